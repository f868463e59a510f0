"""Restatement of the host-side scalar logic around the hot path (no arithmetic kernels).

* coupling maps (utils/constants.py:34-110) and ``remove_permutations_from_coupling_map``
  (utils/utilityfunctions.py:262-269);
* reuse priorities and arg-max pair selection (compilers/adapt/adapt_compiler.py:832-837,
  984-1065);
* layer-absorption counting (adapt_compiler.py:691-706);
* ``minimum_of_sinusoidal`` (utils/utilityfunctions.py:34-57) and
  ``has_stopped_improving`` (:272-278).
"""
import numpy as np


def coupling_map_full(n):
    out = []
    for i in range(1, n):
        for j in range(n - i):
            out.append((j, j + i))
    return out


def coupling_map_linear(n):
    return [(j, j + 1) for j in range(n - 1)]


def remove_permutations(cmap):
    seen, out = set(), []
    for p in cmap:
        k = tuple(sorted(p))
        if k not in seen:
            seen.add(k)
            out.append(p)
    return out


def pair_reuse_priority(history, pair, k, isql=False):
    if len(history) > int(isql) and pair == history[-1]:
        return -1
    if k == 0:
        return 1
    rev = history[::-1]
    try:
        loc = rev.index(pair)
        return 1 - np.exp2(-loc / k)
    except ValueError:
        return 1


def qubit_reuse_priority(history, pair, k, isql=False):
    if len(history) > int(isql) and pair == history[-1]:
        return -1
    if k == 0:
        return 1
    rev = history[::-1]

    def last(q):
        for i, t in enumerate(rev):
            if q in t:
                return i
        return np.inf

    return np.min([1 - np.exp2(-(last(q) + 1) / k) for q in pair])


def reuse_priorities(cmap, history, k, mode="pair", isql=False):
    if not len(history):
        return [1 for _ in cmap]
    f = pair_reuse_priority if mode == "pair" else qubit_reuse_priority
    return [f(history, p, k, isql) for p in cmap]


def best_gradient_pair(cmap, gradients, history, k, mode="pair"):
    combined = np.multiply(gradients, reuse_priorities(cmap, history, k, mode))
    return cmap[int(np.argmax(combined))]


def num_layers_to_absorb(index, layers_as_gates, rotosolve_frequency, max_layers_to_modify):
    since = index % rotosolve_frequency
    nxt = index + (rotosolve_frequency - since)
    lowest = nxt - max_layers_to_modify + 1
    return len([i for i in layers_as_gates if i < lowest])


def normalized_angle(a):
    while a > np.pi or a < -np.pi:
        a = a - 2 * np.pi if a > np.pi else a + 2 * np.pi
    return a


def minimum_of_sinusoidal(v0, vp, vm):
    theta = -(np.pi / 2) - np.arctan2(2 * v0 - vp - vm, vp - vm)
    theta = normalized_angle(theta)
    c = 0.5 * (vp + vm)
    vpi = (vp + vm) - v0
    amp = 0.5 * (((v0 - vpi) ** 2 + (vp - vm) ** 2) ** 0.5)
    return theta, c - amp


def has_stopped_improving(hist, rel_tol=1e-2):
    try:
        fit = np.polyfit(list(range(len(hist))), hist, 1)
        return fit[0] / np.absolute(np.mean(hist)) > -1 * rel_tol
    except np.linalg.LinAlgError:
        return False
