"""Restatement of the host-side scalar logic around the hot path (no arithmetic kernels).

* coupling maps (utils/constants.py:34-110) and ``remove_permutations_from_coupling_map``
  (utils/utilityfunctions.py:262-269);
* reuse priorities and arg-max pair selection (compilers/adapt/adapt_compiler.py:832-837,
  984-1065);
* layer-absorption counting (adapt_compiler.py:691-706);
* ``minimum_of_sinusoidal`` (utils/utilityfunctions.py:34-57),
  ``has_stopped_improving`` (:272-278) and the Rotoselect / Rotosolve call sequence
  (utils/cost_minimiser.py:52-106, 267-368: candidates, order, strict `<`).
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


# --------------------------------------------------------------------------------------------
# Rotoselect / Rotosolve call sequence (utils/cost_minimiser.py:52-106, 267-368)
#
# ``ops`` is a mutable list of [name, qubits, params(list), label]; ``cost_fn(ops)`` evaluates the
# whole circuit (the reference's ``cost_finder``); ``log`` receives one entry per evaluation:
# (gate index, gate name, angle) of the gate being varied, in call order.
# --------------------------------------------------------------------------------------------
SUPPORTED_1Q = ("rx", "ry", "rz")  # circuit_operations SUPPORTED_1Q_GATES order


def _set_gate(ops, i, name, angle):
    """co.replace_1q_gate (circuit_operations_basic.py:70-99): same qubit, new kind and angle,
    label = the kind (create_1q_gate, :20-34); a None kind leaves the gate as it is."""
    if name is None:
        return
    ops[i] = [name, ops[i][1], [float(angle)], name]


def find_best_angle(ops, i, name, cost_fn, log, cost_for_identity=None):
    """cost_minimiser.py:344-368: costs at 0, pi/2, -pi/2 (0 skipped when given), closed-form
    sinusoid minimum; the gate is restored afterwards."""
    orig = list(ops[i])
    costs = []
    angles = [0, np.pi / 2, -np.pi / 2]
    if cost_for_identity is not None:
        costs.append(cost_for_identity)
        angles.remove(0)
    for th in angles:
        _set_gate(ops, i, name, th)
        log.append((i, name, float(th)))
        costs.append(cost_fn(ops))
    th_min, c_min = minimum_of_sinusoidal(costs[0], costs[1], costs[2])
    ops[i] = orig
    return th_min, c_min


def replace_with_best_1q_gate(ops, i, cost_fn, log):
    """cost_minimiser.py:318-342: rx(0) once, then each axis at +-pi/2; strict `<` keeps the
    first axis on exact ties."""
    _set_gate(ops, i, "rx", 0)
    log.append((i, "rx", 0.0))
    c_id = cost_fn(ops)
    best_name, best_angle, best_cost = None, None, 1
    for name in SUPPORTED_1Q:
        ang, c = find_best_angle(ops, i, name, cost_fn, log, c_id)
        if c < best_cost:
            best_name, best_angle, best_cost = name, ang, c
    _set_gate(ops, i, best_name, best_angle)
    return best_cost


def reduce_cost(ops, cost_fn, change_kind, index_range, log):
    """cost_minimiser.py:267-316 (rotosolve_fraction = 1): every supported 1-qubit gate in the
    range, in circuit order."""
    cost = 1
    for i in range(*index_range):
        if ops[i][0] not in SUPPORTED_1Q:
            continue
        if change_kind:
            cost = replace_with_best_1q_gate(ops, i, cost_fn, log)
        else:
            ang, cost = find_best_angle(ops, i, ops[i][3], cost_fn, log)
            _set_gate(ops, i, ops[i][3], ang)
    return cost


def minimize_cost(ops, cost_fn, rotoselect, index_range, log, max_cycles=1000, stop_val=-np.inf, tol=1e-10):
    """cost_minimiser.py:52-106: one evaluation, then cycles of reduce_cost until stop_val, the
    cycle cap, or has_stopped_improving over the last 3 cycles (after more than 3)."""
    hist = []
    log.append(("initial",))
    cost = cost_fn(ops)
    cycles = 0
    while cost > stop_val and cycles < max_cycles:
        cost = reduce_cost(ops, cost_fn, rotoselect, index_range, log)
        cycles += 1
        hist.append(cost)
        if len(hist) > 3 and has_stopped_improving(hist[-3:], tol):
            break
    return cost
