"""Rotoselect / Rotosolve call-sequence parity (cost_minimiser.py:52-106, 267-368) on CPU: the
product's CostMinimiser (generic path: one cost_finder() call per candidate) issues the same
candidate circuits, in the same order, with the same fitted angles and evaluation counts as the
oracle's restatement; both driven by the oracle's statevector cost."""
import numpy as np
import pytest

from oracle import adapt_host
from oracle import sv as osv

N = 5


def _problem(seed):
    """Fixed 'target' brickwork, then a variational block of labelled rotations and CX."""
    rng = np.random.default_rng(seed)
    fixed = []
    for layer in range(3):
        for q in range(N):
            fixed.append([["rx", "ry", "rz"][rng.integers(3)], (q,), [float(rng.uniform(-np.pi, np.pi))], None])
        for q in range(layer % 2, N - 1, 2):
            fixed.append(["cx", (q, q + 1), [], None])
    var = []
    for layer in range(2):
        for q in range(N):
            nm = ["rx", "ry", "rz"][rng.integers(3)]
            var.append([nm, (q,), [float(rng.uniform(-1, 1))], nm])
        for q in range(layer % 2, N - 1, 2):
            var.append(["cx", (q, q + 1), [], None])
    return fixed + var, (len(fixed), len(fixed) + len(var))


def _cost(ops):
    return 1.0 - abs(osv.simulate(N, [(o[0], tuple(o[1]), tuple(o[2])) for o in ops])[0]) ** 2


def _snap(ops, rng):
    return tuple((o[0], round(float(o[2][0]), 12)) for o in ops[rng[0]:rng[1]] if o[0] in ("rx", "ry", "rz"))


def _product_run(ops0, rng, rotoselect, n_cycles):
    from adaptaqc_amd.circuit import Operation, QuantumCircuit
    from adaptaqc_amd.utils.constants import ALG_ROTOSELECT, ALG_ROTOSOLVE
    from adaptaqc_amd.utils.cost_minimiser import CostMinimiser

    qc = QuantumCircuit(N)
    for name, q, p, label in ops0:
        qc.append(Operation(name, len(q), list(p), label), q)
    log = []

    def cost_finder():
        ops = [[i.operation.name, i.qubits, list(i.operation.params), i.operation.label] for i in qc.data]
        log.append(_snap(ops, rng))
        return _cost(ops)

    cm = CostMinimiser(cost_finder, lambda: rng, qc)
    cost = cm.minimize_cost(ALG_ROTOSELECT if rotoselect else ALG_ROTOSOLVE, max_cycles=n_cycles, tol=1e-10)
    final = [[i.operation.name, i.qubits, list(i.operation.params), i.operation.label] for i in qc.data]
    return cost, log, final


def _oracle_run(ops0, rng, rotoselect, n_cycles):
    ops = [list(o[:2]) + [list(o[2]), o[3]] for o in ops0]
    log, calls = [], []

    def cost_fn(o):
        log.append(_snap(o, rng))
        return _cost(o)

    cost = adapt_host.minimize_cost(ops, cost_fn, rotoselect, rng, calls, max_cycles=n_cycles, tol=1e-10)
    return cost, log, ops, calls


@pytest.mark.parametrize("rotoselect", [True, False])
def test_call_sequence_matches_oracle(rotoselect):
    ops0, rng = _problem(3)
    c_p, log_p, fin_p = _product_run(ops0, rng, rotoselect, 2)
    c_o, log_o, fin_o, calls = _oracle_run(ops0, rng, rotoselect, 2)
    n_rot = sum(1 for o in ops0[rng[0]:rng[1]] if o[0] in ("rx", "ry", "rz"))
    per_gate = 7 if rotoselect else 3
    assert len(log_o) == 1 + 2 * per_gate * n_rot  # initial + 2 cycles
    assert len(log_p) == len(log_o)
    for a, b in zip(log_p, log_o):  # identical candidate circuits, call by call
        assert [x[0] for x in a] == [x[0] for x in b]
        np.testing.assert_allclose([x[1] for x in a], [x[1] for x in b], atol=1e-9)
    assert abs(c_p - c_o) < 1e-12
    assert [o[0] for o in fin_p] == [o[0] for o in fin_o]
    # the candidates per gate, in the reference's order: rx(0), then each axis at +pi/2, -pi/2
    if rotoselect:
        first = [c for c in calls[1:8]]
        assert [c[1] for c in first] == ["rx", "rx", "rx", "ry", "ry", "rz", "rz"]
        assert [c[2] for c in first] == [0.0, np.pi / 2, -np.pi / 2, np.pi / 2, -np.pi / 2, np.pi / 2, -np.pi / 2]


def test_exact_tie_keeps_first_axis():
    """A rotation between H(0)CX(0,1) and its inverse: <Phi+|V x I|Phi+> = tr(V)/2 = cos(theta/2) for
    every axis, so all three axes fit to the same cost (0 at theta = 0) -- an exact tie, which the
    reference's strict `<` (cost_minimiser.py:333) gives to rx.  The product picks rx too (near-ties
    within 1e-13 count as ties: the fitted costs differ only by rounding)."""
    ops0 = [["h", (0,), [], None], ["cx", (0, 1), [], None], ["ry", (0,), [0.7], "ry"], ["cx", (0, 1), [], None],
            ["h", (0,), [], None]]
    global N
    n_save, N = N, 2
    try:
        rng = (2, 3)
        _, log_p, fin_p = _product_run(ops0, rng, True, 1)
        costs = [_cost([o if k != 2 else [s[0][0], o[1], [s[0][1]], s[0][0]] for k, o in enumerate(ops0)])
                 for s in log_p[1:]]
        assert len(costs) == 7
        assert fin_p[2][0] == "rx" and abs(fin_p[2][2][0]) < 1e-9
        # the three fitted minima are equal up to rounding
        c_id = costs[0]
        fits = [adapt_host.minimum_of_sinusoidal(c_id, costs[1 + 2 * k], costs[2 + 2 * k])[1] for k in range(3)]
        assert max(fits) - min(fits) < 1e-13
    finally:
        N = n_save
