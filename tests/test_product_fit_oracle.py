"""The chi = 1 variational-compression oracle (oracle/product_fit.py) on CPU: exact on product
states, the 2-qubit optimum is the top singular value of the coefficient matrix, and the result
is a local optimum (no single-site or two-site update raises |<s|psi>|)."""
import numpy as np

from oracle import mps as M
from oracle import product_fit as PF


def _state(n, seed, layers=3):
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(layers):
        for q in range(n):
            ops.append(("ry", (q,), (float(rng.uniform(-1, 1)),)))
            ops.append(("rz", (q,), (float(rng.uniform(-1, 1)),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    return M.run_circuit(n, ops)


def test_product_state_is_recovered_exactly():
    rng = np.random.default_rng(1)
    n = 6
    ops = [("ry", (q,), (float(rng.uniform(-3, 3)),)) for q in range(n)] + \
          [("rz", (q,), (float(rng.uniform(-3, 3)),)) for q in range(n)]
    st = M.run_circuit(n, ops)
    s, fid, sw = PF.product_fit(st.preprocessed(), PF.initial_guess(st.g))
    assert abs(fid - 1.0) < 1e-12 and sw == 10


def test_two_qubit_optimum_is_top_singular_value():
    st = _state(2, 4, layers=4)
    pre = st.preprocessed()
    s, fid, _ = PF.product_fit(pre, PF.initial_guess(st.g))
    coeff = np.array([[M.extract_amplitude(pre, a + 2 * b) for b in range(2)] for a in range(2)])
    assert abs(fid - np.linalg.svd(coeff, compute_uv=False)[0] ** 2) < 1e-12


def test_local_optimality():
    n = 8
    st = _state(n, 7)
    pre = st.preprocessed()
    s, fid, sw = PF.product_fit(pre, PF.initial_guess(st.g), tol=1e-14)
    assert abs(abs(PF.overlap(pre, s)) ** 2 - fid) < 1e-12
    for i in range(n):  # single site: the optimum over s_i alone is |F_i|
        others = [x for x in s]
        l = np.ones(1, dtype=complex)
        for k in range(i):
            l = l @ PF._m(pre[k], others[k])
        r = np.ones(1, dtype=complex)
        for k in range(n - 1, i, -1):
            r = PF._m(pre[k], others[k]) @ r
        F = np.array([l @ pre[i][a] @ r for a in range(2)])
        assert np.linalg.norm(F) ** 2 <= fid * (1 + 1e-9)


def test_oracle_fit_equals_brute_force_best_product_state():
    """The restatement reaches the global optimum on a weakly entangled target (rzz(0.3) chain on a
    rotated product state): equal to an independent maximisation over all per-qubit Bloch angles."""
    from scipy.optimize import minimize

    from adaptaqc_amd import gates as G
    from oracle import sv as osv

    n = 4
    rng = np.random.default_rng(33)
    ops = []
    for q in range(n):
        ops += [("ry", (q,), (float(rng.uniform(0.2, 2.9)),)), ("rz", (q,), (float(rng.uniform(-3, 3)),))]
    for q in range(n - 1):
        ops += [("cx", (q, q + 1), ()), ("rz", (q + 1,), (0.3,)), ("cx", (q, q + 1), ())]
    target = osv.simulate(n, ops)

    def neg_fid(x):
        vs = [np.array([np.cos(x[2 * q] / 2), np.exp(1j * x[2 * q + 1]) * np.sin(x[2 * q] / 2)]).reshape(2, 1)
              for q in range(n)]
        return -abs(np.vdot(G.kron_le(*vs).reshape(-1), target)) ** 2

    r = np.random.default_rng(5)
    best = max(-minimize(neg_fid, r.uniform(-3, 3, 2 * n), method="BFGS", options={"gtol": 1e-12}).fun
               for _ in range(20))
    st = M.run_circuit(n, ops)
    _, fid, _ = PF.product_fit(st.preprocessed(), PF.initial_guess(st.g), 10, 50, 1e-12)
    assert 0.5 < best < 1 - 1e-4
    assert abs(fid - best) < 1e-8
