"""Matrix-product-state restatement of qiskit-aer ~=0.16.0's MPS simulator as the reference drives it.

The reference (adaptaqc/backends/aer_mps_backend.py:27-42,76-78) builds
``AerSimulator(method="matrix_product_state",
matrix_product_state_truncation_threshold=thr, matrix_product_state_max_bond_dimension=chi)``
and runs circuits whose first instruction is ``set_matrix_product_state`` (the cached MPS,
approximate_compiler.py:180-204, adapt_compiler.py:1133-1143).  Restated here from Aer's
published algorithm (``matrix_product_state_internal.cpp`` / ``svd.cpp``):

* State in Vidal form: Gamma_i[sigma] (chi_{i-1} x chi_i), lambda_i on bond (i, i+1).
  Qubit i starts at site i; a permutation ``order`` (site -> qubit) is kept lazily.
* 1-qubit gate: Gamma[loc(q)] <- U Gamma[loc(q)]  (no SVD).
* 2-qubit gate on qubits (a, b) at sites (pa, pb): default ``mps_swap_left`` routing moves the
  higher site down to low+1 by adjacent SWAPs (each a full two-site update, ordering updated),
  then applies the gate on (low, low+1).  The permutation is NOT undone after the gate.
* Two-site update: theta = diag(lam_{l}) G_p diag(lam_p) G_{p+1} diag(lam_{r}), theta' = gate.theta,
  SVD, ``reduce_zeros`` truncation, then divide the outer lambdas back out.
* ``reduce_zeros``: keep s_k with s_k^2 > CHOP (1e-16); cap at max_bond_dimension; drop the
  smallest values while their accumulated s^2 stays below truncation_threshold (keep >= 1);
  renormalise the kept values to unit 2-norm.
* ``save_matrix_product_state`` first sorts qubits back to natural order
  (``move_all_qubits_to_sorted_ordering``: for each target position, bubble the qubit down
  with adjacent swaps).

Parity status: with the truncation threshold non-binding these choices do not change the
represented state; when ``max_chi`` binds, Aer's exact tail rule / renormalisation / routing
could not be verified offline ("parity unpinned").
"""
import numpy as np

from . import gates as G

CHOP = 1e-16


class MPS:
    def __init__(self, n, gammas=None, lambdas=None):
        self.n = n
        if gammas is None:
            gammas = []
            for _ in range(n):
                g = np.zeros((2, 1, 1), dtype=complex)
                g[0, 0, 0] = 1.0
                gammas.append(g)
            lambdas = [np.ones(1) for _ in range(n - 1)]
        self.g = [np.array(x, dtype=complex) for x in gammas]
        self.l = [np.array(x, dtype=float) for x in lambdas]
        self.order = list(range(n))  # site -> qubit
        self.loc = list(range(n))  # qubit -> site
        # test hook: when a list, every two-site update appends (site, singular values before
        # truncation) -- lets tests predict which SVD path the device should take
        self.svd_log = None

    @classmethod
    def from_aer(cls, qiskit_mps):
        """From Aer format ``(list[(G0, G1)], list[lambda])`` (constants.py:17)."""
        gam, lam = qiskit_mps
        g = [np.stack([np.asarray(a, dtype=complex), np.asarray(b, dtype=complex)]) for a, b in gam]
        return cls(len(g), g, [np.asarray(x, dtype=float) for x in lam])

    def copy(self):
        m = MPS(self.n, [x.copy() for x in self.g], [x.copy() for x in self.l])
        m.order = list(self.order)
        m.loc = list(self.loc)
        m.svd_log = self.svd_log
        return m

    def to_aer(self):
        return ([(x[0].copy(), x[1].copy()) for x in self.g], [x.copy() for x in self.l])

    # -- gates -------------------------------------------------------------------------
    def apply_1q(self, q, u):
        p = self.loc[q]
        self.g[p] = np.einsum("ab,bij->aij", u, self.g[p])

    def theta_matrix(self, p, op4=None):
        """theta' = op4 . (lam_l G_p lam_p G_{p+1} lam_r) as a (2 chi_l) x (2 chi_r) matrix, rows
        (s1, l), columns (s2, r) -- the matrix a two-site update decomposes."""
        n = self.n
        ll = self.l[p - 1] if p > 0 else np.ones(1)
        lr = self.l[p + 1] if p + 1 < n - 1 else np.ones(1)
        a = self.g[p] * ll[None, :, None]
        b = self.g[p + 1] * lr[None, None, :]
        theta = np.einsum("aim,m,bmj->aibj", a, self.l[p], b)  # (s1, l, s2, r)
        if op4 is not None:
            theta = np.einsum("cdab,aibj->cidj", op4, theta)
        s1, chl, s2, chr_ = theta.shape
        return theta.reshape(s1 * chl, s2 * chr_)

    def _two_site(self, p, op4, thr, max_chi):
        """op4[s1', s2', s1, s2] acts on sites (p, p+1)."""
        n = self.n
        ll = self.l[p - 1] if p > 0 else np.ones(1)
        lr = self.l[p + 1] if p + 1 < n - 1 else np.ones(1)
        mat = self.theta_matrix(p, op4)
        s1, s2 = 2, 2
        chl, chr_ = mat.shape[0] // 2, mat.shape[1] // 2
        u, s, vh = np.linalg.svd(mat, full_matrices=False)
        if self.svd_log is not None:
            self.svd_log.append((p, s.copy()))
        k = truncation_rank(s, thr, max_chi)
        s = s[:k]
        s = s / np.sqrt(np.sum(s * s))
        u = u[:, :k].reshape(s1, chl, k)
        vh = vh[:k, :].reshape(k, s2, chr_).transpose(1, 0, 2)
        self.g[p] = u / ll[None, :, None]
        self.g[p + 1] = vh / lr[None, None, :]
        self.l[p] = s

    def _swap_sites(self, p, thr, max_chi):
        self._two_site(p, G.SWAP.reshape(2, 2, 2, 2), thr, max_chi)
        qa, qb = self.order[p], self.order[p + 1]
        self.order[p], self.order[p + 1] = qb, qa
        self.loc[qa], self.loc[qb] = p + 1, p

    def apply_2q(self, qa, qb, m, thr=1e-16, max_chi=None):
        """Gate m (Qiskit little-endian over (qa, qb)) with Aer swap-left routing."""
        pa, pb = self.loc[qa], self.loc[qb]
        low, high = min(pa, pb), max(pa, pb)
        for i in range(high, low + 1, -1):  # change_position(high, low+1)
            self._swap_sites(i - 1, thr, max_chi)
        mt = np.asarray(m).reshape(2, 2, 2, 2)  # [b1', b0', b1, b0], b0 <-> qa
        if self.loc[qa] == low:  # qa on site low (s1), qb on low+1 (s2)
            op4 = mt.transpose(1, 0, 3, 2)
        else:
            op4 = mt
        self._two_site(low, op4, thr, max_chi)

    def sort_qubits(self, thr=1e-16, max_chi=None):
        """``move_all_qubits_to_sorted_ordering``."""
        for left in range(self.n):
            pos = self.loc[left]
            for j in range(pos, left, -1):
                self._swap_sites(j - 1, thr, max_chi)

    # -- formats ---------------------------------------------------------------------
    def preprocessed(self):
        """aqc_research ``_preprocess_mps``: A_i[s] = Gamma_i[s] diag(lambda_i) (last site bare)."""
        assert self.order == list(range(self.n))
        out = []
        for i in range(self.n):
            a = self.g[i]
            if i < self.n - 1:
                a = a * self.l[i][None, None, :]
            out.append(a.copy())
        return out


def truncation_rank(s, thr, max_chi):
    """Restatement of qiskit-aer ``reduce_zeros`` (see module docstring)."""
    k = int(np.sum(s * s > CHOP))
    k = max(k, 1)
    if max_chi is not None and max_chi > 0:
        k = min(k, int(max_chi))
    tail = 0.0
    while k > 1 and tail + s[k - 1] ** 2 < thr:
        tail += s[k - 1] ** 2
        k -= 1
    return k


def run_circuit(n, ops, thr=1e-16, max_chi=None, mps=None):
    """``mps_from_circuit``: optional leading MPS state, then gates, then sort (save)."""
    st = mps.copy() if mps is not None else MPS(n)
    for name, qubits, params in ops:
        if name == "set_mps":
            st = MPS.from_aer(params[0])
            continue
        if name in ("barrier", "measure", "id"):
            continue
        m = G.matrix(name, params)
        if len(qubits) == 1:
            st.apply_1q(qubits[0], m)
        elif len(qubits) == 2:
            st.apply_2q(qubits[0], qubits[1], m, thr, max_chi)
        else:
            raise ValueError("MPS oracle supports only 1- and 2-qubit gates")
    st.sort_qubits(thr, max_chi)
    return st


# --------------------------------------------------------------------------------------
# aqc_research.mps_operations restatements (call sites: aer_mps_backend.py:49-93,
# gradients.py:77,94,110).  All take preprocessed lists of (2, chi_l, chi_r) arrays.
# --------------------------------------------------------------------------------------

def mps_dot(a, b):
    """<a|b>, conjugating the FIRST argument (pinned by test_gradients.py:39-73)."""
    env = np.ones((1, 1), dtype=complex)
    for x, y in zip(a, b):
        env = np.einsum("ij,sik,sjl->kl", env, np.conj(x), y, optimize=True)
    return complex(env[0, 0])


def mps_expectation_z(mps, q):
    """<psi|Z_q|psi> by full contraction (``mps_expectation(mps, "Z", q)``)."""
    env = np.ones((1, 1), dtype=complex)
    z = np.array([1.0, -1.0])
    for i, x in enumerate(mps):
        y = x * z[:, None, None] if i == q else x
        env = np.einsum("ij,sik,sjl->kl", env, np.conj(x), y, optimize=True)
    return float(np.real(env[0, 0]))


def extract_amplitude(mps, index):
    """<index|psi> for a little-endian basis index (``extract_amplitude``)."""
    v = np.ones((1,), dtype=complex)
    for i, x in enumerate(mps):
        v = v @ x[(index >> i) & 1]
    return complex(v[0])


def mps_to_vector(mps):
    n = len(mps)
    out = np.zeros(2 ** n, dtype=complex)
    for idx in range(2 ** n):
        out[idx] = extract_amplitude(mps, idx)
    return out


def zero_mps(n):
    return MPS(n).preprocessed()
