"""Owning Python wrappers around libaqchip handles (device-resident statevector / MPS)."""
import ctypes

import numpy as np

from . import _lib


class DeviceSV:
    """2^n complex128 amplitudes resident in HBM (Aer statevector_simulator state)."""

    def __init__(self, n):
        self._l = _lib.lib()
        self.n = int(n)
        h = ctypes.c_void_p()
        _lib.check(self._l.aqc_sv_create(self.n, ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self._l.aqc_sv_destroy(self.h)
            self.h = None

    __del__ = close

    def reset(self):
        _lib.check(self._l.aqc_sv_reset(self.h))

    def copy_from(self, other):
        _lib.check(self._l.aqc_sv_copy(self.h, other.h))

    def apply(self, ops):
        if len(ops) == 0:
            return
        arr = ops if isinstance(ops, np.ndarray) else _lib.ops_array(ops)
        _lib.check(self._l.aqc_sv_apply(self.h, _lib.ptr(arr), len(arr)))

    def amp0(self):
        re, im = ctypes.c_double(), ctypes.c_double()
        _lib.check(self._l.aqc_sv_amp0(self.h, ctypes.byref(re), ctypes.byref(im)))
        return complex(re.value, im.value)

    def z_all(self):
        out = np.zeros(self.n)
        _lib.check(self._l.aqc_sv_z_all(self.h, _lib.dptr(out)))
        return out

    def transition(self, ket, q):
        """2x2 T[a][b] = <self| (|a><b|)_q |ket> (cached Rotoselect / Rotosolve)."""
        out = np.zeros(4, dtype=np.complex128)
        _lib.check(self._l.aqc_sv_transition(self.h, ket.h, int(q), _lib.ptr(out)))
        return out.reshape(2, 2)

    def pair_rdms(self, pairs):
        """4x4 reduced density matrices of qubit pairs (entanglement_measures.py:326-340)."""
        pairs = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1))
        out = np.zeros(len(pairs) // 2 * 16, dtype=np.complex128)
        if len(pairs):
            _lib.check(self._l.aqc_sv_pair_rdms(self.h, _lib.ptr(pairs), len(pairs) // 2, _lib.ptr(out)))
        return out.reshape(-1, 4, 4)

    def get(self):
        out = np.zeros(2 ** self.n, dtype=np.complex128)
        _lib.check(self._l.aqc_sv_get(self.h, _lib.ptr(out)))
        return out

    def set(self, psi):
        psi = np.ascontiguousarray(psi, dtype=np.complex128)
        _lib.check(self._l.aqc_sv_set(self.h, _lib.ptr(psi)))


class DeviceMPS:
    """Vidal-form MPS resident in HBM with Aer MPS-simulator semantics."""

    def __init__(self, n, chi_cap, threshold=1e-16, max_chi=None):
        self._l = _lib.lib()
        self.n = int(n)
        self.chi_cap = int(chi_cap)
        h = ctypes.c_void_p()
        _lib.check(
            self._l.aqc_mps_create(self.n, self.chi_cap, float(threshold), int(max_chi or 0), ctypes.byref(h))
        )
        self.h = h

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self._l.aqc_mps_destroy(self.h)
            self.h = None

    __del__ = close

    # -- state transfer --------------------------------------------------------------
    def set_truncation(self, threshold, max_chi):
        _lib.check(self._l.aqc_mps_set_truncation(self.h, float(threshold), int(max_chi or 0)))

    def load_aer(self, qiskit_mps):
        gam, lam = qiskit_mps
        if len(gam) != self.n:
            raise ValueError("MPS length mismatch")
        dims = [1]
        for a, _ in gam:
            dims.append(np.asarray(a).shape[1])
        dims = np.asarray(dims, dtype=np.int32)
        if dims.max() > self.chi_cap:
            raise ValueError(f"MPS bond dimension {dims.max()} exceeds chi_cap {self.chi_cap}")
        g = np.concatenate(
            [np.stack([np.asarray(a, dtype=np.complex128), np.asarray(b, dtype=np.complex128)]).reshape(-1) for a, b in gam]
        )
        l = np.concatenate([np.asarray(x, dtype=np.float64).reshape(-1) for x in lam]) if len(lam) else np.zeros(1)
        g = np.ascontiguousarray(g)
        l = np.ascontiguousarray(l)
        _lib.check(self._l.aqc_mps_set_vidal(self.h, _lib.ptr(dims), _lib.ptr(g), _lib.ptr(l)))

    def dims(self):
        d = np.zeros(self.n + 1, dtype=np.int32)
        _lib.check(self._l.aqc_mps_get_dims(self.h, _lib.ptr(d)))
        return d

    def to_aer(self):
        """save_matrix_product_state: sorted qubits, Aer format."""
        d = np.zeros(self.n + 1, dtype=np.int32)
        _lib.check(self._l.aqc_mps_get_vidal(self.h, _lib.ptr(d), None, None))
        ng = int(sum(2 * d[i] * d[i + 1] for i in range(self.n)))
        nl = int(sum(d[1:self.n]))
        g = np.zeros(ng, dtype=np.complex128)
        l = np.zeros(max(nl, 1), dtype=np.float64)
        _lib.check(self._l.aqc_mps_get_vidal(self.h, _lib.ptr(d), _lib.ptr(g), _lib.ptr(l)))
        gam, lam = [], []
        off = 0
        for i in range(self.n):
            a, b = int(d[i]), int(d[i + 1])
            t = g[off: off + 2 * a * b].reshape(2, a, b)
            gam.append((t[0].copy(), t[1].copy()))
            off += 2 * a * b
        off = 0
        for bnd in range(1, self.n):
            k = int(d[bnd])
            lam.append(l[off: off + k].copy())
            off += k
        return gam, lam

    def preprocessed(self):
        """aqc_research ``_preprocess_mps`` form: list of (2, chi_l, chi_r) arrays."""
        gam, lam = self.to_aer()
        out = []
        for i, (a, b) in enumerate(gam):
            t = np.stack([a, b])
            if i < self.n - 1:
                t = t * lam[i][None, None, :]
            out.append(t)
        return out

    def copy_from(self, other):
        _lib.check(self._l.aqc_mps_copy(self.h, other.h))

    # -- gates and measurements ------------------------------------------------------
    def apply(self, ops):
        if len(ops) == 0:
            return
        arr = ops if isinstance(ops, np.ndarray) else _lib.ops_array(ops)
        _lib.check(self._l.aqc_mps_apply(self.h, _lib.ptr(arr), len(arr)))

    def sort(self):
        _lib.check(self._l.aqc_mps_sort(self.h))

    def overlap_zero(self):
        """``mps_dot(psi, zero_mps)`` = <psi|0...0>."""
        re, im = ctypes.c_double(), ctypes.c_double()
        _lib.check(self._l.aqc_mps_overlap_zero(self.h, ctypes.byref(re), ctypes.byref(im)))
        return complex(re.value, im.value)

    def dot(self, other):
        """<self|other> (conjugates self)."""
        re, im = ctypes.c_double(), ctypes.c_double()
        _lib.check(self._l.aqc_mps_dot(self.h, other.h, ctypes.byref(re), ctypes.byref(im)))
        return complex(re.value, im.value)

    def z_all(self):
        out = np.zeros(self.n)
        _lib.check(self._l.aqc_mps_z_all(self.h, _lib.ptr(out)))
        return out

    def amps_hw1(self):
        out = np.zeros(2 * self.n)
        _lib.check(self._l.aqc_mps_amps_hw1(self.h, _lib.ptr(out)))
        return out[0::2] + 1j * out[1::2]

    def product_fit(self, svec=None, min_sweeps=10, max_sweeps=50, tol=1e-12):
        """Best product-state approximation (aqc_mps_product_fit): returns (svec (n, 2), fidelity,
        sweeps).  svec None starts from the chi = 1 truncation of the canonical form."""
        guess = svec is None
        s = np.zeros((self.n, 2), dtype=np.complex128) if guess else np.array(svec, dtype=np.complex128)
        s = np.ascontiguousarray(s.reshape(self.n, 2))
        fid = ctypes.c_double()
        sw = ctypes.c_int()
        _lib.check(self._l.aqc_mps_product_fit(self.h, _lib.ptr(s), int(guess), int(min_sweeps), int(max_sweeps),
                                               float(tol), ctypes.byref(fid), ctypes.byref(sw)))
        return s, fid.value, sw.value

    def pair_rdms(self, pairs):
        """4x4 RDMs of qubit pairs by environment chains (aqc_research partial_trace semantics)."""
        pairs = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1))
        out = np.zeros(len(pairs) // 2 * 16, dtype=np.complex128)
        if len(pairs):
            _lib.check(self._l.aqc_mps_pair_rdms(self.h, _lib.ptr(pairs), len(pairs) // 2, _lib.ptr(out)))
        return out.reshape(-1, 4, 4)


def _handles(states):
    arr = (ctypes.c_void_p * len(states))(*[s.h.value for s in states])
    return arr


class OpsBatch:
    """Per-state op lists marshalled once for the C ABI: the pointer array and the counts that
    apply_batch would otherwise rebuild from the Python list on every call (1-2 ms for 1024 lists,
    mostly ``ndarray.ctypes``).  It holds references to its arrays, so their contents may be
    rewritten in place between calls (new angles) and the batch stays valid; replacing an array
    needs a new OpsBatch."""

    def __init__(self, ops_lists):
        self.arrays = [np.ascontiguousarray(o) if isinstance(o, np.ndarray) else _lib.ops_array(o)
                       for o in ops_lists]
        self.ptrs = (ctypes.c_void_p * len(self.arrays))(*[a.ctypes.data if len(a) else 0 for a in self.arrays])
        self.counts = np.asarray([len(a) for a in self.arrays], dtype=np.int32)

    def __len__(self):
        return len(self.arrays)


def apply_batch(states, ops_lists, sort=False, wait=True):
    """Apply per-state op lists (one batched launch sequence, or one fused chain per state); with
    sort=True every state also returns to sorted qubit order in the same schedule (an evaluation's
    replay + save).  ops_lists: a list of op lists / ops arrays, or an OpsBatch.  wait=False
    returns once the work is queued; call check_batch(states) before trusting the states (their
    error flags are read there)."""
    if not states:
        return
    l = _lib.lib()
    batch = ops_lists if isinstance(ops_lists, OpsBatch) else OpsBatch(ops_lists)
    if len(batch) != len(states):
        raise ValueError("apply_batch: one op list per state")
    fn = l.aqc_mps_apply_sort_batch if sort else l.aqc_mps_apply_batch
    if not wait:
        fn = l.aqc_mps_apply_sort_batch_async if sort else l.aqc_mps_apply_batch_async
    _lib.check(fn(_handles(states), len(states), batch.ptrs, _lib.ptr(batch.counts)))


def check_batch(states):
    """Wait for the states' queued work and raise on their error flags (after apply_batch(...,
    wait=False))."""
    if states:
        _lib.check(_lib.lib().aqc_mps_check_batch(_handles(states), len(states)))


EM_METHOD_CODES = {"concurrence": 0, "eof": 1, "negativity": 2, "log_negativity": 3}


def entanglement_measures(rdms, method):
    """Entanglement measure of each 4x4 density matrix on the device (aqc_entanglement_measures)."""
    code = EM_METHOD_CODES[method]
    r = np.ascontiguousarray(np.asarray(rdms, dtype=np.complex128).reshape(-1, 16))
    out = np.zeros(len(r))
    if len(r):
        _lib.check(_lib.lib().aqc_entanglement_measures(_lib.ptr(r), len(r), code, _lib.ptr(out), 0))
    return out


def copy_batch(dst, src):
    """dst[s] <- src[s] for every state in one launch (per-evaluation reload of a cached MPS)."""
    if len(dst) != len(src):
        raise ValueError("copy_batch: dst and src differ in length")
    if not dst:
        return
    _lib.check(_lib.lib().aqc_mps_copy_batch(_handles(dst), _handles(src), len(dst)))


def overlap_zero_batch(states):
    l = _lib.lib()
    out = np.zeros(2 * len(states))
    _lib.check(l.aqc_mps_overlap_zero_batch(_handles(states), len(states), _lib.ptr(out)))
    return out[0::2] + 1j * out[1::2]


def z_all_batch(states):
    """<Z_i> of every state (rows), one set of launches (aqc_mps_z_all_batch)."""
    if not states:
        return np.zeros((0, 0))
    n = states[0].n
    out = np.zeros(len(states) * n)
    _lib.check(_lib.lib().aqc_mps_z_all_batch(_handles(states), len(states), _lib.ptr(out)))
    return out.reshape(len(states), n)


def z_sum_batch(base, states):
    """sum_i <Z_i> of every state (aqc_mps_z_sum_batch): states copied from ``base`` (unchanged
    since) contract only the sites they rewrote, against environments cached on ``base``."""
    out = np.zeros(len(states))
    if states:
        _lib.check(_lib.lib().aqc_mps_z_sum_batch(base.h, _handles(states), len(states), _lib.ptr(out)))
    return out


def zero_hw1_batch(base, states, amps=False):
    """(<psi|0..0> per state, and with ``amps`` the amplitudes <e_i|psi> as rows) through
    aqc_mps_zero_hw1_batch: states copied from ``base`` (unchanged since) contract only the sites
    they rewrote, against rows cached on ``base``."""
    ns = len(states)
    ov = np.zeros(2 * ns)
    a = np.zeros(2 * ns * (states[0].n if ns else 0)) if amps else None
    if ns:
        _lib.check(_lib.lib().aqc_mps_zero_hw1_batch(base.h, _handles(states), ns, _lib.ptr(ov),
                                                     _lib.ptr(a) if amps else None))
    ovc = ov[0::2] + 1j * ov[1::2]
    if not amps:
        return ovc, None
    return ovc, (a[0::2] + 1j * a[1::2]).reshape(ns, -1)


def amps_hw1_batch(states):
    """Amplitudes <e_i|psi> of every state (rows, complex), one set of launches
    (aqc_mps_amps_hw1_batch)."""
    if not states:
        return np.zeros((0, 0), dtype=complex)
    n = states[0].n
    out = np.zeros(2 * len(states) * n)
    _lib.check(_lib.lib().aqc_mps_amps_hw1_batch(_handles(states), len(states), _lib.ptr(out)))
    return (out[0::2] + 1j * out[1::2]).reshape(len(states), n)


def pair_grads_batch(states, svec, pairs, u0, gens, degs, out=None):
    """Per-state gradient norms for every pair; ``out`` may be a device pointer (int): then the call
    returns once the work is queued and is ordered both ways against torch's current stream -- the
    sweep waits for the torch work queued before it (aqc_stream_wait: a fill of ``out``, the
    previous step's reads of it), and torch's stream waits for the sweep (aqc_stream_join), so
    torch ops on ``out`` (the all-gather, the arg-max) see the scores."""
    l = _lib.lib()
    svec = np.ascontiguousarray(np.asarray(svec, dtype=np.complex128).reshape(-1))
    pairs = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1))
    u0 = np.ascontiguousarray(np.asarray(u0, dtype=np.complex128).reshape(16))
    gens = np.ascontiguousarray(np.asarray(gens, dtype=np.complex128).reshape(-1))
    degs = np.ascontiguousarray(np.asarray(degs, dtype=np.float64).reshape(-1))
    npairs = len(pairs) // 2
    ngen = len(degs)
    if out is None:
        host = np.zeros((len(states), npairs))
        outp, is_dev = _lib.ptr(host), 0
    else:
        import torch

        host, outp, is_dev = None, ctypes.c_void_p(int(out)), 1
        _lib.check(l.aqc_stream_wait(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    _lib.check(
        l.aqc_pair_grads_batch(
            _handles(states), len(states), _lib.ptr(svec), _lib.ptr(pairs), npairs, _lib.ptr(u0),
            _lib.ptr(gens) if ngen else None, _lib.ptr(degs) if ngen else None, ngen, outp, is_dev,
        )
    )
    if is_dev:
        import torch

        _lib.check(l.aqc_stream_join(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return host


def argmax_rows(scores, prio):
    """Per-row np.argmax(scores * prio) (first maximum) of a device score matrix on libaqchip's
    kernel (aqc_argmax_scaled_batch), ordered both ways against torch's current stream like a
    device-output sweep.  scores: [S, ld] float64 CUDA tensor (the first len(prio) columns are
    scored), prio: [count] float64 CUDA tensor.  Returns ([S] int64 index, [S] float64 score)."""
    import torch

    l = _lib.lib()
    S, ld = scores.shape
    count = prio.shape[0]
    if not (scores.is_cuda and prio.is_cuda and scores.dtype == torch.float64 and prio.dtype == torch.float64
            and scores.is_contiguous() and prio.is_contiguous() and count <= ld):
        raise ValueError("argmax_rows: contiguous float64 CUDA tensors with len(prio) <= scores.shape[1]")
    out = torch.empty((2, S), dtype=torch.float64, device=scores.device)
    cur = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(l.aqc_stream_wait(cur))
    _lib.check(l.aqc_argmax_scaled_batch(ctypes.c_void_p(scores.data_ptr()), ld, ctypes.c_void_p(prio.data_ptr()),
                                         count, S, ctypes.c_void_p(out.data_ptr())))
    _lib.check(l.aqc_stream_join(cur))
    return out[0].to(torch.int64), out[1]
