"""ctypes binding of libaqchip.so (include/aqc_hip.h).

The HIP library is the only compute path: if it is missing or no GPU is visible, every
backend call raises ``AqcError`` -- there is no CPU fallback.
"""
import atexit
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# AQC_LIB names an alternative build (experiment libraries built in-tree next to this one)
LIB_PATH = os.environ.get("AQC_LIB") or os.path.join(_HERE, "libaqchip.so")

OP_DTYPE = np.dtype(
    [("nq", "<i4"), ("q0", "<i4"), ("q1", "<i4"), ("flags", "<i4"), ("m", "<f8", (32,))], align=True
)
assert OP_DTYPE.itemsize == 272

# every symbol declared in include/aqc_hip.h (the drop-in boundary) and include/aqc_hip_diag.h
# (diagnostics and test hooks)
EXPORTS = (
    "aqc_last_error", "aqc_version", "aqc_init", "aqc_finalize", "aqc_timing_enable",
    "aqc_timing_query", "aqc_timing_reset",
    "aqc_sv_create", "aqc_sv_destroy", "aqc_sv_reset", "aqc_sv_copy", "aqc_sv_apply", "aqc_sv_plan",
    "aqc_sv_amp0", "aqc_sv_z_all", "aqc_sv_get", "aqc_sv_set",
    "aqc_mps_create", "aqc_mps_destroy", "aqc_mps_set_truncation", "aqc_mps_set_vidal",
    "aqc_mps_get_vidal", "aqc_mps_get_dims", "aqc_mps_copy", "aqc_mps_copy_batch", "aqc_mps_apply",
    "aqc_mps_apply_batch", "aqc_mps_apply_sort_batch", "aqc_mps_apply_sort_batch_async", "aqc_mps_apply_batch_async", "aqc_mps_check_batch", "aqc_mps_sort", "aqc_mps_sort_batch", "aqc_mps_overlap_zero",
    "aqc_mps_overlap_zero_batch", "aqc_mps_dot", "aqc_mps_z_all", "aqc_mps_amps_hw1", "aqc_mps_z_all_batch", "aqc_mps_z_sum_batch", "aqc_mps_zero_hw1_batch",
    "aqc_mps_amps_hw1_batch",
    "aqc_pair_grads", "aqc_pair_grads_batch", "aqc_argmax_scaled", "aqc_argmax_scaled_batch", "aqc_mps_jacobi_stats",
    "aqc_mps_set_jacobi_tol", "aqc_mps_set_jacobi_stop", "aqc_mps_set_fused_chain", "aqc_mps_chain_ticks", "aqc_svd_debug",
    "aqc_sv_pair_rdms", "aqc_mps_pair_rdms", "aqc_mps_pair_rdms_batch", "aqc_entanglement_measures",
    "aqc_sv_transition", "aqc_mps_product_fit", "aqc_mps_set_svd_path", "aqc_svd_gram_ticks", "aqc_bj_ticks",
    "aqc_sweep_set_chain_mode", "aqc_stream_join", "aqc_stream_wait", "aqc_svd_gram_stats", "aqc_env_ticks",
    "aqc_comm_unique_id", "aqc_comm_init", "aqc_comm_destroy", "aqc_comm_rank", "aqc_allgather_f64",
    "aqc_allgather_f64_host", "aqc_allreduce_max_f64", "aqc_svd_gram_big_stats", "aqc_svd_gram_big_ticks",
    "aqc_gb_set_spin_limit", "aqc_gb_set_tail", "aqc_gb_set_stages", "aqc_debug_hog", "aqc_pool_stats",
    "aqc_env_fallbacks", "aqc_env_set_single", "aqc_env_set_spin_limit",
)


class AqcError(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None
_initialised_device = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double
_DP = ctypes.POINTER(ctypes.c_double)
_IP = ctypes.POINTER(ctypes.c_int)

_SIGS = {
    "aqc_last_error": ([], ctypes.c_char_p),
    "aqc_version": ([], _I),
    "aqc_init": ([_I], _I),
    "aqc_finalize": ([], _I),
    "aqc_timing_enable": ([_I], _I),
    "aqc_timing_query": ([ctypes.c_char_p, _DP, ctypes.POINTER(ctypes.c_int64), _DP, _DP], _I),
    "aqc_timing_reset": ([], _I),
    "aqc_sv_create": ([_I, ctypes.POINTER(_P)], _I),
    "aqc_sv_destroy": ([_P], _I),
    "aqc_sv_reset": ([_P], _I),
    "aqc_sv_copy": ([_P, _P], _I),
    "aqc_sv_apply": ([_P, _P, _I], _I),
    "aqc_sv_plan": ([_I, _P, _I, _P], _I),
    "aqc_sv_amp0": ([_P, _DP, _DP], _I),
    "aqc_sv_z_all": ([_P, _DP], _I),
    "aqc_sv_get": ([_P, _P], _I),
    "aqc_sv_set": ([_P, _P], _I),
    "aqc_mps_create": ([_I, _I, _D, _I, ctypes.POINTER(_P)], _I),
    "aqc_mps_destroy": ([_P], _I),
    "aqc_mps_set_truncation": ([_P, _D, _I], _I),
    "aqc_mps_set_vidal": ([_P, _P, _P, _P], _I),
    "aqc_mps_get_vidal": ([_P, _P, _P, _P], _I),
    "aqc_mps_get_dims": ([_P, _P], _I),
    "aqc_mps_copy": ([_P, _P], _I),
    "aqc_mps_copy_batch": ([_P, _P, _I], _I),
    "aqc_mps_apply": ([_P, _P, _I], _I),
    "aqc_mps_apply_batch": ([_P, _I, _P, _P], _I),
    "aqc_mps_apply_sort_batch": ([_P, _I, _P, _P], _I),
    "aqc_mps_apply_sort_batch_async": ([_P, _I, _P, _P], _I),
    "aqc_mps_apply_batch_async": ([_P, _I, _P, _P], _I),
    "aqc_mps_check_batch": ([_P, _I], _I),
    "aqc_mps_sort": ([_P], _I),
    "aqc_mps_sort_batch": ([_P, _I], _I),
    "aqc_mps_overlap_zero": ([_P, _DP, _DP], _I),
    "aqc_mps_overlap_zero_batch": ([_P, _I, _P], _I),
    "aqc_mps_dot": ([_P, _P, _DP, _DP], _I),
    "aqc_mps_z_all": ([_P, _P], _I),
    "aqc_mps_amps_hw1": ([_P, _P], _I),
    "aqc_mps_z_all_batch": ([_P, _I, _P], _I),
    "aqc_mps_z_sum_batch": ([_P, _P, _I, _P], _I),
    "aqc_mps_zero_hw1_batch": ([_P, _P, _I, _P, _P], _I),
    "aqc_mps_amps_hw1_batch": ([_P, _I, _P], _I),
    "aqc_pair_grads": ([_P, _P, _P, _I, _P, _P, _P, _I, _P, _I], _I),
    "aqc_pair_grads_batch": ([_P, _I, _P, _P, _I, _P, _P, _P, _I, _P, _I], _I),
    "aqc_argmax_scaled": ([_P, _P, _I, _I, _IP], _I),
    "aqc_argmax_scaled_batch": ([_P, _I, _P, _I, _I, _P], _I),
    "aqc_mps_jacobi_stats": ([_P, _IP], _I),
    "aqc_mps_set_jacobi_tol": ([_D], _I),
    "aqc_mps_set_jacobi_stop": ([_D], _I),
    "aqc_mps_set_fused_chain": ([_I], _I),
    "aqc_mps_chain_ticks": ([_P], _I),
    "aqc_svd_debug": ([_P, _I, _I, _I, _I, _P, _P, _P, _P], _I),
    "aqc_sv_pair_rdms": ([_P, _P, _I, _P], _I),
    "aqc_mps_pair_rdms": ([_P, _P, _I, _P], _I),
    "aqc_mps_pair_rdms_batch": ([_P, _I, _P, _I, _P, _I], _I),
    "aqc_entanglement_measures": ([_P, _I, _I, _P, _I], _I),
    "aqc_sv_transition": ([_P, _P, _I, _P], _I),
    "aqc_mps_product_fit": ([_P, _P, _I, _I, _I, _D, _DP, _IP], _I),
    "aqc_mps_set_svd_path": ([_I, _I], _I),
    "aqc_svd_gram_ticks": ([_P], _I),
    "aqc_bj_ticks": ([_P], _I),
    "aqc_sweep_set_chain_mode": ([_I], _I),
    "aqc_stream_join": ([_P], _I),
    "aqc_stream_wait": ([_P], _I),
    "aqc_svd_gram_stats": ([_P], _I),
    "aqc_env_ticks": ([_P], _I),
    "aqc_comm_unique_id": ([ctypes.c_char_p], _I),
    "aqc_comm_init": ([ctypes.c_char_p, _I, _I, ctypes.POINTER(_P)], _I),
    "aqc_comm_destroy": ([_P], _I),
    "aqc_comm_rank": ([_P, _IP, _IP], _I),
    "aqc_allgather_f64": ([_P, _P, _P, ctypes.c_size_t], _I),
    "aqc_allgather_f64_host": ([_P, _P, _P, ctypes.c_size_t], _I),
    "aqc_allreduce_max_f64": ([_P, _DP], _I),
    "aqc_svd_gram_big_stats": ([_P], _I),
    "aqc_svd_gram_big_ticks": ([_P], _I),
    "aqc_gb_set_spin_limit": ([_D], _I),
    "aqc_env_fallbacks": ([ctypes.POINTER(ctypes.c_longlong)], _I),
    "aqc_env_set_single": ([_I], _I),
    "aqc_env_set_spin_limit": ([_D], _I),
    "aqc_gb_set_tail": ([_I], _I),
    "aqc_gb_set_stages": ([_I], _I),
    "aqc_debug_hog": ([_I, _D], _I),
    "aqc_pool_stats": ([_P], _I),
}


def load(path=LIB_PATH):
    """Load libaqchip.so (does not touch the GPU)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise AqcError(
                f"HIP library not found at {path}; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        # PyTorch first when it is installed: libaqchip and torch both need a libamdhip64.so.7 (the
        # ROCm under /opt/rocm, and torch's bundled one); the first loaded serves the process.  With
        # libaqchip first, torch then ran on the other runtime and found no GPU ("No HIP GPUs are
        # available"); with torch first both share torch's -- the configuration the bench and the
        # GPU suite always ran (they import torch before any library call).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(path)
        missing = []
        for name, (args, res) in _SIGS.items():
            f = getattr(lib, name, None)
            if f is None:
                missing.append(name)
                continue
            f.argtypes = args
            f.restype = res
        # an experiment build (AQC_LIB, tools/ab_libs.sh) may predate newer entry points
        if missing and not os.environ.get("AQC_LIB"):
            raise AqcError(f"{path} lacks entry points {missing}: rebuild it (make -C adaptaqc_amd/csrc)")
        _lib = lib
        return lib


def check(rc):
    if rc != 0:
        msg = load().aqc_last_error().decode(errors="replace")
        raise AqcError(f"libaqchip error {rc}: {msg}")


def device_index():
    """Device for this process: LOCAL_RANK when launched one process per GPU."""
    return int(os.environ.get("AQC_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def lib():
    """The loaded library with this process's device selected (raises without a GPU)."""
    global _initialised_device
    l = load()
    dev = device_index()
    if _initialised_device != dev:
        check(l.aqc_init(dev))
        if _initialised_device is None:
            # drain the device and release the library's lazily created streams / events / buffer
            # sets before the interpreter (and the HIP runtime) tear down
            atexit.register(_finalize)
        _initialised_device = dev
    return l


def _finalize():
    if _lib is not None:
        _lib.aqc_finalize()


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def dptr(a):
    return a.ctypes.data_as(_DP)


def ops_array(ops):
    """[(matrix (2x2 or 4x4 complex), qubits tuple)] -> contiguous aqc_op_t array (filled per
    field over all ops at once: per-op structured-array stores cost ~6 us an op)."""
    n = len(ops)
    arr = np.zeros(n, dtype=OP_DTYPE)
    if n == 0:
        return arr
    nq = np.fromiter((len(q) for _, q in ops), dtype=np.int32, count=n)
    if not np.all((nq == 1) | (nq == 2)):
        raise ValueError("ops_array: only 1- and 2-qubit ops")
    arr["nq"] = nq
    arr["q0"] = np.fromiter((q[0] for _, q in ops), dtype=np.int32, count=n)
    arr["q1"] = np.fromiter((q[1] if len(q) == 2 else 0 for _, q in ops), dtype=np.int32, count=n)
    m = arr["m"]
    for k, width in ((1, 4), (2, 16)):
        idx = np.flatnonzero(nq == k)
        if idx.size:
            mats = np.asarray([ops[i][0] for i in idx], dtype=np.complex128).reshape(idx.size, width)
            m[idx, : 2 * width] = mats.view(np.float64)
    return arr


def timing_enable(on=True):
    check(load().aqc_timing_enable(1 if on else 0))


def timing_reset():
    check(load().aqc_timing_reset())


def timing_query(name):
    ms, b, f = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    n = ctypes.c_int64()
    check(load().aqc_timing_query(name.encode(), ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b), ctypes.byref(f)))
    return {"ms": ms.value, "launches": n.value, "bytes": b.value, "flops": f.value}


def gram_stats():
    """Gram-path counters since the last call (aqc_svd_gram_stats): calls, taken, declined by
    shape, declined at the kept-count decision / eigenvalue floor / failed certificate,
    rank-deficiency certificates run and passed."""
    out = np.zeros(6)
    check(load().aqc_svd_gram_stats(ptr(out)))
    return {"calls": int(out[0]), "taken": int(out[1]), "declined_shape": int(out[2]),
            "declined_floor": int(out[3]), "certificates": int(out[4]), "certified": int(out[5])}


def gram_big_stats():
    """Counters of the multi-workgroup Gram path for 2 chi > 128 since the last call
    (aqc_svd_gram_big_stats): calls, taken, declined, declined at the eigenvalue floor, exchange
    timeouts."""
    out = np.zeros(8)
    check(load().aqc_svd_gram_big_stats(ptr(out)))
    return {"calls": int(out[0]), "taken": int(out[1]), "declined": int(out[2]),
            "declined_floor": int(out[3]), "timeouts": int(out[4]), "certificates": int(out[5]),
            "certified": int(out[6]), "declined_certificate": int(out[7])}
