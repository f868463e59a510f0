"""RCCL collectives through libaqchip's C ABI (``aqc_comm_*``, include/aqc_hip.h), for callers
that shard the candidate sweep without torch.distributed.

The sweep's one exchange: every rank scores its share of the coupling-map pairs,
the scores are all-gathered over xGMI, and every rank takes the same arg-max
(adapt_compiler.py:832-856).  The 128-byte unique id is made on one rank and handed to the others
by the caller (``RcclComm.unique_id()``; e.g. a shared file or the launcher's environment).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

UNIQUE_ID_BYTES = 128


class RcclComm:
    """One RCCL communicator on this process's device (see _lib.device_index)."""

    def __init__(self, unique_id: bytes, rank: int, world: int):
        if len(unique_id) != UNIQUE_ID_BYTES:
            raise ValueError("unique_id must be the 128 bytes of RcclComm.unique_id()")
        self._l = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(self._l.aqc_comm_init(unique_id, int(rank), int(world), ctypes.byref(h)))
        self.h = h
        self.rank, self.world = int(rank), int(world)

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
        _lib.check(_lib.lib().aqc_comm_unique_id(buf))
        return buf.raw

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self._l.aqc_comm_destroy(self.h)
            self.h = None

    __del__ = close

    def allgather(self, local) -> np.ndarray:
        """Host all-gather of float64 scores: (world, len(local)), rank order."""
        x = np.ascontiguousarray(np.asarray(local, dtype=np.float64).reshape(-1))
        out = np.zeros((self.world, len(x)))
        if len(x):
            _lib.check(self._l.aqc_allgather_f64_host(self.h, _lib.ptr(x), _lib.ptr(out), len(x)))
        return out

    def allgather_device(self, send_ptr: int, recv_ptr: int, count: int) -> None:
        """Device all-gather on the library's stream (queued; ordered after a device-output sweep)."""
        _lib.check(self._l.aqc_allgather_f64(self.h, ctypes.c_void_p(int(send_ptr)), ctypes.c_void_p(int(recv_ptr)),
                                             int(count)))

    def allreduce_max(self, value: float) -> float:
        v = ctypes.c_double(float(value))
        _lib.check(self._l.aqc_allreduce_max_f64(self.h, ctypes.byref(v)))
        return v.value


__all__ = ["RcclComm", "UNIQUE_ID_BYTES"]
