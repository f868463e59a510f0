"""adaptaqc_amd -- MI355X-native engine for ADAPT-AQC's overlap / gradient hot path.

Drop-in for the reference's ``adaptaqc.backends`` plugin surface (AerSVBackend /
AerMPSBackend) with the arithmetic in hand-written HIP kernels (libaqchip.so, gfx950).
"""
import os

# qiskit sets this on import; the reference reads it without a default (aer_sv_backend.py:39).
os.environ.setdefault("QISKIT_IN_PARALLEL", "FALSE")

from .circuit import QuantumCircuit  # noqa: E402,F401

__version__ = "0.1.0"
