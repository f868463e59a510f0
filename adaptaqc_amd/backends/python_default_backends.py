"""Shared backend instances (reference adaptaqc/backends/python_default_backends.py:17-19).

Constructing them does not touch the GPU; device state is created on first use.
"""
from .aer_mps_backend import AerMPSBackend
from .aer_sv_backend import AerSVBackend
from .qiskit_sampling_backend import QiskitSamplingBackend

QASM_SIM = QiskitSamplingBackend()
SV_SIM = AerSVBackend()
MPS_SIM = AerMPSBackend()
