# (C) Copyright IBM 2025.
#
# This code is licensed under the Apache License, Version 2.0. You may
# obtain a copy of this license in the LICENSE.txt file in the root directory
# of this source tree or at http://www.apache.org/licenses/LICENSE-2.0.
#
# Any modifications or derivative works of this code must retain this
# copyright notice, and modified files need to carry a notice indicating
# that they have been altered from the originals.
#
# Modified for adaptaqc_amd: this file restates the reference file named in its docstring
# (qiskit-community/adapt-aqc) on top of the MI355X engine (libaqchip); it has been altered
# from the original.

"""Shared backend instances (reference adaptaqc/backends/python_default_backends.py:17-19).

Constructing them does not touch the GPU; device state is created on first use.
"""
from .aer_mps_backend import AerMPSBackend
from .aer_sv_backend import AerSVBackend
from .qiskit_sampling_backend import QiskitSamplingBackend

QASM_SIM = QiskitSamplingBackend()
SV_SIM = AerSVBackend()
MPS_SIM = AerMPSBackend()
