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

"""Shot-sampling backend: OUT OF SCOPE.

Present only so that ``python_default_backends.QASM_SIM`` exists like in the reference; any
use raises ``NotImplementedError`` (the reference's error convention for unsupported paths).
"""
from .aqc_backend import AQCBackend


class QiskitSamplingBackend(AQCBackend):
    def __init__(self, simulator=None):
        self.simulator = simulator

    def _unsupported(self, *_):
        raise NotImplementedError("shot-sampling (qasm_simulator) backend is not part of the MI355X hot path")

    evaluate_global_cost = _unsupported
    evaluate_local_cost = _unsupported
    evaluate_circuit = _unsupported
    measure_qubit_expectation_values = _unsupported
