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

"""Backend plugin surface (reference adaptaqc/backends/aqc_backend.py:14-29)."""
import abc


class AQCBackend(abc.ABC):
    @abc.abstractmethod
    def evaluate_global_cost(self, compiler):
        pass

    @abc.abstractmethod
    def evaluate_local_cost(self, compiler):
        pass

    @abc.abstractmethod
    def evaluate_circuit(self, compiler):
        pass

    @abc.abstractmethod
    def measure_qubit_expectation_values(self, compiler):
        pass
