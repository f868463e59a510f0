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
