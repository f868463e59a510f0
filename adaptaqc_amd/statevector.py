"""Host statevector returned by ``AerSVBackend.evaluate_circuit`` (Aer returns host data too)."""
import numpy as np


class Statevector:
    def __init__(self, data):
        self.data = np.asarray(data, dtype=np.complex128)
        self.num_qubits = int(round(np.log2(len(self.data))))

    def __getitem__(self, i):
        return self.data[i]

    def __len__(self):
        return len(self.data)

    def probabilities(self, qargs=None):
        """Marginal probabilities over ``qargs`` (little-endian), like qiskit's Statevector."""
        p = np.abs(self.data) ** 2
        n = self.num_qubits
        if qargs is None:
            return p
        t = p.reshape([2] * n)
        keep = [n - 1 - q for q in qargs]
        drop = tuple(a for a in range(n) if a not in keep)
        m = t.sum(axis=drop)
        # remaining axes are in descending-qubit order of `keep` sorted; reorder to qargs little-endian
        order = sorted(keep)
        m = np.moveaxis(m, [order.index(a) for a in keep], list(range(len(keep)))[::-1])
        return m.reshape(-1)
