"""Statevectors returned by the SV backend and by ``SVSimulator.run(...).result()``.

``Statevector`` holds host data (Aer returns host data too).  ``DeviceStatevector`` keeps the
amplitudes resident in HBM and copies them to the host only when ``.data`` is read; the drop-in
``partial_trace`` (reference entanglement_measures.py:325-340, called with the result of
``run_circuit_without_transpilation(..., return_statevector=True)``, :71-75) computes its 4x4
RDMs on the device copy and never pulls the 2^n amplitudes over PCIe.
"""
import numpy as np


class Statevector:
    def __init__(self, data):
        self.data = np.asarray(data, dtype=np.complex128)
        self.num_qubits = int(round(np.log2(len(self.data))))

    def __getitem__(self, i):
        return self.data[i]

    def __len__(self):
        return len(self.data)

    def __array__(self, dtype=None, copy=None):
        d = self.data
        return d if dtype is None else d.astype(dtype)

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


class DeviceStatevector(Statevector):
    """A statevector that lives on the device (an owned ``DeviceSV`` snapshot).

    ``data`` is fetched lazily (and once); ``pair_rdm`` runs ``aqc_sv_pair_rdms`` on the device
    copy, memoised per pair."""

    def __init__(self, dev):
        self._dev = dev
        self._host = None
        self._rdms = {}
        self.num_qubits = dev.n

    @property
    def data(self):
        if self._host is None:
            self._host = self._dev.get()
        return self._host

    def __len__(self):
        return 1 << self.num_qubits

    @property
    def device(self):
        return self._dev

    def pair_rdm(self, a, b):
        key = (int(a), int(b))
        if key not in self._rdms:
            self._rdms[key] = self._dev.pair_rdms([key])[0]
        return self._rdms[key]

    def pair_rdms(self, pairs):
        return self._dev.pair_rdms(pairs)
