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

"""Pairwise entanglement measures on MI355X: mirror of adaptaqc/utils/entanglement_measures.py.

``calculate_entanglement_measure`` (reference :39-98) keeps its signature and dispatch: the
4x4 reduced density matrix comes from the device statevector (aqc_sv_pair_rdms, reference
partial_trace :326-340) or the device MPS (aqc_mps_pair_rdms, aqc_research partial_trace), and
the measure from aqc_entanglement_measures (concurrence :278-296, EoF :263-275, negativity and
log-negativity :299-306).  ``pair_entanglement_measures`` is the batched form the compiler's ISL
sweep uses (adapt_compiler.py:955-976): one device state, every pair's RDM in one launch chain,
every measure in one launch.

Not on this path (raise NotImplementedError): the observable lower bound (:101-242, needs shot
sampling) and quantum state tomography (:101-136).
"""
import itertools
import logging

import numpy as np

from ..device import DeviceSV, entanglement_measures

logger = logging.getLogger(__name__)

EM_OBSERVABLE_CONCURRENCE_LOWER_BOUND = "EM_OBSERVABLE_CONCURRENCE_LOWER_BOUND"
EM_TOMOGRAPHY_EOF = "EM_TOMOGRAPHY_EOF"
EM_TOMOGRAPHY_CONCURRENCE = "EM_TOMOGRAPHY_CONCURRENCE"
EM_TOMOGRAPHY_NEGATIVITY = "EM_TOMOGRAPHY_NEGATIVITY"
EM_TOMOGRAPHY_LOG_NEGATIVITY = "EM_TOMOGRAPHY_LOG_NEGATIVITY"

_CODES = {
    EM_TOMOGRAPHY_CONCURRENCE: "concurrence",
    EM_TOMOGRAPHY_EOF: "eof",
    EM_TOMOGRAPHY_NEGATIVITY: "negativity",
    EM_TOMOGRAPHY_LOG_NEGATIVITY: "log_negativity",
}


def _kind(backend):
    from ..backends.aer_mps_backend import AerMPSBackend
    from ..backends.aer_sv_backend import AerSVBackend

    if isinstance(backend, AerMPSBackend):
        return "mps"
    if isinstance(backend, AerSVBackend):
        return "sv"
    return None


def _measure_name(method):
    if method == EM_OBSERVABLE_CONCURRENCE_LOWER_BOUND:
        raise NotImplementedError("the observable concurrence lower bound needs shot sampling, which is "
                                  "outside the MI355X overlap/gradient path")
    if method not in _CODES:
        raise ValueError("Invalid entanglement measure method")
    return _CODES[method]


def calculate_entanglement_measure(method, circuit, qubit_1, qubit_2, backend, backend_options=None,
                                   execute_kwargs=None, mps=None):
    """Entanglement between two qubits of the state prepared by ``circuit`` (reference :39-98)."""
    name = _measure_name(method)
    kind = _kind(backend)
    if kind == "sv":
        from ..circuit import device_ops_array

        st = DeviceSV(circuit.num_qubits)
        st.apply(device_ops_array(circuit))
        rho = st.pair_rdms([(qubit_1, qubit_2)])
    elif kind == "mps":
        from ..device import DeviceMPS
        from ..mps_operations import _as_device

        if mps is None:
            raise ValueError("the MPS backend needs the circuit's MPS (mps=...)")
        dev = mps if isinstance(mps, DeviceMPS) else _as_device(mps, True)
        rho = dev.pair_rdms([(qubit_1, qubit_2)])
    else:
        raise NotImplementedError("quantum state tomography (shot-sampling backends) is outside the MI355X path")
    return float(entanglement_measures(rho, name)[0])


def pair_entanglement_measures(method, compiler, pairs, comm=None):
    """Batched ISL sweep: the measure for every pair of ``pairs`` on the compiler's current state.
    With ``comm`` (sharding.sharded_pair_scores) each rank computes the RDMs and measures of the
    pairs whose first qubit it owns -- its share of the pair-RDM chains -- and one all-gather gives
    every rank the whole list."""
    from ..sharding import sharded_pair_scores

    name = _measure_name(method)
    if not pairs:
        return []

    def score(local):
        rdms = compiler.backend.pair_rdms(compiler, local)
        return [float(x) for x in entanglement_measures(rdms, name)]

    return sharded_pair_scores(score, pairs, compiler.full_circuit.num_qubits, comm)


# -- measures of a single 4x4 density matrix (device kernels) -----------------------------------
def concurrence(rho):
    """Mixed-state concurrence (PhysRevLett.80.2245), reference :278-296."""
    return float(entanglement_measures(np.asarray(rho), "concurrence")[0])


def eof(rho):
    """Entanglement of formation, reference :263-275."""
    return float(entanglement_measures(np.asarray(rho), "eof")[0])


def negativity(rho):
    return float(entanglement_measures(np.asarray(rho), "negativity")[0])


def log_negativity(rho):
    return float(entanglement_measures(np.asarray(rho), "log_negativity")[0])


def partial_trace(statevector, a, b):
    """4x4 RDM of qubits a, b of a statevector (reference :326-340), computed on the device.  A
    device-resident statevector (``SVSimulator.run(...).result().get_statevector()``) is traced
    in place; host data is uploaded first."""
    from ..statevector import DeviceStatevector

    if isinstance(statevector, DeviceStatevector):
        return statevector.pair_rdm(a, b).copy()
    psi = np.asarray(getattr(statevector, "data", statevector), dtype=np.complex128)
    n = int(round(np.log2(len(psi))))
    st = DeviceSV(n)
    st.set(psi)
    return st.pair_rdms([(a, b)])[0]


def partial_transpose(density_matrix, wrt=1):
    """Index permutation of reference :343-356 (host-side data movement)."""
    tp = np.array(density_matrix, copy=True)
    for ja, ka, jb, kb in itertools.product(range(2), range(2), range(2), range(2)):
        if wrt == 1:
            tp[ka * 2 + jb][ja * 2 + kb] = density_matrix[ja * 2 + jb][ka * 2 + kb]
        elif wrt == 2:
            tp[ja * 2 + kb][ka * 2 + jb] = density_matrix[ja * 2 + jb][ka * 2 + kb]
    return tp


def measure_concurrence_lower_bound(circuit, qubit_1, qubit_2, backend, backend_options=None,
                                    execute_kwargs=None):
    raise NotImplementedError("the observable concurrence lower bound needs shot sampling")


def perform_quantum_tomography(circuit, qubit_1, qubit_2, backend, backend_options=None, execute_kwargs=None):
    raise NotImplementedError("quantum state tomography needs a shot-sampling backend")
