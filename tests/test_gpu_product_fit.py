"""starting_circuit="tenpy_product_state" on the device (aqc_mps_product_fit) against the oracle's
restatement (oracle/product_fit.py): same fidelity and sweeps, the same site vectors up to phase,
and the paper's general_gradient configuration (examples/advanced_mps_example.py:41-58) end to end.
Parity with tenpy itself is unpinned (tenpy is absent)."""
import numpy as np
import pytest

import bench
from conftest import to_circuit
from oracle import mps as M
from oracle import product_fit as PF

pytestmark = pytest.mark.gpu


def _ops(n, seed, layers=3):
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(layers):
        for q in range(n):
            ops.append(("ry", (q,), (float(rng.uniform(-1, 1)),)))
            ops.append(("rz", (q,), (float(rng.uniform(-1, 1)),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    return ops


@pytest.mark.parametrize("case", ["circuit12", "bench50"])
def test_product_fit_vs_oracle(case):
    from adaptaqc_amd.device import DeviceMPS

    if case == "circuit12":
        n = 12
        st = M.run_circuit(n, _ops(n, 5))
        aer = st.to_aer()
        cap = 64
    else:
        n = 50
        aer = bench.near_product_mps(n, 64, 1000)
        st = M.MPS.from_aer(aer)
        cap = 64
    d = DeviceMPS(n, cap)
    d.load_aer(aer)
    s_dev, f_dev, sw_dev = d.product_fit(None, 10, 50, 1e-12)
    s_or, f_or, sw_or = PF.product_fit(st.preprocessed(), PF.initial_guess(st.g), 10, 50, 1e-12)
    assert abs(f_dev - f_or) < 1e-10 * max(1.0, f_or)
    assert sw_dev == sw_or
    for a, b in zip(s_dev, s_or):  # equal up to a phase per site
        assert abs(abs(np.vdot(a, b)) - 1.0) < 1e-8
    assert abs(abs(PF.overlap(st.preprocessed(), list(s_dev))) ** 2 - f_dev) < 1e-10
    if case == "bench50":
        assert f_dev > 0.1  # the near-product component is found


def test_tenpy_product_state_starting_circuit():
    """The starting circuit prepares the fitted product state: its overlap with the target equals
    the fit's fidelity, and every gate is a single-qubit rotation."""
    from adaptaqc_amd.backends import AerMPSBackend
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig
    from adaptaqc_amd.device import DeviceMPS
    from adaptaqc_amd.mps_operations import device_mps_from_circuit

    n = 10
    qc = to_circuit(n, _ops(n, 9))
    comp = AdaptCompiler(qc, backend=AerMPSBackend(), adapt_config=AdaptConfig(method="general_gradient"),
                         starting_circuit="tenpy_product_state")
    sc = comp.starting_circuit
    assert all(len(i.qubits) == 1 and i.operation.name in ("rx", "ry", "rz") for i in sc.data)
    target = device_mps_from_circuit(qc.copy())
    start = device_mps_from_circuit(sc.copy())
    assert abs(abs(start.dot(target)) ** 2 - comp.starting_state_fidelity) < 1e-10
    assert comp.starting_state_fidelity > 0.1


def test_paper_configuration_end_to_end():
    """examples/advanced_mps_example.py:41-58 at small size: MPS backend, general_gradient pair
    selection, identity_resolvable layers, rotosolve every 10 layers, tenpy_product_state start."""
    from adaptaqc_amd.backends import AerMPSBackend, mps_sim_with_args
    from adaptaqc_amd.compilers import AdaptCompiler, AdaptConfig
    from adaptaqc_amd.utils.ansatzes import identity_resolvable
    from oracle import sv as osv

    n = 6
    ops = _ops(n, 13, layers=2)
    qc = to_circuit(n, ops)
    cfg = AdaptConfig(method="general_gradient", rotosolve_frequency=10, max_layers_to_modify=100)
    comp = AdaptCompiler(qc, backend=AerMPSBackend(mps_sim_with_args(max_chi=16)), adapt_config=cfg,
                         custom_layer_2q_gate=identity_resolvable(), starting_circuit="tenpy_product_state")
    res = comp.compile()
    assert res.overlap > 1 - 1e-2
    got = osv.simulate(n, [(i.operation.name, i.qubits, tuple(i.operation.params)) for i in res.circuit.data])
    assert abs(np.vdot(osv.simulate(n, ops), got)) ** 2 > 1 - 1e-2
    assert all(m == "general_gradient" for m in res.method_history)
