"""Reference-side binding (adaptaqc_amd.reference_binding) on CPU: ABC registration so the
reference's isinstance switches hold (approximate_compiler.py:113, utilityfunctions.py:122-130),
the rebinding of its simulator entry points, and qiskit-shaped circuits flattened to device ops
(no GPU call)."""
import numpy as np

from qiskit_fakes import from_ir, installed_fake_reference


def test_install_registers_and_patches():
    from adaptaqc_amd import reference_binding as rb
    from adaptaqc_amd.backends import AerMPSBackend, AerSVBackend
    from adaptaqc_amd.mps_operations import mps_from_circuit
    from adaptaqc_amd.utils.gradients import general_grad_of_pairs

    with installed_fake_reference() as mods:
        done = rb.install(import_missing=False)
        assert not done["missing"], done
        RefMPS = mods["adaptaqc.backends.aer_mps_backend"].AerMPSBackend
        RefSV = mods["adaptaqc.backends.aer_sv_backend"].AerSVBackend
        RefBase = mods["adaptaqc.backends.aqc_backend"].AQCBackend
        mps_b, sv_b = AerMPSBackend(), AerSVBackend()
        assert isinstance(mps_b, RefMPS) and isinstance(mps_b, RefBase)
        assert isinstance(sv_b, RefSV) and not isinstance(sv_b, RefMPS)
        assert not isinstance(mps_b, RefSV)
        assert mods["adaptaqc.compilers.approximate_compiler"].mps_from_circuit is mps_from_circuit
        assert mods["aqc_research.mps_operations"].mps_from_circuit is mps_from_circuit
        assert mods["adaptaqc.utils.gradients"].general_grad_of_pairs is general_grad_of_pairs
        # the ISL sweep's per-pair entry points and the batched compiler method
        from adaptaqc_amd.mps_operations import partial_trace as mps_pt
        from adaptaqc_amd.utils.entanglement_measures import partial_trace as sv_pt

        assert mods["aqc_research.mps_operations"].partial_trace is mps_pt
        assert mods["adaptaqc.utils.entanglement_measures"].partial_trace is sv_pt
        AC = mods["adaptaqc.compilers.adapt.adapt_compiler"].AdaptCompiler
        wrapped = AC._get_all_qubit_pair_entanglement_measures
        assert wrapped.__wrapped__.__qualname__.endswith("AdaptCompiler._get_all_qubit_pair_entanglement_measures")
        # the SV simulator handle has the run() the reference's run_circuit_without_transpilation calls
        assert callable(getattr(sv_b.simulator, "run", None))
        # the reference reads these options from backend.simulator (approximate_compiler.py:224-226)
        assert mps_b.simulator.options.matrix_product_state_truncation_threshold == 1e-16
    # uninstalled: the fake modules are gone again, the class method restored
    assert not hasattr(AC._get_all_qubit_pair_entanglement_measures, "__wrapped__")
    import sys

    assert "aqc_research.mps_operations" not in sys.modules


def test_install_without_reference_changes_nothing():
    from adaptaqc_amd import reference_binding as rb

    done = rb.install(import_missing=True)  # no adaptaqc / aqc_research importable here
    assert not done["patched"] and not done["registered"]
    assert len(done["missing"]) == len(rb.PATCHES) + len(rb.REGISTRATIONS)


def test_qiskit_shaped_circuit_flattens_like_ir():
    from adaptaqc_amd.circuit import QuantumCircuit, device_ops, qasm2_dumps

    qc = QuantumCircuit(4)
    qc.rx(0.3, 0)
    qc.cx(0, 3)
    qc.ry(-1.1, 2)
    qc.rzz(0.7, 1, 2)
    qc.unitary(np.diag([1, 1j]), [3])
    qc.h(1)
    a = device_ops(qc)
    b = device_ops(from_ir(qc))
    assert len(a) == len(b) == 6
    for (ma, qa), (mb, qb) in zip(a, b):
        assert qa == qb
        np.testing.assert_allclose(ma, mb)
    text = qasm2_dumps(QuantumCircuit(2).rx(0.5, 0).cx(0, 1))
    assert "rx(0.5) q[0];" in text and "cx q[0],q[1];" in text


def test_isl_wrapper_defers_to_reference_for_other_backends():
    """With a backend that is not this package's, the wrapped ISL method runs the reference's own
    loop (here the fake's restatement, which ends in the reference's tomography branch)."""
    import pytest

    from adaptaqc_amd import reference_binding as rb

    with installed_fake_reference() as mods:
        rb.install(import_missing=False)
        AC = mods["adaptaqc.compilers.adapt.adapt_compiler"].AdaptCompiler

        class OtherBackend:
            pass

        comp = AC(None, OtherBackend(), [(0, 1)])
        with pytest.raises(RuntimeError, match="tomography"):
            comp._get_all_qubit_pair_entanglement_measures()
