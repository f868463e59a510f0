"""Statevector parity on MI355X vs the oracle (tolerance 1e-10 on overlaps, per north_star)."""
import numpy as np
import pytest

from conftest import FakeCompiler, golden_ops, to_circuit
from oracle import sv as osv

pytestmark = pytest.mark.gpu
TOL = 1e-10


def brickwork(n, depth, seed):
    rng = np.random.default_rng(seed)
    ops = []
    for layer in range(depth):
        for q in range(n):
            ops.append((["rx", "ry", "rz"][rng.integers(3)], (q,), (rng.uniform(-np.pi, np.pi),)))
        for q in range(layer % 2, n - 1, 2):
            ops.append(("cx", (q, q + 1), ()))
    return ops


def test_golden_circuits_statevector(goldens):
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceSV

    for seed in range(3):
        ops = golden_ops(goldens, seed)
        qc = to_circuit(8, ops)
        d = DeviceSV(8)
        d.apply(device_ops(qc))
        np.testing.assert_allclose(d.get(), goldens[f"circ{seed}_sv"], atol=1e-12)


@pytest.mark.parametrize("seed", [0, 1])
def test_20_qubit_brickwork_global_cost_and_z(seed):
    """Config 2: 20-qubit random circuit, overlap vs oracle within 1e-10."""
    n = 20
    ops = brickwork(n, 8, seed)
    ops += [("cx", (0, 19), ()), ("cz", (13, 2), ()), ("swap", (5, 17), ())]
    psi = osv.simulate(n, ops)
    from adaptaqc_amd.backends import AerSVBackend

    be = AerSVBackend()
    comp = FakeCompiler(to_circuit(n, ops))
    assert abs(be.evaluate_global_cost(comp) - osv.global_cost(psi)) < TOL
    z = be.measure_qubit_expectation_values(comp)
    np.testing.assert_allclose(z, osv.z_expectations(psi, n), atol=1e-10)
    st = be.evaluate_circuit(comp)
    assert abs(st[0] - psi[0]) < TOL
    np.testing.assert_allclose(st.data, psi, atol=1e-12)


def test_reference_cost_table():
    """test_approximate_compiler.py:114-150 exact costs for |0000>, Neel, GHZ, |++++>."""
    from adaptaqc_amd.backends import AerSVBackend
    from adaptaqc_amd.circuit import QuantumCircuit

    zero = QuantumCircuit(4)
    neel = QuantumCircuit(4)
    neel.x([0, 2])
    ghz = QuantumCircuit(4)
    ghz.h(0)
    for i in range(3):
        ghz.cx(0, i + 1)
    had = QuantumCircuit(4)
    had.h([0, 1, 2, 3])
    be = AerSVBackend()
    got = []
    for c in (zero, neel, ghz, had):
        comp = FakeCompiler(c)
        got += [be.evaluate_global_cost(comp), be.evaluate_local_cost(comp)]
    np.testing.assert_allclose(got, [0, 0, 1, 0.5, 0.5, 0.5, 15 / 16, 0.5], atol=1e-12)


def test_sigma_z_x_h_known_answer():
    """test_utilityfunctions.py:86-95: <Z> = [-1, 0, 1] for x(0), h(1)."""
    from adaptaqc_amd.backends import AerSVBackend
    from adaptaqc_amd.circuit import QuantumCircuit

    qc = QuantumCircuit(3)
    qc.x(0)
    qc.h(1)
    z = AerSVBackend().measure_qubit_expectation_values(FakeCompiler(qc))
    np.testing.assert_array_almost_equal(z, [-1.0, 0.0, 1.0], decimal=15)


def test_ccx_readme_circuit():
    """examples/readme_example.py:14-19 circuit (ccx unrolled on the host)."""
    from adaptaqc_amd.circuit import QuantumCircuit, device_ops
    from adaptaqc_amd.device import DeviceSV

    qc = QuantumCircuit(3)
    qc.rx(1.23, 0)
    qc.cx(0, 1)
    qc.ry(2.5, 1)
    qc.rx(-1.6, 2)
    qc.ccx(2, 1, 0)
    ops = [("rx", (0,), (1.23,)), ("cx", (0, 1), ()), ("ry", (1,), (2.5,)), ("rx", (2,), (-1.6,)), ("ccx", (2, 1, 0), ())]
    d = DeviceSV(3)
    d.apply(device_ops(qc))
    np.testing.assert_allclose(d.get(), osv.simulate(3, ops), atol=1e-12)


def test_soften_raises_on_sv():
    from adaptaqc_amd.backends import AerSVBackend
    from adaptaqc_amd.circuit import QuantumCircuit

    with pytest.raises(NotImplementedError):
        AerSVBackend().evaluate_global_cost(FakeCompiler(QuantumCircuit(2), soften=True))


def test_small_and_segment_edge_sizes():
    """n below, at and above the 10-bit tile; long gate lists spanning many segments."""
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceSV

    for n in (1, 2, 9, 10, 11, 14):
        ops = brickwork(n, 5, n) if n > 1 else [("rx", (0,), (0.3,)), ("rz", (0,), (1.1,))]
        if n >= 4:
            ops += [("cx", (n - 1, 0), ()), ("cz", (1, n - 2), ())]
        d = DeviceSV(n)
        d.apply(device_ops(to_circuit(n, ops)))
        np.testing.assert_allclose(d.get(), osv.simulate(n, ops), atol=1e-12, err_msg=f"n={n}")


def test_gate_fusion_patterns():
    """Host fusion (1q into 2q, repeated and reversed pairs, pending 1q on both sides) is exact."""
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceSV

    rng = np.random.default_rng(17)
    for n in (3, 6, 12):
        ops = []
        for _ in range(120):
            k = rng.integers(6)
            a, b = (int(x) for x in rng.choice(n, 2, replace=False))
            if k < 3:
                ops.append((["rx", "ry", "rz"][k], (a,), (rng.uniform(-np.pi, np.pi),)))
            elif k == 3:
                ops.append(("cx", (a, b), ()))
            elif k == 4:
                ops += [("cx", (a, b), ()), ("cx", (b, a), ()), ("rz", (b,), (0.4,)), ("cz", (a, b), ())]
            else:
                ops += [("h", (a,), ()), ("swap", (a, b), ()), ("ry", (a,), (1.3,))]
        d = DeviceSV(n)
        d.apply(device_ops(to_circuit(n, ops)))
        np.testing.assert_allclose(d.get(), osv.simulate(n, ops), atol=1e-12, err_msg=f"n={n}")


def test_register_tile_path_vs_oracle_and_lds_kernel(monkeypatch):
    """n >= 14 runs the register-resident tile kernel (gates grouped into 4-bit phases):
    random 1q/2q gates incl. fusion patterns, long-range pairs and reversed orders, against the
    oracle and against the per-gate LDS kernel (AQC_SV_TILE=lds)."""
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceSV

    rng = np.random.default_rng(23)
    for n in (14, 15, 17):
        ops = brickwork(n, 4, n)
        for _ in range(150):
            k = rng.integers(6)
            a, b = (int(x) for x in rng.choice(n, 2, replace=False))
            if k < 3:
                ops.append((["rx", "ry", "rz"][k], (a,), (rng.uniform(-np.pi, np.pi),)))
            elif k == 3:
                ops.append(("cx", (a, b), ()))
            elif k == 4:
                ops += [("cx", (a, b), ()), ("cx", (b, a), ()), ("rz", (b,), (0.4,)), ("cz", (a, b), ())]
            else:
                ops += [("h", (a,), ()), ("swap", (a, b), ()), ("ry", (a,), (1.3,))]
        dops = device_ops(to_circuit(n, ops))
        d = DeviceSV(n)
        d.apply(dops)
        got = d.get()
        np.testing.assert_allclose(got, osv.simulate(n, ops), atol=1e-12, err_msg=f"n={n}")
        monkeypatch.setenv("AQC_SV_TILE", "lds")
        d2 = DeviceSV(n)
        monkeypatch.delenv("AQC_SV_TILE")
        d2.apply(dops)
        np.testing.assert_allclose(got, d2.get(), atol=1e-13, err_msg=f"n={n} (lds kernel)")


def test_config2_exact_workload_vs_oracle_goldens():
    """BASELINE config 2 exactly as tools/configs_bench.py times it -- 20 qubits,
    brickwork depth 20, seeds 0..9, with 0 / 10 / 50 thinly-dressed layers -- all 30 circuits
    through the register-tile SV path against the oracle's values (tests/golden/config2_sv.npz, made
    by tests/golden/make_config2_golden.py from oracle/sv.py): global cost within 1e-10, the 20 <Z_i>
    within 1e-10, four projections of the whole state onto seeded random unit vectors within 1e-10.
    The op lists are checked to be the profiled workload's (configs_bench.brickwork_sv_ops)."""
    import os
    import sys

    from adaptaqc_amd import gates as G
    from adaptaqc_amd import _lib
    from adaptaqc_amd.device import DeviceSV

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "tools"))
    import configs_bench
    import make_config2_golden as mk

    gold = np.load(os.path.join(here, "golden", "config2_sv.npz"))
    R = mk.probes()
    d = DeviceSV(mk.N)
    k = 0
    for seed in mk.SEEDS:
        for tail in mk.TAILS:
            named = mk.config2_named_ops(seed, tail)
            ops = configs_bench.brickwork_sv_ops(mk.N, mk.DEPTH, seed, tail)
            assert len(ops) == len(named)
            want = _lib.ops_array([(G.one_qubit(nm, list(p)) if len(q) == 1 else G.TWO_QUBIT[nm], q) for nm, q, p in named])
            np.testing.assert_array_equal(ops, want)
            d.reset()
            d.apply(ops)
            a0 = d.amp0()
            assert abs((1 - abs(a0) ** 2) - (1 - abs(gold["amp0"][k]) ** 2)) < TOL
            assert abs(a0 - gold["amp0"][k]) < TOL
            np.testing.assert_allclose(d.z_all(), gold["z"][k], atol=1e-10)
            psi = d.get()
            np.testing.assert_allclose(R.conj() @ psi, gold["proj"][k], atol=1e-10)
            k += 1


def test_deferred_reset_every_reader():
    """aqc_sv_reset on the register-tile path (n >= 14) launches nothing: the next apply's first
    pass forms |0...0> in its tiles, and every other reader (amp0, get, z_all, pair RDMs, transition,
    copy in either direction, set) sees |0...0> or overwrites it.  Each case follows an apply that
    left a non-trivial state behind, so a reader that skipped the reset would see that state."""
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceSV

    n = 14
    ops = brickwork(n, 4, 5)
    psi = osv.simulate(n, ops)
    dev_ops = device_ops(to_circuit(n, ops))
    e0 = np.zeros(2 ** n, complex)
    e0[0] = 1.0

    def dirty():
        d = DeviceSV(n)
        d.apply(dev_ops)
        d.reset()
        return d

    d = dirty()
    assert abs(d.amp0() - 1.0) < 1e-15
    np.testing.assert_array_equal(dirty().get(), e0)
    np.testing.assert_allclose(dirty().z_all(), np.ones(n), atol=1e-15)
    rd = dirty().pair_rdms([(0, 1)])
    want = np.zeros((4, 4), complex)
    want[0, 0] = 1.0
    np.testing.assert_allclose(np.asarray(rd).reshape(4, 4), want, atol=1e-15)
    # apply after reset: the first pass starts from |0...0>, twice in a row
    d = dirty()
    d.apply(dev_ops)
    np.testing.assert_allclose(d.get(), psi, atol=1e-12)
    d.reset()
    d.apply(dev_ops)
    np.testing.assert_allclose(d.get(), psi, atol=1e-12)
    # copy from a pending source; copy onto a pending destination
    src, dst = dirty(), DeviceSV(n)
    dst.apply(dev_ops)
    dst.copy_from(src)
    np.testing.assert_array_equal(dst.get(), e0)
    src = DeviceSV(n)
    src.apply(dev_ops)
    dst = dirty()
    dst.copy_from(src)
    np.testing.assert_allclose(dst.get(), psi, atol=1e-12)
    # set on a pending state overwrites it
    d = dirty()
    d.set(psi)
    np.testing.assert_allclose(d.get(), psi, atol=0)
    # transition <0|(|a><b|)_q|psi> with a pending bra: row a = 0 only
    bra, ket = dirty(), DeviceSV(n)
    ket.apply(dev_ops)
    t = bra.transition(ket, 3)
    np.testing.assert_allclose(t, [[psi[0], psi[1 << 3]], [0, 0]], atol=1e-15)
    # and a pending ket: <psi|(|a><b|)_q|0> = conj(psi[a << q]) for b = 0
    bra, ket = DeviceSV(n), dirty()
    bra.apply(dev_ops)
    t = bra.transition(ket, 3)
    np.testing.assert_allclose(t, [[np.conj(psi[0]), 0], [np.conj(psi[1 << 3]), 0]], atol=1e-15)


def test_amp0_handed_off_by_the_final_pass():
    """After an apply on the register-tile path the final pass writes <0...0|psi> to the pinned
    host buffer and aqc_sv_amp0 reads it without a copy: equal to the state's first amplitude after
    applies, an empty apply (state unchanged), a reset, a copy into the handle and a set."""
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceSV

    n = 15
    ops_a = device_ops(to_circuit(n, brickwork(n, 4, 8)))
    ops_b = device_ops(to_circuit(n, brickwork(n, 3, 9)))
    d, e = DeviceSV(n), DeviceSV(n)
    d.apply(ops_a)
    a = d.amp0()
    assert abs(a - d.get()[0]) == 0.0
    d.apply([])  # no ops: the state and its handed-off amp 0 stay
    assert d.amp0() == a
    d.apply(ops_b)
    b = d.amp0()
    assert abs(b - d.get()[0]) == 0.0 and abs(b - a) > 1e-6
    d.reset()
    assert d.amp0() == 1.0
    e.apply(ops_a)
    d.copy_from(e)
    assert d.amp0() == a
    psi = np.zeros(2 ** n, complex)
    psi[0], psi[5] = 0.6, 0.8
    d.set(psi)
    assert abs(d.amp0() - 0.6) < 1e-15


def test_copy_then_destroy_source_then_reuse_block():
    """aqc_sv_copy queues a copy that reads the source on the destination's stream.  The
    source destroyed right after, and a new state of the same size taking its pooled block and
    writing it at once, must not corrupt the copy (the source's stream waits for the copy)."""
    from adaptaqc_amd.circuit import device_ops
    from adaptaqc_amd.device import DeviceSV

    n = 20
    ops = brickwork(n, 6, 5)
    want = osv.simulate(n, ops)
    dops = device_ops(to_circuit(n, ops))
    for _ in range(3):
        src = DeviceSV(n)
        src.apply(dops)
        dst = DeviceSV(n)
        dst.copy_from(src)
        src.close()
        other = DeviceSV(n)  # (same size: the pool hands out src's block)
        other.apply(device_ops(to_circuit(n, brickwork(n, 8, 9))))
        other.amp0()
        np.testing.assert_allclose(dst.get(), want, atol=1e-12)
        dst.close()
        other.close()
