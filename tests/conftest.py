import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X; exercises libaqchip compute paths")


@pytest.fixture(scope="session")
def goldens():
    return np.load(os.path.join(GOLDEN, "oracle_goldens.npz"))


@pytest.fixture(scope="session")
def random_mps():
    from oracle.fixtures import unpack_npz_dict

    z = np.load(os.path.join(GOLDEN, "random_mps.npz"))
    return {int(s): unpack_npz_dict(z, f"s{int(s)}_") for s in z["seeds"]}


def golden_ops(g, seed):
    """Seeded random-circuit ops stored in oracle_goldens.npz -> [(name, qubits, params)]."""
    names = g[f"circ{seed}_ops_names"]
    qs = g[f"circ{seed}_ops_q"]
    ps = g[f"circ{seed}_ops_p"]
    out = []
    for nm, q, p in zip(names, qs, ps):
        nm = str(nm)
        qq = tuple(int(x) for x in q if x >= 0)
        out.append((nm, qq, (float(p),) if nm in ("rx", "ry", "rz") else ()))
    return out


def to_circuit(n, ops):
    from adaptaqc_amd.circuit import QuantumCircuit

    qc = QuantumCircuit(n)
    for nm, q, p in ops:
        if nm in ("rx", "ry", "rz"):
            getattr(qc, nm)(p[0], q[0])
        elif len(q) == 1:
            getattr(qc, nm)(q[0])
        else:
            getattr(qc, nm)(*q)
    return qc


class FakeCompiler:
    """The attributes the reference backends read from ``compiler``."""

    def __init__(self, full_circuit, soften=False, history=(), sufficient_cost=1e-2):
        from types import SimpleNamespace

        self.full_circuit = full_circuit
        self.soften_global_cost = soften
        self.global_cost_history = list(history)
        self.adapt_config = SimpleNamespace(sufficient_cost=sufficient_cost)
        self.backend_options = {}
        self.execute_kwargs = {}
