"""Reference-side binding: drop the MI355X engine into qiskit-community/adapt-aqc itself.

The reference chooses its MPS / statevector code paths by class (``isinstance(backend,
AerMPSBackend)``, approximate_compiler.py:113, :223; ``isinstance(backend, AerSVBackend)``,
utilityfunctions.py:122-130) and reaches the simulators through four module-level names:

* ``adaptaqc.compilers.approximate_compiler.mps_from_circuit`` (:133, :198, :230: zero state,
  target MPS, tenpy starting state),
* ``aqc_research.mps_operations.mps_from_circuit`` as ``mpsops.mps_from_circuit``
  (adapt_compiler.py:1129, the MPS-cache absorption),
* ``adaptaqc.utils.gradients.general_grad_of_pairs`` (adapt_compiler.py:846, the candidate sweep),
* the backend methods of aqc_backend.py:14-29 (every cost evaluation),
* the ISL sweep (the reference's default method, adapt_config.py:25):
  ``AdaptCompiler._get_all_qubit_pair_entanglement_measures`` (adapt_compiler.py:955-976) calls
  ``calculate_entanglement_measure`` per coupling-map pair, which reaches
  ``backend.simulator.run(...).result().get_statevector()`` through
  ``co.run_circuit_without_transpilation`` (circuit_operations_running.py:58-63) and then
  ``entanglement_measures.partial_trace`` (:75) on SV, or ``mpsops.partial_trace`` (:77) on the MPS
  from ``backend.evaluate_circuit``.  ``SVSimulator.run`` simulates on the device (an unchanged
  circuit once per sweep), and both ``partial_trace`` names are rebound to device RDMs.  The
  compiler method itself is wrapped so that, with one of this package's backends, the whole sweep
  is one device state, one all-pair RDM launch chain and one measure launch; with any other
  backend, or the observable lower bound, the reference's own method runs.

``install()`` registers this package's backends as virtual subclasses of the reference's
``AerMPSBackend`` / ``AerSVBackend`` (``ABCMeta.register``: both derive from the ABC
``AQCBackend``) and points those names at the device implementations, which accept the
reference's qiskit circuits (``CircuitInstruction`` with ``Qubit`` objects resolved through
``find_bit``; gate matrices from the standard names or ``to_matrix()``).  A backend instance keeps
its device copy of the cached MPS across evaluations (uploaded once per cached payload), so the
reference's evaluation loop pays no per-call create / upload.

Usage, in the reference's environment::

    from adaptaqc_amd import reference_binding
    reference_binding.install()
    from adaptaqc_amd.backends import AerMPSBackend as HipMPSBackend, mps_sim_with_args
    compiler = AdaptCompiler(target, backend=HipMPSBackend(mps_sim_with_args(max_chi=64)), ...)

Nothing here imports qiskit; with the reference absent ``install()`` reports what it could not
find and changes nothing.
"""
from __future__ import annotations

import importlib
import sys

from .backends.aer_mps_backend import AerMPSBackend as HipMPSBackend
from .backends.aer_sv_backend import AerSVBackend as HipSVBackend
from .mps_operations import mps_from_circuit as device_mps_from_circuit
from .mps_operations import partial_trace as device_mps_partial_trace
from .utils.entanglement_measures import partial_trace as device_sv_partial_trace
from .utils.gradients import general_grad_of_pairs as device_general_grad_of_pairs


class _Wrap:
    """A replacement built from the original attribute (``factory(original) -> replacement``)."""

    def __init__(self, factory):
        self.factory = factory


def _batched_isl(original):
    """``AdaptCompiler._get_all_qubit_pair_entanglement_measures`` (adapt_compiler.py:955-976) for
    this package's backends: the same ``circ_mps`` side effect and per-pair list in coupling-map
    order, computed as one device state + all-pair RDMs (aqc_sv_pair_rdms / aqc_mps_pair_rdms) +
    one aqc_entanglement_measures launch."""
    from .device import entanglement_measures
    from .utils.entanglement_measures import _CODES

    def _get_all_qubit_pair_entanglement_measures(self):
        backend = getattr(self, "backend", None)
        method = getattr(self, "entanglement_measure_method", None)
        if not isinstance(backend, (HipSVBackend, HipMPSBackend)) or method not in _CODES:
            return original(self)
        pairs = [(int(c), int(t)) for c, t in self.coupling_map]
        if isinstance(backend, HipMPSBackend):
            self.circ_mps = backend.evaluate_circuit(self)
            rdms = self.circ_mps.pair_rdms(pairs) if pairs else []
        else:
            self.circ_mps = None
            rdms = backend.pair_rdms(self, pairs) if pairs else []
        if not pairs:
            return []
        return [float(x) for x in entanglement_measures(rdms, _CODES[method])]

    _get_all_qubit_pair_entanglement_measures.__wrapped__ = original
    return _get_all_qubit_pair_entanglement_measures


# ---- the reference's own Rotoselect / Rotosolve, batched (cost_minimiser.py:267-368) --------------
# The reference's CostMinimiser asks ``self.cost_finder()`` (the compiler's evaluate_cost,
# approximate_compiler.py:150-158, 514-527) once per candidate: 1 + 3 x 2 = 7 evaluations per gate in
# replace_with_best_1q_gate, 3 (2 with the identity cost given) in find_best_angle, each a full
# replay.  With this package's backends, the wrappers below take all
# candidates of a gate from one batched evaluation of utils/cached_rotations.py (statevector: a 2x2
# transition matrix of the prefix and the undone suffix; MPS: the cached prefix MPS and all
# candidates replayed through the suffix in one lock-step batch), and then run the reference's own
# code on those numbers: its SUPPORTED_1Q_GATES order, its minimum_of_sinusoidal, its strict `<`,
# its co.replace_1q_gate edits of full_circuit, and cost_evaluation_counter advanced by the number
# of evaluate_cost calls it would have made.  An evaluator lives for one _reduce_cost sweep (the
# gates are visited in index order; only the gate just optimised changes between them).  The local
# and softened costs batch the same way (every candidate's <Z_i> or HW-1 amplitudes in one set of
# launches; on the statevector backend the local cost from a cached prefix state).  Anything else
# (the softened cost on SV, other backends, NLopt / SciPy paths) runs the reference's code.

def _rotations_evaluator(minimiser):
    from .utils.cached_rotations import MPSPrefixBatch, SVPrefixBatch, SVTransitionSweep, _cost_kind

    compiler = getattr(minimiser.cost_finder, "__self__", None)
    if compiler is None or getattr(compiler, "full_circuit", None) is not minimiser.full_circuit:
        return None
    kind = _cost_kind(compiler)  # the branch evaluate_cost takes (approximate_compiler.py:514-527)
    backend = getattr(compiler, "backend", None)
    if isinstance(backend, HipMPSBackend):
        return MPSPrefixBatch(compiler, kind)
    if isinstance(backend, HipSVBackend):
        if kind == "global":
            return SVTransitionSweep(compiler)
        if kind == "local":
            return SVPrefixBatch(compiler)
    return None


def _reference_module(name):
    return sys.modules.get(name)


def _batched_reduce_cost(original):
    def _reduce_cost(self, *args, **kwargs):
        prev = getattr(self, "_aqc_rotations", None)
        self._aqc_rotations = _rotations_evaluator(self)
        try:
            return original(self, *args, **kwargs)
        finally:
            self._aqc_rotations = prev

    _reduce_cost.__wrapped__ = original
    return _reduce_cost


def _candidate(name, theta):
    from .utils.cached_rotations import rotation

    return rotation(name, theta)


def _batched_replace_with_best_1q_gate(original):
    def replace_with_best_1q_gate(self, gate_index):
        ev = getattr(self, "_aqc_rotations", None)
        cm = _reference_module(type(self).__module__)
        if ev is None or cm is None:
            return original(self, gate_index)
        names = list(cm.SUPPORTED_1Q_GATES)
        ev.goto(gate_index)
        mats = [_candidate("rx", 0.0)]
        for name in names:
            mats += [_candidate(name, cm.np.pi / 2), _candidate(name, -cm.np.pi / 2)]
        c = ev.costs(gate_index, mats)
        ev.count(len(mats))
        # cost_minimiser.py:327-342 on those numbers (find_best_angle's replace / restore of the
        # gate is a no-op on the circuit once it holds rx(0))
        cm.co.replace_1q_gate(self.full_circuit, gate_index, "rx", 0)
        cost_identity = c[0]
        best_gate_name, best_gate_angle, best_gate_cost = None, None, 1
        for k, gate_name in enumerate(names):
            min_angle, cost = cm.minimum_of_sinusoidal(cost_identity, c[1 + 2 * k], c[2 + 2 * k])
            if cost < best_gate_cost:
                best_gate_name, best_gate_angle, best_gate_cost = gate_name, min_angle, cost
        cm.co.replace_1q_gate(self.full_circuit, gate_index, best_gate_name, best_gate_angle)
        return best_gate_cost

    replace_with_best_1q_gate.__wrapped__ = original
    return replace_with_best_1q_gate


def _batched_find_best_angle(original):
    def find_best_angle(self, gate_index, gate_name, cost_for_identity=None):
        ev = getattr(self, "_aqc_rotations", None)
        cm = _reference_module(type(self).__module__)
        if ev is None or cm is None:
            return original(self, gate_index, gate_name, cost_for_identity)
        # cost_minimiser.py:344-368: [0, pi/2, -pi/2], the identity cost reused when given
        angles = [0, cm.np.pi / 2, -cm.np.pi / 2]
        costs = []
        if cost_for_identity is not None:
            costs.append(cost_for_identity)
            angles.remove(0)
        ev.goto(gate_index)
        costs += ev.costs(gate_index, [_candidate(gate_name, float(t)) for t in angles])
        ev.count(len(angles))
        return cm.minimum_of_sinusoidal(costs[0], costs[1], costs[2])

    find_best_angle.__wrapped__ = original
    return find_best_angle


# (module, attribute path, replacement) -- the reference's own call sites resolve these names at
# call time (module globals, module attributes, class attributes), so rebinding them is enough
PATCHES = (
    ("adaptaqc.compilers.approximate_compiler", "mps_from_circuit", device_mps_from_circuit),
    ("aqc_research.mps_operations", "mps_from_circuit", device_mps_from_circuit),
    ("aqc_research.mps_operations", "partial_trace", device_mps_partial_trace),
    ("adaptaqc.utils.entanglement_measures", "partial_trace", device_sv_partial_trace),
    ("adaptaqc.utils.gradients", "general_grad_of_pairs", device_general_grad_of_pairs),
    ("adaptaqc.compilers.adapt.adapt_compiler", "AdaptCompiler._get_all_qubit_pair_entanglement_measures",
     _Wrap(_batched_isl)),
    ("adaptaqc.utils.cost_minimiser", "CostMinimiser._reduce_cost", _Wrap(_batched_reduce_cost)),
    ("adaptaqc.utils.cost_minimiser", "CostMinimiser.replace_with_best_1q_gate",
     _Wrap(_batched_replace_with_best_1q_gate)),
    ("adaptaqc.utils.cost_minimiser", "CostMinimiser.find_best_angle", _Wrap(_batched_find_best_angle)),
)
REGISTRATIONS = (
    ("adaptaqc.backends.aer_mps_backend", "AerMPSBackend", HipMPSBackend),
    ("adaptaqc.backends.aer_sv_backend", "AerSVBackend", HipSVBackend),
)

_saved = {}


def _module(name, import_missing):
    if name in sys.modules:
        return sys.modules[name]
    if not import_missing:
        return None
    try:
        return importlib.import_module(name)
    except ImportError:
        return None


def install(import_missing: bool = True) -> dict:
    """Register the device backends with the reference's ABCs and rebind its simulator entry
    points.  Returns {"registered": [...], "patched": [...], "missing": [...]}."""
    done = {"registered": [], "patched": [], "missing": []}
    for mod_name, cls_name, impl in REGISTRATIONS:
        mod = _module(mod_name, import_missing)
        base = getattr(mod, cls_name, None) if mod is not None else None
        if base is None or not hasattr(base, "register"):
            done["missing"].append(f"{mod_name}.{cls_name}")
            continue
        base.register(impl)
        done["registered"].append(f"{mod_name}.{cls_name} <- {impl.__module__}.{impl.__name__}")
    for mod_name, path, impl in PATCHES:
        owner = _module(mod_name, import_missing)
        *parents, attr = path.split(".")
        for p in parents:
            owner = getattr(owner, p, None) if owner is not None else None
        if owner is None or not hasattr(owner, attr):
            done["missing"].append(f"{mod_name}.{path}")
            continue
        key = (mod_name, path)
        if key not in _saved:
            _saved[key] = (owner, getattr(owner, attr))
        if isinstance(impl, _Wrap):
            impl = impl.factory(_saved[key][1])
        setattr(owner, attr, impl)
        done["patched"].append(f"{mod_name}.{path}")
    return done


def uninstall() -> None:
    """Restore the patched names (ABC registrations cannot be undone and stay)."""
    for (mod_name, path), (owner, orig) in list(_saved.items()):
        setattr(owner, path.split(".")[-1], orig)
        del _saved[(mod_name, path)]


__all__ = ["install", "uninstall", "HipMPSBackend", "HipSVBackend", "PATCHES", "REGISTRATIONS"]
