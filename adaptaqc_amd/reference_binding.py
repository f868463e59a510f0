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
