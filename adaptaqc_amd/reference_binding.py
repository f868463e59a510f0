"""Reference-side binding: drop the MI355X engine into qiskit-community/adapt-aqc itself.

The reference chooses its MPS / statevector code paths by class (``isinstance(backend,
AerMPSBackend)``, approximate_compiler.py:113, :223; ``isinstance(backend, AerSVBackend)``,
utilityfunctions.py:122-130) and reaches the simulators through four module-level names:

* ``adaptaqc.compilers.approximate_compiler.mps_from_circuit`` (:133, :198, :230: zero state,
  target MPS, tenpy starting state),
* ``aqc_research.mps_operations.mps_from_circuit`` as ``mpsops.mps_from_circuit``
  (adapt_compiler.py:1129, the MPS-cache absorption),
* ``adaptaqc.utils.gradients.general_grad_of_pairs`` (adapt_compiler.py:846, the candidate sweep),
* the backend methods of aqc_backend.py:14-29 (every cost evaluation).

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
from .utils.gradients import general_grad_of_pairs as device_general_grad_of_pairs

# (module, attribute, replacement) -- the reference's own call sites resolve these names at call
# time, so rebinding the module attribute is enough
PATCHES = (
    ("adaptaqc.compilers.approximate_compiler", "mps_from_circuit", device_mps_from_circuit),
    ("aqc_research.mps_operations", "mps_from_circuit", device_mps_from_circuit),
    ("adaptaqc.utils.gradients", "general_grad_of_pairs", device_general_grad_of_pairs),
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
    for mod_name, attr, impl in PATCHES:
        mod = _module(mod_name, import_missing)
        if mod is None or not hasattr(mod, attr):
            done["missing"].append(f"{mod_name}.{attr}")
            continue
        key = (mod_name, attr)
        if key not in _saved:
            _saved[key] = getattr(mod, attr)
        setattr(mod, attr, impl)
        done["patched"].append(f"{mod_name}.{attr}")
    return done


def uninstall() -> None:
    """Restore the patched names (ABC registrations cannot be undone and stay)."""
    for (mod_name, attr), orig in list(_saved.items()):
        mod = sys.modules.get(mod_name)
        if mod is not None:
            setattr(mod, attr, orig)
        del _saved[(mod_name, attr)]


__all__ = ["install", "uninstall", "HipMPSBackend", "HipSVBackend", "PATCHES", "REGISTRATIONS"]
