"""Load the reference's ``paper/random_mps/target_seed_*.pkl`` fixtures without executing code.

The pickles hold Aer-format MPS ``(list[(G0, G1)], list[lambda])``.  They are read with an
unpickler that resolves only numpy's array-reconstruction globals; anything else raises.
``tests/golden/make_golden.py`` converts them once into ``tests/golden/random_mps.npz``
(the reference does not exist on the GPU box).
"""
import importlib
import pickle

_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"),
    ("numpy", "ndarray"),
    ("numpy", "dtype"),
}


class _NumpyOnly(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) not in _ALLOWED:
            raise pickle.UnpicklingError(f"refusing global {module}.{name}")
        if module == "numpy.core.multiarray":
            module = "numpy._core.multiarray"
        return getattr(importlib.import_module(module), name)


def load_aer_mps_pickle(path):
    with open(path, "rb") as f:
        return _NumpyOnly(f).load()


def pack_npz_dict(qmps, prefix):
    gam, lam = qmps
    d = {f"{prefix}n": len(gam)}
    for i, (a, b) in enumerate(gam):
        d[f"{prefix}g{i}"] = __import__("numpy").stack([a, b])
    for i, x in enumerate(lam):
        d[f"{prefix}l{i}"] = x
    return d


def unpack_npz_dict(z, prefix):
    n = int(z[f"{prefix}n"])
    gam = [(z[f"{prefix}g{i}"][0], z[f"{prefix}g{i}"][1]) for i in range(n)]
    lam = [z[f"{prefix}l{i}"] for i in range(n - 1)]
    return gam, lam
