"""The C-ABI library loads and exports every symbol include/*.h declares -- the drop-in boundary
(aqc_hip.h) and the diagnostics / test hooks (aqc_hip_diag.h) -- with no GPU needed."""
import os
import re

from conftest import ROOT


def _header_symbols(names=("aqc_hip.h", "aqc_hip_diag.h")):
    out = set()
    for name in names:
        src = open(os.path.join(ROOT, "include", name)).read()
        out |= set(re.findall(r"^(?:int|const char\*)\s+(aqc_\w+)\(", src, flags=re.M))
    return sorted(out)


def test_library_exports_header_symbols():
    from adaptaqc_amd import _lib

    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 35
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.EXPORTS), "ctypes table out of sync with the headers"
    boundary = set(_header_symbols(("aqc_hip.h",)))
    assert not boundary & set(_header_symbols(("aqc_hip_diag.h",))), "a symbol declared in both headers"
    assert "aqc_svd_debug" not in boundary and "aqc_debug_hog" not in boundary


def test_library_version_and_error_channel():
    from adaptaqc_amd import _lib

    lib = _lib.load()
    assert lib.aqc_version() == 1
    assert isinstance(lib.aqc_last_error(), bytes)


def test_no_oracle_in_product():
    """The product package never imports the oracle (oracle/__init__.py contract)."""
    pkg = os.path.join(ROOT, "adaptaqc_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                text = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in text and "from oracle" not in text, f
