"""CPU: the C-ABI library loads, exports every symbol include/trivy_amd.h declares,
and refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from trivy_amd._lib import lib, EXPORTED, LIB_PATH


def declared_symbols():
    out = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if fn.endswith(".h"):
            text = open(os.path.join(ROOT, "include", fn)).read()
            text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
            out |= set(re.findall(r"\b(tvm_[a-z_0-9]+)\s*\(", text))
    return out


def test_exports_every_declared_symbol():
    L = ctypes.CDLL(LIB_PATH)
    missing = [s for s in sorted(declared_symbols()) if not hasattr(L, s)]
    assert not missing
    assert declared_symbols() == set(EXPORTED)


def test_abi_version():
    assert lib().tvm_abi_version() == 1
    assert b"gfx950" in lib().tvm_version()


def test_engine_requires_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import trivy_amd
    db = trivy_amd.load_fixture_files([os.path.join(ROOT, "tests/golden/fixtures/ospkg/debian/debian.json")])
    with pytest.raises(RuntimeError, match="no HIP device"):
        trivy_amd.Engine(db)


def test_db_flatten_stats():
    import trivy_amd
    db = trivy_amd.load_fixture_files([os.path.join(ROOT, "tests/golden/fixtures/ospkg/debian/debian.json"),
                                       os.path.join(ROOT, "tests/golden/fixtures/ospkg/debian/data-source.json")])
    st = db.stats()
    assert st["platforms"] == 1 and st["keys"] == 1 and st["advisories"] == 3 and st["rows"] == 3


import golden_tables as gt  # noqa: E402

_SUPPORTED = [c for d in gt.OS_DRIVERS for c in gt.os_supported_cases(d)]


@pytest.mark.parametrize("case", _SUPPORTED, ids=[c[0] for c in _SUPPORTED])
def test_supported_versions_host(case):
    """Driver.IsSupportedVersion of every driver (host-side; *_test.go tables)."""
    from trivy_amd.detector.ospkg import is_supported_version
    cid, family, os_ver, now, want = case
    assert is_supported_version(family, os_ver, now) == want, cid


@pytest.mark.parametrize("driver", gt.OS_DRIVERS)
def test_every_fixture_flattens(driver):
    """Every OS fixture set loads; poisoned buckets stay loadable (errors are lazy)."""
    import glob
    import trivy_amd
    for f in sorted(glob.glob(os.path.join(gt.GOLDEN, "fixtures", "ospkg", driver, "*.json"))):
        st = trivy_amd.load_fixture_files([f]).stats()
        assert st["platforms"] >= 0
