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


def test_supported_versions_host():
    from trivy_amd.detector.ospkg import is_supported_version
    from conftest import load_case_file, parse_now
    for drv in ["debian", "ubuntu"]:
        for c in load_case_file(drv)["supported"]:
            assert is_supported_version(c["family"], c["os_ver"], parse_now(c["now"])) == c["want"], c["name"]
