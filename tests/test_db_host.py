"""Host-only (no GPU): every committed bolt-fixture file flattens through the product's
JSON decoder and finalize() (db.cpp DB::finalize), the load-time step that replaces
trivy-db's db.Init + per-call Get."""
import glob
import os

import pytest

import trivy_amd

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = sorted(glob.glob(os.path.join(HERE, "golden", "fixtures", "**", "*.json"), recursive=True))


@pytest.mark.parametrize("path", FIX, ids=[os.path.relpath(p, HERE) for p in FIX])
def test_fixture_flattens(path):
    db = trivy_amd.load_fixture_files([path])
    st = db.stats()
    assert all(v >= 0 for v in st.values())


def test_all_fixtures_together():
    db = trivy_amd.load_fixture_files(FIX)
    st = db.stats()
    assert st["keys"] > 50 and st["rows"] > 50 and st["advisories"] > 50
