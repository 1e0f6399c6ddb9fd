"""CPU: batch-API host helpers and the C3/C5 synthetic DBs load and finalize (no GPU)."""
import numpy as np

from tools import synth_mix as sm
from trivy_amd.batch import arena_of


def test_arena_of_columns():
    names = np.array([b"a", b"bcd", b"", b"ef"], dtype="S")
    arena, [(no, nl), (vo, vl)] = arena_of(names, [b"1", b"", b"22", b"333"])
    assert arena == b"abcdef122333"
    assert [arena[o:o + n] for o, n in zip(no, nl)] == [b"a", b"bcd", b"", b"ef"]
    assert [arena[o:o + n] for o, n in zip(vo, vl)] == [b"1", b"", b"22", b"333"]
    a2, [(o, n)] = arena_of([])
    assert a2 == b"" and len(o) == 0


def test_mix_dbs_finalize():
    import trivy_amd
    for plats in (sm.C5_PLATS, sm.C3_PLATS):
        sdb = sm.make_mix_db(plats, 200, seed=9)
        st = sdb.put(trivy_amd.DB()).finalize().stats()
        assert st["platforms"] >= len(plats) and st["advisories"] > 0 and st["rows"] >= st["advisories"] // 2
        b = sm.make_mix_batch(sdb, 5000, [1] * len(plats), seed=1)
        assert len(b) == 5000
