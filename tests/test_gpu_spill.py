"""GPU: a long installed key whose scratch reservation fails (the batch scratch is sized
exactly by Engine::scratch_words, so only the TVM_TEST_SPILL_CAP hook can make it fail) fails
the pass with ERR_SPILL and leaves NO rows on that package - not even ROW_ALWAYS (unfixed)
rows, which would otherwise match a package whose key was never written - while every other
package of the batch keeps exactly the oracle's pairs."""
import numpy as np
import pytest

from oracle import match as om
from tools.synth import SynthBatch, make_batch, make_db

pytestmark = pytest.mark.gpu


def test_spill_failure_leaves_no_rows(monkeypatch, oracle_built):
    from test_gpu_parity import build_engine
    from trivy_amd.batch import MatchBatch
    sdb = make_db(["debian 12"], 400, seed=31, unfixed=0.5)
    eng = build_engine(sdb)
    base = make_batch(sdb, 8, 300, [1], seed=5, miss=0.0)
    names, vers = list(base.names), list(base.versions)
    long_ix = list(range(3, len(names), 37))
    for i in long_ix:  # a dpkg key far beyond 32 bytes: generic encoder + the batch scratch
        vers[i] = b"1:" + b".".join(str(k).encode() for k in range(2, 40)) + b"-1"
    batch = SynthBatch(base.plat, names, vers, list(base.targets))
    opk, oad = om.match(om.Prepared(sdb, batch), n_threads=4)
    long_set = set(long_ix)
    assert sum(1 for p in opk.tolist() if p in long_set) > 10  # the long packages do match rows
    monkeypatch.setenv("TVM_TEST_SPILL_CAP", "0")
    mb = MatchBatch(eng)
    arena, noff, nlen, voff, vlen = batch.arena()
    for p, b0, b1 in batch.targets:
        mb.add_arena(sdb.platforms[p], b1 - b0, arena, noff[b0:], nlen[b0:], voff[b0:], vlen[b0:])
    mb.upload(max(64 * len(batch), 2 * len(opk))).launch()
    total, errp, bits = mb.status()
    assert bits & 1, bits  # ERR_SPILL: the pass reports failure
    pairs = mb.pairs()
    got_long = [p for p in pairs[:, 0].tolist() if p in long_set]
    assert got_long == []
    keep = ~np.isin(opk, long_ix)
    assert np.array_equal(pairs[:, 0], opk[keep]) and np.array_equal(pairs[:, 1], oad[keep])
    mb.close()
