"""Debug: the Red Hat chain step by step with timestamps (GPU)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tools import synth_mix as sm
t0 = time.time()
def log(*a):
    print(f"[{time.time()-t0:7.2f}]", *a, flush=True)
import trivy_amd
from tools.synth_vuln import vuln_arena
from trivy_amd.batch import MatchBatch
sdb = sm.make_mix_db(sm.C5_PLATS, 1500, seed=0xC5C5)
db = sdb.put(trivy_amd.DB())
ids = sm.MixDB.vuln_ids_of(sdb)
db.put_arena(*vuln_arena(ids))
db.finalize()
log("db")
eng = trivy_amd.Engine(db, 0)
log("engine")
batch = sm.make_mix_batch(sdb, 24_000, sm.C5_WEIGHTS, seed=31)
mb = MatchBatch(eng)
firsts = sm.add_to(mb, sdb, batch)
log("added", len(mb))
total, errp, bits = mb.run()
log("run", total, errp, bits)
raw = mb.pairs()
log("pairs", len(raw))
mb.redhat_merge()
log("merge enqueued")
mb.launch(0, sync=True)
log("synced")
print(mb.status(), flush=True)
mp = mb.pairs()
log("merged pairs", len(mp))
mb.fill()
log("fill")
n = mb.filter(mb.filter_opts())
log("filter", n)
