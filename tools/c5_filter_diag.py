#!/usr/bin/env python3
"""GPU diagnostic (measurement only): where result.Filter drops C5 pairs.  Builds a C5 batch
of N packages (bench.py's Mix workload), runs match -> Red Hat merge -> FillInfo -> Filter with
the default options, and breaks the dropped pairs down by platform kind and by cause: the
package has a twin (same name, version, release) in its target, or the package's list holds
the VulnerabilityID more than once."""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(n=1_000_000):
    import argparse
    import bench
    import trivy_amd
    from trivy_amd.batch import MatchBatch, advisory_vuln_id
    args = argparse.Namespace(packages=n)
    wl = bench.Mix(args, "c5")
    db = trivy_amd.DB()
    wl.load(db, vulns=True)
    eng = trivy_amd.Engine(db.finalize(), 0)
    mb = MatchBatch(eng)
    wl.fill(mb)
    total, errp, bits = mb.run()
    raw = mb.pairs()
    mb.redhat_merge()
    merged = mb.pairs()
    mb.fill()
    kept = mb.filter(mb.filter_opts())
    fp = mb.filtered_pairs(kept)
    print(f"raw {len(raw)} merged {len(merged)} kept {kept} ignored {mb.n_ignored}", flush=True)
    kind = np.empty(wl.n, dtype=object)
    twin = np.zeros(wl.n, dtype=bool)
    for s, (p, g) in zip(wl.starts, wl.batch.groups):
        m = len(g["key"])
        kind[s:s + m] = wl.sdb.plats[p][1]
        key = [(i // wl.per_target, g["name"][i], g["ver"][i]) for i in range(m)]
        c = collections.Counter(key)
        twin[s:s + m] = [c[k] > 1 for k in key]
    m_set = collections.Counter(map(tuple, merged.tolist()))
    f_set = collections.Counter(map(tuple, fp.tolist()))
    dropped = m_set - f_set
    vid_cache = {}

    def vid(a):
        if a not in vid_cache:
            vid_cache[a] = advisory_vuln_id(db, a)
        return vid_cache[a]
    per_pkg = collections.defaultdict(list)
    for p, a in merged.tolist():
        per_pkg[p].append(vid(a))
    rep = {p: len(v) != len(set(v)) for p, v in per_pkg.items()}
    br = collections.Counter()
    for (p, a), c in dropped.items():
        br[(kind[p], "twin" if twin[p] else "-", "repeated-id" if rep.get(p) else "-")] += c
    for k, c in br.most_common(20):
        print(k, c)
    allk = collections.Counter()
    for (p, a), c in m_set.items():
        allk[(kind[p], "twin" if twin[p] else "-", "repeated-id" if rep.get(p) else "-")] += c
    print("all merged pairs by class:")
    for k, c in allk.most_common(20):
        print(k, c)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000)
