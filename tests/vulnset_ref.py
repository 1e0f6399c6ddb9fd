"""The whole-batch DetectedVulnerability checker (test infrastructure): the oracle's expected
set for a tools/synth_mix.py batch, in the form tvm_match_vulns hands it out - per
DetectedVulnerability its package and its record (the advisory side), records compared as
canonical keys.

Expected set: the matches of oracle/mixmatch.c over the WHOLE batch (oracle/mix_c.py
Prepared / match, pinned to the Python oracle drivers by tests/test_cport.py), each turned
into a record by the oracle drivers' own epilogues (oracle/drivers.py advisory_record /
redhat_group_record, oracle/library.py advisory_record - the functions debian_detect,
redhat_detect, library.detect ... build their output with); Red Hat groups from the members
ORC_MIX_MEMBERS reports.  tests/test_vulnset_ref.py checks this construction against the
oracle drivers' per-target output on the CPU.
"""
import json

import numpy as np

from oracle import drivers as od
from oracle import library as ol
from oracle import mix_c


def rec_key(rec, flags):
    """Canonical key of a record: the DetectedVulnerability fields it sets (Go zero values
    dropped) and the copy flags."""
    return json.dumps([{k: x for k, x in rec.items() if x not in ("", 0, None, [], {})}, int(flags)], sort_keys=True)


class Keys:
    """Record key -> small int (shared by the oracle and the GPU side of one comparison)."""

    def __init__(self):
        self.ids = {}

    def __call__(self, key):
        return self.ids.setdefault(key, len(self.ids))


def expected(sm, sdb, batch, keys, threads=8, columnar=False):
    """(pkg int64[], record id int64[], installed list per package) of the whole batch, in the
    drivers' output order (by package; per package advisory / Get order, Red Hat by ID).
    columnar: the oracle digests the packages column-wise (mix_c.Prepared columnar form, for
    batches of 10-20M packages)."""
    sample = [(p, g, np.arange(len(g["key"]))) for p, g in batch.groups]
    prep = mix_c.Prepared(sm, sdb, sample, columnar=columnar)
    pk, en = mix_c.match(prep, threads, members=True)
    pk, en = pk.copy(), en.copy()
    plat_of = prep.plat_of
    fam = prep.plat_family
    rh_plat = np.array([f == "redhat" for f in fam], dtype=bool)
    rep = en >= 0
    is_rh = rh_plat[plat_of[pk]] if len(pk) else np.zeros(0, dtype=bool)
    out_pkg = pk[rep]
    out_rec = np.zeros(len(out_pkg), dtype=np.int64)
    rep_idx = np.nonzero(rep)[0]
    # records of plain entries, once per distinct entry
    plain = ~is_rh[rep_idx]
    ents = en[rep_idx[plain]]
    uniq, inv = np.unique(ents, return_inverse=True)
    ids = np.zeros(len(uniq), dtype=np.int64)
    # the platform of each distinct entry: take it from one of its rows
    first_row = np.zeros(len(uniq), dtype=np.int64)
    first_row[inv[::-1]] = rep_idx[plain][::-1]
    for k, e in enumerate(uniq.tolist()):
        f = fam[int(plat_of[pk[first_row[k]]])]
        a = prep.entries[e]["adv"]
        ids[k] = keys(rec_key(*(ol.advisory_record(a) if f is None else od.advisory_record(f, a))))
    out_rec[plain] = ids[inv]
    # Red Hat groups: the representative row, then its members (-(entry + 1))
    rh_rows = np.nonzero(~plain)[0]
    if len(rh_rows):
        pos = rep_idx[rh_rows]
        nxt = np.append(rep_idx[1:], len(en))[rh_rows]
        single = {}
        for r, a0, a1 in zip(rh_rows.tolist(), pos.tolist(), nxt.tolist()):
            mem = [-int(x) - 1 for x in en[a0 + 1:a1]]
            if len(mem) == 1:
                k = single.get(mem[0])
                if k is None:
                    k = single[mem[0]] = keys(rec_key(*od.redhat_group_record([prep.entries[mem[0]]["adv"]])))
            else:
                k = keys(rec_key(*od.redhat_group_record([prep.entries[m]["adv"] for m in mem])))
            out_rec[r] = k
    return out_pkg, out_rec, prep.installed


def gpu_side(vs, keys):
    """(pkg, record id) of a trivy_amd.batch.VulnSet, records keyed like expected()."""
    from trivy_amd.batch import vuln_record
    uniq, inv = np.unique(vs.rec, return_inverse=True)
    ids = np.zeros(len(uniq), dtype=np.int64)
    for k, r in enumerate(uniq.tolist()):
        d = dict(vs.record(r))
        flags = d.pop("_copy")
        ids[k] = keys(rec_key(d, flags))
    return vs.pkg.astype(np.int64), ids[inv]
