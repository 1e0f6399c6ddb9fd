"""Host side of the batch VEX filter (trivy_amd/vex.py): the reference's TestVEX_Filter cases
and seeded documents of all three formats, against the oracle (oracle/vex.py).  CPU only."""
import json
import os

import numpy as np
import pytest

from oracle import vex as ov
from tools import synth_vex as sv
from trivy_amd import vex as tv

HERE = os.path.join(os.path.dirname(__file__), "golden", "vex")
TABLE = json.load(open(os.path.join(HERE, "cases.json")))


@pytest.mark.parametrize("case", TABLE["cases"], ids=[c["name"] for c in TABLE["cases"]])
def test_suppressions_reference_cases(case):
    """pkg/vex/vex_test.go:66-373: one package per listed vulnerability, one result whose
    root is the case's BOM root."""
    rep = case.get("report") or {}
    text = open(os.path.join(HERE, case["file"])).read()
    if case.get("wantErr"):
        with pytest.raises(tv.VEXError, match=case["wantErr"]):
            tv.VEX.new(text, rep.get("ArtifactType", ""), rep.get("SerialNumber", ""), rep.get("Version", 0))
        return
    v = tv.VEX.new(text, rep.get("ArtifactType", ""), rep.get("SerialNumber", ""), rep.get("Version", 0))
    vulns = [TABLE["vulns"][k] for k in case["vulns"]]
    purls = [ov.purl_string(x["PkgIdentifier"]["PURL"]) for x in vulns]
    refs = [x["PkgIdentifier"].get("BOMRef", "") for x in vulns]
    root = TABLE["boms"][case["bom"]] if case["bom"] else None
    pk, ids = v.suppressions(purls, refs, np.zeros(len(vulns), dtype=np.int64),
                             [ov.purl_string(root) if root else None])
    drop = set(zip(pk.tolist(), ids))
    kept = [x for i, x in enumerate(vulns) if (i, x["VulnerabilityID"]) not in drop]
    assert kept == [TABLE["vulns"][k] for k in case["want"]]


def _synthetic(seed, n_results=6, per=40):
    rng = np.random.default_rng(seed)
    plats = ["debian 12", "ubuntu 22.04"]
    purls, refs, result_of, findings, roots = [], [], [], [], []
    for r in range(n_results):
        roots.append(sv.root_of(r) if r % 3 else None)
        for k in range(per):
            j = int(rng.integers(25))  # shared names across results, some repeats inside one
            plat = plats[j % 2]
            arch = "amd64" if j % 3 else None
            purls.append(sv.purl_of(plat, "lib+pkg%d" % j, "1.%d-%d" % (j % 4, j % 2), arch))
            refs.append("ref-%d-%d" % (r, k))
            result_of.append(r)
            for v in rng.choice(30, size=3, replace=False):
                findings.append((len(purls) - 1, "CVE-2023-%04d" % v))
    return rng, purls, refs, np.array(result_of), roots, findings


def _oracle_drop(ovex, purls, refs, result_of, roots, findings):
    out = set()
    for pk, vid in findings:
        vuln = {"VulnerabilityID": vid, "PkgIdentifier": {"PURL": ov.purl_from_string(purls[pk]),
                                                          "BOMRef": refs[pk]}}
        root = roots[result_of[pk]]
        if not ovex.keep(vuln, ov.purl_from_string(root) if root else None):
            out.add((pk, vid))
    return out


@pytest.mark.parametrize("kind", ["openvex", "cyclonedx", "csaf"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_suppressions_vs_oracle(kind, seed):
    rng, purls, refs, result_of, roots, findings = _synthetic(seed)
    if kind == "openvex":
        text = sv.openvex(rng, findings, purls, len(roots))
    elif kind == "cyclonedx":
        text = sv.cyclonedx(rng, findings, purls, refs)
    else:
        text = sv.csaf(rng, findings, purls)
    at = "cyclonedx" if kind == "cyclonedx" else ""
    pv = tv.VEX.new(text, at, sv.SERIAL, 1)
    pk, ids = pv.suppressions(purls, refs, result_of, roots)
    fset = set(findings)
    got = {x for x in zip(pk.tolist(), ids) if x in fset}  # the set may name findings the batch lacks
    want = _oracle_drop(ov.VEX.new(text, at, sv.SERIAL, 1), purls, refs, result_of, roots, findings)
    assert got == want
    assert 0 < len(want) < len(findings)
