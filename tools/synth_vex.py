"""Seeded VEX documents (OpenVEX, CycloneDX, CSAF) aimed at a batch's packages, for the
parity tests of the VEX filter (trivy_amd/vex.py + filter.hip vs oracle/vex.py)."""
import json
import urllib.parse

import numpy as np

SERIAL = "urn:uuid:3e671687-395b-41f5-a30f-a58921a69b79"


def purl_of(platform, name, version, arch=None):
    """The PURL trivy gives an OS package (pkg/purl): pkg:deb/<os>/<name>@<ver>?distro=<os>-<ver>."""
    fam, _, ver = platform.partition(" ")
    s = "pkg:deb/%s/%s@%s" % (fam, urllib.parse.quote(name, safe=""), urllib.parse.quote(version, safe=""))
    q = ([("arch", arch)] if arch else []) + [("distro", "%s-%s" % (fam, ver))]
    return s + "?" + "&".join("%s=%s" % kv for kv in q)


def root_of(r):
    return "pkg:oci/image%d@sha256:%064x?tag=%d" % (r % 3, r, r)


def _strip(purl, rng):
    """A more general pattern of a package PURL: versionless and/or qualifier-less."""
    base, _, q = purl.partition("?")
    k = rng.integers(4)
    if k == 0:
        return purl
    if k == 1:
        return base
    if k == 2:
        return base.rpartition("@")[0]
    return base.rpartition("@")[0] + "?" + q


def openvex(rng, findings, purls, n_results, n_stmts=60):
    """findings: [(package, vuln ID)]; purls[package]."""
    stmts = []
    statuses = ["not_affected", "fixed", "affected", "under_investigation"]
    hot = [findings[i] for i in rng.integers(len(findings), size=8)]  # repeated statements: timestamp order decides
    for _ in range(n_stmts):
        pk, vid = hot[rng.integers(len(hot))] if rng.random() < 0.5 else findings[rng.integers(len(findings))]
        st = {"vulnerability": {"name": vid} if rng.random() < 0.8 else {"name": "GHSA-" + vid, "aliases": [vid]},
              "status": statuses[rng.integers(4)]}
        if rng.random() < 0.5:
            st["timestamp"] = "2023-01-%02dT%02d:00:00.%09dZ" % (rng.integers(10, 20), rng.integers(24),
                                                               rng.integers(10 ** 9))
        if rng.random() < 0.3:  # root image + subcomponent
            r = int(rng.integers(n_results))
            prod = {"@id": root_of(r).partition("@")[0] if rng.random() < 0.5 else root_of(r),
                    "subcomponents": [{"@id": _strip(purls[pk], rng)}]}
        elif rng.random() < 0.2:
            prod = {"@id": "urn:x-image:%d" % pk, "identifiers": {"purl": _strip(purls[pk], rng)}}
        else:
            prod = {"@id": _strip(purls[pk], rng)}
        st["products"] = [prod]
        stmts.append(st)
    return json.dumps({"@context": "https://openvex.dev/ns/v0.2.0", "timestamp": "2023-01-16T19:07:16.853479631-06:00",
                       "statements": stmts})


def cyclonedx(rng, findings, purls, bom_refs, n_vulns=60):
    vulns = []
    states = ["not_affected", "resolved", "exploitable", "in_triage", "false_positive", None]
    for _ in range(n_vulns):
        pk, vid = findings[rng.integers(len(findings))]
        affects = []
        for _ in range(1 + rng.integers(3)):
            q, _ = findings[rng.integers(len(findings))] if rng.random() < 0.5 else (pk, None)
            ref = bom_refs[q] if rng.random() < 0.5 else purls[q]
            serial = SERIAL if rng.random() < 0.9 else "urn:uuid:00000000-0000-4000-8000-000000000000"
            affects.append({"ref": "urn:cdx:%s/%d#%s" % (serial[9:], 1, ref)})
        v = {"id": vid, "affects": affects}
        s = states[rng.integers(len(states))]
        if s:
            v["analysis"] = {"state": s}
        vulns.append(v)
    return json.dumps({"bomFormat": "CycloneDX", "specVersion": "1.5", "version": 1, "vulnerabilities": vulns})


def csaf(rng, findings, purls, n_vulns=40):
    prods, rels, vulns = [], [], []
    for k in range(n_vulns):
        pk, vid = findings[rng.integers(len(findings))]
        pid = "P%d" % k
        if rng.random() < 0.3:  # a component of another product, named through a relationship
            prods.append({"product_id": pid + "-c", "product_identification_helper": {"purl": _strip(purls[pk], rng)}})
            prods.append({"product_id": pid + "-app", "product_identification_helper": {"purl": "pkg:oci/app%d" % k}})
            rels.append({"category": ["default_component_of", "installed_on", "optional_component_of"][k % 3],
                         "product_reference": pid + "-c", "relates_to_product_reference": pid + "-app",
                         "full_product_name": {"product_id": pid, "name": "x"}})
        else:
            prods.append({"product_id": pid, "product_identification_helper": {"purl": _strip(purls[pk], rng)}})
        st = ["known_not_affected", "fixed", "known_affected"][rng.integers(3)]
        vulns.append({"cve": vid, "product_status": {st: [pid]}})
    branches = [{"category": "vendor", "name": "v", "branches": [
        {"category": "product_version", "name": p["product_id"], "product": dict(p, name=p["product_id"])}
        for p in prods]}]
    return json.dumps({"document": {"category": "csaf_vex"}, "product_tree": {"branches": branches,
                                                                             "relationships": rels},
                       "vulnerabilities": vulns})
