#!/usr/bin/env python3
"""Harvest library-detection vectors from the reference's integration goldens (DATA).

TEST INFRASTRUCTURE.  Reads /root/reference/integration/testdata/*.json.golden (the
expected `trivy` JSON reports of the reference's integration tests,
integration/integration_test.go:204-255) and keeps, per lang-pkgs Result, the
detector-produced subset of every DetectedVulnerability (the goldens
include FillInfo fields, so only the detector subset is compared).  The packages listed
are exactly the vulnerable ones, so each package's expected vulnerability set is
complete.  The DB these goldens were produced against is every YAML file of
integration/testdata/fixtures/db (converted to tests/golden/fixtures/integration/).

Output: tests/golden/integration_lib.json
"""
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
FIELDS = ["VulnerabilityID", "PkgID", "PkgName", "InstalledVersion", "FixedVersion", "PkgPath", "DataSource"]


def main(ref="/root/reference"):
    out = []
    for f in sorted(glob.glob(os.path.join(ref, "integration/testdata/*.json.golden"))):
        with open(f, encoding="utf-8") as fh:
            d = json.load(fh)
        for r in d.get("Results") or []:
            if r.get("Class") != "lang-pkgs" or not r.get("Vulnerabilities"):
                continue
            pkgs, want = {}, []
            for v in r["Vulnerabilities"]:
                key = (v.get("PkgID", ""), v["PkgName"], v["InstalledVersion"], v.get("PkgPath", ""))
                pkgs[key] = {"ID": key[0], "Name": key[1], "Version": key[2], "FilePath": key[3]}
                want.append({k: v[k] for k in FIELDS if v.get(k)})
            out.append({"golden": os.path.basename(f), "target": r.get("Target"), "type": r["Type"],
                        "pkgs": list(pkgs.values()), "want": want})
    with open(os.path.join(HERE, "integration_lib.json"), "w", encoding="utf-8") as fh:
        json.dump(out, fh, indent=1, ensure_ascii=False)
        fh.write("\n")
    print(f"{len(out)} lang-pkgs results")


if __name__ == "__main__":
    main(*sys.argv[1:])
