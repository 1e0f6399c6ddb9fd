#!/usr/bin/env python3
"""Harvest the SBOM-scan vectors of the reference's integration tests (DATA).

TEST INFRASTRUCTURE.  integration/sbom_test.go:30-153 scans three CycloneDX SBOMs and the centos-7 image again as an
in-toto attestation, SPDX tag-value and SPDX JSON
(integration/testdata/fixtures/sbom/*, copied as data to tests/golden/sbom/) against the
integration DB (integration/testdata/fixtures/db, converted to
tests/golden/fixtures/integration/) and compares with integration/testdata/*.json.golden.
This keeps, per Result of those goldens, its class / type and the detector-produced
subset of every DetectedVulnerability (the goldens also hold FillInfo fields).

Output: tests/golden/sbom_cases.json
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
FIELDS = ["VulnerabilityID", "PkgID", "PkgName", "InstalledVersion", "FixedVersion", "PkgPath", "DataSource"]
CASES = [("centos7 cyclonedx", "centos-7-cyclonedx.json", "centos-7.json.golden"),
         ("fluentd-multiple-lockfiles cyclonedx", "fluentd-multiple-lockfiles-cyclonedx.json",
          "fluentd-multiple-lockfiles.json.golden"),
         ("minikube KBOM", "minikube-kbom.json", "minikube-kbom.json.golden"),
         # integration/sbom_test.go:84-153: the same image as in-toto, SPDX tag-value, SPDX JSON
         ("centos7 in in-toto attestation", "centos-7-cyclonedx.intoto.jsonl", "centos-7.json.golden"),
         ("centos7 spdx tag-value", "centos-7-spdx.txt", "centos-7.json.golden"),
         ("centos7 spdx json", "centos-7-spdx.json", "centos-7.json.golden")]


def main(ref="/root/reference"):
    out = []
    for name, sbom, golden in CASES:
        with open(os.path.join(ref, "integration/testdata", golden), encoding="utf-8") as fh:
            d = json.load(fh)
        results = [{"Class": r.get("Class"), "Type": r.get("Type"),
                    "Vulnerabilities": [{k: v[k] for k in FIELDS if v.get(k)} for v in r.get("Vulnerabilities") or []]}
                   for r in d.get("Results") or []]
        out.append({"name": name, "sbom": sbom, "golden": golden, "os": d["Metadata"].get("OS"),
                    "results": results})
    with open(os.path.join(HERE, "sbom_cases.json"), "w", encoding="utf-8") as fh:
        json.dump(out, fh, indent=1, ensure_ascii=False)


if __name__ == "__main__":
    main()
