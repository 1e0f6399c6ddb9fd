#!/usr/bin/env python3
"""Harvest FillInfo vectors from the reference's integration goldens (DATA).

TEST INFRASTRUCTURE.  Reads /root/reference/integration/testdata/*.json.golden (the
expected `trivy` JSON reports, integration/integration_test.go:204-255) and turns every
reported vulnerability into one FillInfo case (pkg/vulnerability/vulnerability.go:60-109):

  input  = what the detector handed to FillInfo: VulnerabilityID, FixedVersion,
           DataSource; Status only when the result is unfixed and not "affected" (a
           vendor status the detector copied, debian.go:95 / redhat.go:160); and the
           detector's package-specific SeveritySource + Severity when the golden's
           SeveritySource is the detector's own (debian.go:89-92 "debian",
           redhat.go:161 "redhat") for a target of that family;
  want   = the FillInfo fields of the golden: Status, Severity, SeveritySource,
           PrimaryURL and the joined Vulnerability detail (Title, Description, CweIDs,
           VendorSeverity, CVSS, References, PublishedDate, LastModifiedDate).

The vulnerability DB these goldens were produced against is
integration/testdata/fixtures/db/vulnerability.yaml (converted to
tests/golden/fixtures/integration/vulnerability.json).

Output: tests/golden/fillinfo_integration.json
"""
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
DETAIL = ["Title", "Description", "CweIDs", "VendorSeverity", "CVSS", "References", "PublishedDate",
          "LastModifiedDate"]
# dbTypes.Status marshals as these names (trivy-db pkg/types/status.go); cases carry ints
STATUS = ["unknown", "not_affected", "affected", "fixed", "under_investigation", "will_not_fix", "fix_deferred",
          "end_of_life"]
# spring4shell-jre8: the example WASM post-scan module rewrites the severity after
# FillInfo (integration/module_test.go:21 "severity update"), so it is not a FillInfo vector
SKIP = {"spring4shell-jre8.json.golden"}
DETECTOR_SEVERITY_SOURCE = {"debian": "debian", "redhat": "redhat", "centos": "redhat"}


def main(ref="/root/reference"):
    out = []
    for f in sorted(glob.glob(os.path.join(ref, "integration/testdata/*.json.golden"))):
        if os.path.basename(f) in SKIP:
            continue
        with open(f, encoding="utf-8") as fh:
            d = json.load(fh)
        for r in d.get("Results") or []:
            for v in r.get("Vulnerabilities") or []:
                inp = {k: v[k] for k in ("VulnerabilityID", "FixedVersion", "DataSource") if v.get(k)}
                if not v.get("FixedVersion") and v.get("Status") not in (None, "affected"):
                    inp["Status"] = STATUS.index(v["Status"])
                own = DETECTOR_SEVERITY_SOURCE.get(r.get("Type", ""))
                if r.get("Class") == "os-pkgs" and own and v.get("SeveritySource") == own:
                    inp["SeveritySource"] = own
                    inp["Vulnerability"] = {"Severity": v.get("Severity", "")}
                want = {k: v[k] for k in ("Severity", "SeveritySource", "PrimaryURL") if v.get(k)}
                want["Status"] = STATUS.index(v["Status"])
                want["Vulnerability"] = {k: v[k] for k in DETAIL if v.get(k)}
                out.append({"golden": os.path.basename(f), "target": r.get("Target"), "class": r.get("Class"),
                            "input": inp, "want": want})
    with open(os.path.join(HERE, "fillinfo_integration.json"), "w", encoding="utf-8") as fh:
        json.dump(out, fh, indent=1, ensure_ascii=False)
        fh.write("\n")
    print(f"{len(out)} FillInfo cases")


if __name__ == "__main__":
    main(*sys.argv[1:])
