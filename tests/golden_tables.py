"""Access to the reference's transcribed Go test tables (tests/golden/tables/, written by
tests/golden/extract_go_tables.py) in the shape the drivers take."""
import datetime
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TABLES = os.path.join(GOLDEN, "tables")

# ubuntu.go:147 reads time.Now(); the tables were written against the reference snapshot
REF_NOW = "2025-01-14T00:00:00Z"

OS_DRIVERS = ["alma", "alpine", "amazon", "chainguard", "debian", "mariner", "oracle", "photon", "redhat",
              "rocky", "suse", "ubuntu", "wolfi"]
FAMILY = {"alma": "alma", "alpine": "alpine", "amazon": "amazon", "chainguard": "chainguard", "debian": "debian",
          "mariner": "cbl-mariner", "oracle": "oracle", "photon": "photon", "redhat": "redhat", "rocky": "rocky",
          "ubuntu": "ubuntu", "wolfi": "wolfi"}
SUSE_FAMILY = {"opensuse": "opensuse.leap", "sles": "suse linux enterprise server"}


def parse_now(s):
    return int(datetime.datetime.strptime(s, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=datetime.timezone.utc)
               .timestamp())


def load(rel):
    with open(os.path.join(TABLES, rel), encoding="utf-8") as f:
        return json.load(f)


def table(rel, func):
    for t in load(rel)["tables"]:
        if t["func"] == func:
            return t["cases"]
    raise KeyError(func)


def fixture_files(driver, fixtures):
    """testdata/fixtures/x.yaml of the driver -> tests/golden/fixtures/ospkg/<driver>/x.json"""
    out = []
    for f in fixtures or []:
        base = os.path.basename(f)[:-len(".yaml")]
        out.append(os.path.join(GOLDEN, "fixtures", "ospkg", driver, base + ".json"))
    return out


def os_detect_cases(driver):
    """[(id, fixture paths, family, os_ver, repo, pkgs, want, want_err, now)]"""
    out = []
    for c in table(f"detector__ospkg__{driver}__{driver}_test.json", "TestScanner_Detect"):
        fam = SUSE_FAMILY[c["distribution"]] if driver == "suse" else FAMILY[driver]
        a = c["args"]
        err = c.get("wantErr")
        if err is True:
            err = ""
        out.append((f"{driver}/{c['name']}", fixture_files(driver, c.get("fixtures")), fam, a.get("osVer", ""),
                    a.get("repo"), a.get("pkgs") or [], c.get("want") or [], err, parse_now(REF_NOW)))
    return out


def os_supported_cases(driver):
    """[(id, family, os_ver, now, want)]"""
    rel = f"detector__ospkg__{driver}__{driver}_test.json"
    try:
        cases = table(rel, "TestScanner_IsSupportedVersion")
    except KeyError:
        return []
    out = []
    for c in cases:
        if driver == "oracle":
            fam, ver, want = c["osFamily"], c["osVersion"], c["expected"]
        else:
            fam, ver, want = c["args"]["osFamily"], c["args"]["osVer"], c["want"]
        if driver == "suse":
            fam = SUSE_FAMILY.get(c.get("distribution"), fam)
        out.append((f"{driver}/{c['name']}", fam, ver, parse_now(c["now"]), want))
    return out
