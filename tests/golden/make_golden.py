#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/fixtures/.

This is TEST INFRASTRUCTURE.  It reads the reference's bolt-fixtures YAML data
files (DATA, not source) and re-emits them as JSON key/value records: the exact
records `dbtest.InitDB` (reference pkg/dbtest/db.go:17-36) would have put into
a temporary bbolt file through github.com/aquasecurity/bolt-fixtures
(go.mod:15).  bolt-fixtures decodes YAML into Go values and stores each leaf
`value:` as `json.Marshal(value)`; we reproduce that encoding:

* maps are emitted with sorted keys (Go's json.Marshal orders map keys);
* integral YAML floats (`Severity: 1.0`) become JSON integers, exactly as
  Go's float64 formatting would print them (SURVEY.md §8a′ "YAML numbers");
* YAML timestamps stay strings (go-yaml leaves them as strings when decoding
  into interface{}).

Output format: one JSON file per fixture, a list of records
    {"path": ["debian 9", "apache2", "CVE-2012-3499"], "value": "<json text>"}
where `path` is the bucket chain plus the final key.

The driver test tables (inputs / expected outputs of the reference's *_test.go) are
transcribed as data by tests/golden/extract_go_tables.py into tests/golden/tables/.

Usage:  python tests/golden/make_golden.py [/root/reference]
"""
import json
import math
import os
import re
import sys

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "fixtures")

# fixture directories (relative to the reference root) whose YAML we convert
FIXTURE_DIRS = [
    "pkg/detector/library/testdata/fixtures",
    "integration/testdata/fixtures/db",
    "pkg/vulnerability/testdata/fixtures",
]
OSPKG_ROOT = "pkg/detector/ospkg"


class _NoTimestampLoader(yaml.SafeLoader):
    """SafeLoader without the implicit timestamp resolver (go-yaml keeps them as strings)."""


_NoTimestampLoader.yaml_implicit_resolvers = {
    k: [(tag, rx) for tag, rx in v if tag != "tag:yaml.org,2002:timestamp"]
    for k, v in yaml.SafeLoader.yaml_implicit_resolvers.items()
}


def _go_json(v):
    """json.Marshal as Go would print the YAML-decoded value."""
    if isinstance(v, bool) or v is None or isinstance(v, str):
        return json.dumps(v, ensure_ascii=False)
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        if math.isfinite(v) and v == int(v) and abs(v) < 1e21:
            return str(int(v))
        return repr(v)
    if isinstance(v, list):
        return "[" + ",".join(_go_json(x) for x in v) + "]"
    if isinstance(v, dict):
        items = sorted((str(k), x) for k, x in v.items())
        return "{" + ",".join(json.dumps(k, ensure_ascii=False) + ":" + _go_json(x) for k, x in items) + "}"
    raise TypeError(type(v))


def _walk(node, prefix, out):
    for item in node or []:
        if "bucket" in item:
            _walk(item.get("pairs"), prefix + [str(item["bucket"])], out)
        else:
            out.append({"path": prefix + [str(item["key"])], "value": _go_json(item.get("value"))})


# A double-quoted block-sequence item followed by a stray ',' ends go-yaml's parse of
# the document there (integration/testdata/fixtures/db/vulnerability.yaml:1367): the
# goldens show the quoted URL kept (spring4shell-jre11.json.golden:246) and everything
# after it absent - that entry's PublishedDate/LastModifiedDate (same golden) and the
# whole CVE-2020-14155 record (conan.json.golden:149-159 has no detail, Severity UNKNOWN).
# PyYAML rejects the line, so the document is cut the same way before parsing.
_QUOTED_ITEM_COMMA = re.compile(r'^(\s*- "[^"\n]*"),\s*$', re.M)


def convert(path):
    with open(path, encoding="utf-8") as f:
        text = f.read()
    m = _QUOTED_ITEM_COMMA.search(text)
    if m:
        text = text[:m.start()] + m.group(1) + "\n"
    doc = yaml.load(text, Loader=_NoTimestampLoader)
    recs = []
    _walk(doc, [], recs)
    return recs


def main(ref="/root/reference"):
    jobs = []
    osroot = os.path.join(ref, OSPKG_ROOT)
    for drv in sorted(os.listdir(osroot)):
        d = os.path.join(osroot, drv, "testdata", "fixtures")
        if os.path.isdir(d):
            jobs.append((d, os.path.join("ospkg", drv)))
    for rel in FIXTURE_DIRS:
        tag = "library" if "library" in rel else "vulnerability" if "vulnerability" in rel else "integration"
        jobs.append((os.path.join(ref, rel), tag))
    n = 0
    for src_dir, tag in jobs:
        dst_dir = os.path.join(OUT, tag)
        os.makedirs(dst_dir, exist_ok=True)
        for fn in sorted(os.listdir(src_dir)):
            if not fn.endswith(".yaml"):
                continue
            try:
                recs = convert(os.path.join(src_dir, fn))
            except yaml.YAMLError as e:
                # integration/.../vulnerability.yaml (FillInfo data, out of scope) has a
                # trailing comma PyYAML rejects; skip it and say so.
                print(f"skip {tag}/{fn}: {str(e).splitlines()[0]}")
                continue
            with open(os.path.join(dst_dir, fn[:-5] + ".json"), "w", encoding="utf-8") as f:
                json.dump(recs, f, indent=1, ensure_ascii=False)
                f.write("\n")
            n += 1
    print(f"wrote {n} fixture files under {OUT}")


if __name__ == "__main__":
    main(*sys.argv[1:])
