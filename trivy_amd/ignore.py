"""Ignore-file findings compiled against a batch (mirror of pkg/result/ignore.go
IgnoreConfig.MatchVulnerability for the batch result filter).

filterVulnerabilities (pkg/result/filter.go:117-122) drops a vulnerability when the
ignore file holds a finding with its ID whose paths match the target or the package path
(no paths: any) and whose PURLs match the package (no PURLs: any; trivy purl.Match,
pkg/purl/purl.go:249-274).  On the batch path packages carry no PkgPath and results no
target path, so:
  * findings without paths or PURLs   -> plain IDs (tvm_filter_opts.ignore_ids);
  * findings with PURLs, no paths     -> (package, ID) pairs for the packages whose PURL
                                         one of the finding's PURLs matches, and for every
                                         package without a PURL (matchPURL, :116-126)
                                         (tvm_filter_opts.ignore_pair_*), resolved through
                                         a (type, namespace, name) index of the batch;
  * findings with paths               -> rejected (they need the target / package path).
Expired findings must already be pruned (ParseIgnoreFile + Prune do that).
"""
import numpy as np

from .vex import PURL


def split_findings(findings, purls):
    """(plain IDs, (package indices uint32, IDs)) for the batch whose package i has the PURL
    string purls[i] (None: no PURL).  findings: [{"ID", "Paths", "PURLs" (strings)}]."""
    plain, pairs = [], set()
    index = {}
    parsed = [PURL.parse(p) if p else None for p in purls]
    no_purl = [i for i, p in enumerate(parsed) if p is None]
    for i, p in enumerate(parsed):
        if p is not None:
            index.setdefault(p.base(), []).append(i)
    for f in findings:
        if f.get("Paths"):
            raise ValueError("ignore findings with paths need the target / package path: not on the batch path")
        if not f.get("PURLs"):
            plain.append(f["ID"])
            continue
        for s in f["PURLs"]:
            c = PURL.parse(s)
            if c is None:
                raise ValueError("invalid PURL in ignore finding: " + s)
            pairs.update((i, f["ID"]) for i in index.get(c.base(), ()) if c.trivy_matches(parsed[i]))
        # matchPURL (ignore.go:116-126): a package without a PURL is matched by any finding
        pairs.update((i, f["ID"]) for i in no_purl)
    items = sorted(pairs)
    return plain, (np.array([p for p, _ in items], dtype=np.uint32), [v for _, v in items])
