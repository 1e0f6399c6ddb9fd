"""Ignore-file findings compiled against a batch (mirror of pkg/result/ignore.go
IgnoreConfig.MatchVulnerability for the batch result filter).

filterVulnerabilities (pkg/result/filter.go:117-122) drops a vulnerability into
ModifiedFindings when MatchVulnerability(ID, result Target, PkgPath, PURL) returns a
finding: the first finding, in file order, with that ID whose paths match (doublestar)
first the Target, then - a second pass over all findings - the PkgPath (no paths: any),
and whose PURLs match the package's PURL (no PURLs, or a package without a PURL: any;
purl.Match, pkg/purl/purl.go:249-274).

The host compiles the findings into three kinds of rules over the batch (tvm_ignore_rules),
each tagged with the precedence (pass << 31 | finding index) of the finding it came from;
the GPU takes, per pair, the smallest precedence among the rules that hit it, which is the
finding MatchVulnerability returns:
  * every package (no paths, no PURLs)                        -> ALL rules;
  * one package (PURLs: the packages whose PURL one matches,  -> PKG rules, resolved
    through a (type, namespace, name) index of the batch);
  * a class of packages: packages without a PURL (matchPURL,  -> CLS rules + one class per
    ignore.go:116-126) and, for findings with paths, the         package
    packages sharing (Target, PkgPath, has-PURL).
Rules grow with findings x classes and with true PURL matches, never with findings x
packages.  Expired findings must already be pruned (ParseIgnoreFile + Prune do that).
"""
import numpy as np

from . import glob
from .vex import PURL

PASS_PKGPATH = 1 << 31


class IgnoreRules:
    """tvm_ignore_rules for one batch: ids (distinct vulnerability IDs), rule arrays
    (uint32), pkg_class (uint32 per package or None)."""

    def __init__(self, n_pkgs):
        self.n_pkgs = n_pkgs
        self._ids = {}
        self.all_ = ([], [])
        self.pkg = ([], [], [])
        self.cls = ([], [], [])
        self.pkg_class = None

    def id_index(self, vid):
        return self._ids.setdefault(vid, len(self._ids))

    @property
    def ids(self):
        return list(self._ids)

    def arrays(self):
        u = lambda x: np.ascontiguousarray(x, dtype=np.uint32)  # noqa: E731
        return ([u(x) for x in self.all_], [u(x) for x in self.pkg], [u(x) for x in self.cls],
                None if self.pkg_class is None else u(self.pkg_class))

    def __len__(self):
        return len(self.all_[0]) + len(self.pkg[0]) + len(self.cls[0])


def compile_rules(findings, purls, results=None, pkg_paths=None):
    """IgnoreRules for a batch whose package i has the PURL string purls[i] (None: no PURL)
    and the PkgPath pkg_paths[i] (default ""); results = [(Target, begin, end)] covering the
    packages (needed only when a finding has paths).  findings: [{"ID", "Paths", "PURLs"
    (strings)}] in file order."""
    n = len(purls)
    rules = IgnoreRules(n)
    parsed = [PURL.parse(p) if p else None for p in purls]
    index = {}
    for i, p in enumerate(parsed):
        if p is not None:
            index.setdefault(p.base(), []).append(i)
    paths = pkg_paths if pkg_paths is not None else [""] * n
    with_paths = any(f.get("Paths") for f in findings)
    if with_paths:
        if results is None:
            raise ValueError("ignore findings with paths need the results' Target paths")
        target = [None] * n
        for t, b, e in results:
            target[b:e] = [t] * (e - b)
        if any(t is None for t in target):
            raise ValueError("results must cover every package")
        key = [(target[i], paths[i], parsed[i] is not None) for i in range(n)]
    else:
        key = [(None, None, parsed[i] is not None) for i in range(n)]
    classes = {}
    pkg_class = np.array([classes.setdefault(k, len(classes)) for k in key], dtype=np.uint32)
    used_cls = False
    for k, f in enumerate(findings):
        vid, pats = f["ID"], f.get("Paths") or []
        cons = []
        for s in f.get("PURLs") or []:
            c = PURL.parse(s)
            if c is None:
                raise ValueError("invalid PURL in ignore finding: " + s)
            cons.append(c)
        idx = rules.id_index(vid)
        if not pats and not cons:
            rules.all_[0].append(idx)
            rules.all_[1].append(k)
            continue
        # per class: the pass this finding matches in (0 Target / no paths, 1 PkgPath)
        cls_prec = {}
        for (tgt, ppath, has), c in classes.items():
            if not pats or glob.match_any(pats, tgt):
                cls_prec[c] = k
            elif glob.match_any(pats, ppath):
                cls_prec[c] = PASS_PKGPATH | k
        for (tgt, ppath, has), c in classes.items():
            if c in cls_prec and (not cons or not has):  # no PURL constraint, or a package without a PURL
                rules.cls[0].append(c)
                rules.cls[1].append(idx)
                rules.cls[2].append(cls_prec[c])
                used_cls = True
        if cons:  # packages with a PURL that one constraint matches (their class decides the pass)
            hit = set()
            for c in cons:
                hit.update(i for i in index.get(c.base(), ()) if c.trivy_matches(parsed[i]))
            for i in sorted(hit):
                prec = cls_prec.get(int(pkg_class[i]))
                if prec is not None:
                    rules.pkg[0].append(i)
                    rules.pkg[1].append(idx)
                    rules.pkg[2].append(prec)
    if used_cls:
        rules.pkg_class = pkg_class
    return rules


def plain_rules(ids, n_pkgs):
    """IgnoreRules of a .trivyignore without paths / PURLs: ALL rules in file order."""
    rules = IgnoreRules(n_pkgs)
    for k, vid in enumerate(ids):
        rules.all_[0].append(rules.id_index(vid))
        rules.all_[1].append(k)
    return rules
