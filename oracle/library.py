"""ORACLE - TEST INFRASTRUCTURE ONLY.

Direct (pairwise, no sort keys, no interval algebra) restatement of the reference's
library detection path, used by tests/ as the checker of the GPU product:

  pkg/detector/library/driver.go:25-93    NewDriver: LangType -> (ecosystem, comparer)
  pkg/detector/library/driver.go:111-159  DetectVulnerabilities, createFixedVersions
  pkg/detector/library/detect.go:11-42    Detect / detect (Layer, PkgPath, PkgIdentifier)
  pkg/detector/library/compare/compare.go:21-78 and */compare.go   IsVulnerable + matchVersion
and the third-party modules those call (absent here; published algorithms restated,
pinned by the reference's compare_test.go tables, driver_test.go and the integration
fixtures/goldens - every choice no reference vector pins is marked UNPINNED):

  GENERIC  github.com/aquasecurity/go-version v0.0.0-20210121072130-637058cfe492 (go.mod:19)
  NPM      github.com/aquasecurity/go-npm-version v0.0.0-20201110091526-0b796d180798 (go.mod:17)
  PEP440   github.com/aquasecurity/go-pep440-version v0.0.0-20210121094942-22b2f8951d46 (go.mod:18)
  MAVEN    github.com/masahiro331/go-mvn-version v0.0.0-20210429150710-d3157d602a08 (go.mod:73)
  GEM      github.com/aquasecurity/go-gem-version v0.0.0-20201115065557-8eed6fe000ce (go.mod:16)
  BITNAMI  github.com/bitnami/go-version v0.0.0-20231130084017-bb00604d650c (go.mod:37)
  trivy-db GetAdvisories prefix scan + vulnerability.NormalizePkgName (go.mod:25)
"""
import functools
import json
import re

from .drivers import DecodeError, decode_advisory


class VersionError(Exception):
    pass


class ConstraintError(Exception):
    pass


def _cmp(a, b):
    return (a > b) - (a < b)


# ===================================================================== GENERIC ======
# hashicorp-style version: v?N(.N)*, pre-release "-ident(.ident)*" (or starting with a
# letter without the dash), build metadata "+..." ignored for ordering.
_GEN_RE = re.compile(r"^v?([0-9]+(?:\.[0-9]+)*)"
                     r"(?:-([0-9A-Za-z\-~]+(?:\.[0-9A-Za-z\-~]+)*)|([A-Za-z\-~][0-9A-Za-z\-~]*(?:\.[0-9A-Za-z\-~]+)*))?"
                     r"(?:\+([0-9A-Za-z\-~]+(?:\.[0-9A-Za-z\-~]+)*))?$")
_GEN_VER = (r"v?[0-9]+(?:\.[0-9]+)*(?:-[0-9A-Za-z\-~]+(?:\.[0-9A-Za-z\-~]+)*|[A-Za-z\-~][0-9A-Za-z\-~]*"
            r"(?:\.[0-9A-Za-z\-~]+)*)?(?:\+[0-9A-Za-z\-~]+(?:\.[0-9A-Za-z\-~]+)*)?")
U64 = 2 ** 64 - 1


class GenVer:
    def __init__(self, s, revision_dash=False):
        m = _GEN_RE.match(s)
        if not m:
            raise VersionError(f"malformed version: {s}")
        self.segs = [int(x) for x in m.group(1).split(".")]
        if any(x > U64 for x in self.segs):
            raise VersionError(f"malformed version: {s}")
        pre = m.group(2) if m.group(2) is not None else m.group(3)
        self.rev = 0
        if revision_dash and m.group(2) is not None and m.group(2).isdigit():
            # bitnami: "-N" is a package revision, not a pre-release (UNPINNED: rev 0 == none)
            self.rev, pre = int(m.group(2)), None
        self.pre = pre.split(".") if pre else []

    def key_tuple(self):
        return self.segs

    def compare(self, o):
        n = max(len(self.segs), len(o.segs))
        a = self.segs + [0] * (n - len(self.segs))
        b = o.segs + [0] * (n - len(o.segs))
        if a != b:
            return _cmp(a, b)
        c = _cmp_pre(self.pre, o.pre)
        if c:
            return c
        return _cmp(self.rev, o.rev)


def _cmp_ident(x, y):
    xn, yn = x.isdigit(), y.isdigit()
    if xn and yn:
        return _cmp(int(x), int(y))
    if xn != yn:
        return -1 if xn else 1
    return _cmp(x, y)


def _cmp_pre(a, b):
    """semver pre-release precedence: none > some; identifiers numeric < alphanumeric."""
    if not a and not b:
        return 0
    if not a:
        return 1
    if not b:
        return -1
    for x, y in zip(a, b):
        c = _cmp_ident(x, y)
        if c:
            return c
    return _cmp(len(a), len(b))


def _bump(segs, prefix_len):
    """The version just above every version whose first prefix_len segments equal segs'."""
    s = list(segs[:prefix_len])
    s[-1] += 1
    return s


def _gen_op_check(op, v, c, specified):
    """One go-version comparator.  specified = number of segments written in c."""
    cmpv = v.compare(c)
    if op in ("", "=", "=="):
        return cmpv == 0
    if op == "!=":
        return cmpv != 0
    if op == ">":
        return cmpv > 0
    if op == "<":
        return cmpv < 0
    if op in (">=", "=>"):
        return cmpv >= 0
    if op in ("<=", "=<"):
        return cmpv <= 0
    segs = c.segs[:specified]
    if op == "~>":
        # pessimistic (UNPINNED): >= c and < c with its second-to-last written segment bumped
        if cmpv < 0:
            return False
        n = max(1, specified - 1)
        return _lt_segs(v, _bump(segs, n))
    if op == "~":
        # tilde (UNPINNED): >= c, < next minor (or next major when only the major is written)
        if cmpv < 0:
            return False
        return _lt_segs(v, _bump(segs, 2 if specified >= 2 else 1))
    if op == "^":
        # caret (UNPINNED): >= c, < bump of the first non-zero written segment
        if cmpv < 0:
            return False
        i = 0
        while i < specified - 1 and segs[i] == 0:
            i += 1
        return _lt_segs(v, _bump(segs, i + 1))
    raise ConstraintError(op)


def _lt_segs(v, upper):
    """v < upper.0.0... as a release with the lowest possible pre-release (all of upper's
    pre-releases are excluded too)."""
    n = max(len(v.segs), len(upper))
    a = v.segs + [0] * (n - len(v.segs))
    b = upper + [0] * (n - len(upper))
    return a < b


_GEN_OPS = ["~>", ">=", "=>", "<=", "=<", "!=", "==", ">", "<", "=", "~", "^", ""]
_GEN_OPS_RE = "|".join(re.escape(o) for o in _GEN_OPS)
_GEN_VALID = re.compile(r"^\s*(\s*(" + _GEN_OPS_RE + r")\s*(" + _GEN_VER + r")\s*,?)*\s*$")
_GEN_ONE = re.compile(r"(" + _GEN_OPS_RE + r")\s*(" + _GEN_VER + r")")


def _specified(vs):
    vs = vs[1:] if vs.startswith("v") else vs
    m = re.match(r"[0-9]+(?:\.[0-9]+)*", vs)
    return len(m.group(0).split("."))


def gen_match(ver, constraint, revision_dash=False):
    v = GenVer(ver, revision_dash)
    alts = []
    for alt in constraint.split("||"):
        if not _GEN_VALID.match(alt):
            raise ConstraintError(f"improper constraint: {alt}")
        cs = []
        for op, vs in _GEN_ONE.findall(alt):
            cs.append((op, GenVer(vs, revision_dash), _specified(vs)))
        alts.append(cs)
    return any(all(_gen_op_check(op, v, c, n) for op, c, n in cs) for cs in alts)


# ========================================================================= NPM ======
# node-semver ranges (no includePrerelease): ||, whitespace/comma AND, hyphen ranges,
# x-ranges, ~ and ^, and the pre-release rule: a version with a pre-release tag only
# satisfies a comparator set that holds a comparator with a pre-release on the same
# [major, minor, patch].
_NPM_VER = re.compile(r"^\s*[v=]*\s*([0-9]+)\.([0-9]+)\.([0-9]+)"
                      r"(?:-?([0-9A-Za-z\-]+(?:\.[0-9A-Za-z\-]+)*))?(?:\+([0-9A-Za-z\-]+(?:\.[0-9A-Za-z\-]+)*))?\s*$")


class NpmVer:
    def __init__(self, s):
        m = _NPM_VER.match(s)
        if not m:
            raise VersionError(f"invalid semantic version: {s}")
        self.t = (int(m.group(1)), int(m.group(2)), int(m.group(3)))
        if max(self.t) > U64:  # UNPINNED: numeric fields are 64-bit
            raise VersionError(f"invalid semantic version: {s}")
        self.pre = m.group(4).split(".") if m.group(4) else []

    @staticmethod
    def make(t, pre):
        v = NpmVer.__new__(NpmVer)
        v.t, v.pre = tuple(t), list(pre)
        return v

    def compare(self, o):
        if self.t != o.t:
            return _cmp(self.t, o.t)
        return _cmp_pre(self.pre, o.pre)


_XR = r"(?:x|X|\*|[0-9]+)"
_PARTIAL = re.compile(r"^[v=]*(" + _XR + r")(?:\.(" + _XR + r")(?:\.(" + _XR + r")"
                      r"(?:-?([0-9A-Za-z\-]+(?:\.[0-9A-Za-z\-]+)*))?(?:\+[0-9A-Za-z\-]+(?:\.[0-9A-Za-z\-]+)*)?)?)?$")


def _partial(s):
    m = _PARTIAL.match(s)
    if not m:
        raise ConstraintError(f"invalid comparator: {s}")
    parts = [m.group(1), m.group(2), m.group(3)]
    nums = []
    for p in parts:
        if p is None or p in ("x", "X", "*"):
            break
        nums.append(int(p))
    pre = m.group(4).split(".") if (m.group(4) and len(nums) == 3) else []
    return nums, pre


def _cmp_lo(op, nums, pre):
    """Desugar one primitive comparator to (op, NpmVer) list."""
    n = len(nums)
    if n == 0:
        return [(">=", NpmVer.make((0, 0, 0), []))] if op in ("", "=", ">=", "<=") else \
            ([("<", NpmVer.make((0, 0, 0), ["0"]))] if op in ("<", ">") else [])
    full = nums + [0] * (3 - n)
    if n == 3:
        return [(op or "=", NpmVer.make(full, pre))]
    up = list(nums)
    up[-1] += 1
    up = up + [0] * (3 - n)
    if op in ("", "="):
        return [(">=", NpmVer.make(full, [])), ("<", NpmVer.make(up, ["0"]))]
    if op == ">":
        return [(">=", NpmVer.make(up, []))]
    if op == ">=":
        return [(">=", NpmVer.make(full, []))]
    if op == "<":
        return [("<", NpmVer.make(full, ["0"]))]
    if op == "<=":
        return [("<", NpmVer.make(up, ["0"]))]
    raise ConstraintError(op)


def _tilde(nums, pre):
    n = len(nums)
    if n == 0:
        return [(">=", NpmVer.make((0, 0, 0), []))]
    full = nums + [0] * (3 - n)
    up = [nums[0] + 1, 0, 0] if n == 1 else [nums[0], nums[1] + 1, 0]
    return [(">=", NpmVer.make(full, pre if n == 3 else [])), ("<", NpmVer.make(up, ["0"]))]


def _caret(nums, pre):
    n = len(nums)
    if n == 0:
        return [(">=", NpmVer.make((0, 0, 0), []))]
    full = nums + [0] * (3 - n)
    if nums[0] != 0 or n == 1:
        up = [nums[0] + 1, 0, 0]
    elif n == 2 or nums[1] != 0:
        up = [0, nums[1] + 1, 0]
    else:
        up = [0, 0, nums[2] + 1]
    return [(">=", NpmVer.make(full, pre if n == 3 else [])), ("<", NpmVer.make(up, ["0"]))]


_NPM_TOKEN = re.compile(r"(<=|>=|<|>|=|~>|~|\^)?\s*([^\s<>=~^,]+)")


def _npm_set(s):
    s = s.replace(",", " ").strip()
    hy = re.match(r"^(\S+)\s+-\s+(\S+)$", s)
    if hy:
        lo, lpre = _partial(hy.group(1))
        hi, hpre = _partial(hy.group(2))
        out = [(">=", NpmVer.make(lo + [0] * (3 - len(lo)), lpre if len(lo) == 3 else []))] if lo else []
        if len(hi) == 3:
            out.append(("<=", NpmVer.make(hi, hpre)))
        elif hi:
            up = list(hi)
            up[-1] += 1
            out.append(("<", NpmVer.make(up + [0] * (3 - len(hi)), ["0"])))
        return out or [(">=", NpmVer.make((0, 0, 0), []))]
    out = []
    pos = 0
    s2 = s
    while pos < len(s2):
        while pos < len(s2) and s2[pos].isspace():
            pos += 1
        if pos >= len(s2):
            break
        m = _NPM_TOKEN.match(s2, pos)
        if not m or m.end() == pos:
            raise ConstraintError(f"invalid range: {s}")
        op, ver = m.group(1) or "", m.group(2)
        nums, pre = _partial(ver)
        if op in ("~", "~>"):
            out += _tilde(nums, pre)
        elif op == "^":
            out += _caret(nums, pre)
        else:
            out += _cmp_lo(op, nums, pre)
        pos = m.end()
    return out or [(">=", NpmVer.make((0, 0, 0), []))]


def _npm_test(op, v, c):
    r = v.compare(c)
    return {"=": r == 0, "": r == 0, "<": r < 0, "<=": r <= 0, ">": r > 0, ">=": r >= 0}[op]


def npm_match(ver, constraint):
    v = NpmVer(ver)
    sets = [_npm_set(alt) for alt in constraint.split("||")]  # NewConstraints parses every set first
    for cs in sets:
        if not all(_npm_test(op, v, c) for op, c in cs):
            continue
        if v.pre and not any(c.pre and c.t == v.t for _, c in cs):
            continue
        return True
    return False


# ====================================================================== PEP 440 ======
_PEP_RE = re.compile(
    r"^\s*v?(?:(?P<epoch>[0-9]+)!)?(?P<release>[0-9]+(?:\.[0-9]+)*)"
    r"(?P<pre>[-_\.]?(?P<pre_l>alpha|a|beta|b|preview|pre|c|rc)[-_\.]?(?P<pre_n>[0-9]+)?)?"
    r"(?P<post>(?:-(?P<post_n1>[0-9]+))|(?:[-_\.]?(?P<post_l>post|rev|r)[-_\.]?(?P<post_n2>[0-9]+)?))?"
    r"(?P<dev>[-_\.]?(?P<dev_l>dev)[-_\.]?(?P<dev_n>[0-9]+)?)?"
    r"(?:\+(?P<local>[a-z0-9]+(?:[-_\.][a-z0-9]+)*))?\s*$", re.I)
_PRE_NORM = {"a": 0, "alpha": 0, "b": 1, "beta": 1, "c": 2, "rc": 2, "pre": 2, "preview": 2}


class PepVer:
    def __init__(self, s):
        m = _PEP_RE.match(s)
        if not m:
            raise VersionError(f"malformed version: {s}")
        self.epoch = int(m.group("epoch") or 0)
        self.release = [int(x) for x in m.group("release").split(".")]
        self.pre = (_PRE_NORM[m.group("pre_l").lower()], int(m.group("pre_n") or 0)) if m.group("pre_l") else None
        if m.group("post"):
            self.post = int(m.group("post_n1") or m.group("post_n2") or 0)
        else:
            self.post = None
        self.dev = int(m.group("dev_n") or 0) if m.group("dev_l") else None
        nums = [self.epoch] + self.release + [x for x in (self.pre and self.pre[1], self.post, self.dev) if x]
        if max(nums) > U64:  # UNPINNED: numeric fields are 64-bit
            raise VersionError(f"malformed version: {s}")
        loc = m.group("local")
        self.local = tuple(int(x) if x.isdigit() else x.lower() for x in re.split(r"[-_\.]", loc)) if loc else None

    @property
    def is_prerelease(self):
        return self.pre is not None or self.dev is not None

    @property
    def is_postrelease(self):
        return self.post is not None

    def base(self):
        r = list(self.release)
        while len(r) > 1 and r[-1] == 0:
            r.pop()
        return (self.epoch, tuple(r))

    def public_key(self):
        r = list(self.release)
        while r and r[-1] == 0:
            r.pop()
        if self.pre is None and self.post is None and self.dev is not None:
            pre = (-1,)
        elif self.pre is None:
            pre = (3,)
        else:
            pre = (1,) + self.pre
        post = (0,) if self.post is None else (1, self.post)
        dev = (2,) if self.dev is None else (1, self.dev)
        return (self.epoch, tuple(r), pre, post, dev)

    def key(self):
        if self.local is None:
            loc = (0,)
        else:
            loc = (1,) + tuple((1, x, "") if isinstance(x, int) else (0, 0, x) for x in self.local)
        return self.public_key() + (loc,)

    def compare(self, o):
        return _cmp(self.key(), o.key())


def _pep_prefix_match(v, spec_ver):
    """==V.* : same epoch and v's zero-padded release starts with V's release."""
    s = PepVer(spec_ver)
    if v.epoch != s.epoch:
        return False
    n = len(s.release)
    r = v.release + [0] * max(0, n - len(v.release))
    return r[:n] == s.release


def _pep_check(op, v, spec):
    if spec == "*":
        return True
    if op == "~=":
        s = PepVer(spec)
        if len(s.release) < 2:
            raise ConstraintError("~= needs two release segments")
        prefix = ".".join(str(x) for x in s.release[:-1])
        if s.epoch:
            prefix = f"{s.epoch}!{prefix}"
        return _pep_check(">=", v, spec) and _pep_prefix_match(v, prefix)
    if op in ("==", "!=") and spec.endswith(".*"):
        r = _pep_prefix_match(v, spec[:-2])
        return r if op == "==" else not r
    s = PepVer(spec)
    if op in ("==", "!=", "==="):
        if op == "===":
            r = v.compare(s) == 0  # UNPINNED: arbitrary equality approximated by version equality
            return r
        if s.local is None:
            r = v.public_key() == s.public_key()
        else:
            r = v.key() == s.key()
        return r if op == "==" else not r
    pv = v.public_key()
    if op == "<=":
        return pv <= s.public_key()
    if op == ">=":
        return pv >= s.public_key()
    if op == "<":
        if not v.compare(s) < 0:
            return False
        if not s.is_prerelease and v.is_prerelease and v.base() == s.base():
            return False
        return True
    if op == ">":
        if not v.compare(s) > 0:
            return False
        if not s.is_postrelease and v.is_postrelease and v.base() == s.base():
            return False
        if v.local is not None and v.base() == s.base():
            return False
        return True
    raise ConstraintError(op)


_PEP_SPEC = re.compile(r"\s*(~=|===|==|!=|<=|>=|<|>)?\s*([^\s,<>=!~]+)\s*")


def pep_match(ver, constraint):
    v = PepVer(ver)
    alts = []
    for alt in constraint.split("||"):
        a = alt.strip()
        cs = []
        if a == "*":
            cs.append(("==", "*"))
        else:
            pos = 0
            while pos < len(a):
                if a[pos] in ", ":
                    pos += 1
                    continue
                m = _PEP_SPEC.match(a, pos)
                if not m:
                    raise ConstraintError(f"improper constraint: {alt}")
                sv = m.group(2)
                op = m.group(1) or "=="
                # NewSpecifiers validates every specifier up front
                pv = PepVer(sv[:-2] if sv.endswith(".*") else sv)
                if op == "~=" and len(pv.release) < 2:
                    raise ConstraintError(f"~= needs two release segments: {sv}")
                cs.append((op, sv))
                pos = m.end()
        if not cs:
            raise ConstraintError(f"improper constraint: {alt}")
        alts.append(cs)
    return any(all(_pep_check(op, v, s) for op, s in cs) for cs in alts)


# ======================================================================== MAVEN ======
# org.apache.maven.artifact.versioning.ComparableVersion (Maven 3), as ported by
# go-mvn-version: items are ints, qualifier strings and sub-lists ('-' or digit/letter
# transitions open a sub-list); trailing nulls are removed; comparison pads with null.
_QUALS = ["alpha", "beta", "milestone", "rc", "snapshot", "", "sp"]
_ALIAS = {"ga": "", "final": "", "release": "", "cr": "rc"}


class _MInt:
    def __init__(self, v):
        self.v = v

    def is_null(self):
        return self.v == 0


class _MStr:
    def __init__(self, s, followed_by_digit):
        if followed_by_digit and len(s) == 1:
            s = {"a": "alpha", "b": "beta", "m": "milestone"}.get(s, s)
        self.s = _ALIAS.get(s, s)

    def is_null(self):
        return self.s == ""

    def qkey(self):
        return str(_QUALS.index(self.s)) if self.s in _QUALS else f"{len(_QUALS)}-{self.s}"


class _MList(list):
    def is_null(self):
        return len(self) == 0

    def normalize(self):
        for i in range(len(self) - 1, -1, -1):
            it = self[i]
            if it.is_null():
                del self[i]
            elif not isinstance(it, _MList):
                break


def _m_item(is_digit, buf):
    return _MInt(int(buf)) if is_digit else _MStr(buf, False)


def mvn_parse(version):
    version = version.lower()
    items = lst = _MList()
    stack = [lst]
    is_digit = False
    start = 0
    for i, c in enumerate(version):
        if c == ".":
            lst.append(_MInt(0) if i == start else _m_item(is_digit, version[start:i]))
            start = i + 1
        elif c == "-":
            lst.append(_MInt(0) if i == start else _m_item(is_digit, version[start:i]))
            start = i + 1
            nl = _MList()
            lst.append(nl)
            lst = nl
            stack.append(lst)
        elif c.isdigit() and c.isascii():
            if not is_digit and i > start:
                lst.append(_MStr(version[start:i], True))
                start = i
                nl = _MList()
                lst.append(nl)
                lst = nl
                stack.append(lst)
            is_digit = True
        else:
            if is_digit and i > start:
                lst.append(_m_item(True, version[start:i]))
                start = i
                nl = _MList()
                lst.append(nl)
                lst = nl
                stack.append(lst)
            is_digit = False
    if len(version) > start:
        lst.append(_m_item(is_digit, version[start:]))
    while stack:
        stack.pop().normalize()
    return items


def _m_cmp(a, b):
    """Item.compareTo; a is an item (never None), b may be None."""
    if isinstance(a, _MInt):
        if b is None:
            return 0 if a.v == 0 else 1
        if isinstance(b, _MInt):
            return _cmp(a.v, b.v)
        return 1
    if isinstance(a, _MStr):
        if b is None:
            return _cmp(a.qkey(), _MStr("", False).qkey())
        if isinstance(b, _MInt):
            return -1
        if isinstance(b, _MStr):
            return _cmp(a.qkey(), b.qkey())
        return -1
    # list
    if b is None:
        return 0 if len(a) == 0 else _m_cmp(a[0], None)
    if isinstance(b, _MInt):
        return -1
    if isinstance(b, _MStr):
        return 1
    for i in range(max(len(a), len(b))):
        x = a[i] if i < len(a) else None
        y = b[i] if i < len(b) else None
        r = (0 if y is None else -_m_cmp(y, None)) if x is None else _m_cmp(x, y)
        if r:
            return r
    return 0


_MVN_VALID = re.compile(r"^[0-9A-Za-z][0-9A-Za-z.\-_+]*$")


class MvnVer:
    def __init__(self, s):
        s = s.strip()
        if not _MVN_VALID.match(s):
            raise VersionError(f"malformed version: {s}")
        self.items = mvn_parse(s)

    def compare(self, o):
        return _m_cmp(self.items, o.items)


_MVN_TOK = re.compile(r"(>=|<=|!=|==|=|>|<)?\s*([^\s<>=!,]+)")


def _mvn_ranges(spec):
    """Maven range spec "[a,b),(c,]" -> list of (lo, lo_incl, hi, hi_incl) (None = unbounded)."""
    out = []
    pos = 0
    s = spec.strip()
    while pos < len(s):
        if s[pos] in ", ":
            pos += 1
            continue
        if s[pos] not in "[(":
            raise ConstraintError(f"bad range: {spec}")
        end = min([i for i in (s.find("]", pos), s.find(")", pos)) if i >= 0] or [-1])
        if end < 0:
            raise ConstraintError(f"bad range: {spec}")
        body = s[pos + 1:end]
        lo_incl, hi_incl = s[pos] == "[", s[end] == "]"
        if "," in body:
            lo, hi = [x.strip() for x in body.split(",", 1)]
            out.append((MvnVer(lo) if lo else None, lo_incl, MvnVer(hi) if hi else None, hi_incl))
        else:
            if not (lo_incl and hi_incl) or not body.strip():
                raise ConstraintError(f"bad range: {spec}")
            v = MvnVer(body)
            out.append((v, True, v, True))
        pos = end + 1
    return out


def mvn_match(ver, constraint):
    v = MvnVer(ver)
    alts = []
    for alt in constraint.split("||"):
        a = alt.strip()
        if a.startswith("[") or a.startswith("("):
            alts.append(("range", _mvn_ranges(a)))
            continue
        cs = []
        pos = 0
        while pos < len(a):
            if a[pos] in ", \t":
                pos += 1
                continue
            m = _MVN_TOK.match(a, pos)
            if not m:
                raise ConstraintError(f"improper constraint: {alt}")
            cs.append((m.group(1) or "=", MvnVer(m.group(2))))
            pos = m.end()
        if not cs:
            raise ConstraintError(f"improper constraint: {alt}")
        alts.append(("ops", cs))
    for kind, body in alts:
        if kind == "range":
            for lo, li, hi, hi_i in body:
                ok = lo is None or (v.compare(lo) >= 0 if li else v.compare(lo) > 0)
                ok = ok and (hi is None or (v.compare(hi) <= 0 if hi_i else v.compare(hi) < 0))
                if ok:
                    return True
        else:
            if all({"=": v.compare(c) == 0, "==": v.compare(c) == 0, "!=": v.compare(c) != 0,
                    ">": v.compare(c) > 0, "<": v.compare(c) < 0, ">=": v.compare(c) >= 0,
                    "<=": v.compare(c) <= 0}[op] for op, c in body):
                return True
    return False


# ====================================================================== RUBYGEMS ======
_GEM_RE = re.compile(r"^\s*([0-9]+(?:\.[0-9a-zA-Z]+)*(?:-[0-9A-Za-z-]+(?:\.[0-9A-Za-z-]+)*)?)?\s*$")


class GemVer:
    def __init__(self, s):
        m = _GEM_RE.match(s)
        if not m:
            raise VersionError(f"Malformed version number string {s}")
        v = (m.group(1) or "0").replace("-", ".pre.")
        self.segments = [int(x) if x.isdigit() else x for x in re.findall(r"[0-9]+|[a-zA-Z]+", v)]
        self.prerelease = bool(re.search(r"[a-zA-Z]", v))

    def canonical(self):
        idx = next((i for i, s in enumerate(self.segments) if isinstance(s, str)), len(self.segments))
        num, strs = self.segments[:idx], self.segments[idx:]
        while num and num[-1] == 0:
            num.pop()
        while strs and strs[-1] == 0:
            strs.pop()
        return num + strs

    def compare(self, o):
        a, b = self.canonical(), o.canonical()
        for i in range(max(len(a), len(b))):
            x = a[i] if i < len(a) else 0
            y = b[i] if i < len(b) else 0
            if x == y:
                continue
            if isinstance(x, str) and not isinstance(y, str):
                return -1
            if not isinstance(x, str) and isinstance(y, str):
                return 1
            return _cmp(x, y)
        return 0

    def release(self):
        r = GemVer.__new__(GemVer)
        r.segments = [s for s in self.segments[:next((i for i, s in enumerate(self.segments) if isinstance(s, str)),
                                                       len(self.segments))]]
        r.prerelease = False
        return r

    def bump(self):
        segs = list(self.segments)
        while any(isinstance(s, str) for s in segs):
            segs.pop()
        if len(segs) > 1:
            segs.pop()
        segs[-1] += 1
        r = GemVer.__new__(GemVer)
        r.segments, r.prerelease = segs, False
        return r


_GEM_REQ = re.compile(r"^\s*(=|!=|>=|<=|>|<|~>)?\s*(\S.*?)\s*$")


def gem_match(ver, constraint):
    v = GemVer(ver)
    alts = []
    for alt in constraint.split("||"):
        cs = []
        for part in alt.split(","):
            m = _GEM_REQ.match(part)
            if not m:
                raise ConstraintError(f"Illformed requirement [{part}]")
            cs.append((m.group(1) or "=", GemVer(m.group(2))))
        alts.append(cs)

    def ok(op, r):
        c = v.compare(r)
        if op == "~>":
            return c >= 0 and v.release().compare(r.bump()) < 0
        return {"=": c == 0, "!=": c != 0, ">": c > 0, "<": c < 0, ">=": c >= 0, "<=": c <= 0}[op]
    return any(all(ok(op, r) for op, r in cs) for cs in alts)


# ======================================================================= BITNAMI ======
def bitnami_match(ver, constraint):
    return gen_match(ver, constraint, revision_dash=True)


MATCHERS = {"generic": gen_match, "npm": npm_match, "pep440": pep_match, "maven": mvn_match, "gem": gem_match,
            "bitnami": bitnami_match}


def match(grammar, ver, constraint):
    """matchVersion: (bool, error) -> True/False, raising on a parse error."""
    return MATCHERS[grammar](ver, constraint)


def is_vulnerable(grammar, ver, adv):
    """compare.IsVulnerable (compare.go:21-55)."""
    vuln = adv.get("VulnerableVersions") or []
    patched = adv.get("PatchedVersions") or []
    unaffected = adv.get("UnaffectedVersions") or []
    if any(v == "" for v in vuln + patched):
        return True
    matched = False
    if vuln:
        try:
            matched = match(grammar, ver, " || ".join(vuln))
        except (VersionError, ConstraintError):
            return False
        if not matched:
            return False
    secure = patched + unaffected
    if not secure:
        return matched
    try:
        return not match(grammar, ver, " || ".join(secure))
    except (VersionError, ConstraintError):
        return False


def create_fixed_versions(adv):
    """driver.go:139-159."""
    def uniq_join(xs):
        out = []
        for x in xs:
            if x not in out:
                out.append(x)
        return ", ".join(out)
    if adv.get("PatchedVersions"):
        return uniq_join(adv["PatchedVersions"])
    fixed = []
    for v in adv.get("VulnerableVersions") or []:
        for s in v.split(","):
            s = s.strip()
            if not s.startswith("<=") and s.startswith("<"):
                fixed.append(s[1:].strip())
    return uniq_join(fixed)


# LangType -> (ecosystem, grammar) (driver.go:25-93)
LANG = {}
for _t in ("bundler", "gemspec"):
    LANG[_t] = ("rubygems", "gem")
for _t in ("rustbinary", "cargo"):
    LANG[_t] = ("cargo", "generic")
LANG["composer"] = ("composer", "generic")
for _t in ("gobinary", "gomod"):
    LANG[_t] = ("go", "generic")
for _t in ("jar", "pom", "gradle"):
    LANG[_t] = ("maven", "maven")
for _t in ("npm", "yarn", "pnpm", "node-pkg", "javascript"):
    LANG[_t] = ("npm", "npm")
for _t in ("nuget", "dotnet-core", "packages-props"):
    LANG[_t] = ("nuget", "generic")
for _t in ("pipenv", "poetry", "pip", "python-pkg"):
    LANG[_t] = ("pip", "pep440")
LANG["pub"] = ("pub", "generic")
LANG["hex"] = ("erlang", "generic")
LANG["conan"] = ("conan", "generic")
LANG["swift"] = ("swift", "generic")
LANG["cocoapods"] = ("cocoapods", "gem")
LANG["bitnami"] = ("bitnami", "bitnami")
LANG["kubernetes"] = ("k8s", "generic")


def normalize_pkg_name(eco, name):
    """trivy-db vulnerability.NormalizePkgName: pip names lower-cased, '_' -> '-'."""
    if eco == "pip":
        return name.lower().replace("_", "-")
    return name


def get_advisories_prefix(db, prefix, name):
    """trivy-db ForEachAdvisory over every root bucket starting with prefix (bbolt key
    order); a later root overwrites an earlier one for the same vulnID; then
    GetAdvisories decodes each value (first error fails the call)."""
    values = {}
    for (kind, root), node in sorted(db.tree.items(), key=lambda kv: kv[0][1].encode()):
        if kind != "b" or not root.startswith(prefix):
            continue
        b = node.get(("b", name))
        if not b:
            continue
        src = db.data_source(root)
        for (k2, vid), val in sorted(b.items(), key=lambda kv: kv[0][1].encode()):
            if k2 != "k" or val == "":
                continue
            values[vid] = (val, src)
    out = []
    for vid in sorted(values, key=lambda x: x.encode()):
        val, src = values[vid]
        a = decode_advisory(val)
        a["VulnerabilityID"] = vid
        if src:
            a["DataSource"] = src
        elif "DataSource" in a:
            a["DataSource"] = {k: a["DataSource"][k] for k in ("ID", "Name", "URL") if a["DataSource"].get(k)}
        out.append(a)
    return out


def detect_vulnerabilities(db, lang, pkg_id, name, ver):
    """(*Driver).DetectVulnerabilities (driver.go:111-137)."""
    eco, grammar = LANG[lang]
    try:
        advs = get_advisories_prefix(db, eco + "::", normalize_pkg_name(eco, name))
    except DecodeError as e:
        raise DecodeError(f"failed to get {eco} advisories: failed to unmarshal advisory JSON: {e}")
    return [library_vuln(a, pkg_id, name, ver) for a in advs if is_vulnerable(grammar, ver, a)]


def library_vuln(a, pkg_id, name, ver):
    """driver.go:125-132: the DetectedVulnerability of advisory a for (pkgID, pkgName, pkgVer)."""
    v = {"VulnerabilityID": a["VulnerabilityID"], "PkgID": pkg_id, "PkgName": name, "InstalledVersion": ver,
         "FixedVersion": create_fixed_versions(a), "DataSource": a.get("DataSource")}
    return {k: x for k, x in v.items() if x}


def wrap_vuln(v, p):
    """detect.go:33-37: library.Detect adds the package's Layer, PkgPath and PkgIdentifier."""
    for k_in, k_out in (("Layer", "Layer"), ("FilePath", "PkgPath"), ("Identifier", "PkgIdentifier")):
        if p.get(k_in):
            v[k_out] = p[k_in]
    return v


def advisory_record(a):
    """The record (drivers.record_of) library.Detect builds from advisory a."""
    from .drivers import _STUB, record_of
    return record_of(wrap_vuln(library_vuln(a, _STUB["ID"], _STUB["Name"], _STUB["Version"]), _STUB))


def detect(db, lang, pkgs):
    """library.Detect (detect.go:11-42): None for an unsupported type."""
    if lang not in LANG:
        return None
    eco = LANG[lang][0]
    out = []
    for p in pkgs:
        try:
            vs = detect_vulnerabilities(db, lang, p.get("ID", ""), p.get("Name", ""), p.get("Version", ""))
        except DecodeError as e:
            raise DecodeError(f"failed to scan {eco} vulnerabilities: failed to detect {eco} vulnerabilities: {e}")
        out += [wrap_vuln(v, p) for v in vs]
    return out
