#!/usr/bin/env python3
"""Transcribe the reference's Go test tables into JSON data (test infrastructure).

Reads the reference's `*_test.go` files AS TEXT and re-emits the literal values of
every `tests := []struct{...}{...}` / `map[string]struct{...}{...}` table - inputs and
expected outputs only, no code - into `tests/golden/tables/<relpath>.json`.  Each case
keeps the Go field names (`args.osVer`, `want`, `wantErr`, ...); identifiers are
resolved through a small constant table (trivy-db enum values, data-source IDs, ftypes
constants) and `time.Date(...)` calls become RFC 3339 strings.

Usage:  python tests/golden/extract_go_tables.py [/root/reference]
"""
import datetime
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "tables")

# Test files whose tables are transcribed (relative to the reference root).
FILES = [
    "pkg/detector/ospkg/alma/alma_test.go",
    "pkg/detector/ospkg/alpine/alpine_test.go",
    "pkg/detector/ospkg/amazon/amazon_test.go",
    "pkg/detector/ospkg/chainguard/chainguard_test.go",
    "pkg/detector/ospkg/debian/debian_test.go",
    "pkg/detector/ospkg/mariner/mariner_test.go",
    "pkg/detector/ospkg/oracle/oracle_test.go",
    "pkg/detector/ospkg/photon/photon_test.go",
    "pkg/detector/ospkg/redhat/redhat_test.go",
    "pkg/detector/ospkg/rocky/rocky_test.go",
    "pkg/detector/ospkg/suse/suse_test.go",
    "pkg/detector/ospkg/ubuntu/ubuntu_test.go",
    "pkg/detector/ospkg/wolfi/wolfi_test.go",
    "pkg/detector/library/driver_test.go",
    "pkg/detector/library/compare/compare_test.go",
    "pkg/detector/library/compare/bitnami/compare_test.go",
    "pkg/detector/library/compare/maven/compare_test.go",
    "pkg/detector/library/compare/npm/compare_test.go",
    "pkg/detector/library/compare/pep440/compare_test.go",
    "pkg/detector/library/compare/rubygems/compare_test.go",
    "pkg/scanner/utils/utils_test.go",
    "pkg/vulnerability/vulnerability_test.go",
    "pkg/result/filter_test.go",
    "pkg/fanal/analyzer/pkg/dpkg/dpkg_test.go",
    "pkg/fanal/analyzer/pkg/apk/apk_test.go",
    "pkg/fanal/analyzer/pkg/rpm/rpm_test.go",
    "pkg/fanal/analyzer/pkg/rpm/rpmqa_test.go",
]

# trivy-db / trivy constants used in the tables (values from trivy-db pkg/types and
# pkg/vulnsrc/vulnerability, pinned go.mod:25; ftypes from pkg/fanal/types/const.go).
SEVERITIES = ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"]
STATUSES = ["Unknown", "NotAffected", "Affected", "Fixed", "UnderInvestigation", "WillNotFix", "FixDeferred",
            "EndOfLife"]
CONST = {"true": True, "false": False, "nil": None, "time.UTC": "UTC"}
for i, s in enumerate(SEVERITIES):
    CONST["dbTypes.Severity" + s.capitalize()] = i
    CONST["types.Severity" + s.capitalize()] = i
for i, s in enumerate(STATUSES):
    CONST["dbTypes.Status" + s] = i
SOURCE_IDS = {
    "Alpine": "alpine", "Debian": "debian", "Ubuntu": "ubuntu", "Amazon": "amazon", "RedHat": "redhat",
    "RedHatOVAL": "redhat-oval", "Alma": "alma", "Rocky": "rocky", "OracleOVAL": "oracle-oval",
    "SuseCVRF": "suse-cvrf", "Photon": "photon", "CBLMariner": "cbl-mariner", "Wolfi": "wolfi",
    "Chainguard": "chainguard", "GHSA": "ghsa", "GLAD": "glad", "OSV": "osv", "NVD": "nvd", "GoVulnDB": "go",
    "RubySec": "ruby-advisory-db", "PhpSecurityAdvisories": "php-security-advisories",
    "NodejsSecurityWg": "nodejs-security-wg", "K8sVulnDB": "k8s", "Bitnami": "bitnami",
}
for k, v in SOURCE_IDS.items():
    CONST["vulnerability." + k] = v
FTYPES = {
    "Alpine": "alpine", "Alma": "alma", "Amazon": "amazon", "CBLMariner": "cbl-mariner", "CentOS": "centos",
    "Chainguard": "chainguard", "Debian": "debian", "Fedora": "fedora", "OpenSUSE": "opensuse",
    "OpenSUSELeap": "opensuse.leap", "OpenSUSETumbleweed": "opensuse.tumbleweed", "Oracle": "oracle",
    "Photon": "photon", "RedHat": "redhat", "Rocky": "rocky", "SLES": "suse linux enterprise server",
    "Ubuntu": "ubuntu", "Wolfi": "wolfi",
    "Bundler": "bundler", "GemSpec": "gemspec", "Cargo": "cargo", "Composer": "composer", "Npm": "npm",
    "NuGet": "nuget", "DotNetCore": "dotnet-core", "Pip": "pip", "Pipenv": "pipenv", "Poetry": "poetry",
    "CondaPkg": "conda-pkg", "PythonPkg": "python-pkg", "NodePkg": "node-pkg", "Yarn": "yarn", "Pnpm": "pnpm",
    "Jar": "jar", "Pom": "pom", "Gradle": "gradle", "GoBinary": "gobinary", "GoModule": "gomod",
    "JavaScript": "javascript", "RustBinary": "rustbinary", "Conan": "conan", "Cocoapods": "cocoapods",
    "Swift": "swift", "Pub": "pub", "Hex": "hex", "Bitnami": "bitnami", "K8sUpstream": "kubernetes",
}
for k, v in FTYPES.items():
    CONST["ftypes." + k] = v
# github.com/package-url/packageurl-go type constants
for k in ("Golang", "Npm", "Maven", "PyPi", "Apk", "Rpm", "Deb", "Gem", "Cargo", "Composer", "Nuget", "Conan",
          "Cocoapods", "Hex", "Pub", "Swift", "Bitnami", "Conda", "Docker", "OCI", "Generic"):
    CONST["packageurl.Type" + k] = k.lower()
CONST["types.ClassLangPkg"] = "lang-pkgs"
CONST["types.ClassOSPkg"] = "os-pkgs"
CONST["types.ClassConfig"] = "config"
CONST["types.ClassSecret"] = "secret"
CONST["types.ClassLicense"] = "license"
CONST["types.ClassLicenseFile"] = "license-file"
CONST["types.FindingStatusIgnored"] = "ignored"
CONST["types.FindingStatusNotAffected"] = "not_affected"
CONST["types.FindingStatusFixed"] = "fixed"
CONST["types.FindingStatusUnderInvestigation"] = "under_investigation"
CONST["suse.OpenSUSE"] = "opensuse"                 # suse.go Type enum (iota)
CONST["suse.SUSEEnterpriseLinux"] = "sles"


class Tok:
    __slots__ = ("k", "v")

    def __init__(self, k, v):
        self.k, self.v = k, v

    def __repr__(self):
        return f"{self.k}:{self.v!r}"


_GO_ESC = {"n": "\n", "t": "\t", "r": "\r", "\\": "\\", '"': '"', "'": "'", "a": "\a", "b": "\b", "f": "\f",
           "v": "\v"}


def _unquote(body):
    out, i = [], 0
    while i < len(body):
        c = body[i]
        if c != "\\":
            out.append(c)
            i += 1
            continue
        e = body[i + 1]
        if e in _GO_ESC:
            out.append(_GO_ESC[e])
            i += 2
        elif e == "x":
            out.append(chr(int(body[i + 2:i + 4], 16)))
            i += 4
        elif e == "u":
            out.append(chr(int(body[i + 2:i + 6], 16)))
            i += 6
        elif e == "U":
            out.append(chr(int(body[i + 2:i + 10], 16)))
            i += 10
        else:
            raise ValueError("escape " + e)
    return "".join(out)


def tokenize(src):
    toks, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if c.isspace():
            i += 1
        elif src.startswith("//", i):
            i = src.find("\n", i)
            i = n if i < 0 else i
        elif src.startswith("/*", i):
            i = src.find("*/", i) + 2
        elif c == "`":
            j = src.find("`", i + 1)
            toks.append(Tok("str", src[i + 1:j]))
            i = j + 1
        elif c == '"':
            j = i + 1
            while src[j] != '"':
                j += 2 if src[j] == "\\" else 1
            toks.append(Tok("str", _unquote(src[i + 1:j])))
            i = j + 1
        elif c == "'":
            j = src.find("'", i + 1)
            toks.append(Tok("num", ord(_unquote(src[i + 1:j]))))
            i = j + 1
        elif c.isdigit():
            m = re.match(r"0x[0-9a-fA-F]+|\d+\.\d*(e[-+]?\d+)?|\d+", src[i:])
            s = m.group(0)
            toks.append(Tok("num", int(s, 0) if s.isdigit() or s.startswith("0x") else float(s)))
            i += len(s)
        elif c.isalpha() or c == "_":
            m = re.match(r"[A-Za-z_][A-Za-z0-9_]*", src[i:])
            toks.append(Tok("id", m.group(0)))
            i += len(m.group(0))
        elif src.startswith(":=", i):
            toks.append(Tok("p", ":="))
            i += 2
        else:
            toks.append(Tok("p", c))
            i += 1
    return toks


class Parser:
    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, o=0):
        return self.t[self.i + o] if self.i + o < len(self.t) else Tok("eof", None)

    def next(self):
        t = self.t[self.i]
        self.i += 1
        return t

    def expect(self, v):
        t = self.next()
        if t.v != v:
            raise SyntaxError(f"expected {v!r}, got {t!r} at {self.i}")
        return t

    def skip_balanced(self, open_, close):
        self.expect(open_)
        depth = 1
        while depth:
            t = self.next()
            if t.k == "p" and t.v == open_:
                depth += 1
            elif t.k == "p" and t.v == close:
                depth -= 1

    def qualident(self):
        name = self.next().v
        while self.peek().v == "." and self.peek(1).k == "id":
            self.next()
            name += "." + self.next().v
        return name

    def parse_type(self):
        t = self.peek()
        if t.v == "[":
            self.next()
            if self.peek().v != "]":
                self.next()
            self.expect("]")
            return "[]" + self.parse_type()
        if t.v == "*":
            self.next()
            return "*" + self.parse_type()
        if t.v == "map":
            self.next()
            self.expect("[")
            k = self.parse_type()
            self.expect("]")
            return f"map[{k}]" + self.parse_type()
        if t.v == "struct":
            self.next()
            self.skip_balanced("{", "}")
            return "struct"
        if t.v == "interface":
            self.next()
            self.skip_balanced("{", "}")
            return "interface"
        if t.v == "func":
            self.next()
            self.skip_balanced("(", ")")
            if self.peek().k == "id":
                self.parse_type()
            return "func"
        return self.qualident()

    def composite(self, typ):
        self.expect("{")
        keyed, items = {}, []
        elem_typ = typ[2:] if typ and typ.startswith("[]") else None
        if typ and typ.startswith("map["):
            depth, j = 0, 4
            while True:
                if typ[j] == "[":
                    depth += 1
                elif typ[j] == "]":
                    if depth == 0:
                        break
                    depth -= 1
                j += 1
            elem_typ = typ[j + 1:]
        while self.peek().v != "}":
            if self.peek().v == "{":
                v = self.composite(elem_typ)
                if self.peek().v == ":":  # composite key (unused here)
                    raise SyntaxError("composite key")
                items.append(v)
            else:
                v = self.value(elem_typ)
                if self.peek().v == ":":
                    self.next()
                    key = v if not isinstance(v, dict) or "__ident__" not in v else v["__ident__"]
                    if self.peek().v == "{":
                        keyed[key] = self.composite(elem_typ if typ and typ.startswith("map[") else None)
                    else:
                        keyed[key] = self.value(elem_typ if typ and typ.startswith("map[") else None)
                else:
                    items.append(v)
            if self.peek().v == ",":
                self.next()
        self.expect("}")
        if keyed and items:
            raise SyntaxError("mixed composite")
        if keyed:
            return keyed
        if not items and not (typ and (typ.startswith("[]") or typ.startswith("*[]"))):
            return {}
        return items

    def value(self, hint=None):
        v = self.unary(hint)
        while self.peek().v == "+" and isinstance(v, str):
            self.next()
            v += self.unary(hint)
        return v

    def unary(self, hint=None):
        t = self.peek()
        if t.v == "&":
            self.next()
            return self.unary(hint)
        if t.v == "-":
            self.next()
            return -self.unary(hint)
        if t.k == "str":
            self.next()
            return t.v
        if t.k == "num":
            self.next()
            return t.v
        if t.v == "{":
            return self.composite(hint)
        if t.v in ("[", "map", "struct"):
            typ = self.parse_type()
            if self.peek().v == "(":  # conversion, e.g. []T(nil)
                self.next()
                v = self.value()
                self.expect(")")
                return v
            return self.composite(typ)
        if t.k == "id":
            if t.v == "func":
                raise SyntaxError("func literal")
            name = self.qualident()
            if self.peek().v == "{":
                return self.composite(name)
            if self.peek().v == "(":
                self.next()
                args = []
                while self.peek().v != ")":
                    args.append(self.value())
                    if self.peek().v == ",":
                        self.next()
                self.next()
                return call(name, args)
            return ident(name)
        raise SyntaxError(f"unexpected {t!r}")


def ident(name):
    if name in CONST:
        return CONST[name]
    for suffix in (".String",):
        if name.endswith(suffix) and name[:-len(suffix)] in CONST:
            return CONST[name[:-len(suffix)]]
    return {"__ident__": name}


def call(name, args):
    if name == "time.Date":
        y, mo, d, h, mi, s = args[:6]
        y, mo = y + (mo - 1) // 12, (mo - 1) % 12 + 1  # Go normalises out-of-range fields
        t = datetime.datetime(y, mo, 1) + datetime.timedelta(days=d - 1, hours=h, minutes=mi, seconds=s)
        return t.strftime("%Y-%m-%dT%H:%M:%SZ")
    if name.endswith(".String") and not args:
        base = name[:-len(".String")]
        if base in CONST:
            v = CONST[base]
            if base.startswith(("dbTypes.Severity", "types.Severity")):
                return SEVERITIES[v]
            return v
    if name in ("lo.ToPtr", "utils.ToPtr") and len(args) == 1:
        return args[0]
    return {"__call__": name, "args": args}


def _subst(v, env):
    """Replaces {"__ident__": name} references to the test's local `var (...)` values."""
    if isinstance(v, dict):
        if set(v) == {"__ident__"} and v["__ident__"] in env:
            return env[v["__ident__"]]
        return {k: _subst(x, env) for k, x in v.items()}
    if isinstance(v, list):
        return [_subst(x, env) for x in v]
    return v


def _local_vars(toks, start, end):
    """name -> value of every `var ( name = value ... )` block in toks[start:end]."""
    env = {}
    for k in range(start, end):
        if toks[k].v == "var" and toks[k + 1].v == "(":
            p = Parser(toks)
            p.i = k + 2
            while p.peek().v != ")":
                name = p.next().v
                p.expect("=")
                env[name] = _subst(p.value(), env)
    return env


def _toplevel_vars(toks):
    """name -> value of every single `var name = value` declaration (package level)."""
    env = {}
    for k in range(len(toks) - 2):
        if toks[k].v == "var" and toks[k + 1].k == "id" and toks[k + 2].v == "=" and toks[k + 1].v != "tests":
            p = Parser(toks)
            p.i = k + 3
            try:
                env[toks[k + 1].v] = _subst(p.value(), env)
            except Exception:  # not a literal: not data
                pass
    return env


def extract(path):
    src = open(path, encoding="utf-8").read()
    toks = tokenize(src)
    tables = []
    top = _toplevel_vars(toks)
    i = 0
    # the enclosing test function of each table
    while i < len(toks):
        t = toks[i]
        is_var = i > 0 and toks[i - 1].v == "var" and i + 1 < len(toks) and toks[i + 1].v == "="
        if t.k == "id" and t.v == "tests" and i + 1 < len(toks) and (toks[i + 1].v == ":=" or is_var):
            fn, fstart = None, 0
            for j in range(i, 0, -1):
                if toks[j].v == "func" and toks[j + 1].k == "id" and toks[j + 1].v.startswith("Test"):
                    fn, fstart = toks[j + 1].v, j
                    break
            env = dict(top)
            env.update(_local_vars(toks, fstart, i))
            p = Parser(toks)
            p.i = i + 2
            typ = p.parse_type()
            body = _subst(p.composite(typ), env)
            if isinstance(body, dict):  # map[string]struct: name -> case
                body = [dict(v, name=k) if isinstance(v, dict) else {"name": k, "value": v} for k, v in body.items()]
            tables.append({"func": fn, "cases": body})
            i = p.i
        else:
            i += 1
    return tables


def main(ref="/root/reference"):
    for rel in FILES:
        tables = extract(os.path.join(ref, rel))
        dst = os.path.join(OUT, rel.replace("pkg/", "", 1).replace("/", "__").replace(".go", ".json"))
        os.makedirs(OUT, exist_ok=True)
        with open(dst, "w", encoding="utf-8") as f:
            json.dump({"ref": rel, "tables": tables}, f, indent=1, ensure_ascii=False)
            f.write("\n")
        print(f"{rel}: {sum(len(t['cases']) for t in tables)} cases in {len(tables)} tables")


if __name__ == "__main__":
    main(*sys.argv[1:])
