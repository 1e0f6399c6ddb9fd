"""doublestar v4 Match for ignore-file paths (github.com/bmatcuk/doublestar/v4, pinned by the
reference's go.mod; called from pkg/result/ignore.go:102-114 matchPath).

Semantics restated: the pattern and the path are '/'-separated; in a component '*' is any
run of non-'/' characters, '?' one non-'/' character, '[...]' a class ('!' or '^' negates,
ranges allowed), '{a,b}' alternatives, '\\' escapes the next character; a component that
is exactly '**' matches zero or more whole components.  A malformed pattern matches
nothing (Match returns ErrBadPattern; the reference validates patterns when it parses the
ignore file).

Each pattern is compiled once to one anchored regular expression over "/" + path: a plain
component becomes "/" + its regex, a '**' component "(?:/[^/]*)*", so '**' can absorb
zero components together with their separators.
"""
import functools
import re

_ANY = "(?:/[^/]*)*"


def _component(c):
    """Regex of one pattern component, or None when it is malformed."""
    out, i = [], 0
    while i < len(c):
        ch = c[i]
        if ch == "\\":
            if i + 1 >= len(c):
                return None
            out.append(re.escape(c[i + 1]))
            i += 2
        elif ch == "*":
            out.append("[^/]*")
            i += 1
        elif ch == "?":
            out.append("[^/]")
            i += 1
        elif ch == "[":
            k = i + 1
            neg = k < len(c) and c[k] in "!^"
            if neg:
                k += 1
            end = c.find("]", k + 1 if k < len(c) and c[k] == "]" else k)
            if end < 0:
                return None
            body = c[k:end].replace("\\", "\\\\")
            if not body:
                return None
            out.append("[" + ("^" if neg else "") + body + "]")
            i = end + 1
        elif ch == "{":
            end = c.find("}", i)
            if end < 0:
                return None
            alts = [_component(a) for a in c[i + 1:end].split(",")]
            if any(a is None for a in alts):
                return None
            out.append("(?:" + "|".join(alts) + ")")
            i = end + 1
        else:
            out.append(re.escape(ch))
            i += 1
    return "".join(out)


@functools.lru_cache(maxsize=4096)
def compile_pattern(pattern):
    """Compiled matcher of a pattern, or None when malformed."""
    parts = []
    for comp in pattern.split("/"):
        if comp == "**":
            parts.append(_ANY)
            continue
        rx = _component(comp)
        if rx is None:
            return None
        parts.append("/" + rx)
    return re.compile("".join(parts), re.S)


def match(pattern, path):
    """doublestar.Match(pattern, path) (errors count as no match)."""
    rx = compile_pattern(pattern)
    return rx is not None and rx.fullmatch("/" + path) is not None


def match_any(patterns, path):
    """ignore.go matchPath: no patterns match everything."""
    return not patterns or any(match(p, path) for p in patterns)
