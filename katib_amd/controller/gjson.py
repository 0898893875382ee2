"""Tiny GJSON subset used for trial success/failure conditions
(reference ``pkg/controller.v1beta1/trial/util/job_util.go:30-120``).

Supported syntax - enough for every default and example condition:
``a.b.c`` paths, ``#(key==value)#`` (all matches) / ``#(key==value)`` (first
match) queries with ``== != < <= > >= %`` and string / number / bool literals,
``#`` (array length) and ``|`` pipes. A result "matches" when it is an object or
a non-empty array (job_util.go:67-88), or a true-ish scalar.
"""

from __future__ import annotations

import fnmatch
import re
from typing import Any, List

_QUERY = re.compile(r"^#\((.+?)(==|!=|<=|>=|<|>|%)(.+)\)(#?)$")


def _split_path(path: str) -> List[str]:
    parts, cur, depth = [], "", 0
    for ch in path:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "." and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur:
        parts.append(cur)
    return parts


def _literal(s: str):
    s = s.strip()
    if len(s) >= 2 and s[0] == s[-1] == '"':
        return s[1:-1]
    if s in ("true", "false"):
        return s == "true"
    try:
        return float(s)
    except ValueError:
        return s


def _cmp(a, op, b) -> bool:
    if isinstance(b, (int, float)) and not isinstance(b, bool):
        try:
            a = float(a)
        except (TypeError, ValueError):
            return False
    if op == "==":
        return a == b
    if op == "!=":
        return a != b
    if op == "%":
        return isinstance(a, str) and fnmatch.fnmatchcase(a, str(b))
    try:
        return {"<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b}[op]
    except TypeError:
        return False


def _apply(value: Any, part: str):
    m = _QUERY.match(part)
    if m:
        key, op, lit, allm = m.group(1).strip(), m.group(2), _literal(m.group(3)), m.group(4) == "#"
        if not isinstance(value, list):
            return None
        hits = [v for v in value if isinstance(v, dict) and _cmp(v.get(key), op, lit)]
        if allm:
            return hits
        return hits[0] if hits else None
    if part == "#":
        return len(value) if isinstance(value, list) else None
    if isinstance(value, dict):
        return value.get(part)
    if isinstance(value, list):
        if part.isdigit():
            i = int(part)
            return value[i] if i < len(value) else None
        # implicit map over arrays: a.#.b style
        out = [v.get(part) for v in value if isinstance(v, dict) and part in v]
        return out
    return None


def get(obj: Any, expr: str):
    cur = obj
    for seg in expr.split("|"):
        seg = seg.strip()
        if not seg:
            continue
        for part in _split_path(seg):
            cur = _apply(cur, part)
            if cur is None:
                return None
    return cur


def matches(obj: Any, expr: str) -> bool:
    if not expr:
        return False
    r = get(obj, expr)
    if isinstance(r, dict):
        return True
    if isinstance(r, list):
        return len(r) > 0
    if isinstance(r, bool):
        return r
    if isinstance(r, str):
        return r.lower() == "true"
    return False
