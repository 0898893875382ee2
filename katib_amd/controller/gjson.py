"""Tiny GJSON subset used for trial success/failure conditions
(reference ``pkg/controller.v1beta1/trial/util/job_util.go:30-120``).

Supported syntax - enough for every default and example condition:
``a.b.c`` paths, ``#(key==value)#`` (all matches) / ``#(key==value)`` (first
match) queries with ``== != < <= > >= %`` and string / number / bool literals,
``#`` (array length), ``|`` pipes, ``[a,b]`` multipaths and the ``@this`` modifier.
A result "matches" when it is an object or a non-empty array (job_util.go:67-88), or
a true-ish scalar. ``deployed_job_status`` is GetDeployedJobStatus (job_util.go:58-120).
"""

from __future__ import annotations

import fnmatch
import re
from typing import Any, Dict, List, Optional

_QUERY = re.compile(r"^#\((.+?)(==|!=|<=|>=|<|>|%)(.+)\)(#?)$")


def _split_path(path: str) -> List[str]:
    parts, cur, depth = [], "", 0
    for ch in path:
        if ch in "([":
            depth += 1
        elif ch in ")]":
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


def _split_top(s: str, sep: str) -> List[str]:
    parts, cur, depth = [], "", 0
    for ch in s:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if ch == sep and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    return parts


def _apply(value: Any, part: str):
    if part == "@this":
        return value
    if len(part) >= 2 and part[0] == "[" and part[-1] == "]":  # multipath: one result per member path
        out = [get(value, p.strip()) for p in _split_top(part[1:-1], ",") if p.strip()]
        return [v for v in out if v is not None]
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
    for seg in _split_top(expr, "|"):
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


def _is_condition(r) -> bool:
    return isinstance(r, dict) or (isinstance(r, list) and len(r) > 0)


def deployed_job_status(job: Any, success_condition: str, failure_condition: str,
                        trial_running: bool = False) -> Optional[Dict[str, str]]:
    """Failure is checked first; the matched object (or the first element of a matched
    array) supplies ``reason``/``message``. ``None`` means "no status update" (the
    trial is already running and neither condition holds)."""
    for expr, cond in ((failure_condition, "Failed"), (success_condition, "Succeeded")):
        r = get(job, expr) if expr else None
        if _is_condition(r):
            first = r[0] if isinstance(r, list) else r
            out = {"condition": cond}
            if isinstance(first, dict):
                for k in ("reason", "message"):
                    if first.get(k):
                        out[k] = str(first[k])
            return out
    name = ((job or {}).get("metadata") or {}).get("name") if isinstance(job, dict) else None
    if not trial_running and name:
        return {"condition": "Running"}
    return None
