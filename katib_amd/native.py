"""Loader for the in-tree native runtime (``_native`` C++ extension).

The extension is built in-tree by ``__graft_entry__.build()`` /
``katib_amd._build.build_native``; if it is missing (fresh checkout) it is built
on first use with the system g++ (a few seconds) - never silently replaced by a
Python fallback.
"""

from __future__ import annotations

import importlib
import threading

_lock = threading.Lock()
_mod = None


def load():
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            try:
                _mod = importlib.import_module("katib_amd._native")
            except ImportError:
                from ._build import build_native

                build_native()
                _mod = importlib.import_module("katib_amd._native")
    return _mod
