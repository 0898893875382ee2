"""Loader of the in-tree HIP extension (``katib_amd._hipkern``).

``KATIB_AMD_HIPKERN=<path to .so>`` loads a tuning variant built with
``_build.build_hip(defines=..., out=...)`` instead (same module name, so every importer
sees the same kernels); unset, the in-tree build is imported. A missing build raises:
the HIP paths never fall back silently.
"""

from __future__ import annotations

import importlib
import importlib.util
import os
import sys


def hipkern():
    mod = sys.modules.get("katib_amd._hipkern")
    if mod is not None:
        return mod
    path = os.environ.get("KATIB_AMD_HIPKERN")
    try:
        if path:
            spec = importlib.util.spec_from_file_location("katib_amd._hipkern", path)
            mod = importlib.util.module_from_spec(spec)
            sys.modules["katib_amd._hipkern"] = mod
            spec.loader.exec_module(mod)
            return mod
        return importlib.import_module("katib_amd._hipkern")
    except ImportError as e:
        sys.modules.pop("katib_amd._hipkern", None)
        raise ImportError("katib_amd._hipkern is not built (run __graft_entry__.build()): %s" % e)
