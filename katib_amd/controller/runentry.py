"""Run one ``entrypoint``/``Function`` trial in a fresh process (multi-GPU trials, or
when warm workers are disabled). Same contract as :mod:`katib_amd.controller.worker`."""

import json
import sys

from .worker import _run_entrypoint, _run_function


def main():
    spec = json.loads(sys.argv[1])
    if spec.get("function"):
        _run_function(spec["function"], spec["function"].get("params", {}))
    else:
        _run_entrypoint(spec["entrypoint"], spec.get("args", []))


if __name__ == "__main__":
    main()
