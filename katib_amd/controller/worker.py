"""Warm trial worker: one long-lived process per GPU slot.

Started by the scheduler through the native runtime (``TrialRuntime.spawn_worker``)
with ``HIP_VISIBLE_DEVICES`` pinned to its slot. It initialises the HIP context
once (``--warm``), then executes trial after trial:

    scheduler -> stdin : one JSON payload line per trial
    worker    -> stdout: the trial's own output (metrics lines), then "\\x1eEND <code>"

Exit codes: 0 success, 1 failure, 3 stopped on request (early stop / kill /
deadline - delivered as SIGUSR1 and raised inside the trial as
:class:`TrialStopped`). Reusing the process removes interpreter start, ``import
torch`` and HIP context creation (seconds per trial) from every trial, which is
what dominates trials/hour for short trials.
"""

from __future__ import annotations

import importlib
import json
import os
import signal
import sys
import traceback

MARK = "\x1e"


class TrialStopped(BaseException):
    """Raised asynchronously in the trial when the scheduler stops it."""


_current = {"trial": None}


def _on_usr1(signum, frame):
    if _current["trial"] is not None:
        raise TrialStopped()


def _run_function(fn_spec, params):
    ns = {"__name__": "__katib_objective__"}
    exec(compile(fn_spec["source"], "<katib-objective>", "exec"), ns)
    fn = ns[fn_spec["entry"]]
    return fn(params)


def _run_entrypoint(entry, args):
    mod, _, fname = entry.partition(":")
    m = importlib.import_module(mod)
    fn = getattr(m, fname or "main")
    return fn(list(args))


def main():
    warm = "--warm" in sys.argv
    sys.stdout.reconfigure(line_buffering=True)
    signal.signal(signal.SIGUSR1, _on_usr1)
    if warm and os.environ.get("HIP_VISIBLE_DEVICES", "") != "":
        try:
            import torch

            if torch.cuda.is_available():
                torch.empty(1, device="cuda")
                torch.cuda.synchronize()
        except Exception as e:  # a broken device must not hide the worker: trials will fail loudly
            print("katib-amd worker: GPU warm-up failed: %s" % e, flush=True)
    print(MARK + "READY", flush=True)
    base_env = dict(os.environ)
    base_cwd = os.getcwd()
    for line in sys.stdin:
        line = line.strip()
        if not line:
            continue
        payload = json.loads(line)
        code = 0
        os.environ.clear()
        os.environ.update(base_env)
        os.environ.update(payload.get("env", {}))
        os.environ["KATIB_TRIAL_NAME"] = payload.get("trial", "")
        cwd = payload.get("cwd") or base_cwd
        try:
            os.makedirs(cwd, exist_ok=True)
            os.chdir(cwd)
            _current["trial"] = payload.get("trial")
            if payload.get("function"):
                _run_function(payload["function"], payload["function"].get("params", {}))
            else:
                _run_entrypoint(payload["entrypoint"], payload.get("args", []))
        except TrialStopped:
            code = 3
        except SystemExit as e:
            code = int(e.code) if isinstance(e.code, int) else (0 if e.code is None else 1)
        except BaseException:
            traceback.print_exc(file=sys.stdout)
            code = 1
        finally:
            _current["trial"] = None
        sys.stdout.flush()
        sys.stderr.flush()
        print(MARK + "END %d" % code, flush=True)
        try:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()
        except Exception:
            pass


if __name__ == "__main__":
    main()
