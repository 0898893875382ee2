"""Fork server ("zygote") for cold Python trial processes.

A ``batch/v1 Job`` trial whose command is ``python3 -m <module> ...`` (the reference's B1 shape,
``docs/workflow-design.md:39-108``: every trial a fresh container) pays interpreter start and
``import torch`` before its first line of training - most of a short trial. The zygote is one
long-lived interpreter per scheduler that has already imported torch and the preload modules
(``KATIB_AMD_ZYGOTE_PRELOAD``) but never touches the GPU (no HIP call, no
``torch.cuda.is_available()``: a HIP context does not survive ``fork``). Per trial it forks a fresh
child that applies the trial's environment (``HIP_VISIBLE_DEVICES`` included, before the child's
first HIP call), working directory and argv, and runs the module as ``__main__``: each child
initialises HIP itself, and nothing ever ``exec``s after GPU initialisation.

Process tree: the scheduler (a child subreaper, ``PR_SET_CHILD_SUBREAPER``) starts the zygote; the
zygote double-forks, so the trial process is re-parented to the scheduler, which then supervises it
exactly like one it spawned itself (``TrialRuntime.adopt``: the same waitpid reaping, process-group
kills, stdout pipe, metrics collection and deadlines). Requests travel over a ``SOCK_SEQPACKET``
unix socket: one JSON message ``{"argv", "env", "cwd"}`` with the trial's stdout pipe attached
(``SCM_RIGHTS``); the reply is ``{"pid": ...}`` or ``{"error": ...}``.

Reference behaviour kept: a trial is still a separate process with its own environment, exit
code and stdout (``pkg/webhook/v1beta1/pod/inject_webhook.go:152-197`` wraps the container
command; the collector reads its output), so the fork server is invisible to trial code.
"""

from __future__ import annotations

import argparse
import ctypes
import importlib
import json
import os
import shutil
import signal
import socket
import struct
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

PR_SET_PDEATHSIG = 1
PR_SET_CHILD_SUBREAPER = 36
DEFAULT_PRELOAD = "torch,katib_amd.workloads.common,katib_amd.workloads.mnist_mlp"


def _prctl(option: int, arg: int) -> bool:
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        return libc.prctl(option, arg, 0, 0, 0) == 0
    except (OSError, AttributeError):
        return False


# ------------------------------------------------------------------------------------ server
def _run_child(req: Dict, out_fd: int, keep_parent: int) -> None:
    """In the forked trial process: become the trial, run it, exit with its code. Never returns."""
    code = 1
    try:
        os.setpgid(0, 0)
        # the intermediate parent exits right away; once re-parented to the scheduler, arm the
        # parent-death signal so a dying scheduler takes its trials along (as the exec path does)
        deadline = time.time() + 2.0
        while os.getppid() == keep_parent and time.time() < deadline:
            time.sleep(0.0005)
        _prctl(PR_SET_PDEATHSIG, signal.SIGKILL)
        for s in (signal.SIGTERM, signal.SIGINT, signal.SIGUSR1, signal.SIGCHLD, signal.SIGPIPE):
            signal.signal(s, signal.SIG_DFL)
        devnull = os.open(os.devnull, os.O_RDONLY)
        os.dup2(devnull, 0)
        os.dup2(out_fd, 1)
        os.dup2(out_fd, 2)
        os.close(devnull)
        os.close(out_fd)
        os.environ.clear()
        os.environ.update(req.get("env") or {})
        if req.get("cwd"):
            os.chdir(req["cwd"])
        argv: List[str] = list(req["argv"])
        _child_imports(argv)
        # stdout is a pipe: line buffering keeps metrics flowing to the collector as they are printed
        sys.stdout.reconfigure(line_buffering=True)
        sys.stderr.reconfigure(line_buffering=True)
        nthreads = os.environ.get("OMP_NUM_THREADS")
        if nthreads and nthreads.isdigit() and "torch" in sys.modules:
            sys.modules["torch"].set_num_threads(int(nthreads))
        _restore_blas_threads()
        import runpy

        try:
            if argv[1] == "-m":
                sys.argv = [argv[2]] + argv[3:]
                runpy.run_module(argv[2], run_name="__main__", alter_sys=True)
            elif argv[1] == "-c":
                sys.argv = ["-c"] + argv[3:]
                exec(compile(argv[2], "<string>", "exec"), {"__name__": "__main__", "__builtins__": __builtins__})
            else:
                sys.argv = argv[1:]
                runpy.run_path(argv[1], run_name="__main__")
            code = 0
        except SystemExit as e:
            if e.code is None:
                code = 0
            elif isinstance(e.code, int):
                code = e.code
            else:
                print(e.code, file=sys.stderr)
                code = 1
        except BaseException:  # noqa: BLE001 - the trial's own failure: traceback, exit 1 (like python)
            import traceback

            traceback.print_exc()
            code = 1
    finally:
        try:
            import atexit

            atexit._run_exitfuncs()  # what interpreter exit would run (trial code's own handlers)
        except Exception:  # noqa: BLE001
            pass
        try:
            sys.stdout.flush()
            sys.stderr.flush()
        except Exception:  # noqa: BLE001
            pass
        os._exit(code & 0xFF)


# sys.path entries of this interpreter's installation (stdlib, site-packages, .pth additions): what a
# freshly exec'd interpreter has after its script directory and PYTHONPATH. Set by serve().
_SITE_PATH: List[str] = []


def _site_path() -> List[str]:
    """sys.path minus entry 0 (the server's launch directory) and this server's own PYTHONPATH."""
    own = [os.path.abspath(p) for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p]
    return [p for p in sys.path[1:] if not p or os.path.abspath(p) not in own]


def _child_imports(argv: List[str]) -> None:
    """Make imports in the forked trial resolve as they would after ``exec``:

    * ``sys.path`` = [the script directory (``script.py``), the working directory (``-m``) or ''
      (``-c``)] + the trial environment's ``PYTHONPATH`` + the installation's paths - the server's
      own launch directory and PYTHONPATH do not leak into the trial;
    * every ``katib_amd`` module the server preloaded (other than this server) is dropped from
      ``sys.modules``: such modules read ``KATIB_*`` switches and phase clocks at import time, so the
      trial re-imports them under ITS environment (torch and other third-party modules stay loaded -
      that is the saving the server exists for);
    * finder caches are invalidated, the working directory having changed under them."""
    if argv[1] == "-m":
        head = os.getcwd()
    elif argv[1] == "-c":
        head = ""
    else:
        head = os.path.dirname(os.path.realpath(argv[1]))
    extra = [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p]
    sys.path[:] = [head] + extra + [p for p in _SITE_PATH if p not in extra]
    for name in list(sys.modules):
        if (name == "katib_amd" or name.startswith("katib_amd.")) and name not in (
                "katib_amd", "katib_amd.controller", "katib_amd.controller.zygote"):
            del sys.modules[name]
    for k in ("", "."):
        sys.path_importer_cache.pop(k, None)
    importlib.invalidate_caches()


def _restore_blas_threads() -> None:
    """The server runs with ``OPENBLAS_NUM_THREADS=1`` (numpy's OpenBLAS otherwise starts a thread
    pool at import, and a forked child would inherit it half-copied); the trial gets the BLAS pool
    an exec'd interpreter would have started under its environment."""
    if "numpy" not in sys.modules:
        return
    n = os.environ.get("OPENBLAS_NUM_THREADS") or os.environ.get("OMP_NUM_THREADS")
    want = int(n) if n and n.isdigit() else (os.cpu_count() or 1)
    if want <= 1:
        return
    try:
        import threadpoolctl

        threadpoolctl.threadpool_limits(limits=want, user_api="blas")
    except Exception:  # noqa: BLE001 - a single-threaded BLAS is slower, never wrong
        pass


def os_threads() -> int:
    """Threads of this process as the kernel counts them (native pools included, which
    ``threading.active_count()`` does not see)."""
    try:
        return len(os.listdir("/proc/self/task"))
    except OSError:
        return threading.active_count()


def _handle(conn: socket.socket, listener: socket.socket) -> None:
    msg, fds, _, _ = socket.recv_fds(conn, 1 << 20, 1)
    if not msg:
        return
    try:
        req = json.loads(msg.decode())
        if len(fds) != 1:
            raise ValueError("expected one stdout descriptor")
        argv = req.get("argv") or []
        if len(argv) < 2:
            raise ValueError("argv needs an interpreter argument")
    except (ValueError, json.JSONDecodeError) as e:
        for fd in fds:
            os.close(fd)
        conn.send(json.dumps({"error": str(e)}).encode())
        return
    out_fd = fds[0]
    sys.stdout.flush()
    sys.stderr.flush()
    r, w = os.pipe()
    pid1 = os.fork()
    if pid1 == 0:  # intermediate: fork the trial and exit, so the trial is re-parented to the subreaper
        try:
            os.close(r)
            conn.close()
            listener.close()
            inter = os.getpid()
            pid2 = os.fork()
            if pid2 == 0:
                os.close(w)
                _run_child(req, out_fd, inter)
            os.write(w, struct.pack("i", pid2))
        finally:
            os._exit(0)
    os.close(w)
    os.close(out_fd)
    os.waitpid(pid1, 0)
    data = os.read(r, 4)
    os.close(r)
    if len(data) != 4:
        conn.send(json.dumps({"error": "fork failed"}).encode())
        return
    conn.send(json.dumps({"pid": struct.unpack("i", data)[0]}).encode())


def serve(path: str, preload: List[str]) -> int:
    t0 = time.time()
    loaded = []
    for mod in preload:
        if not mod:
            continue
        try:
            importlib.import_module(mod)
            loaded.append(mod)
        except Exception as e:  # noqa: BLE001 - a missing preload only costs the child its import
            print("zygote: preload %s failed: %s" % (mod, e), file=sys.stderr, flush=True)
    if "torch" in sys.modules:
        # torch.optim's first optimizer construction imports torch._dynamo (~1.3 s of pure Python,
        # measured on MI355X: scripts/trial_model_phase_probe.py): do it here, once, on a CPU
        # tensor - no kernel runs and no thread pool starts
        try:
            import torch

            torch.optim.SGD([torch.zeros(1, requires_grad=True)], lr=0.1)
            loaded.append("torch.optim(+_dynamo)")
        except Exception as e:  # noqa: BLE001
            print("zygote: optimizer warm-up failed: %s" % e, file=sys.stderr, flush=True)
    if "torch" in sys.modules and sys.modules["torch"].cuda.is_initialized():
        print("zygote: refusing to serve - the GPU was initialised during preload", file=sys.stderr, flush=True)
        return 3
    # fork() copies only the calling thread: a mutex another thread holds (an intra-op pool a torch
    # build starts at import, an OpenMP runtime) stays locked forever in every forked trial. Refuse
    # to serve rather than hand out trials that can deadlock; the scheduler then execs them.
    threads = os_threads()
    if threads > 1:
        print("zygote: refusing to serve - %d threads after preload (fork is only safe from a "
              "single-threaded process)" % threads, file=sys.stderr, flush=True)
        return 4
    _SITE_PATH[:] = _site_path()
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass
    listener = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    listener.bind(path)
    os.chmod(path, 0o600)
    listener.listen(64)
    print(json.dumps({"ready": True, "pid": os.getpid(), "preloaded": loaded, "threads": threads,
                      "preload_s": round(time.time() - t0, 3)}), flush=True)
    signal.signal(signal.SIGTERM, lambda *_: (listener.close(), os._exit(0)))
    # the scheduler may start this server from a helper thread, so the parent-death signal (tied to
    # the creating THREAD) cannot be used: poll the parent instead and exit once re-parented
    parent = os.getppid()
    listener.settimeout(1.0)
    while True:
        try:
            conn, _ = listener.accept()
        except socket.timeout:
            if os.getppid() != parent:
                return 0
            continue
        except OSError:
            return 0
        conn.settimeout(None)
        with conn:
            try:
                _handle(conn, listener)
            except Exception as e:  # noqa: BLE001 - one bad request must not take the server down
                try:
                    conn.send(json.dumps({"error": "zygote: %s" % e}).encode())
                except OSError:
                    pass


# ------------------------------------------------------------------------------------ client
class Zygote:
    """Scheduler-side handle: starts the fork server and spawns trial processes through it."""

    def __init__(self, state_dir: str, preload: Optional[str] = None, timeout: float = 120.0):
        self.path = os.path.join(state_dir, "zygote-%d.sock" % os.getpid())
        if len(self.path) > 100:  # sun_path limit
            import tempfile

            self.path = os.path.join(tempfile.gettempdir(), "katib-amd-zygote-%d.sock" % os.getpid())
        if not _prctl(PR_SET_CHILD_SUBREAPER, 1):
            raise RuntimeError("prctl(PR_SET_CHILD_SUBREAPER) failed")
        preload = preload if preload is not None else os.environ.get("KATIB_AMD_ZYGOTE_PRELOAD", DEFAULT_PRELOAD)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ)
        env["PYTHONPATH"] = os.pathsep.join(p for p in (root, env.get("PYTHONPATH", "")) if p)
        env["OPENBLAS_NUM_THREADS"] = "1"  # no BLAS thread pool in the forking process (_restore_blas_threads)
        self.proc = subprocess.Popen([sys.executable, "-m", "katib_amd.controller.zygote", "--socket", self.path,
                                      "--preload", preload], stdout=subprocess.PIPE, stdin=subprocess.DEVNULL,
                                     env=env, text=True)
        line = ""
        t0 = time.time()
        while time.time() - t0 < timeout:
            line = self.proc.stdout.readline()
            if line.startswith("{") or not line:
                break
        if not line.startswith("{"):
            self.close()
            raise RuntimeError("zygote did not start")
        self.info = json.loads(line)
        self.lock = threading.Lock()

    @staticmethod
    def eligible(argv: List[str]) -> bool:
        """``<this interpreter> -m module ...`` / ``-c code ...`` / ``script.py ...`` with no other
        interpreter flags: what the fork server can run exactly as ``exec`` would."""
        if len(argv) < 2:
            return False
        exe = argv[0] if os.path.sep in argv[0] else shutil.which(argv[0])
        if not exe or os.path.realpath(exe) != os.path.realpath(sys.executable):
            return False
        if argv[1] in ("-m", "-c"):
            return len(argv) >= 3
        return argv[1].endswith(".py") and not argv[1].startswith("-")

    def spawn(self, argv: List[str], env: Dict[str, str], cwd: str, out_fd: int) -> int:
        """Fork a trial process; returns its pid (re-parented to this process)."""
        msg = json.dumps({"argv": list(argv), "env": dict(env), "cwd": cwd}).encode()
        with self.lock:
            with socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET) as s:
                s.settimeout(30.0)
                s.connect(self.path)
                socket.send_fds(s, [msg], [out_fd])
                rep = json.loads(s.recv(1 << 16).decode() or "{}")
        if "pid" not in rep:
            raise RuntimeError(rep.get("error", "zygote: no reply"))
        return int(rep["pid"])

    def alive(self) -> bool:
        return self.proc.poll() is None

    def close(self):
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        try:
            os.unlink(self.path)
        except OSError:
            pass


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="katib-amd trial fork server")
    ap.add_argument("--socket", required=True)
    ap.add_argument("--preload", default=DEFAULT_PRELOAD)
    a = ap.parse_args(argv)
    return serve(a.socket, [m.strip() for m in a.preload.split(",")])


if __name__ == "__main__":
    sys.exit(main())
