"""In-tree builders for the native pieces.

* ``_native``  - C++17 runtime (store, parser, supervisor, samplers), g++ + pybind11.
* ``_hipkern`` - HIP/CDNA4 kernels for gfx950, built with hipcc through
  ``torch.utils.cpp_extension`` conventions but as an explicit in-tree ``.so`` so
  the artefact travels with the repo snapshot to the GPU box.

Both builds are incremental: a target is rebuilt only when a source is newer.
"""

from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
import time

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
NATIVE_SRC = os.path.join(PKG_DIR, "csrc", "native")
HIP_SRC = os.path.join(PKG_DIR, "csrc", "hip")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _newer(target: str, sources) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _local_includes(src: str, root: str, seen=None):
    """Headers of ``root`` that ``src`` includes with ``#include "..."``, transitively: a
    translation unit is recompiled only when one of ITS headers changes."""
    seen = set() if seen is None else seen
    try:
        lines = open(src, errors="replace").read().splitlines()
    except OSError:
        return seen
    for ln in lines:
        ln = ln.strip()
        if ln.startswith("#include") and '"' in ln:
            h = os.path.join(root, ln.split('"')[1])
            if os.path.exists(h) and h not in seen:
                seen.add(h)
                _local_includes(h, root, seen)
    return seen


def native_target() -> str:
    return os.path.join(PKG_DIR, "_native" + EXT_SUFFIX)


def build_native(force: bool = False, verbose: bool = False) -> str:
    import pybind11

    srcs = sorted(glob.glob(os.path.join(NATIVE_SRC, "*.cpp")))
    deps = srcs + sorted(glob.glob(os.path.join(NATIVE_SRC, "*.hpp")))
    out = native_target()
    if not force and not _newer(out, deps):
        return out
    inc = [pybind11.get_include(), sysconfig.get_paths()["include"], NATIVE_SRC]
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-result"]
    cmd += [f"-I{i}" for i in inc] + srcs + ["-o", out + ".tmp", "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build_selftest(sanitize: str = "address,undefined", out_dir: str = "", verbose: bool = False) -> str:
    """Standalone native self-test executable (csrc/native/tests/native_selftest.cpp) linked
    with the runtime sources, optionally under ``-fsanitize=<sanitize>`` (host code only:
    ``address,undefined`` or ``thread``); sanitizer runtimes are linked statically so the
    binary runs without any preloading."""
    srcs = [s for s in sorted(glob.glob(os.path.join(NATIVE_SRC, "*.cpp"))) if not s.endswith("bindings.cpp")]
    srcs.append(os.path.join(NATIVE_SRC, "tests", "native_selftest.cpp"))
    deps = srcs + sorted(glob.glob(os.path.join(NATIVE_SRC, "*.hpp")))
    tag = sanitize.replace(",", "_") if sanitize else "plain"
    out_dir = out_dir or os.path.join(NATIVE_SRC, "build")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "native_selftest_" + tag)
    if not _newer(out, deps):
        return out
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-Wall", "-Wno-unused-result", f"-I{NATIVE_SRC}"]
    if sanitize:
        cmd += [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
        cmd += ["-static-libtsan"] if "thread" in sanitize else ["-static-libasan", "-static-libubsan"]
    cmd += srcs + ["-o", out + ".tmp", "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


# Per-translation-unit compiler flags: MFMA accumulators in VGPRs instead of AGPRs where the kernels
# read or rescale accumulators inside their loops. transformer.hip (flash attention): the online softmax
# reads every score tile, with AGPR accumulators each tile cost ~190 v_accvgpr moves (attn_fwd_k 1124 ->
# 911 instructions, 208 -> 160 VGPRs; 293 -> 450 TFLOP/s with the softmax changes, profiles/attention_r05.log).
# darts_ops_fwd.hip / darts_ops_pwb.hip (DARTS pointwise MFMA): darts-gpu.yaml step 41.86 -> 40.71 ms, B5
# neutral (profiles/darts_vgpr_form_ab_r05.log).
_VGPR_FORM = ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
HIP_TU_FLAGS = {"transformer.hip": _VGPR_FORM, "darts_ops_fwd.hip": _VGPR_FORM, "darts_ops_pwb.hip": _VGPR_FORM}


def hip_target() -> str:
    return os.path.join(PKG_DIR, "_hipkern" + EXT_SUFFIX)


def build_hip(force: bool = False, verbose: bool = False, arch: str = "gfx950", defines=(), out: str = "",
              build_dir: str = "", tu_flags=None) -> str:
    """Compile every ``csrc/hip/*.hip`` kernel file + the torch binding into one .so.
    ``defines`` / ``out`` / ``build_dir`` build a tuning variant elsewhere (e.g.
    ``defines=["KATIB_HIP_REP=8"]``), loadable with ``KATIB_AMD_HIPKERN=<path>``."""
    import torch
    from torch.utils import cpp_extension as ce

    srcs = sorted(glob.glob(os.path.join(HIP_SRC, "*.hip"))) + sorted(glob.glob(os.path.join(HIP_SRC, "*.cpp")))
    deps = srcs + sorted(glob.glob(os.path.join(HIP_SRC, "*.h")))
    out = out or hip_target()
    if not srcs:
        return ""
    if not force and not _newer(out, deps):
        return out
    t_start = time.time()
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    hipcc = os.path.join(rocm, "bin", "hipcc")
    torch_inc = ce.include_paths()  # torch + torch/csrc/api
    py_inc = sysconfig.get_paths()["include"]
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    build_dir = build_dir or os.path.join(PKG_DIR, "csrc", "hip", "build")
    os.makedirs(build_dir, exist_ok=True)
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={arch}", "-D__HIP_PLATFORM_AMD__=1",
              "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_hipkern", "-DTORCH_API_INCLUDE_EXTENSION_H",
              "-D_GLIBCXX_USE_CXX11_ABI=" + str(int(torch._C._GLIBCXX_USE_CXX11_ABI)),
              "-fno-gpu-rdc", "-Wno-unused-result", "-Wno-deprecated-declarations"] + ["-D" + d for d in defines]
    inc = [f"-I{p}" for p in torch_inc + [py_inc, HIP_SRC]]
    objs, cmds = [], []
    for s in srcs:
        o = os.path.join(build_dir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + sorted(_local_includes(s, HIP_SRC))):
            lang = ["-x", "hip"] if s.endswith(".hip") else []
            extra = (HIP_TU_FLAGS if tu_flags is None else tu_flags).get(os.path.basename(s), [])
            cmds.append([hipcc] + common + extra + inc + lang + ["-c", s, "-o", o])
    # One hipcc per translation unit, run concurrently (bounded by MAX_JOBS / CPU count).
    jobs = max(1, min(len(cmds) or 1, int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 4), 16))
    pending, running = list(cmds), []
    while pending or running:
        while pending and len(running) < jobs:
            cmd = pending.pop(0)
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            running.append((cmd, subprocess.Popen(cmd), time.time()))
        cmd, proc, t0 = running.pop(0)
        if proc.wait() != 0:
            for _, p, _ in running:
                p.wait()
            raise subprocess.CalledProcessError(proc.returncode, cmd)
        # date the object to when its compile STARTED: a source edited while hipcc ran (whose
        # device and host passes may then have read different versions) stays newer than the
        # object, so the next build recompiles it instead of linking a torn object
        os.utime(cmd[-1], (t0, t0))
    link = [hipcc, "-shared", "-fPIC", f"--offload-arch={arch}"] + objs + [
        f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
        f"-Wl,-rpath,{torch_lib}", "-o", out + ".tmp"]
    if verbose:
        print(" ".join(link), file=sys.stderr)
    subprocess.check_call(link)
    os.replace(out + ".tmp", out)
    os.utime(out, (t_start, t_start))
    return out


def zbf16_target() -> str:
    return os.path.join(PKG_DIR, "_hipkern_zbf16" + EXT_SUFFIX)


def build_hip_zbf16(force: bool = False, verbose: bool = False) -> str:
    """The bf16-intermediates variant of the HIP extension (``-DKATIB_DARTS_ZBF16``: the DARTS
    edge kernels store depthwise outputs and pre-BN op outputs as bf16), loaded with
    ``KATIB_AMD_HIPKERN=<this path>`` by ``bench.py --dtype bf16`` and its GPU tests."""
    return build_hip(force=force, verbose=verbose, defines=["KATIB_DARTS_ZBF16"], out=zbf16_target(),
                     build_dir=os.path.join(PKG_DIR, "csrc", "hip", "build_zbf16"))


def stamps_target() -> str:
    return os.path.join(PKG_DIR, "_hipkern_stamps" + EXT_SUFFIX)


def build_hip_stamps(force: bool = False, verbose: bool = False) -> str:
    """Diagnostic variant (``-DKATIB_HIP_STAMPS``): the DARTS plane / pool kernels record per-workgroup
    phase timestamps of one armed launch (``stamps_arm``; ``scripts/darts_phase_stamps.py``). Never
    loaded by default; ``KATIB_AMD_HIPKERN=<this path>`` selects it."""
    return build_hip(force=force, verbose=verbose, defines=["KATIB_HIP_STAMPS"], out=stamps_target(),
                     build_dir=os.path.join(PKG_DIR, "csrc", "hip", "build_stamps"))


if __name__ == "__main__":
    print(build_native(verbose=True))
    print(build_hip(verbose=True))
