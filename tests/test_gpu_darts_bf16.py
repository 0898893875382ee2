"""bf16-intermediates DARTS build (``_hipkern_zbf16``: depthwise outputs and pre-BN op outputs
stored as bf16, everything else fp32) against the fp32 PyTorch oracle: 30 captured
second-order search steps agree on the genotype up to near ties (choices the fp32 oracle's own
alphas separate by less than twice the measured drift), the loss trajectory within bf16
tolerance, the alpha trajectory within 15 % of its displacement. Runs in a child process because the
variant extension replaces the fp32 one module-wide."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bf16_intermediates_trajectory_matches_fp32_oracle():
    from katib_amd import _build

    so = _build.zbf16_target()
    if not os.path.exists(so):
        pytest.fail("bf16 variant not built (run __graft_entry__.build())")
    env = dict(os.environ, KATIB_AMD_HIPKERN=so)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "darts_bf16_worker.py")], env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(res)
    assert res["zbf16"], "the child did not load the bf16 variant"
    # bf16 rounding may flip choices the fp32 oracle itself separates by less than twice the
    # measured alpha drift (near ties); any decisive difference fails
    assert res["genotype_decisive_diffs"] == 0, (res["genotype_torch"], res["genotype_hip"])
    assert res["genotype_equal"] or res["genotype_near_tie_diffs"] <= 2, res
    assert res["alpha_displacement"] > 1e-2
    assert res["alpha_drift"] <= 0.15 * res["alpha_displacement"], res
    assert res["loss_max_abs_diff"] < 5e-2, res
    assert res["W_rel"] < 5e-2, res
