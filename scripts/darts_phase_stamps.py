#!/usr/bin/env python3
"""Per-workgroup phase timestamps of the DARTS plane kernels on the B5 step (diagnostic build).

Loads the ``_hipkern_stamps`` variant (``_build.build_hip_stamps``, ``-DKATIB_HIP_STAMPS``), runs
the B5 search step eagerly and, for each armed launch of the depthwise backward, dw-pw forward and
pool backward kernels, prints: workgroups, the launch span (first workgroup start -> last
workgroup end, device clock), the spread of workgroup start times (dispatch / residency waves) and
the median / p90 duration of every phase inside a workgroup. Usage:
    python scripts/darts_phase_stamps.py [--config b5|default] [--calls 4]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from katib_amd import _build  # noqa: E402

os.environ.setdefault("KATIB_AMD_HIPKERN", _build.stamps_target())

import torch  # noqa: E402

KINDS = {1: ("dw_bwd_plane_multi", ["prologue", "stage", "input-grad", "wgrad", "flush"]),
         2: ("dwpw_plane_multi", ["prologue", "stage", "compute", "stats"]),
         3: ("pool_bwd_multi", ["coeffs", "stage", "gather+store"])}


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="b5")
    ap.add_argument("--calls", type=int, default=6)
    args = ap.parse_args()
    sys.path.insert(0, ROOT)
    import bench
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops

    dev = torch.device("cuda", 0)
    dops.set_backend("hip")
    from katib_amd.ops import hip_darts as hd

    K = hd._K
    assert K.stamps_compiled(), "not the stamps build (KATIB_AMD_HIPKERN)"
    cfg = bench.CONFIGS[args.config]
    layout = DartsLayout(bench.PRIMS, init_channels=cfg["init_channels"], num_layers=cfg["num_layers"],
                         num_nodes=cfg["num_nodes"], stem_multiplier=cfg["stem_multiplier"])
    search = DartsSearch(layout, dev, capture=False)
    x = torch.randn(128, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (128,), device=dev)
    for _ in range(3):
        search.step(x, y, x, y)
    torch.cuda.synchronize()
    buf = torch.zeros(65536 * 8, dtype=torch.int64, device=dev)
    for kind, (name, phases) in KINDS.items():
        print("== %s" % name)
        print("%5s %6s %8s %8s %8s | %s" % ("call", "WGs", "span_us", "start90", "startmx",
                                           " | ".join("%s p50/p90" % p for p in phases)))
        for call in range(args.calls):
            buf.zero_()
            K.stamps_arm(kind, call, buf)
            search.step(x, y, x, y)
            torch.cuda.synchronize()
            K.stamps_arm(0, 0, buf)
            st = buf.view(65536, 8).cpu()
            rows = st[st[:, 0] > 0]
            if rows.shape[0] == 0:
                break
            t0 = int(rows[:, 0].min())
            npz = len(phases) + 1
            end = rows[:, len(phases)]
            span = (int(end.max()) - t0) / 100.0  # 100 MHz -> us
            starts = [(int(r) - t0) / 100.0 for r in rows[:, 0]]
            cols = []
            for k in range(1, npz):
                d = [(int(r[k]) - int(r[k - 1])) / 100.0 for r in rows if r[k] > 0 and r[k - 1] > 0]
                cols.append("%5.2f/%5.2f" % (pct(d, 0.5), pct(d, 0.9)))
            print("%5d %6d %8.2f %8.2f %8.2f | %s" % (call, rows.shape[0], span, pct(starts, 0.9), max(starts),
                                                      " | ".join(cols)), flush=True)


if __name__ == "__main__":
    main()
