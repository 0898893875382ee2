"""Run-to-run determinism of the HIP DARTS search step on one GPU: two identical single-process
searches (same seed, same data), compared bitwise after 1 and after STEPS steps - weights, alphas,
BN running statistics. Run against the default kernel library or a variant
(KATIB_AMD_HIPKERN=<.so>, e.g. one built with KATIB_HIP_REP=2048 so that every workgroup of a
persistent grid owns its own reduction replica)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from katib_amd.models.darts import DartsLayout  # noqa: E402
from katib_amd.models.darts_search import DartsSearch  # noqa: E402
from katib_amd.ops import darts as dops  # noqa: E402
from katib_amd.parallel.comm import Comm  # noqa: E402


def main():
    steps = int(os.environ.get("STEPS", "30"))
    capture = os.environ.get("CAPTURE", "1") == "1"
    dev = torch.device("cuda", 0)
    dops.set_backend("hip")
    layout = DartsLayout(["separable_convolution_3x3", "dilated_convolution_3x3", "dilated_convolution_5x5",
                          "avg_pooling_3x3", "max_pooling_3x3", "skip_connection"], init_channels=4, num_layers=2,
                         num_nodes=3, stem_multiplier=1)
    B = 128
    g = torch.Generator().manual_seed(11)
    proto = torch.randn(10, 3, 1, 1, generator=g)
    data = []
    for _ in range(steps):
        ty, vy = torch.randint(0, 10, (B,), generator=g), torch.randint(0, 10, (B,), generator=g)
        tx = proto[ty] + 0.5 * torch.randn(B, 3, 32, 32, generator=g)
        vx = proto[vy] + 0.5 * torch.randn(B, 3, 32, 32, generator=g)
        data.append([t.to(dev) for t in (tx, ty, vx, vy)])
    runs = []
    for _ in range(2):
        s = DartsSearch(layout, dev, Comm(device=dev), seed=3, capture=capture)
        snaps = []
        for i, (tx, ty, vx, vy) in enumerate(data):
            s.step(tx, ty, vx, vy)
            if i == 0 or i == steps - 1:
                torch.cuda.synchronize()
                snaps.append({"W": s.W.clone(), "A": s.A.clone(), "bn": s.bn.mean.clone()})
        runs.append((snaps, str(s.genotype())))
    out = {"steps": steps, "capture": capture, "lib": os.environ.get("KATIB_AMD_HIPKERN", "default")}
    for j, tag in enumerate(("step1", "final")):
        for k in ("W", "A", "bn"):
            a, b = runs[0][0][j][k], runs[1][0][j][k]
            out["%s_%s_equal" % (tag, k)] = bool(torch.equal(a, b))
            out["%s_%s_maxdiff" % (tag, k)] = float((a - b).abs().max())
            out["%s_%s_ndiff" % (tag, k)] = int((a != b).sum())
    out["geno_equal"] = runs[0][1] == runs[1][1]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
