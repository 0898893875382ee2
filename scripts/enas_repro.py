"""Bisect of the ENAS child training collapse seen in the enas-cifar10 experiment on MI355X:
one architecture, 3 epochs, with / without the captured train step (CapturedStep).
argv: "<capture>[:variant]" with variant in
  noeval  - no validation passes between epochs
  torchbn - nn.BatchNorm2d instead of the HIP NHWC batch norm
  noconv  - PyTorch conv instead of the HIP implicit-GEMM conv
  nodw    - PyTorch depthwise conv instead of the HIP depthwise kernels
  adamfe  - torch Adam (foreach, capturable) instead of the fused one"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from katib_amd.ops import batchnorm as hbn  # noqa: E402
from katib_amd.ops import conv as hconv  # noqa: E402
from katib_amd.ops import dwconv as hdw  # noqa: E402
from katib_amd.workloads import enas_child  # noqa: E402

cfg = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "enas_repro_arch.json")))
orig = dict(bn=hbn.BatchNorm2d.forward, conv=hconv.supported, dw=hdw.supported, adam=torch.optim.Adam)


class _AdamForeach(torch.optim.Adam):
    def __init__(self, params, **kw):
        kw.pop("fused", None)
        super().__init__(params, foreach=True, **kw)


for spec in sys.argv[1:] or ["1", "0"]:
    capture, _, variant = spec.partition(":")
    print("=== capture", capture, variant, flush=True)
    hbn.BatchNorm2d.forward, hconv.supported, hdw.supported = orig["bn"], orig["conv"], orig["dw"]
    enas_child.torch.optim.Adam = orig["adam"]
    if variant == "torchbn":
        hbn.BatchNorm2d.forward = lambda self, x, residual=None, relu=False: torch.nn.BatchNorm2d.forward(self, x)
    elif variant == "noconv":
        hconv.supported = lambda *a, **k: False
    elif variant == "nodw":
        hdw.supported = lambda *a, **k: False
    elif variant == "adamfe":
        enas_child.torch.optim.Adam = _AdamForeach
    extra = ["--num-valid=0"] if variant == "noeval" else []
    enas_child.main(extra + ["--num_epochs=3", "--num-train=20000", "--capture=" + capture,
                             "--architecture=" + json.dumps(cfg["architecture"]), "--nn_config=" + cfg["nn_config"]])
