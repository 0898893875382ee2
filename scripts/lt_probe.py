"""Which hipBLASLt epilogues have bf16 solutions on this GPU (scripts/gpu_r05dd.sh diagnostics)."""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from katib_amd.ops.transformer import _kern  # noqa: E402

k = _kern()
torch.zeros(1, device="cuda")
EPI = {"DEFAULT": 1, "BIAS": 4, "GELU": 32, "GELU_BIAS": 36, "GELU_AUX": 160, "GELU_AUX_BIAS": 164, "DGELU": 192,
       "DGELU_BGRAD": 208, "BGRADA": 256, "BGRADB": 512}
BF16, F32 = 14, 0  # hipDataType HIP_R_16BF, HIP_R_32F
for name, e in EPI.items():
    for ta, tb in itertools.product((0, 1), (0, 1)):
        for bt, at in ((-1, -1), (BF16, -1), (F32, -1), (BF16, BF16), (F32, BF16), (F32, F32)):
            r = k.lt_probe(e, ta, tb, 3072, 16384, 768, bt, at)
            if r != 0:
                print(f"{name:14s} ta={ta} tb={tb} bias_t={bt:2d} aux_t={at:2d} -> {r}", flush=True)
print("probe done", flush=True)
