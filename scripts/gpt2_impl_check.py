"""Compare the GPT-2 trial implementations on one GPU: flat HIP model vs nn.Module (eager / captured)."""
import sys

sys.path.insert(0, ".")
from katib_amd.workloads import gpt2_pbt  # noqa: E402
from katib_amd.workloads.gpt2_pbt import GPTConfig  # noqa: E402

gpt2_pbt.PRESETS["t"] = GPTConfig(vocab=1000, ctx=128, n_layer=2, n_head=4, d=256)
common = ["--model", "t", "--batch-size", "8", "--lr", "3e-3", "--num-tokens", "200000", "--p2p", "0", "--steps", "40"]
for extra in (["--impl", "flat"], ["--impl", "module", "--capture", "0"], ["--impl", "module", "--capture", "1"]):
    print(extra, gpt2_pbt.main(common + extra), flush=True)
