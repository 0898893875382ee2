#!/usr/bin/env python3
"""Where the cold MLP trial's 'model' phase goes (launch-side time between the dataset on the device
and the first training step): times each setup statement of workloads/mnist_mlp.main separately,
in a fresh process (first use of each kernel family included)."""
import sys
import time

t = [("start", time.time())]


def mark(n):
    t.append((n, time.time()))


import torch  # noqa: E402

mark("import_torch")
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from katib_amd.workloads import mnist_mlp as mm  # noqa: E402
from katib_amd.workloads.common import CapturedStep, device, teacher_vectors  # noqa: E402

mark("import_katib")
opt_name = sys.argv[1] if len(sys.argv) > 1 else "adam"
dev = device()
torch.zeros(1, device=dev).add_(1)
torch.cuda.synchronize()
mark("hip_init")
x, y = teacher_vectors(70000, seed=1234, dev=dev)
torch.cuda.synchronize()
mark("data")
torch.manual_seed(0)
model = mm.DeepMLP(256, 3)
mark("model_ctor")
model = model.to(dev)
torch.cuda.synchronize()
mark("model_to_dev")
if opt_name == "adam":
    opt = torch.optim.Adam(model.parameters(), lr=0.01, capturable=True)
elif opt_name == "ftrl":
    opt = mm.Ftrl(model.parameters(), lr=0.01)
else:
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9)
torch.cuda.synchronize()
mark("optimizer")
for p_ in model.parameters():
    p_.grad = torch.zeros_like(p_)
torch.cuda.synchronize()
mark("zero_grads")
if opt_name == "adam":
    opt.step()
    torch.cuda.synchronize()
mark("adam_prestep")
idx = torch.zeros(64, dtype=torch.long, device=dev)
import torch.nn.functional as F  # noqa: E402


def step():
    xb, yb = x.index_select(0, idx), y.index_select(0, idx)
    with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
        loss = F.cross_entropy(model(xb), yb)
    opt.zero_grad(set_to_none=False)
    loss.backward()
    opt.step()
    return loss


step()
torch.cuda.synchronize()
mark("first_eager_step")
step()
torch.cuda.synchronize()
mark("second_eager_step")
cs = CapturedStep(step, warmup=1)
cs()
cs()
torch.cuda.synchronize()
mark("capture")
for (a, ta), (b, tb) in zip(t, t[1:]):
    print("%-20s %7.3f s" % (b, tb - ta))
print("total %.3f s" % (t[-1][1] - t[0][1]))
