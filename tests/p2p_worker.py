"""Producer / consumer processes for tests/test_gpu_p2p.py."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from katib_amd.parallel import p2p_ckpt  # noqa: E402


def state(dev):
    g = torch.Generator(device=dev).manual_seed(3)
    return {"model": {"w": torch.randn(1000, 333, device=dev, generator=g),
                      "b": torch.arange(17, device=dev, dtype=torch.int64)},
            "optim": {"state": {0: {"step": torch.tensor(5.0, device=dev)}}, "param_groups": [{"lr": 0.1}]},
            "step": 42}


if __name__ == "__main__":
    role, d = sys.argv[1], sys.argv[2]
    dev = torch.device("cuda", int(os.environ.get("P2P_DEVICE", "0")))
    if role == "producer":
        assert p2p_ckpt.publish(state(dev), d)
        print("published", flush=True)
        t0 = time.time()
        while not os.path.exists(os.path.join(d, "done")) and time.time() - t0 < 120:
            time.sleep(0.1)
    else:
        got = p2p_ckpt.fetch(d, dev)
        ref = state(dev)
        ok = got is not None and torch.equal(got["model"]["w"], ref["model"]["w"]) and \
            torch.equal(got["model"]["b"], ref["model"]["b"]) and got["step"] == 42 and \
            float(got["optim"]["state"][0]["step"]) == 5.0 and got["optim"]["param_groups"][0]["lr"] == 0.1
        open(os.path.join(d, "done"), "w").write("ok" if ok else "bad")
        print("fetched ok" if ok else "fetch mismatch", flush=True)
        sys.exit(0 if ok else 1)
