#!/usr/bin/env python3
"""Marginal cost of one kernel launch inside the captured B5 DARTS step graph vs in a bare graph.

(a) B5 step graph as is; (b) the same step with K extra 1-element kernels appended per segment
(at:: add_) and (c) K extra fold_f64 launches (our extension's launch path); (d) a bare graph of
K at:: add_ kernels; (e) a bare graph alternating a 2 MB streaming kernel and a tiny kernel.
Prints ms per replay / per step and the per-extra-kernel cost."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / reps


def graph_of(body):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    return g


def main():
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops
    from katib_amd.workloads.data import cifar10

    dops.set_backend("hip")
    from katib_amd.ops import hip_darts as hd

    dev = torch.device("cuda", 0)
    K = int(os.environ.get("PROBE_K", "200"))
    out = {}
    tiny = torch.zeros(1, device=dev)
    f64 = torch.zeros(64 * hd.REP, dtype=torch.float64, device=dev)
    # bare graphs
    g = graph_of(lambda: [tiny.add_(1.0) for _ in range(K)])
    out["bare_at_add_us"] = timeit(g.replay) * 1e3 / K
    g = graph_of(lambda: [hd._K.fold_f64([(f64, 64, 64)]) for _ in range(K)])
    out["bare_fold_f64_us"] = timeit(g.replay) * 1e3 / K
    big = torch.zeros(1 << 19, device=dev)  # 2 MB
    g = graph_of(lambda: [big.add_(1.0) for _ in range(K)])
    out["bare_2MB_add_us"] = timeit(g.replay) * 1e3 / K
    g = graph_of(lambda: [(big.add_(1.0), tiny.add_(1.0)) for _ in range(K)])
    out["bare_2MB_plus_tiny_us_per_pair"] = timeit(g.replay) * 1e3 / K

    prims = ["separable_convolution_3x3", "dilated_convolution_3x3", "dilated_convolution_5x5", "avg_pooling_3x3",
             "max_pooling_3x3", "skip_connection"]
    layout = DartsLayout(prims, init_channels=4, num_layers=2, num_nodes=3, stem_multiplier=1)
    ds = cifar10(dev, n=512)
    (tx, ty), (vx, vy) = next(zip(ds.subset(0, 256).batches(128, seed=0), ds.subset(256, 512).batches(128, seed=1)))

    def run(extra):
        s = DartsSearch(layout, dev, capture=True)
        if extra:
            orig = s._seg_weight_update

            def patched():
                orig()
                for _ in range(K):
                    extra()
            s._seg_weight_update = patched
        return timeit(lambda: s.step(tx, ty, vx, vy), reps=20)

    base = run(None)
    out["step_ms"] = base
    out["step_plus_K_at_add_ms"] = run(lambda: tiny.add_(1.0))
    out["step_plus_K_fold_ms"] = run(lambda: hd._K.fold_f64([(f64, 64, 64)]))
    out["marginal_at_add_us"] = (out["step_plus_K_at_add_ms"] - base) * 1e3 / K
    out["marginal_fold_us"] = (out["step_plus_K_fold_ms"] - base) * 1e3 / K
    print(json.dumps({k: round(v, 4) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
