#!/usr/bin/env python3
"""Do independent branches of a captured HIP graph run concurrently on this stack?

Captures the same 2 x CHAIN small dependent kernels (a) on one stream and (b) as two
independent chains forked onto two streams inside one capture, replays both, and
prints ms per replay. Decides whether the DARTS Hessian passes (two independent
forward/backward chains) can overlap inside the step graph."""
import json
import time

import torch


def build(chains, n, chain, streams):
    g = torch.cuda.CUDAGraph()
    side = [torch.cuda.Stream() for _ in chains]  # created before capture
    cap = torch.cuda.Stream()
    with torch.cuda.graph(g, stream=cap):
        main = torch.cuda.current_stream()
        if streams == 1:
            for _ in range(chain):
                for x in chains:
                    x.mul_(1.0001).add_(1e-4)
        else:
            for s in side:
                s.wait_stream(main)
            for x, s in zip(chains, side):
                with torch.cuda.stream(s):
                    for _ in range(chain):
                        x.mul_(1.0001).add_(1e-4)
            for s in side:
                main.wait_stream(s)
    return g


def timeit(g, reps=50):
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / reps


def main():
    out = {}
    for n in (1 << 14, 1 << 20, 1 << 22):
        for nch in (2, 4):
            xs = [torch.zeros(n, device="cuda") for _ in range(nch)]
            chain = 200
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):  # warm-up outside capture
                for x in xs:
                    x.mul_(1.0).add_(0.0)
            torch.cuda.current_stream().wait_stream(s)
            g1 = build(xs, n, chain, 1)
            g2 = build(xs, n, chain, 2)
            for x in xs:
                x.zero_()
            g2.replay()
            torch.cuda.synchronize()
            ok = all(float(x[0]) > 0 for x in xs)  # every forked chain really ran
            out["n=%d chains=%d" % (n, nch)] = {"serial_ms": round(timeit(g1), 3),
                                                "forked_ms": round(timeit(g2), 3),
                                                "forked_ran": ok, "kernels": 2 * chain * nch}
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
