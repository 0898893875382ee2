#!/usr/bin/env python3
"""Labelled PROJECTION of the DARTS data-parallel step on 1/2/4/8 MI355X:
what the driver's N-GPU bench should show, predicted from single-GPU measurements, so the
eventual 1->8 curve is checked against a model instead of being discovered.

Model (strong scaling, the bench default: global batch 128, SyncBN over all ranks):
    step(N) = floor(128 / N) + R x t_rv(N)
  floor(b)  measured dp1 step at per-rank batch b (profiles/experiments_r05.log, batch sweep)
  R         rendezvous per step measured by the 2-rank run of the same step (`rendezvous_per_step`
            key: SyncBN folds + gradient all-reduces, all inside the captured graph)
  t_rv(N)   one-shot xGMI rendezvous floor from scripts/rendezvous_probe.py (2 / 4 ranks sharing
            one GPU through IPC: launch + flag handshake, not link bandwidth; 8 ranks extrapolated
            linearly in the peer count). The folds are serial points of the step, so they add.
Weak scaling (batch 128 per rank, per-rank BN): only the gradient all-reduces rendezvous (4 per
step, one per flat gradient vector), so step(N) = floor(128) + 4 t_rv(N).

Prints the table; `profiles/dp_projection_r05.log` is its output.
"""

FLOOR_MS = {  # per-rank batch -> measured dp1 step (ms), round 5
    "b5": {128: 6.23, 64: 4.67, 32: 3.70, 16: 3.32},
    "default": {128: 41.74, 64: 24.73, 32: 16.60, 16: 12.66},
}
RENDEZVOUS = {"b5": 175, "default": 315}  # measured, 2 ranks (gpurun_out/r05f.log, r05n.log)
# 2, 4 measured (mid of 5.6-6.6 / 8.7-11.8 us) with every rank on ONE GPU, so the ranks' fold kernels
# time-share the device; 8 extrapolated linearly. On 8 separate GPUs the peers' flags are polled in
# parallel, so the 2-rank figure is the optimistic bound (last column of the SyncBN tables).
T_RV_US = {1: 0.0, 2: 6.1, 4: 10.3, 8: 18.5}
GRAD_ALLREDUCES = 4


def main():
    print("DARTS DP projection (NOT a measurement; inputs measured on one MI355X, see scripts/dp_projection.py)")
    for cfg in ("b5", "default"):
        f, R = FLOOR_MS[cfg], RENDEZVOUS[cfg]
        base = f[128]
        print(f"\n== {cfg}: strong scaling, global batch 128, SyncBN ({R} rendezvous/step)")
        print(" N | per-rank batch | floor ms | rendezvous ms | step ms | speedup vs 1 GPU | images/s"
              " | step ms if t_rv stays at the 2-rank figure")
        for n in (1, 2, 4, 8):
            b = 128 // n
            rv = 0.0 if n == 1 else R * T_RV_US[n] / 1000.0
            step = f[b] + rv
            opt = f[b] + (0.0 if n == 1 else R * T_RV_US[2] / 1000.0)
            print(f" {n} | {b:>14} | {f[b]:8.2f} | {rv:13.2f} | {step:7.2f} | {base / step:16.2f} | {128 / step * 1000:8.0f}"
                  f" | {opt:7.2f} ({base / opt:.2f}x)")
        print(f"== {cfg}: strong scaling, global batch 128, per-rank BN (--sync-bn 0: BN over 128/N images, "
              f"{GRAD_ALLREDUCES} rendezvous/step)")
        print(" N | step ms | speedup vs 1 GPU")
        for n in (1, 2, 4, 8):
            rv = 0.0 if n == 1 else GRAD_ALLREDUCES * T_RV_US[n] / 1000.0
            step = f[128 // n] + rv
            print(f" {n} | {step:7.2f} | {base / step:16.2f}")
        print(f"== {cfg}: weak scaling, batch 128 per rank, per-rank BN ({GRAD_ALLREDUCES} rendezvous/step)")
        print(" N | step ms | images/s | efficiency")
        for n in (1, 2, 4, 8):
            rv = 0.0 if n == 1 else GRAD_ALLREDUCES * T_RV_US[n] / 1000.0
            step = base + rv
            print(f" {n} | {step:7.2f} | {128 * n / step * 1000:8.0f} | {base / step:10.3f}")
    print("\nReading: strong scaling of B5 is bound twice over - by the SyncBN rendezvous (175 serial folds of ~6-18 us"
          "\nagainst a 3.3-4.7 ms per-rank floor: ~1.1x at 2-4 GPUs, flat at 8) and, without SyncBN, by the per-rank"
          "\nfloor itself (batch 16 still costs 3.3 ms: the step is launch / latency bound, 1.8x at 8). The default"
          "\nconfig (larger per-rank work) projects 1.6x / 2.1x / 2.3x with SyncBN. Weak scaling keeps >= 98%"
          "\nefficiency at 8 ranks.")


if __name__ == "__main__":
    main()
