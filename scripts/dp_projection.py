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

Prints the table; `profiles/dp_projection_r06.log` is its output.
"""

FLOOR_MS = {  # per-rank batch -> measured dp1 step (ms), round 6 final kernels (profiles/dp_floors_r06.log)
    "b5": {128: 5.33, 64: 3.92, 32: 3.17, 16: 2.87},
    "default": {128: 38.29, 64: 22.47, 32: 15.21, 16: 11.86},
}
# SyncBN rendezvous on the step's critical path, measured with 2 ranks (profiles/dp_rendezvous_r06.log): the
# concurrent Hessian branches fold through two workspaces side by side, so of 175 (B5) / 315 (default)
# rendezvous per step 141 / 253 are serial - exactly the count of the stacked mode, where each twin pair of
# folds is one rendezvous.
RENDEZVOUS = {"b5": 141, "default": 253}
# SyncBN fold rendezvous floor (us) with the single-workgroup small-payload path of fold_sync (round 6):
# 2 / 4 ranks measured (scripts/rendezvous_probe.py, 1 workgroup, 64-2048 floats: 4.1-4.25 / 5.0-5.2 us,
# profiles/rendezvous_r06.log) with every rank on ONE GPU, 8 extrapolated linearly in the peer count
# (+0.45 us per peer). Round 5 ran 16 workgroups: 6.1 / 10.3 / 18.5.
T_RV_US = {1: 0.0, 2: 4.2, 4: 5.1, 8: 6.9}
# gradient-bucket all-reduces (one-shot, B5-size vectors ~9.5k floats, 16 workgroups): 5.9 / 9.7 us, 8 extrapolated
T_GRAD_US = {1: 0.0, 2: 5.9, 4: 9.7, 8: 17.3}
GRAD_ALLREDUCES = 4


def main():
    print("DARTS DP projection (NOT a measurement; inputs measured on one MI355X, see scripts/dp_projection.py)")
    for cfg in ("b5", "default"):
        f, R = FLOOR_MS[cfg], RENDEZVOUS[cfg]
        base = f[128]
        print(f"\n== {cfg}: strong scaling, global batch 128, SyncBN ({R} serial rendezvous/step)")
        print(" N | per-rank batch | floor ms | rendezvous ms | step ms | speedup vs 1 GPU | images/s"
              " | step ms if t_rv stays at the 2-rank figure")
        for n in (1, 2, 4, 8):
            b = 128 // n
            rv = 0.0 if n == 1 else (R - GRAD_ALLREDUCES) * T_RV_US[n] / 1000.0 + GRAD_ALLREDUCES * T_GRAD_US[n] / 1000.0
            step = f[b] + rv
            opt = f[b] + (0.0 if n == 1 else (R - GRAD_ALLREDUCES) * T_RV_US[2] / 1000.0
                          + GRAD_ALLREDUCES * T_GRAD_US[2] / 1000.0)
            print(f" {n} | {b:>14} | {f[b]:8.2f} | {rv:13.2f} | {step:7.2f} | {base / step:16.2f} | {128 / step * 1000:8.0f}"
                  f" | {opt:7.2f} ({base / opt:.2f}x)")
        print(f"== {cfg}: strong scaling, global batch 128, per-rank BN (--sync-bn 0: BN over 128/N images, "
              f"{GRAD_ALLREDUCES} rendezvous/step)")
        print(" N | step ms | speedup vs 1 GPU")
        for n in (1, 2, 4, 8):
            rv = 0.0 if n == 1 else GRAD_ALLREDUCES * T_GRAD_US[n] / 1000.0
            step = f[128 // n] + rv
            print(f" {n} | {step:7.2f} | {base / step:16.2f}")
        print(f"== {cfg}: weak scaling, batch 128 per rank, per-rank BN ({GRAD_ALLREDUCES} rendezvous/step)")
        print(" N | step ms | images/s | efficiency")
        for n in (1, 2, 4, 8):
            rv = 0.0 if n == 1 else GRAD_ALLREDUCES * T_GRAD_US[n] / 1000.0
            step = base + rv
            print(f" {n} | {step:7.2f} | {128 * n / step * 1000:8.0f} | {base / step:10.3f}")
    print("\nReading: with the single-workgroup fold rendezvous (4.2 / 5.1 us at 2 / 4 ranks instead of 6.1 / 10.3) and"
          "\nthe serial count the concurrent Hessian branches really pay (141 of 175 on B5), the round-6 floors"
          "\n(B5 5.33 ms, default 38.3 ms at batch 128) give the table above; per-rank BN (the reference's DDP"
          "\nsemantics) and weak scaling are unchanged in kind.")


if __name__ == "__main__":
    main()
