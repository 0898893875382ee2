"""Child process of tests/test_gpu_darts_bf16.py: loads the bf16-intermediates build of the HIP
extension (KATIB_AMD_HIPKERN, set by the parent) and compares it with the fp32 PyTorch oracle.
Prints one JSON line."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

ALL = ["max_pooling_3x3", "avg_pooling_3x3", "skip_connection", "separable_convolution_3x3",
       "separable_convolution_5x5", "dilated_convolution_3x3", "dilated_convolution_5x5"]


def rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def margin_check(alt, alh, tol, k=2):
    """Compare the genotype choices (models/darts.py SearchSpace.parse: per node the top-k edges by
    their strongest non-'none' alpha, and that alpha's op) of the oracle alphas ``alt`` and the
    HIP alphas ``alh``. A differing choice is a near tie when the oracle's own alphas separate the
    two alternatives by at most ``tol`` (twice the measured alpha drift); otherwise decisive."""
    near = decisive = 0
    for At, Ah in zip(alt, alh):
        st, ot = At[:, :-1].max(1)
        sh, oh = Ah[:, :-1].max(1)
        et = set(torch.topk(st, k).indices.tolist())
        eh = set(torch.topk(sh, k).indices.tolist())
        for e_new in eh - et:
            for e_old in et - eh:
                if abs(float(st[e_new] - st[e_old])) <= tol:
                    near += 1
                else:
                    decisive += 1
        for e in et & eh:
            if int(ot[e]) != int(oh[e]):
                if abs(float(At[e, ot[e]] - At[e, oh[e]])) <= tol:
                    near += 1
                else:
                    decisive += 1
    return near, decisive


def main():
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops
    from katib_amd.ops import hip_darts

    out = {"zbf16": hip_darts.ZDT == torch.bfloat16}
    dev = torch.device("cuda", 0)
    # one captured step, then a 30-step trajectory (as test_search_trajectory_30_steps_matches_torch)
    layout = DartsLayout(ALL, init_channels=4, num_layers=2, num_nodes=3, stem_multiplier=1)
    gen = torch.Generator(device=dev).manual_seed(21)
    proto = torch.randn(10, 3, 1, 1, device=dev, generator=gen)
    batches = []
    for _ in range(4):
        ty = torch.randint(0, 10, (32,), device=dev, generator=gen)
        vy = torch.randint(0, 10, (32,), device=dev, generator=gen)
        tx = proto[ty] + 0.5 * torch.randn(32, 3, 32, 32, device=dev, generator=gen)
        vx = proto[vy] + 0.5 * torch.randn(32, 3, 32, 32, device=dev, generator=gen)
        batches.append((tx, ty, vx, vy))
    res = {}
    for backend in ("torch", "hip"):
        dops.set_backend(backend)
        s = DartsSearch(layout, dev, capture=backend == "hip", settings={"alpha_lr": 3e-2})
        A0 = s.A.clone()
        first = None
        losses = []
        for i in range(30):
            losses.append(float(s.step(*batches[i % 4])))
            if i == 0:
                first = (s.W.clone(), s.A.clone())
        torch.cuda.synchronize()
        alphas = [a.detach().clone() for a in list(s.An) + list(s.Ar)]
        res[backend] = (losses, s.W.clone(), s.A.clone(), A0, str(s.genotype()), first, alphas)
    dops.set_backend("torch")
    (lt, Wt, At, A0, gt, ft, alt), (lh, Wh, Ah, _, gh, fh, alh) = res["torch"], res["hip"]
    drift = float((Ah - At).abs().max())
    near, decisive = margin_check(alt, alh, 2 * drift)
    out.update({
        "step1_W_rel": rel(fh[0], ft[0]),
        "step1_alpha_abs": float((fh[1] - ft[1]).abs().max()),
        "loss_max_abs_diff": max(abs(a - b) for a, b in zip(lt, lh)),
        "loss_first": [lt[0], lh[0]],
        "alpha_displacement": float((At - A0).abs().max()),
        "alpha_drift": float((Ah - At).abs().max()),
        "W_rel": rel(Wh, Wt),
        "genotype_equal": gt == gh,
        "genotype_near_tie_diffs": near,
        "genotype_decisive_diffs": decisive,
        "genotype_torch": gt,
        "genotype_hip": gh,
    })
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
