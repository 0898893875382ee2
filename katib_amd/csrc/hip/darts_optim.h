// DARTS search-step optimizer kernels: the architect's virtual step and
// finite-difference Hessian perturbations, Adam on the architecture weights and the clipped
// momentum-SGD weight update, each one launch over the flat fp32 parameter buffers instead
// of a chain of ~10-20 elementwise framework ops.
//
// Reference: examples/v1beta1/trial-images/darts-cnn-cifar10/architect.py:30-135 (virtual
// step w' = w - xi (mu m + g + wd w), eps = 0.01 / ||dw'||, alpha.grad = dalpha - xi (dalpha+ -
// dalpha-) / (2 eps)), run_trial.py:113-116,195-205 (Adam(betas=(0.5, 0.999), weight decay) on
// alphas; clip_grad_norm_ + SGD(momentum, weight decay) on weights).
//
// Norms are two launches without atomics or memsets: sumsq writes one fp64 partial per
// workgroup (every slot overwritten), and every workgroup of the consuming kernel re-reduces
// the <= kMaxParts partials in a fixed order, so results are deterministic. Device scalars
// (lr, eps, Adam step) keep the whole step host-sync free for HIP-graph replay.
#pragma once
#include <hip/hip_runtime.h>

namespace katib_hip {
namespace optim {

constexpr int kThreads = 256;
constexpr int kMaxParts = 256;

// number of workgroups (= partials) sumsq uses for n elements
int sumsq_parts(int n);
void launch_sumsq(const float* x, int n, double* parts, hipStream_t st);

struct VirtualStepArgs {
  float* wv;          // out: w' = w - lr * (mu * mom + g + wd * w)
  const float* w;
  const float* mom;
  const float* g;
  const float* lr;    // device scalar
  float mu, wd;
  int n;
  float* av;          // out: alpha' = alpha
  const float* a;
  int na;
  float* zero_w;      // zeroed (virtual weight-gradient row), n_zero_w elements
  int n_zero_w;
  float* zero_a;      // zeroed (virtual alpha gradients), na elements
};
void launch_virtual_step(const VirtualStepArgs& a, hipStream_t st);

// phase 0: eps = 0.01 / sqrt(sum parts) -> *eps; w += d * eps; ga = 0
// phase 1: w -= d * (2 eps); gap = ga; ga = 0
// phase 2: w += d * eps; alpha_grad = gav - lr * (gap - ga) / (2 eps)
//          [+ BN running statistics of the two concurrent passes merged, below]
// Concurrent form (the +eps and -eps passes as two independent graph branches):
// phase 3: eps -> *eps; wp = w + d * eps; wm = wp - d * (2 eps) (the sequential rounding);
//          ga = gap = 0; bn_plus = bn_zero = bn (running stats [mean | var], nbn floats)
// phase 2 with n = 0 then leaves w alone and, when nbn > 0, sets
//          bn = (1 - m) * bn_plus + bn - (1 - m) * bn_zero
//          = the two sequential momentum updates (+ pass on bn_plus, - pass on bn, both from r0)
struct HessianArgs {
  float* w;
  const float* d;     // dw' (virtual weight gradient)
  int n;
  float* eps;         // device scalar (written in phase 0)
  const double* parts;
  int nparts;
  float* ga;          // alpha gradient accumulator of the perturbed passes
  float* gap;         // dalpha+ copy
  const float* gav;   // dalpha of the unrolled pass
  float* alpha_grad;  // out (phase 2)
  const float* lr;
  int na;
  int phase;
  float* wp = nullptr;       // phase 3 outputs
  float* wm = nullptr;
  float* bn = nullptr;       // running statistics merged in phase 2 / snapshotted in phase 3
  float* bn_plus = nullptr;
  float* bn_zero = nullptr;
  int nbn = 0;
  float bn_momentum = 0.1f;
};
void launch_hessian(const HessianArgs& a, hipStream_t st);

// one workgroup: t += 1; g = grad + wd * a; m, v moments; a -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
struct AdamArgs {
  float* a;
  const float* grad;
  float* m;
  float* v;
  float* t;           // device step counter
  float lr, b1, b2, wd, eps;
  int n;
  float* zero;        // optional extra buffer zeroed by the same launch (nzero elements)
  int nzero;
};
void launch_adam(const AdamArgs& a, hipStream_t st);

// coef = min(clip / (||g|| + 1e-6), 1); g *= coef; mom = mu * mom + g + wd * w; w -= lr * mom
struct SgdArgs {
  float* w;
  float* g;
  float* mom;
  const float* lr;
  const double* parts;
  int nparts;
  float clip, mu, wd;
  int n;
};
void launch_sgd_clip(const SgdArgs& a, hipStream_t st);

}  // namespace optim
}  // namespace katib_hip
