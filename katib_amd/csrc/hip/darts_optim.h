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
  float* g_zero = nullptr;  // optional: g's buffer zeroed after use (the model gradient row for the next pass)
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
  int zero_g = 0;  // 1: g left zeroed (for the next step's first pass) instead of holding the clipped gradient
};
void launch_sgd_clip(const SgdArgs& a, hipStream_t st);

// Architecture-weight softmax of the DARTS network forward (model.py:147-148): softmax over the
// primitives of every row of up to two [rows][K] alpha matrices (normal, reduce cells) in one
// workgroup; the same launch optionally zeroes an f64 buffer (the step's BN-reduction arena), so
// the step's first two launches become one.
struct AlphaSoftmaxArgs {
  const float* a[2];
  float* w[2];
  int rows[2];
  int nmat, K;
  double* zero;  // optional, nzero doubles
  long long nzero;
};
void launch_alpha_softmax(const AlphaSoftmaxArgs& a, hipStream_t st);

// d(loss)/d(alpha) from the edges' d(loss)/d(softmax weight) (kRep f64 replicas each, summed here)
// through the softmax Jacobian, d alpha_k = w_k (g_k - sum_j w_j g_j), summed over every edge that
// shares the row (cells of one type share their alphas) and written or added into the alpha
// gradient rows: one launch replaces the replica fold, the row concatenation, the dtype copy, the
// softmax backward and the gradient accumulation of the autograd path. Workgroup per row.
constexpr int kAlphaGradMax = 128;  // both stacked Hessian passes' entries
struct AlphaGradArgs {
  const double* g[kAlphaGradMax];
  int rstride[kAlphaGradMax];
  const float* w[kAlphaGradMax];   // softmax weights of the entry's row
  float* dst[kAlphaGradMax];       // destination rows, K floats each
  int row_start[kAlphaGradMax + 1];  // entries of destination row r: [row_start[r], row_start[r + 1])
  int n, nrows, K, accumulate;
};
void launch_alpha_grad(const AlphaGradArgs& a, hipStream_t st);

}  // namespace optim
}  // namespace katib_hip
