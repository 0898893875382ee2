// Fused DARTS network head (SURVEY K9 + K11): global average pool -> classifier -> log-softmax +
// NLL, and its backward, as one workgroup per sample instead of ~6 forward and ~10 backward
// framework launches (mean reduce, GEMM, log_softmax, nll, fills; nll/log_softmax backward, two
// GEMMs, bias reduce, pool backward, grad accumulation).
//
// Reference: examples/v1beta1/trial-images/darts-cnn-cifar10/model.py:156-161 (gap + linear),
// model.py:185 / run_trial.py:199-207 (nn.CrossEntropyLoss, mean reduction).
//
// head_fwd   per sample n: pooled[n][c] = mean_hw x; logits = pooled W^T + b; loss_n = lse - logit_y;
//            dl[n][k] = (softmax_k - [k == y]) / N   (d loss / d logits for a unit upstream gradient)
// head_loss  loss = sum_n loss_n / N   (one workgroup, fixed order)
// head_bwd   per sample n, g = upstream gradient (device scalar): dx[n][c][:] = g (dl[n] W)[c] / HW;
//            weight / bias gradients accumulate g dl[n][k] pooled[n][c] into replica n % kRep.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace katib_hip {
namespace head {

constexpr int kMaxC = 1024;
constexpr int kMaxK = 64;

struct FwdArgs {
  const float* x;     // [N][C][HW]
  const float* w;     // [K][C]
  const float* b;     // [K]
  const int64_t* y;   // [N] class indices
  float* pooled;      // [N][C]
  float* logits;      // [N][K]
  float* dl;          // [N][K]
  float* loss_n;      // [N]
  int N, C, HW, K;
  int nodes = 1;      // > 1: x is node-major [nodes][N][C / nodes][HW] (a DARTS cell output, never concatenated)
};
void launch_fwd(const FwdArgs& a, hipStream_t st);
void launch_loss(const float* loss_n, int N, float* loss, hipStream_t st);

struct BwdArgs {
  const float* dl;
  const float* pooled;
  const float* w;
  const float* gout;  // device scalar upstream gradient
  float* dx;          // [N][C][HW] (written), nullptr = not needed
  float* gw;          // weight-gradient replica 0 (replica r at gw + r * gw_stride), nullptr = skip
  int gw_stride;
  float* gb;
  int gb_stride;
  int N, C, HW, K;
  int nodes = 1;      // dx layout, as FwdArgs::nodes
};
void launch_bwd(const BwdArgs& a, hipStream_t st);

}  // namespace head
}  // namespace katib_hip
