// Kernels that close the fused ResNet-18 train step (ops/resnet_step.py) so that every launch
// in the captured step is a katib_hip kernel: the batch gather + channel pad of the input, the
// classifier head (global average pool + linear + cross-entropy, forward and backward in one
// pass) and its weight gradient, and one multi-tensor SGD launch that also re-emits the bf16
// filter images the convolutions read and zeroes the fp32 gradient accumulators.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdint>

namespace katib_hip {
namespace rn {

typedef __hip_bfloat16 bf16;

// xb[b][p][0..C8) = tx[idx[b]][p][0..C) zero-padded to C8 (NHWC bf16), p < HW.
hipError_t launch_gather(const bf16* tx, const int64_t* idx, bf16* xb, int B, int HW, int C, int C8, int64_t n_src,
                         hipStream_t st);

struct HeadArgs {
  const bf16* x;        // [B][HW][C] final activation
  const float* w;       // [K][C]
  const float* bias;    // [K]
  const int64_t* ty;    // labels of the whole set
  const int64_t* idx;   // [B] batch indices into ty
  int64_t n_labels;
  bf16* dx;             // [B][HW][C] gradient of x
  float* pooled;        // [B][C] scratch
  float* dl;            // [B][K] scratch: d loss / d logits (mean over the batch folded in)
  float* loss_n;        // [B] scratch
  float* gw;            // [K][C] weight gradient (written)
  float* gb;            // [K] bias gradient (written)
  float* loss_acc;      // scalar, += mean loss (may be nullptr)
  int B, HW, C, K;
};
constexpr int kHeadMaxC = 2048;
constexpr int kHeadMaxK = 64;
// Two launches: per-sample forward + backward, then the batch reductions (weight / bias
// gradient, mean loss) in a fixed order (no atomics: bitwise reproducible).
hipError_t launch_head(const HeadArgs& a, hipStream_t st);

// One parameter tensor of the fused SGD. Conv filters (wk != nullptr): p / m are the fp32 master
// and momentum in [K][RS][C] order (channels_last storage of [K][C][R][S]), g the fp32 gradient
// accumulator [K][RS][C8] the wgrad kernel adds into; the kernel writes wk = bf16 [K][RS][C8]
// (zero-padded) and, when wt != nullptr, wt = bf16 [C8][RS][K] for the input-gradient GEMM.
// Flat tensors (wk == nullptr): n elements of p / g / m.
struct SgdSeg {
  float* p;
  float* g;
  float* m;
  bf16* wk;
  bf16* wt;
  int K, C, C8, RS;
  int n;
  int tile0;  // first workgroup of this segment in the launch
};
// update = 0: only (re)write the bf16 filter images from p (initialisation).
hipError_t launch_sgd(const SgdSeg* segs_dev, int nseg, int total_tiles, float lr, float momentum, float wd,
                      int nesterov, int update, hipStream_t st);
// Workgroups a segment needs.
int sgd_tiles(const SgdSeg& s);

}  // namespace rn
}  // namespace katib_hip
