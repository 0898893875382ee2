// ENAS LSTM controller on gfx950: arc sampling + REINFORCE training in one persistent workgroup.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace katib_hip {
namespace enas {

constexpr int kThreads = 256;
constexpr int kMaxH = 64;       // 4H gate columns <= 256 threads (one column per thread)
constexpr int kMaxOps = 1024;
constexpr int kMaxLayers = 64;
constexpr int kLogFields = 8;   // loss, entropy, grad_norm, baseline, skip_rate, sum CE, mean KL, advantage

// Flat parameter layout (same order as the torch controller's parameters()):
// w_lstm [2H, 4H], g_emb [1, H], w_emb [n_ops, H], w_soft [H, n_ops], attn_w_1 [H, H], attn_w_2 [H, H], attn_v [H, 1]
struct Offsets {
  int wl, g, we, ws, w1, w2, v, n;
};

__host__ __device__ inline Offsets offsets(int H, int n_ops) {
  Offsets o;
  o.wl = 0;
  o.g = o.wl + 8 * H * H;
  o.we = o.g + H;
  o.ws = o.we + n_ops * H;
  o.w1 = o.ws + H * n_ops;
  o.w2 = o.w1 + H * H;
  o.v = o.w2 + H * H;
  o.n = o.v + H;
  return o;
}

__host__ __device__ inline int arc_len(int L) { return L + L * (L - 1) / 2; }

// per-layer tape record: op probabilities, tanh(z) of the op logits, h W2, all_h[l], all_h[l] W1, skip logits,
// and (backward) d op-logits, d (h W2)
__host__ __device__ inline int layer_rec(int H, int n_ops, int L) { return 3 * n_ops + 4 * H + L; }

// per-block scratch: 2L LSTM calls x [xh 2H | gates 4H | c_prev H | c_new H | d pre-activations 4H],
// L layer records, dAllH / dAllHW [L][H]
constexpr int kCallRec = 12;  // floats per LSTM call, in units of H
__host__ __device__ inline int64_t tape_floats(int H, int n_ops, int L) {
  return (int64_t)2 * kCallRec * H * L + (int64_t)L * layer_rec(H, n_ops, L) + (int64_t)2 * L * H;
}

struct Args {
  float* P;          // [n] parameters (updated in place by training)
  float* M;          // [n] Adam first moment
  float* V;          // [n] Adam second moment
  float* G;          // [n] gradient scratch (training)
  float* tape;       // [blocks][tape_floats]
  int* arcs;         // [blocks][arc_len] sampled arcs (sampling) / [nsteps][arc_len] (training)
  const int* forced;  // optional replayed arcs, row stride forced_stride (0 = one arc for every step/block)
  int forced_stride;
  float* logs;       // [nsteps][kLogFields] (training)
  float* baseline;   // [1] REINFORCE baseline (training, in/out)
  int L, n_ops, H;
  int use_temp, use_tanh, use_ew, use_sw;
  float temperature, tanh_c, entropy_weight, skip_target, skip_weight, baseline_decay;
  float lr, beta1, beta2, eps;
  float baseline_rate, omb1, omb2;  // 1 - baseline_decay, 1 - beta1, 1 - beta2 (rounded once, on the host)
  int adam_t0;       // Adam steps taken before this launch
  int nsteps;        // 0: sample one arc per block; > 0: that many REINFORCE steps in ONE block
  float reward;
  unsigned long long seed, rng_offset;
  long long* phase_clocks;  // optional [5]: wall-clock ticks per phase summed over steps (profiling)
};

size_t lds_bytes(int H, int n_ops, int L);
void launch(const Args& a, int blocks, hipStream_t st);

}  // namespace enas
}  // namespace katib_hip
