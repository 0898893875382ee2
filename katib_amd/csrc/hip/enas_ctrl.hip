// ENAS LSTM controller (reference pkg/suggestion/v1beta1/nas/enas/Controller.py:19-257) on gfx950.
//
// The reference runs the controller as a TF graph on the suggestion pod's CPU: every sampling
// step is a chain of [1 x 2H] x [2H x 4H] products, logits, a categorical draw and a skip
// attention over the previous layers - hundreds of tiny dependent ops per arc, 50 REINFORCE
// steps per GetSuggestions call. Here one workgroup owns the whole controller:
//
//   * w_lstm (2H x 4H fp32, 128 KB at H = 64) is staged once into LDS with a padded row
//     stride (4H + 1) so that both the forward product (thread j reads column j) and the
//     backward transposed product (thread k reads row k) are bank-conflict free.
//   * one thread per gate column; [x, h] is broadcast from LDS. The backward pass records
//     each step's upstream vectors on the tape (pre-activation gradients of every LSTM call,
//     op-logit gradients, attention-query gradients), and every weight gradient is then ONE
//     outer-product sum - e.g. dW_lstm = [2H x 2L] x [2L x 4H] - staged through the (by then
//     free) LDS weight tile and computed on MFMA (v_mfma_f32_16x16x4_f32) instead of 2L
//     rank-1 read-modify-writes of global memory.
//   * op sampling is Gumbel-max over the shaped logits with a counter-based RNG (exact
//     categorical draw, one block-wide argmax); skip decisions are Bernoulli(sigma(2 s)).
//   * training = forward with a tape in global scratch -> advantage (EMA baseline, entropy
//     bonus) -> hand-written BPTT through LSTM / logits / attention / skip averaging ->
//     global norm -> Adam, all inside the launch; `nsteps` REINFORCE steps run back to back,
//     so one GetSuggestions call is ONE kernel launch (plus one for sampling its arcs, one
//     workgroup per arc).
//
// All shapes are checked on the host (enas_bind.cpp).
#include <hip/hip_runtime.h>

#include <cmath>

#include "enas_ctrl.h"

namespace katib_hip {
namespace enas {

namespace {

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide reductions (all kThreads threads must call; red = 4 LDS floats)
__device__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wsum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__device__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wmax(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// index of the largest key (smallest index on ties); red = 8 LDS floats
__device__ int block_argmax(float key, int idx, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float k2 = __shfl_xor(key, o, 64);
    int i2 = __shfl_xor(idx, o, 64);
    if (k2 > key || (k2 == key && i2 < idx)) {
      key = k2;
      idx = i2;
    }
  }
  __syncthreads();
  if (lane == 0) {
    red[wave] = key;
    reinterpret_cast<int*>(red)[4 + wave] = idx;
  }
  __syncthreads();
  float bk = red[0];
  int bi = reinterpret_cast<int*>(red)[4];
  for (int w = 1; w < 4; ++w) {
    float k2 = red[w];
    int i2 = reinterpret_cast<int*>(red)[4 + w];
    if (k2 > bk || (k2 == bk && i2 < bi)) {
      bk = k2;
      bi = i2;
    }
  }
  return bi;
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// uniform in (0, 1), counter based: (seed, stream, counter) -> independent draws
__device__ __forceinline__ float uniform01(unsigned long long seed, unsigned long long stream,
                                           unsigned long long ctr) {
  unsigned long long x = mix64(seed ^ mix64(stream * 0x632BE59BD9B4E019ull + ctr));
  return ((float)(x >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }
// log(sigmoid(x)), stable for both signs
__device__ __forceinline__ float log_sigmoid(float x) { return fminf(x, 0.f) - log1pf(expf(-fabsf(x))); }

struct Ctx {
  const Args* a;
  Offsets o;
  int H, H2, H4, WS, n_ops, L;
  float* sW;    // [2H][4H + 1]
  float* sXH;   // [2H]
  float* sG;    // [4H] gates (forward) / pre-activation gradients (backward)
  float* sH;    // [H]
  float* sC;    // [H]
  float* sInp;  // [H] input of the next LSTM call
  float* sLog;  // [n_ops] shaped logits (forward) / logit gradients (backward)
  float* sQ;    // [L] attention logits (forward) / their gradients (backward)
  float* sHW2;  // [H]
  float* sDH;   // [H]
  float* sDC;   // [H]
  float* sDInp; // [H]
  float* sDHW2; // [H]
  float* sDXH;  // [2H]
  float* sRed;  // [16]
  int* sArc;    // [arc_len]
  float* tape;
  __device__ float* call(int k) const { return tape + (size_t)k * kCallRec * H; }  // xh|gates|c_prev|c_new|dpre
  __device__ float* layer(int l) const { return tape + (size_t)2 * kCallRec * H * L + (size_t)l * layer_rec(H, n_ops, L); }
  // layer record fields
  __device__ float* probs(int l) const { return layer(l); }
  __device__ float* th(int l) const { return layer(l) + n_ops; }
  __device__ float* hw2(int l) const { return layer(l) + 2 * n_ops; }
  __device__ float* ah(int l) const { return layer(l) + 2 * n_ops + H; }
  __device__ float* ahw(int l) const { return layer(l) + 2 * n_ops + 2 * H; }
  __device__ float* s1(int l) const { return layer(l) + 2 * n_ops + 3 * H; }
  __device__ float* dlog(int l) const { return layer(l) + 2 * n_ops + 3 * H + L; }
  __device__ float* dhw2(int l) const { return layer(l) + 3 * n_ops + 3 * H + L; }
  __device__ float* dallh(int i) const { return layer(L) + (size_t)i * H; }
  __device__ float* dallhw(int i) const { return dallh(L) + (size_t)i * H; }
};

// shaping of a raw logit: z = x / T; s = c * tanh(z)
__device__ __forceinline__ float shape(const Args& a, float x, float& thz) {
  float z = a.use_temp ? x / a.temperature : x;
  thz = tanhf(z);
  return a.use_tanh ? a.tanh_c * thz : z;
}

// d raw logit from d shaped logit
__device__ __forceinline__ float unshape(const Args& a, float ds, float thz) {
  float dz = a.use_tanh ? ds * a.tanh_c * (1.f - thz * thz) : ds;
  return a.use_temp ? dz / a.temperature : dz;
}

// LSTM cell forward for call k; sXH = [x, h] already staged. Updates sH, sC; records the call.
__device__ void lstm_fwd(const Ctx& c, int k) {
  const int tid = threadIdx.x, H = c.H;
  float* rec = c.call(k);
  if (tid < c.H4) {
    const float* w = c.sW + tid;
    float acc = 0.f;
    #pragma unroll 8
    for (int q = 0; q < c.H2; ++q) acc += c.sXH[q] * w[q * c.WS];
    const float g = tid < 3 * H ? sigmoidf(acc) : tanhf(acc);  // i, f, o | g
    c.sG[tid] = g;
    rec[c.H2 + tid] = g;
  }
  if (tid < c.H2) rec[tid] = c.sXH[tid];
  __syncthreads();
  if (tid < H) {
    const float cp = c.sC[tid];
    const float cn = c.sG[tid] * c.sG[3 * H + tid] + c.sG[H + tid] * cp;
    c.sC[tid] = cn;
    c.sH[tid] = c.sG[2 * H + tid] * tanhf(cn);
    rec[6 * H + tid] = cp;
    rec[7 * H + tid] = cn;
  }
  __syncthreads();
}

// LSTM cell backward for call k: consumes sDH / sDC (gradients w.r.t. this call's h / c
// outputs), leaves d h_prev in sDH, d c_prev in sDC and d x in sDXH[0, H); records the
// pre-activation gradient for the weight-gradient product.
__device__ void lstm_bwd(const Ctx& c, int k) {
  const int tid = threadIdx.x, H = c.H;
  float* rec = c.call(k);
  if (tid < c.H2) c.sXH[tid] = rec[tid];
  if (tid < H) {
    const float gi = rec[c.H2 + tid], gf = rec[c.H2 + H + tid], go = rec[c.H2 + 2 * H + tid],
                gg = rec[c.H2 + 3 * H + tid];
    const float cp = rec[6 * H + tid], cn = rec[7 * H + tid];
    const float tc = tanhf(cn);
    const float dh = c.sDH[tid];
    const float dcn = c.sDC[tid] + dh * go * (1.f - tc * tc);
    c.sDC[tid] = dcn * gf;
    c.sG[tid] = dcn * gg * gi * (1.f - gi);
    c.sG[H + tid] = dcn * cp * gf * (1.f - gf);
    c.sG[2 * H + tid] = dh * tc * go * (1.f - go);
    c.sG[3 * H + tid] = dcn * gi * (1.f - gg * gg);
  }
  __syncthreads();
  if (tid < c.H4) rec[8 * H + tid] = c.sG[tid];
  if (tid < c.H2) {
    const float* w = c.sW + tid * c.WS;
    float acc = 0.f;
    #pragma unroll 8
    for (int j = 0; j < c.H4; ++j) acc += w[j] * c.sG[j];
    c.sDXH[tid] = acc;
  }
  __syncthreads();
  if (tid < H) c.sDH[tid] = c.sDXH[H + tid];
  __syncthreads();
}

struct FwdSums {
  float logp, ent, kl, skips;
};

// One arc: forward pass with tape. `stream` selects the RNG stream; `forced` replays an arc.
__device__ FwdSums sample_arc(const Ctx& c, unsigned long long stream, const int* forced) {
  const Args& a = *c.a;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, H = c.H;
  const float* P = a.P;
  FwdSums s{0.f, 0.f, 0.f, 0.f};
  if (tid < H) {
    c.sH[tid] = 0.f;
    c.sC[tid] = 0.f;
    c.sInp[tid] = P[c.o.g + tid];
  }
  __syncthreads();
  const unsigned long long per_layer = (unsigned long long)(c.n_ops + c.L);
  for (int l = 0; l < c.L; ++l) {
    const int pos = l + l * (l - 1) / 2;
    // ---- call 2l: LSTM(inputs)
    if (tid < H) {
      c.sXH[tid] = c.sInp[tid];
      c.sXH[H + tid] = c.sH[tid];
    }
    __syncthreads();
    lstm_fwd(c, 2 * l);
    // ---- op logits: h W_soft, shaped, softmax, categorical draw
    float mx = -INFINITY;
    for (int t = tid; t < c.n_ops; t += kThreads) {
      float acc = 0.f;
      #pragma unroll 8
      for (int q = 0; q < H; ++q) acc += c.sH[q] * P[c.o.ws + q * c.n_ops + t];
      float thz;
      const float sl = shape(a, acc, thz);
      c.sLog[t] = sl;
      c.th(l)[t] = thz;
      mx = fmaxf(mx, sl);
    }
    mx = block_max(mx, c.sRed);
    float se = 0.f;
    for (int t = tid; t < c.n_ops; t += kThreads) se += expf(c.sLog[t] - mx);
    const float lse = mx + logf(block_sum(se, c.sRed));
    float bestk = -INFINITY;
    int besti = 0x7fffffff;
    for (int t = tid; t < c.n_ops; t += kThreads) {
      c.probs(l)[t] = expf(c.sLog[t] - lse);
      if (!forced) {
        const float u = uniform01(a.seed, stream, (unsigned long long)l * per_layer + t);
        const float key = c.sLog[t] - logf(-logf(u));  // Gumbel-max
        if (key > bestk) {
          bestk = key;
          besti = t;
        }
      }
    }
    const int op = forced ? forced[pos] : block_argmax(bestk, besti, c.sRed + 8);
    const float lp = c.sLog[op] - lse;
    s.logp += lp;
    s.ent += -lp * expf(lp);
    if (tid == 0) c.sArc[pos] = op;
    // ---- call 2l+1: LSTM(w_emb[op])
    if (tid < H) {
      c.sXH[tid] = P[c.o.we + op * H + tid];
      c.sXH[H + tid] = c.sH[tid];
    }
    __syncthreads();
    lstm_fwd(c, 2 * l + 1);
    if (l > 0) {
      // ---- skip attention over the previous layers: q_i = tanh(h W2 + all_h[i] W1) v
      if (tid < H) {
        float acc = 0.f;
        #pragma unroll 8
        for (int q = 0; q < H; ++q) acc += c.sH[q] * P[c.o.w2 + q * H + tid];
        c.sHW2[tid] = acc;
        c.hw2(l)[tid] = acc;
      }
      __syncthreads();
      for (int i = wave; i < l; i += kThreads / 64) {
        float val = lane < H ? P[c.o.v + lane] * tanhf(c.sHW2[lane] + c.ahw(i)[lane]) : 0.f;
        val = wsum(val);
        if (lane == 0) c.sQ[i] = val;
      }
      __syncthreads();
      float lps = 0.f, ents = 0.f, kls = 0.f, sk = 0.f;
      const float t1 = a.skip_target, t0 = 1.f - a.skip_target;
      for (int i = tid; i < l; i += kThreads) {
        float thz;
        const float s1 = shape(a, c.sQ[i], thz);  // class 1 logit; class 0 = -s1 (odd shaping)
        c.s1(l)[i] = s1;
        int skip;
        if (forced) {
          skip = forced[pos + 1 + i];
        } else {
          const float u = uniform01(a.seed, stream, (unsigned long long)l * per_layer + c.n_ops + i);
          skip = u < sigmoidf(2.f * s1) ? 1 : 0;
        }
        const float lpi = log_sigmoid(skip ? 2.f * s1 : -2.f * s1);
        lps += lpi;
        ents += -lpi * expf(lpi);
        const float sp1 = sigmoidf(s1), sp0 = sigmoidf(-s1);
        kls += sp0 * logf(sp0 / t0) + sp1 * logf(sp1 / t1);
        sk += (float)skip;
        c.sArc[pos + 1 + i] = skip;
      }
      s.logp += block_sum(lps, c.sRed);
      s.ent += block_sum(ents, c.sRed);
      s.kl += block_sum(kls, c.sRed);
      const float S = block_sum(sk, c.sRed);
      s.skips += S;
      // next input: skip-weighted mean of the previous layers' outputs
      if (tid < H) {
        float acc = 0.f;
        for (int i = 0; i < l; ++i)
          if (c.sArc[pos + 1 + i]) acc += c.ah(i)[tid];
        c.sInp[tid] = acc / (1.f + S);
      }
    } else if (tid < H) {
      c.sInp[tid] = P[c.o.g + tid];
    }
    // ---- all_h[l] = h, all_h_w[l] = h W1
    if (tid < H) {
      c.ah(l)[tid] = c.sH[tid];
      float acc = 0.f;
      #pragma unroll 8
      for (int q = 0; q < H; ++q) acc += c.sH[q] * P[c.o.w1 + q * H + tid];
      c.ahw(l)[tid] = acc;
    }
    __syncthreads();
  }
  return s;
}

// out[m][n] = sum_k A_k[m] * B_k[n], A_k = a0 + k * as, B_k = b0 + k * bs (tape vectors): an M x N
// product with inner dimension K, staged through the LDS weight tile (dead between the end of
// the backward pass and the next stage_w) in chunks of K, on MFMA 16x16x4 with zero padding.
__device__ void outer_sum(const Ctx& c, float* out, const float* a0, int as, const float* b0, int bs, int M, int N,
                          int K) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cap = c.H2 * c.WS;
  const int kc_max = max(4, (cap / (M + N)) & ~3);
  const int mb = (M + 15) / 16, nb = (N + 15) / 16;
  if (K <= 0) {
    for (int i = tid; i < M * N; i += kThreads) out[i] = 0.f;
    return;
  }
  for (int kb = 0; kb < K; kb += kc_max) {
    const int kc = min(kc_max, K - kb), kp = (kc + 3) & ~3;
    float* sA = c.sW;           // [kp][M]
    float* sB = c.sW + kp * M;  // [kp][N]
    __syncthreads();
#pragma unroll 4
    for (int i = tid; i < kp * M; i += kThreads) {
      const int k = i / M, m = i - k * M;
      sA[i] = k < kc ? a0[(size_t)(kb + k) * as + m] : 0.f;
    }
#pragma unroll 4
    for (int i = tid; i < kp * N; i += kThreads) {
      const int k = i / N, n = i - k * N;
      sB[i] = k < kc ? b0[(size_t)(kb + k) * bs + n] : 0.f;
    }
    __syncthreads();
    for (int t = wave; t < mb * nb; t += kThreads / 64) {
      const int m0 = (t / nb) * 16, n0 = (t % nb) * 16;
      const int mm = m0 + (lane & 15), nn = n0 + (lane & 15);
      f4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < kp; k0 += 4) {
        const int k = k0 + (lane >> 4);
        const float av = mm < M ? sA[k * M + mm] : 0.f;
        const float bv = nn < N ? sB[k * N + nn] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + (lane >> 4) * 4 + r;
        if (row < M && nn < N) {
          float* o = out + (size_t)row * N + nn;
          *o = kb == 0 ? acc[r] : *o + acc[r];
        }
      }
    }
  }
  __syncthreads();
}

// all deferred weight gradients of one backward pass
__device__ void weight_grads(const Ctx& c) {
  const int H = c.H, L = c.L, lr = layer_rec(H, c.n_ops, L), cs = kCallRec * H;
  float* G = c.a->G;
  outer_sum(c, G + c.o.wl, c.call(0), cs, c.call(0) + 8 * H, cs, c.H2, c.H4, 2 * L);          // [x,h] (x) dpre
  outer_sum(c, G + c.o.ws, c.call(1) + H, 2 * cs, c.dlog(0), lr, H, c.n_ops, L);              // h_{2l} (x) dlogits
  outer_sum(c, G + c.o.w1, c.ah(0), lr, c.dallhw(0), H, H, H, L);                             // all_h (x) d keys
  outer_sum(c, G + c.o.w2, c.ah(L > 1 ? 1 : 0), lr, c.dhw2(L > 1 ? 1 : 0), lr, H, H, L - 1);  // h (x) d query
}

// REINFORCE backward through the taped arc. A = advantage, ckl = d loss / d (sum of a
// layer's KL terms). g_emb / w_emb / attn_v gradients accumulate into G (zeroed by the
// caller); the matrix gradients are recorded on the tape for weight_grads.
__device__ void backward(const Ctx& c, float A, float ckl) {
  const Args& a = *c.a;
  const int tid = threadIdx.x, H = c.H;
  const float* P = a.P;
  float* G = a.G;
  if (tid < H) {
    c.sDH[tid] = 0.f;
    c.sDC[tid] = 0.f;
    c.sDInp[tid] = 0.f;
  }
  __syncthreads();
  const float t1 = a.skip_target, t0 = 1.f - a.skip_target;
  for (int l = c.L - 1; l >= 0; --l) {
    const int pos = l + l * (l - 1) / 2;
    const int op = c.sArc[pos];
    const float* hl = c.ah(l);  // h_{2l+1}
    // ---- inputs of layer l+1 (sDInp = their gradient)
    if (l >= 1) {
      float S = 0.f;
      for (int i = 0; i < l; ++i) S += (float)c.sArc[pos + 1 + i];
      const float inv = 1.f / (1.f + S);
      for (int idx = tid; idx < l * H; idx += kThreads) {
        const int i = idx / H, m = idx - i * H;
        if (c.sArc[pos + 1 + i]) c.dallh(i)[m] += c.sDInp[m] * inv;
      }
    } else if (tid < H) {
      G[c.o.g + tid] += c.sDInp[tid];
    }
    // ---- skip attention (layer l >= 1)
    if (l >= 1) {
      for (int i = tid; i < l; i += kThreads) {
        const float s1 = c.s1(l)[i];
        const int skip = c.sArc[pos + 1 + i];
        const float p1 = sigmoidf(2.f * s1), p0 = 1.f - p1;
        const float sp1 = sigmoidf(s1), sp0 = sigmoidf(-s1);
        const float ds1 = A * (p1 - (skip ? 1.f : 0.f)) + ckl * sp1 * (1.f - sp1) * (logf(sp1 / t1) + 1.f);
        const float ds0 = A * (p0 - (skip ? 0.f : 1.f)) + ckl * sp0 * (1.f - sp0) * (logf(sp0 / t0) + 1.f);
        // both classes are shaped from +-q: tanh(z0) = -tanh(z1)
        const float thz1 = a.use_tanh ? s1 / a.tanh_c : 0.f;  // only read when shaping uses tanh
        c.sQ[i] = unshape(a, ds1, thz1) - unshape(a, ds0, -thz1);
      }
      __syncthreads();
      if (tid < H) {
        const float vm = P[c.o.v + tid], hw2 = c.hw2(l)[tid];
        float dv = 0.f, dhw2 = 0.f;
        for (int i = 0; i < l; ++i) {
          const float t = tanhf(hw2 + c.ahw(i)[tid]);
          const float dq = c.sQ[i];
          dv += dq * t;
          const float dpre = dq * vm * (1.f - t * t);
          dhw2 += dpre;
          c.dallhw(i)[tid] += dpre;
        }
        G[c.o.v + tid] += dv;
        c.sDHW2[tid] = dhw2;
      }
      __syncthreads();
      if (tid < H) {
        float acc = 0.f;
        #pragma unroll 8
        for (int m = 0; m < H; ++m) acc += P[c.o.w2 + tid * H + m] * c.sDHW2[m];
        c.sDH[tid] += acc;
        c.dhw2(l)[tid] = c.sDHW2[tid];  // dW2 += h (x) this, in weight_grads
      }
    }
    __syncthreads();
    // ---- h_{2l+1} feeds the attention keys (W1) of later layers and their skip inputs
    if (tid < H) {
      const float* dk = c.dallhw(l);
      float acc = 0.f;
      #pragma unroll 8
      for (int m = 0; m < H; ++m) acc += P[c.o.w1 + tid * H + m] * dk[m];
      c.sDH[tid] += acc + c.dallh(l)[tid];
    }
    __syncthreads();
    // ---- call 2l+1: input w_emb[op]
    lstm_bwd(c, 2 * l + 1);
    if (tid < H) G[c.o.we + op * H + tid] += c.sDXH[tid];
    // ---- op logits from h_{2l} (= the recurrent input recorded by call 2l+1)
    for (int t = tid; t < c.n_ops; t += kThreads) {
      const float ds = A * (c.probs(l)[t] - (t == op ? 1.f : 0.f));
      const float dl = unshape(a, ds, c.th(l)[t]);
      c.sLog[t] = dl;
      c.dlog(l)[t] = dl;  // dW_soft += h_{2l} (x) this, in weight_grads
    }
    __syncthreads();
    if (tid < H) {
      float acc = 0.f;
      #pragma unroll 8
      for (int t = 0; t < c.n_ops; ++t) acc += P[c.o.ws + tid * c.n_ops + t] * c.sLog[t];
      c.sDH[tid] += acc;
    }
    __syncthreads();
    // ---- call 2l: input inp_l
    lstm_bwd(c, 2 * l);
    if (tid < H) {
      c.sDInp[tid] = c.sDXH[tid];
      if (l == 0) G[c.o.g + tid] += c.sDXH[tid];  // inp_0 = g_emb
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kThreads, 1) enas_ctrl_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Ctx c;
  c.a = &a;
  c.H = a.H;
  c.H2 = 2 * a.H;
  c.H4 = 4 * a.H;
  c.WS = c.H4 + 1;
  c.n_ops = a.n_ops;
  c.L = a.L;
  c.o = offsets(a.H, a.n_ops);
  float* p = smem;
  c.sW = p;    p += c.H2 * c.WS;
  c.sXH = p;   p += c.H2;
  c.sG = p;    p += c.H4;
  c.sH = p;    p += c.H;
  c.sC = p;    p += c.H;
  c.sInp = p;  p += c.H;
  c.sLog = p;  p += c.n_ops;
  c.sQ = p;    p += c.L;
  c.sHW2 = p;  p += c.H;
  c.sDH = p;   p += c.H;
  c.sDC = p;   p += c.H;
  c.sDInp = p; p += c.H;
  c.sDHW2 = p; p += c.H;
  c.sDXH = p;  p += c.H2;
  c.sRed = p;  p += 16;
  c.sArc = reinterpret_cast<int*>(p);
  const int alen = arc_len(a.L);
  c.tape = a.tape + (size_t)blockIdx.x * tape_floats(a.H, a.n_ops, a.L);
  const int tid = threadIdx.x;

  auto stage_w = [&]() {
    for (int i = tid; i < c.H2 * c.H4; i += kThreads) c.sW[(i / c.H4) * c.WS + i % c.H4] = a.P[c.o.wl + i];
    __syncthreads();
  };
  stage_w();

  if (a.nsteps == 0) {  // sampling: one arc per workgroup
    const int* forced = a.forced ? a.forced + (size_t)blockIdx.x * a.forced_stride : nullptr;
    sample_arc(c, a.rng_offset + blockIdx.x, forced);
    for (int i = tid; i < alen; i += kThreads) a.arcs[(size_t)blockIdx.x * alen + i] = c.sArc[i];
    return;
  }

  // training: nsteps REINFORCE steps in this (single) workgroup
  float baseline = a.baseline[0];
  const float norm = a.L > 1 ? 0.5f * a.L * (a.L - 1) : 0.f;
  const float ckl = (a.use_sw && a.L > 1) ? a.skip_weight / (float)(a.L - 1) : 0.f;
  for (int s = 0; s < a.nsteps; ++s) {
    const int* forced = a.forced ? a.forced + (size_t)s * a.forced_stride : nullptr;
    long long tk = wall_clock64();
    auto tick = [&](int ph) {  // phase timing (thread 0, only when requested)
      if (a.phase_clocks && tid == 0) {
        const long long now = wall_clock64();
        a.phase_clocks[ph] += now - tk;
        tk = now;
      }
    };
    FwdSums fs = sample_arc(c, a.rng_offset + s, forced);
    tick(0);
    // advantage with the EMA baseline (updated first, as the reference's control dependency)
    float r = a.reward + (a.use_ew ? a.entropy_weight * fs.ent : 0.f);
    baseline -= a.baseline_rate * (baseline - r);
    const float A = r - baseline;
    const float kl_mean = a.L > 1 ? fs.kl / (float)(a.L - 1) : 0.f;
    const float loss = -fs.logp * A + (a.use_sw ? a.skip_weight * kl_mean : 0.f);
    // zero the gradients that accumulate during the pass (the matrix ones are written whole)
    if (tid < c.H) {
      a.G[c.o.g + tid] = 0.f;
      a.G[c.o.v + tid] = 0.f;
    }
    for (int i = tid; i < c.n_ops * c.H; i += kThreads) a.G[c.o.we + i] = 0.f;
    for (int i = tid; i < 2 * c.L * c.H; i += kThreads) c.dallh(0)[i] = 0.f;
    __syncthreads();
    backward(c, A, ckl);
    tick(1);
    weight_grads(c);
    tick(2);
    // Adam (torch.optim.Adam arithmetic: lerp first moment, bias-corrected denominator),
    // with the gradient's global norm (logged) accumulated in the same pass
    const int t = a.adam_t0 + s + 1;
    const float bc1 = (float)(1.0 - pow((double)a.beta1, (double)t));
    const float bc2s = (float)sqrt(1.0 - pow((double)a.beta2, (double)t));
    const float step = a.lr / bc1;
    float ss = 0.f;
    {
      const float* __restrict__ G = a.G;
      float* __restrict__ M = a.M;
      float* __restrict__ V = a.V;
      float* __restrict__ P = a.P;
      auto upd = [&](float g, float& m, float& v, float& p) {
        ss += g * g;
        m = m + a.omb1 * (g - m);
        v = v * a.beta2 + a.omb2 * g * g;
        p = p - step * m / (sqrtf(v) / bc2s + a.eps);
      };
      typedef float f4 __attribute__((ext_vector_type(4)));
      const int n4 = (c.o.n % 4 == 0) ? c.o.n / 4 : 0;  // 16-byte path (torch buffers are 16-B aligned)
#pragma unroll 4
      for (int i = tid; i < n4; i += kThreads) {
        const f4 g = reinterpret_cast<const f4*>(G)[i];
        f4 m = reinterpret_cast<f4*>(M)[i], v = reinterpret_cast<f4*>(V)[i], p = reinterpret_cast<f4*>(P)[i];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float mu = m[u], vu = v[u], pu = p[u];
          upd(g[u], mu, vu, pu);
          m[u] = mu;
          v[u] = vu;
          p[u] = pu;
        }
        reinterpret_cast<f4*>(M)[i] = m;
        reinterpret_cast<f4*>(V)[i] = v;
        reinterpret_cast<f4*>(P)[i] = p;
      }
      for (int i = 4 * n4 + tid; i < c.o.n; i += kThreads) upd(G[i], M[i], V[i], P[i]);
    }
    const float gnorm = sqrtf(block_sum(ss, c.sRed));
    tick(3);
    for (int i = tid; i < alen; i += kThreads) a.arcs[(size_t)s * alen + i] = c.sArc[i];
    if (tid == 0) {
      float* lg = a.logs + (size_t)s * kLogFields;
      lg[0] = loss;
      lg[1] = fs.ent;
      lg[2] = gnorm;
      lg[3] = baseline;
      lg[4] = norm > 0.f ? fs.skips / norm : 0.f;
      lg[5] = -fs.logp;
      lg[6] = kl_mean;
      lg[7] = A;
    }
    __syncthreads();
    stage_w();  // the next step samples with the updated weights
    tick(4);
  }
  if (tid == 0) a.baseline[0] = baseline;
}

}  // namespace

size_t lds_bytes(int H, int n_ops, int L) {
  const int H2 = 2 * H, H4 = 4 * H;
  size_t floats = (size_t)H2 * (H4 + 1) + H2 + H4 + 3 * H + n_ops + L + 5 * H + H2 + 16;
  return floats * sizeof(float) + (size_t)arc_len(L) * sizeof(int);
}

void launch(const Args& a, int blocks, hipStream_t st) {
  const size_t lds = lds_bytes(a.H, a.n_ops, a.L);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&enas_ctrl_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)lds);
  hipLaunchKernelGGL(enas_ctrl_kernel, dim3(blocks), dim3(kThreads), lds, st, a);
}

}  // namespace enas
}  // namespace katib_hip
