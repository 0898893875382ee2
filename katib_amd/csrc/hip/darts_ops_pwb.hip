// DARTS pointwise backward kernels (pw_bwd tiles, pw_bwd_px narrow layers, pw_bwd_wave wide layers)
// and their launch heuristics. See darts_ops.hip for the design notes.
#include "darts_ops_dev.h"

namespace katib_hip {


// ------------------------------------------------------------------------------------------------
// pw_bwd: dz (on the fly) -> dd = pw^T dz ; dW_pw += dz (x) a_in.
// mode 0 (dw-pw stage): a_in = stored depthwise output d; writes dd [N,Cin,Ho,Wo].
// mode 1 (StdConv / FR half): a_in = relu(x) at strided positions; gx += dd * (x > 0).
// grid: persistent over 64-pixel tiles; weight grads accumulated in registers across tiles.
// ------------------------------------------------------------------------------------------------
template <bool MFMA, int MBLK = 4>
__global__ void __launch_bounds__(256) pw_bwd_kernel(PwBwdBatch bt) {
  const PwBwdArgs& a = bt.e[blockIdx.y];
  constexpr int P = 64, PS = P + 1;  // padded LDS rows: per-channel row reads hit distinct banks
  const int Cin = a.Cin, Cout = a.Cout, Ho = a.Ho, Wo = a.Wo, HWo = Ho * Wo;
  const int ntiles = a.N * HWo / P;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sDz = smem;             // [Cout][PS]
  float* sA = sDz + Cout * PS;   // [Cin][PS]
  float* sMean = sA + Cin * PS;  // [Cout]
  float* sInv = sMean + Cout;
  float* sM1 = sInv + Cout;      // [Cout]
  float* sM2 = sM1 + Cout;
  float* sW = sM2 + Cout;        // [1]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const float wv = (tid == 0 && a.gs.w) ? a.gs.w[a.gs.widx] : 1.f;  // issued with the coefficient loads
  bn_gs_coop(a.gs, a.co_off, Cout, sMean, sInv, sM1, sM2);
  if (tid == 0) sW[0] = wv;
  __syncthreads();
  const float wk = sW[0];
  typedef float f4 __attribute__((ext_vector_type(4)));
  // weight-grad accumulators live in registers across tiles.
  // scalar path: pairs (co, ci) = tid + 256*j; MFMA path: 16x16 blocks b = wave + 4*j
  // Cout*Cin <= 8192 (the 128 -> 64 preprocess of darts-gpu.yaml's last cell); MFMA: MBLK 16x16
  // blocks per wave (4 waves x MBLK x 256), 8 only where needed (more accumulators, fewer waves)
  constexpr int MAXJ = 32;
  float gacc[MFMA ? 1 : MAXJ];
  f4 macc[MFMA ? MBLK : 1];
#pragma unroll
  for (int j = 0; j < (MFMA ? 1 : MAXJ); ++j) gacc[j] = 0.f;
#pragma unroll
  for (int j = 0; j < (MFMA ? MBLK : 1); ++j) macc[j] = f4{0, 0, 0, 0};
  const int npairs = Cout * Cin;
  const int nbi = Cin / 16, nblk = (Cout / 16) * nbi;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int pix0 = t * P, n = pix0 / HWo, prem = pix0 % HWo;
    #pragma unroll 4  // keep several global loads of the staging pass in flight
    for (int i = tid; i < Cout * P; i += 256) {
      int co = i / P, p = i % P;
      size_t gi = ((size_t)n * a.CoutTotal + a.co_off + co) * HWo + prem + p;
      sDz[co * PS + p] = bn_bwd_val(a.gs, gi, sMean[co], sInv[co], wk, sM1[co], sM2[co]);
    }
    #pragma unroll 4  // keep several global loads of the staging pass in flight
    for (int i = tid; i < Cin * P; i += 256) {
      int ci = i / P, p = i % P;
      int pp = prem + p;
      float v;
      if (a.mode == 0) {
        v = z2f(a.ain[((size_t)n * Cin + ci) * HWo + pp]);
      } else {
        int oy = pp / Wo, ox = pp % Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
        v = (iy < a.H && ix < a.W)
                ? fmaxf(a.x[plane_off(n, ci, a.N, Cin, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix], 0.f)
                : 0.f;
      }
      sA[ci * PS + p] = v;
    }
    __syncthreads();
    if (a.gW) {
      if (MFMA) {
        // gW[co][ci] += sum_p dz[co][p] * a[ci][p]  (M = co, N = ci, K = pixels)
#pragma unroll
        for (int j = 0; j < MBLK; ++j) {
          int b = wave + 4 * j;
          if (b < nblk) {
            int cob = (b / nbi) * 16, cib = (b % nbi) * 16;
            for (int p0 = 0; p0 < P; p0 += 4) {
              float av = sDz[(cob + (lane & 15)) * PS + p0 + (lane >> 4)];
              float bv = sA[(cib + (lane & 15)) * PS + p0 + (lane >> 4)];
              macc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, macc[j], 0, 0, 0);
            }
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < MAXJ; ++j) {
          int pr = tid + 256 * j;
          if (pr < npairs) {
            int co = pr / Cin, ci = pr % Cin;
            float s = 0.f;
            for (int p = 0; p < P; ++p) s += sDz[co * PS + p] * sA[ci * PS + p];
            gacc[j] += s;
          }
        }
      }
    }
    // dd[ci][p] = sum_co pw[co][ci] dz[co][p]
    if (a.need_dx) {
      if (MFMA) {
        for (int cib = wave * 16; cib < Cin; cib += 64) {
          f4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
          for (int k0 = 0; k0 < Cout; k0 += 4) {
            float av = a.pw[(k0 + (lane >> 4)) * Cin + cib + (lane & 15)];
#pragma unroll
            for (int pb = 0; pb < 4; ++pb) {
              float bv = sDz[(k0 + (lane >> 4)) * PS + pb * 16 + (lane & 15)];
              acc[pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[pb], 0, 0, 0);
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            int ci = cib + (lane >> 4) * 4 + r;
#pragma unroll
            for (int pb = 0; pb < 4; ++pb) {
              int pp = prem + pb * 16 + (lane & 15);
              float v = acc[pb][r];
              if (a.mode == 0) {
                a.dd[((size_t)n * Cin + ci) * HWo + pp] = v;
              } else {
                int oy = pp / Wo, ox = pp % Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
                if (iy < a.H && ix < a.W) {
                  size_t xi = plane_off(n, ci, a.N, Cin, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix;
                  if (a.overwrite) a.gx[xi] = a.x[xi] > 0.f ? v : 0.f;
                  else if (a.x[xi] > 0.f) a.gx[xi] += v;
                }
              }
            }
          }
        }
      } else {
        for (int ci = wave; ci < Cin; ci += 4) {
          const int ciu = __builtin_amdgcn_readfirstlane(ci);
          float v = 0.f;
          for (int co = 0; co < Cout; ++co) v += a.pw[co * Cin + ciu] * sDz[co * PS + lane];
          int pp = prem + lane;
          if (a.mode == 0) {
            a.dd[((size_t)n * Cin + ciu) * HWo + pp] = v;
          } else {
            int oy = pp / Wo, ox = pp % Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
            if (iy < a.H && ix < a.W) {
              size_t xi = plane_off(n, ciu, a.N, Cin, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix;
              if (a.overwrite) a.gx[xi] = a.x[xi] > 0.f ? v : 0.f;
              else if (a.x[xi] > 0.f) a.gx[xi] += v;
            }
          }
        }
      }
    }
    __syncthreads();
  }
  if (a.gW) {
    float* gW = a.gW + (size_t)rep_slot() * a.gstride;
    if (MFMA) {
#pragma unroll
      for (int j = 0; j < MBLK; ++j) {
        int b = wave + 4 * j;
        if (b < nblk) {
          int cob = (b / nbi) * 16, cib = (b % nbi) * 16;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            atomicAdd(gW + (cob + (lane >> 4) * 4 + r) * Cin + cib + (lane & 15), macc[j][r]);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        int pr = tid + 256 * j;
        if (pr < npairs) atomicAdd(gW + pr, gacc[j]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// pw_bwd_px: pw_bwd for narrow layers (Cin * Cout <= 96, the C = 4..12 channels of small
// supernets). The tiled kernel above spends most of its time in the weight-gradient sum, where
// Cin * Cout threads (16 of 256 at C = 4) each walk the tile's 64 pixels through LDS. Here
// every thread owns whole pixels with ALL channels in registers: dz (BN backward on the fly),
// the layer input, dd = pw^T dz, and a private Cin x Cout weight-gradient accumulator; loads
// and stores are coalesced across the wave (consecutive pixels), there is no LDS staging and
// no barrier until the block's single reduction of its accumulators (wave shuffles, then one
// LDS add per wave and one global atomic vector per block into the block's replica).
// ------------------------------------------------------------------------------------------------
template <int CI, int CO, bool V4>
__global__ void __launch_bounds__(256) pw_bwd_px_kernel(PwBwdBatch bt) {
  const PwBwdArgs& a = bt.e[blockIdx.y];
  const int HWo = a.Ho * a.Wo, Wo = a.Wo;
  const int total = a.N * HWo;
  __shared__ float sC[4 * CO + 1];
  __shared__ float sGW[CI * CO];
  const int tid = threadIdx.x, lane = tid & 63;
  const float wv = (tid == 0 && a.gs.w) ? a.gs.w[a.gs.widx] : 1.f;  // issued with the coefficient loads
  bn_gs_coop(a.gs, a.co_off, CO, sC, sC + CO, sC + 2 * CO, sC + 3 * CO);  // BN-backward sums may arrive unfolded
  if (tid == 0) sC[4 * CO] = wv;
  for (int i = tid; i < CI * CO; i += 256) sGW[i] = 0.f;
  __syncthreads();
  float mean[CO], inv[CO], m1[CO], m2[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) {
    mean[c] = sC[c];
    inv[c] = sC[CO + c];
    m1[c] = sC[2 * CO + c];
    m2[c] = sC[3 * CO + c];
  }
  const float wk = sC[4 * CO];
  float wpw[CI * CO];  // pointwise weights in registers (the loop's stores could alias them)
#pragma unroll
  for (int i = 0; i < CI * CO; ++i) wpw[i] = a.pw[i];
  float gacc[CI * CO];
#pragma unroll
  for (int i = 0; i < CI * CO; ++i) gacc[i] = 0.f;
  const bool want_w = a.gW != nullptr;
  if (V4) {
    // 4 consecutive pixels per thread with 16-byte loads/stores (HWo % 4 == 0; mode 0, or
    // mode 1 at stride 1 / offset 0 where the input plane is the output plane)
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int t = blockIdx.x * 256 + tid; t < total / 4; t += gridDim.x * 256) {
      const int p = t * 4, n = p / HWo, pp = p - n * HWo;
      f4 dz[CO], av[CI];
#pragma unroll
      for (int c = 0; c < CO; ++c) {
        const size_t gi = ((size_t)n * a.CoutTotal + a.co_off + c) * HWo + pp;
        const f4 zz = zld4(a.gs.z + gi), gg = *reinterpret_cast<const f4*>(a.gs.g + gi);
        dz[c] = wk * inv[c] * (gg - m1[c] - ((zz - mean[c]) * inv[c]) * m2[c]);
      }
#pragma unroll
      for (int c = 0; c < CI; ++c) {
        const size_t o = a.mode == 0 ? ((size_t)n * CI + c) * HWo + pp : plane_off(n, c, a.N, CI, a.xnodes, HWo) + pp;
        av[c] = a.mode == 0 ? zld4(a.ain + o) : *reinterpret_cast<const f4*>(a.x + o);
        if (a.mode != 0) {
          av[c].x = fmaxf(av[c].x, 0.f);
          av[c].y = fmaxf(av[c].y, 0.f);
          av[c].z = fmaxf(av[c].z, 0.f);
          av[c].w = fmaxf(av[c].w, 0.f);
        }
      }
      if (want_w) {
#pragma unroll
        for (int co = 0; co < CO; ++co)
#pragma unroll
          for (int ci = 0; ci < CI; ++ci) {
            const f4 t2 = dz[co] * av[ci];
            gacc[co * CI + ci] += (t2.x + t2.y) + (t2.z + t2.w);
          }
      }
      if (a.need_dx) {
#pragma unroll
        for (int ci = 0; ci < CI; ++ci) {
          f4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int co = 0; co < CO; ++co) v += wpw[co * CI + ci] * dz[co];
          const size_t o = a.mode == 0 ? ((size_t)n * CI + ci) * HWo + pp : plane_off(n, ci, a.N, CI, a.xnodes, HWo) + pp;
          if (a.mode == 0) {
            *reinterpret_cast<f4*>(a.dd + o) = v;
          } else {
            f4 m;
            m.x = av[ci].x > 0.f ? v.x : 0.f;
            m.y = av[ci].y > 0.f ? v.y : 0.f;
            m.z = av[ci].z > 0.f ? v.z : 0.f;
            m.w = av[ci].w > 0.f ? v.w : 0.f;
            f4* g = reinterpret_cast<f4*>(a.gx + o);
            *g = a.overwrite ? m : *g + m;
          }
        }
      }
    }
  }
  for (int p = blockIdx.x * 256 + tid; p < (V4 ? 0 : total); p += gridDim.x * 256) {
    const int n = p / HWo, pp = p - n * HWo;
    float dz[CO], av[CI];
#pragma unroll
    for (int c = 0; c < CO; ++c)
      dz[c] = bn_bwd_val(a.gs, ((size_t)n * a.CoutTotal + a.co_off + c) * HWo + pp, mean[c], inv[c], wk, m1[c], m2[c]);
    size_t xi0 = 0;
    bool inb = true;
    if (a.mode == 0) {
#pragma unroll
      for (int c = 0; c < CI; ++c) av[c] = z2f(a.ain[((size_t)n * CI + c) * HWo + pp]);
    } else {
      const int oy = pp / Wo, ox = pp - oy * Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
      inb = iy < a.H && ix < a.W;
      xi0 = inb ? (size_t)iy * a.W + ix : 0;  // pixel inside the channel plane (plane_off below)
      // every channel loaded unconditionally (out-of-band pixels read pixel 0 and are masked):
      // a load under `inb ?` made hipcc branch around each load and wait vmcnt(0) per channel,
      // CI serial round trips per pixel
      float raw[CI];
#pragma unroll
      for (int c = 0; c < CI; ++c) raw[c] = a.x[plane_off(n, c, a.N, CI, a.xnodes, (size_t)a.H * a.W) + xi0];
#pragma unroll
      for (int c = 0; c < CI; ++c) av[c] = inb ? fmaxf(raw[c], 0.f) : 0.f;
    }
    if (want_w) {
#pragma unroll
      for (int co = 0; co < CO; ++co)
#pragma unroll
        for (int ci = 0; ci < CI; ++ci) gacc[co * CI + ci] += dz[co] * av[ci];
    }
    if (a.need_dx) {
#pragma unroll
      for (int ci = 0; ci < CI; ++ci) {
        float v = 0.f;
#pragma unroll
        for (int co = 0; co < CO; ++co) v += wpw[co * CI + ci] * dz[co];
        if (a.mode == 0) {
          a.dd[((size_t)n * CI + ci) * HWo + pp] = v;
        } else if (a.overwrite) {  // stride 1: every input pixel is some thread's own
          a.gx[plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W) + xi0] = av[ci] > 0.f ? v : 0.f;
        } else if (inb && av[ci] > 0.f) {  // relu'(x): x > 0  <=>  relu(x) > 0
          a.gx[plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W) + xi0] += v;
        }
      }
    }
  }
  if (!want_w) return;
  wave_sums_to_lds<CI * CO>(gacc, sGW, lane);
  __syncthreads();
  float* gW = a.gW + (size_t)rep_slot() * a.gstride;
  for (int i = tid; i < CI * CO; i += 256) atomicAdd(gW + i, sGW[i]);
}


// ------------------------------------------------------------------------------------------------
// pw_bwd_wave: pw_bwd for the 16..64-channel layers of darts-gpu.yaml-sized supernets (Cin, Cout
// multiples of 16). The tiled kernel above stages a 64-pixel tile per workgroup between two
// barriers and runs its MFMA chains on one wave when Cin = Cout = 16, so each workgroup walks a
// serial load -> barrier -> compute chain per tile. Here every WAVE owns whole 64-pixel chunks
// and never waits for the others until the final weight-gradient reduction:
//   loads   lane (c = lane & 15, q = lane >> 4) reads 16 consecutive pixels q*16 .. q*16+15 of
//           channel c of every 16-channel block with 16-byte loads: dz (BN backward on the fly)
//           and the layer input, straight into MFMA operand registers;
//   dW      v_mfma_f32_16x16x4f32 with K = pixels: step j feeds pixel q*16 + j of lane group q
//           as k-index q, so the 16 steps cover the chunk with no data movement;
//   dd      pw^T dz needs dz with channels on the K axis: the wave writes its dz chunk to a
//           wave-private LDS tile (no workgroup barrier) and reads it back in B-operand order.
// ------------------------------------------------------------------------------------------------
// NS > 1 (small planes): work item = (chunk, group of CI / NS input channels): the wave forms dz for
// every output channel but the weight gradients and dd of its input-channel group only. (A group
// fixed per workgroup - a quarter of the weight-gradient flush atomics at NS = 4 - measured a wash on
// the darts-gpu.yaml step: the waves sharing a chunk's z / g loads in one CU's caches are worth as
// much as the atomics saved, profiles/darts_default_ab_r04.log.)
template <int CI, int CO, int NS = 1>
__global__ void __launch_bounds__(256) pw_bwd_wave_kernel(PwBwdBatch bt) {
  static_assert(CI % 16 == 0 && CO % 16 == 0 && CI <= 128 && CO <= 64 && (CI / 16) % NS == 0, "16-channel blocks");
  constexpr int BO = CO / 16, BI = CI / 16 / NS, RS = 64 + 4;  // LDS tile row stride (floats)
  typedef float f4 __attribute__((ext_vector_type(4)));
  const PwBwdArgs& a = bt.e[blockIdx.y];
  const int HWo = a.Ho * a.Wo, Wo = a.Wo;
  const int nchunks = a.N * HWo / 64;  // HWo % 64 == 0 (host-checked)
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [4 waves][CO][RS]
  __shared__ float sC[4 * CO + 1];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int c16 = lane & 15, q = lane >> 4;
  const float wv = (tid == 0 && a.gs.w) ? a.gs.w[a.gs.widx] : 1.f;  // issued with the coefficient loads
  bn_gs_coop(a.gs, a.co_off, CO, sC, sC + CO, sC + 2 * CO, sC + 3 * CO);
  if (tid == 0) sC[4 * CO] = wv;
  __syncthreads();
  const float wk = sC[4 * CO];
  float mean[BO], inv[BO], m1[BO], m2[BO];
#pragma unroll
  for (int bo = 0; bo < BO; ++bo) {
    const int c = bo * 16 + c16;
    mean[bo] = sC[c];
    inv[bo] = sC[CO + c];
    m1[bo] = sC[2 * CO + c];
    m2[bo] = sC[3 * CO + c];
  }
  const bool want_w = a.gW != nullptr;
  // contiguous input rows: the dw-pw stage, or a stride-1 StdConv whose input plane is the output plane
  const bool flat = a.mode == 0 || (a.S == 1 && a.off == 0 && a.H == a.Ho && a.W == a.Wo);
  const bool fr2 = a.mode != 0 && a.S == 2 && a.H == 2 * a.Ho && a.W == 2 * a.Wo && a.W % 4 == 0 && a.off <= 1 &&
                   ((uintptr_t)a.x & 15) == 0;
  float* sT = smem + wave * CO * RS;
  const int ci0 = ((blockIdx.x * 4 + wave) % NS) * BI * 16;  // the wave's input-channel group (fixed: stride % NS == 0)
  f4 macc[BO][BI];
#pragma unroll
  for (int bo = 0; bo < BO; ++bo)
#pragma unroll
    for (int bi = 0; bi < BI; ++bi) macc[bo][bi] = f4{0.f, 0.f, 0.f, 0.f};
  for (int w = blockIdx.x * 4 + wave; w < nchunks * NS; w += gridDim.x * 4) {
    const int pix0 = (w / NS) * 64, n = pix0 / HWo, prem = pix0 - n * HWo;
    const int pq = prem + q * 16;  // this lane's pixels pq .. pq + 15
    float dz[BO][16];
#pragma unroll
    for (int bo = 0; bo < BO; ++bo) {
      const size_t gi = ((size_t)n * a.CoutTotal + a.co_off + bo * 16 + c16) * HWo + pq;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f4 zz = zld4(a.gs.z + gi + 4 * t);
        const f4 gg = *reinterpret_cast<const f4*>(a.gs.g + gi + 4 * t);
        const f4 v = wk * inv[bo] * (gg - m1[bo] - ((zz - mean[bo]) * inv[bo]) * m2[bo]);
        dz[bo][4 * t] = v.x;
        dz[bo][4 * t + 1] = v.y;
        dz[bo][4 * t + 2] = v.z;
        dz[bo][4 * t + 3] = v.w;
      }
    }
    if (want_w) {
      float av[BI][16];
#pragma unroll
      for (int bi = 0; bi < BI; ++bi) {
        const int ci = ci0 + bi * 16 + c16;
        if (flat) {
          const size_t so = a.mode == 0 ? ((size_t)n * CI + ci) * HWo + pq : plane_off(n, ci, a.N, CI, a.xnodes, HWo) + pq;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            f4 v = a.mode == 0 ? zld4(a.ain + so + 4 * t) : *reinterpret_cast<const f4*>(a.x + so + 4 * t);
            if (a.mode != 0) v = f4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
            av[bi][4 * t] = v.x;
            av[bi][4 * t + 1] = v.y;
            av[bi][4 * t + 2] = v.z;
            av[bi][4 * t + 3] = v.w;
          }
        } else if (fr2) {
          const float* plane = a.x + plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W);
#pragma unroll
          for (int j = 0; j < 16; j += 2) fr2_pair(plane, a.W, Wo, a.off, pq + j, av[bi][j], av[bi][j + 1]);
        } else {  // FactorizedReduce half: relu(x) at (oy*S + off, ox*S + off)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int pp = pq + j, oy = pp / Wo, ox = pp - oy * Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
            av[bi][j] = (iy < a.H && ix < a.W)
                            ? fmaxf(a.x[plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix], 0.f)
                            : 0.f;
          }
        }
      }
      // gW[co][ci] += sum_p dz[co][p] a[ci][p]: A[i = co][k = p], B[k = p][j = ci]
#pragma unroll
      for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int bo = 0; bo < BO; ++bo)
#pragma unroll
          for (int bi = 0; bi < BI; ++bi)
            macc[bo][bi] = __builtin_amdgcn_mfma_f32_16x16x4f32(dz[bo][j], av[bi][j], macc[bo][bi], 0, 0, 0);
    }
    if (!a.need_dx) continue;
    // dz chunk -> wave-private LDS tile [co][p]
    wave_lds_sync();  // the previous chunk's tile reads are done
#pragma unroll
    for (int bo = 0; bo < BO; ++bo)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        *reinterpret_cast<f4*>(sT + (bo * 16 + c16) * RS + q * 16 + 4 * t) =
            f4{dz[bo][4 * t], dz[bo][4 * t + 1], dz[bo][4 * t + 2], dz[bo][4 * t + 3]};
    wave_lds_sync();
    // dd[ci][p] = sum_co pw[co][ci] dz[co][p]: A[i = ci][k = co] = pw[co][ci], B[k = co][j = p]
#pragma unroll
    for (int bi = 0; bi < BI; ++bi) {
      f4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
      for (int k0 = 0; k0 < CO; k0 += 4) {
        const float av = a.pw[(k0 + q) * CI + ci0 + bi * 16 + c16];
#pragma unroll
        for (int pb = 0; pb < 4; ++pb)
          acc[pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sT[(k0 + q) * RS + pb * 16 + c16], acc[pb], 0, 0, 0);
      }
      // D map: row (ci) = bi*16 + q*4 + r, col (pixel) = pb*16 + c16
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ci = ci0 + bi * 16 + q * 4 + r;
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          const int pp = prem + pb * 16 + c16;
          const float v = acc[pb][r];
          if (a.mode == 0) {
            a.dd[((size_t)n * CI + ci) * HWo + pp] = v;
          } else {
            const int oy = pp / Wo, ox = pp - oy * Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
            if (iy < a.H && ix < a.W) {
              const size_t xi = plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix;
              if (a.overwrite) a.gx[xi] = a.x[xi] > 0.f ? v : 0.f;
              else if (a.x[xi] > 0.f) a.gx[xi] += v;
            }
          }
        }
      }
    }
  }
  if (!want_w) return;
  // the 4 waves' partial 16x16 blocks -> one LDS sum -> one atomic vector per workgroup
  __syncthreads();
  float* sG = smem;  // [CO][CI]
  for (int i = tid; i < CO * CI; i += 256) sG[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int bo = 0; bo < BO; ++bo)
#pragma unroll
    for (int bi = 0; bi < BI; ++bi)
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(sG + (bo * 16 + q * 4 + r) * CI + ci0 + bi * 16 + c16, macc[bo][bi][r]);
  __syncthreads();
  float* gW = a.gW + (size_t)rep_slot() * a.gstride;
  for (int i = tid; i < CO * CI; i += 256) atomicAdd(gW + i, sG[i]);
}

template <int CI, int CO>
static bool try_pw_bwd_px(const PwBwdBatch& b, hipStream_t st) {
  const PwBwdArgs& a = b.e[0];
  if (a.Cin != CI || a.Cout != CO) return false;
  const int total = a.N * a.Ho * a.Wo;
  // one pixel per thread: the 4-pixel vector form (pw_bwd_px_kernel<..., true>) measured slower at C = 8
  // (register pressure: 21.7 vs 17.6 us) and neutral at C = 4 on MI355X, so it is not launched
  const int per_edge = std::max(1, std::min((total + 255) / 256, max_blocks() / std::max(2 * b.n, 1)));
  hipLaunchKernelGGL((pw_bwd_px_kernel<CI, CO, false>), dim3(per_edge, b.n), dim3(256), 0, st, b);
  return true;
}

template <int CI, int CO>
static bool try_pw_bwd_wave(const PwBwdBatch& b, hipStream_t st) {
  const PwBwdArgs& a = b.e[0];
  if (a.Cin != CI || a.Cout != CO || (a.Ho * a.Wo) % 64 != 0) return false;
  for (int e = 0; e < b.n; ++e) {  // 16-byte operand loads
    const PwBwdArgs& x = b.e[e];
    const bool flat = x.mode == 0 || (x.S == 1 && x.off == 0 && x.H == x.Ho && x.W == x.Wo);
    const uintptr_t bits = (uintptr_t)x.gs.z | (uintptr_t)x.gs.g | (flat ? (x.mode == 0 ? (uintptr_t)x.ain : (uintptr_t)x.x) : (uintptr_t)0);
    if (bits & 15) return false;
  }
  constexpr int BI = CI / 16;
  const int chunks = a.N * a.Ho * a.Wo / 64;
  // split the input channels over waves while the launch has fewer than ~4 waves per SIMD
  int ns = 1;
  while (BI % (2 * ns) == 0 && chunks * ns * b.n < 4096) ns *= 2;
  const int per_edge = std::max(1, std::min((chunks * ns + 3) / 4, max_blocks() / std::max(b.n, 1)));
  const size_t lds = sizeof(float) * 4 * CO * (64 + 4);
  const dim3 grid(per_edge, b.n);
  if (ns == 1) hipLaunchKernelGGL((pw_bwd_wave_kernel<CI, CO, 1>), grid, dim3(256), lds, st, b);
  else if constexpr (BI % 2 == 0) {
    if (ns == 2) hipLaunchKernelGGL((pw_bwd_wave_kernel<CI, CO, 2>), grid, dim3(256), lds, st, b);
    else if constexpr (BI % 4 == 0) hipLaunchKernelGGL((pw_bwd_wave_kernel<CI, CO, 4>), grid, dim3(256), lds, st, b);
  }
  return true;
}

void launch_pw_bwd(const PwBwdBatch& b, hipStream_t st) {
  const PwBwdArgs& a = b.e[0];
  // narrow layers: pixel-per-thread kernel (see pw_bwd_px_kernel)
  if (try_pw_bwd_px<4, 4>(b, st) || try_pw_bwd_px<8, 8>(b, st) || try_pw_bwd_px<4, 8>(b, st) ||
      try_pw_bwd_px<8, 4>(b, st) || try_pw_bwd_px<12, 8>(b, st) || try_pw_bwd_px<2, 2>(b, st) ||
      try_pw_bwd_px<4, 2>(b, st) || try_pw_bwd_px<2, 4>(b, st))
    return;
  // 16..64-channel layers: wave-per-chunk MFMA kernel (see pw_bwd_wave_kernel)
  if (try_pw_bwd_wave<16, 16>(b, st) || try_pw_bwd_wave<32, 32>(b, st) || try_pw_bwd_wave<64, 64>(b, st) ||
      try_pw_bwd_wave<48, 16>(b, st) || try_pw_bwd_wave<48, 32>(b, st) || try_pw_bwd_wave<64, 32>(b, st) ||
      try_pw_bwd_wave<32, 16>(b, st) || try_pw_bwd_wave<128, 64>(b, st))
    return;
  int ntiles = a.N * a.Ho * a.Wo / 64;
  dim3 grid(per_edge_blocks(ntiles, b.n), b.n);
  size_t lds = sizeof(float) * (a.Cout * 65 + a.Cin * 65 + 4 * a.Cout + 4);
  const int nblk = (a.Cin % 16 == 0 && a.Cout % 16 == 0) ? (a.Cin / 16) * (a.Cout / 16) : 1 << 30;
  if (nblk <= 16) hipLaunchKernelGGL((pw_bwd_kernel<true, 4>), grid, dim3(256), lds, st, b);
  else if (nblk <= 32) hipLaunchKernelGGL((pw_bwd_kernel<true, 8>), grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL((pw_bwd_kernel<false>), grid, dim3(256), lds, st, b);
}


}  // namespace katib_hip
