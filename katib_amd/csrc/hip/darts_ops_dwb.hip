// DARTS depthwise / pooling backward kernels (dw_bwd tiles, dw_bwd_plane, pool_bwd, fused edge_bwd)
// and their launch heuristics. See darts_ops.hip for the design notes.
#include "darts_ops_dev.h"

namespace katib_hip {

// ------------------------------------------------------------------------------------------------
// dw_bwd: transposed depthwise. For own output rows [oy0, oy0+TR): dW_dw += dd * act(in);
// for own input rows [oy0*S, (oy0+TR)*S): ga = sum_taps dw * dd, masked by act'(in).
// PREBN: input = z_prev (pre-BN), act = relu(BN(.)) -> writes g_prev and reductions for BN bwd.
// else  : input = x, act = relu -> gx += ga * (x > 0).
// ------------------------------------------------------------------------------------------------
template <int K, int DIL, int S, bool PREBN>
__global__ void __launch_bounds__(256) dw_bwd_kernel(DwBwdBatch bt) {
  const DwBwdArgs& a = bt.e[blockIdx.y];
  constexpr int P = 64, KK = K * K;
  const int C = a.C, H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int TR = P / Wo;
  const int tiles = Ho / TR;
  const int ntiles = a.N * tiles;
  const int pad = a.pad;
  const int r = (K - 1) / 2 * DIL;         // == pad for these ops
  const int h = (r + S - 1) / S;           // halo output rows
  const int OR = TR + 2 * h;               // staged dd rows
  const int IR = (TR - 1) * S + (K - 1) * DIL + 1;
  const int IW = (Wo - 1) * S + (K - 1) * DIL + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sDD = smem;                        // [CH][OR][Wo]
  float* sIn = sDD + a.chunk * OR * Wo;     // [CH][IR][IW]
  float* sMean = sIn + a.chunk * IR * IW;   // [C]
  float* sInv = sMean + C;
  float* sRed = sInv + C;                   // [2C] block-local BN-bwd partials (PREBN)
  float* sGW = sRed + 2 * C;                // [C*K*K] block-local depthwise weight grads
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int c = tid; c < C; c += 256) {
    if (PREBN) bn_coeffs(a.inbn, c, sMean[c], sInv[c]);
    sRed[c] = 0.f;
    sRed[C + c] = 0.f;
  }
  if (a.gW)
    for (int i = tid; i < C * KK; i += 256) sGW[i] = 0.f;
  __syncthreads();
  const int own_in = TR * S;  // own input rows [oy0*S, oy0*S + own_in)
  const int nq = own_in * W;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int n = t / tiles, oy0 = (t % tiles) * TR;
    const int iy0 = oy0 * S - pad;
    const size_t xin = (size_t)n * C * H * W;
    const float* ddn = a.dd + (size_t)n * C * Ho * Wo;
    for (int c0 = 0; c0 < C; c0 += a.chunk) {
      const int cn = min(a.chunk, C - c0);
      #pragma unroll 4  // keep several global loads of the staging pass in flight
      for (int i = tid; i < cn * OR * Wo; i += 256) {
        int cc = i / (OR * Wo), rr = (i / Wo) % OR, q = i % Wo;
        int oy = oy0 - h + rr;
        sDD[i] = (oy >= 0 && oy < Ho) ? ddn[((size_t)(c0 + cc) * Ho + oy) * Wo + q] : 0.f;
      }
      if (a.gW) {
        #pragma unroll 4  // keep several global loads of the staging pass in flight
        for (int i = tid; i < cn * IR * IW; i += 256) {
          int cc = i / (IR * IW), rr = (i / IW) % IR, q = i % IW;
          int iy = iy0 + rr, ix = -pad + q, c = c0 + cc;
          float v = 0.f;
          if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
            v = xval<PREBN>(a.x, xin + ((size_t)c * H + iy) * W + ix);
            if (PREBN) v = (v - sMean[c]) * sInv[c];
            v = fmaxf(v, 0.f);
          }
          sIn[i] = v;
        }
      }
      __syncthreads();
      // weight grads: thread per (channel, tap), summed over the tile's 64 output pixels
      if (a.gW) {
        for (int job = tid; job < cn * KK; job += 256) {
          const int cc = job / KK, tap = job % KK, ky = tap / K, kx = tap % K;
          const float* dd = sDD + (cc * OR + h) * Wo;
          const float* in = sIn + (cc * IR + ky * DIL) * IW + kx * DIL;
          float s = 0.f;
          for (int ty = 0; ty < TR; ++ty)
            for (int tx = 0; tx < Wo; ++tx) s += dd[ty * Wo + tx] * in[ty * S * IW + tx * S];
          sGW[(c0 + cc) * KK + tap] += s;  // unique owner
        }
      }
      // input grads for own input rows: the tap geometry depends only on the pixel q, so it
      // is computed once per pixel (branch-free masks) and reused for every channel. A tile
      // owns nq = 64*S*S input pixels: at stride 1 the block's 4 waves take 4 channel groups
      // of the same 64 pixels (wave-uniform channel -> scalar weight loads, wave-level sums).
      const int qspan = (nq < 256 && 256 % nq == 0) ? nq : 256;
      const int G = 256 / qspan;
      for (int q0 = 0; q0 < nq; q0 += qspan) {
        const int q = q0 + tid % qspan;
        const int cg = __builtin_amdgcn_readfirstlane(tid / qspan);
        const int rr = q / W, ix = q - rr * W;
        const int iy = oy0 * S + rr;
        const bool ok = q < nq && iy < H;
        int srow[K], ocol[K];
        float mrow[K], mcol[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          int ty = iy + pad - k * DIL;  // = oy * S when valid
          int oy = ty >= 0 ? ty / S : -1;
          bool v = ok && ty >= 0 && (ty % S) == 0 && oy < Ho;
          srow[k] = v ? oy - (oy0 - h) : 0;
          mrow[k] = v ? 1.f : 0.f;
          int tx = ix + pad - k * DIL;
          int ox = tx >= 0 ? tx / S : -1;
          bool u = ok && tx >= 0 && (tx % S) == 0 && ox < Wo;
          ocol[k] = u ? ox : 0;
          mcol[k] = u ? 1.f : 0.f;
        }
        for (int cc = cg; cc < cn; cc += G) {
          const int c = c0 + cc;
          const float* wk = a.dw + c * KK;  // wave-uniform -> scalar loads
          const float* dd = sDD + cc * OR * Wo;
          float ga = 0.f;
#pragma unroll
          for (int ky = 0; ky < K; ++ky) {
            float rowacc = 0.f;
#pragma unroll
            for (int kx = 0; kx < K; ++kx) rowacc += mcol[kx] * wk[ky * K + kx] * dd[srow[ky] * Wo + ocol[kx]];
            ga += mrow[ky] * rowacc;
          }
          const size_t xi = ((size_t)(n * C + c) * H + iy) * W + ix;
          if (PREBN) {
            float g = 0.f, gy = 0.f;
            if (ok) {
              float y = (xval<true>(a.x, xi) - sMean[c]) * sInv[c];
              g = y > 0.f ? ga : 0.f;
              gy = g * y;
              a.gout[xi] = g;
            }
            if (a.red) {
              g = wave_sum(g);
              gy = wave_sum(gy);
              if (lane == 0) {
                atomicAdd(sRed + c, g);  // one LDS atomic per wave per channel
                atomicAdd(sRed + C + c, gy);
              }
            }
          } else if (ok) {
            const float gm = xval<false>(a.x, xi) > 0.f ? ga : 0.f;
            if (a.overwrite) a.gout[xi] = gm;
            else if (gm != 0.f) a.gout[xi] += gm;
          }
        }
      }
      __syncthreads();
    }
  }
  if (PREBN && a.red)
    for (int i = tid; i < 2 * C; i += 256) atomicAdd(a.red + rep_slot() * 2 * C + i, (double)sRed[i]);
  if (a.gW)
    for (int i = tid; i < C * KK; i += 256) atomicAdd(a.gW + (size_t)rep_slot() * a.gstride + i, sGW[i]);
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// ------------------------------------------------------------------------------------------------
// pool_bwd: gx += avg^T(dz_avg) + max^T(dz_max) + wid * dout (identity skip), per (n,c) plane
// ------------------------------------------------------------------------------------------------
template <int S, bool V4 = false>
__device__ __forceinline__ void pool_bwd_body(const PoolBwdArgs& a, const int bx) {
  const int C = a.C, H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo, HWo = Ho * Wo;
  const int nc = bx, c = nc % C;
  const size_t ob = (size_t)nc * HWo;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sGa = smem;                                          // [HWo] dz_avg / window count
  float* sGm = smem + HWo;                                    // [HWo] dz_max
  unsigned char* sArg = (unsigned char*)(smem + 2 * HWo);     // [HWo] argmax tap
  // the plane's BN coefficients: four threads each sum one pair over the replicas
  __shared__ float sCo[8];
  KSTAMP(0);
  // all four replica pair-sums in ONE memory round trip: wave 0's 16-lane groups take the avg
  // pool's BN statistics, the max pool's, and the two BN-backward sums (S1, S2) each - folded
  // (rep 1) or not (rep kRep: two loads per lane). One thread per BN walking kRep replicas in
  // rounds of 8 was four dependent round trips (~2.8 us of a ~10 us workgroup, phase stamps r06)
  if (threadIdx.x < 64) {
    const int grp = threadIdx.x >> 4, j = threadIdx.x & 15;
    const GradSrc& gs = grp & 1 ? a.gm : a.ga;
    const bool on = gs.z != nullptr, stats = grp < 2;
    const BNRef& b = gs.bn;
    double s = 0.0, s2 = 0.0;
    if (on && stats && !b.eval) {
      for (int r = j; r < b.rep; r += 16) {
        s += b.sums[(size_t)r * b.rstride + c];
        s2 += b.sums[(size_t)r * b.rstride + b.C + c];
      }
    } else if (on && !stats && !gs.eval) {
      const int rep = gs.rep, rs = gs.rep == 1 ? 0 : gs.rstride;
      const size_t off2 = gs.S2 - gs.S1;
      for (int r = j; r < rep; r += 16) {
        s += gs.S1[(size_t)r * rs + c];
        s2 += gs.S1[(size_t)r * rs + off2 + c];
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      s += __shfl_xor(s, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    if (j == 0) {
      float* o = sCo + 4 * (grp & 1) + (stats ? 0 : 2);
      if (!on) {
        o[0] = 0.f;
        o[1] = stats ? 1.f : 0.f;
      } else if (stats) {
        if (b.eval) {
          o[0] = b.rmean[c];
          o[1] = rsqrtf(b.rvar[c] + b.eps);
        } else {  // as bn_moments / bn_coeffs
          const double m = s * (double)b.inv_count;
          double v = s2 * (double)b.inv_count - m * m;
          if (v < 0) v = 0;
          o[0] = (float)m;
          o[1] = rsqrtf((float)v + b.eps);
        }
      } else {  // as gs_means
        o[0] = gs.eval ? 0.f : (float)(s * (double)gs.bn.inv_count);
        o[1] = gs.eval ? 0.f : (float)(s2 * (double)gs.bn.inv_count);
      }
    }
  }
  __syncthreads();
  KSTAMP(1);
  const float ma = sCo[0], ia = sCo[1], a1 = a.ga.z ? sCo[2] : 0.f, a2 = a.ga.z ? sCo[3] : 0.f;
  const float mm = sCo[4], im = sCo[5], m1 = a.gm.z ? sCo[6] : 0.f, m2 = a.gm.z ? sCo[7] : 0.f;
  const float wa = a.ga.w ? a.ga.w[a.ga.widx] : 0.f;
  const float wm = a.gm.w ? a.gm.w[a.gm.widx] : 0.f;
  const float wid = (a.w && a.id_idx >= 0) ? a.w[a.id_idx] : 0.f;
  if constexpr (V4) {
    // 4 consecutive outputs / input pixels per thread: every operand one 16-byte (amax: 4-byte)
    // access instead of four 4-byte ones - a quarter of the memory requests in flight for the
    // same bytes (HWo, H*W % 4 == 0 and every operand 16-byte aligned: host-checked)
    typedef float f4 __attribute__((ext_vector_type(4)));
    const float* gsrc = a.ga.z ? a.ga.g : a.gm.g;  // both pools read the edge's dout
    for (int o4 = threadIdx.x * 4; o4 < HWo; o4 += 1024) {
      const f4 g = *reinterpret_cast<const f4*>(gsrc + ob + o4);
      if (a.ga.z) {
        const f4 z = zld4(a.ga.z + ob + o4);
        const f4 d = wa * ia * (g - a1 - ((z - ma) * ia) * a2);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int o = o4 + t, oy = o / Wo, ox = o - oy * Wo;
          const int y0 = max(oy * S - 1, 0), y1 = min(oy * S + 1, H - 1);
          const int x0 = max(ox * S - 1, 0), x1 = min(ox * S + 1, W - 1);
          sGa[o] = d[t] / (float)((y1 - y0 + 1) * (x1 - x0 + 1));
        }
      } else {
        *reinterpret_cast<f4*>(sGa + o4) = f4{0.f, 0.f, 0.f, 0.f};
      }
      if (a.gm.z) {
        const f4 z = zld4(a.gm.z + ob + o4);
        *reinterpret_cast<f4*>(sGm + o4) = wm * im * (g - m1 - ((z - mm) * im) * m2);
        *reinterpret_cast<unsigned*>(sArg + o4) = *reinterpret_cast<const unsigned*>(a.amax + ob + o4);
      } else {
        *reinterpret_cast<f4*>(sGm + o4) = f4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<unsigned*>(sArg + o4) = 0xffffffffu;
      }
    }
    __syncthreads();
    KSTAMP(2);
    const size_t pb = (size_t)nc * H * W;
    for (int q4 = threadIdx.x * 4; q4 < H * W; q4 += 1024) {
      f4 g = {0.f, 0.f, 0.f, 0.f};
      if (a.dout_id) g = wid * *reinterpret_cast<const f4*>(a.dout_id + pb + q4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j < a.nextra) g += *reinterpret_cast<const f4*>(a.extra[j] + pb + q4);
      const int iy = q4 / W, ix0 = q4 - iy * W;  // 4 pixels of one row (W % 4 == 0)
      if constexpr (S == 1) {
        // stride 1: the quad's 3 x 6 window of outputs (rows iy - 1 .. iy + 1, columns ix0 - 1 ..
        // ix0 + 4; Ho = H, Wo = W) read once - a 16-byte / 4-byte LDS read for the middle four
        // columns and two scalars per row and array - instead of 9 neighbours x 3 arrays per pixel
        // (27 reads per row instead of 108 per quad); out-of-range neighbours read as ga = gm = 0 and
        // tap 255, and the sums run in the per-pixel loop's order
        float wa[3][6], wm[3][6];
        unsigned char wt[3][6];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const int oy = iy - 1 + r;
          const bool rok = oy >= 0 && oy < Ho;
          const int o = (rok ? oy : 0) * Wo + ix0;
          const f4 ga4 = *reinterpret_cast<const f4*>(sGa + o), gm4 = *reinterpret_cast<const f4*>(sGm + o);
          const unsigned t4 = *reinterpret_cast<const unsigned*>(sArg + o);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            wa[r][k + 1] = rok ? ga4[k] : 0.f;
            wm[r][k + 1] = rok ? gm4[k] : 0.f;
            wt[r][k + 1] = rok ? (unsigned char)(t4 >> (8 * k)) : 255;
          }
          const bool lok = rok && ix0 > 0, hok = rok && ix0 + 4 < Wo;
          wa[r][0] = lok ? sGa[o - 1] : 0.f;
          wm[r][0] = lok ? sGm[o - 1] : 0.f;
          wt[r][0] = lok ? sArg[o - 1] : 255;
          wa[r][5] = hok ? sGa[o + 4] : 0.f;
          wm[r][5] = hok ? sGm[o + 4] : 0.f;
          wt[r][5] = hok ? sArg[o + 4] : 255;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float v = 0.f;
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int cx = 0; cx < 3; ++cx) {  // output (iy - 1 + r, ix0 + t - 1 + cx): tap (2 - r) * 3 + (2 - cx)
              v += wa[r][t + cx];
              if (wt[r][t + cx] == (2 - r) * 3 + (2 - cx)) v += wm[r][t + cx];
            }
          g[t] += v;
        }
        f4* dst = reinterpret_cast<f4*>(a.gx + pb + q4);
        *dst = a.overwrite ? g : *dst + g;
        continue;
      }
      if constexpr (S == 2) {
        // stride 2: the quad (ix0 = 4k) meets output columns 2k .. 2k + 2 and output rows m = iy / 2
        // and, for odd iy, m + 1 - a 2 x 3 window read once (an 8-byte pair + a scalar per row and
        // array); pixel t reads columns t / 2 .. (t + 1) / 2. Out-of-range outputs read as 0 / tap 255
        float wa[2][3], wm[2][3];
        unsigned char wt[2][3];
        const int m = iy >> 1, k2 = ix0 >> 1;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int oy = m + r;
          const bool rok = oy < Ho && (r == 0 || (iy & 1));
          const int o = (rok ? oy : m) * Wo + k2;
          typedef float f2 __attribute__((ext_vector_type(2)));
          const f2 ga2 = *reinterpret_cast<const f2*>(sGa + o), gm2 = *reinterpret_cast<const f2*>(sGm + o);
          const unsigned short t2 = *reinterpret_cast<const unsigned short*>(sArg + o);
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            wa[r][c] = rok ? ga2[c] : 0.f;
            wm[r][c] = rok ? gm2[c] : 0.f;
            wt[r][c] = rok ? (unsigned char)(t2 >> (8 * c)) : 255;
          }
          const bool hok = rok && k2 + 2 < Wo;
          wa[r][2] = hok ? sGa[o + 2] : 0.f;
          wm[r][2] = hok ? sGm[o + 2] : 0.f;
          wt[r][2] = hok ? sArg[o + 2] : 255;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float v = 0.f;
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = t / 2; c <= (t + 1) / 2; ++c) {  // output (m + r, 2k + c)
              v += wa[r][c];
              if (wt[r][c] == (iy - 2 * (m + r) + 1) * 3 + (t - 2 * c + 1)) v += wm[r][c];
            }
          g[t] += v;
        }
        f4* dst = reinterpret_cast<f4*>(a.gx + pb + q4);
        *dst = a.overwrite ? g : *dst + g;
        continue;
      }
      const int oy_lo = iy - 1 < 0 ? 0 : (iy - 1 + S - 1) / S, oy_hi = min((iy + 1) / S, Ho - 1);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int ix = ix0 + t;
        const int ox_lo = ix - 1 < 0 ? 0 : (ix - 1 + S - 1) / S, ox_hi = min((ix + 1) / S, Wo - 1);
        float v = 0.f;
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
          for (int ox = ox_lo; ox <= ox_hi; ++ox) {
            const int o = oy * Wo + ox;
            v += sGa[o];
            if (sArg[o] == (iy - oy * S + 1) * 3 + (ix - ox * S + 1)) v += sGm[o];
          }
        g[t] += v;
      }
      f4* dst = reinterpret_cast<f4*>(a.gx + pb + q4);
      *dst = a.overwrite ? g : *dst + g;
    }
    KSTAMP(3);
    return;
  }
  for (int o = threadIdx.x; o < HWo; o += 256) {
    int oy = o / Wo, ox = o % Wo;
    if (a.ga.z) {
      int y0 = max(oy * S - 1, 0), y1 = min(oy * S + 1, H - 1);
      int x0 = max(ox * S - 1, 0), x1 = min(ox * S + 1, W - 1);
      sGa[o] = bn_bwd_val(a.ga, ob + o, ma, ia, wa, a1, a2) / (float)((y1 - y0 + 1) * (x1 - x0 + 1));
    } else {
      sGa[o] = 0.f;
    }
    if (a.gm.z) {
      sGm[o] = bn_bwd_val(a.gm, ob + o, mm, im, wm, m1, m2);
      sArg[o] = a.amax[ob + o];
    } else {
      sGm[o] = 0.f;
      sArg[o] = 255;
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < H * W; q += 256) {
    int iy = q / W, ix = q % W;
    float g = 0.f;
    // outputs whose 3x3 window (pad 1) covers (iy, ix): oy*S - 1 <= iy <= oy*S + 1
    int oy_lo = iy - 1 < 0 ? 0 : (iy - 1 + S - 1) / S, oy_hi = min((iy + 1) / S, Ho - 1);
    int ox_lo = ix - 1 < 0 ? 0 : (ix - 1 + S - 1) / S, ox_hi = min((ix + 1) / S, Wo - 1);
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        int o = oy * Wo + ox;
        g += sGa[o];
        int tap = (iy - oy * S + 1) * 3 + (ix - ox * S + 1);
        if (sArg[o] == tap) g += sGm[o];
      }
    }
    if (a.dout_id) g += wid * a.dout_id[(size_t)nc * H * W + q];
#pragma unroll
    for (int j = 0; j < 4; ++j)  // the node's conv input grads (constant indices: a dynamic index into
      if (j < a.nextra) g += a.extra[j][(size_t)nc * H * W + q];  // the argument copy sends it to scratch)
    if (a.overwrite) a.gx[(size_t)nc * H * W + q] = g;
    else a.gx[(size_t)nc * H * W + q] += g;
  }
}
template <int S>
__global__ void __launch_bounds__(256) pool_bwd_kernel(PoolBwdBatch bt) {
  pool_bwd_body<S>(bt.e[blockIdx.y], blockIdx.x);
}

// stride-1 and stride-2 pool backward of a node in one launch (different edges: different gx)
template <bool V4>
__global__ void __launch_bounds__(256) pool_bwd_multi_kernel(PoolBwdBatch bt) {
  const PoolBwdArgs a = bt.e[blockIdx.y];  // copy: see dwpw_plane_multi_kernel
  if ((int)blockIdx.x >= a.N * a.C) return;
  if (a.S == 1) pool_bwd_body<1, V4>(a, blockIdx.x);
  else pool_bwd_body<2, V4>(a, blockIdx.x);
}


// ------------------------------------------------------------------------------------------------
// dw_bwd_plane: dw_bwd for narrow layers (C <= 16), the backward twin of dwpw_plane. One
// workgroup per (image, band of input rows): the dd rows the band's input pixels reach (plus a
// zero border of PO = ceil(pad/S), so every tap lands inside the staged grid) and act(in) of the
// band are staged with one coalesced burst (and, when accumulating, the current input gradient),
// then
//   input grads : thread per own input pixel, all channels: ga = sum_taps w * dd (transposed
//                 depthwise gather from LDS), masked by act'(in); PREBN keeps the BN-backward
//                 sums per thread and reduces once per block;
//   weight grads: thread per (channel, tap[, pixel part]) summing act(in) * dd over the band.
// Every input pixel belongs to exactly one band, so both sums are complete without overlap.
// Replaces the 64-pixel tiles whose halo rows were re-staged per tile behind two barriers.
// ------------------------------------------------------------------------------------------------
template <int K, int DIL, int S, bool PREBN, int C>
__device__ __forceinline__ void dw_bwd_plane_body(const DwBwdArgs& a, const int bx, const int nb, const int dbg) {
  constexpr int KK = K * K, PAD = (K - 1) / 2 * DIL, PO = (PAD + S - 1) / S, SH = S == 2 ? 1 : 0;
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  // channel groups: depthwise backward never mixes channels, so wider layers run as a.C / C
  // independent C-channel groups (blockIdx.x = (image * nb + band) * G + group)
  const int G = a.C / C, grp = bx % G, nbx = bx / G, c0 = grp * C;
  const int n = nbx / nb, band = nbx - n * nb;
  const int BRi = H / nb, iy0 = band * BRi, nrow = BRi;
  const int oyA = (iy0 - PAD) >> SH;                 // floor division (S in {1, 2})
  const int oyB = (iy0 + nrow - 1 + PAD) >> SH;
  const int ODR = oyB - oyA + 1, ODW = lds_pitch(Wo + 2 * PO), NP = nrow * W;  // row pitch: lds_pitch
  const bool accum = !PREBN && !a.overwrite;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sWt = smem;                    // [C][KK] depthwise weights (dwb_head_floats)
  float* sGW = smem + C * 25;           // [C][KK] block-local depthwise weight gradients
  float* sDD = smem + dwb_head_floats(C);  // [C][ODR][ODW]
  float* sIn = sDD + C * ODR * ODW;     // [C][nrow][W] act(in)
  float* sOld = sIn + C * NP;           // [C][nrow][W] current gradient (accumulate mode)
  __shared__ float sMean[C], sInv[C], sRed[2 * C];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  KSTAMP(0);
  // the group's depthwise weights in LDS, loaded with the prologue: read from global memory
  // inside the tap loops, every weight was its own load + s_waitcnt vmcnt(0) (the compiler may
  // not hoist them above the gradient stores, which could alias) - 9-25 serial round trips per
  // channel in the middle of the compute phase
  for (int i = tid; i < C * KK; i += 256) {
    sGW[i] = 0.f;
    sWt[i] = a.dw[c0 * KK + i];
  }
  if (tid < C) {
    if (PREBN) bn_coeffs(a.inbn, c0 + tid, sMean[tid], sInv[tid]);
    sRed[tid] = 0.f;
    sRed[C + tid] = 0.f;
  }
  // only the input-BN staging reads the prologue's LDS (sMean / sInv) before the staging barrier
  if (PREBN) __syncthreads();
  KSTAMP(1);
  // staging with 16-byte loads (the band's rows are contiguous per channel; W, Wo % 4 == 0):
  // many wide loads in flight per wave, which the one-row-per-wave scalar loop lacked
  const float* ddn = a.dd + ((size_t)n * a.C + c0) * Ho * Wo;
  const size_t xn = ((size_t)n * a.C + c0) * H * W;
  const int va = max(oyA, 0), vb = min(oyB, Ho - 1), vrows = vb - va + 1;  // staged dd rows inside [0, Ho)
  {
    const int q4 = vrows * Wo / 4;  // float4s per channel
#pragma unroll 4
    for (int i = tid; i < C * q4; i += 256) {
      const int c = i / q4, o = (i - c * q4) * 4, r = o / Wo, ox = o - r * Wo;
      const float4 v = *reinterpret_cast<const float4*>(ddn + ((size_t)c * Ho + va) * Wo + o);
      float* d = sDD + (c * ODR + va - oyA + r) * ODW + PO + ox;
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
    // zero border: rows outside [0, Ho) and the PO columns on each side
    for (int i = tid; i < C * ODR; i += 256) {
      const int c = i / ODR, oy = oyA + i - c * ODR;
      float* d = sDD + i * ODW;
      if (oy < 0 || oy >= Ho) {
        for (int q = 0; q < ODW; ++q) d[q] = 0.f;
      } else {
        for (int q = 0; q < PO; ++q) d[q] = d[PO + Wo + q] = 0.f;
      }
    }
  }
  {
    const int q4 = NP / 4;
#pragma unroll 4
    for (int i = tid; i < C * q4; i += 256) {
      const int c = i / q4, o = (i - c * q4) * 4;
      float4 v = xval4<PREBN>(a.x, xn + ((size_t)c * H + iy0) * W + o);
      if (PREBN) {
        const float m = sMean[c], iv = sInv[c];
        v.x = (v.x - m) * iv;
        v.y = (v.y - m) * iv;
        v.z = (v.z - m) * iv;
        v.w = (v.w - m) * iv;
      }
      v.x = fmaxf(v.x, 0.f);
      v.y = fmaxf(v.y, 0.f);
      v.z = fmaxf(v.z, 0.f);
      v.w = fmaxf(v.w, 0.f);
      *reinterpret_cast<float4*>(sIn + c * NP + o) = v;
    }
    if (accum) {
      const float* gsrc = a.gout + ((size_t)n * a.C + c0) * H * W;
#pragma unroll 4
      for (int i = tid; i < C * q4; i += 256) {
        const int c = i / q4, o = (i - c * q4) * 4;
        *reinterpret_cast<float4*>(sOld + c * NP + o) =
            *reinterpret_cast<const float4*>(gsrc + ((size_t)c * H + iy0) * W + o);
      }
    }
  }
  __syncthreads();
  KSTAMP(2);
  // input gradients of the band's own pixels
  float st1[C], st2[C];
#pragma unroll
  for (int c = 0; c < C; ++c) st1[c] = st2[c] = 0.f;
  float* gn = a.gout + ((size_t)n * a.C + c0) * H * W;
  if (S == 1 && a.vin) {
    // stride 1: 4 consecutive input pixels of one row per thread (W % 4 == 0, as the staging
    // assumes): the taps' column offsets are shared, and the gradient leaves as one 16-byte store
    // per channel instead of four 4-byte ones
    // The staged dd row the 4 pixels meet through every column tap is dd columns ix .. ix + 3 + 2 PAD
    // (PO = PAD at stride 1): NQ aligned 16-byte quads from ix (ODW = lds_pitch, a multiple of 4),
    // read as ds_read_b128 per tap row instead of 4 K ds_read_b32 at a 4-float lane stride (8 of
    // 32 banks: 4-way conflicts)
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int NQ = (4 + 2 * PAD + 3) / 4;
    // work item = (channel, pixel quad), channel-major: with the channel loop inside the thread
    // only NP / 4 threads had work (64 of 256 for an 8-row band of a 32-wide plane), each walking
    // C channels with nothing to hide its LDS latency behind; now every thread takes one item and a
    // wave holds one channel whenever NP / 4 is a multiple of 64 (uniform weight reads)
    const int NQ4 = NP / 4;
    for (int j = tid; j < ((dbg & 1) ? 0 : C * NQ4); j += 256) {
      const int c = j / NQ4, p = (j - c * NQ4) * 4;
      const int r = p / W, ix = p - r * W, iy = iy0 + r;
      int srow[K];
#pragma unroll
      for (int k = 0; k < K; ++k) srow[k] = (iy + PAD - k * DIL - oyA) * ODW + ix;
      KEEP_WEIGHT_READS_LOCAL();
      const float* wk = sWt + c * KK;
      const float* dd = sDD + c * ODR * ODW;
      f4 ga = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        float v[4 * NQ];  // v[m] = dd column ix + m
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const float4 t = *reinterpret_cast<const float4*>(dd + srow[ky] + 4 * q);
          v[4 * q] = t.x;
          v[4 * q + 1] = t.y;
          v[4 * q + 2] = t.z;
          v[4 * q + 3] = t.w;
        }
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const float w = wk[ky * K + kx];
          const int o = 2 * PAD - kx * DIL;  // pixel ix + t meets dd column ix + t + o
          ga.x += w * v[o];
          ga.y += w * v[o + 1];
          ga.z += w * v[o + 2];
          ga.w += w * v[o + 3];
        }
      }
      const int li = (c * nrow + r) * W + ix;
      const f4 act = *reinterpret_cast<const f4*>(sIn + li);
      const f4 g = {act.x > 0.f ? ga.x : 0.f, act.y > 0.f ? ga.y : 0.f, act.z > 0.f ? ga.z : 0.f,
                    act.w > 0.f ? ga.w : 0.f};
      f4* dst = reinterpret_cast<f4*>(gn + ((size_t)c * H + iy) * W + ix);
      if (PREBN) {
        *dst = g;
        const float t1 = (g.x + g.y) + (g.z + g.w);
        const float t2 = (g.x * act.x + g.y * act.y) + (g.z * act.z + g.w * act.w);
#pragma unroll
        for (int cc = 0; cc < C; ++cc)  // select into the register arrays (no dynamic index)
          if (cc == c) {
            st1[cc] += t1;
            st2[cc] += t2;
          }
      } else {
        *dst = accum ? *reinterpret_cast<const f4*>(sOld + li) + g : g;
      }
    }
  }
  if constexpr (S == 2) {
    // stride 2: input pixel (iy, ix) meets tap (ky, kx) only when iy + PAD - ky*DIL and
    // ix + PAD - kx*DIL are both even. Threads walk the band class by class (row parity, column
    // parity; nrow, W even), so when a class spans whole waves (NPc % 64 == 0) the valid taps are
    // wave-uniform and the others are skipped by scalar branches instead of masked multiply-adds:
    // a quarter of the work (a dilated tap set is all-or-nothing per class).
    const int hw2 = W / 2, NPc = (nrow / 2) * hw2;
    for (int q = tid; q < ((dbg & 1) || !a.vin ? 0 : NP); q += 256) {
      const int cls = NPc % 64 == 0 ? __builtin_amdgcn_readfirstlane(q / NPc) : q / NPc;
      const int qq = q - cls * NPc, rr = qq / hw2, xx = qq - rr * hw2;
      const int r = 2 * rr + (cls >> 1), ix = 2 * xx + (cls & 1), iy = iy0 + r;
      const int iyc = iy0 + (cls >> 1), ixc = cls & 1;  // class representatives (parities only)
      int srow[K], scol[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        srow[k] = (((iy + PAD - k * DIL) >> 1) - oyA) * ODW;
        scol[k] = ((ix + PAD - k * DIL) >> 1) + PO;
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        KEEP_WEIGHT_READS_LOCAL();
        const float* wk = sWt + c * KK;  // LDS broadcast reads
        const float* dd = sDD + c * ODR * ODW;
        float ga = 0.f;
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
          if ((iyc + PAD - ky * DIL) & 1) continue;
#pragma unroll
          for (int kx = 0; kx < K; ++kx) {
            if ((ixc + PAD - kx * DIL) & 1) continue;
            ga += wk[ky * K + kx] * dd[srow[ky] + scol[kx]];
          }
        }
        const int li = (c * nrow + r) * W + ix;
        const float act = sIn[li];
        const size_t gi = ((size_t)c * H + iy) * W + ix;
        const float g = act > 0.f ? ga : 0.f;
        if (PREBN) {
          gn[gi] = g;
          st1[c] += g;
          st2[c] += g * act;
        } else {
          gn[gi] = accum ? sOld[li] + g : g;
        }
      }
    }
  }
  for (int p = tid; p < ((dbg & 1) || a.vin ? 0 : NP); p += 256) {
    const int r = p / W, ix = p - r * W, iy = iy0 + r;
    int srow[K], scol[K];
    float mrow[K], mcol[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int t = iy + PAD - k * DIL, u = ix + PAD - k * DIL;
      srow[k] = ((t >> SH) - oyA) * ODW;
      scol[k] = (u >> SH) + PO;
      mrow[k] = (S == 1 || (t & 1) == 0) ? 1.f : 0.f;
      mcol[k] = (S == 1 || (u & 1) == 0) ? 1.f : 0.f;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      KEEP_WEIGHT_READS_LOCAL();
        const float* wk = sWt + c * KK;  // LDS broadcast reads
      const float* dd = sDD + c * ODR * ODW;
      float ga = 0.f;
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        float rowacc = 0.f;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const float v = wk[ky * K + kx] * dd[srow[ky] + scol[kx]];
          rowacc += S == 1 ? v : mcol[kx] * v;
        }
        ga += S == 1 ? rowacc : mrow[ky] * rowacc;
      }
      const int li = (c * nrow + r) * W + ix;
      const float act = sIn[li];
      const size_t gi = ((size_t)c * H + iy) * W + ix;
      const float g = act > 0.f ? ga : 0.f;
      if (PREBN) {
        gn[gi] = g;
        st1[c] += g;
        st2[c] += g * act;  // g * y == g * relu(y)
      } else {
        gn[gi] = accum ? sOld[li] + g : g;
      }
    }
  }
  if (PREBN && a.red) {
    float st[2 * C];  // [sum g | sum g*y], reduce-scattered over the wave
#pragma unroll
    for (int c = 0; c < C; ++c) st[c] = st1[c], st[C + c] = st2[c];
    const float v = wave_reduce_scatter<2 * C>(st);
    if ((lane & (32 / C - 1)) == 0) atomicAdd(sRed + wave_scatter_index<2 * C>(lane), v);
  }
  KSTAMP(3);
  // depthwise weight gradients over the band: thread per (channel, tap, pixel part)
  if (a.gW && !(dbg & 2) && S == 1) {
    // stride 1: job = (channel, ky, own row). A 4-pixel quad of the input row (one 16-byte LDS
    // read) and the 4 + 2*PAD dd values it meets across all K column taps (registers) feed
    // 4*K multiply-adds: ~1.5 per LDS read against 0.5 for a pixel-by-pixel walk per tap
    // job = (row part, channel, ky, row); when the C * K * nrow jobs leave threads idle, each row
    // is split into XP column parts (XP | W / 4), a partial sum each
    const int JB = C * K * nrow, W4 = W / 4;
    int XP = 1;
    while (XP * 2 * JB <= 256 && W4 % (XP * 2) == 0) XP *= 2;
    const int XW = W / XP;
    for (int j = tid; j < JB * XP; j += 256) {
      const int xp = j / JB, jj = j - xp * JB;
      const int c = jj / (K * nrow), rem = jj - c * K * nrow, ky = rem / nrow, r = rem - ky * nrow;
      const float* ddr = sDD + (c * ODR + iy0 + r + PAD - ky * DIL - oyA) * ODW + PO;
      const float* inr = sIn + c * NP + r * W;
      float acc[K];
#pragma unroll
      for (int kx = 0; kx < K; ++kx) acc[kx] = 0.f;
      for (int ix = xp * XW; ix < (xp + 1) * XW; ix += 4) {
        const float4 v = *reinterpret_cast<const float4*>(inr + ix);
        // dseg[m] = dd[ix - PAD + m]: dd column ix - PAD + PO + m = ix + m (PO = PAD at stride 1),
        // whole aligned quads from ix (ds_read_b128; ODW = lds_pitch)
        constexpr int NQ = (4 + 2 * PAD + 3) / 4;
        float dseg[4 * NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const float4 t = *reinterpret_cast<const float4*>(ddr - PO + ix + 4 * q);
          dseg[4 * q] = t.x;
          dseg[4 * q + 1] = t.y;
          dseg[4 * q + 2] = t.z;
          dseg[4 * q + 3] = t.w;
        }
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int o = 2 * PAD - kx * DIL;  // in[ix + q] meets dd[ix + q + PAD - kx*DIL]
          acc[kx] += v.x * dseg[o] + v.y * dseg[o + 1] + v.z * dseg[o + 2] + v.w * dseg[o + 3];
        }
      }
#pragma unroll
      for (int kx = 0; kx < K; ++kx) atomicAdd(sGW + c * KK + ky * K + kx, acc[kx]);
    }
  } else if (a.gW && !(dbg & 2)) {
    constexpr int JOBS = C * KK, T = JOBS >= 256 ? 1 : 256 / JOBS;
    for (int j = tid; j < JOBS * T; j += 256) {
      const int job = j / T, part = j - job * T;
      const int c = job / KK, tap = job - c * KK, ky = tap / K, kx = tap - ky * K;
      const float* dd = sDD + c * ODR * ODW;
      const float* in = sIn + c * NP;
      float acc = 0.f;
      for (int r = 0; r < nrow; ++r) {
        const int t = iy0 + r + PAD - ky * DIL;
        if (S == 2 && (t & 1)) continue;
        const float* ddr = dd + ((t >> SH) - oyA) * ODW + PO;
        const float* inr = in + r * W;
        for (int ix = part * S + ((S == 2) ? ((PAD - kx * DIL) & 1) : 0); ix < W; ix += T * S)
          acc += inr[ix] * ddr[(ix + PAD - kx * DIL) >> SH];
      }
      atomicAdd(sGW + job, acc);
    }
  }
  KSTAMP(4);
  __syncthreads();
  if (PREBN && a.red && tid < 2 * C)  // red replica layout [sum g: a.C | sum g*y: a.C]
    atomicAdd(a.red + rep_slot() * 2 * a.C + (tid < C ? c0 + tid : a.C + c0 + tid - C), (double)sRed[tid]);
  if (a.gW)
    for (int i = tid; i < C * KK; i += 256) atomicAdd(a.gW + (size_t)rep_slot() * a.gstride + c0 * KK + i, sGW[i]);
  KSTAMP(5);
}

template <int K, int DIL, int S, bool PREBN, int C>
__global__ void __launch_bounds__(256) dw_bwd_plane_kernel(DwBwdBatch bt, int nb, int dbg) {
  dw_bwd_plane_body<K, DIL, S, PREBN, C>(bt.e[blockIdx.y], blockIdx.x, nb, dbg);
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// Mixed-variant depthwise backward: one launch for entries of different kernel size / dilation /
// stride / input BN that write DISTINCT outputs - a node's separable second stages (3x3 and 5x5,
// input BN), or a node's stage-1 separable and dilated convolutions each writing its own
// (masked) input-gradient buffer that the pool backward then sums into gx. Each entry carries
// its variant (dw_bwd_variant), band count and workgroup count.
#define DWB_CASE(KK, DD, SS, PB) \
  case dw_bwd_variant(KK, DD, SS, PB): dw_bwd_plane_body<KK, DD, SS, PB, C>(a, blockIdx.x, a.nbands, 0); break;
template <int C>
__global__ void __launch_bounds__(256) dw_bwd_plane_multi_kernel(DwBwdBatch bt) {
  const DwBwdArgs a = bt.e[blockIdx.y];  // copy: see dwpw_plane_multi_kernel
  if ((int)blockIdx.x < a.nblk) {
    switch (a.variant) {
      DWB_CASE(3, 1, 1, true) DWB_CASE(5, 1, 1, true)
      DWB_CASE(3, 1, 1, false) DWB_CASE(3, 1, 2, false) DWB_CASE(5, 1, 1, false) DWB_CASE(5, 1, 2, false)
      DWB_CASE(3, 2, 1, false) DWB_CASE(3, 2, 2, false) DWB_CASE(5, 2, 1, false) DWB_CASE(5, 2, 2, false)
      default: break;
    }
  }
  if (bt.tail.ctr) fold_tail(bt.tail);
}
#undef DWB_CASE

// ------------------------------------------------------------------------------------------------
// edge_bwd: the whole input gradient of one edge in one pass (cf. dw_bwd_plane_kernel, whose band
// layout it shares). Workgroup = (image, band of input rows, C-channel group); act = relu(x) of
// the band is staged once and the gradient is accumulated in LDS:
//   conv slots (sep 3x3 / 5x5 stage 1, dil 3x3 / 5x5): dd of the slot staged with its halo, the
//     transposed depthwise gather added to sGX, the slot's depthwise weight gradient reduced in
//     LDS and flushed with one atomic per weight (replica rep_slot());
//   pools: dz_avg / window count and dz_max (BN backward on the fly from the combine reductions)
//     of the output rows the band reaches, plus the argmax taps, staged and gathered;
//   identity: w_id * dout.
// gx = relu'(x) * conv + pool + identity, written (or added) once per element. Replaces the
// per-(K, S) dw_bwd launches, the pool backward and the identity add of a node: 4-10 launches
// that each re-read and re-wrote gx.
// ------------------------------------------------------------------------------------------------
template <int K, int DIL, int S, int C>
__device__ __forceinline__ void edge_conv_part(const EdgeBwdArgs& a, const int v, const int n, const int c0,
                                               const int iy0, const int nrow, float* sDD, const float* sAct,
                                               float* sGX, float* sGW) {
  constexpr int KK = K * K, PAD = (K - 1) / 2 * DIL, PO = (PAD + S - 1) / S, SH = S == 2 ? 1 : 0;
  const int W = a.W, Ho = a.Ho, Wo = a.Wo, NP = nrow * W;
  const int oyA = (iy0 - PAD) >> SH, oyB = (iy0 + nrow - 1 + PAD) >> SH;
  const int ODR = oyB - oyA + 1, ODW = Wo + 2 * PO;
  const int tid = threadIdx.x;
  const float* ddn = a.dd[v] + ((size_t)n * a.C + c0) * Ho * Wo;
  const int va = max(oyA, 0), vb = min(oyB, Ho - 1), vrows = vb - va + 1;
  {
    const int q4 = vrows * Wo / 4;
#pragma unroll 4
    for (int i = tid; i < C * q4; i += 256) {
      const int c = i / q4, o = (i - c * q4) * 4, r = o / Wo, ox = o - r * Wo;
      const float4 f = *reinterpret_cast<const float4*>(ddn + ((size_t)c * Ho + va) * Wo + o);
      float* d = sDD + (c * ODR + va - oyA + r) * ODW + PO + ox;
      d[0] = f.x;
      d[1] = f.y;
      d[2] = f.z;
      d[3] = f.w;
    }
    for (int i = tid; i < C * ODR; i += 256) {
      const int c = i / ODR, oy = oyA + i - c * ODR;
      float* d = sDD + i * ODW;
      if (oy < 0 || oy >= Ho) {
        for (int q = 0; q < ODW; ++q) d[q] = 0.f;
      } else {
        for (int q = 0; q < PO; ++q) d[q] = d[PO + Wo + q] = 0.f;
      }
    }
    for (int i = tid; i < C * KK; i += 256) sGW[i] = 0.f;
  }
  __syncthreads();
  for (int p = tid; p < NP; p += 256) {
    const int r = p / W, ix = p - r * W, iy = iy0 + r;
    int srow[K], scol[K];
    float mrow[K], mcol[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int t = iy + PAD - k * DIL, u = ix + PAD - k * DIL;
      srow[k] = ((t >> SH) - oyA) * ODW;
      scol[k] = (u >> SH) + PO;
      mrow[k] = (S == 1 || (t & 1) == 0) ? 1.f : 0.f;
      mcol[k] = (S == 1 || (u & 1) == 0) ? 1.f : 0.f;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float* wk = a.dw[v] + (c0 + c) * KK;  // uniform -> scalar loads
      const float* dd = sDD + c * ODR * ODW;
      float ga = 0.f;
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        float rowacc = 0.f;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const float t = wk[ky * K + kx] * dd[srow[ky] + scol[kx]];
          rowacc += S == 1 ? t : mcol[kx] * t;
        }
        ga += S == 1 ? rowacc : mrow[ky] * rowacc;
      }
      sGX[c * NP + p] += ga;  // own pixel: no other thread touches it
    }
  }
  if (a.gW[v]) {
    if (S == 1) {
      // job = (channel, ky, own row): 4-pixel input quads against the dd row segment they meet
      const int JB = C * K * nrow;
      for (int j = tid; j < JB; j += 256) {
        const int c = j / (K * nrow), rem = j - c * K * nrow, ky = rem / nrow, r = rem - ky * nrow;
        const float* ddr = sDD + (c * ODR + iy0 + r + PAD - ky * DIL - oyA) * ODW + PO;
        const float* inr = sAct + c * NP + r * W;
        float acc[K];
#pragma unroll
        for (int kx = 0; kx < K; ++kx) acc[kx] = 0.f;
        for (int ix = 0; ix < W; ix += 4) {
          const float4 f = *reinterpret_cast<const float4*>(inr + ix);
          float dseg[4 + 2 * PAD];
#pragma unroll
          for (int m = 0; m < 4 + 2 * PAD; ++m) dseg[m] = ddr[ix - PAD + m];
#pragma unroll
          for (int kx = 0; kx < K; ++kx) {
            const int o = 2 * PAD - kx * DIL;
            acc[kx] += f.x * dseg[o] + f.y * dseg[o + 1] + f.z * dseg[o + 2] + f.w * dseg[o + 3];
          }
        }
#pragma unroll
        for (int kx = 0; kx < K; ++kx) atomicAdd(sGW + c * KK + ky * K + kx, acc[kx]);
      }
    } else {
      constexpr int JOBS = C * KK, T = JOBS >= 256 ? 1 : 256 / JOBS;
      for (int j = tid; j < JOBS * T; j += 256) {
        const int job = j / T, part = j - job * T;
        const int c = job / KK, tap = job - c * KK, ky = tap / K, kx = tap - ky * K;
        const float* dd = sDD + c * ODR * ODW;
        const float* in = sAct + c * NP;
        float acc = 0.f;
        for (int r = 0; r < nrow; ++r) {
          const int t = iy0 + r + PAD - ky * DIL;
          if (t & 1) continue;
          const float* ddr = dd + ((t >> SH) - oyA) * ODW + PO;
          const float* inr = in + r * W;
          for (int ix = part * S + ((PAD - kx * DIL) & 1); ix < W; ix += T * S)
            acc += inr[ix] * ddr[(ix + PAD - kx * DIL) >> SH];
        }
        atomicAdd(sGW + job, acc);
      }
    }
  }
  __syncthreads();
  if (a.gW[v])
    for (int i = tid; i < C * KK; i += 256) atomicAdd(a.gW[v] + (size_t)rep_slot() * a.gstride[v] + c0 * KK + i, sGW[i]);
  __syncthreads();  // sDD / sGW are restaged by the next slot
}

template <int S, int C>
__device__ __forceinline__ void edge_bwd_body(const EdgeBwdArgs& a, const int bx) {
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int G = a.C / C, grp = bx % G, nbx = bx / G, c0 = grp * C;
  const int n = nbx / a.nb, band = nbx - n * a.nb;
  const int nrow = H / a.nb, iy0 = band * nrow, NP = nrow * W;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sAct = smem;           // [C][NP] relu(x)
  float* sGX = sAct + C * NP;   // [C][NP] conv gradient (pre-mask)
  float* sDD = sGX + C * NP;    // staging: one conv slot's dd band, or the pool gradients
  __shared__ float sGW[C * 25];
  __shared__ float sCo[C][10];
  const int tid = threadIdx.x;
  const float* xn = a.x + ((size_t)n * a.C + c0) * H * W;
  {
    const int q4 = NP / 4;
#pragma unroll 4
    for (int i = tid; i < C * q4; i += 256) {
      const int c = i / q4, o = (i - c * q4) * 4;
      float4 f = *reinterpret_cast<const float4*>(xn + ((size_t)c * H + iy0) * W + o);
      f.x = fmaxf(f.x, 0.f);
      f.y = fmaxf(f.y, 0.f);
      f.z = fmaxf(f.z, 0.f);
      f.w = fmaxf(f.w, 0.f);
      *reinterpret_cast<float4*>(sAct + c * NP + o) = f;
      *reinterpret_cast<float4*>(sGX + c * NP + o) = float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const bool pa = a.ga.z != nullptr, pm = a.gm.z != nullptr;
  if (tid < C) {  // pool BN coefficients and softmax weights per channel
    float* co = sCo[tid];
    co[0] = 0.f; co[1] = 1.f; co[2] = 0.f; co[3] = 0.f; co[4] = 0.f; co[5] = 1.f; co[6] = 0.f; co[7] = 0.f;
    if (pa) {
      bn_coeffs(a.ga.bn, c0 + tid, co[0], co[1]);
      gs_means(a.ga, c0 + tid, co[2], co[3]);
    }
    if (pm) {
      bn_coeffs(a.gm.bn, c0 + tid, co[4], co[5]);
      gs_means(a.gm, c0 + tid, co[6], co[7]);
    }
    co[8] = pa && a.ga.w ? a.ga.w[a.ga.widx] : 1.f;
    co[9] = pm && a.gm.w ? a.gm.w[a.gm.widx] : 1.f;
  }
  __syncthreads();
  if (a.conv_mask & 1) edge_conv_part<3, 1, S, C>(a, 0, n, c0, iy0, nrow, sDD, sAct, sGX, sGW);
  if (a.conv_mask & 2) edge_conv_part<5, 1, S, C>(a, 1, n, c0, iy0, nrow, sDD, sAct, sGX, sGW);
  if (a.conv_mask & 4) edge_conv_part<3, 2, S, C>(a, 2, n, c0, iy0, nrow, sDD, sAct, sGX, sGW);
  if (a.conv_mask & 8) edge_conv_part<5, 2, S, C>(a, 3, n, c0, iy0, nrow, sDD, sAct, sGX, sGW);
  // pools: output rows whose 3x3 window (pad 1) touches the band's input rows
  const int poA = max(0, (iy0 - 1 + S - 1) / S), poB = min(Ho - 1, (iy0 + nrow) / S);
  const int PR = poB - poA + 1, PP = PR * Wo;
  float* sGa = sDD;
  float* sGm = sDD + C * PP;
  unsigned char* sArg = reinterpret_cast<unsigned char*>(sDD + 2 * C * PP);
  if (pa || pm) {
    for (int i = tid; i < C * PP; i += 256) {
      const int c = i / PP, o = poA * Wo + (i - c * PP), oy = o / Wo, ox = o - oy * Wo;
      const size_t idx = ((size_t)n * a.C + c0 + c) * Ho * Wo + o;
      const float* co = sCo[c];
      float gav = 0.f, gmv = 0.f;
      unsigned char arg = 255;
      if (pa) {
        const int y0 = max(oy * S - 1, 0), y1 = min(oy * S + 1, H - 1);
        const int x0 = max(ox * S - 1, 0), x1 = min(ox * S + 1, W - 1);
        gav = bn_bwd_val(a.ga, idx, co[0], co[1], co[8], co[2], co[3]) / (float)((y1 - y0 + 1) * (x1 - x0 + 1));
      }
      if (pm) {
        gmv = bn_bwd_val(a.gm, idx, co[4], co[5], co[9], co[6], co[7]);
        arg = a.amax[idx];
      }
      sGa[i] = gav;
      sGm[i] = gmv;
      sArg[i] = arg;
    }
    __syncthreads();
  }
  const float wid = (a.dout_id && a.w && a.id_idx >= 0) ? a.w[a.id_idx] : 0.f;
  for (int p = tid; p < NP; p += 256) {
    const int r = p / W, ix = p - r * W, iy = iy0 + r;
    const int oy_lo = iy - 1 < 0 ? 0 : (iy - 1 + S - 1) / S, oy_hi = min((iy + 1) / S, Ho - 1);
    const int ox_lo = ix - 1 < 0 ? 0 : (ix - 1 + S - 1) / S, ox_hi = min((ix + 1) / S, Wo - 1);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float g = sAct[c * NP + p] > 0.f ? sGX[c * NP + p] : 0.f;
      if (pa || pm) {
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
          for (int ox = ox_lo; ox <= ox_hi; ++ox) {
            const int o = c * PP + (oy - poA) * Wo + ox;
            g += sGa[o];
            if (sArg[o] == (iy - oy * S + 1) * 3 + (ix - ox * S + 1)) g += sGm[o];
          }
      }
      const size_t gi = ((size_t)n * a.C + c0 + c) * H * W + (size_t)iy * W + ix;
      if (a.dout_id) g += wid * a.dout_id[gi];
      a.gx[gi] = a.overwrite ? g : a.gx[gi] + g;
    }
  }
}

template <int C>
__global__ void __launch_bounds__(256) edge_bwd_kernel(EdgeBwdBatch bt) {
  const EdgeBwdArgs a = bt.e[blockIdx.y];  // copy: see dwpw_plane_multi_kernel
  if ((int)blockIdx.x >= a.nblk) return;
  if (a.S == 1) edge_bwd_body<1, C>(a, blockIdx.x);
  else edge_bwd_body<2, C>(a, blockIdx.x);
}

// LDS floats of one edge_bwd band: act + gradient planes, then the larger of the widest conv
// slot's staged dd band and the pool staging
static size_t edge_bwd_floats(const EdgeBwdArgs& a, int nb, int CG) {
  const int nrow = a.H / nb, S = a.S, sh = S == 2 ? 1 : 0;
  auto fdiv = [sh](int v) { return v >= 0 ? v >> sh : -((-v + (1 << sh) - 1) >> sh); };
  size_t stage = 0;
  const int pads[4] = {1, 2, 2, 4};
  for (int v = 0; v < 4; ++v) {
    if (!(a.conv_mask & (1 << v))) continue;
    const int PAD = pads[v], PO = (PAD + S - 1) / S;
    const int ODR = fdiv(nrow - 1 + PAD) - fdiv(-PAD) + 2;
    stage = std::max(stage, (size_t)CG * ODR * (a.Wo + 2 * PO));
  }
  if (a.ga.z || a.gm.z) {
    const size_t PP = (size_t)(nrow / S + 3) * a.Wo;
    stage = std::max(stage, 2 * CG * PP + (CG * PP + 3) / 4);
  }
  return 2 * (size_t)CG * nrow * a.W + stage;
}

bool launch_edge_bwd(EdgeBwdBatch b, hipStream_t st) {
  if (b.n < 1) return true;
  const int C = b.e[0].C, N = b.e[0].N;
  if (!(C == 4 || (C % 8 == 0 && C <= kMaxC))) return false;
  const int CG = C == 4 ? 4 : 8, G = C / CG;
  int maxblk = 0;
  size_t lds = 0;
  for (int i = 0; i < b.n; ++i) {
    EdgeBwdArgs& a = b.e[i];
    if (a.C != C || a.N != N || a.H != a.Ho * a.S || a.W != a.Wo * a.S || a.W % 4 || a.Wo % 4) return false;
    uintptr_t bits = (uintptr_t)a.x;
    for (int v = 0; v < 4; ++v)
      if (a.conv_mask & (1 << v)) bits |= (uintptr_t)a.dd[v];
    if (bits & 15) return false;
    // bands: LDS per workgroup <= lds_kb and >= min_wg workgroups per launch
    constexpr int lds_kb = 48;
    constexpr int min_wg = 1024;
    int nb = 1;
    while (nb < 32 && a.H % (2 * nb) == 0 &&
           (edge_bwd_floats(a, nb, CG) * 4 > (size_t)lds_kb * 1024 || N * nb * G * b.n < min_wg))
      nb *= 2;
    if (edge_bwd_floats(a, nb, CG) * 4 > 64 * 1024) return false;
    a.nb = nb;
    a.nblk = N * nb * G;
    maxblk = std::max(maxblk, a.nblk);
    lds = std::max(lds, edge_bwd_floats(a, nb, CG) * sizeof(float));
  }
  const dim3 grid(maxblk, b.n);
  if (CG == 4) hipLaunchKernelGGL(edge_bwd_kernel<4>, grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL(edge_bwd_kernel<8>, grid, dim3(256), lds, st, b);
  return true;
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
void launch_pool_bwd_multi(const PoolBwdBatch& b, hipStream_t st) {
  int maxblk = 0;
  size_t lds = 0;
  bool v4 = true;
  auto al = [](const void* p, uintptr_t m) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & (m - 1)) == 0; };
  for (int i = 0; i < b.n; ++i) {
    const PoolBwdArgs& a = b.e[i];
    maxblk = std::max(maxblk, a.N * a.C);
    lds = std::max(lds, sizeof(float) * 2 * a.Ho * a.Wo + a.Ho * a.Wo + 16);
    v4 = v4 && (a.Ho * a.Wo) % 4 == 0 && (a.H * a.W) % 4 == 0 && a.W % 4 == 0 && al(a.ga.g, 16) && al(a.gm.g, 16) &&
         al(a.ga.z, 4 * sizeof(zt)) && al(a.gm.z, 4 * sizeof(zt)) && al(a.amax, 4) && al(a.dout_id, 16) &&
         al(a.gx, 16) && (!a.ga.z || !a.gm.z || a.ga.g == a.gm.g);
    for (int j = 0; j < a.nextra; ++j) v4 = v4 && al(a.extra[j], 16);
  }
  KSTAMP_ARM(kStampPoolBwd, st)
  if (v4) hipLaunchKernelGGL(pool_bwd_multi_kernel<true>, dim3(maxblk, b.n), dim3(256), lds, st, b);
  else hipLaunchKernelGGL(pool_bwd_multi_kernel<false>, dim3(maxblk, b.n), dim3(256), lds, st, b);
  KSTAMP_DISARM(st)
}

// LDS floats of one dw_bwd_plane band (nb bands per image)
static size_t dw_plane_floats(const DwBwdArgs& a, int K, int DIL, int S, int nb, bool accum, int C) {
  const int PAD = (K - 1) / 2 * DIL, PO = (PAD + S - 1) / S, sh = S == 2 ? 1 : 0, BRi = a.H / nb;
  auto fdiv = [sh](int v) { return v >= 0 ? v >> sh : -((-v + (1 << sh) - 1) >> sh); };
  const int ODR = fdiv(BRi - 1 + PAD) - fdiv(-PAD) + 2;  // +1: odd bands start at odd rows
  return (size_t)dwb_head_floats(C) + (size_t)C * ODR * lds_pitch(a.Wo + 2 * PO) +
         (size_t)C * BRi * a.W * (accum ? 2 : 1);
}

template <int K, int DIL, int S, int C>
static void launch_dw_bwd_plane_t(const DwBwdBatch& b, bool prebn, hipStream_t st) {
  const DwBwdArgs& a = b.e[0];
  bool accum = false;
  for (int i = 0; i < b.n; ++i) accum |= !prebn && !b.e[i].overwrite;
  // bands: as few as possible (less halo) while the launch still has ~4 workgroups per CU and a
  // band stays within 40 KB of LDS
  int nb = 1;
  const int G = a.C / C;  // channel groups per image
  while (nb < 8 && a.H % (2 * nb) == 0 &&
         (dw_plane_floats(a, K, DIL, S, nb, accum, C) * 4 > 40 * 1024 || a.N * nb * G * b.n < 1024))
    nb *= 2;
  const size_t lds = sizeof(float) * dw_plane_floats(a, K, DIL, S, nb, accum, C);
  dim3 grid(a.N * nb * G, b.n);
  constexpr int dbg = 0;  // timing probes
  if (prebn) hipLaunchKernelGGL((dw_bwd_plane_kernel<K, DIL, S, true, C>), grid, dim3(256), lds, st, b, nb, dbg);
  else hipLaunchKernelGGL((dw_bwd_plane_kernel<K, DIL, S, false, C>), grid, dim3(256), lds, st, b, nb, dbg);
}

static bool aligned16(const DwBwdBatch& b) {
  for (int i = 0; i < b.n; ++i)
    if (((uintptr_t)b.e[i].x | (uintptr_t)b.e[i].dd | (uintptr_t)b.e[i].gout) & 15) return false;
  return true;
}

// plane path: narrow layers whose spatial sizes divide exactly by the stride
static bool dw_plane_ok(const DwBwdBatch& b, int K, int DIL, int S) {
  const DwBwdArgs& a = b.e[0];
  return (a.C == 4 || a.C == 8 || (a.C % 16 == 0 && a.C <= kMaxC)) && a.H == a.Ho * S && a.W == a.Wo * S &&
         a.pad == (K - 1) / 2 * DIL && a.Wo % 4 == 0 && aligned16(b);
}

template <int K, int DIL, int S>
static void launch_dw_bwd_t(const DwBwdBatch& b, bool prebn, hipStream_t st) {
  const DwBwdArgs& a = b.e[0];
  if (dw_plane_ok(b, K, DIL, S)) {
    // wide layers run in channel groups of grp (4, 8 or 16) channels: 8 measured
    // 48.2 vs 50.8 ms per darts-gpu.yaml step against 16 (half the LDS per band: fewer, taller bands),
    // and 4 beats 8 on the round-4 kernels (B5 6.37 vs 6.44 ms, default 41.98 vs 42.20 ms,
    // profiles/darts_dwb_group_ab_r04.log)
    constexpr int grp = 4;
    if (a.C == 4 || grp == 4) return launch_dw_bwd_plane_t<K, DIL, S, 4>(b, prebn, st);
    if (a.C == 8 || grp == 8) return launch_dw_bwd_plane_t<K, DIL, S, 8>(b, prebn, st);
    return launch_dw_bwd_plane_t<K, DIL, S, 16>(b, prebn, st);
  }
  const int TR = 64 / a.Wo;
  const int r = (K - 1) / 2 * DIL, h = (r + S - 1) / S, OR = TR + 2 * h;
  const int IR = (TR - 1) * S + (K - 1) * DIL + 1;
  const int IW = (a.Wo - 1) * S + (K - 1) * DIL + 1;
  size_t lds = sizeof(float) * (a.chunk * OR * a.Wo + a.chunk * IR * IW + 4 * a.C + (a.gW ? a.C * K * K : 0));
  dim3 grid(per_edge_blocks(a.N * (a.Ho / TR), b.n), b.n);
  if (prebn) hipLaunchKernelGGL((dw_bwd_kernel<K, DIL, S, true>), grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL((dw_bwd_kernel<K, DIL, S, false>), grid, dim3(256), lds, st, b);
}

bool launch_dw_bwd_multi(DwBwdBatch b, hipStream_t st) {
  if (b.n < 1) return true;
  const DwBwdArgs& a0 = b.e[0];
  if (!(a0.C == 4 || a0.C == 8 || (a0.C % 16 == 0 && a0.C <= kMaxC)) || !aligned16(b)) return false;
  constexpr int grp = 4;
  const int C = (a0.C == 4 || grp == 4) ? 4 : 8;  // channel groups as launch_dw_bwd_t
  if (a0.C % C) return false;
  int maxblk = 0;
  size_t lds = 0;
  for (int i = 0; i < b.n; ++i) {
    DwBwdArgs& a = b.e[i];
    const int K = dw_variant_k(a.variant), DIL = dw_variant_dil(a.variant), S = dw_variant_s(a.variant);
    const bool prebn = dw_variant_prebn(a.variant);
    // the plane kernel's layout (dw_plane_ok) and an overwriting (never accumulating) input BN-free entry
    if (a.C != a0.C || a.H != a.Ho * S || a.W != a.Wo * S || a.pad != (K - 1) / 2 * DIL || a.Wo % 4 ||
        (prebn && (DIL != 1 || S != 1)) || (!prebn && !a.overwrite))
      return false;
    int nb = 1;
    const int G = a.C / C;
    constexpr int min_wg = 512;
    while (nb < 8 && a.H % (2 * nb) == 0 &&
           (dw_plane_floats(a, K, DIL, S, nb, false, C) * 4 > 40 * 1024 || a.N * nb * G * b.n < min_wg))
      nb *= 2;
    a.nbands = nb;
    a.nblk = a.N * nb * G;
    a.vin = S == 1 ? (vec_mask() >> (C == 4 ? 2 : 3)) & 1 : (vec_mask() >> 4) & 1;
    maxblk = std::max(maxblk, a.nblk);
    lds = std::max(lds, sizeof(float) * dw_plane_floats(a, K, DIL, S, nb, false, C));
  }
  KSTAMP_ARM(kStampDwBwd, st)
  if (C == 4) hipLaunchKernelGGL(dw_bwd_plane_multi_kernel<4>, dim3(maxblk, b.n), dim3(256), lds, st, b);
  else hipLaunchKernelGGL(dw_bwd_plane_multi_kernel<8>, dim3(maxblk, b.n), dim3(256), lds, st, b);
  KSTAMP_DISARM(st)
  return true;
}

void launch_dw_bwd(const DwBwdBatch& b, int K, int dil, int S, bool prebn, hipStream_t st) {
#define DISPATCH(KK, DD, SS) \
  if (K == KK && dil == DD && S == SS) return launch_dw_bwd_t<KK, DD, SS>(b, prebn, st);
  DISPATCH(3, 1, 1) DISPATCH(3, 1, 2) DISPATCH(5, 1, 1) DISPATCH(5, 1, 2)
  DISPATCH(3, 2, 1) DISPATCH(3, 2, 2) DISPATCH(5, 2, 1) DISPATCH(5, 2, 2)
#undef DISPATCH
}
void launch_pool_bwd(const PoolBwdBatch& b, int S, hipStream_t st) {
  const PoolBwdArgs& a = b.e[0];
  size_t lds = sizeof(float) * 2 * a.Ho * a.Wo + a.Ho * a.Wo + 16;
  dim3 grid(a.N * a.C, b.n);
  if (S == 1) hipLaunchKernelGGL(pool_bwd_kernel<1>, grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL(pool_bwd_kernel<2>, grid, dim3(256), lds, st, b);
}

}  // namespace katib_hip
