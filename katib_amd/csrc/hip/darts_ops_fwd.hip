// DARTS forward edge kernels: dw-pw stages (plane / tile / split), pointwise StdConv / FactorizedReduce
// (pw_fwd, pw_fwd_wave), avg + max pooling - launch heuristics and the single-variant instantiations.
// Kernel templates: darts_ops_fwd_k.h. See darts_ops.hip for the design notes.
#include "darts_ops_fwd_k.h"

namespace katib_hip {


template <int K, int DIL, int S, int C>
static void launch_dwpw_plane_t(const DwPwFwdBatch& b, bool prebn, hipStream_t st) {
  const DwPwFwdArgs& a = b.e[0];
  const int nb = a.chunk, BR = (a.Ho + nb - 1) / nb;
  const size_t lds = sizeof(float) * (plane_head_floats(C) + C * ((BR - 1) * S + (K - 1) * DIL + 1) * lds_pitch(a.W + 2 * a.pad));
  dim3 grid(a.N * nb, b.n);
  // 16-byte staging when every row is whole float4s and every input is 16-byte aligned
  bool vec = a.W % 4 == 0;
  for (int i = 0; i < b.n; ++i) vec &= ((uintptr_t)b.e[i].x & 15) == 0;
  if (vec) {
    if (prebn) hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, true, C, true>), grid, dim3(256), lds, st, b);
    else hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, false, C, true>), grid, dim3(256), lds, st, b);
  } else {
    if (prebn) hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, true, C, false>), grid, dim3(256), lds, st, b);
    else hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, false, C, false>), grid, dim3(256), lds, st, b);
  }
}

// row-band kernel for C = 4 / 8 / 16 (the staged band fits 64 KB of LDS by construction)
static bool plane_ok(const DwPwFwdArgs& a) { return a.C == 4 || a.C == 8 || a.C == 16; }

template <int CI, int CO>
static bool try_pw_fwd_wave(const PwFwdBatch& b, hipStream_t st);

template <int K, int DIL, int S, int CG>
static bool try_dwpw_split_g(const DwPwFwdBatch& b, bool prebn, hipStream_t st, bool split16);

// layers of 16..64 channels: depthwise on channel groups (dwpw_plane_kernel<..., PW = false>), then
// the pointwise + BN statistics as an MFMA GEMM over d (pw_fwd_wave_kernel). At C = 16 this measured
// faster than the fused plane kernel (50.7 vs 52.5 ms per darts-gpu.yaml step); the fused form
// keeps the fused kernel there.
template <int K, int DIL, int S>
static bool try_dwpw_split(const DwPwFwdBatch& b, bool prebn, hipStream_t st) {
  const DwPwFwdArgs& a = b.e[0];
  constexpr bool split16 = true;
  constexpr int grp = 8;
  if (grp == 4) return try_dwpw_split_g<K, DIL, S, 4>(b, prebn, st, split16);
  if (grp == 8) return try_dwpw_split_g<K, DIL, S, 8>(b, prebn, st, split16);
  return try_dwpw_split_g<K, DIL, S, 16>(b, prebn, st, split16);
}

template <int K, int DIL, int S, int CG>
static bool try_dwpw_split_g(const DwPwFwdBatch& b, bool prebn, hipStream_t st, bool split16) {
  const DwPwFwdArgs& a = b.e[0];
  if (a.C % 16 != 0 || a.C > 64 || (a.C == 16 && !split16) ||
      (a.Ho * a.Wo) % 64 != 0 || a.W % 4 != 0)
    return false;
  for (int i = 0; i < b.n; ++i)
    if (((uintptr_t)b.e[i].x | (uintptr_t)b.e[i].d | (uintptr_t)b.e[i].z) & 15) return false;
  const int G = a.C / CG;
  int nb = std::max(1, std::min(a.Ho / 4, 2048 / std::max(a.N * b.n * G, 1)));
  auto band_bytes = [&](int v) {
    const int BR = (a.Ho + v - 1) / v;
    return ((size_t)plane_head_floats(CG) + (size_t)CG * ((BR - 1) * S + (K - 1) * DIL + 1) * lds_pitch(a.W + 2 * a.pad)) * sizeof(float);
  };
  while (band_bytes(nb) > 65536 && nb < a.Ho) ++nb;
  DwPwFwdBatch db = b;
  db.tail.ctr = nullptr;  // the statistics come from the pointwise launch below, which folds them
  for (int i = 0; i < b.n; ++i) db.e[i].chunk = nb;
  dim3 grid(a.N * nb * G, b.n);
  const size_t lds = band_bytes(nb);
  if (prebn) hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, true, CG, true, false>), grid, dim3(256), lds, st, db);
  else hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, false, CG, true, false>), grid, dim3(256), lds, st, db);
  PwFwdBatch pb{};
  pb.n = b.n;
  pb.tail = b.tail;
  for (int i = 0; i < b.n; ++i) {
    const DwPwFwdArgs& e = b.e[i];
    PwFwdArgs& p = pb.e[i];
    p.x = e.d; p.pw = e.pw; p.z = e.z; p.stats = e.stats;
    p.N = e.N; p.Cin = e.C; p.Cout = e.C; p.CoutTotal = e.C; p.co_off = 0;
    p.H = e.Ho; p.W = e.Wo; p.Ho = e.Ho; p.Wo = e.Wo; p.S = 1; p.off = 0; p.relu = 0;
  }
  if (try_pw_fwd_wave<16, 16>(pb, st) || try_pw_fwd_wave<32, 32>(pb, st) || try_pw_fwd_wave<64, 64>(pb, st))
    return true;
  launch_pw_fwd(pb, st);  // C = 48: the generic dispatch
  return true;
}

template <int K, int DIL, int S>
static void launch_dwpw_fwd_t(const DwPwFwdBatch& b, bool prebn, hipStream_t st) {
  const DwPwFwdArgs& a = b.e[0];
  if (try_dwpw_split<K, DIL, S>(b, prebn, st)) return;
  if (plane_ok(a)) {
    if (a.C == 4) return launch_dwpw_plane_t<K, DIL, S, 4>(b, prebn, st);
    if (a.C == 8) return launch_dwpw_plane_t<K, DIL, S, 8>(b, prebn, st);
    return launch_dwpw_plane_t<K, DIL, S, 16>(b, prebn, st);
  }
  const int TR = 64 / a.Wo;
  const int IR = (TR - 1) * S + (K - 1) * DIL + 1;
  const int IW = (a.Wo - 1) * S + (K - 1) * DIL + 1;
  size_t lds = sizeof(float) * (a.C * 64 + a.chunk * IR * IW + 4 * a.C);
  dim3 grid(per_edge_blocks(a.N * (a.Ho / TR), b.n), b.n);
  if (prebn) hipLaunchKernelGGL((dwpw_fwd_kernel<K, DIL, S, true>), grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL((dwpw_fwd_kernel<K, DIL, S, false>), grid, dim3(256), lds, st, b);
}

void launch_dwpw_fwd(const DwPwFwdBatch& b, int K, int dil, int S, bool prebn, hipStream_t st) {
#define DISPATCH(KK, DD, SS) \
  if (K == KK && dil == DD && S == SS) return launch_dwpw_fwd_t<KK, DD, SS>(b, prebn, st);
  DISPATCH(3, 1, 1) DISPATCH(3, 1, 2) DISPATCH(5, 1, 1) DISPATCH(5, 1, 2)
  DISPATCH(3, 2, 1) DISPATCH(3, 2, 2) DISPATCH(5, 2, 1) DISPATCH(5, 2, 2)
#undef DISPATCH
}

// ------------------------------------------------------------------------------------------------
// Mixed-variant launches (one per node stage instead of one per (K, dil, S) group). The entries
// must share the channel count; returns false (nothing launched) when they do not fit the plane
// kernels, and the caller falls back to the per-group launches.
// ------------------------------------------------------------------------------------------------

// per-entry band counts / variants of a dw-pw multi batch; false: the entries do not fit the plane kernels
static bool dwpw_multi_prep(DwPwMultiBatch& b, bool& fused, int& maxblk, size_t& lds) {
  const int C = b.e[0].C, N = b.e[0].N;
  constexpr bool split16 = true;
  fused = C == 4 || C == 8 || (C == 16 && !split16);
  const bool split = !fused && C % 16 == 0 && C <= 64;
  if (!fused && !split) return false;
  const int CG = fused ? C : 8, G = C / CG;
  maxblk = 0;
  lds = 0;
  for (int i = 0; i < b.n; ++i) {
    DwPwFwdArgs& a = b.e[i];
    if (a.C != C || a.N != N) return false;
    const int code = a.variant >> 2;
    const int K = (code & 4) ? 5 : 3, DIL = (code & 2) ? 2 : 1, S = (code & 1) ? 2 : 1;
    const bool aligned = ((((uintptr_t)a.x) | (uintptr_t)a.d | (uintptr_t)a.z) & 15) == 0;
    if (split && (!aligned || (a.Ho * a.Wo) % 64 != 0 || a.W % 4 != 0)) return false;
    int nb = std::max(1, std::min(a.Ho / 4, 512 / std::max(N * b.n * G, 1)));
    auto band_bytes = [&](int v) {
      const int BR = (a.Ho + v - 1) / v;
      return ((size_t)plane_head_floats(CG) + (size_t)CG * ((BR - 1) * S + (K - 1) * DIL + 1) * lds_pitch(a.W + 2 * a.pad)) * sizeof(float);
    };
    while (band_bytes(nb) > 65536 && nb < a.Ho) ++nb;
    a.chunk = nb;
    a.nblk = N * nb * G;
    const bool vec = a.W % 4 == 0 && (((uintptr_t)a.x) & 15) == 0;
    a.variant = (a.variant & ~1) | (vec ? 1 : 0);
    a.vout = (vec_mask() >> (CG == 4 ? 0 : 1)) & 1;
    maxblk = std::max(maxblk, a.nblk);
    lds = std::max(lds, band_bytes(nb));
  }
  return true;
}

bool launch_dwpw_multi(DwPwMultiBatch b, hipStream_t st) {
  if (b.n < 1) return true;
  const int C = b.e[0].C;
  bool fused;
  int maxblk;
  size_t lds;
  if (!dwpw_multi_prep(b, fused, maxblk, lds)) return false;
  const dim3 grid(maxblk, b.n);
  if (fused) {
    // (phase stamps: armed in the launching translation unit, darts_ops_fwd_m{4,8,16}.hip)
    if (C == 4) launch_dwpw_plane_multi_t<4>(true, grid, lds, st, b);
    else if (C == 8) launch_dwpw_plane_multi_t<8>(true, grid, lds, st, b);
    else launch_dwpw_plane_multi_t<16>(true, grid, lds, st, b);
    return true;
  }
  {
    DwPwMultiBatch db = b;
    db.tail.ctr = nullptr;  // statistics (and their fold) come from the pointwise launch
    launch_dwpw_plane_multi_t<8>(false, grid, lds, st, db);
  }
  // the pointwise halves + BN statistics of every entry: one MFMA wave launch
  PwFwdBatch pb{};
  pb.n = b.n;
  pb.tail = b.tail;  // per-entry launches below share the counter: they run one after another
  for (int i = 0; i < b.n; ++i) {
    const DwPwFwdArgs& e = b.e[i];
    PwFwdArgs& p = pb.e[i];
    p.x = e.d; p.pw = e.pw; p.z = e.z; p.stats = e.stats;
    p.N = e.N; p.Cin = e.C; p.Cout = e.C; p.CoutTotal = e.C; p.co_off = 0;
    p.H = e.Ho; p.W = e.Wo; p.Ho = e.Ho; p.Wo = e.Wo; p.S = 1; p.off = 0; p.relu = 0;
  }
  bool same_hw = true;
  for (int i = 1; i < b.n; ++i) same_hw &= b.e[i].Ho == b.e[0].Ho && b.e[i].Wo == b.e[0].Wo;
  if (same_hw && (try_pw_fwd_wave<16, 16>(pb, st) || try_pw_fwd_wave<32, 32>(pb, st) || try_pw_fwd_wave<64, 64>(pb, st)))
    return true;
  for (int i = 0; i < b.n; ++i) {  // mixed output sizes (stride-1 and stride-2 entries): per entry
    PwFwdBatch one{};
    one.n = 1;
    one.tail = pb.tail;
    one.e[0] = pb.e[i];
    if (!(try_pw_fwd_wave<16, 16>(one, st) || try_pw_fwd_wave<32, 32>(one, st) || try_pw_fwd_wave<64, 64>(one, st)))
      launch_pw_fwd(one, st);
  }
  return true;
}

// workgroups per pool entry, and whether the LDS-staged 4-pixel path applies (lds: its plane bytes)
static bool pool_fwd_prep(PoolFwdArgs* e, int n, int& maxblk, size_t& lds) {
  // 4 outputs per thread from a register window loaded straight from global memory (round 6; the
  // round-4 LDS-staged form was slower: a barrier round trip per staged plane, 42 -> 68 us per call
  // on the darts-gpu.yaml step, profiles/darts_default_ab_r04.log)
  bool v4 = true;
  auto al = [](const void* p, uintptr_t m) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & (m - 1)) == 0; };
  maxblk = 0;
  lds = 0;
  for (int i = 0; i < n; ++i) {
    PoolFwdArgs& a = e[i];
    a.nblk = a.C * channel_groups(a.N, a.C, n);
    maxblk = std::max(maxblk, a.nblk);
    v4 = v4 && a.W % 4 == 0 && a.Wo % 4 == 0 && (a.S == 1 || a.W == 2 * a.Wo) && al(a.x, 16) &&
         al(a.zavg, 4 * sizeof(zt)) && al(a.zmax, 4 * sizeof(zt)) && al(a.amax, 4);
  }
  return v4;
}

void launch_pool_fwd_multi(PoolFwdBatch b, hipStream_t st) {
  int maxblk;
  size_t lds;
  if (pool_fwd_prep(b.e, b.n, maxblk, lds))
    hipLaunchKernelGGL(pool_fwd_multi_kernel<true>, dim3(maxblk, b.n), dim3(256), lds, st, b);
  else hipLaunchKernelGGL(pool_fwd_multi_kernel<false>, dim3(maxblk, b.n), dim3(256), 0, st, b);
}

bool launch_dwpw_pool_multi(DwPwMultiBatch b, const PoolFwdBatch& pb, hipStream_t st) {
  constexpr bool off = false;
  if (off || b.n < 1 || pb.n < 1 || b.tail.ctr || pb.tail.ctr || b.n + pb.n > 65535) return false;
  const int C = b.e[0].C;
  bool fused;
  int maxblk;
  size_t lds;
  if (!dwpw_multi_prep(b, fused, maxblk, lds) || !fused || (C != 4 && C != 8)) return false;
  PoolFwdEntries pe{};
  pe.n = pb.n;
  for (int i = 0; i < pb.n; ++i) pe.e[i] = pb.e[i];
  int pblk;
  size_t plds;
  if (!pool_fwd_prep(pe.e, pe.n, pblk, plds)) return false;  // the joint kernel carries the 4-pixel pool only
  const dim3 grid(std::max(maxblk, pblk), b.n + pb.n);
  lds = std::max(lds, plds);
  if (C == 4) launch_dwpw_pool_t<4>(grid, lds, st, b, pe);
  else launch_dwpw_pool_t<8>(grid, lds, st, b, pe);
  return true;
}

template <int CI, int CO>
static bool try_pw_fwd_wave(const PwFwdBatch& b, hipStream_t st) {
  const PwFwdArgs& a = b.e[0];
  constexpr int BO = CO / 16;
  if (a.Cin != CI || a.Cout != CO || (a.Ho * a.Wo) % 64 != 0) return false;
  for (int e = 0; e < b.n; ++e) {  // 16-byte loads (flat input) and stores
    const PwFwdArgs& x = b.e[e];
    const bool flat = !x.relu || (x.S == 1 && x.off == 0 && x.H == x.Ho && x.W == x.Wo);
    if ((((uintptr_t)x.z) | (flat ? (uintptr_t)x.x : 0)) & 15) return false;
  }
  const int chunks = a.N * a.Ho * a.Wo / 64;
  // split the output channels over waves while the launch has fewer than ~4 waves per SIMD
  int ns = 1;
  while (BO % (2 * ns) == 0 && chunks * ns * b.n < 4096) ns *= 2;
  const int per_edge = std::max(1, std::min((chunks * ns + 3) / 4, max_blocks() / std::max(b.n, 1)));
  const dim3 grid(per_edge, b.n);
  if (ns == 1) hipLaunchKernelGGL((pw_fwd_wave_kernel<CI, CO, 1>), grid, dim3(256), 0, st, b);
  else if constexpr (BO % 2 == 0) {
    if (ns == 2) hipLaunchKernelGGL((pw_fwd_wave_kernel<CI, CO, 2>), grid, dim3(256), 0, st, b);
    else if constexpr (BO % 4 == 0) hipLaunchKernelGGL((pw_fwd_wave_kernel<CI, CO, 4>), grid, dim3(256), 0, st, b);
  }
  return true;
}

void launch_pw_fwd(const PwFwdBatch& b, hipStream_t st) {
  const PwFwdArgs& a = b.e[0];
  // (narrow layers stay on the 64-pixel tiles below: a pixel-quad-per-thread kernel had too few
  // waves at B5 sizes - 32-128 workgroups - and measured 333 vs 281 us per step,
  // profiles/darts_vec_ab_r04.log)
  if (try_pw_fwd_wave<48, 16>(b, st) || try_pw_fwd_wave<48, 32>(b, st) || try_pw_fwd_wave<64, 32>(b, st) ||
      try_pw_fwd_wave<32, 16>(b, st) || try_pw_fwd_wave<16, 16>(b, st) || try_pw_fwd_wave<32, 32>(b, st) ||
      try_pw_fwd_wave<64, 64>(b, st) || try_pw_fwd_wave<128, 64>(b, st))  // 128 -> 64: last-cell preprocess
    return;
  size_t lds = sizeof(float) * (a.Cin * 64 + 2 * a.Cout);
  dim3 grid(per_edge_blocks(a.N * a.Ho * a.Wo / 64, b.n), b.n);
  hipLaunchKernelGGL(pw_fwd_kernel, grid, dim3(256), lds, st, b);
}

void launch_pool_fwd(const PoolFwdBatch& b, int S, hipStream_t st) {
  const PoolFwdArgs& a = b.e[0];
  dim3 grid(a.C * channel_groups(a.N, a.C, b.n), b.n);
  if (S == 1) hipLaunchKernelGGL(pool_fwd_kernel<1>, grid, dim3(256), 0, st, b);
  else hipLaunchKernelGGL(pool_fwd_kernel<2>, grid, dim3(256), 0, st, b);
}

}  // namespace katib_hip
