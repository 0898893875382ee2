// One-shot all-reduce over xGMI for small / mid-size messages.
//
// MI355X nodes are a full mesh: every GPU has a dedicated xGMI link to each of its 7
// peers. A ring all-reduce walks one link at a time and pays 2(W-1) latency hops; for
// the DARTS gradient vectors (37 KB .. 1.8 MB) that is pure latency. Here every rank
// publishes its input in an IPC-mapped staging buffer and each workgroup reads its slice
// from all W-1 peers at once (all links busy in parallel), summing in rank order so
// every rank produces bit-identical results (DP replicas stay in lockstep).
//
// Synchronisation (no host involvement, HIP-graph capturable):
//  * every rank owns a signal page in uncached device memory; peers write
//    flags[block][src] = epoch into it, the owner polls them;
//  * epoch is a per-block counter kept on the device (flags are monotonic, never reset);
//  * staging is double-buffered by epoch parity, so no closing barrier is needed: block b
//    of rank r enters call k only after every peer's block b signalled call k-1, i.e.
//    after every peer finished call k-2, the last reader of this parity half. This needs
//    the same grid size on every call (fixed at workspace creation);
//  * producer side: stores -> s_waitcnt(0) -> barrier -> system-scope release fence
//    (buffer_wbl2 sc0 sc1: the L2 is not coherent with xGMI readers) -> explicit
//    s_waitcnt(0) (the compiler drops the fence's own wait after a drained counter) ->
//    flag stores (sc0 sc1);
//    consumer side: poll (sc0 sc1 loads) -> barrier -> system-scope acquire
//    (buffer_inv sc0 sc1) -> peer loads;
//  * every wait is bounded by the 100 MHz wall clock; on timeout the kernel raises an
//    error word in its signal page and drains (the host checks it), so a missing peer
//    can never hang the GPU.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "xgmi_allreduce.h"

namespace katib_hip {
namespace xgmi {

namespace {

__device__ inline uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int V>
struct VecT;
template <>
struct VecT<4> {
  using T = float4;
};
template <>
struct VecT<1> {
  using T = float;
};

__device__ inline float4 vadd(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ inline float vadd(float a, float b) { return a + b; }
__device__ inline float4 vscale(float4 a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }
__device__ inline float vscale(float a, float s) { return a * s; }

template <int V>
__global__ __launch_bounds__(kThreads) void oneshot_kernel(AllReduceArgs a) {
  using vec = typename VecT<V>::T;
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  uint32_t* mysig = a.sig[a.rank];
  __shared__ uint32_t s_e;
  if (tid == 0) s_e = ld_sys(mysig + kSigEpoch + b) + 1u;
  __syncthreads();
  const uint32_t e = s_e;
  const int64_t half = (int64_t)(e & 1u) * a.cap;

  // this block's slice, in vectors; the n % V scalar tail belongs to the last block
  const int64_t nv = a.n / V;
  const int64_t per = (nv + nb - 1) / nb;
  const int64_t lo = min(nv, (int64_t)b * per), hi = min(nv, lo + per);
  const int64_t tail0 = nv * V;
  const bool has_tail = (b == nb - 1) && tail0 < a.n;

  // 1. publish my slice
  {
    const vec* in = reinterpret_cast<const vec*>(a.in);
    vec* mine = reinterpret_cast<vec*>(a.buf[a.rank] + half);
    for (int64_t i = lo + tid; i < hi; i += kThreads) mine[i] = in[i];
    if (has_tail && tid < a.n - tail0) a.buf[a.rank][half + tail0 + tid] = a.in[tail0 + tid];
  }
  __builtin_amdgcn_s_waitcnt(0);  // this wave's stores are in L2
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // write L2 back: peers read over xGMI
    __builtin_amdgcn_s_waitcnt(0);                  // ... and wait for the write-back
    for (int p = 0; p < a.world; ++p)
      if (p != a.rank) st_sys(a.sig[p] + b * kMaxRanks + a.rank, e);
  }
  // 2. wait for every peer's block b (bounded)
  if (tid < a.world && tid != a.rank) {
    const uint32_t* f = mysig + b * kMaxRanks + tid;
    const uint64_t t0 = wall_clock64();
    while (ld_sys(f) < e) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        st_sys(mysig + kSigErr, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // drop stale L2/L1 lines of peer buffers

  // 3. sum in rank order (identical bits on every rank)
  {
    const vec* in = reinterpret_cast<const vec*>(a.in);
    vec* out = reinterpret_cast<vec*>(a.out);
    for (int64_t i = lo + tid; i < hi; i += kThreads) {
      vec acc = (a.rank == 0) ? in[i] : reinterpret_cast<const vec*>(a.buf[0] + half)[i];
      for (int p = 1; p < a.world; ++p) {
        const vec v = (p == a.rank) ? in[i] : reinterpret_cast<const vec*>(a.buf[p] + half)[i];
        acc = vadd(acc, v);
      }
      out[i] = vscale(acc, a.scale);
    }
    if (has_tail && tid < a.n - tail0) {
      const int64_t i = tail0 + tid;
      float acc = (a.rank == 0) ? a.in[i] : a.buf[0][half + i];
      for (int p = 1; p < a.world; ++p) acc += (p == a.rank) ? a.in[i] : a.buf[p][half + i];
      a.out[i] = acc * a.scale;
    }
  }
  if (tid == 0) st_sys(mysig + kSigEpoch + b, e);
}

// fold + cross-rank sum of f64 segments (SyncBN), same hand-off protocol as oneshot_kernel
// Small payloads (every SyncBN fold of the B5 supernet: a few hundred doubles) run on block 0 alone: one
// flag per peer instead of one per (block, peer) - the handshake, not the bytes, is the cost there
// (2 / 4 ranks: 4.1 / 5.0 us per rendezvous on 1 workgroup vs 5.9 / 8.7 on 16, profiles/rendezvous_r06.log).
// The other blocks return at once (the decision is the same on every rank: same segments), so their
// epochs do not move; block 0 stages small calls in a region of its own at the top of each half, which
// no multi-block call touches (those are limited to cap / 2 - kSmallFold doubles), so block 0's parity
// alternation protects both regions exactly as in the uniform case.
__global__ __launch_bounds__(kThreads) void fold_sync_kernel(AllReduceArgs a, FoldF64Args f, uint64_t mask) {
  const bool small = f.total <= kSmallFold;
  if (small && blockIdx.x > 0) return;
  const int b = blockIdx.x, nb = small ? 1 : gridDim.x, tid = threadIdx.x;
  uint32_t* mysig = a.sig[a.rank];
  __shared__ uint32_t s_e;
  if (tid == 0) s_e = ld_sys(mysig + kSigEpoch + b) + 1u;
  __syncthreads();
  const uint32_t e = s_e;
  const int64_t half = (int64_t)(e & 1u) * (a.cap / 2) + (small ? a.cap / 2 - kSmallFold : 0);  // in doubles
  const int per = (f.total + nb - 1) / nb;
  const int lo = min(f.total, b * per), hi = min(f.total, lo + per);
  double* mine = reinterpret_cast<double*>(a.buf[a.rank]) + half;

  // 1. fold my slice: local segments are final, synchronised ones are published
  for (int g = lo + tid; g < hi; g += kThreads) {
    int seg = 0, i = g;
    while (seg < f.nseg - 1 && i >= f.n[seg]) i -= f.n[seg++];
    double* p = f.p[seg] + i;
    const int rs = f.rstride[seg];
    double v[kRep];
#pragma unroll
    for (int r = 0; r < kRep; ++r) v[r] = p[(size_t)r * rs];
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < kRep; ++r) acc += v[r];
#pragma unroll
    for (int r = 1; r < kRep; ++r) p[(size_t)r * rs] = 0.0;
    if ((mask >> seg) & 1ull) mine[g] = acc;
    else p[0] = acc;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // write L2 back: peers read over xGMI
    __builtin_amdgcn_s_waitcnt(0);
    for (int p = 0; p < a.world; ++p)
      if (p != a.rank) st_sys(a.sig[p] + b * kMaxRanks + a.rank, e);
  }
  // 2. wait for every peer's block b (bounded)
  if (tid < a.world && tid != a.rank) {
    const uint32_t* fl = mysig + b * kMaxRanks + tid;
    const uint64_t t0 = wall_clock64();
    while (ld_sys(fl) < e) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        st_sys(mysig + kSigErr, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  // 3. synchronised segments: sum in rank order into replica 0
  for (int g = lo + tid; g < hi; g += kThreads) {
    int seg = 0, i = g;
    while (seg < f.nseg - 1 && i >= f.n[seg]) i -= f.n[seg++];
    if (!((mask >> seg) & 1ull)) continue;
    double acc = reinterpret_cast<const double*>(a.buf[0])[half + g];
    for (int p = 1; p < a.world; ++p) acc += reinterpret_cast<const double*>(a.buf[p])[half + g];
    f.p[seg][i] = acc;
  }
  if (tid == 0) st_sys(mysig + kSigEpoch + b, e);
}

}  // namespace

hipError_t launch_fold_sync(const AllReduceArgs& a, const FoldF64Args& f, uint64_t sync_mask, int blocks,
                            hipStream_t stream) {
  hipLaunchKernelGGL(fold_sync_kernel, dim3(blocks), dim3(kThreads), 0, stream, a, f, sync_mask);
  return hipGetLastError();
}

hipError_t launch_oneshot(const AllReduceArgs& a, int blocks, bool vec4, hipStream_t stream) {
  if (vec4)
    hipLaunchKernelGGL(oneshot_kernel<4>, dim3(blocks), dim3(kThreads), 0, stream, a);
  else
    hipLaunchKernelGGL(oneshot_kernel<1>, dim3(blocks), dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace xgmi
}  // namespace katib_hip
