// Cell-persistent DARTS feasibility probe (VERDICT r03 "next" #2): what does one grid-wide barrier
// inside a persistent cooperative kernel cost on MI355X, against one kernel boundary inside a
// replayed HIP graph -- the two ways a chain of dependent DARTS ops (each a full pass over a
// 0.5-2 MB B5 activation) can be sequenced?
//
//   launch_empty   K empty kernels captured in one graph                    -> us per launch
//   barrier_empty  one cooperative kernel running K grid.sync()s            -> us per barrier
//   launch_pass    K dependent 2 MB y = a x + b passes, one kernel each, in a graph (2048 WGs)
//   coop_pass      the same K passes in one cooperative kernel, grid.sync() between passes
//                  (256 or 512 WGs = 1 or 2 per CU, grid-stride float4 loops)
//   own_barrier / own_pass   the same with a hand-rolled atomic sense-reversal barrier
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/grid_barrier_probe scripts/grid_barrier_probe.hip
// Every wave of the cooperative kernels runs exactly K iterations and reaches every barrier, so the
// grid always drains.
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

namespace cg = cooperative_groups;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

__global__ void empty_kernel() {}

__global__ void pass_kernel(const float4* __restrict__ x, float4* __restrict__ y, int n4, float a, float b) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    float4 v = x[i];
    y[i] = make_float4(a * v.x + b, a * v.y + b, a * v.z + b, a * v.w + b);
  }
}

__global__ void coop_barrier_kernel(int K, float* sink) {
  cg::grid_group g = cg::this_grid();
  for (int k = 0; k < K; ++k) g.sync();
  if (blockIdx.x == 0 && threadIdx.x == 0) sink[0] = (float)K;
}

__global__ void coop_pass_kernel(float4* b0, float4* b1, int n4, int K, float a, float b) {
  cg::grid_group g = cg::this_grid();
  for (int k = 0; k < K; ++k) {
    const float4* x = (k & 1) ? b1 : b0;
    float4* y = (k & 1) ? b0 : b1;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
      float4 v = x[i];
      y[i] = make_float4(a * v.x + b, a * v.y + b, a * v.z + b, a * v.w + b);
    }
    g.sync();
  }
}

// Hand-rolled sense-reversal barrier (what a cell-persistent kernel would use instead of the
// cooperative-groups one): one device-scope arrival counter and a generation word, both touched
// only through vector-memory atomics; the spin is bounded so a lost arrival cannot wedge the GPU
// (the kernel then records the failure in err and every wave still leaves).
__device__ __forceinline__ void bar_sync(unsigned* count, unsigned* gen, unsigned nblocks, unsigned& mygen, int* err) {
  __syncthreads();
  if (threadIdx.x == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
    const unsigned g = mygen;
    if (__hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1l << 20)) {  // ~50 ms: a broken barrier ends the probe, never hangs it
          atomicOr(err, 1);
          break;
        }
      }
    }
    mygen = g + 1;
  }
  __syncthreads();
}

__global__ void own_barrier_kernel(int K, unsigned* count, unsigned* gen, int* err) {
  unsigned mygen = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int k = 0; k < K; ++k) bar_sync(count, gen, gridDim.x, mygen, err);
}

__global__ void own_pass_kernel(float4* b0, float4* b1, int n4, int K, float a, float b, unsigned* count, unsigned* gen,
                                int* err) {
  unsigned mygen = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int k = 0; k < K; ++k) {
    const float4* x = (k & 1) ? b1 : b0;
    float4* y = (k & 1) ? b0 : b1;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
      float4 v = x[i];
      y[i] = make_float4(a * v.x + b, a * v.y + b, a * v.z + b, a * v.w + b);
    }
    bar_sync(count, gen, gridDim.x, mygen, err);
  }
}

// Round 5: a hierarchical per-XCD barrier. Workgroups are dispatched to the
// 8 XCDs round-robin (XCD = blockIdx.x & 7), so each XCD's workgroups first meet at a counter of
// their own (one 128-byte line per XCD); the last arrival of an XCD is the only one that touches
// the global counter, and on release the 8 XCD leaders alone poll the global generation word and
// forward it to a per-XCD generation word the rest of their XCD polls. Fewer same-address
// atomics (8 instead of 256 at the global counter) and 8 instead of 256 global pollers.
struct HierBar {
  unsigned* xcount;  // [8 x 32]: per-XCD arrival counters, 128 B apart
  unsigned* xgen;    // [8 x 32]: per-XCD generation words
  unsigned* count;   // global arrivals (one per XCD)
  unsigned* gen;     // global generation
};

__device__ __forceinline__ bool spin_until_changed(unsigned* w, unsigned g, int* err) {
  long spins = 0;
  while (__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1l << 20)) {
      atomicOr(err, 2);
      return false;
    }
  }
  return true;
}

__device__ __forceinline__ void hier_sync(const HierBar& b, unsigned& mygen, int* err) {
  __syncthreads();
  if (threadIdx.x == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
    const unsigned nblk = gridDim.x, xcd = blockIdx.x & 7u;
    const unsigned in_xcd = nblk / 8 + (xcd < (nblk & 7u) ? 1u : 0u);
    const unsigned nx = nblk < 8 ? nblk : 8;
    const unsigned g = mygen;
    unsigned* xc = b.xcount + xcd * 32;
    unsigned* xg = b.xgen + xcd * 32;
    if (__hip_atomic_fetch_add(xc, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == in_xcd - 1) {
      __hip_atomic_store(xc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // XCD leader
      if (__hip_atomic_fetch_add(b.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nx - 1) {
        __hip_atomic_store(b.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(b.gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        spin_until_changed(b.gen, g, err);
      }
      __hip_atomic_fetch_add(xg, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      spin_until_changed(xg, g, err);
    }
    mygen = g + 1;
  }
  __syncthreads();
}

__global__ void hier_barrier_kernel(int K, HierBar b, int* err) {
  unsigned mygen = __hip_atomic_load(b.xgen + (blockIdx.x & 7u) * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int k = 0; k < K; ++k) hier_sync(b, mygen, err);
}

__global__ void hier_pass_kernel(float4* b0, float4* b1, int n4, int K, float a, float bb, HierBar b, int* err) {
  unsigned mygen = __hip_atomic_load(b.xgen + (blockIdx.x & 7u) * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int k = 0; k < K; ++k) {
    const float4* x = (k & 1) ? b1 : b0;
    float4* y = (k & 1) ? b0 : b1;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
      float4 v = x[i];
      y[i] = make_float4(a * v.x + bb, a * v.y + bb, a * v.z + bb, a * v.w + bb);
    }
    hier_sync(b, mygen, err);
  }
}

template <class F>
static float time_ms(F&& f, hipStream_t st, int reps) {
  for (int i = 0; i < 3; ++i) f();
  CHECK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(e1, st));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 200;
  const int n = 1 << 19;  // 2 MB of fp32, a B5 C=4 activation at batch 128 x 32 x 32
  const int n4 = n / 4;
  const int reps = 20;
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  if (!prop.cooperativeLaunch) {
    std::printf("{\"error\": \"no cooperative launch\"}\n");
    return 1;
  }
  float4 *b0, *b1;
  float* sink;
  CHECK(hipMalloc(&b0, n * sizeof(float)));
  CHECK(hipMalloc(&b1, n * sizeof(float)));
  CHECK(hipMalloc(&sink, sizeof(float)));
  unsigned *ctr, *gen;
  int* err;
  CHECK(hipMalloc(&ctr, sizeof(unsigned)));
  CHECK(hipMalloc(&gen, sizeof(unsigned)));
  CHECK(hipMalloc(&err, sizeof(int)));
  CHECK(hipMemset(ctr, 0, sizeof(unsigned)));
  CHECK(hipMemset(gen, 0, sizeof(unsigned)));
  CHECK(hipMemset(err, 0, sizeof(int)));
  HierBar hb;
  CHECK(hipMalloc(&hb.xcount, 8 * 32 * sizeof(unsigned)));
  CHECK(hipMalloc(&hb.xgen, 8 * 32 * sizeof(unsigned)));
  CHECK(hipMalloc(&hb.count, 64 * sizeof(unsigned)));
  CHECK(hipMalloc(&hb.gen, 64 * sizeof(unsigned)));
  CHECK(hipMemsetAsync(b0, 0, n * sizeof(float), st));
  CHECK(hipMemsetAsync(b1, 0, n * sizeof(float), st));

  auto graph_of = [&](auto&& body) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    body();
    CHECK(hipStreamEndCapture(st, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHECK(hipGraphDestroy(g));
    return ge;
  };

  hipGraphExec_t g_empty = graph_of([&] {
    for (int k = 0; k < K; ++k) empty_kernel<<<1, 64, 0, st>>>();
  });
  hipGraphExec_t g_pass = graph_of([&] {
    for (int k = 0; k < K; ++k)
      pass_kernel<<<2048, 256, 0, st>>>((k & 1) ? b1 : b0, (k & 1) ? b0 : b1, n4, 0.5f, 1.0f);
  });
  const float ms_empty = time_ms([&] { CHECK(hipGraphLaunch(g_empty, st)); }, st, reps);
  const float ms_pass = time_ms([&] { CHECK(hipGraphLaunch(g_pass, st)); }, st, reps);

  std::printf("{\"K\": %d, \"bytes_per_pass\": %d, \"cus\": %d, \"launch_empty_us\": %.3f, \"launch_pass_us\": %.3f",
              K, 2 * n * 4, prop.multiProcessorCount, ms_empty * 1e3f / K, ms_pass * 1e3f / K);
  for (int per_cu = 1; per_cu <= 2; ++per_cu) {
    const int blocks = prop.multiProcessorCount * per_cu;
    int Kv = K;
    void* bargs[] = {&Kv, &sink};
    const float ms_bar = time_ms([&] {
      CHECK(hipLaunchCooperativeKernel((const void*)coop_barrier_kernel, dim3(blocks), dim3(256), bargs, 0, st));
    }, st, reps);
    float a = 0.5f, bb = 1.0f;
    int n4v = n4;
    void* pargs[] = {&b0, &b1, &n4v, &Kv, &a, &bb};
    const float ms_coop = time_ms([&] {
      CHECK(hipLaunchCooperativeKernel((const void*)coop_pass_kernel, dim3(blocks), dim3(256), pargs, 0, st));
    }, st, reps);
    std::printf(", \"barrier_empty_us_%dwg\": %.3f, \"coop_pass_us_%dwg\": %.3f", blocks, ms_bar * 1e3f / K, blocks,
                ms_coop * 1e3f / K);
    // the hand-rolled barrier, launched cooperatively too (co-residency of every workgroup checked)
    void* oargs[] = {&Kv, &ctr, &gen, &err};
    const float ms_own = time_ms([&] {
      CHECK(hipLaunchCooperativeKernel((const void*)own_barrier_kernel, dim3(blocks), dim3(256), oargs, 0, st));
    }, st, reps);
    void* opargs[] = {&b0, &b1, &n4v, &Kv, &a, &bb, &ctr, &gen, &err};
    const float ms_own_pass = time_ms([&] {
      CHECK(hipLaunchCooperativeKernel((const void*)own_pass_kernel, dim3(blocks), dim3(256), opargs, 0, st));
    }, st, reps);
    std::printf(", \"own_barrier_us_%dwg\": %.3f, \"own_pass_us_%dwg\": %.3f", blocks, ms_own * 1e3f / K, blocks,
                ms_own_pass * 1e3f / K);
    // hierarchical per-XCD barrier (all generation words start at 0 and advance together)
    CHECK(hipMemset(hb.xcount, 0, 8 * 32 * sizeof(unsigned)));
    CHECK(hipMemset(hb.xgen, 0, 8 * 32 * sizeof(unsigned)));
    CHECK(hipMemset(hb.count, 0, sizeof(unsigned)));
    CHECK(hipMemset(hb.gen, 0, sizeof(unsigned)));
    CHECK(hipDeviceSynchronize());
    void* hargs[] = {&Kv, &hb, &err};
    const float ms_hier = time_ms([&] {
      CHECK(hipLaunchCooperativeKernel((const void*)hier_barrier_kernel, dim3(blocks), dim3(256), hargs, 0, st));
    }, st, reps);
    void* hpargs[] = {&b0, &b1, &n4v, &Kv, &a, &bb, &hb, &err};
    const float ms_hier_pass = time_ms([&] {
      CHECK(hipLaunchCooperativeKernel((const void*)hier_pass_kernel, dim3(blocks), dim3(256), hpargs, 0, st));
    }, st, reps);
    std::printf(", \"hier_xcd_barrier_us_%dwg\": %.3f, \"hier_xcd_pass_us_%dwg\": %.3f", blocks, ms_hier * 1e3f / K,
                blocks, ms_hier_pass * 1e3f / K);
  }
  int herr = 0;
  CHECK(hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost));
  std::printf(", \"own_barrier_timeouts\": %d", herr);  // bit 1: flat barrier, bit 2: hierarchical
  std::printf("}\n");
  CHECK(hipGraphExecDestroy(g_empty));
  CHECK(hipGraphExecDestroy(g_pass));
  CHECK(hipFree(b0));
  CHECK(hipFree(b1));
  CHECK(hipFree(sink));
  CHECK(hipFree(ctr));
  CHECK(hipFree(gen));
  CHECK(hipFree(err));
  CHECK(hipFree(hb.xcount));
  CHECK(hipFree(hb.xgen));
  CHECK(hipFree(hb.count));
  CHECK(hipFree(hb.gen));
  return 0;
}
