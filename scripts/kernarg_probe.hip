// Does the kernarg size change the per-launch cost inside a replayed HIP graph? The DARTS edge
// launches pass their per-entry batches by value (1-4 KB). K empty kernels with a 16 B .. 4 KB
// by-value argument, captured in one graph, replayed 20 times: us per launch.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/kernarg_probe scripts/kernarg_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

template <int B>
struct Arg {
  int v[B / 4];
};

template <int B>
__global__ void k_arg(Arg<B> a, int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.v[B / 4 - 1] == 12345) out[0] = a.v[0];
}

template <int B>
static float per_launch_us(hipStream_t st, int K, int blocks, int* out) {
  Arg<B> a{};
  for (int i = 0; i < B / 4; ++i) a.v[i] = i;
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < K; ++k) k_arg<B><<<blocks, 256, 0, st>>>(a, out);
  CHECK(hipStreamEndCapture(st, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CHECK(hipGraphLaunch(ge, st));
  CHECK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, st));
  const int reps = 20;
  for (int i = 0; i < reps; ++i) CHECK(hipGraphLaunch(ge, st));
  CHECK(hipEventRecord(e1, st));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms * 1e3f / (reps * K);
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 200;
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* out;
  CHECK(hipMalloc(&out, sizeof(int)));
  for (int blocks : {1, 2048}) {
    std::printf("{\"K\": %d, \"blocks\": %d, \"us_16B\": %.3f, \"us_256B\": %.3f, \"us_1KB\": %.3f, \"us_2KB\": %.3f, \"us_3KB\": %.3f, \"us_4000B\": %.3f}\n",
                K, blocks, per_launch_us<16>(st, K, blocks, out), per_launch_us<256>(st, K, blocks, out),
                per_launch_us<1024>(st, K, blocks, out), per_launch_us<2048>(st, K, blocks, out),
                per_launch_us<3072>(st, K, blocks, out), per_launch_us<4000>(st, K, blocks, out));
  }
  CHECK(hipFree(out));
  return 0;
}
