// Does the HIP runtime (ROCm 7.2, gfx950) pass kernel arguments larger than 4 KB by value, eagerly
// and inside a captured graph? Each kernel sums its by-value int array; the host checks the sums.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
struct Blob {
  int v[N];
};

template <int N>
__global__ void sum_k(Blob<N> b, long long* out) {
  long long s = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) s += b.v[i];
  __shared__ long long sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int i = 0; i < 256; ++i) t += sh[i];
    out[blockIdx.x] = t;
  }
}

template <int N>
int run(long long* d, hipStream_t st, bool graph) {
  Blob<N> b;
  long long want = 0;
  for (int i = 0; i < N; ++i) {
    b.v[i] = i * 7 + 3;
    want += b.v[i];
  }
  hipMemset(d, 0, 8 * 4);
  hipError_t e;
  if (graph) {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    hipLaunchKernelGGL(sum_k<N>, dim3(4), dim3(256), 0, st, b, d);
    e = hipGetLastError();
    hipStreamEndCapture(st, &g);
    if (e == hipSuccess) e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int i = 0; i < N; ++i) b.v[i] = -1;  // the graph must have copied the arguments
    if (e == hipSuccess) e = hipGraphLaunch(ge, st);
  } else {
    hipLaunchKernelGGL(sum_k<N>, dim3(4), dim3(256), 0, st, b, d);
    e = hipGetLastError();
  }
  hipError_t e2 = hipStreamSynchronize(st);
  long long h[4] = {0, 0, 0, 0};
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const bool ok = e == hipSuccess && e2 == hipSuccess && h[0] == want && h[3] == want;
  printf("{\"bytes\": %d, \"graph\": %d, \"launch\": \"%s\", \"sync\": \"%s\", \"ok\": %s}\n", (int)sizeof(Blob<N>),
         graph ? 1 : 0, hipGetErrorString(e), hipGetErrorString(e2), ok ? "true" : "false");
  return ok ? 0 : 1;
}

int main() {
  long long* d;
  hipMalloc(&d, 8 * 4);
  hipStream_t st;
  hipStreamCreate(&st);
  int bad = 0;
  for (int graph = 0; graph < 2; ++graph) {
    bad += run<1000>(d, st, graph);
    bad += run<2000>(d, st, graph);
    bad += run<4000>(d, st, graph);
    bad += run<7000>(d, st, graph);
  }
  printf("{\"failures\": %d}\n", bad);
  return 0;
}
