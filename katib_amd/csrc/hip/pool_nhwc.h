// NHWC bf16 max / average pooling ('valid' padding) for the ENAS child network (pool_nhwc.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace katib_hip {
namespace poolnhwc {

struct Geom {
  int N, H, W, C;  // input [N][H][W][C], C % 8 == 0
  int P, S;        // window, stride
  int OH, OW;      // (H - P) / S + 1, (W - P) / S + 1
};

// y [N][OH][OW][C] bf16; arg [N][OH][OW][C] uint8 winning tap (max only)
hipError_t launch_fwd(const Geom& g, bool is_max, const void* x, void* y, void* arg, hipStream_t st);
// gx [N][H][W][C] bf16 written in full (zeros where no window reaches)
hipError_t launch_bwd(const Geom& g, bool is_max, const void* gy, const void* arg, void* gx, hipStream_t st);

}  // namespace poolnhwc
}  // namespace katib_hip
