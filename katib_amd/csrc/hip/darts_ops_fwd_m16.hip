// Mixed-variant dw-pw (and joint dw-pw + pool) kernels for C = 16 channel groups: one translation
// unit per channel count so their 32-variant bodies compile in parallel.
#include "darts_ops_fwd_k.h"

namespace katib_hip {

template <>
void launch_dwpw_plane_multi_t<16>(bool pw, dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b) {
  (void)pw;
  KSTAMP_ARM(kStampDwPw, st)
  hipLaunchKernelGGL((dwpw_plane_multi_kernel<16, true>), grid, dim3(256), lds, st, b);
  KSTAMP_DISARM(st)
}

}  // namespace katib_hip
