// Mixed-variant dw-pw (and joint dw-pw + pool) kernels for C = 8 channel groups: one translation
// unit per channel count so their 32-variant bodies compile in parallel.
#include "darts_ops_fwd_k.h"

namespace katib_hip {

template <>
void launch_dwpw_plane_multi_t<8>(bool pw, dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b) {
  if (!pw) {
    hipLaunchKernelGGL((dwpw_plane_multi_kernel<8, false>), grid, dim3(256), lds, st, b);
    return;
  }
  KSTAMP_ARM(kStampDwPw, st)
  hipLaunchKernelGGL((dwpw_plane_multi_kernel<8, true>), grid, dim3(256), lds, st, b);
  KSTAMP_DISARM(st)
}

template <>
void launch_dwpw_pool_t<8>(dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b, const PoolFwdEntries& pe) {
  hipLaunchKernelGGL((dwpw_pool_multi_kernel<8, true>), grid, dim3(256), lds, st, b, pe);
}

}  // namespace katib_hip
