// Argument blocks for the DARTS edge kernels (darts_ops.hip). Passed by value.
#pragma once
#include <hip/hip_runtime.h>

namespace katib_hip {

constexpr int kMaxOps = 8;
constexpr int kMaxC = 256;

struct BNRef {              // where a BN layer's normalisation statistics come from
  const double* sums;       // training: [2*C] = (sum, sum of squares) of the pre-BN tensor
  float* rmean;             // running stats (read in eval, updated by combine in training)
  float* rvar;
  float inv_count;          // 1 / (N*H*W)
  float eps;
  int eval;
  int C;
};

struct GradSrc {            // d(loss)/d(z) evaluated on the fly: BN backward of a weighted op
  const float* g;           // upstream gradient (dout of the edge, or a stored stage gradient)
  const float* z;           // pre-BN tensor
  const double* S1;         // [C] sum g
  const double* S2;         // [C] sum g * zhat
  BNRef bn;
  const float* w;           // softmax weights (nullptr -> 1)
  int widx;
  int eval;
};

struct DwPwFwdArgs {
  const float* x; BNRef inbn; const float* dw; const float* pw;
  float* d; float* z; double* stats;
  int N, C, H, W, Ho, Wo, pad, chunk, use_mfma;
};

struct PwFwdArgs {
  const float* x; const float* pw; float* z; double* stats;
  int N, Cin, Cout, CoutTotal, co_off, H, W, Ho, Wo, S, off;
};

struct PoolFwdArgs {
  const float* x; float* zavg; float* zmax; double* stats_avg; double* stats_max; unsigned char* amax;
  int N, C, H, W, Ho, Wo;
};

struct CombineFwdArgs {
  const float* z[kMaxOps]; BNRef bn[kMaxOps]; int widx[kMaxOps]; int nops;
  BNRef upd[kMaxOps]; int nupd;  // extra BN layers whose running stats are updated here (not summed)
  const float* w; int id_idx; const float* xid; const float* gamma; const float* beta;
  float* out; int N, C, HW; float momentum; int update_running; int accumulate;
};

struct CombineBwdArgs {
  const float* dout; const float* z[kMaxOps]; BNRef bn[kMaxOps]; int nops;
  const float* xid; double* red; int N, C, HW;
  double* gw; int widx[kMaxOps]; int id_idx;  // optional: d(loss)/d(softmax weight) per primitive
};

struct PwBwdArgs {
  GradSrc gs; const float* pw; const float* ain; const float* x; float* dd; float* gx; float* gW;
  int N, Cin, Cout, CoutTotal, co_off, H, W, Ho, Wo, S, off, mode, need_dx;
};

struct DwBwdArgs {
  const float* x; BNRef inbn; const float* dw; const float* dd; float* gout; float* gW; double* red;
  int N, C, H, W, Ho, Wo, pad, chunk;
};

struct PoolBwdArgs {
  GradSrc ga; GradSrc gm; const float* x; const float* dout_id; const float* w; int id_idx; float* gx;
  const unsigned char* amax;
  int N, C, H, W, Ho, Wo;
};

void launch_dwpw_fwd(const DwPwFwdArgs& a, int K, int dil, int S, bool prebn, hipStream_t st);
void launch_dw_bwd(const DwBwdArgs& a, int K, int dil, int S, bool prebn, hipStream_t st);
void launch_pw_fwd(const PwFwdArgs& a, hipStream_t st);
void launch_pool_fwd(const PoolFwdArgs& a, int S, hipStream_t st);
void launch_pool_bwd(const PoolBwdArgs& a, int S, hipStream_t st);
void launch_combine_fwd(const CombineFwdArgs& a, hipStream_t st);
void launch_combine_bwd_reduce(const CombineBwdArgs& a, hipStream_t st);
void launch_pw_bwd(const PwBwdArgs& a, hipStream_t st);
int max_blocks();
void set_max_blocks(int n);

}  // namespace katib_hip
