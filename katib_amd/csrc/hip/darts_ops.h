// Argument blocks for the DARTS edge kernels (darts_ops.hip). Passed by value.
#pragma once
#include <hip/hip_runtime.h>

namespace katib_hip {

constexpr int kMaxOps = 8;
constexpr int kMaxC = 256;
// Cross-workgroup sums (BN statistics, BN-backward reductions, weight gradients) go to kRep
// replicas of the accumulator, workgroup b adding into replica b % kRep: global float atomics
// execute memory-side and same-address adds serialise, so bounding the adders per address
// (grid / kRep) keeps every flush short. Consumers sum the replicas (bn_moments / prologues);
// weight-gradient replicas are folded once per backward pass (fold_rows).
#ifndef KATIB_HIP_REP
#define KATIB_HIP_REP 32
#endif
constexpr int kRep = KATIB_HIP_REP;

struct BNRef {              // where a BN layer's normalisation statistics come from
  const double* sums;       // training: replica r at sums + r*rstride: [2*C] = (sum, sum of squares)
  float* rmean;             // running stats (read in eval, updated by combine in training)
  float* rvar;
  float inv_count;          // 1 / (N*H*W)
  float eps;
  int eval;
  int C;
  int rep;                  // replicas to sum (1 or kRep)
  int rstride;              // doubles between replicas
};

struct GradSrc {            // d(loss)/d(z) evaluated on the fly: BN backward of a weighted op
  const float* g;           // upstream gradient (dout of the edge, or a stored stage gradient)
  const float* z;           // pre-BN tensor
  const double* S1;         // [C] sum g            (replica r at + r*rstride)
  const double* S2;         // [C] sum g * zhat
  BNRef bn;
  const float* w;           // softmax weights (nullptr -> 1)
  int widx;
  int eval;
  int rep;
  int rstride;
};

struct DwPwFwdArgs {
  const float* x; BNRef inbn; const float* dw; const float* pw;
  float* d; float* z; double* stats;  // stats: kRep replicas of [2C]
  int N, C, H, W, Ho, Wo, pad, chunk, use_mfma;
  int variant;  // dwpw_plane_multi_kernel: ((K == 5) * 4 + (dil == 2) * 2 + (S == 2)) * 4 + prebn * 2 + vec
  int nblk;     // dwpw_plane_multi_kernel: workgroups of this entry (grid.x is the max over entries)
};

struct PwFwdArgs {
  const float* x; const float* pw; float* z; double* stats;  // stats: kRep replicas of [2*CoutTotal]
  int N, Cin, Cout, CoutTotal, co_off, H, W, Ho, Wo, S, off;
  int relu;  // 1: input = relu(x) (StdConv / FactorizedReduce); 0: identity (pointwise half of a dw-pw stage)
};

struct PoolFwdArgs {
  const float* x; float* zavg; float* zmax; double* stats_avg; double* stats_max; unsigned char* amax;
  int N, C, H, W, Ho, Wo;  // stats: kRep replicas of [2C] each
  int S, nblk;             // pool_fwd_multi_kernel: per-entry stride and workgroups
};

struct CombineFwdArgs {
  const float* z[kMaxOps]; BNRef bn[kMaxOps]; int widx[kMaxOps]; int nops;
  BNRef upd[kMaxOps]; int nupd;  // extra BN layers whose running stats are updated here (not summed)
  const float* w; int id_idx; const float* xid; const float* gamma; const float* beta;
  float* out; int N, C, HW; float momentum; int update_running; int accumulate;
};

struct CombineBwdArgs {
  const float* dout; const float* z[kMaxOps]; BNRef bn[kMaxOps]; int nops;
  const float* xid; double* red; int N, C, HW;  // red: kRep replicas of [(nops+1)*C + 1]
  double* gw; int widx[kMaxOps]; int id_idx;  // optional: d(loss)/d(softmax weight), kRep replicas of [nw]
  int rstride, gwstride;
};

struct PwBwdArgs {
  GradSrc gs; const float* pw; const float* ain; const float* x; float* dd; float* gx; float* gW;
  int gstride;  // floats between gW replicas (0: single accumulator)
  int N, Cin, Cout, CoutTotal, co_off, H, W, Ho, Wo, S, off, mode, need_dx;
  int overwrite;  // mode 1, stride 1: gx = masked grad instead of += (the kernel covers every pixel)
};

struct DwBwdArgs {
  const float* x; BNRef inbn; const float* dw; const float* dd; float* gout; float* gW; double* red;
  int gstride;  // floats between gW replicas (0: single accumulator); red: kRep replicas of [2C]
  int N, C, H, W, Ho, Wo, pad, chunk;
  int overwrite;  // non-PREBN: gout = masked grad (first writer of this input gradient) instead of +=
};

struct FoldArgs {  // buf[0][i] = sum_r buf[r][i]; rows 1.. zeroed
  float* buf; int n; int rows;
};

constexpr int kMaxSeg = 64;
struct FoldF64Args {  // per segment: p[i] = sum_{r < kRep} p[r*rstride + i]; replicas 1.. zeroed
  double* p[kMaxSeg]; int n[kMaxSeg]; int rstride[kMaxSeg]; int nseg; int total;
};

struct PoolBwdArgs {
  GradSrc ga; GradSrc gm; const float* x; const float* dout_id; const float* w; int id_idx; float* gx;
  const unsigned char* amax;
  int overwrite;  // gx = result instead of +=
  int N, C, H, W, Ho, Wo;
  int S;          // pool_bwd_multi_kernel: per-entry stride
};

// Edge batches: one launch runs the same kernel for up to M edges of a DARTS node that share
// shapes (blockIdx.y = edge). Passed by value in the kernarg segment (kept <= 4 KB).
template <typename A, int M>
struct Batch {
  A e[M];
  int n;
  static constexpr int kCap = M;
};
using DwPwFwdBatch = Batch<DwPwFwdArgs, 8>;
using CombineFwdBatch = Batch<CombineFwdArgs, 3>;
using PwFwdBatch = Batch<PwFwdArgs, 16>;
using PoolFwdBatch = Batch<PoolFwdArgs, 8>;
using CombineBwdBatch = Batch<CombineBwdArgs, 4>;
using PwBwdBatch = Batch<PwBwdArgs, 8>;
using DwBwdBatch = Batch<DwBwdArgs, 8>;
using PoolBwdBatch = Batch<PoolBwdArgs, 8>;
using DwPwMultiBatch = Batch<DwPwFwdArgs, 16>;  // a node's stage-1 (or stage-2) dw-pw entries, mixed K/dil/S
static_assert(sizeof(DwPwMultiBatch) <= 4096 && sizeof(PoolBwdBatch) <= 4096 && sizeof(PwFwdBatch) <= 4096,
              "kernel argument blocks must fit the 4 KB kernarg segment");
static_assert(sizeof(DwPwFwdBatch) <= 4096 && sizeof(CombineFwdBatch) <= 4096 && sizeof(PwFwdBatch) <= 4096 && sizeof(PoolFwdBatch) <= 4096 &&
                  sizeof(CombineBwdBatch) <= 4096 && sizeof(PwBwdBatch) <= 4096 && sizeof(DwBwdBatch) <= 4096 &&
                  sizeof(PoolBwdBatch) <= 4096,
              "kernel argument batches must fit the 4 KB kernarg budget");

void launch_dwpw_fwd(const DwPwFwdBatch& b, int K, int dil, int S, bool prebn, hipStream_t st);
void launch_dw_bwd(const DwBwdBatch& b, int K, int dil, int S, bool prebn, hipStream_t st);
void launch_pw_fwd(const PwFwdBatch& b, hipStream_t st);
void launch_pool_fwd(const PoolFwdBatch& b, int S, hipStream_t st);
void launch_pool_bwd(const PoolBwdBatch& b, int S, hipStream_t st);
// mixed-variant launches: one launch for entries with different kernel size / dilation / stride
bool launch_dwpw_multi(DwPwMultiBatch b, hipStream_t st);
void launch_pool_fwd_multi(PoolFwdBatch b, hipStream_t st);
void launch_pool_bwd_multi(const PoolBwdBatch& b, hipStream_t st);
void launch_combine_fwd(const CombineFwdBatch& b, hipStream_t st);
void launch_combine_bwd_reduce(const CombineBwdBatch& b, hipStream_t st);
void launch_pw_bwd(const PwBwdBatch& b, hipStream_t st);
int max_blocks();
void launch_fold_rows(const FoldArgs& a, hipStream_t st);
void launch_fold_f64(const FoldF64Args& a, hipStream_t st);
void set_max_blocks(int n);

}  // namespace katib_hip
