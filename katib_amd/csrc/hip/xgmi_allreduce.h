// One-shot xGMI all-reduce: shared host/device declarations (see xgmi_allreduce.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "darts_ops.h"  // FoldF64Args (SyncBN: fold + cross-rank sum of the DARTS BN reductions)

namespace katib_hip {
namespace xgmi {

constexpr int kMaxRanks = 8;     // one MI355X node
constexpr int kMaxBlocks = 256;  // fixed grid per workspace, <= kMaxBlocks
constexpr int kThreads = 512;
// signal page (uint32 words): flags[kMaxBlocks][kMaxRanks] | epoch[kMaxBlocks] | err
constexpr int kSigEpoch = kMaxBlocks * kMaxRanks;
constexpr int kSigErr = kSigEpoch + kMaxBlocks;
constexpr int kSigWords = kSigErr + 64;

constexpr int kSmallFold = 4096;  // fold_sync: totals up to this many doubles run on one workgroup

struct AllReduceArgs {
  const float* in;
  float* out;
  int64_t n;
  int64_t cap;  // floats per staging half (multiple of 4)
  float scale;
  int rank, world;
  uint64_t timeout_ticks;  // wall_clock64 ticks (100 MHz)
  float* buf[kMaxRanks];   // staging [2][cap] of every rank (mine + IPC-mapped peers)
  uint32_t* sig[kMaxRanks];
};

hipError_t launch_oneshot(const AllReduceArgs& a, int blocks, bool vec4, hipStream_t stream);
// SyncBN for the DARTS supernet: fold the kRep replicas of every segment (as fold_f64) and, for
// the segments whose bit is set in sync_mask (BN statistics / BN-backward sums), also sum the folded
// values over the ranks in rank order (fp64, identical bits on every rank); the other segments
// (d alpha) stay local. a.in / a.out / a.n / a.scale are unused; staging holds cap / 2 doubles.
hipError_t launch_fold_sync(const AllReduceArgs& a, const FoldF64Args& f, uint64_t sync_mask, int blocks,
                            hipStream_t stream);

}  // namespace xgmi
}  // namespace katib_hip
