// One-shot xGMI all-reduce: shared host/device declarations (see xgmi_allreduce.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace katib_hip {
namespace xgmi {

constexpr int kMaxRanks = 8;     // one MI355X node
constexpr int kMaxBlocks = 256;  // fixed grid per workspace, <= kMaxBlocks
constexpr int kThreads = 512;
// signal page (uint32 words): flags[kMaxBlocks][kMaxRanks] | epoch[kMaxBlocks] | err
constexpr int kSigEpoch = kMaxBlocks * kMaxRanks;
constexpr int kSigErr = kSigEpoch + kMaxBlocks;
constexpr int kSigWords = kSigErr + 64;

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

}  // namespace xgmi
}  // namespace katib_hip
