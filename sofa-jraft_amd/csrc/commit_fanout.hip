// commit_fanout.hip -- batched commit fan-out after a quorum epoch.
//
// Reference, per group whose commit index moved during the epoch:
//   BallotBox.commitAt -> waiter.onCommitted(lastCommittedIndex)   (core/BallotBox.java:131-137)
//   FSMCallerImpl.onCommitted enqueues COMMITTED; runApplyTask coalesces a batch to its max
//     committed index and calls doCommitted(max)                   (core/FSMCallerImpl.java:239-244,362-373)
//   doCommitted: nothing if lastAppliedIndex >= committedIndex      (:462-470), else
//     ClosureQueueImpl.popClosureUntil(committedIndex)              (closure/ClosureQueueImpl.java:113-142):
//       queue empty or committedIndex < firstIndex -> returns committedIndex + 1, pops nothing
//       committedIndex > firstIndex + size - 1     -> returns -1 (doCommitted then fails
//                                                     Requires.requireTrue, :480), pops nothing
//       otherwise pops [firstIndex, committedIndex], firstIndex = committedIndex + 1,
//       returns the old firstIndex
//     and applies log entries (lastAppliedIndex, committedIndex] with those closures.
// Several onCommitted calls in one epoch carry increasing indices, and popping [f, c1] then
// [c1+1, c2] leaves the same queue as popping [f, c2]: the post-epoch state depends only on
// the epoch's last committed index.  One exception: a commit beyond the closure queue
// (INVALID, only reachable when the queue is inconsistent with the log) is reported with
// nothing popped, where the reference may first pop a prefix through an earlier onCommitted
// of the same epoch and then fail.  tests/test_commit_fanout.py checks this closed form
// against a call-by-call replay (oracle/jraft_oracle.c jo_commit_fanout_replay).
//
// Three launches (HBM-bound; bytes per group in DESIGN.md §4.5):
//   fanout_eval     one thread per group per tile slot: status, popClosureUntil result,
//                   in-place ClosureQueue (firstIndex, size); per-tile count of groups the
//                   host must act on (APPLY or INVALID)
//   fanout_scan     one block: exclusive scan of the tile counts, total -> num_listed
//   fanout_compact  the listed group ids in ascending order (deterministic, no atomics)
#include "jrq_device.h"

namespace jrq {

constexpr int kFanBlock = 1024;
constexpr int kFanPerThread = 4;
constexpr int kFanTile = kFanBlock * kFanPerThread;  // groups per tile

// include/jrq.h jrq_fanout_status
constexpr uint8_t kFanNone = 0, kFanApply = 1, kFanSkip = 2, kFanInvalid = 3;

__device__ __forceinline__ bool listed(uint8_t st) { return st == kFanApply || st == kFanInvalid; }

// Tile slot k of thread t is group base + k*kFanBlock + t: every load is a coalesced stream.
__global__ __launch_bounds__(kFanBlock) void fanout_eval(JrqFanoutArgs a) {
  const uint32_t base = blockIdx.x * kFanTile + threadIdx.x;
  uint32_t mine = 0;
#pragma unroll
  for (int k = 0; k < kFanPerThread; ++k) {
    const uint32_t g = base + k * kFanBlock;
    if (g >= a.G) break;
    const int64_t c = a.committed[g];
    uint8_t st = kFanNone;
    int64_t first_closure = 0;
    if (c > a.prev_committed[g]) {  // onCommitted(c) was called for this group
      if (a.last_applied[g] >= c) {
        st = kFanSkip;
      } else {
        const int64_t f = a.cq_first[g];
        const int64_t n = a.cq_size[g];
        if (n == 0 || c < f) {
          st = kFanApply;
          first_closure = c + 1;
        } else if (c > f + n - 1) {
          st = kFanInvalid;
          first_closure = -1;
        } else {
          st = kFanApply;
          first_closure = f;
          a.cq_first[g] = c + 1;
          a.cq_size[g] = n - (c - f + 1);
        }
      }
    }
    a.first_closure[g] = first_closure;
    a.status[g] = st;
    mine += listed(st) ? 1u : 0u;
  }
  __shared__ uint64_t w[kFanBlock / 64];
  uint64_t total;
  (void)block_exclusive_scan(mine, w, &total);
  if (threadIdx.x == 0) a.tile_count[blockIdx.x] = static_cast<uint32_t>(total);
}

__global__ __launch_bounds__(kFanBlock) void fanout_scan(JrqFanoutArgs a, uint32_t ntiles) {
  __shared__ uint64_t w[kFanBlock / 64];
  uint64_t carry = 0;
  for (uint32_t c = 0; c < ntiles; c += kFanBlock) {
    const uint32_t i = c + threadIdx.x;
    const uint64_t v = i < ntiles ? a.tile_count[i] : 0;
    uint64_t total;
    const uint64_t ex = block_exclusive_scan(v, w, &total);
    if (i < ntiles) a.tile_count[i] = static_cast<uint32_t>(carry + ex);
    carry += total;
  }
  if (threadIdx.x == 0) *a.num_listed = static_cast<uint32_t>(carry);
}

// Thread t owns the 4 consecutive groups base + 4t .. base + 4t + 3 (ascending order).
__global__ __launch_bounds__(kFanBlock) void fanout_compact(JrqFanoutArgs a) {
  const uint32_t base = blockIdx.x * kFanTile + threadIdx.x * kFanPerThread;
  bool f[kFanPerThread];
  uint32_t mine = 0;
#pragma unroll
  for (int k = 0; k < kFanPerThread; ++k) {
    f[k] = base + k < a.G && listed(a.status[base + k]);
    mine += f[k] ? 1u : 0u;
  }
  __shared__ uint64_t w[kFanBlock / 64];
  uint64_t total;
  uint32_t pos = a.tile_count[blockIdx.x] + static_cast<uint32_t>(block_exclusive_scan(mine, w, &total));
#pragma unroll
  for (int k = 0; k < kFanPerThread; ++k)
    if (f[k]) a.listed[pos++] = base + k;
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_fanout(
    const JrqFanoutArgs* a, hipStream_t stream) {
  const uint32_t ntiles = (a->G + jrq::kFanTile - 1) / jrq::kFanTile;
  hipLaunchKernelGGL(jrq::fanout_eval, dim3(ntiles), dim3(jrq::kFanBlock), 0, stream, *a);
  hipLaunchKernelGGL(jrq::fanout_scan, dim3(1), dim3(jrq::kFanBlock), 0, stream, *a, ntiles);
  hipLaunchKernelGGL(jrq::fanout_compact, dim3(ntiles), dim3(jrq::kFanBlock), 0, stream, *a);
  return hipGetLastError();
}
