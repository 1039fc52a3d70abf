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
// One launch, HBM-bound (bytes per group in DESIGN.md §4.5): one lane per group per tile
// slot computes the status, the popClosureUntil result and the in-place ClosureQueue
// (firstIndex, size); a wave ballot over 64 consecutive groups writes one word of the
// `listed` bitmap (APPLY or INVALID: the groups the host must act on), and the workgroups'
// counts meet in one counter (the last workgroup publishes it).  The host walks the set bits in ascending group order.
#include "jrq_device.h"

namespace jrq {

constexpr int kFanBlock = 1024;
constexpr int kFanPerThread = 4;
constexpr int kFanTile = kFanBlock * kFanPerThread;  // groups per tile

// include/jrq.h jrq_fanout_status
constexpr uint8_t kFanNone = 0, kFanApply = 1, kFanSkip = 2, kFanInvalid = 3;

__device__ __forceinline__ bool listed(uint8_t st) { return st == kFanApply || st == kFanInvalid; }

// Tile slot k of thread t is group base + k*kFanBlock + t: every load is a coalesced stream,
// and the 64 lanes of a wave hold 64 consecutive groups (one bitmap word).
__global__ __launch_bounds__(kFanBlock) void fanout_eval(JrqFanoutArgs a) {
  __shared__ uint32_t block_listed;
  if (threadIdx.x == 0) block_listed = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * kFanTile + threadIdx.x;
  uint32_t mine = 0;
#pragma unroll
  for (int k = 0; k < kFanPerThread; ++k) {
    const uint32_t g = base + k * kFanBlock;
    const uint32_t g0 = g - (threadIdx.x & 63u);  // first group of this wave's word
    if (g0 >= a.G) break;                          // wave-uniform
    uint8_t st = kFanNone;
    if (g < a.G) {
      const int64_t c = a.committed[g];
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
    }
    const uint64_t word = __ballot(listed(st));
    if ((threadIdx.x & 63u) == 0) a.listed[g0 >> 6] = word;
    mine += static_cast<uint32_t>(__popcll(word));
  }
  // one global atomic per workgroup (per-wave atomics on one address serialise at L2); the
  // last workgroup to finish publishes the sum and re-zeroes the counters for the next launch
  if ((threadIdx.x & 63u) == 0 && mine) atomicAdd(&block_listed, mine);
  __syncthreads();
  // (one 64-bit atomic carries both: blocks done << 32 | listed sum -- no fence needed)
  if (threadIdx.x == 0) {
    const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr),
                                             (1ull << 32) | block_listed);
    if ((old >> 32) == gridDim.x - 1u) {
      *a.num_listed = static_cast<uint32_t>(old) + block_listed;
      atomicExch(reinterpret_cast<unsigned long long*>(a.ctr), 0ull);
    }
  }
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_fanout(
    const JrqFanoutArgs* a, hipStream_t stream) {
  const uint32_t ntiles = (a->G + jrq::kFanTile - 1) / jrq::kFanTile;
  hipLaunchKernelGGL(jrq::fanout_eval, dim3(ntiles), dim3(jrq::kFanBlock), 0, stream, *a);
  return hipGetLastError();
}
