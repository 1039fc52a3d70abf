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

#ifndef JRQ_FAN_BLOCK
#define JRQ_FAN_BLOCK 1024
#endif
#ifndef JRQ_FAN_PER_THREAD
#define JRQ_FAN_PER_THREAD 4
#endif
constexpr int kFanBlock = JRQ_FAN_BLOCK;
constexpr int kFanPerThread = JRQ_FAN_PER_THREAD;
constexpr int kFanTile = kFanBlock * kFanPerThread;  // groups per tile

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

// (fan_one: the per-group closed form above, jrq_device.h, shared with the table's fused epoch)

// Bits 0..31 of x to the even bits, of y to the odd bits (a pair lane's two groups are
// adjacent in the bitmap).
__device__ __forceinline__ uint64_t interleave32(uint64_t x, uint64_t y) {
  auto spread = [](uint64_t v) {
    v &= 0xFFFFFFFFull;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
  };
  return spread(x) | (spread(y) << 1);
}

// Two adjacent groups per lane (r05), as the headline epoch kernel reads its streams: every
// int64 stream with 16-B nt loads (1 KiB per wave instruction, where fanout_eval's one group
// per lane moved 512 B), all five issued before the first decision, two pair slots per lane
// (kFanBlock * 4 groups per workgroup, the same 256 workgroups for 1M groups: one counter
// atomic each).  The queue words are written back only by a lane whose pair pops.  A wave's 64
// pairs are two bitmap words: the even and odd groups' ballots interleaved.  Needs even G,
// 16-B aligned int64 arrays and 2-B aligned status (jrq_launch_fanout checks; else fanout_eval).
__global__ __launch_bounds__(kFanBlock) void fanout_pair(JrqFanoutArgs a) {
  using i64x2 = __attribute__((ext_vector_type(2))) int64_t;
  __shared__ uint32_t block_listed;
  if (threadIdx.x == 0) block_listed = 0;
  __syncthreads();
  constexpr int kSlots = kFanPerThread / 2;
  const uint32_t pairs = a.G >> 1;
  const uint32_t base = blockIdx.x * (kFanBlock * kSlots) + threadIdx.x;
  i64x2 pc[kSlots], cc[kSlots], ap[kSlots], cf[kSlots], cs[kSlots];
#pragma unroll
  for (int k = 0; k < kSlots; ++k) {  // every load first (a pair past G reads pair 0, unused)
    const uint32_t i = base + k * kFanBlock;
    const size_t g = 2 * static_cast<size_t>(i < pairs ? i : 0u);
    pc[k] = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(a.prev_committed + g));
    cc[k] = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(a.committed + g));
    ap[k] = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(a.last_applied + g));
    cf[k] = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(a.cq_first + g));
    cs[k] = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(a.cq_size + g));
  }
  uint32_t mine = 0;
#pragma unroll
  for (int k = 0; k < kSlots; ++k) {
    const uint32_t i = base + k * kFanBlock;
    const uint32_t i0 = i - (threadIdx.x & 63u);  // this wave's first pair
    if (i0 >= pairs) break;                        // wave-uniform
    uint8_t s0 = kFanNone, s1 = kFanNone;
    if (i < pairs) {
      const size_t g = 2 * static_cast<size_t>(i);
      int64_t f0 = cf[k].x, n0 = cs[k].x, f1 = cf[k].y, n1 = cs[k].y, fc0, fc1;
      s0 = fan_one(pc[k].x, cc[k].x, ap[k].x, f0, n0, fc0);
      s1 = fan_one(pc[k].y, cc[k].y, ap[k].y, f1, n1, fc1);
      i64x2 fc;
      fc.x = fc0;
      fc.y = fc1;
      *reinterpret_cast<i64x2*>(a.first_closure + g) = fc;
      *reinterpret_cast<uint16_t*>(a.status + g) = static_cast<uint16_t>(s0 | (s1 << 8));
      if (f0 != cf[k].x || f1 != cf[k].y) {  // a pop moved firstIndex
        i64x2 nf, nn;
        nf.x = f0;
        nf.y = f1;
        nn.x = n0;
        nn.y = n1;
        *reinterpret_cast<i64x2*>(a.cq_first + g) = nf;
        *reinterpret_cast<i64x2*>(a.cq_size + g) = nn;
      }
    }
    const uint64_t be = __ballot(listed(s0)), bo = __ballot(listed(s1));
    const uint32_t w0 = i0 >> 5;  // bitmap word of this wave's first 64 groups
    if ((threadIdx.x & 63u) == 0) {
      a.listed[w0] = interleave32(be, bo);
      if (2ull * i0 + 64 < a.G) a.listed[w0 + 1] = interleave32(be >> 32, bo >> 32);
    }
    mine += static_cast<uint32_t>(__popcll(be) + __popcll(bo));
  }
  if ((threadIdx.x & 63u) == 0 && mine) atomicAdd(&block_listed, mine);
  __syncthreads();
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

#ifndef JRQ_FANOUT_PAIR
#define JRQ_FANOUT_PAIR 1
#endif

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_fanout(
    const JrqFanoutArgs* a, hipStream_t stream) {
  auto al = [](const void* p, uintptr_t n) { return (reinterpret_cast<uintptr_t>(p) & (n - 1)) == 0; };
  const bool pair = JRQ_FANOUT_PAIR && a->G % 2 == 0 && al(a->prev_committed, 16) &&
                    al(a->committed, 16) && al(a->last_applied, 16) && al(a->cq_first, 16) &&
                    al(a->cq_size, 16) && al(a->first_closure, 16) && al(a->status, 2);
  const uint32_t ntiles = (a->G + jrq::kFanTile - 1) / jrq::kFanTile;
  if (pair)
    hipLaunchKernelGGL(jrq::fanout_pair, dim3(ntiles), dim3(jrq::kFanBlock), 0, stream, *a);
  else
    hipLaunchKernelGGL(jrq::fanout_eval, dim3(ntiles), dim3(jrq::kFanBlock), 0, stream, *a);
  return hipGetLastError();
}
