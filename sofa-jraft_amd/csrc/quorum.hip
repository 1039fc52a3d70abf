// quorum.hip -- batched BallotBox.commitAt evaluation for millions of Raft groups (gfx950).
//
// Replaces, for G groups per launch, the per-(entry, ack) loop of
//   BallotBox.commitAt     jraft-core/.../core/BallotBox.java:96-139
//   Ballot.grant/isGranted jraft-core/.../entity/Ballot.java:100-140
// including joint-consensus ballots (Ballot.init with conf + oldConf, :63-85).
//
// Formulation (exact under the Replicator invariant that a peer's acks on pending
// indices are contiguous from pendingIndex -- Replicator.java:1387-1392, 1401; see
// DESIGN.md §Quorum for the proof and the oracle replay that pins it):
//   entry i in [pendingIndex, lastAppended] is granted  <=>
//     |{p in newMask : match[p] >= i}| >= newQ  and  |{p in oldMask : match[p] >= i}| >= oldQ
//   <=> i <= kth(newMask, newQ) and i <= kth(oldMask, oldQ)     (kth = q-th largest match)
//   so a conf run [s, e] commits up to min(e, kN, kO) when that is >= max(s, pendingIndex),
//   and committed = max(lastCommitted, max over runs).
// The result does not depend on the order of the epoch's acks, as for the reference
// (every grant is idempotent and a commit takes the max granted index).
//
// One lane per group, grid-stride; every per-peer match row is a coalesced int64 stream.
// HBM-bound: 8P + 41 bytes per group decision (roofline).
#include "jrq_device.h"

namespace jrq {

constexpr int64_t kI64Min = INT64_MIN;
constexpr int64_t kI64Max = INT64_MAX;

// q-th largest of v[p] over the peers in `mask` (q >= 1); kI64Min if fewer than q members.
// P <= 16: rank-by-counting, branch-free, P^2 compares on 64-bit values in registers.
template <int P>
__device__ __forceinline__ int64_t kth_largest(const int64_t (&v)[P], uint32_t mask, uint32_t q) {
  int64_t best = kI64Min;
#pragma unroll
  for (int a = 0; a < P; ++a) {
    // members at least as large as v[a] (ties count): v[a] qualifies as a q-th-largest bound
    uint32_t ge = 0;
#pragma unroll
    for (int b = 0; b < P; ++b) ge += ((mask >> b) & 1u) & (v[b] >= v[a] ? 1u : 0u);
    const bool ok = ((mask >> a) & 1u) && ge >= q;
    best = (ok && v[a] > best) ? v[a] : best;
  }
  return best;
}

template <int P>
__device__ __forceinline__ int64_t run_bound(const int64_t (&m)[P], uint64_t cw) {
  const uint32_t nmask = static_cast<uint32_t>(cw & 0xFFFFu);
  const uint32_t omask = static_cast<uint32_t>((cw >> 16) & 0xFFFFu);
  const uint32_t nq = static_cast<uint32_t>((cw >> 32) & 0xFFu);
  const uint32_t oq = static_cast<uint32_t>((cw >> 40) & 0xFFu);
  // quorum 0 is always met (Ballot.isGranted: quorum <= 0, Ballot.java:138-140)
  const int64_t kn = nq == 0 ? kI64Max : kth_largest<P>(m, nmask, nq);
  const int64_t ko = oq == 0 ? kI64Max : kth_largest<P>(m, omask, oq);
  return kn < ko ? kn : ko;
}

template <int P>
__global__ __launch_bounds__(256) void quorum_epoch_kernel(JrqQuorumArgs a) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < a.G; g += stride) {
    const int64_t pi = a.pending_index[g];
    const int64_t lc = a.last_committed[g];
    if (pi == 0) {  // commitAt returns false: not the leader (BallotBox.java:101-103)
      a.committed[g] = lc;
      a.status[g] = kStNotLeader;
      continue;
    }
    const int64_t la = a.last_appended[g];
    int64_t m[P];
    uint8_t st = 0;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int64_t v = a.match[static_cast<size_t>(p) * a.match_ld + g];
      // an ack past the queue would throw ArrayIndexOutOfBoundsException and change
      // nothing (BallotBox.java:107-109): that peer grants no entry in this epoch
      const bool oor = v > la;
      st |= oor ? kStOutOfRange : 0;
      m[p] = oor ? kI64Min : v;
    }
    int64_t best = lc;
    if (a.run_off == nullptr) {
      const uint64_t cw = a.conf[g];
      if ((cw & 0xFFFFu) == 0 && la >= pi) st |= kStEmptyConf;
      int64_t cand = run_bound<P>(m, cw);
      cand = cand < la ? cand : la;
      best = (cand >= pi && cand > best) ? cand : best;
    } else {
      const uint32_t r0 = a.run_off[g], r1 = a.run_off[g + 1];
      for (uint32_t r = r0; r < r1; ++r) {
        const int64_t s = (r == r0) ? pi : (a.run_start[r] > pi ? a.run_start[r] : pi);
        const int64_t e = (r + 1 < r1) ? a.run_start[r + 1] - 1 : la;
        const int64_t ee = e < la ? e : la;
        if (ee < s) continue;  // run entirely committed already (or empty)
        const uint64_t cw = a.run_conf[r];
        if ((cw & 0xFFFFu) == 0) st |= kStEmptyConf;
        int64_t cand = run_bound<P>(m, cw);
        cand = cand < ee ? cand : ee;
        best = (cand >= s && cand > best) ? cand : best;
      }
    }
    a.committed[g] = best;
    a.status[g] = st;
  }
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_quorum(const JrqQuorumArgs* args, int grid, hipStream_t stream) {
  const dim3 blk(256);
  switch (args->num_peers) {
#define JRQ_CASE(P)                                                                  \
  case P:                                                                            \
    hipLaunchKernelGGL(jrq::quorum_epoch_kernel<P>, dim3(grid), blk, 0, stream, *args); \
    break;
    JRQ_CASE(1) JRQ_CASE(2) JRQ_CASE(3) JRQ_CASE(4) JRQ_CASE(5) JRQ_CASE(6) JRQ_CASE(7)
    JRQ_CASE(8) JRQ_CASE(9) JRQ_CASE(10) JRQ_CASE(11) JRQ_CASE(12) JRQ_CASE(13) JRQ_CASE(14)
    JRQ_CASE(15) JRQ_CASE(16)
#undef JRQ_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
