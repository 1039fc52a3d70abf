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

// Acks past the queue would throw ArrayIndexOutOfBoundsException and change nothing
// (BallotBox.java:107-109): that peer grants no entry in this epoch.
template <int P>
__device__ __forceinline__ uint8_t mask_out_of_range(int64_t (&m)[P], int64_t la) {
  uint8_t st = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const bool oor = m[p] > la;
    st |= oor ? kStOutOfRange : 0;
    m[p] = oor ? kI64Min : m[p];
  }
  return st;
}

// One group with a single conf word (no conf change inside the pending window).
template <int P>
__device__ __forceinline__ void decide_single(int64_t pi, int64_t la, int64_t lc, uint64_t cw,
                                              int64_t (&m)[P], int64_t& out, uint8_t& st_out) {
  uint8_t st = mask_out_of_range<P>(m, la);
  if ((cw & 0xFFFFu) == 0 && la >= pi) st |= kStEmptyConf;
  int64_t cand = run_bound<P>(m, cw);
  cand = cand < la ? cand : la;
  const int64_t best = (cand >= pi && cand > lc) ? cand : lc;
  // commitAt returns false when not the leader (BallotBox.java:101-103): state unchanged
  out = pi == 0 ? lc : best;
  st_out = pi == 0 ? kStNotLeader : st;
}

// General path: one lane per group, optional conf runs.  Every load of the group is
// issued before any decision, so a group costs one memory round trip.
template <int P>
__global__ __launch_bounds__(256) void quorum_epoch_kernel(JrqQuorumArgs a) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < a.G; g += stride) {
    const int64_t pi = a.pending_index[g];
    const int64_t lc = a.last_committed[g];
    const int64_t la = a.last_appended[g];
    int64_t m[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m[p] = a.match[static_cast<size_t>(p) * a.match_ld + g];
    if (a.run_off == nullptr) {
      const uint64_t cw = a.conf[g];
      int64_t out;
      uint8_t st;
      decide_single<P>(pi, la, lc, cw, m, out, st);
      a.committed[g] = out;
      a.status[g] = st;
      continue;
    }
    const uint32_t r0 = a.run_off[g], r1 = a.run_off[g + 1];
    if (pi == 0) {
      a.committed[g] = lc;
      a.status[g] = kStNotLeader;
      continue;
    }
    uint8_t st = mask_out_of_range<P>(m, la);
    int64_t best = lc;
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
    a.committed[g] = best;
    a.status[g] = st;
  }
}

typedef int64_t i64x2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ i64x2 ld2(const int64_t* p) {
  const i64x2* q = reinterpret_cast<const i64x2*>(p);
  if (NT) return __builtin_nontemporal_load(q);
  return *q;
}

// Fast path (no run table, 16-B aligned arrays, even match_ld): one lane decides two
// adjacent groups per unit; every stream is read with 16-byte loads (1 KiB per wave
// instruction) and the two status bytes are stored as one 16-bit word.  A lane takes U
// units 256 pairs apart (its workgroup's block of 256*U pairs) and issues every load of
// all U units before the first decision; NT marks the streams non-temporal (read once,
// never re-read: no point keeping them in L2 / MALL).
template <int P, int U, bool NT>
__global__ __launch_bounds__(256) void quorum_epoch_pair_kernel(JrqQuorumArgs a) {
  const uint32_t pairs = a.G >> 1;
  const uint32_t step = gridDim.x * 256u * U;
  for (uint32_t t0 = blockIdx.x * 256u * U + threadIdx.x; t0 < pairs; t0 += step) {
    i64x2 pi[U], lc[U], la[U], cw[U], m[U][P];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t t = t0 + 256u * u;
      if (t >= pairs) continue;
      const uint32_t g = t << 1;
      pi[u] = ld2<NT>(a.pending_index + g);
      lc[u] = ld2<NT>(a.last_committed + g);
      la[u] = ld2<NT>(a.last_appended + g);
      cw[u] = ld2<NT>(reinterpret_cast<const int64_t*>(a.conf) + g);
#pragma unroll
      for (int p = 0; p < P; ++p) m[u][p] = ld2<NT>(a.match + static_cast<size_t>(p) * a.match_ld + g);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t t = t0 + 256u * u;
      if (t >= pairs) continue;
      const uint32_t g = t << 1;
      int64_t m0[P], m1[P];
#pragma unroll
      for (int p = 0; p < P; ++p) {
        m0[p] = m[u][p].x;
        m1[p] = m[u][p].y;
      }
      int64_t o0, o1;
      uint8_t s0, s1;
      decide_single<P>(pi[u].x, la[u].x, lc[u].x, static_cast<uint64_t>(cw[u].x), m0, o0, s0);
      decide_single<P>(pi[u].y, la[u].y, lc[u].y, static_cast<uint64_t>(cw[u].y), m1, o1, s1);
      i64x2 out;
      out.x = o0;
      out.y = o1;
      const uint16_t st = static_cast<uint16_t>(s0 | (s1 << 8));
      if (NT) {
        __builtin_nontemporal_store(out, reinterpret_cast<i64x2*>(a.committed + g));
        __builtin_nontemporal_store(st, reinterpret_cast<uint16_t*>(a.status + g));
      } else {
        *reinterpret_cast<i64x2*>(a.committed + g) = out;
        *reinterpret_cast<uint16_t*>(a.status + g) = st;
      }
    }
  }
  // odd G: the last group goes through the scalar decision
  if ((a.G & 1u) && blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t g = a.G - 1;
    int64_t m[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m[p] = a.match[static_cast<size_t>(p) * a.match_ld + g];
    int64_t out;
    uint8_t st;
    decide_single<P>(a.pending_index[g], a.last_appended[g], a.last_committed[g], a.conf[g], m,
                     out, st);
    a.committed[g] = out;
    a.status[g] = st;
  }
}

// K successive epochs of the same groups in one launch (hard part 4: a
// 10k-group epoch is launch-bound).  Between epochs the group state moves as BallotBox
// moves it: a commit sets lastCommittedIndex and pendingIndex = lastCommittedIndex + 1
// (BallotBox.java:131-134); a group that is not the leader stays so.  Epoch k reads its
// own match snapshot and lastAppended (entries appended since); the conf is per group.
// One lane per group; the loads of 4 epochs are issued before their decisions (8 measured
// slower on C2: 31.6 vs 27.8 us for 64 epochs).
template <int P>
__global__ __launch_bounds__(256) void quorum_epochs_kernel(JrqQuorumArgs a, uint32_t K,
                                                            uint64_t match_eld, uint64_t la_eld) {
  constexpr uint32_t kEpochUnroll = 4;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < a.G; g += stride) {
    int64_t pi = a.pending_index[g];
    int64_t lc = a.last_committed[g];
    const uint64_t cw = a.conf[g];
    for (uint32_t k0 = 0; k0 < K; k0 += kEpochUnroll) {
      int64_t m[kEpochUnroll][P], la[kEpochUnroll];
#pragma unroll
      for (uint32_t u = 0; u < kEpochUnroll; ++u) {
        if (k0 + u >= K) break;
        const size_t k = k0 + u;
        la[u] = a.last_appended[k * la_eld + g];
#pragma unroll
        for (int p = 0; p < P; ++p)
          m[u][p] = a.match[k * match_eld + static_cast<size_t>(p) * a.match_ld + g];
      }
#pragma unroll
      for (uint32_t u = 0; u < kEpochUnroll; ++u) {
        if (k0 + u >= K) break;
        const size_t k = k0 + u;
        int64_t out;
        uint8_t st;
        decide_single<P>(pi, la[u], lc, cw, m[u], out, st);
        a.committed[k * a.G + g] = out;
        a.status[k * a.G + g] = st;
        if (pi != 0 && out > lc) pi = out + 1;
        lc = out;
      }
    }
  }
}

// ------------------------------------------------------------------ lease ---
// NodeImpl.checkDeadNodes0 (jraft-core/.../core/NodeImpl.java:1970-2000) for one conf:
// the leader itself is alive; another member is alive when now - lastRpcSendTimestamp <=
// leaderLeaseTimeoutMs (Java long arithmetic: wrapping subtraction); the lease starts at
// the oldest alive timestamp (Long.MAX_VALUE if none); the check passes when
// alive >= quorum (peers.size()/2 + 1).
template <int P>
__device__ __forceinline__ bool alive_quorum(const int64_t (&ts)[P], uint32_t mask, uint32_t q,
                                             uint32_t self, int64_t now, int64_t timeout,
                                             int64_t& start, uint16_t& dead) {
  uint32_t alive = 0;
  start = kI64Max;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const bool member = (mask >> p) & 1u;
    const bool is_self = static_cast<uint32_t>(p) == self;
    const int64_t age = static_cast<int64_t>(static_cast<uint64_t>(now) - static_cast<uint64_t>(ts[p]));
    const bool fresh = age <= timeout;
    alive += (member && (is_self || fresh)) ? 1u : 0u;
    start = (member && !is_self && fresh && ts[p] < start) ? ts[p] : start;
    dead |= (member && !is_self && !fresh) ? static_cast<uint16_t>(1u << p) : 0;
  }
  return alive >= q;
}

// NodeImpl.handleStepDownTimeout (:2003-2016): check the conf, then the old conf when it
// is not empty; every passing check moves lastLeaderTimestamp to its lease start.
template <int P>
__global__ __launch_bounds__(256) void lease_check_kernel(JrqLeaseArgs a) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < a.G; g += stride) {
    int64_t ts[P];
#pragma unroll
    for (int p = 0; p < P; ++p)
      ts[p] = __builtin_nontemporal_load(a.last_rpc_ts + static_cast<size_t>(p) * a.ld + g);
    const uint64_t cw = __builtin_nontemporal_load(a.conf + g);
    const uint32_t self = a.self_slot[g];
    int64_t lead = a.lease_start[g];
    uint16_t dead = 0;
    int64_t start;
    uint8_t ok = 0;
    if (alive_quorum<P>(ts, cw & 0xFFFFu, (cw >> 32) & 0xFFu, self, a.now_ms, a.lease_timeout_ms,
                        start, dead)) {
      lead = start;
      ok |= 1;
    }
    const uint32_t omask = (cw >> 16) & 0xFFFFu;
    if (omask != 0) {
      if (alive_quorum<P>(ts, omask, (cw >> 40) & 0xFFu, self, a.now_ms, a.lease_timeout_ms,
                          start, dead)) {
        lead = start;
        ok |= 2;
      }
    } else {
      ok |= 2;  // no old conf to check
    }
    a.ok[g] = ok;
    a.lease_start[g] = lead;
    if (a.dead) a.dead[g] = dead;
  }
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_lease(
    const JrqLeaseArgs* args, int num_cus, hipStream_t stream) {
  const uint64_t need = (static_cast<uint64_t>(args->G) + 255) / 256;
  const uint64_t cap = static_cast<uint64_t>(num_cus) * 8;
  const dim3 grid(static_cast<unsigned>(need < cap ? (need ? need : 1) : cap)), blk(256);
  switch (args->num_peers) {
#define JRQ_CASE(P)                                                                    \
  case P:                                                                              \
    hipLaunchKernelGGL(jrq::lease_check_kernel<P>, grid, blk, 0, stream, *args); \
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

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_quorum(
    const JrqQuorumArgs* args, int num_cus, hipStream_t stream) {
  const dim3 blk(256);
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  const JrqQuorumArgs& a = *args;
  const bool pair = a.run_off == nullptr && (a.match_ld & 1u) == 0 && al16(a.match) &&
                    al16(a.pending_index) && al16(a.last_appended) && al16(a.last_committed) &&
                    al16(a.conf) && al16(a.committed) &&
                    (reinterpret_cast<uintptr_t>(a.status) & 1u) == 0 && a.G >= 2;
  // pair-kernel variant (A/B knob JRQ_Q_VARIANT): 0 = 1 unit/lane, 1 = 1 unit/lane with
  // non-temporal streams (default: 4.96 vs 4.58-4.74 TB/s on C3), 2 = 2 units/lane,
  // 3 = 2 units/lane non-temporal
  static const int variant = [] {
    const char* v = std::getenv("JRQ_Q_VARIANT");
    return v ? std::atoi(v) : 1;
  }();
  const int units = (variant == 2 || variant == 3) ? 2 : 1;
  // enough 256-thread blocks for one lane per group (pair: per two per unit), at most 8 per CU
  const uint64_t lanes = pair ? ((a.G >> 1) + units - 1) / units : a.G;
  const uint64_t need = (lanes + 255) / 256;
  const uint64_t cap = static_cast<uint64_t>(num_cus) * 8;
  const int grid = static_cast<int>(need < cap ? (need ? need : 1) : cap);
  switch (args->num_peers) {
#define JRQ_CASE(P)                                                                            \
  case P:                                                                                      \
    if (!pair)                                                                                 \
      hipLaunchKernelGGL(jrq::quorum_epoch_kernel<P>, dim3(grid), blk, 0, stream, *args);      \
    else if (variant == 0)                                                                     \
      hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<P, 1, false>), dim3(grid), blk, 0,    \
                         stream, *args);                                                       \
    else if (variant == 2)                                                                     \
      hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<P, 2, false>), dim3(grid), blk, 0,    \
                         stream, *args);                                                       \
    else if (variant == 3)                                                                     \
      hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<P, 2, true>), dim3(grid), blk, 0,     \
                         stream, *args);                                                       \
    else                                                                                       \
      hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<P, 1, true>), dim3(grid), blk, 0,     \
                         stream, *args);                                                       \
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

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_quorum_epochs(
    const JrqQuorumArgs* args, uint32_t K, uint64_t match_eld, uint64_t la_eld, int num_cus,
    hipStream_t stream) {
  const uint64_t need = (static_cast<uint64_t>(args->G) + 255) / 256;
  const uint64_t cap = static_cast<uint64_t>(num_cus) * 8;
  const dim3 grid(static_cast<unsigned>(need < cap ? (need ? need : 1) : cap)), blk(256);
  switch (args->num_peers) {
#define JRQ_CASE(P)                                                                      \
  case P:                                                                                \
    hipLaunchKernelGGL(jrq::quorum_epochs_kernel<P>, grid, blk, 0, stream, *args, K,     \
                       match_eld, la_eld);                                               \
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
