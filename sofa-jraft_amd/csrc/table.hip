// table.hip -- the resident group table (include/jrq.h jrq_table): BallotBox state of G groups
// kept in HBM across epochs, incremental updates, and an epoch that returns only the groups
// whose commit advanced.
//
// Replaces, for a long-running multi-Raft host, the per-group state and calls of
//   BallotBox.commitAt / appendPendingTask / resetPendingIndex / clearPendingTasks
//   (jraft-core/.../core/BallotBox.java:96-215) and Ballot.grant/isGranted (entity/Ballot.java:
//   100-140), with the formulation of quorum.hip (quorum_core.h).
//
// Kernels:
//   table_states_kernel  group headers (one lane per header; rare: leader changes, conf runs)
//   table_recs_kernel    8-B update records: match of one peer slot / queue size of one group
//   table_epoch_kernel   one epoch over every group, in place; a commit writes lastCommitted
//                        (pendingIndex becomes JRQ_PI_FOLLOWS_LC once), and the group is
//                        appended to a compacted list with one 64-bit atomic per workgroup.
// HBM per group per epoch: reads match 8P + pendingIndex, lastAppended, lastCommitted, conf
// 32 B; writes 8 B lastCommitted + 8 B list entry per committing group.
#include "quorum_core.h"

namespace jrq {

typedef int64_t i64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ i64x2 tld2(const int64_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(p));
}

// Runs of a flagged group: run 0 = the conf word (starts at or before pendingIndex), runs
// 1..kTableMaxRuns-1 in the inline slots (start INT64_MAX = unused: an empty run).
struct TableRuns {
  const JrqTableArgs* t;
  uint32_t g;
  uint64_t c0;
  __device__ int64_t start(uint32_t r) const {
    return r == 0 ? kI64Min : t->xstart[static_cast<size_t>(r - 1) * t->ld + g];
  }
  __device__ uint64_t conf(uint32_t r) const {
    return r == 0 ? c0 : t->xconf[static_cast<size_t>(r - 1) * t->ld + g];
  }
};

// Writes of a committing group: lastCommitted, and pendingIndex -> JRQ_PI_FOLLOWS_LC once.
__device__ __forceinline__ void table_commit_one(const JrqTableArgs& t, uint32_t g, int64_t pr,
                                                 int64_t out) {
  t.lc[g] = out;
  if (pr != kPiFollowsLc) t.pi[g] = kPiFollowsLc;
}

// 1024-thread workgroups of 2048 groups (63 VGPRs: 2 workgroups per CU resident).  The
// compacted list is cut into kTableSegments segments, workgroup b appending to segment
// b % kTableSegments: same-address atomics serialise (~14 ns each, tools/table_probe.hip: one
// counter for 512 workgroups cost 7 us of a 25 us epoch), so each counter sees 1/16 of them,
// and the last arriver of each segment publishes its count -- no global arrival counter.
constexpr uint32_t kTableBlock = kTableBlockGroups / 2;

// The run walk of a group with JRQ_CONF_RUNS, reloading it (L2-hot): lastCommitted after the
// epoch, status, and the writes of a commit.
template <int P>
__device__ __forceinline__ int64_t table_runs_one(const JrqTableArgs& t, uint32_t h, int64_t& pi,
                                               uint8_t& st) {
  const int64_t pr = t.pi[h], lc = t.lc[h], la = t.la[h];
  const uint64_t cw = t.conf[h];
  int64_t m[P];
#pragma unroll
  for (int p = 0; p < P; ++p) m[p] = t.match[static_cast<size_t>(p) * t.ld + h];
  pi = pr == kPiFollowsLc ? lc + 1 : pr;
  int64_t out = lc;
  st = kStNotLeader;
  if (pi != 0) {
    st = mask_out_of_range<P>(m, la);
    const TableRuns R{&t, h, cw & ~kConfRuns};
    out = runs_best<P>(R, kTableMaxRuns, pi, la, lc, m, st);
  }
  if (out > lc) table_commit_one(t, h, pr, out);
  return out - lc;
}

template <int P>
__global__ __launch_bounds__(kTableBlock) JRQ_SGPRS_8WAVES void table_epoch_kernel(JrqTableArgs t) {
  constexpr uint32_t kWaves = kTableBlock / 64;
  __shared__ uint32_t wave_cnt[kWaves];
  __shared__ uint32_t blk_base;
  const uint32_t pairs = (t.G + 1) >> 1;  // ld covers the pad group of an odd G (not a leader)
  const uint32_t tt = blockIdx.x * kTableBlock + threadIdx.x;
  const uint32_t g = tt << 1;
  bool c0 = false, c1 = false, f0 = false, f1 = false;
  uint64_t e0 = 0, e1 = 0;
  if (tt < pairs) {
    const i64x2 pr = tld2(t.pi + g);
    const i64x2 lc = tld2(t.lc + g);
    const i64x2 la = tld2(t.la + g);
    const i64x2 cw = tld2(reinterpret_cast<const int64_t*>(t.conf) + g);
    i64x2 mv[P];
#pragma unroll
    for (int p = 0; p < P; ++p) mv[p] = tld2(t.match + static_cast<size_t>(p) * t.ld + g);
    const int64_t pi0 = pr.x == kPiFollowsLc ? lc.x + 1 : pr.x;
    const int64_t pi1 = pr.y == kPiFollowsLc ? lc.y + 1 : pr.y;
    f0 = static_cast<uint64_t>(cw.x) >> 63;
    f1 = static_cast<uint64_t>(cw.y) >> 63;
    int64_t m0[P], m1[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      m0[p] = mv[p].x;
      m1[p] = mv[p].y;
    }
    int64_t o0, o1;
    uint8_t s0, s1;
    decide_single<P>(pi0, la.x, lc.x, static_cast<uint64_t>(cw.x), m0, o0, s0);
    decide_single<P>(pi1, la.y, lc.y, static_cast<uint64_t>(cw.y), m1, o1, s1);
    // a group with a conf change inside its pending window (JRQ_CONF_RUNS) is decided again
    // below with its runs; its single-conf result here is discarded
    c0 = !f0 && o0 > lc.x;  // decide_single returns lastCommitted unless a commit happened
    c1 = !f1 && o1 > lc.y;
    if (c0 && c1) {
      i64x2 o;
      o.x = o0;
      o.y = o1;
      __builtin_nontemporal_store(o, reinterpret_cast<i64x2*>(t.lc + g));
      // pendingIndex = lastCommittedIndex + 1 from now on (BallotBox.java:131-132): one
      // store per group and leadership, the steady state writes lastCommitted only
      if (pr.x != kPiFollowsLc) t.pi[g] = kPiFollowsLc;
      if (pr.y != kPiFollowsLc) t.pi[g + 1] = kPiFollowsLc;
    } else {
      if (c0) table_commit_one(t, g, pr.x, o0);
      if (c1) table_commit_one(t, g + 1, pr.y, o1);
    }
    if (t.status) {  // a flagged group's status is written by the run walk
      if (g + 1 < t.G && !f0 && !f1)
        __builtin_nontemporal_store(static_cast<uint16_t>(s0 | (s1 << 8)),
                                    reinterpret_cast<uint16_t*>(t.status + g));
      else {
        if (!f0) t.status[g] = s0;
        if (!f1 && g + 1 < t.G) t.status[g + 1] = s1;
      }
    }
    e0 = (static_cast<uint64_t>(o0 - pi0 + 1) << 32) | g;
    e1 = (static_cast<uint64_t>(o1 - pi1 + 1) << 32) | (g + 1);
  }
  // flagged groups walk their conf runs in the lane that holds them, after the fast path's
  // registers are dead (skipped by a wave none of whose groups is flagged).
  // No workgroup barrier: a barrier here measured +4.7 us per 1M-group epoch
  // (tools/table_probe.hip).
  if (__builtin_expect(f0, 0)) {
    int64_t pi;
    uint8_t st;
    const int64_t d = table_runs_one<P>(t, g, pi, st);
    if (t.status) t.status[g] = st;
    c0 = d > 0;
    e0 = (static_cast<uint64_t>(t.lc[g] - pi + 1) << 32) | g;
  }
  if (__builtin_expect(f1, 0)) {
    int64_t pi;
    uint8_t st;
    const int64_t d = table_runs_one<P>(t, g + 1, pi, st);
    if (t.status) t.status[g + 1] = st;
    c1 = d > 0;
    e1 = (static_cast<uint64_t>(t.lc[g + 1] - pi + 1) << 32) | (g + 1);
  }
  // compaction: lane-major order inside a wave, waves in order inside the workgroup; one
  // 64-bit atomic per workgroup ({workgroups done << 32 | entries}) on its segment's counter
  // reserves the workgroup's slice, and the last workgroup of a segment publishes its count
  // and re-zeroes the counter
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t b0 = __ballot(c0), b1 = __ballot(c1);
  const uint64_t below = (1ull << lane) - 1ull;
  const uint32_t pre = __popcll(b0 & below) + __popcll(b1 & below);
  if (lane == 0) wave_cnt[w] = __popcll(b0) + __popcll(b1);
  __syncthreads();
  const uint32_t seg = blockIdx.x % kTableSegments;
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (uint32_t u = 0; u < kWaves; ++u) tot += wave_cnt[u];
    const unsigned long long old = atomicAdd(t.ctr + seg, (1ull << 32) | tot);
    blk_base = seg * t.seg_cap + static_cast<uint32_t>(old);
    const uint32_t seg_blocks = (gridDim.x - seg + kTableSegments - 1) / kTableSegments;
    if (static_cast<uint32_t>(old >> 32) + 1u == seg_blocks) {  // the segment is complete
      t.n_changed[seg] = static_cast<uint32_t>(old) + tot;
      atomicExch(t.ctr + seg, 0ull);
    }
  }
  __syncthreads();
  uint32_t pos = blk_base + pre;
  for (uint32_t u = 0; u < w; ++u) pos += wave_cnt[u];
  if (c0) t.changed[pos++] = e0;
  if (c1) t.changed[pos] = e1;
}

// Group headers: one lane per header (a group appears at most once per call).
__global__ __launch_bounds__(256) void table_states_kernel(JrqTableArgs t, const JrqGroupState* s,
                                                          uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const JrqGroupState st = s[i];
  const uint32_t g = st.group;
  if (g >= t.G || st.num_runs > kTableMaxRuns) {  // counted, reported by jrq_table_check
    atomicAdd(t.invalid, 1u);
    return;
  }
  const uint32_t nr = st.num_runs;
  t.pi[g] = st.pending_index;
  t.la[g] = st.last_appended;
  t.lc[g] = st.last_committed;
  const uint64_t c0 = nr ? (st.run_conf[0] & ~kConfRuns) : 0;
  t.conf[g] = c0 | (nr > 1 ? kConfRuns : 0ull);
#pragma unroll
  for (int k = 1; k < kTableMaxRuns; ++k) {
    const size_t o = static_cast<size_t>(k - 1) * t.ld + g;
    t.xstart[o] = static_cast<uint32_t>(k) < nr ? st.run_start[k] : kI64Max;
    t.xconf[o] = static_cast<uint32_t>(k) < nr ? (st.run_conf[k] & ~kConfRuns) : 0ull;
  }
  if (st.flags & 1u)  // JRQ_STATE_RESET_MATCH: a new leader's replicators start over
    for (uint32_t p = 0; p < t.P; ++p) t.match[static_cast<size_t>(p) * t.ld + g] = st.pending_index - 1;
}

// 8-byte update records (include/jrq.h JRQ_REC): value relative to the group's pendingIndex.
__global__ __launch_bounds__(256) void table_recs_kernel(JrqTableArgs t, const uint64_t* recs,
                                                         uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t r = recs[i];
  const uint32_t f = static_cast<uint32_t>(r & 31u);
  const uint32_t g = static_cast<uint32_t>(r >> 5) & ((1u << 27) - 1u);
  const uint32_t v = static_cast<uint32_t>(r >> 32);
  if (g >= t.G || f > 16u || (f < 16u && f >= t.P)) {  // counted, reported by jrq_table_check
    atomicAdd(t.invalid, 1u);
    return;
  }
  const int64_t pr = t.pi[g], lc = t.lc[g];
  const int64_t val = (pr == kPiFollowsLc ? lc + 1 : pr) - 1 + static_cast<int64_t>(v);
  if (f == 16u) t.la[g] = val;
  else t.match[static_cast<size_t>(f) * t.ld + g] = val;
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_update(
    const JrqTableArgs* a, const JrqGroupState* states, uint32_t n_states, const uint64_t* recs,
    uint32_t n_recs, hipStream_t stream) {
  if (n_states)
    hipLaunchKernelGGL(jrq::table_states_kernel, dim3((n_states + 255) / 256), dim3(256), 0,
                       stream, *a, states, n_states);
  if (n_recs)
    hipLaunchKernelGGL(jrq::table_recs_kernel, dim3((n_recs + 255) / 256), dim3(256), 0, stream,
                       *a, recs, n_recs);
  return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) uint32_t jrq_table_seg_cap(uint32_t G) {
  const uint32_t blocks = (G + jrq::kTableBlockGroups - 1) / jrq::kTableBlockGroups;
  return (blocks + jrq::kTableSegments - 1) / jrq::kTableSegments * jrq::kTableBlockGroups;
}

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_epoch(
    const JrqTableArgs* a, hipStream_t stream) {
  const uint32_t pairs = (a->G + 1) >> 1;
  const dim3 grid((pairs + jrq::kTableBlock - 1) / jrq::kTableBlock), blk(jrq::kTableBlock);
  if (grid.x < jrq::kTableSegments)  // segments no workgroup appends to: count 0
    (void)hipMemsetAsync(a->n_changed + grid.x, 0, 4 * (jrq::kTableSegments - grid.x), stream);
  switch (a->P) {
#define JRQ_CASE(P)                                                                   \
  case P:                                                                             \
    hipLaunchKernelGGL(jrq::table_epoch_kernel<P>, grid, blk, 0, stream, *a);         \
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
