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

// 16 B at byte offset `off` of a wave-uniform row base: the scalar-base form of the load (one
// 32-bit offset VGPR shared by every row instead of a 64-bit address per row; with 64-bit
// addresses the epoch kernel ran out of its 64 VGPRs and spilled loaded words mid-issue).  The
// empty asm pins the base in SGPRs, so the compiler cannot fold a row's p * ld into a per-lane
// 64-bit address again.
typedef __attribute__((address_space(1))) const i64x2 gi64x2;
typedef __attribute__((address_space(1))) const char gchar;
__device__ __forceinline__ i64x2 tld2o(const int64_t* base, uint32_t off) {
  gchar* b = (gchar*)base;
  asm volatile("" : "+s"(b));
  return __builtin_nontemporal_load(reinterpret_cast<const gi64x2*>(b + off));
}

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

// The run walk of one flagged group, run r of it on lane r of an aligned lane quad (the table
// holds at most kTableMaxRuns = 4 runs): each lane loads the group (the quad's loads of it
// coalesce) and its run's start, next start and conf word, all in one batch; the quad then
// max-reduces the runs' candidates.  Returns the group's candidate (kI64Min: none) and status.
template <int P>
__device__ __forceinline__ int64_t table_run_lane(const JrqTableArgs& t, uint32_t h, uint32_t r,
                                                  int64_t& pr, int64_t& lc, int64_t& pi,
                                                  uint8_t& st) {
  static_assert(kTableMaxRuns == 4, "one run per lane of a quad");
  pr = t.pi[h];
  lc = t.lc[h];
  const int64_t la = t.la[h];
  const size_t o = static_cast<size_t>(r) * t.ld + h;  // run r's slot is r - 1; next run's is r
  const uint64_t cw = r == 0 ? (t.conf[h] & ~kConfRuns) : t.xconf[o - t.ld];
  const int64_t rs = r == 0 ? kI64Min : t.xstart[o - t.ld];
  const int64_t nx = r + 1 < kTableMaxRuns ? t.xstart[o] : kI64Max;
  int64_t m[P];
#pragma unroll
  for (int p = 0; p < P; ++p) m[p] = t.match[static_cast<size_t>(p) * t.ld + h];
  pi = pr == kPiFollowsLc ? lc + 1 : pr;
  if (pi == 0) {
    st = kStNotLeader;
    return kI64Min;
  }
  st = mask_out_of_range<P>(m, la);
  const int64_t s = rs > pi ? rs : pi;
  const int64_t e = nx == kI64Max ? la : nx - 1;
  return run_candidate<P>(m, cw, s, e < la ? e : la, st);
}

// One epoch over every group of the table.  1024-thread workgroups of 2048 groups (two per
// lane, 16-B loads), 2 resident per CU.
// A group with a conf change inside its pending window (JRQ_CONF_RUNS) is skipped by the
// single-conf decision and walked by its own wave afterwards: its dynamic state (pendingIndex,
// lastCommitted, lastAppended, match) is what its owner lane loaded, left in the wave's slice of
// LDS (the first 16 flagged groups of a wave; a wave-local hand-off, no barrier), and its runs
// come from the wave's flagged-entry slots (table_flags_kernel writes them with every header
// update: only headers change runs), spread over a lane quad by shuffles, one conf run per lane
// (the table holds at most 4).  The wave copies its first four entries to LDS beside its
// single-conf loads and counts its flagged groups by ballot, and it walks them before issuing
// any store, so a flagged group costs no dependent round trip to memory, no wait for the wave's
// stores and no workgroup barrier (round 2 deferred flagged groups to an LDS list behind a
// barrier and reloaded them: +25 % on C3 with 1 % flagged, tools/flag_probe.hip; round 3's
// first walk came after the stores and read entries through a generic pointer, and every flat
// load drained the wave's stores).  Beyond 4 flagged groups in one wave the walk reads the
// further entries from memory, beyond 16 it reloads the group too.
// The one barrier left is the compaction's: list entries are staged per wave in LDS, and one
// 64-bit atomic per workgroup ({done << 32 | entries}) on its segment's counter (workgroup b
// -> segment b % kTableSegments: same-address atomics serialise, ~14 ns each,
// tools/table_probe.hip) reserves its slice; the last workgroup of a segment publishes the
// segment's count and re-zeroes the counter.
template <int P>
__global__ __launch_bounds__(kTableBlock, 8) JRQ_SGPRS_8WAVES void table_epoch_kernel(JrqTableArgs t) {
  constexpr uint32_t kWaves = kTableBlock / 64;
  constexpr uint32_t kHand = 16;  // flagged groups per wave handed over through LDS
  constexpr uint32_t kEntLds = 4; // flagged-entry slots per wave copied to LDS up front
  __shared__ uint32_t wave_cnt[kWaves];
  __shared__ uint64_t staged[kWaves][128];
  __shared__ int64_t hand[kWaves][kHand][P + 3];  // {pendingIndex word, lc, la, match[P]}
  __shared__ __attribute__((aligned(16))) int64_t ent4[kWaves][kEntLds][8];  // entries 0-3
  __shared__ uint32_t blk_base;
  const uint32_t pairs = (t.G + 1) >> 1;
  const uint32_t tt = blockIdx.x * kTableBlock + threadIdx.x;
  const uint32_t g = tt << 1;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  // The wave's first four flagged-entry slots go straight to its LDS slice (an LDS-DMA load,
  // 256 B per wave, ~1 % of the epoch's bytes; no registers held across the single-conf path),
  // whatever the wave's count: the count is the wave's own ballot of its flagged groups (the
  // flags kernel's count of the same 128 groups).  Loading the count and branching on it here
  // put a full memory round trip in front of every wave's single-conf loads.
  const uint32_t wid = blockIdx.x * kWaves + w;
  const int64_t* const ent = reinterpret_cast<const int64_t*>(t.flag_ent) + static_cast<size_t>(wid) * kFlagSlots * 8;
  if (lane < 4 * kEntLds)  // lane l: bytes 16 l .. 16 l + 15 of entries 0-3 (64 B each)
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ent + lane * 2), &ent4[w][0][0], 16, 0, 0);
  bool c0 = false, c1 = false, f0 = false, f1 = false, w0 = false, w1 = false;
  int64_t o0 = 0, o1 = 0;
  uint32_t s01 = 0;
  if (tt < pairs) {
    const uint32_t go = g * 8u;  // (g < 2^27)
    const i64x2 pr = tld2o(t.pi, go);
    const i64x2 lc = tld2o(t.lc, go);
    const i64x2 la = tld2o(t.la, go);
    const i64x2 cw = tld2o(reinterpret_cast<const int64_t*>(t.conf), go);
    i64x2 mv[P];
#pragma unroll
    for (int p = 0; p < P; ++p) mv[p] = tld2o(t.match + static_cast<size_t>(p) * t.ld, go);
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
    // a flagged group's state -> the wave's hand-off slot of its rank (the flags kernel's
    // entry order: the first groups of the pairs, then the second ones)
    const uint64_t bf0 = __ballot(f0), bf1 = __ballot(f1);
    const uint32_t k0 = __popcll(bf0 & below), k1 = __popcll(bf0) + __popcll(bf1 & below);
    if (f0 && k0 < kHand) {
      int64_t* hs = hand[w][k0];
      hs[0] = pr.x;
      hs[1] = lc.x;
      hs[2] = la.x;
#pragma unroll
      for (int p = 0; p < P; ++p) hs[3 + p] = m0[p];
    }
    if (f1 && k1 < kHand) {
      int64_t* hs = hand[w][k1];
      hs[0] = pr.y;
      hs[1] = lc.y;
      hs[2] = la.y;
#pragma unroll
      for (int p = 0; p < P; ++p) hs[3 + p] = m1[p];
    }
    uint8_t s0, s1;
    // (the 64-bit decision: the 32-bit one of the pair kernel, decide_single_rel, took this
    // kernel past its 64 VGPRs -- 10 spills at P = 5)
    decide_single<P>(pi0, la.x, lc.x, static_cast<uint64_t>(cw.x), m0, o0, s0);
    decide_single<P>(pi1, la.y, lc.y, static_cast<uint64_t>(cw.y), m1, o1, s1);
    // a flagged group is decided by the walk (its single-conf result here is discarded)
    c0 = !f0 && o0 > lc.x;  // decide_single returns lastCommitted unless a commit happened
    c1 = !f1 && o1 > lc.y;
    // pendingIndex = lastCommittedIndex + 1 from now on (BallotBox.java:131-132): one store per
    // group and leadership, the steady state writes lastCommitted only
    w0 = pr.x != kPiFollowsLc;
    w1 = pr.y != kPiFollowsLc;
    s01 = s0 | (static_cast<uint32_t>(s1) << 8);
    // list entries -> the wave's slice of LDS (ballot prefixes, no atomics)
    const uint64_t b0 = __ballot(c0), b1 = __ballot(c1);
    if (c0) staged[w][__popcll(b0 & below)] = (static_cast<uint64_t>(o0 - pi0 + 1) << 32) | g;
    if (c1) staged[w][__popcll(b0) + __popcll(b1 & below)] = (static_cast<uint64_t>(o1 - pi1 + 1) << 32) | (g + 1);
  }
  uint32_t cnt = __popcll(__ballot(c0)) + __popcll(__ballot(c1));
  // The walk, before any of the wave's stores: its reads (LDS, and the entries past the first
  // four from memory) then wait for nothing but themselves.  With the single-conf stores issued
  // first, every wait of the walk (vmcnt counts stores too) drained the wave's stores.
  // Flagged group i of the wave on quad i % 16, one conf run per lane.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (the hand-off slots: this wave's)
  __builtin_amdgcn_wave_barrier();
  // eight lanes per flagged group: run r = (lane >> 1) & 3 of group slot lane >> 3, the lane
  // pair splitting the run's two quorum checks (new conf, old conf: one q-th largest each,
  // joined by one shuffle) -- the walk's VALU is what a flagged wave adds, and the two
  // sorting networks were most of it
  const uint32_t q = lane >> 3, r = (lane >> 1) & 3u, mh = lane & 1u;
  // this wave's flagged groups (f0 / f1 are false on lanes past the table)
  const uint32_t nflag = __popcll(__ballot(f0)) + __popcll(__ballot(f1));
  for (uint32_t base = 0; base < nflag; base += 8) {  // (wave-uniform)
    const uint32_t i = base + q;
    bool act = i < nflag;
    // the entry {group, start1, start2, start3, conf0 .. conf3}: run r's start, the next run's
    // start and run r's conf word (entries 0-3 from LDS, later ones from memory; values, not a
    // pointer that could be either: a generic pointer makes flat loads, which wait for every
    // outstanding memory operation)
    int64_t eh = 0, ers = kI64Min, enx = kI64Max;
    uint64_t rc = 0;
    if (act && i < kEntLds) {
      eh = ent4[w][i][0];
      if (r != 0) ers = ent4[w][i][r];
      if (r != 3) enx = ent4[w][i][r + 1];
      rc = static_cast<uint64_t>(ent4[w][i][4 + r]);
    } else if (act) {
      const int64_t* e = ent + static_cast<size_t>(i) * 8;
      eh = e[0];
      if (r != 0) ers = e[r];
      if (r != 3) enx = e[r + 1];
      rc = static_cast<uint64_t>(e[4 + r]);
    }
    const uint32_t h = static_cast<uint32_t>(eh);
    const int64_t rs = ers, nx = enx;
    act = act && h < t.G;  // (the flags kernel writes only table groups: a guard, not a case)
    int64_t cand64 = kI64Min, hpr = 0, hlc = 0, hla = 0, pi = 0;
    uint8_t st = 0;
    bool relp = false;
    uint32_t kx = 0xFFFFFFFFu, sr = 0, er = 0;
    if (act) {
      int64_t hm[P];
      if (i < kHand) {  // from the owner lane, through LDS
        const int64_t* hs = hand[w][i];
        hpr = hs[0];
        hlc = hs[1];
        hla = hs[2];
#pragma unroll
        for (int p = 0; p < P; ++p) hm[p] = hs[3 + p];
      } else {  // more flagged groups than hand-off slots: reload (rare)
        hpr = t.pi[h];
        hlc = t.lc[h];
        hla = t.la[h];
#pragma unroll
        for (int p = 0; p < P; ++p) hm[p] = t.match[static_cast<size_t>(p) * t.ld + h];
      }
      pi = hpr == kPiFollowsLc ? hlc + 1 : hpr;
      if (pi == 0) {
        st = kStNotLeader;
      } else {
        const int64_t s = rs > pi ? rs : pi;
        const int64_t e = nx == kI64Max ? hla : nx - 1;
        const int64_t ee = e < hla ? e : hla;
        // the walk runs when every load of the wave has landed and the VALU is the busy
        // unit: 32-bit arithmetic relative to pendingIndex for every real group (half the
        // VALU of the 64-bit rank count), 64-bit outside rel_domain
        if (rel_domain(pi, hla)) {
          RelGroup<P> rg;
          rel_map<P>(pi, hla, hm, rg);
          st = rg.st;
          if (ee >= s) {  // run_candidate_rel, this lane's half of it
            if ((rc & 0xFFFFu) == 0) st |= kStEmptyConf;
            relp = true;
            sr = static_cast<uint32_t>(s - pi) + 1u;
            er = static_cast<uint32_t>(ee - pi) + 1u;
            const uint32_t msk = static_cast<uint32_t>((rc >> (mh ? 16 : 0)) & 0xFFFFu);
            const uint32_t qq = static_cast<uint32_t>((rc >> (mh ? 40 : 32)) & 0xFFu);
            kx = qq == 0 ? rg.W : kth_largest_rel<P>(rg.r, msk, qq);
          }
        } else {  // both lanes of the pair: the whole 64-bit run_candidate
          st = mask_out_of_range<P>(hm, hla);
          cand64 = run_candidate<P>(hm, rc, s, ee, st);
        }
      }
    }
    // the pair's two bounds (every lane exchanges: the wave stays converged)
    const uint32_t kp = dpp32<kDppXor1>(kx);
    int64_t cand = cand64;
    if (relp) {
      uint32_t c = kx < kp ? kx : kp;
      c = c < er ? c : er;
      cand = c >= sr ? pi - 1 + static_cast<int64_t>(c) : kI64Min;
    }
    // max over the group's 8 lanes, complete on its lead lane (the lane pairs agree already)
    cand = max(cand, dpp64<kDppXor2>(cand));
    cand = max(cand, dpp64<kDppHalfMirror>(cand));
    uint32_t s32 = st;
    s32 |= dpp32<kDppXor1>(s32);
    s32 |= dpp32<kDppXor2>(s32);
    s32 |= dpp32<kDppHalfMirror>(s32);
    const bool lead = (lane & 7u) == 0;
    const bool commit = act && lead && cand > hlc;  // pi == 0 (not the leader): kI64Min
    if (act && lead) {
      if (t.status) t.status[h] = static_cast<uint8_t>(s32);
      if (commit) table_commit_one(t, h, hpr, cand);
    }
    const uint64_t bc = __ballot(commit);
    if (commit) staged[w][cnt + __popcll(bc & below)] = (static_cast<uint64_t>(cand - pi + 1) << 32) | h;
    cnt += __popcll(bc);
  }
  // the single-conf results
  if (tt < pairs) {
    if (c0 && c1) {
      i64x2 o;
      o.x = o0;
      o.y = o1;
      __builtin_nontemporal_store(o, reinterpret_cast<i64x2*>(t.lc + g));
      if (w0) t.pi[g] = kPiFollowsLc;
      if (w1) t.pi[g + 1] = kPiFollowsLc;
    } else {
      if (c0) {
        t.lc[g] = o0;
        if (w0) t.pi[g] = kPiFollowsLc;
      }
      if (c1) {
        t.lc[g + 1] = o1;
        if (w1) t.pi[g + 1] = kPiFollowsLc;
      }
    }
    if (t.status) {  // a flagged group's status is written by the walk
      if (g + 1 < t.G && !f0 && !f1)
        __builtin_nontemporal_store(static_cast<uint16_t>(s01), reinterpret_cast<uint16_t*>(t.status + g));
      else {
        if (!f0) t.status[g] = static_cast<uint8_t>(s01);
        if (!f1 && g + 1 < t.G) t.status[g + 1] = static_cast<uint8_t>(s01 >> 8);
      }
    }
  }
  if (lane == 0) wave_cnt[w] = cnt;
  lds_barrier();  // (the results' stores stay in flight)
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
  lds_barrier();
  uint32_t pos = blk_base;
  for (uint32_t u = 0; u < w; ++u) pos += wave_cnt[u];
  for (uint32_t i = lane; i < cnt; i += 64) t.changed[pos + i] = staged[w][i];
}

// The flagged-entry slots: per 128-group wave range of the epoch kernel, its groups flagged
// JRQ_CONF_RUNS, each as a 64-B entry {group, start1 | start2, start3 | conf0, conf1 | conf2,
// conf3} (run starts and conf words; unused runs: start INT64_MAX, conf 0), and their count.
// Rebuilt after every update that carries group headers (only headers change runs and flags);
// the waves map exactly as the epoch kernel's (1024-thread workgroups, two groups per lane),
// no barrier, no atomics.
constexpr uint32_t kFlagBlock = kTableBlockGroups / 2;
__global__ __launch_bounds__(kFlagBlock) void table_flags_kernel(JrqTableArgs t) {
  const uint32_t pairs = (t.G + 1) >> 1;
  const uint32_t tt = blockIdx.x * kFlagBlock + threadIdx.x;
  const uint32_t g = tt << 1;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wid = blockIdx.x * (kFlagBlock / 64) + (threadIdx.x >> 6);
  bool f0 = false, f1 = false;
  if (tt < pairs) {
    const i64x2 cw = tld2(reinterpret_cast<const int64_t*>(t.conf) + g);
    f0 = static_cast<uint64_t>(cw.x) >> 63;
    f1 = (static_cast<uint64_t>(cw.y) >> 63) && g + 1 < t.G;
  }
  const uint64_t below = (1ull << lane) - 1ull;
  const uint64_t b0 = __ballot(f0), b1 = __ballot(f1);
  int64_t* const ent = reinterpret_cast<int64_t*>(t.flag_ent) + static_cast<size_t>(wid) * kFlagSlots * 8;
  auto put = [&](uint32_t k, uint32_t h) {
    int64_t* e = ent + k * 8;
    e[0] = h;
    for (int r = 1; r < kTableMaxRuns; ++r) e[r] = t.xstart[static_cast<size_t>(r - 1) * t.ld + h];
    e[4] = static_cast<int64_t>(t.conf[h] & ~kConfRuns);
    for (int r = 1; r < kTableMaxRuns; ++r)
      e[4 + r] = static_cast<int64_t>(t.xconf[static_cast<size_t>(r - 1) * t.ld + h]);
  };
  if (f0) put(__popcll(b0 & below), g);
  if (f1) put(__popcll(b0) + __popcll(b1 & below), g + 1);
  if (lane == 0) t.flag_wcnt[wid] = __popcll(b0) + __popcll(b1);
}

// Group headers: one lane per header (a group appears at most once per call).
__global__ __launch_bounds__(256) void table_states_kernel(JrqTableArgs t, const JrqGroupState* s,
                                                          uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const JrqGroupState st = s[i];
  const uint32_t g = st.group;
  const uint32_t nr = st.num_runs;
  // pendingIndex resolved (JRQ_PI_FOLLOWS_LC = lastCommitted + 1)
  const int64_t pi = st.pending_index == kPiFollowsLc ? st.last_committed + 1 : st.pending_index;
  // counted, reported by jrq_table_check: out-of-range group or run count, and a leader with
  // pending entries but no conf run (conf word 0 = quorum 0, which would grant every entry)
  if (g >= t.G || nr > kTableMaxRuns || (nr == 0 && pi != 0 && st.last_appended >= pi)) {
    atomicAdd(t.invalid, 1u);
    return;
  }
  t.pi[g] = st.pending_index;
  t.la[g] = st.last_appended;
  t.lc[g] = st.last_committed;
  const uint64_t c0 = nr ? (st.run_conf[0] & ~kConfRuns) : 0;
  t.conf[g] = c0 | (nr > 1 ? kConfRuns : 0ull);  // (table_flags_kernel lists the flagged)
#pragma unroll
  for (int k = 1; k < kTableMaxRuns; ++k) {
    const size_t o = static_cast<size_t>(k - 1) * t.ld + g;
    t.xstart[o] = static_cast<uint32_t>(k) < nr ? st.run_start[k] : kI64Max;
    t.xconf[o] = static_cast<uint32_t>(k) < nr ? (st.run_conf[k] & ~kConfRuns) : 0ull;
  }
  if (st.flags & 1u)  // JRQ_STATE_RESET_MATCH: a new leader's replicators start over
    for (uint32_t p = 0; p < t.P; ++p) t.match[static_cast<size_t>(p) * t.ld + g] = pi - 1;
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
  const int64_t pi = pr == kPiFollowsLc ? lc + 1 : pr;
  const int64_t val = pi - 1 + static_cast<int64_t>(v);
  if (f == 16u) {
    // entries pending on a group without a conf run (conf word 0: no header named one) could
    // never be decided as the reference decides them: refused and counted like any bad record
    if (t.conf[g] == 0 && pi != 0 && val >= pi) {
      atomicAdd(t.invalid, 1u);
      return;
    }
    t.la[g] = val;
  } else {
    t.match[static_cast<size_t>(f) * t.ld + g] = val;
  }
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_update(
    const JrqTableArgs* a, const JrqGroupState* states, uint32_t n_states, const uint64_t* recs,
    uint32_t n_recs, hipStream_t stream) {
  if (n_states) {
    hipLaunchKernelGGL(jrq::table_states_kernel, dim3((n_states + 255) / 256), dim3(256), 0,
                       stream, *a, states, n_states);
    const uint32_t pairs = (a->G + 1) >> 1;
    hipLaunchKernelGGL(jrq::table_flags_kernel, dim3((pairs + jrq::kFlagBlock - 1) / jrq::kFlagBlock),
                       dim3(jrq::kFlagBlock), 0, stream, *a);
  }
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
