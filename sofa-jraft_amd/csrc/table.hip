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
//                        listed in its wave's fixed slice of the changed list.
//   table_list_*         host variant only: the slices gathered back to back.
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

// Stores at byte offset `off` of a wave-uniform base, as tld2o loads (the base stays in SGPRs).
typedef __attribute__((address_space(1))) i64x2 gi64x2w;
typedef __attribute__((address_space(1))) int64_t gi64w;
typedef __attribute__((address_space(1))) char gcharw;
__device__ __forceinline__ void tst2o(int64_t* base, uint32_t off, i64x2 v);
__device__ __forceinline__ void tst1o(int64_t* base, uint32_t off, int64_t v) {
  gcharw* b = (gcharw*)base;
  asm volatile("" : "+s"(b));
  *reinterpret_cast<gi64w*>(b + off) = v;
}

// Cache policy of the epoch's stores (A/B knob, tools/ab_build.sh): nt -- plain stores measured
// 2 % slower here (21.75 vs 22.14 us), while the pair kernel's are 1.5-7 % faster plain
#ifndef JRQ_TABLE_NT_STORES
#define JRQ_TABLE_NT_STORES 1
#endif
#ifndef JRQ_TABLE_AB_NODECIDE
#define JRQ_TABLE_AB_NODECIDE 0
#endif
#ifndef JRQ_TABLE_AB_NOLIST
#define JRQ_TABLE_AB_NOLIST 0
#endif
// (timing only: 1 = no lastCommitted stores; 2 = lastCommitted stored to a separate row -- the
// first cold xstart row, which a table without conf runs never reads)
#ifndef JRQ_TABLE_AB_LC
#define JRQ_TABLE_AB_LC 0
#endif
template <class T>
__device__ __forceinline__ void st_tab(T v, T* p) {
#if JRQ_TABLE_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void tst2o(int64_t* base, uint32_t off, i64x2 v) {
  gcharw* b = (gcharw*)base;
  asm volatile("" : "+s"(b));
#if JRQ_TABLE_NT_STORES
  __builtin_nontemporal_store(v, reinterpret_cast<gi64x2w*>(b + off));
#else
  *reinterpret_cast<gi64x2w*>(b + off) = v;
#endif
}

// Word `comp` (0/1) of the 16 B lane `src` holds in v (every lane calls it: two ds_bpermute
// per word).
__device__ __forceinline__ int64_t ent_field(const i64x2& v, uint32_t src, uint32_t comp) {
  const int s = static_cast<int>(src);
  const uint32_t xl = __shfl(static_cast<uint32_t>(v.x), s), xh = __shfl(static_cast<uint32_t>(static_cast<uint64_t>(v.x) >> 32), s);
  const uint32_t yl = __shfl(static_cast<uint32_t>(v.y), s), yh = __shfl(static_cast<uint32_t>(static_cast<uint64_t>(v.y) >> 32), s);
  const uint64_t x = (static_cast<uint64_t>(xh) << 32) | xl, y = (static_cast<uint64_t>(yh) << 32) | yl;
  return static_cast<int64_t>(comp ? y : x);
}

// Writes of a committing group: lastCommitted, and pendingIndex -> JRQ_PI_FOLLOWS_LC once.
__device__ __forceinline__ void table_commit_one(const JrqTableArgs& t, uint32_t g, int64_t pr,
                                                 int64_t out) {
  tf(t.lc, t, g) = out;
  if (pr != kPiFollowsLc) tf(t.pi, t, g) = kPiFollowsLc;
}

// The epoch's changed list comes in fixed slices, one per 256-group wave range: wave w (groups
// [256 w, 256 w + 256)) writes its entries at changed[256 w ..] and their count at
// n_changed[w].  No reservation: round 3 staged the entries in LDS and reserved each
// workgroup's share with one 64-bit atomic on 16 segment counters, whose round trip at the end
// of every workgroup (plus the barrier in front of it) cost ~1.5 us of a 21 us epoch
// (round 3's tools/table_probe.hip).
// Shape: 256-thread workgroups, two group pairs per lane -- pair A = groups (256 w + 2 l,
// +1), pair B = pair A + 128, each stream read with 16-B loads (1 KiB per wave instruction),
// every load of both pairs issued before the first decision.  At the 32-bit decision's ~75
// VGPRs one pair per lane fits 6 waves per SIMD: a 1M-group epoch (8192 waves of 128 groups)
// then needs 1.33 rounds of the chip's 6144 wave slots; two pairs per lane at <= 128 VGPRs
// fit 4 waves per SIMD, 4096 waves of 256 groups: one round.
constexpr uint32_t kTableEpochBlock = 64 * kTableBlockWaves;

// One epoch over every group of the table, in place.  The single-conf decision runs in 32-bit
// arithmetic relative to pendingIndex (rel_map / rel_cand, the pair kernel's); groups outside
// rel_domain (never a real group) are decided again with 64-bit arithmetic in a wave-uniform
// pass at the end.
// A group with a conf change inside its pending window (JRQ_CONF_RUNS) is skipped by the
// single-conf decision and walked by its own wave afterwards: its dynamic state (pendingIndex,
// lastCommitted, lastAppended, match) is what its owner lane loaded, left in the wave's slice of
// LDS (the first 16 flagged groups of a wave; a wave-local hand-off, no barrier), and its runs
// come from the wave's flagged-entry slots (table_flags_kernel writes them with every header
// update: only headers change runs), eight lanes per group (one conf run per lane pair, the
// pair splitting the run's new-conf and old-conf q-th largest).  The wave copies its first four
// entries to LDS beside its single-conf loads and counts its flagged groups by ballot.  Beyond 4
// flagged groups in one wave the walk reads the further entries from memory, beyond 16 it
// reloads the group.  No workgroup barrier, no atomics: each wave writes its own list slice and
// count.
template <int P>
__global__ __launch_bounds__(kTableEpochBlock, P <= 5 ? 4 : 2) JRQ_SGPRS_8WAVES void table_epoch_kernel(JrqTableArgs t) {
  constexpr uint32_t kWaves = kTableEpochBlock / 64;
  constexpr uint32_t kHand = 16;  // flagged groups per wave handed over through LDS
  constexpr uint32_t kEntLds = 4; // flagged-entry slots per wave copied to LDS up front
  __shared__ int64_t hand[kWaves][kHand][P + 3];  // {pendingIndex word, lc, la, match[P]}
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  // wave wid holds groups [256 wid, 256 wid + 256): its flagged-entry slots, list slice, count
  const uint32_t wid = blockIdx.x * kWaves + w;
  const uint32_t gA = wid * kTableSlice + 2u * lane;  // pair A = (gA, gA + 1), B = A + 128
  uint64_t* const slice = t.changed + static_cast<size_t>(wid) * kTableSlice;
  int64_t* const tile = t.match + static_cast<size_t>(__builtin_amdgcn_readfirstlane(wid)) * t.ts;
  // The wave's first four flagged-entry slots are loaded up front, beside the single-conf loads,
  // whatever the wave's count: 16 B per lane on lanes 0-15 (entry i = lanes 4i .. 4i + 3), read
  // by the walk through lane shuffles.  (The count is the wave's own ballot of its flagged
  // groups, the flags kernel's count of the same 256 groups: loading the count and branching on
  // it put a full memory round trip in front of every wave's single-conf loads.  Round 3 copied
  // the entries into LDS with an LDS-DMA load; with one in flight the compiler waited for every
  // load of the wave, vmcnt(0), before the first LDS write -- the flagged hand-off -- so pair
  // B's loads held up pair A's decisions.)
  const int64_t* const ent = reinterpret_cast<const int64_t*>(t.flag_ent) + static_cast<size_t>(wid) * kFlagSlots * 8;
  i64x2 ev;
  ev.x = 0;
  ev.y = 0;
  if (lane < 4 * kEntLds) ev = *reinterpret_cast<const i64x2*>(ent + lane * 2);
  // per group k = 0..3 (A.x, A.y, B.x, B.y): live (inside the table), flagged, committing,
  // outside rel_domain; commit value, delta, status
  bool live[2], f[4], c[4], x[4], wpi[4];
  int64_t o[4];
  uint32_t d[4], st4 = 0;
  {
    i64x2 pr[2], lc[2], la[2], cw[2], mv[2][P];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t g = gA + 128u * h;
      live[h] = g < t.G;
      // the wave's tile (one contiguous block: its groups' every hot field), pair offset in it
      const uint32_t go = (2u * lane + 128u * h) * 8u;
      pr[h] = tld2o(tile + P * 256, go);
      lc[h] = tld2o(tile + (P + 2) * 256, go);
      la[h] = tld2o(tile + (P + 1) * 256, go);
      cw[h] = tld2o(tile + (P + 3) * 256, go);
#pragma unroll
      for (int p = 0; p < P; ++p) mv[h][p] = tld2o(tile + p * 256, go);
    }
    uint32_t kbase = 0;  // hand-off ranks: A.x, A.y, B.x, B.y groups in the flags kernel's order
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int h = k >> 1;
      const bool y = k & 1;
      const uint32_t g = gA + 128u * h + (y ? 1u : 0u);
      const int64_t prk = y ? pr[h].y : pr[h].x, lck = y ? lc[h].y : lc[h].x;
      const int64_t lak = y ? la[h].y : la[h].x;
      const uint64_t cwk = static_cast<uint64_t>(y ? cw[h].y : cw[h].x);
      const bool in = live[h] && g < t.G;
      f[k] = in && (cwk >> 63);
      const uint64_t bf = __ballot(f[k]);
      const uint32_t rk = kbase + __popcll(bf & below);
      kbase += __popcll(bf);
      int64_t m[P];
#pragma unroll
      for (int p = 0; p < P; ++p) m[p] = y ? mv[h][p].y : mv[h][p].x;
      if (f[k] && rk < kHand) {  // a flagged group's state -> the wave's hand-off slot
        int64_t* hs = hand[w][rk];
        hs[0] = prk;
        hs[1] = lck;
        hs[2] = lak;
#pragma unroll
        for (int p = 0; p < P; ++p) hs[3 + p] = m[p];
      }
      const int64_t pi = prk == kPiFollowsLc ? lck + 1 : prk;
#if JRQ_TABLE_AB_NODECIDE  // diagnosis only (tools/ab_build.sh): loads and stores, no decision
      uint8_t s = static_cast<uint8_t>(cwk & 1u) | static_cast<uint8_t>(m[P - 1] & 2);
      const uint32_t r = static_cast<uint32_t>(lak - pi + 1);
#else
      RelGroup<P> rg;
      rel_map<P>(pi, lak, m, rg);
      uint8_t s;
      const uint32_t r = rel_cand<P>(cwk, rg, s);
#endif
      s = pi == 0 ? kStNotLeader : s;
      x[k] = in && !f[k] && !rel_domain(pi, lak);
      o[k] = pi - 1 + static_cast<int64_t>(r);
      // a flagged group is decided by the walk (its single-conf result here is discarded)
      c[k] = in && !f[k] && !x[k] && pi != 0 && r >= 1u && o[k] > lck;
      d[k] = r;
      // pendingIndex = lastCommittedIndex + 1 from now on (BallotBox.java:131-132): one store
      // per group and leadership, the steady state writes lastCommitted only
      wpi[k] = prk != kPiFollowsLc;
      st4 |= static_cast<uint32_t>(s) << (8 * k);
    }
  }
  // the single-conf results and their list entries (ballot ranks: one contiguous run per store)
  uint32_t cnt = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t g = gA + 128u * h;
    const bool ca = c[2 * h], cb = c[2 * h + 1];
    const uint32_t go = (2u * lane + 128u * h) * 8u;  // groups g, g + 1 in the wave's tile
#if JRQ_TABLE_AB_LC == 2
    int64_t* const lcb = t.xstart + static_cast<size_t>(__builtin_amdgcn_readfirstlane(wid)) * 256;
#else
    int64_t* const lcb = tile + (P + 2) * 256;
#endif
#if JRQ_TABLE_AB_LC != 1
    if (ca && cb) {
      i64x2 v;
      v.x = o[2 * h];
      v.y = o[2 * h + 1];
      tst2o(lcb, go, v);
    } else {
      if (ca) tst1o(lcb, go, o[2 * h]);
      if (cb) tst1o(lcb, go + 8u, o[2 * h + 1]);
    }
#endif
    if (ca && wpi[2 * h]) tst1o(tile + P * 256, go, kPiFollowsLc);
    if (cb && wpi[2 * h + 1]) tst1o(tile + P * 256, go + 8u, kPiFollowsLc);
    const uint64_t ba = __ballot(ca), bb = __ballot(cb);
#if !JRQ_TABLE_AB_NOLIST  // (diagnosis knob: no list entries)
    if (ca) slice[cnt + __popcll(ba & below)] = (static_cast<uint64_t>(d[2 * h]) << 32) | g;
    if (cb) slice[cnt + __popcll(ba) + __popcll(bb & below)] = (static_cast<uint64_t>(d[2 * h + 1]) << 32) | (g + 1);
#endif
    cnt += __popcll(ba) + __popcll(bb);
    if (t.status && live[h]) {  // a flagged (or 64-bit) group's status is written by its own pass
      const uint32_t s2 = (st4 >> (16 * h)) & 0xFFFFu;
      const bool ka = !f[2 * h] && !x[2 * h], kb = !f[2 * h + 1] && !x[2 * h + 1] && g + 1 < t.G;
      if (ka && kb)
        st_tab(static_cast<uint16_t>(s2), reinterpret_cast<uint16_t*>(t.status + g));
      else {
        if (ka) t.status[g] = static_cast<uint8_t>(s2);
        if (kb) t.status[g + 1] = static_cast<uint8_t>(s2 >> 8);
      }
    }
  }
  // The walk.  Its reads are LDS (the hand-off slots and entries 0-3) except in waves with
  // more than 4 / 16 flagged groups.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (the hand-off slots: this wave's)
  __builtin_amdgcn_wave_barrier();
  // eight lanes per flagged group: run r = (lane >> 1) & 3 of group slot lane >> 3, the lane
  // pair splitting the run's two quorum checks (new conf, old conf: one q-th largest each,
  // joined by one exchange)
  const uint32_t q = lane >> 3, r = (lane >> 1) & 3u, mh = lane & 1u;
  const uint32_t nflag = __popcll(__ballot(f[0])) + __popcll(__ballot(f[1])) +
                         __popcll(__ballot(f[2])) + __popcll(__ballot(f[3]));
  for (uint32_t base = 0; base < nflag; base += 8) {  // (wave-uniform)
    const uint32_t i = base + q;
    bool act = i < nflag;
    // the entry {group, start1, start2, start3, conf0 .. conf3}: run r's start, the next run's
    // start and run r's conf word (entries 0-3 from LDS, later ones from memory; values, not a
    // pointer that could be either: a generic pointer makes flat loads, which wait for every
    // outstanding memory operation)
    int64_t eh = 0, ers = kI64Min, enx = kI64Max;
    uint64_t rc = 0;
    // entries 0-3 from the lanes holding them (every lane shuffles: the wave is converged here)
    const uint32_t ie = i < kEntLds ? i : 0u;
    const int64_t f0 = ent_field(ev, 4u * ie, 0u);
    const int64_t fr = ent_field(ev, 4u * ie + (r >> 1), r & 1u);
    const int64_t fn = ent_field(ev, 4u * ie + ((r + 1) >> 1), (r + 1) & 1u);
    const int64_t fc = ent_field(ev, 4u * ie + ((4u + r) >> 1), (4u + r) & 1u);
    if (act && i < kEntLds) {
      eh = f0;
      if (r != 0) ers = fr;
      if (r != 3) enx = fn;
      rc = static_cast<uint64_t>(fc);
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
        hpr = tf(t.pi, t, h);
        hlc = tf(t.lc, t, h);
        hla = tf(t.la, t, h);
#pragma unroll
        for (int p = 0; p < P; ++p) hm[p] = tf(t.match + p * 256, t, h);
      }
      pi = hpr == kPiFollowsLc ? hlc + 1 : hpr;
      if (pi == 0) {
        st = kStNotLeader;
      } else {
        const int64_t s = rs > pi ? rs : pi;
        const int64_t e = nx == kI64Max ? hla : nx - 1;
        const int64_t ee = e < hla ? e : hla;
        // 32-bit arithmetic relative to pendingIndex for every real group, 64-bit outside
        // rel_domain
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
      uint32_t cc = kx < kp ? kx : kp;
      cc = cc < er ? cc : er;
      cand = cc >= sr ? pi - 1 + static_cast<int64_t>(cc) : kI64Min;
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
    if (commit) slice[cnt + __popcll(bc & below)] = (static_cast<uint64_t>(cand - pi + 1) << 32) | h;
    cnt += __popcll(bc);
  }
  // groups outside rel_domain (negative or huge indexes, 4-billion-entry windows; never a real
  // group): the 64-bit decision from reloaded words, in a wave-uniform branch kept out of the
  // fast path's registers
  if (__builtin_expect(__ballot(x[0] || x[1] || x[2] || x[3]) != 0, 0)) {
#pragma unroll 1
    for (uint32_t k = 0; k < 4; ++k) {
      const bool mine = k == 0 ? x[0] : k == 1 ? x[1] : k == 2 ? x[2] : x[3];
      const uint32_t h = gA + 128u * (k >> 1) + (k & 1u);
      int64_t out = 0, pr = 0, pi = 0, lc = 0;
      uint8_t st = 0;
      if (mine) {
        pr = tf(t.pi, t, h);
        lc = tf(t.lc, t, h);
        const int64_t la = tf(t.la, t, h);
        int64_t m[P];
#pragma unroll
        for (int p = 0; p < P; ++p) m[p] = tf(t.match + p * 256, t, h);
        pi = pr == kPiFollowsLc ? lc + 1 : pr;
        decide_single<P>(pi, la, lc, tf(t.conf, t, h), m, out, st);
        if (t.status) t.status[h] = st;
      }
      const bool commit = mine && out > lc;
      if (commit) table_commit_one(t, h, pr, out);
      const uint64_t bc = __ballot(commit);
      if (commit) slice[cnt + __popcll(bc & below)] = (static_cast<uint64_t>(out - pi + 1) << 32) | h;
      cnt += __popcll(bc);
    }
  }
  if (lane == 0 && static_cast<uint64_t>(wid) * kTableSlice < t.G) t.n_changed[wid] = cnt;
}

// Host variant of the epoch: the slices' counts scanned into offsets (one workgroup; a
// 1M-group table has 8192 slices) and the slices gathered back to back (one wave per slice),
// so that only the entries cross PCIe.  total_out[0] = the number of entries.
constexpr uint32_t kScanBlock = 1024;
__global__ __launch_bounds__(kScanBlock) void table_list_scan_kernel(const uint32_t* __restrict__ n,
                                                                     uint32_t slices,
                                                                     uint32_t* __restrict__ off,
                                                                     uint32_t* __restrict__ total_out) {
  __shared__ uint32_t wsum[kScanBlock / 64];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  for (uint32_t b = 0; b < slices; b += kScanBlock) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t v = i < slices ? n[i] : 0u;
    uint32_t x = v;  // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= static_cast<uint32_t>(o)) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = carry;
    for (uint32_t u = 0; u < w; ++u) before += wsum[u];
    if (i < slices) off[i] = before + x - v;
    __syncthreads();
    if (threadIdx.x == kScanBlock - 1) carry = before + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) total_out[0] = carry;
}

__global__ __launch_bounds__(512) void table_list_gather_kernel(const uint64_t* __restrict__ changed,
                                                                const uint32_t* __restrict__ n,
                                                                const uint32_t* __restrict__ off,
                                                                uint32_t slices,
                                                                uint64_t* __restrict__ out) {
  const uint32_t s = blockIdx.x * 8u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (s >= slices) return;
  const uint32_t k = n[s], o = off[s];
  for (uint32_t i = lane; i < k; i += 64) out[o + i] = changed[static_cast<size_t>(s) * kTableSlice + i];
}

// The flagged-entry slots: per 256-group wave range of the epoch kernel, its groups flagged
// JRQ_CONF_RUNS, each as a 64-B entry {group, start1 | start2, start3 | conf0, conf1 | conf2,
// conf3} (run starts and conf words; unused runs: start INT64_MAX, conf 0), and their count.
// Rebuilt after every update that carries group headers (only headers change runs and flags);
// the waves map exactly as the epoch kernel's (lane l: pairs A = 256 w + 2 l and B = A + 128,
// entries in the order A.x, A.y, B.x, B.y groups by ballot rank), no barrier, no atomics.
constexpr uint32_t kFlagBlock = 64 * kTableBlockWaves;
__global__ __launch_bounds__(kFlagBlock) void table_flags_kernel(JrqTableArgs t) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wid = blockIdx.x * (kFlagBlock / 64) + (threadIdx.x >> 6);
  const uint32_t gA = wid * kTableSlice + 2u * lane;
  const uint64_t below = (1ull << lane) - 1ull;
  int64_t* const ent = reinterpret_cast<int64_t*>(t.flag_ent) + static_cast<size_t>(wid) * kFlagSlots * 8;
  auto put = [&](uint32_t k, uint32_t h) {
    int64_t* e = ent + k * 8;
    e[0] = h;
    for (int r = 1; r < kTableMaxRuns; ++r) e[r] = t.xstart[static_cast<size_t>(r - 1) * t.ld + h];
    e[4] = static_cast<int64_t>(tf(t.conf, t, h) & ~kConfRuns);
    for (int r = 1; r < kTableMaxRuns; ++r)
      e[4 + r] = static_cast<int64_t>(t.xconf[static_cast<size_t>(r - 1) * t.ld + h]);
  };
  uint32_t base = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t g = gA + 128u * h;
    bool f0 = false, f1 = false;
    if (g < t.G) {
      const i64x2 cw = tld2(reinterpret_cast<const int64_t*>(&tf(t.conf, t, g)));
      f0 = static_cast<uint64_t>(cw.x) >> 63;
      f1 = (static_cast<uint64_t>(cw.y) >> 63) && g + 1 < t.G;
    }
    const uint64_t b0 = __ballot(f0), b1 = __ballot(f1);
    if (f0) put(base + __popcll(b0 & below), g);
    if (f1) put(base + __popcll(b0) + __popcll(b1 & below), g + 1);
    base += __popcll(b0) + __popcll(b1);
  }
  if (lane == 0) t.flag_wcnt[wid] = base;
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
  tf(t.pi, t, g) = st.pending_index;
  tf(t.la, t, g) = st.last_appended;
  tf(t.lc, t, g) = st.last_committed;
  const uint64_t c0 = nr ? (st.run_conf[0] & ~kConfRuns) : 0;
  tf(t.conf, t, g) = c0 | (nr > 1 ? kConfRuns : 0ull);  // (table_flags_kernel lists the flagged)
#pragma unroll
  for (int k = 1; k < kTableMaxRuns; ++k) {
    const size_t o = static_cast<size_t>(k - 1) * t.ld + g;
    t.xstart[o] = static_cast<uint32_t>(k) < nr ? st.run_start[k] : kI64Max;
    t.xconf[o] = static_cast<uint32_t>(k) < nr ? (st.run_conf[k] & ~kConfRuns) : 0ull;
  }
  if (st.flags & 1u)  // JRQ_STATE_RESET_MATCH: a new leader's replicators start over
    for (uint32_t p = 0; p < t.P; ++p) tf(t.match + p * 256, t, g) = pi - 1;
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
  const int64_t pr = tf(t.pi, t, g), lc = tf(t.lc, t, g);
  const int64_t pi = pr == kPiFollowsLc ? lc + 1 : pr;
  const int64_t val = pi - 1 + static_cast<int64_t>(v);
  if (f == 16u) {
    // entries pending on a group without a conf run (conf word 0: no header named one) could
    // never be decided as the reference decides them: refused and counted like any bad record
    if (tf(t.conf, t, g) == 0 && pi != 0 && val >= pi) {
      atomicAdd(t.invalid, 1u);
      return;
    }
    tf(t.la, t, g) = val;
  } else {
    tf(t.match + f * 256, t, g) = val;
  }
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_update(
    const JrqTableArgs* a, const JrqGroupState* states, uint32_t n_states, const uint64_t* recs,
    uint32_t n_recs, hipStream_t stream) {
  if (n_states) {
    hipLaunchKernelGGL(jrq::table_states_kernel, dim3((n_states + 255) / 256), dim3(256), 0,
                       stream, *a, states, n_states);
    const uint32_t waves = (a->G + jrq::kTableSlice - 1) / jrq::kTableSlice;
    hipLaunchKernelGGL(jrq::table_flags_kernel, dim3((waves + jrq::kFlagBlock / 64 - 1) / (jrq::kFlagBlock / 64)),
                       dim3(jrq::kFlagBlock), 0, stream, *a);
  }
  if (n_recs)
    hipLaunchKernelGGL(jrq::table_recs_kernel, dim3((n_recs + 255) / 256), dim3(256), 0, stream,
                       *a, recs, n_recs);
  return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_list_gather(
    const uint64_t* changed, const uint32_t* n, uint32_t slices, uint32_t* off, uint32_t* total,
    uint64_t* out, hipStream_t stream) {
  hipLaunchKernelGGL(jrq::table_list_scan_kernel, dim3(1), dim3(jrq::kScanBlock), 0, stream, n, slices,
                     off, total);
  hipLaunchKernelGGL(jrq::table_list_gather_kernel, dim3((slices + 7) / 8), dim3(512), 0, stream,
                     changed, n, off, slices, out);
  return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_epoch(
    const JrqTableArgs* a, hipStream_t stream) {
  const uint32_t waves = (a->G + jrq::kTableSlice - 1) / jrq::kTableSlice;
  const dim3 grid((waves + jrq::kTableEpochBlock / 64 - 1) / (jrq::kTableEpochBlock / 64)), blk(jrq::kTableEpochBlock);
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
