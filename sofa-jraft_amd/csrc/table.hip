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
// HBM per group per epoch: reads match 4P (u32 words against the group's match base) +
// pendingIndex, lastAppended, lastCommitted, conf 32 B; writes 8 B lastCommitted + 4 B list
// delta per committing group, 36 B of map + count per 256 groups.
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

// Four u32 (one lane's groups of a match row) at byte offset `off` of a wave-uniform base.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
__device__ __forceinline__ u32x4 tld4o(const int64_t* base, uint32_t off) {
  gchar* b = (gchar*)base;
  asm volatile("" : "+s"(b));
  return __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(b + off));
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

// Writes of a committing group: lastCommitted, pendingIndex -> JRQ_PI_FOLLOWS_LC once, and, when
// the new pendingIndex moves the group's match base (once per 2^30 entries), its match words
// re-expressed against the new base (m = base + word; words below it saturate at 0).
template <int P>
__device__ __forceinline__ void table_rebase(const JrqTableArgs& t, uint32_t g, int64_t b0, int64_t b1) {
  const uint64_t sh = static_cast<uint64_t>(b1 - b0);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const uint32_t s = tm(t, p, g);
    tm(t, p, g) = s > sh ? static_cast<uint32_t>(s - sh) : 0u;
  }
}
template <int P>
__device__ __forceinline__ void table_commit_one(const JrqTableArgs& t, uint32_t g, int64_t pr,
                                                 int64_t pi, int64_t out) {
  tf(t.lc, t, g) = out;
  if (pr != kPiFollowsLc) tf(t.pi, t, g) = kPiFollowsLc;
  const int64_t b0 = mbase(pi), b1 = mbase(out + 1);
  if (b1 != b0) table_rebase<P>(t, g, b0, b1);
}

// Absolute match of a u32 word under base b.
__device__ __forceinline__ int64_t mabs(int64_t b, uint32_t s) { return b + static_cast<int64_t>(s); }

// The changed list of an epoch comes in fixed slices, one per 256-group wave range: slice s
// (groups [256 s, 256 s + 256), decided by one wave) is 256 words at changed + 256 s: words
// 0-3 a 256-bit map of the groups whose commit advanced (bit i = group 256 s + i), then from
// byte 32 their deltas commit - pendingIndex + 1 as u32, in group order; n_changed[s] = how
// many.  12 B per committing group + 4 B per 256 groups, where round 4's (delta << 32 | group)
// words took 16 (the list's 8 B per group cost ~2 us of a 19-us C3 epoch:
// tools/probes/table_shape_probe.hip, profiles/r05b_table_diag.json).  No reservation, no
// atomics: round 3 reserved each workgroup's share with a 64-bit atomic, ~1.5 us per epoch.
constexpr uint32_t kSliceMapWords = 4;

__device__ __forceinline__ uint64_t spread_bits(uint32_t x) {  // bit i -> bit 2i
  uint64_t v = x;
  v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
  v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
  v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
  v = (v | (v << 2)) & 0x3333333333333333ull;
  v = (v | (v << 1)) & 0x5555555555555555ull;
  return v;
}

// Shape: 256-thread workgroups, four groups per lane as two pairs -- pair A = groups (256 w +
// 2 l, +1), pair B = pair A + 128: each int64 stream read with 16-B loads (1 KiB per wave
// instruction), each u32 match row with one 16-B load per lane (its four groups: mslot()),
// every load issued before the first decision: P + 8 load instructions per wave for 256
// groups.  At <= 128 VGPRs 4 waves per SIMD fit, 4096 waves of 256 groups: a 1M-group epoch in
// one round.  (Round 4 measured one pair per lane at 512 threads the same on the read side:
// tools/probes/table_shape_probe.hip.)
constexpr uint32_t kTableEpochBlock = 64 * kTableBlockWaves;

// One epoch over every group of the table, in place.  The single-conf decision runs in 32-bit
// arithmetic relative to pendingIndex (rel_cand, the pair kernel's) straight from the u32 match
// words: r = word - (pi - 1 - base) for a word inside the window; groups outside rel_domain
// (never a real group) are decided again with 64-bit arithmetic in a wave-uniform pass.
// A group with a conf change inside its pending window (JRQ_CONF_RUNS) is skipped by the
// single-conf decision and walked by its own wave afterwards: its dynamic state (pendingIndex,
// lastCommitted, lastAppended, absolute match) is what its owner lane loaded, left in the wave's
// slice of LDS (the first 16 flagged groups of a wave; a wave-local hand-off, no barrier), and
// its runs come from the wave's flagged-entry slots (table_flags_kernel writes them with every
// header update: only headers change runs), eight lanes per group (one conf run per lane pair,
// the pair splitting the run's new-conf and old-conf q-th largest).  The walk hands each
// group's delta back to its owner lane through LDS, so the wave writes its list slice once, in
// group order, after every decision.  No workgroup barrier, no atomics.
template <int P>
__global__ __launch_bounds__(kTableEpochBlock, P <= 5 ? 4 : 2) JRQ_SGPRS_8WAVES void table_epoch_kernel(JrqTableArgs t) {
  constexpr uint32_t kWaves = kTableEpochBlock / 64;
  constexpr uint32_t kHand = 16;  // flagged groups per wave handed over through LDS
  constexpr uint32_t kEntLds = 4; // flagged-entry slots per wave copied to lanes up front
  __shared__ int64_t hand[kWaves][kHand][P + 3];   // {pendingIndex word, lc, la, match[P]}
  __shared__ uint32_t walked[kWaves][kFlagSlots];  // the walk's delta per flagged rank (0: none)
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  // wave wid holds groups [256 wid, 256 wid + 256): its flagged-entry slots, list slice, count
  const uint32_t wid = blockIdx.x * kWaves + w;
  const uint32_t gA = wid * kTableSlice + 2u * lane;  // pair A = (gA, gA + 1), B = A + 128
  uint64_t* const slice = t.changed + static_cast<size_t>(wid) * kTableSlice;
  int64_t* const tile = reinterpret_cast<int64_t*>(t.match) + static_cast<size_t>(__builtin_amdgcn_readfirstlane(wid)) * t.ts;
  const int64_t* const ent = reinterpret_cast<const int64_t*>(t.flag_ent) + static_cast<size_t>(wid) * kFlagSlots * 8;
  // The wave's first four flagged-entry slots, loaded up front beside the single-conf loads
  // whatever the wave's count: 16 B per lane on lanes 0-15 (entry i = lanes 4i .. 4i + 3), read
  // by the walk through lane shuffles.  (Loading the count first and branching on it put a
  // memory round trip in front of every wave's loads.)
  i64x2 ev;
  ev.x = 0;
  ev.y = 0;
  if (lane < 4 * kEntLds) ev = *reinterpret_cast<const i64x2*>(ent + lane * 2);
  // per group k = 0..3 (A.x, A.y, B.x, B.y): live (inside the table), flagged, committing,
  // outside rel_domain; commit delta, flagged rank, status
  bool live[2], f[4], c[4], x[4], wpi[4], xb[4];
  uint32_t d[4], rk[4], st4 = 0;
  int64_t outv[4], bk[4];
  {
    i64x2 pr[2], lc[2], la[2], cw[2];
    u32x4 mq[P];
    const uint32_t go = 16u * lane;  // byte offset of pair A in a 2-KiB int64 row
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      live[h] = gA + 128u * h < t.G;
      pr[h] = tld2o(tile + 128 * P, go + 1024u * h);
      lc[h] = tld2o(tile + 128 * P + 512, go + 1024u * h);
      la[h] = tld2o(tile + 128 * P + 256, go + 1024u * h);
      cw[h] = tld2o(tile + 128 * P + 768, go + 1024u * h);
    }
#pragma unroll
    for (int p = 0; p < P; ++p) mq[p] = tld4o(tile + 128 * p, go);  // groups A.x, A.y, B.x, B.y
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
      rk[k] = kbase + __popcll(bf & below);
      kbase += __popcll(bf);
      uint32_t s[P];
#pragma unroll
      for (int p = 0; p < P; ++p) s[p] = k == 0 ? mq[p].x : k == 1 ? mq[p].y : k == 2 ? mq[p].z : mq[p].w;
      const int64_t pi = prk == kPiFollowsLc ? lck + 1 : prk;
      const int64_t b = mbase(pi);
      if (f[k] && rk[k] < kHand) {  // a flagged group's state -> the wave's hand-off slot
        int64_t* hs = hand[w][rk[k]];
        hs[0] = prk;
        hs[1] = lck;
        hs[2] = lak;
#pragma unroll
        for (int p = 0; p < P; ++p) hs[3 + p] = mabs(b, s[p]);
      }
#if JRQ_TABLE_AB_NODECIDE  // diagnosis only (tools/ab_build.sh): loads and stores, no decision
      uint8_t st = static_cast<uint8_t>(cwk & 1u) | static_cast<uint8_t>(s[P - 1] & 2u);
      const uint32_t r = static_cast<uint32_t>(lak - pi + 1);
#else
      // the window [pi, la] in the words' terms: a word u maps to r = u - o in [1, W] (o =
      // pi - 1 - base < 2^30), an ack past lastAppended is u > la - base
      RelGroup<P> rg;
      const uint32_t o = static_cast<uint32_t>(pi - 1 - b), lab = static_cast<uint32_t>(lak - b);
      rg.W = lak >= pi ? static_cast<uint32_t>(lak - pi) + 1u : 0u;
      rg.st = 0;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const uint32_t dd = s[p] - o - 1u;
        rg.st |= s[p] > lab ? kStOutOfRange : 0;
        rg.r[p] = dd < rg.W ? dd + 1u : 0u;
      }
      uint8_t st;
      const uint32_t r = rel_cand<P>(cwk, rg, st);
#endif
      st = pi == 0 ? kStNotLeader : st;
      // (the u32 words need a window below 2^31, which header / record checks guarantee)
      x[k] = in && !f[k] && !(pi == 0 || (pi > 0 && pi < (int64_t{1} << 62) &&
                                            (lak < pi || lak - pi < int64_t{0x7FFFFFFF})));
      // a flagged group is decided by the walk (its single-conf result here is discarded)
      c[k] = in && !f[k] && !x[k] && pi != 0 && r >= 1u && pi - 1 + static_cast<int64_t>(r) > lck;
      d[k] = r;
      outv[k] = pi - 1 + static_cast<int64_t>(r);
      bk[k] = b;
      // pendingIndex = lastCommittedIndex + 1 from now on (BallotBox.java:131-132): one store
      // per group and leadership, the steady state writes lastCommitted only; a commit that
      // moves the match base (once per 2^30 entries) re-expresses the group's words
      wpi[k] = prk != kPiFollowsLc;
      xb[k] = c[k] && mbase(outv[k] + 1) != b;
      st4 |= static_cast<uint32_t>(st) << (8 * k);
    }
    // the single-conf commits' lastCommitted, a pair at a time (the stores leave before the walk)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool ca = c[2 * h], cb = c[2 * h + 1];
      const uint32_t off = go + 1024u * h;
#if JRQ_TABLE_AB_LC != 1
      int64_t* const lcb = tile + 128 * P + 512;
      if (ca && cb) {
        i64x2 v;
        v.x = outv[2 * h];
        v.y = outv[2 * h + 1];
        tst2o(lcb, off, v);
      } else {
        if (ca) tst1o(lcb, off, outv[2 * h]);
        if (cb) tst1o(lcb, off + 8u, outv[2 * h + 1]);
      }
#endif
      if (ca && wpi[2 * h]) tst1o(tile + 128 * P, off, kPiFollowsLc);
      if (cb && wpi[2 * h + 1]) tst1o(tile + 128 * P, off + 8u, kPiFollowsLc);
    }
    if (__builtin_expect(__ballot(xb[0] || xb[1] || xb[2] || xb[3]) != 0, 0)) {
#pragma unroll 1
      for (uint32_t k = 0; k < 4; ++k) {
        const bool mine = k == 0 ? xb[0] : k == 1 ? xb[1] : k == 2 ? xb[2] : xb[3];
        const int64_t b0 = k == 0 ? bk[0] : k == 1 ? bk[1] : k == 2 ? bk[2] : bk[3];
        const int64_t o = k == 0 ? outv[0] : k == 1 ? outv[1] : k == 2 ? outv[2] : outv[3];
        if (mine) table_rebase<P>(t, gA + 128u * (k >> 1) + (k & 1u), b0, mbase(o + 1));
      }
    }
  }
  if (t.status) {  // (a flagged or 64-bit group's status is written by its own pass)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t g = gA + 128u * h;
      if (!live[h]) continue;
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
    // start and run r's conf word (entries 0-3 from the lanes holding them, later ones from
    // memory; values, not a pointer that could be either: a generic pointer makes flat loads,
    // which wait for every outstanding memory operation)
    int64_t eh = 0, ers = kI64Min, enx = kI64Max;
    uint64_t rc = 0;
    const uint32_t ie = i < kEntLds ? i : 0u;  // (every lane shuffles: the wave is converged)
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
        const int64_t bb = mbase(hpr == kPiFollowsLc ? hlc + 1 : hpr);
#pragma unroll
        for (int p = 0; p < P; ++p) hm[p] = mabs(bb, tm(t, p, h));
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
      if (commit) table_commit_one<P>(t, h, hpr, pi, cand);
      walked[w][i] = commit ? static_cast<uint32_t>(cand - pi + 1) : 0u;
    }
  }
  // groups outside rel_domain (negative or huge indexes; never a real group): the 64-bit
  // decision from reloaded words, in a wave-uniform branch kept out of the fast path's registers
  if (__builtin_expect(__ballot(x[0] || x[1] || x[2] || x[3]) != 0, 0)) {
#pragma unroll 1
    for (uint32_t k = 0; k < 4; ++k) {
      const bool mine = k == 0 ? x[0] : k == 1 ? x[1] : k == 2 ? x[2] : x[3];
      const uint32_t h = gA + 128u * (k >> 1) + (k & 1u);
      if (!mine) continue;
      const int64_t pr = tf(t.pi, t, h), lc = tf(t.lc, t, h), la = tf(t.la, t, h);
      const int64_t pi = pr == kPiFollowsLc ? lc + 1 : pr;
      const int64_t bb = mbase(pi);
      int64_t m[P];
#pragma unroll
      for (int p = 0; p < P; ++p) m[p] = mabs(bb, tm(t, p, h));
      int64_t out = 0;
      uint8_t st = 0;
      decide_single<P>(pi, la, lc, tf(t.conf, t, h), m, out, st);
      if (t.status) t.status[h] = st;
      const bool commit = out > lc;
      if (commit) table_commit_one<P>(t, h, pr, pi, out);
      const uint32_t dk = commit ? static_cast<uint32_t>(out - pi + 1) : 0u;
      if (k == 0) { c[0] = commit; d[0] = dk; }
      if (k == 1) { c[1] = commit; d[1] = dk; }
      if (k == 2) { c[2] = commit; d[2] = dk; }
      if (k == 3) { c[3] = commit; d[3] = dk; }
    }
  }
  // the walked groups' results back to their owner lanes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (f[k]) {
      const uint32_t dk = walked[w][rk[k]];
      c[k] = dk != 0;
      d[k] = dk;
    }
  // the list slice, in group order: the map (pair A's groups are bits 0-127 as 2 l, 2 l + 1,
  // pair B's bits 128-255), then the deltas at their ranks (a lane's committing groups sit at
  // consecutive ranks: one 8-B store per pair when both commit)
  const uint64_t bA0 = __ballot(c[0]), bA1 = __ballot(c[1]), bB0 = __ballot(c[2]), bB1 = __ballot(c[3]);
  const uint32_t nA = __popcll(bA0) + __popcll(bA1);
  const uint32_t cnt = nA + __popcll(bB0) + __popcll(bB1);
  // (a wave past the table's last slice -- the grid is whole workgroups -- owns no slice: the
  // caller's list has room for jrq_table_slices(t) slices only)
  const bool owns = static_cast<uint64_t>(wid) * kTableSlice < t.G;
#if !JRQ_TABLE_AB_NOLIST  // (diagnosis knob: no list)
  if (lane < kSliceMapWords && owns) {
    const uint64_t lo = lane < 2 ? bA0 : bB0, hi = lane < 2 ? bA1 : bB1;
    const uint32_t sh = (lane & 1u) * 32u;
    slice[lane] = spread_bits(static_cast<uint32_t>(lo >> sh)) | (spread_bits(static_cast<uint32_t>(hi >> sh)) << 1);
  }
  uint32_t* const deltas = reinterpret_cast<uint32_t*>(slice + kSliceMapWords);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint64_t b0 = h ? bB0 : bA0, b1 = h ? bB1 : bA1;
    const uint32_t at = (h ? nA : 0u) + __popcll(b0 & below) + __popcll(b1 & below);
    const bool c0 = c[2 * h], c1 = c[2 * h + 1];
    if (c0 && c1 && !(at & 1u)) {
      *reinterpret_cast<uint64_t*>(deltas + at) = static_cast<uint64_t>(d[2 * h]) | (static_cast<uint64_t>(d[2 * h + 1]) << 32);
    } else {
      if (c0) deltas[at] = d[2 * h];
      if (c1) deltas[at + (c0 ? 1u : 0u)] = d[2 * h + 1];
    }
  }
#endif
  if (lane == 0 && owns) t.n_changed[wid] = cnt;
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

// One wave per slice: lane l takes the slice's groups 4 l .. 4 l + 3 (a nibble of its map),
// their ranks from the map's popcounts, and writes each listed group as the host list's word
// (delta << 32 | group).
__global__ __launch_bounds__(512) void table_list_gather_kernel(const uint64_t* __restrict__ changed,
                                                                const uint32_t* __restrict__ n,
                                                                const uint32_t* __restrict__ off,
                                                                uint32_t slices,
                                                                uint64_t* __restrict__ out) {
  const uint32_t s = blockIdx.x * 8u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (s >= slices || n[s] == 0) return;
  const uint64_t* sl = changed + static_cast<size_t>(s) * kTableSlice;
  const uint32_t* deltas = reinterpret_cast<const uint32_t*>(sl + kSliceMapWords);
  const uint32_t wd = lane >> 4, sh = 4u * (lane & 15u);
  const uint64_t word = sl[wd];
  uint32_t at = off[s] + __popcll(word & ((1ull << sh) - 1ull));
  uint32_t rank = __popcll(word & ((1ull << sh) - 1ull));
  for (uint32_t u = 0; u < wd; ++u) {
    const uint32_t pc = __popcll(sl[u]);
    at += pc;
    rank += pc;
  }
  uint32_t nib = static_cast<uint32_t>(word >> sh) & 15u;
  while (nib) {
    const uint32_t b = __builtin_ctz(nib);
    nib &= nib - 1u;
    out[at++] = (static_cast<uint64_t>(deltas[rank++]) << 32) | (s * kTableSlice + 4u * lane + b);
  }
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
  // counted, reported by jrq_table_check: out-of-range group or run count, a leader with
  // pending entries but no conf run (conf word 0 = quorum 0, which would grant every entry), a
  // negative pendingIndex or one past 2^62, and a pending queue longer than a Java ArrayList
  // holds (2^31 - 1: the u32 match words rely on it)
  // lastAppended below pendingIndex - 1 (a queue of negative size, which no BallotBox holds: the
  // epoch's u32 out-of-range test assumes lastAppended >= the match base)
  if (g >= t.G || nr > kTableMaxRuns || (nr == 0 && pi != 0 && st.last_appended >= pi) || pi < 0 ||
      pi >= (int64_t{1} << 62) || (pi > 0 && st.last_appended < pi - 1) ||
      (pi > 0 && st.last_appended >= pi && st.last_appended - pi >= int64_t{0x7FFFFFFF})) {
    atomicAdd(t.invalid, 1u);
    return;
  }
  // the group's match base before and after: its words re-expressed when it moves
  const int64_t pr0 = tf(t.pi, t, g), lc0 = tf(t.lc, t, g);
  const int64_t b0 = mbase(pr0 == kPiFollowsLc ? lc0 + 1 : pr0), b1 = mbase(pi);
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
  if (st.flags & 1u) {  // JRQ_STATE_RESET_MATCH: a new leader's replicators start over
    const uint32_t w = pi > 0 ? static_cast<uint32_t>(pi - 1 - b1) : 0u;
    for (uint32_t p = 0; p < t.P; ++p) tm(t, p, g) = w;
  } else if (b1 > b0) {
    const uint64_t d = static_cast<uint64_t>(b1 - b0);
    for (uint32_t p = 0; p < t.P; ++p) {
      const uint32_t v = tm(t, p, g);
      tm(t, p, g) = v > d ? static_cast<uint32_t>(v - d) : 0u;
    }
  } else if (b1 < b0) {
    // A lower base without RESET_MATCH (outside the host's contract: within a leadership
    // pendingIndex only grows, Replicator.java:1387-1401; resetPendingIndex resets the matches).
    // A word of 0 means "at or below the old base" -- its true match is unknown, so it stays 0
    // under the new base (never grants) instead of reading back as exactly the old base, which
    // could count as an ack of entries no peer acknowledged.  Others saturate.
    const uint64_t d = static_cast<uint64_t>(b0 - b1);
    for (uint32_t p = 0; p < t.P; ++p) {
      const uint32_t w0 = tm(t, p, g);
      const uint64_t v = w0 + d;
      tm(t, p, g) = w0 == 0 ? 0u : v > 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(v);
    }
  }
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
    // never be decided as the reference decides them, and a queue longer than an ArrayList
    // (2^31 - 1 entries) is not one BallotBox can hold: refused and counted like any bad record
    if ((tf(t.conf, t, g) == 0 && pi != 0 && val >= pi) || v > 0x7FFFFFFFu) {
      atomicAdd(t.invalid, 1u);
      return;
    }
    tf(t.la, t, g) = val;
  } else {  // the u32 word against the group's match base (saturating: past 2^32 is out of range)
    const int64_t rel = val - mbase(pi);
    tm(t, f, g) = rel <= 0 ? 0u : (rel > 0xFFFFFFFFll ? 0xFFFFFFFFu : static_cast<uint32_t>(rel));
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
