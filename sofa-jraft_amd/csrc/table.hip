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
// delta per committing group, 20 B of map + count per 128 groups.
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

// A committing group whose new pendingIndex moves its match base (once per 2^30 entries): its
// match words re-expressed against the new base (m = base + word; words below it saturate at 0).
template <int P>
__device__ __forceinline__ void table_rebase(const JrqTableArgs& t, uint32_t g, int64_t b0, int64_t b1) {
  const uint64_t sh = static_cast<uint64_t>(b1 - b0);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const uint32_t s = tm(t, p, g);
    tm(t, p, g) = s > sh ? static_cast<uint32_t>(s - sh) : 0u;
  }
}
// Absolute match of a u32 word under base b.
__device__ __forceinline__ int64_t mabs(int64_t b, uint32_t s) { return b + static_cast<int64_t>(s); }

// The changed list of an epoch comes in fixed slices, one per 128-group epoch wave: slice s
// (groups [128 s, 128 s + 128), decided by one wave) is 128 words at changed + 128 s: words
// 0-1 a 128-bit map of the groups whose commit advanced (bit i = group 128 s + i), then from
// byte 16 their deltas commit - pendingIndex + 1 as u32, in group order; n_changed[s] = how
// many.  12 B per committing group + 4 B per 128 groups.  No reservation, no atomics: each
// slice is written by the one wave that decides its groups.
constexpr uint32_t kSliceMapWords = 2;

__device__ __forceinline__ uint64_t spread_bits(uint32_t x) {  // bit i -> bit 2i
  uint64_t v = x;
  v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
  v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
  v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
  v = (v | (v << 2)) & 0x3333333333333333ull;
  v = (v | (v << 1)) & 0x5555555555555555ull;
  return v;
}

// Eight u32 words (one lane's pair of groups of a match row) at byte offset `off` of a
// wave-uniform base.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u32x2 gu32x2;
__device__ __forceinline__ u32x2 tld2u(const int64_t* base, uint32_t off) {
  gchar* b = (gchar*)base;
  asm volatile("" : "+s"(b));
  return __builtin_nontemporal_load(reinterpret_cast<const gu32x2*>(b + off));
}

// Shape (r06, "v4"): one wave per 128 groups (half a tile), two adjacent groups per lane -- the
// pair kernel's shape.  Every int64 stream of the pair with one 16-B load (1 KiB per wave
// instruction), every u32 match row with one 8-B load (512 B), all P + 4 loads issued before
// the first decision.  <= 64 VGPRs at P <= 5: 8 waves per SIMD, a 1M-group epoch's 8192 waves
// in one round, each with half of round 5's four-group chain (that kernel's single round of
// 4096 waves at 4 per SIMD left every wave's loads, then decisions, then stores in the same
// phase: 0.45 of spec).
constexpr uint32_t kTableEpochBlock = 64 * kTableBlockWaves;
#ifndef JRQ_TABLE_OCC  // waves per SIMD the epoch is compiled for at P <= 5 (A/B knob)
#define JRQ_TABLE_OCC 7
#endif

// Runs of a flagged group from its flagged-entry slot {group, start1, start2, start3, conf0,
// conf1, conf2, conf3} (unused runs: start INT64_MAX, conf 0).
struct EntRuns {
  int64_t e[8];
  __device__ int64_t start(uint32_t r) const { return r == 0 ? kI64Min : e[r]; }
  __device__ uint64_t conf(uint32_t r) const { return static_cast<uint64_t>(e[4 + r]); }
};

// The relative form of one group (rel_map from the u32 words): pi resolved, the window [pi, la]
// in the words' terms -- a word u maps to r = u - o in [1, W] (o = pi - 1 - base < 2^30); an
// ack past lastAppended is u > la - base (la >= pi - 1 >= base: headers with a smaller
// lastAppended are refused).
template <int P>
__device__ __forceinline__ void map_words(int64_t pi, int64_t la, const uint32_t (&s)[P], RelGroup<P>& g) {
  const int64_t b = mbase(pi);
  const uint32_t o = static_cast<uint32_t>(pi - 1 - b), lab = static_cast<uint32_t>(la - b);
  g.W = la >= pi ? static_cast<uint32_t>(la - pi) + 1u : 0u;
  g.st = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const uint32_t dd = s[p] - o - 1u;
    g.st |= s[p] > lab ? kStOutOfRange : 0;
    g.r[p] = dd < g.W ? dd + 1u : 0u;
  }
}

// One epoch over every group of the table, in place.  The single-conf decision runs in 32-bit
// arithmetic relative to pendingIndex (rel_cand, the pair kernel's) straight from the u32 match
// words.  A group with a conf change inside its pending window (JRQ_CONF_RUNS) is skipped by
// that decision and decided afterwards by its own lane: its loaded state (pendingIndex word,
// lastCommitted, lastAppended, match words) parked in the wave's slice of LDS during the
// decisions (registers stay free for the single-conf path), its runs from the wave's
// flagged-entry slots -- the first four loaded up front by lanes 0-15 beside the group loads
// whatever the wave's count (a branch on the count would put a memory round trip in front of
// every wave's loads), later ones by their owners.  Groups outside rel_domain (negative or huge
// indexes; never a real group) are decided again with 64-bit arithmetic from reloaded words in
// a wave-uniform branch.  No barrier beyond the wave's own, no atomics.
#ifndef JRQ_TABLE_LAZY_ENT  // (r06 A/B knob) flagged-entry words read where the walk uses them
#define JRQ_TABLE_LAZY_ENT 0
#endif
#ifndef JRQ_TABLE_ENT_LDS  // flagged-entry slots per unit loaded up front (4: lanes 32-63 repeat)
#define JRQ_TABLE_ENT_LDS 4
#endif
constexpr uint32_t kEntLds = JRQ_TABLE_ENT_LDS;

// One unit's loads (128 groups, half a tile; the unit's list slice and flagged-entry slots are
// its own): every int64 stream of the lane's pair with one 16-B load (1 KiB per wave
// instruction), every u32 match row with one 8-B load (512 B), and the lane's word of the unit's
// first kEntLds flagged-entry slots (64 B each; lanes 32-63 read lanes 0-31's words again: no
// branch, no extra line).  `u` is wave-uniform.
template <int P>
struct UnitIn {
  int64_t ev;
  i64x2 pr, la, lc, cw;
  u32x2 mq[P];
  i64x2 ap, cf, cs;  // the fused fan-out's FSMCaller rows (kFan only)
};

template <int P, bool kFan>
__device__ __forceinline__ void unit_load(const JrqTableArgs& t, uint32_t u, uint32_t lane, UnitIn<P>& in) {
  const int64_t* const tile = reinterpret_cast<const int64_t*>(t.match) + static_cast<size_t>(u >> 1) * t.ts;
  const int64_t* const ent = reinterpret_cast<const int64_t*>(t.flag_ent) + static_cast<size_t>(u) * kFlagSlots * 8;
  in.ev = __builtin_nontemporal_load(ent + (lane & (8 * kEntLds - 1)));
  const uint32_t go = 16u * lane + 1024u * (u & 1u);  // the pair's byte offset in a 2-KiB int64 row
  in.pr = tld2o(tile + 128 * P, go);
  in.la = tld2o(tile + 128 * P + 256, go);
  in.lc = tld2o(tile + 128 * P + 512, go);
  in.cw = tld2o(tile + 128 * P + 768, go);
#pragma unroll
  for (int p = 0; p < P; ++p) in.mq[p] = tld2u(tile + 128 * p, 8u * lane + 512u * (u & 1u));
  if (kFan) {  // the pair's lastAppliedIndex, ClosureQueue firstIndex and size (pad lanes: group 0's)
    const uint32_t g0 = u * kListSlice + 2u * lane;
    const size_t gp = g0 < t.G ? g0 : 0u;
    in.ap = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(t.fsm + gp));
    in.cf = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(t.fsm + t.ld + gp));
    in.cs = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(t.fsm + 2 * t.ld + gp));
  }
}

// The unit's decisions and writes, from its loads.
template <int P, bool kFan>
__device__ __forceinline__ void unit_decide(const JrqTableArgs& t, uint32_t u, uint32_t lane,
                                            int64_t (&entw)[kEntLds][8], const UnitIn<P>& ui) {
  const uint64_t below = (1ull << lane) - 1ull;
  const uint32_t g0 = u * kListSlice + 2u * lane;  // this lane's pair (g0, g0 + 1)
  int64_t* const tile = reinterpret_cast<int64_t*>(t.match) + static_cast<size_t>(u >> 1) * t.ts;
  const int64_t* const ent = reinterpret_cast<const int64_t*>(t.flag_ent) + static_cast<size_t>(u) * kFlagSlots * 8;
  if (lane < 8 * kEntLds) entw[lane >> 3][lane & 7u] = ui.ev;
  bool f[2], c[2], x[2], wpi[2];
  uint32_t d[2], st[2], rk[2];
  int64_t outv[2], pir[2];
  uint64_t bf[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t g = g0 + j;
    const int64_t prk = j ? ui.pr.y : ui.pr.x, lck = j ? ui.lc.y : ui.lc.x, lak = j ? ui.la.y : ui.la.x;
    const uint64_t cwk = static_cast<uint64_t>(j ? ui.cw.y : ui.cw.x);
    const bool in = g < t.G;
    f[j] = in && (cwk >> 63);
    bf[j] = __ballot(f[j]);
    rk[j] = (j ? __popcll(bf[0]) : 0u) + __popcll(bf[j] & below);
    const int64_t pi = prk == kPiFollowsLc ? lck + 1 : prk;
    uint32_t s[P];
#pragma unroll
    for (int p = 0; p < P; ++p) s[p] = j ? ui.mq[p].y : ui.mq[p].x;
    RelGroup<P> rg;
    map_words<P>(pi, lak, s, rg);
    uint8_t s8;
    const uint32_t r = rel_cand<P>(cwk, rg, s8);
    st[j] = pi == 0 ? kStNotLeader : s8;
    x[j] = in && !rel_domain(pi, lak);
    c[j] = in && !f[j] && !x[j] && pi != 0 && r >= 1u && pi - 1 + static_cast<int64_t>(r) > lck;
    d[j] = r;
    outv[j] = pi - 1 + static_cast<int64_t>(r);
    pir[j] = pi;
    wpi[j] = prk != kPiFollowsLc;
    // a flagged group (a conf change inside its window): its lane decides its runs right here,
    // from the same relative words, the runs from its flagged-entry slot (LDS for the first
    // kEntLds of the wave, memory beyond)
    if (__builtin_expect(bf[j] != 0, 0)) {  // (wave-uniform)
      // the parked entries are read by other lanes: LDS operations of one wave complete in
      // issue order, so only the compiler's order is needed (a fence here made the waitcnt
      // pass drain every load in flight, the next unit's among them, at the join below)
      asm volatile("" ::: "memory");
      if (f[j] && !x[j]) {
        uint32_t k = rk[j];
        asm volatile("" : "+v"(k));
#if JRQ_TABLE_LAZY_ENT
        // the slot's words read where they are used (LDS for the first kEntLds slots, memory
        // beyond): no array of them live across the walk (register pressure sets occupancy)
        const int64_t* const eg = ent + static_cast<size_t>(k) * 8;
        const bool inl = k < kEntLds;
        const uint32_t kl = inl ? k : 0u;
        auto est = [&](uint32_t q) -> int64_t { return inl ? entw[kl][q] : eg[q]; };
        auto ecf = [&](uint32_t q) -> uint64_t { return static_cast<uint64_t>(inl ? entw[kl][4 + q] : eg[4 + q]); };
#else
        int64_t es[kTableMaxRuns];
        uint64_t ec[kTableMaxRuns];
        if (k < kEntLds) {
          const int64_t* e = entw[k];
#pragma unroll
          for (int q = 1; q < kTableMaxRuns; ++q) es[q] = e[q];
#pragma unroll
          for (int q = 1; q < kTableMaxRuns; ++q) ec[q] = static_cast<uint64_t>(e[4 + q]);
        } else {
          const int64_t* e = ent + static_cast<size_t>(k) * 8;
#pragma unroll
          for (int q = 1; q < kTableMaxRuns; ++q) es[q] = e[q];
#pragma unroll
          for (int q = 1; q < kTableMaxRuns; ++q) ec[q] = static_cast<uint64_t>(e[4 + q]);
          // settled here (a rare branch): a load still pending where it joins the common path
          // made the waitcnt pass drain every load in flight there -- the next unit's too
          __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
        auto est = [&](uint32_t q) -> int64_t { return es[q]; };
        auto ecf = [&](uint32_t q) -> uint64_t { return ec[q]; };
#endif
        uint8_t sw = rg.st;
        int64_t best = kI64Min;
        if (pi != 0) {
          {  // run 0, [pi, start1 - 1] under the group's conf word: its bound is r, the
             // single-conf decision's (the same q-th largests), so no sort of its own
            const int64_t s1 = est(1);
            const int64_t e = s1 == kI64Max ? lak : s1 - 1;
            const int64_t ee = e < lak ? e : lak;
            if (ee >= pi) {
              if ((cwk & 0xFFFFu) == 0) sw |= kStEmptyConf;
              const uint32_t er = static_cast<uint32_t>(ee - pi) + 1u;
              const uint32_t cc = r < er ? r : er;
              if (cc >= 1u) best = pi - 1 + static_cast<int64_t>(cc);
            }
          }
#pragma unroll
          for (uint32_t q = 1; q < kTableMaxRuns; ++q) {
            const int64_t sq = est(q);
            if (sq == kI64Max) break;  // unused runs (they come last)
            const int64_t nx = q + 1 < kTableMaxRuns ? est(q + 1) : kI64Max;
            const int64_t sr = sq > pi ? sq : pi;
            const int64_t e = nx == kI64Max ? lak : nx - 1;
            const int64_t ee = e < lak ? e : lak;
            const int64_t cand = run_candidate_rel<P>(rg, ecf(q), pi, sr, ee, sw);
            best = cand > best ? cand : best;
          }
        }
        st[j] = pi == 0 ? kStNotLeader : sw;
        c[j] = pi != 0 && best > lck;
        outv[j] = best;
        d[j] = static_cast<uint32_t>(best - pi + 1);
      }
    }
  }
  // groups outside rel_domain (negative or huge indexes; never a real group): the 64-bit
  // decision from reloaded words, flagged or not, kept out of the fast path's registers
  if (__builtin_expect(__ballot(x[0] || x[1]) != 0, 0)) {
#pragma unroll 1
    for (uint32_t j = 0; j < 2; ++j) {
      const bool mine = j ? x[1] : x[0];
      if (!mine) continue;
      uint32_t h = g0 + j;
      asm volatile("" : "+v"(h));
      const int64_t prx = tf(t.pi, t, h), lcx = tf(t.lc, t, h), lax = tf(t.la, t, h);
      const int64_t pi = prx == kPiFollowsLc ? lcx + 1 : prx;
      const int64_t bb = mbase(pi);
      const uint64_t cwx = tf(t.conf, t, h);
      int64_t m[P];
#pragma unroll
      for (int p = 0; p < P; ++p) m[p] = mabs(bb, tm(t, p, h));
      int64_t out = lcx;
      uint8_t s8 = 0;
      if (cwx >> 63) {  // its runs from the cold rows (run 0's conf in the conf word)
        EntRuns R;
        R.e[0] = h;
        for (int r = 1; r < kTableMaxRuns; ++r) {
          R.e[r] = t.xstart[static_cast<size_t>(r - 1) * t.ld + h];
          R.e[4 + r] = static_cast<int64_t>(t.xconf[static_cast<size_t>(r - 1) * t.ld + h]);
        }
        R.e[4] = static_cast<int64_t>(cwx & ~kConfRuns);
        uint32_t nr = 1;
        while (nr < kTableMaxRuns && R.e[nr] != kI64Max) ++nr;
        s8 = mask_out_of_range<P>(m, lax);
        out = pi == 0 ? lcx : runs_best<P>(R, nr, pi, lax, lcx, m, s8);
        s8 = pi == 0 ? kStNotLeader : s8;
      } else {
        decide_single<P>(pi, lax, lcx, cwx, m, out, s8);
      }
      const bool commit = out > lcx;
      const uint32_t dj = static_cast<uint32_t>(out - pi + 1);
      if (j == 0) { c[0] = commit; d[0] = dj; outv[0] = out; st[0] = s8; }
      else        { c[1] = commit; d[1] = dj; outv[1] = out; st[1] = s8; }
    }
  }
  // state writes of the committing groups: lastCommitted (a pair at a time), pendingIndex ->
  // JRQ_PI_FOLLOWS_LC once (BallotBox.java:131-132: the steady state writes lastCommitted only),
  // and, when the new pendingIndex moves the match base (once per 2^30 entries), the words
  // re-expressed against it
  {
    int64_t* const lcb = tile + 128 * P + 512;
    // the pair's row offset again, from the lane id (mbcnt) and the wave's half (an SGPR):
    // recomputed, not kept live across the decisions (it was spilled and reloaded per store)
    const uint32_t go = 16u * __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) +
                        1024u * (u & 1u);
#if JRQ_TABLE_AB_LC != 1
    if (c[0] && c[1]) {
      i64x2 v;
      v.x = outv[0];
      v.y = outv[1];
      tst2o(lcb, go, v);
    } else {
      if (c[0]) tst1o(lcb, go, outv[0]);
      if (c[1]) tst1o(lcb, go + 8u, outv[1]);
    }
#endif
    if (c[0] && wpi[0]) tst1o(tile + 128 * P, go, kPiFollowsLc);
    if (c[1] && wpi[1]) tst1o(tile + 128 * P, go + 8u, kPiFollowsLc);
    const bool xb0 = c[0] && mbase(outv[0] + 1) != mbase(pir[0]);
    const bool xb1 = c[1] && mbase(outv[1] + 1) != mbase(pir[1]);
    if (__builtin_expect(__ballot(xb0 || xb1) != 0, 0)) {
      if (xb0) table_rebase<P>(t, g0, mbase(pir[0]), mbase(outv[0] + 1));
      if (xb1) table_rebase<P>(t, g0 + 1, mbase(pir[1]), mbase(outv[1] + 1));
    }
  }
  if (t.status && g0 < t.G) {
    if (g0 + 1 < t.G)
      st_tab(static_cast<uint16_t>(st[0] | (st[1] << 8)), reinterpret_cast<uint16_t*>(t.status + g0));
    else
      t.status[g0] = static_cast<uint8_t>(st[0]);
  }
  // the list slice, in group order: the map (lane l's pair = bits 2 l, 2 l + 1), then the deltas
  // at their ranks (one 8-B store when both groups of the pair commit at an even rank)
  const uint64_t b0 = __ballot(c[0]), b1 = __ballot(c[1]);
  const uint32_t cnt = __popcll(b0) + __popcll(b1);
  // (a wave past the table's last slice -- the grid is whole workgroups -- owns no slice: the
  // caller's list has room for jrq_table_slices(t) slices only)
  const bool owns = static_cast<uint64_t>(u) * kListSlice < t.G;
  uint64_t* const slice = t.changed + static_cast<size_t>(u) * kListSlice;
#if !JRQ_TABLE_AB_NOLIST  // (diagnosis knob: no list)
  if (lane < kSliceMapWords && owns) {
    const uint32_t sh = lane * 32u;
    slice[lane] = spread_bits(static_cast<uint32_t>(b0 >> sh)) | (spread_bits(static_cast<uint32_t>(b1 >> sh)) << 1);
  }
  uint32_t* const deltas = reinterpret_cast<uint32_t*>(slice + kSliceMapWords);
  const uint32_t at = __popcll(b0 & below) + __popcll(b1 & below);
  if (c[0] && c[1] && !(at & 1u)) {
    *reinterpret_cast<uint64_t*>(deltas + at) = static_cast<uint64_t>(d[0]) | (static_cast<uint64_t>(d[1]) << 32);
  } else {
    if (c[0]) deltas[at] = d[0];
    if (c[1]) deltas[at + (c[0] ? 1u : 0u)] = d[1];
  }
#endif
  if (lane == 0 && owns) t.n_changed[u] = cnt;
  // the fused fan-out (jrq_table_epoch_fanout): each committing group's doCommitted /
  // popClosureUntil on its new lastCommittedIndex (fan_one), the queue written back where it
  // popped, the result at the group's delta rank in the slice's fan arrays
  if (kFan) {
    int64_t f0 = ui.cf.x, n0 = ui.cs.x, f1 = ui.cf.y, n1 = ui.cs.y, fc0 = 0, fc1 = 0;
    const uint8_t s0 = c[0] ? fan_one(ui.lc.x, outv[0], ui.ap.x, f0, n0, fc0) : kFanNone;
    const uint8_t s1 = c[1] ? fan_one(ui.lc.y, outv[1], ui.ap.y, f1, n1, fc1) : kFanNone;
    if (f0 != ui.cf.x || f1 != ui.cf.y) {  // a pop moved firstIndex
      i64x2 nf, nn;
      nf.x = f0;
      nf.y = f1;
      nn.x = n0;
      nn.y = n1;
      *reinterpret_cast<i64x2*>(t.fsm + t.ld + g0) = nf;
      *reinterpret_cast<i64x2*>(t.fsm + 2 * t.ld + g0) = nn;
    }
    const uint32_t r0 = __popcll(b0 & below) + __popcll(b1 & below);
    int64_t* const ff = t.fan_first + static_cast<size_t>(u) * kListSlice;
    uint8_t* const fs = t.fan_status + static_cast<size_t>(u) * kListSlice;
    if (c[0]) {
      ff[r0] = fc0;
      fs[r0] = s0;
    }
    if (c[1]) {
      const uint32_t r1 = r0 + (c[0] ? 1u : 0u);
      ff[r1] = fc1;
      fs[r1] = s1;
    }
  }
}


// JRQ_TABLE_UNITS (r06 A/B knob): units per wave.  1: one wave per unit (8192 waves for 1M
// groups, JRQ_TABLE_OCC per SIMD).  2: one wave per tile, both halves' loads issued before the
// first half's decisions, so a wave decides one unit while the other's loads are in flight.
#ifndef JRQ_TABLE_UNITS
#define JRQ_TABLE_UNITS 1
#endif
template <int P, bool kFan>
__global__ __launch_bounds__(kTableEpochBlock, JRQ_TABLE_UNITS == 2 ? 4 : (P <= 5 ? (kFan ? 6 : JRQ_TABLE_OCC) : (P <= 10 ? 4 : 2)))
JRQ_SGPRS_8WAVES void table_epoch_kernel(JrqTableArgs t) {
  constexpr uint32_t kWaves = kTableEpochBlock / 64;
  __shared__ int64_t entl[kWaves][kEntLds][8];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + w);
#if JRQ_TABLE_UNITS == 2
  UnitIn<P> a, b;
  unit_load<P, kFan>(t, 2u * wid, lane, a);
  unit_load<P, kFan>(t, 2u * wid + 1u, lane, b);
  unit_decide<P, kFan>(t, 2u * wid, lane, entl[w], a);
  asm volatile("" ::: "memory");  // (the first unit's LDS reads before the second's parking)
  unit_decide<P, kFan>(t, 2u * wid + 1u, lane, entl[w], b);
#else
  UnitIn<P> a;
  unit_load<P, kFan>(t, wid, lane, a);
  unit_decide<P, kFan>(t, wid, lane, entl[w], a);
#endif
}

// jrq_table_fsm_update: n groups' FSMCaller state (lastAppliedIndex, ClosureQueue firstIndex and
// size), one group per lane; a group past the table is skipped and counted.
__global__ __launch_bounds__(256) void table_fsm_kernel(JrqTableArgs t, const uint32_t* __restrict__ groups,
                                                        const int64_t* __restrict__ applied,
                                                        const int64_t* __restrict__ first,
                                                        const int64_t* __restrict__ size, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t g = groups[i];
    if (g >= t.G) {
      atomicAdd(t.invalid, 1u);
      continue;
    }
    t.fsm[g] = applied[i];
    t.fsm[t.ld + g] = first[i];
    t.fsm[2 * t.ld + g] = size[i];
  }
}

// Host variant of the fused fan-out: each slice's fan results (ranks 0 .. n[s) of its fan arrays)
// gathered behind the slices before it, in the host list's order (one wave per slice).
__global__ __launch_bounds__(512) void table_fan_gather_kernel(const int64_t* __restrict__ ff,
                                                               const uint8_t* __restrict__ fs,
                                                               const uint32_t* __restrict__ n,
                                                               const uint32_t* __restrict__ off,
                                                               uint32_t slices, int64_t* __restrict__ out_first,
                                                               uint8_t* __restrict__ out_status) {
  const uint32_t s = blockIdx.x * 8u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (s >= slices) return;
  const uint32_t cnt = n[s], o = off[s];
  for (uint32_t r = lane; r < cnt; r += 64u) {
    out_first[o + r] = ff[static_cast<size_t>(s) * kListSlice + r];
    out_status[o + r] = fs[static_cast<size_t>(s) * kListSlice + r];
  }
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

// One wave per slice: lane l takes the slice's groups 2 l, 2 l + 1 (two bits of its map), their
// ranks from the map's popcounts, and writes each listed group as the host list's word (delta
// << 32 | group).
__global__ __launch_bounds__(512) void table_list_gather_kernel(const uint64_t* __restrict__ changed,
                                                                const uint32_t* __restrict__ n,
                                                                const uint32_t* __restrict__ off,
                                                                uint32_t slices,
                                                                uint64_t* __restrict__ out) {
  const uint32_t s = blockIdx.x * 8u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (s >= slices || n[s] == 0) return;
  const uint64_t* sl = changed + static_cast<size_t>(s) * kListSlice;
  const uint32_t* deltas = reinterpret_cast<const uint32_t*>(sl + kSliceMapWords);
  const uint32_t wd = lane >> 5, sh = 2u * (lane & 31u);
  const uint64_t word = sl[wd];
  uint32_t rank = __popcll(word & ((1ull << sh) - 1ull)) + (wd ? static_cast<uint32_t>(__popcll(sl[0])) : 0u);
  uint32_t at = off[s] + rank;
  uint32_t bits = static_cast<uint32_t>(word >> sh) & 3u;
  while (bits) {
    const uint32_t b = __builtin_ctz(bits);
    bits &= bits - 1u;
    out[at++] = (static_cast<uint64_t>(deltas[rank++]) << 32) | (s * kListSlice + 2u * lane + b);
  }
}

// The flagged-entry slots: per 128-group epoch wave, its groups flagged JRQ_CONF_RUNS, each as
// a 64-B entry {group, start1, start2, start3, conf0, conf1, conf2, conf3} (run starts and conf
// words; unused runs: start INT64_MAX, conf 0), and their count.  Rebuilt after every update
// that carries group headers (only headers change runs and flags); the waves map exactly as the
// epoch kernel's (lane l: groups 128 w + 2 l, + 1; entries in the order of the even groups' ballot
// ranks, then the odd groups'), no barrier, no atomics.
constexpr uint32_t kFlagBlock = 64 * kTableBlockWaves;
__global__ __launch_bounds__(kFlagBlock) void table_flags_kernel(JrqTableArgs t) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wid = blockIdx.x * (kFlagBlock / 64) + (threadIdx.x >> 6);
  const uint32_t g = wid * kListSlice + 2u * lane;
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
  bool f0 = false, f1 = false;
  if (g < t.G) {
    const i64x2 cw = tld2(reinterpret_cast<const int64_t*>(&tf(t.conf, t, g)));
    f0 = static_cast<uint64_t>(cw.x) >> 63;
    f1 = (static_cast<uint64_t>(cw.y) >> 63) && g + 1 < t.G;
  }
  const uint64_t b0 = __ballot(f0), b1 = __ballot(f1);
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
  if (st.flags & 2u) t.rstamp[g] = static_cast<uint64_t>(st.run_start[0]);  // JRQ_STATE_STAMP
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

// Order-free ack records (include/jrq.h JRQ_ACK): one lane per record.  The record's segment
// (a binary search over the few segment starts) gives its stamp; a record stamped before its
// group's last reset is dropped.  The absolute index is the one within 2^31 of pendingIndex - 1
// whose low 32 bits the record carries; a match raises its slot's u32 word (against the group's
// match base, saturating: below the base it changes nothing), a lastAppended the group's queue
// end -- both as atomic maxima, so records apply in any order.
// Record i of the update: in segment s (the last whose first record seg_off[s] is <= i), at
// seg_ptr[s][i - seg_off[s]] -- a segment's records are contiguous wherever they are (the staging
// buffer, or a caller's device region filled by jrq_table_ack_push).
__global__ __launch_bounds__(256) void table_acks_kernel(JrqTableArgs t, const uint64_t* const* __restrict__ seg_ptr,
                                                         uint32_t n, const uint32_t* __restrict__ seg_off,
                                                         const uint64_t* __restrict__ seg_stamp, uint32_t nseg) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint32_t lo = 0, hi = nseg;  // the last segment starting at or before i
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (seg_off[mid] <= i) lo = mid;
    else hi = mid;
  }
  const uint64_t r = seg_ptr[lo][i - seg_off[lo]];
  const uint32_t f = static_cast<uint32_t>(r & 31u);
  const uint32_t g = static_cast<uint32_t>(r >> 5) & ((1u << 27) - 1u);
  const uint32_t low = static_cast<uint32_t>(r >> 32);
  if (g >= t.G || f > 16u || (f < 16u && f >= t.P)) {
    atomicAdd(t.invalid, 1u);
    return;
  }
  if (seg_stamp[lo] < t.rstamp[g]) return;  // recorded before the group's last reset
  const int64_t pr = tf(t.pi, t, g), lc = tf(t.lc, t, g);
  const int64_t pi = pr == kPiFollowsLc ? lc + 1 : pr;
  if (pi <= 0) return;  // not the leader: commitAt refuses (BallotBox.java:101-103)
  const int64_t a = (pi - 1) + static_cast<int64_t>(static_cast<int32_t>(low - static_cast<uint32_t>(pi - 1)));
  if (f == 16u) {
    // a queue longer than an ArrayList, or entries pending without a conf run: refused, counted
    if (a - pi >= int64_t{0x7FFFFFFF} || (tf(t.conf, t, g) == 0 && a >= pi)) {
      atomicAdd(t.invalid, 1u);
      return;
    }
    atomicMax(reinterpret_cast<long long*>(&tf(t.la, t, g)), static_cast<long long>(a));
  } else {
    const int64_t rel = a - mbase(pi);
    if (rel <= 0) return;
    atomicMax(&tm(t, f, g), rel > 0xFFFFFFFFll ? 0xFFFFFFFFu : static_cast<uint32_t>(rel));
  }
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_acks(
    const JrqTableArgs* a, const uint64_t* const* seg_ptr, uint32_t n, const uint32_t* seg_off,
    const uint64_t* seg_stamp, uint32_t nseg, hipStream_t stream) {
  if (n)
    hipLaunchKernelGGL(jrq::table_acks_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, *a, seg_ptr, n,
                       seg_off, seg_stamp, nseg);
  return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_update(
    const JrqTableArgs* a, const JrqGroupState* states, uint32_t n_states, const uint64_t* recs,
    uint32_t n_recs, hipStream_t stream) {
  if (n_states) {
    hipLaunchKernelGGL(jrq::table_states_kernel, dim3((n_states + 255) / 256), dim3(256), 0,
                       stream, *a, states, n_states);
    const uint32_t waves = (a->G + jrq::kListSlice - 1) / jrq::kListSlice;
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
  const uint32_t units = (a->G + jrq::kListSlice - 1) / jrq::kListSlice;
  const uint32_t waves = (units + JRQ_TABLE_UNITS - 1) / JRQ_TABLE_UNITS;
  const dim3 grid((waves + jrq::kTableEpochBlock / 64 - 1) / (jrq::kTableEpochBlock / 64)), blk(jrq::kTableEpochBlock);
  switch (a->P) {
#define JRQ_CASE(P)                                                                   \
  case P:                                                                             \
    if (a->fan_first)                                                                 \
      hipLaunchKernelGGL((jrq::table_epoch_kernel<P, true>), grid, blk, 0, stream, *a); \
    else                                                                              \
      hipLaunchKernelGGL((jrq::table_epoch_kernel<P, false>), grid, blk, 0, stream, *a); \
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

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_fsm(
    const JrqTableArgs* a, const uint32_t* groups, const int64_t* applied, const int64_t* first,
    const int64_t* size, uint32_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(jrq::table_fsm_kernel, dim3(blocks < 4096 ? blocks : 4096), dim3(256), 0, stream, *a,
                     groups, applied, first, size, n);
  return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_table_fan_gather(
    const int64_t* ff, const uint8_t* fs, const uint32_t* n, const uint32_t* off, uint32_t slices,
    int64_t* out_first, uint8_t* out_status, hipStream_t stream) {
  if (slices == 0) return hipSuccess;
  hipLaunchKernelGGL(jrq::table_fan_gather_kernel, dim3((slices + 7) / 8), dim3(512), 0, stream, ff, fs, n,
                     off, slices, out_first, out_status);
  return hipGetLastError();
}
