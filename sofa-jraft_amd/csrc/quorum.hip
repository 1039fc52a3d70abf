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
// Groups whose conf word carries JRQ_CONF_RUNS walk their conf runs (run table); every other
// group is decided from its conf word alone.  HBM-bound: 8P + 41 bytes per group decision
// (roofline).
#include "quorum_core.h"

namespace jrq {

// The CSR run table of the stateless ABI: runs [r0, r1) of one group.
struct CsrRuns {
  const int64_t* run_start;
  const uint64_t* run_conf;
  uint32_t r0;
  __device__ int64_t start(uint32_t r) const { return run_start[r0 + r]; }
  __device__ uint64_t conf(uint32_t r) const { return run_conf[r0 + r]; }
};

template <int P>
__device__ __forceinline__ int64_t csr_runs_best(const JrqQuorumArgs& a, uint32_t r0, uint32_t r1,
                                                 int64_t pi, int64_t la, int64_t lc,
                                                 const int64_t (&m)[P], uint8_t& st) {
  const CsrRuns R{a.run_start, a.run_conf, r0};
  return runs_best<P>(R, r1 - r0, pi, la, lc, m, st);
}

// A group flagged JRQ_CONF_RUNS: its runs from the CSR run table.
template <int P>
__device__ __forceinline__ void decide_runs(const JrqQuorumArgs& a, uint32_t g, int64_t pi,
                                            int64_t la, int64_t lc, int64_t (&m)[P],
                                            int64_t& out, uint8_t& st_out) {
  if (pi == 0) {
    out = lc;
    st_out = kStNotLeader;
    return;
  }
  uint8_t st = mask_out_of_range<P>(m, la);
  out = csr_runs_best<P>(a, a.run_off[g], a.run_off[g + 1], pi, la, lc, m, st);
  st_out = st;
}

template <int P>
__device__ __forceinline__ void decide(const JrqQuorumArgs& a, uint32_t g, int64_t pi, int64_t la,
                                       int64_t lc, uint64_t cw, int64_t (&m)[P], int64_t& out,
                                       uint8_t& st) {
  if (a.run_off != nullptr && (cw & kConfRuns))
    decide_runs<P>(a, g, pi, la, lc, m, out, st);
  else
    decide_single<P>(pi, la, lc, cw, m, out, st);
}

// General path (unaligned arrays, odd strides): one lane per group.  Every load of the group
// is issued before any decision, so a group costs one memory round trip (two more for a
// group that walks its runs).
template <int P>
__global__ __launch_bounds__(256) JRQ_SGPRS_8WAVES void quorum_epoch_kernel(JrqQuorumArgs a) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < a.G; g += stride) {
    const int64_t pi = a.pending_index[g];
    const int64_t lc = a.last_committed[g];
    const int64_t la = a.last_appended[g];
    const uint64_t cw = a.conf[g];
    int64_t m[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m[p] = a.match[static_cast<size_t>(p) * a.match_ld + g];
    int64_t out;
    uint8_t st;
    decide<P>(a, g, pi, la, lc, cw, m, out, st);
    a.committed[g] = out;
    a.status[g] = st;
  }
}

typedef int64_t i64x2 __attribute__((ext_vector_type(2)));

// The pair kernel's cache policy for its streams (A/B knobs, tools/ab_build.sh): nt loads (each
// input is read once per epoch), plain stores -- nt stores of the 16-B committed pairs and
// 2-B status words measured 7 % slower on C3 (15.95 vs 14.79 us, in-process A/B; nt loads
// 4.6 % faster than plain ones)
#ifndef JRQ_PAIR_NT_LOADS
#define JRQ_PAIR_NT_LOADS 1
#endif
#ifndef JRQ_PAIR_NT_STORES
#define JRQ_PAIR_NT_STORES 0
#endif
__device__ __forceinline__ i64x2 ld2nt(const int64_t* p) {
#if JRQ_PAIR_NT_LOADS
  return __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(p));
#else
  return *reinterpret_cast<const i64x2*>(p);
#endif
}
template <class T>
__device__ __forceinline__ void st_pair(T v, T* p) {
#if JRQ_PAIR_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// Fast path (16-B aligned arrays, even match_ld): one lane decides two adjacent groups; every
// stream is read with 16-byte non-temporal loads (1 KiB per wave instruction; each input is
// read once per epoch, so it is not kept in L2 / MALL) and the two status bytes are stored as
// one 16-bit word.  512-thread workgroups: 256 and 1024 measured 6-8 % slower on C3
// (round 3's round 3's tools/table_probe.hip).
// kRuns (run tables given): a group flagged JRQ_CONF_RUNS (a conf change inside its pending
// window) is skipped by the single-conf decision and walked by its own wave afterwards, four
// lanes per group (runs r, r + 4, ... on lane r of the quad, candidates max-reduced over the
// quad); its state (pendingIndex, lastCommitted, lastAppended, match) comes from the owner lane
// through the wave's slice of LDS (the first 16 flagged groups of a wave; a wave-local hand-off),
// so the walk costs the run table's two dependent loads and no workgroup barrier.  Round 2
// deferred flagged groups to a workgroup list behind __syncthreads() -- which also waits for
// every store of the fast path -- and reloaded them.  Without run tables the kernel is the
// kRuns = false instantiation: no LDS, no walk.
// The single-conf decision runs in 32-bit arithmetic relative to pendingIndex
// (decide_single_rel, quorum_core.h: C3 16.4 -> 15.6 us per epoch in round 3's tools/pair_probe.hip,
// against 15.1 us for the loads and stores alone).
// Workgroup size of the pair kernel by input layout: in-process A/B (r05, 30 interleaved
// rounds, profiles/r05e_ab_pair_block.log): rows 15.8 us at 512 threads, 15.2 at 1024, 16.6 at
// 256; tiles 14.8 at 512 and at 256, 15.0 at 1024.
#ifndef JRQ_PAIR_BLOCK_ROWS
#define JRQ_PAIR_BLOCK_ROWS 1024
#endif
#ifndef JRQ_PAIR_BLOCK_TILES
#define JRQ_PAIR_BLOCK_TILES 512
#endif
constexpr uint32_t pair_block(bool tiles) { return tiles ? JRQ_PAIR_BLOCK_TILES : JRQ_PAIR_BLOCK_ROWS; }
#ifndef JRQ_PAIR_XCD_TILES
#define JRQ_PAIR_XCD_TILES 0
#endif

// kTiles: the inputs in the resident table's tiles (JrqQuorumArgs::ts != 0: 256-group tiles,
// every field of a tile's groups in one contiguous block; jrq_quorum_epoch_tiles_dev), the
// outputs as rows.  A wave's pairs sit in one half of one tile.
template <int P, bool kRuns, bool kTiles>
__global__ __launch_bounds__(pair_block(kTiles)) JRQ_SGPRS_8WAVES void quorum_epoch_pair_kernel(JrqQuorumArgs a) {
  constexpr uint32_t kPairBlock = pair_block(kTiles);
  // word of group g in a field's row (tiles: the field's row in tile 0)
  auto at = [&](uint32_t g) -> size_t {
    return kTiles ? static_cast<size_t>(g >> 8) * a.ts + (g & 255u) : static_cast<size_t>(g);
  };
  auto mrow = [&](int p) -> const int64_t* {
    return a.match + (kTiles ? static_cast<size_t>(p) * 256u : static_cast<size_t>(p) * a.match_ld);
  };
  constexpr uint32_t kWaves = kPairBlock / 64;
  constexpr uint32_t kHand = 16;
  __shared__ int64_t hand[kRuns ? kWaves : 1][kHand][P + 3];  // {pi, lc, la, match[P]}
  __shared__ uint32_t flagged[kRuns ? kWaves : 1][128];
  const uint32_t pairs = a.G >> 1;
#if JRQ_PAIR_XCD_TILES
  // A/B knob (tools/ab_build.sh): workgroups in XCD-contiguous order -- block b runs on XCD
  // b % 8 (round-robin dispatch), so tile = that XCD's run position b / 8 inside its own
  // contiguous range of tiles, and each XCD streams one region of every row
  const uint32_t nb = gridDim.x, xq = nb / 8, xr = nb % 8, xcd = blockIdx.x % 8;
  const uint32_t tile = xcd * xq + (xcd < xr ? xcd : xr) + blockIdx.x / 8;
  const uint32_t t = tile * kPairBlock + threadIdx.x;
#else
  const uint32_t t = blockIdx.x * kPairBlock + threadIdx.x;
#endif
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  bool f0 = false, f1 = false;
  bool slow = false;  // a group outside decide_single_rel's domain (never in a real batch)
  if (t < pairs) {
    const uint32_t g = t << 1;
    const size_t gi = at(g);
    const i64x2 pi = ld2nt(a.pending_index + gi);
    const i64x2 lc = ld2nt(a.last_committed + gi);
    const i64x2 la = ld2nt(a.last_appended + gi);
    const i64x2 cw = ld2nt(reinterpret_cast<const int64_t*>(a.conf) + gi);
    i64x2 m[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m[p] = ld2nt(mrow(p) + gi);
    f0 = kRuns && (static_cast<uint64_t>(cw.x) & kConfRuns);
    f1 = kRuns && (static_cast<uint64_t>(cw.y) & kConfRuns);
    int64_t m0[P], m1[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      m0[p] = m[p].x;
      m1[p] = m[p].y;
    }
    if (kRuns) {  // flagged groups -> the wave's list and hand-off slots (ballot ranks)
      const uint64_t b0 = __ballot(f0), b1 = __ballot(f1);
      const uint32_t k0 = __popcll(b0 & below), k1 = __popcll(b0) + __popcll(b1 & below);
      auto put = [&](uint32_t k, uint32_t h, int64_t p_, int64_t c_, int64_t l_, const int64_t(&mm)[P]) {
        flagged[w][k] = h;
        if (k < kHand) {
          int64_t* hs = hand[w][k];
          hs[0] = p_;
          hs[1] = c_;
          hs[2] = l_;
#pragma unroll
          for (int q = 0; q < P; ++q) hs[3 + q] = mm[q];
        }
      };
      if (f0) put(k0, g, pi.x, lc.x, la.x, m0);
      if (f1) put(k1, g + 1, pi.y, lc.y, la.y, m1);
    }
    int64_t o0, o1;
    uint8_t s0, s1;
    decide_single_rel<P>(pi.x, la.x, lc.x, static_cast<uint64_t>(cw.x), m0, o0, s0);
    decide_single_rel<P>(pi.y, la.y, lc.y, static_cast<uint64_t>(cw.y), m1, o1, s1);
    slow = !(rel_domain(pi.x, la.x) && rel_domain(pi.y, la.y));
    if (!f0 && !f1) {
      i64x2 out;
      out.x = o0;
      out.y = o1;
      st_pair(out, reinterpret_cast<i64x2*>(a.committed + g));
      st_pair(static_cast<uint16_t>(s0 | (s1 << 8)),
                                  reinterpret_cast<uint16_t*>(a.status + g));
    } else {  // rare: a flagged group's outputs are written by the walk only
      if (!f0) {
        a.committed[g] = o0;
        a.status[g] = s0;
      }
      if (!f1) {
        a.committed[g + 1] = o1;
        a.status[g + 1] = s1;
      }
    }
  }
  if (kRuns) {
    const uint32_t nflag = __popcll(__ballot(f0)) + __popcll(__ballot(f1));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (this wave's slots only)
    __builtin_amdgcn_wave_barrier();
    const uint32_t q = lane >> 2, r = lane & 3u;
    for (uint32_t base = 0; base < nflag; base += 16) {  // (wave-uniform)
      const uint32_t i = base + q;
      const bool act = i < nflag;
      const uint32_t h = act ? flagged[w][i] : 0u;
      int64_t hpi = 0, hlc = 0, hla = 0, hm[P];
      if (act && i < kHand) {
        const int64_t* hs = hand[w][i];
        hpi = hs[0];
        hlc = hs[1];
        hla = hs[2];
#pragma unroll
        for (int p = 0; p < P; ++p) hm[p] = hs[3 + p];
      } else if (act) {  // more flagged groups than hand-off slots: reload (rare)
        hpi = a.pending_index[at(h)];
        hlc = a.last_committed[at(h)];
        hla = a.last_appended[at(h)];
#pragma unroll
        for (int p = 0; p < P; ++p) hm[p] = mrow(p)[at(h)];
      }
      int64_t cand = kI64Min;
      uint8_t st = 0;
      if (act && hpi != 0) {
        st = mask_out_of_range<P>(hm, hla);
        const uint32_t r0 = a.run_off[h], nr = a.run_off[h + 1] - r0;
        for (uint32_t rr = r; rr < nr; rr += 4) {  // runs_best (quorum_core.h), spread over the quad
          const int64_t rs = a.run_start[r0 + rr];
          const int64_t s = (rr == 0) ? hpi : (rs > hpi ? rs : hpi);
          const int64_t e = (rr + 1 < nr) ? a.run_start[r0 + rr + 1] - 1 : hla;
          const int64_t c = run_candidate<P>(hm, a.run_conf[r0 + rr], s, e < hla ? e : hla, st);
          cand = c > cand ? c : cand;
        }
      }
      cand = max(cand, dpp64<kDppXor1>(cand));
      cand = max(cand, dpp64<kDppXor2>(cand));
      uint32_t s32 = st;
      s32 |= dpp32<kDppXor1>(s32);
      s32 |= dpp32<kDppXor2>(s32);
      if (act && r == 0) {
        // decide_runs: not the leader -> unchanged (BallotBox.java:101-103)
        a.committed[h] = hpi == 0 ? hlc : (cand > hlc ? cand : hlc);
        a.status[h] = hpi == 0 ? kStNotLeader : static_cast<uint8_t>(s32);
      }
    }
  }
  // groups outside the 32-bit domain: decided again with 64-bit arithmetic from reloaded
  // words, after (and over) the fast path's stores -- a wave-uniform branch, never taken by a
  // real batch, kept out of the fast path's registers
  if (__builtin_expect(__ballot(slow) != 0, 0) && slow) {
#pragma unroll 1
    for (uint32_t g = t << 1; g < (t << 1) + 2; ++g) {
      if (kRuns && (a.conf[at(g)] & kConfRuns)) continue;  // (the walk decided it, exactly)
      int64_t m[P];
#pragma unroll
      for (int p = 0; p < P; ++p) m[p] = mrow(p)[at(g)];
      int64_t out;
      uint8_t st;
      decide_single<P>(a.pending_index[at(g)], a.last_appended[at(g)], a.last_committed[at(g)],
                       a.conf[at(g)], m, out, st);
      a.committed[g] = out;
      a.status[g] = st;
    }
  }
  // odd G: the last group goes through the scalar decision
  if ((a.G & 1u) && t == 0) {
    const uint32_t g = a.G - 1;
    int64_t m[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m[p] = mrow(p)[at(g)];
    int64_t out;
    uint8_t st;
    decide<P>(a, g, a.pending_index[at(g)], a.last_appended[at(g)], a.last_committed[at(g)],
              a.conf[at(g)], m, out, st);
    a.committed[g] = out;
    a.status[g] = st;
  }
}

// ------------------------------------------------------ K epochs per launch ---
// K successive epochs of the same G groups (hard part 4: a 10k-group epoch is
// launch-bound).  Between epochs the group state moves as BallotBox moves it: a commit sets
// lastCommittedIndex and pendingIndex = lastCommittedIndex + 1 (BallotBox.java:131-134); a
// group that is not the leader stays so.  That carried state is a thresholded prefix max:
//   v_k = max over the group's runs r of { cand_rk : cand_rk >= s_r },
//         cand_rk = min(end_r, la_k, bound_r(match_k)),  s_r = max(start_r, pi_0) (first: pi_0)
//   committed_k = max(lc_0, max_{j <= k} v_j)
//   pi_k = committed_{k-1} + 1 once a commit happened (max_{j<k} v_j > lc_0), else pi_0
// (a candidate in [s_r, committed_{k-1}] that the reference would refuse because it is below
// pi_k cannot raise the max, so the threshold may stay at pi_0).  v_k depends on epoch k's
// inputs only: lanes run over (group, epoch) -- a workgroup holds a tile of 32 groups, each
// half-wave a chunk of C epochs of them -- and a scan over the chunk maxima in LDS stitches
// the prefix.  Loads stay coalesced (32 consecutive groups = 256 B per row and epoch); small
// tiles spread a 10k-group batch over all 256 CUs.
// A chunk = C epochs of the tile's T groups on T lanes, at most W waves per workgroup,
// super-chunks beyond that.  Product shape (EpochChunk, r05): tiles of T = 16 groups (a
// quarter-wave chunk still loads whole 128-B lines: 16 groups x 8 B per row and epoch), at most
// 4 waves, and 16 loads per lane (C = 4 epochs at P = 3) -- or 32 (C = 8) for a launch of 192+
// epochs, whose workgroups then walk half as many super-chunks.  In-process A/B on the GPU
// (tools/ab_inproc.py, profiles/r05e_ab_epochs_shapes.log), C2 at 256 / 64 epochs per launch:
// round 4's T = 32, 8 waves, C = 4: 26.1 / 8.3 us; T = 16, 4 waves, C = 4: 24.5 / 7.4;
// C = 8: 22.8 / 8.8 (so C = 8 only for long launches); 2 or 8 waves, T = 32 with 16 waves: all
// slower.
#ifndef JRQ_EPOCHS_DEEP_LOADS
#define JRQ_EPOCHS_DEEP_LOADS 32
#endif
#ifndef JRQ_EPOCHS_WAVES
#define JRQ_EPOCHS_WAVES 4
#endif
template <int P, bool kDeep>
struct EpochChunk {
  static constexpr int kLoads = kDeep ? JRQ_EPOCHS_DEEP_LOADS : 16;
  static constexpr int kC = (kLoads / (P + 1)) < 1 ? 1 : ((kLoads / (P + 1)) > 8 ? 8 : kLoads / (P + 1));
  static constexpr int kMaxWaves = JRQ_EPOCHS_WAVES;
  static constexpr int kTile = 16;  // groups per workgroup
};
constexpr uint32_t kEpochsDeepK = 192;  // epochs per launch from which EpochChunk<P, true> runs

template <int P, int C, int T, int W>
__global__ __launch_bounds__(64 * W) void quorum_epochs_kernel(JrqQuorumArgs a, uint32_t K,
                                                               uint64_t match_eld,
                                                               uint64_t la_eld) {
  static_assert(T == 16 || T == 32 || T == 64, "a chunk is a quarter, a half or a whole wave");
  constexpr uint32_t kPerWave = 64 / T;
  __shared__ int64_t chunk_max[kPerWave * W][T];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gl = lane & (T - 1u);
  const uint32_t chunk = (threadIdx.x >> 6) * kPerWave + lane / T;  // this lane's chunk
  const uint32_t nchunks = (blockDim.x >> 6) * kPerWave;
  // tiles in XCD-contiguous order: workgroups are dealt round-robin to the 8 XCDs, so block b
  // takes tile (b % 8)'s run position b / 8 -- the tiles that share DRAM pages (8 per 2 KiB of
  // a row) then go out from one XCD back to back (-4 %, round 3's tools/epochs_probe.hip mode 4)
  const uint32_t nb = gridDim.x, xq = nb / 8, xr = nb % 8, xcd = blockIdx.x % 8;
  const uint32_t tile = xcd * xq + (xcd < xr ? xcd : xr) + blockIdx.x / 8;
  const uint32_t g = tile * T + gl;
  const bool live = g < a.G;
  // Every load is unconditional (a dead lane reads group 0, an epoch past K reads epoch K-1;
  // both results are discarded): per-lane conditions around them made the compiler wait for
  // each epoch's loads before issuing the next epoch's -- C round trips instead of one.
  const uint32_t gs = live ? g : 0u;
  const int64_t pi0 = live ? a.pending_index[gs] : 0;
  const int64_t lc0 = live ? a.last_committed[gs] : 0;
  const uint64_t cw = live ? a.conf[gs] : 0;
  int64_t carry = kI64Min;  // max v over the epochs of earlier super-chunks
  for (uint32_t base = 0; base < K; base += nchunks * C) {
    const uint32_t k0 = base + chunk * C;
    int64_t la[C], pre[C];
    uint8_t st[C];
    bool runs;
    uint32_t r0, r1;
    {
      int64_t m[C][P];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const size_t k = k0 + c < K ? k0 + c : K - 1;
        la[c] = __builtin_nontemporal_load(a.last_appended + k * la_eld + gs);
#pragma unroll
        for (int p = 0; p < P; ++p)
          m[c][p] = __builtin_nontemporal_load(a.match + k * match_eld +
                                               static_cast<size_t>(p) * a.match_ld + gs);
      }
      // conf runs of a flagged group: its CSR bounds, after the epoch loads are out
      runs = a.run_off != nullptr && (cw & kConfRuns);
      r0 = runs ? a.run_off[g] : 0;
      r1 = runs ? a.run_off[g + 1] : 0;
      int64_t run_max = kI64Min;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        st[c] = 0;
        if (live && k0 + c < K) {
          st[c] = mask_out_of_range<P>(m[c], la[c]);
          int64_t v;
          if (!runs) {
            int64_t cand = run_bound<P>(m[c], cw);
            cand = cand < la[c] ? cand : la[c];
            v = cand >= pi0 ? cand : kI64Min;
          } else {
            uint8_t unused = 0;
            v = csr_runs_best<P>(a, r0, r1, pi0, la[c], kI64Min, m[c], unused);
          }
          run_max = v > run_max ? v : run_max;
        }
        pre[c] = run_max;  // inclusive max over this chunk
      }
    }
    chunk_max[chunk][gl] = pre[C - 1];
    __syncthreads();
    int64_t excl = carry, all = carry;
    for (uint32_t u = 0; u < nchunks; ++u) {
      const int64_t t = chunk_max[u][gl];
      if (u < chunk) excl = t > excl ? t : excl;
      all = t > all ? t : all;
    }
    if (base + nchunks * C < K) __syncthreads();  // the next super-chunk rewrites chunk_max
    carry = all;
    if (!live) continue;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const uint32_t k = k0 + c;
      if (k >= K) break;
      const int64_t prev = c == 0 ? excl : (pre[c - 1] > excl ? pre[c - 1] : excl);
      const int64_t mk = pre[c] > excl ? pre[c] : excl;
      int64_t out = mk > lc0 ? mk : lc0;
      uint8_t s = st[c];
      if (pi0 == 0) {
        out = lc0;
        s = kStNotLeader;
      } else {
        const int64_t pik = prev > lc0 ? prev + 1 : pi0;  // pendingIndex before epoch k
        if (!runs) {
          if ((cw & 0xFFFFu) == 0 && la[c] >= pik) s |= kStEmptyConf;
        } else {  // runs still pending at epoch k with an empty conf (L2-hot re-read)
          for (uint32_t r = r0; r < r1; ++r) {
            const int64_t sr = (r == r0) ? pik : (a.run_start[r] > pik ? a.run_start[r] : pik);
            const int64_t er = (r + 1 < r1) ? a.run_start[r + 1] - 1 : la[c];
            if ((er < la[c] ? er : la[c]) >= sr && (a.run_conf[r] & 0xFFFFu) == 0)
              s |= kStEmptyConf;
          }
        }
      }
      a.committed[static_cast<size_t>(k) * a.G + g] = out;
      a.status[static_cast<size_t>(k) * a.G + g] = s;
    }
  }
}

// K epochs of a large batch (r05): with G/2 >= 2048 lanes per CU there is parallelism enough
// over the groups alone, so one lane takes two adjacent groups through all K epochs in order,
// carrying the prefix max in registers -- no chunk stitch, no LDS, no barrier -- and reads every
// stream with 16-B loads (1 KiB per wave instruction; the chunk kernel's tiles of 32 groups
// read 256-B row segments).  The same carried state as quorum_epochs_kernel.
// One group's epoch candidate v_k (kI64Min: none) and its out-of-range flags.
template <int P>
__device__ __forceinline__ int64_t epoch_candidate(const JrqQuorumArgs& a, bool runs, uint32_t r0,
                                                   uint32_t r1, int64_t pi0, int64_t la,
                                                   uint64_t cw, int64_t (&m)[P], uint8_t& st) {
  if (!runs && rel_domain(pi0, la) && pi0 != 0) {  // 32-bit, relative to pendingIndex_0
    RelGroup<P> g;
    rel_map<P>(pi0, la, m, g);
    st = g.st;
    uint8_t unused;
    const uint32_t r = rel_cand<P>(cw, g, unused);
    return r >= 1u ? pi0 - 1 + static_cast<int64_t>(r) : kI64Min;
  }
  st = mask_out_of_range<P>(m, la);
  if (!runs) {
    int64_t cand = run_bound<P>(m, cw);
    cand = cand < la ? cand : la;
    return cand >= pi0 ? cand : kI64Min;
  }
  uint8_t unused = 0;
  return csr_runs_best<P>(a, r0, r1, pi0, la, kI64Min, m, unused);
}

// Status of epoch k beyond the out-of-range flags: not the leader, or an empty conf over an
// entry still pending (pik = pendingIndex before epoch k).
__device__ __forceinline__ uint8_t epoch_status(const JrqQuorumArgs& a, bool runs, uint32_t r0,
                                                uint32_t r1, int64_t pi0, int64_t pik, int64_t la,
                                                uint64_t cw, uint8_t st) {
  if (pi0 == 0) return kStNotLeader;
  if (!runs) return ((cw & 0xFFFFu) == 0 && la >= pik) ? static_cast<uint8_t>(st | kStEmptyConf) : st;
  for (uint32_t r = r0; r < r1; ++r) {  // runs still pending at epoch k with an empty conf
    const int64_t sr = (r == r0) ? pik : (a.run_start[r] > pik ? a.run_start[r] : pik);
    const int64_t er = (r + 1 < r1) ? a.run_start[r + 1] - 1 : la;
    if ((er < la ? er : la) >= sr && (a.run_conf[r] & 0xFFFFu) == 0) st |= kStEmptyConf;
  }
  return st;
}

// kRuns: the batch carries run tables (a.run_off); without them the walk is compiled out.
// kTiles: every epoch's inputs in the 256-group tiles of jrq_quorum_epoch_tiles_dev (a.ts =
// the tile stride; epoch k's tiles match_eld words after epoch 0's), so a wave reads each
// epoch's match and lastAppended fields as one contiguous block of its tile.
#ifndef JRQ_EPOCHS_PAIR_BLOCK
#define JRQ_EPOCHS_PAIR_BLOCK 256
#endif
#ifndef JRQ_EPOCHS_PAIR_UNROLL
#define JRQ_EPOCHS_PAIR_UNROLL 1
#endif
template <int P, bool kRuns, bool kTiles>
__global__ __launch_bounds__(JRQ_EPOCHS_PAIR_BLOCK) void quorum_epochs_pair_kernel(JrqQuorumArgs a, uint32_t K,
                                                                                 uint64_t match_eld,
                                                                                 uint64_t la_eld) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t pairs = a.G >> 1;
  const bool tail = i == pairs && (a.G & 1u);  // the odd last group, on one more lane
  if (i >= pairs && !tail) return;
  const uint32_t g = tail ? a.G - 1 : 2 * i;
  const int n = tail ? 1 : 2;
  // word of group g in a field's row (tiles: in tile 0; a pair never straddles a tile)
  const size_t at = kTiles ? static_cast<size_t>(g >> 8) * a.ts + (g & 255u) : static_cast<size_t>(g);
  const size_t mstride = kTiles ? 256u : static_cast<size_t>(a.match_ld);
  int64_t pi0[2], lc0[2], vmax[2] = {kI64Min, kI64Min};
  uint64_t cw[2];
  bool runs[2];
  uint32_t r0[2], r1[2];
  if (!tail) {
    const i64x2 p2 = ld2nt(a.pending_index + at), l2 = ld2nt(a.last_committed + at);
    const i64x2 c2 = ld2nt(reinterpret_cast<const int64_t*>(a.conf) + at);
    pi0[0] = p2.x; pi0[1] = p2.y;
    lc0[0] = l2.x; lc0[1] = l2.y;
    cw[0] = static_cast<uint64_t>(c2.x); cw[1] = static_cast<uint64_t>(c2.y);
  } else {
    pi0[0] = a.pending_index[at]; lc0[0] = a.last_committed[at]; cw[0] = a.conf[at];
    pi0[1] = 0; lc0[1] = 0; cw[1] = 0;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    runs[h] = kRuns && h < n && (cw[h] & kConfRuns);
    r0[h] = runs[h] ? a.run_off[g + h] : 0;
    r1[h] = runs[h] ? a.run_off[g + h + 1] : 0;
  }
#pragma unroll JRQ_EPOCHS_PAIR_UNROLL
  for (uint32_t k = 0; k < K; ++k) {
    int64_t la[2], m[2][P];
    if (!tail) {
      const i64x2 l2 = ld2nt(a.last_appended + k * la_eld + at);
      la[0] = l2.x; la[1] = l2.y;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const i64x2 v = ld2nt(a.match + k * match_eld + static_cast<size_t>(p) * mstride + at);
        m[0][p] = v.x;
        m[1][p] = v.y;
      }
    } else {
      la[0] = a.last_appended[k * la_eld + at];
      la[1] = 0;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        m[0][p] = a.match[k * match_eld + static_cast<size_t>(p) * mstride + at];
        m[1][p] = 0;
      }
    }
    int64_t out[2];
    uint8_t s[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t prev = vmax[h];  // max v over the earlier epochs
      uint8_t st = 0;
      const int64_t v = epoch_candidate<P>(a, runs[h], r0[h], r1[h], pi0[h], la[h], cw[h], m[h], st);
      vmax[h] = v > vmax[h] ? v : vmax[h];
      out[h] = pi0[h] == 0 ? lc0[h] : (vmax[h] > lc0[h] ? vmax[h] : lc0[h]);
      const int64_t pik = prev > lc0[h] ? prev + 1 : pi0[h];
      s[h] = epoch_status(a, runs[h], r0[h], r1[h], pi0[h], pik, la[h], cw[h], st);
    }
    const size_t o = static_cast<size_t>(k) * a.G + g;
    if (!tail) {
      i64x2 c2;
      c2.x = out[0];
      c2.y = out[1];
      st_pair(c2, reinterpret_cast<i64x2*>(a.committed + o));
      st_pair(static_cast<uint16_t>(s[0] | (s[1] << 8)), reinterpret_cast<uint16_t*>(a.status + o));
    } else {
      a.committed[o] = out[0];
      a.status[o] = s[0];
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

// --------------------------------------------------------------- ReadIndex ---
// NodeImpl.readLeader's ReadOnlySafe round (jraft-core/.../core/NodeImpl.java:1343-1396) and
// its ReadIndexHeartbeatResponseClosure (:1246-1291): quorum = peers.size()/2 + 1 (getQuorum,
// :1321-1327; <= 1 answers at once), a heartbeat to every conf peer but the leader, and per
// response, in arrival order: ackSuccess or ackFailures + 1, then success when ackSuccess + 1
// >= quorum, else failure when ackFailures >= failPeersThreshold (quorum - 1 for an even
// peer count, quorum for an odd one); the first verdict stands.  Restated without the loop:
// the verdict is whichever threshold the arrival order crosses first -- the arrival key of
// the (quorum-1)-th success against that of the threshold-th failure (key = position * 16 +
// slot, so equal positions resolve by slot, as the oracle orders them).
template <int P>
__device__ __forceinline__ uint8_t readindex_verdict(uint64_t cw, uint64_t ord, uint32_t okm,
                                                     uint32_t self) {
  // a conf naming a slot >= num_peers has a peer no response can come from: not decidable
  // from this batch's inputs (the reference has no slots), so it is reported, not left pending
  if ((static_cast<uint32_t>(cw & 0xFFFFu) >> P) != 0) return kRiInvalid;
  const uint32_t mask = static_cast<uint32_t>(cw & 0xFFFFu);
  const uint32_t n = __builtin_popcount(mask);  // peers.size()
  const uint32_t q = n ? n / 2 + 1 : 0;
  if (q <= 1) return kRiSuccess;  // the fast path answers at once
  const uint32_t need_ok = q - 1, need_fail = (n % 2 == 0) ? q - 1 : q;
  // per responding slot a sort key: kind (failure = 1) above the arrival key position * 16 +
  // slot, so that a success sorts before every failure; 0xFFFF = no response from that slot
  uint32_t kk[P];
  uint32_t n_ok = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const uint32_t pos = static_cast<uint32_t>(ord >> (4 * p)) & 0xFu;
    const bool resp = ((mask >> p) & 1u) && static_cast<uint32_t>(p) != self && pos != 0;
    const uint32_t fail = ((okm >> p) & 1u) ^ 1u;
    kk[p] = resp ? (fail << 12) | (pos * 16u + static_cast<uint32_t>(p)) : 0xFFFFu;
    n_ok += (resp && !fail) ? 1u : 0u;
  }
  // the crossing keys: the need-th smallest key among the successes / the failures (the rank
  // of a failure counts every success below it: subtract them)
  uint32_t t_ok = ~0u, t_fail = ~0u;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    uint32_t rank = 0;
#pragma unroll
    for (int r = 0; r < P; ++r) rank += kk[r] <= kk[p] ? 1u : 0u;
    const bool fail = kk[p] >> 12 == 1u;
    if (kk[p] != 0xFFFFu && !fail && rank == need_ok) t_ok = kk[p];
    if (kk[p] != 0xFFFFu && fail && rank - n_ok == need_fail) t_fail = kk[p] & 0xFFFu;
  }
  return t_ok < t_fail ? kRiSuccess : (t_fail != ~0u ? kRiFailure : kRiPending);
}

// kQuad: four consecutive groups per lane -- two 16-B loads each of conf and order, 8 B of
// ok masks, 4 of self slots, one 4-B verdict store (the one-group form moved 1-8 B per lane
// per instruction); needs 16-B aligned conf / order, 8-B ok, 4-B self and result.
template <int P, bool kQuad>
__global__ __launch_bounds__(256) void readindex_quorum_kernel(JrqReadIndexArgs a) {
  const uint32_t stride = gridDim.x * blockDim.x;
  if (!kQuad) {
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < a.G; g += stride)
      a.result[g] = readindex_verdict<P>(__builtin_nontemporal_load(a.conf + g),
                                         __builtin_nontemporal_load(a.order + g), a.ok_mask[g],
                                         a.self_slot[g]);
    return;
  }
  const uint32_t quads = a.G / 4;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < quads; i += stride) {
    using u64x2 = __attribute__((ext_vector_type(2))) uint64_t;
    const u64x2 c0 = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(a.conf) + 2 * i);
    const u64x2 c1 = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(a.conf) + 2 * i + 1);
    const u64x2 o0 = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(a.order) + 2 * i);
    const u64x2 o1 = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(a.order) + 2 * i + 1);
    const uint64_t ok4 = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(a.ok_mask) + i);
    const uint32_t s4 = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(a.self_slot) + i);
    uint32_t r = readindex_verdict<P>(c0.x, o0.x, static_cast<uint32_t>(ok4 & 0xFFFFu), s4 & 0xFFu);
    r |= static_cast<uint32_t>(readindex_verdict<P>(c0.y, o0.y, static_cast<uint32_t>((ok4 >> 16) & 0xFFFFu),
                                                    (s4 >> 8) & 0xFFu)) << 8;
    r |= static_cast<uint32_t>(readindex_verdict<P>(c1.x, o1.x, static_cast<uint32_t>((ok4 >> 32) & 0xFFFFu),
                                                    (s4 >> 16) & 0xFFu)) << 16;
    r |= static_cast<uint32_t>(readindex_verdict<P>(c1.y, o1.y, static_cast<uint32_t>(ok4 >> 48),
                                                    s4 >> 24)) << 24;
    reinterpret_cast<uint32_t*>(a.result)[i] = r;
  }
  // the last G % 4 groups, one per lane of the first wave
  const uint32_t g = quads * 4 + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x * blockDim.x + threadIdx.x < (a.G & 3u))
    a.result[g] = readindex_verdict<P>(a.conf[g], a.order[g], a.ok_mask[g], a.self_slot[g]);
}

// ------------------------------------------------------------- leader tick ---
// One group's lease check (NodeImpl.handleStepDownTimeout -> checkDeadNodes, :2003-2016):
// the conf, then the old conf when not empty; each passing check moves the lease start.
template <int P>
__device__ __forceinline__ void lease_one(const int64_t (&ts)[P], uint64_t cw, uint32_t self,
                                          int64_t now, int64_t timeout, int64_t& lead,
                                          uint8_t& ok, uint16_t& dead) {
  int64_t start;
  ok = 0;
  dead = 0;
  if (alive_quorum<P>(ts, cw & 0xFFFFu, (cw >> 32) & 0xFFu, self, now, timeout, start, dead)) {
    lead = start;
    ok |= 1;
  }
  const uint32_t omask = (cw >> 16) & 0xFFFFu;
  if (omask != 0) {
    if (alive_quorum<P>(ts, omask, (cw >> 40) & 0xFFu, self, now, timeout, start, dead)) {
      lead = start;
      ok |= 2;
    }
  } else {
    ok |= 2;
  }
}

// The leader's periodic tick over G leader groups in one launch: the lease check and, when
// kRI, the ReadIndex heartbeat round of the same groups (readindex_verdict), which read the
// same conf word and self slot.  Two adjacent groups per lane, as the headline epoch kernel
// (quorum_epoch_pair_kernel): every int64 stream (P timestamp rows, conf, lease start, order)
// is read with 16-B nt loads, 1 KiB per wave instruction, the byte / u16 fields two at a time;
// the whole grid at once.  Round 4 ran the two as separate launches of one group per lane
// (lease 0.68 of HBM, ReadIndex 0.32: the 21-MB ReadIndex launch was latency-bound).
// Needs 16-B aligned ts rows (even ld) / conf / lease_start / order, 4-B ok_mask and dead,
// 2-B self_slot / ok / ri_result (jrq_launch_tick checks; else the one-group kernels run).
// (JRQ_TICK_SGPR_CAP, an A/B knob: the 8-waves SGPR budget of the pair kernel -- a few SGPRs
// spill to VGPR lanes at P = 5 -- against the compiler's own ~106 SGPRs, 6 waves per SIMD)
#ifndef JRQ_TICK_SGPR_CAP
#define JRQ_TICK_SGPR_CAP 1
#endif
#if JRQ_TICK_SGPR_CAP
#define JRQ_TICK_ATTR JRQ_SGPRS_8WAVES
#else
#define JRQ_TICK_ATTR
#endif
template <int P, bool kRI>
#ifndef JRQ_TICK_BLOCK
#define JRQ_TICK_BLOCK 512
#endif
__global__ __launch_bounds__(JRQ_TICK_BLOCK) JRQ_TICK_ATTR void leader_tick_pair_kernel(JrqLeaseArgs a) {
  using u64x2 = __attribute__((ext_vector_type(2))) uint64_t;
  using i64x2 = __attribute__((ext_vector_type(2))) int64_t;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t pairs = a.G >> 1;
  if (i < pairs) {
    const size_t g = 2 * static_cast<size_t>(i);
    int64_t t0[P], t1[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const i64x2 v = __builtin_nontemporal_load(
          reinterpret_cast<const i64x2*>(a.last_rpc_ts + static_cast<size_t>(p) * a.ld + g));
      t0[p] = v.x;
      t1[p] = v.y;
    }
    const u64x2 cw = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(a.conf + g));
    const uint32_t s2 = __builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(a.self_slot + g));
    i64x2 lead = __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(a.lease_start + g));
    u64x2 ord = {0, 0};
    uint32_t okm2 = 0;
    if (kRI) {
      ord = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(a.order + g));
      okm2 = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(a.ri_ok_mask + g));
    }
    int64_t l0 = lead.x, l1 = lead.y;
    uint8_t ok0, ok1;
    uint16_t d0, d1;
    lease_one<P>(t0, cw.x, s2 & 0xFFu, a.now_ms, a.lease_timeout_ms, l0, ok0, d0);
    lease_one<P>(t1, cw.y, s2 >> 8, a.now_ms, a.lease_timeout_ms, l1, ok1, d1);
    lead.x = l0;
    lead.y = l1;
    *reinterpret_cast<uint16_t*>(a.ok + g) = static_cast<uint16_t>(ok0 | (ok1 << 8));
    *reinterpret_cast<i64x2*>(a.lease_start + g) = lead;
    if (a.dead) *reinterpret_cast<uint32_t*>(a.dead + g) = static_cast<uint32_t>(d0) | (static_cast<uint32_t>(d1) << 16);
    if (kRI) {
      const uint32_t r0 = readindex_verdict<P>(cw.x, ord.x, okm2 & 0xFFFFu, s2 & 0xFFu);
      const uint32_t r1 = readindex_verdict<P>(cw.y, ord.y, okm2 >> 16, s2 >> 8);
      *reinterpret_cast<uint16_t*>(a.ri_result + g) = static_cast<uint16_t>(r0 | (r1 << 8));
    }
  } else if (i == pairs && (a.G & 1u)) {  // the odd last group, one lane
    const size_t g = a.G - 1;
    int64_t t[P];
#pragma unroll
    for (int p = 0; p < P; ++p) t[p] = a.last_rpc_ts[static_cast<size_t>(p) * a.ld + g];
    const uint64_t cw = a.conf[g];
    int64_t l = a.lease_start[g];
    uint8_t ok;
    uint16_t d;
    lease_one<P>(t, cw, a.self_slot[g], a.now_ms, a.lease_timeout_ms, l, ok, d);
    a.ok[g] = ok;
    a.lease_start[g] = l;
    if (a.dead) a.dead[g] = d;
    if (kRI) a.ri_result[g] = readindex_verdict<P>(cw, a.order[g], a.ri_ok_mask[g], a.self_slot[g]);
  }
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_readindex(
    const JrqReadIndexArgs* args, int num_cus, hipStream_t stream) {
  const bool quad = ((reinterpret_cast<uintptr_t>(args->conf) | reinterpret_cast<uintptr_t>(args->order)) & 15u) == 0 &&
                    (reinterpret_cast<uintptr_t>(args->ok_mask) & 7u) == 0 &&
                    ((reinterpret_cast<uintptr_t>(args->self_slot) | reinterpret_cast<uintptr_t>(args->result)) & 3u) == 0;
  const uint64_t lanes = quad ? (static_cast<uint64_t>(args->G) + 3) / 4 : args->G;
  const uint64_t need = (lanes + 255) / 256;
  const uint64_t cap = static_cast<uint64_t>(num_cus) * 8;
  const dim3 grid(static_cast<unsigned>(need < cap ? (need ? need : 1) : cap)), blk(256);
  switch (args->num_peers) {
#define JRQ_CASE(P)                                                                                \
  case P:                                                                                          \
    if (quad)                                                                                      \
      hipLaunchKernelGGL((jrq::readindex_quorum_kernel<P, true>), grid, blk, 0, stream, *args);  \
    else                                                                                           \
      hipLaunchKernelGGL((jrq::readindex_quorum_kernel<P, false>), grid, blk, 0, stream, *args); \
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

// The lease check, with the ReadIndex round fused when args->order is set (the leader tick):
// the pair kernel when the arrays allow its wide accesses, else the one-group kernels.
extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_lease(
    const JrqLeaseArgs* args, int num_cus, hipStream_t stream) {
  auto al = [](const void* p, uintptr_t n) { return (reinterpret_cast<uintptr_t>(p) & (n - 1)) == 0; };
  const JrqLeaseArgs& a = *args;
  const bool ri = a.order != nullptr;
  const bool pair = a.G >= 2 && (a.ld & 1u) == 0 && al(a.last_rpc_ts, 16) && al(a.conf, 16) &&
                    al(a.lease_start, 16) && al(a.self_slot, 2) && al(a.ok, 2) && al(a.dead, 4) &&
                    (!ri || (al(a.order, 16) && al(a.ri_ok_mask, 4) && al(a.ri_result, 2)));
  if (pair) {
    const uint64_t lanes = static_cast<uint64_t>(a.G) / 2 + 1;  // + the odd tail's lane
    const dim3 grid(static_cast<unsigned>((lanes + JRQ_TICK_BLOCK - 1) / JRQ_TICK_BLOCK)), blk(JRQ_TICK_BLOCK);
    switch (a.num_peers) {
#define JRQ_CASE(P)                                                                             \
  case P:                                                                                       \
    if (ri)                                                                                     \
      hipLaunchKernelGGL((jrq::leader_tick_pair_kernel<P, true>), grid, blk, 0, stream, a);   \
    else                                                                                        \
      hipLaunchKernelGGL((jrq::leader_tick_pair_kernel<P, false>), grid, blk, 0, stream, a);  \
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
  if (ri) {  // unaligned leader tick: the ReadIndex kernel after the lease kernel below
    JrqReadIndexArgs r{};
    r.conf = a.conf;
    r.self_slot = a.self_slot;
    r.order = a.order;
    r.ok_mask = a.ri_ok_mask;
    r.num_peers = a.num_peers;
    r.G = a.G;
    r.result = a.ri_result;
    const hipError_t s = jrq_launch_readindex(&r, num_cus, stream);
    if (s != hipSuccess) return s;
  }
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
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  const JrqQuorumArgs& a = *args;
  const bool pair = (a.match_ld & 1u) == 0 && al16(a.match) && al16(a.pending_index) &&
                    al16(a.last_appended) && al16(a.last_committed) && al16(a.conf) &&
                    al16(a.committed) && (reinterpret_cast<uintptr_t>(a.status) & 1u) == 0 &&
                    a.G >= 2;
  if (a.ts && !pair) return hipErrorInvalidValue;  // (tiled inputs: the pair kernel only)
  // pair kernel: one lane per two groups, the whole grid at once; scalar kernel: one lane per
  // group, at most 8 workgroups per CU, grid-stride beyond
  const uint64_t lanes = pair ? (a.G >> 1) : a.G;
  const uint32_t bs = pair ? jrq::pair_block(a.ts != 0) : 256u;
  const dim3 blk(bs);
  const uint64_t need = (lanes + bs - 1) / bs;
  const uint64_t cap = pair ? need : static_cast<uint64_t>(num_cus) * 8;
  const dim3 grid(static_cast<unsigned>(need < cap ? (need ? need : 1) : cap));
  switch (args->num_peers) {
#define JRQ_CASE(P)                                                                      \
  case P:                                                                                \
    if (pair && a.ts && a.run_off)                                                       \
      hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<P, true, true>), grid, blk, 0, stream, *args); \
    else if (pair && a.ts)                                                               \
      hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<P, false, true>), grid, blk, 0, stream, *args); \
    else if (pair && a.run_off)                                                          \
      hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<P, true, false>), grid, blk, 0, stream, *args); \
    else if (pair)                                                                       \
      hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<P, false, false>), grid, blk, 0, stream, *args); \
    else                                                                                 \
      hipLaunchKernelGGL(jrq::quorum_epoch_kernel<P>, grid, blk, 0, stream, *args);      \
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

// Waves per workgroup of quorum_epochs_kernel: enough for ceil(K / C) chunks, at most wmax.
static inline uint32_t jrq_epochs_waves(uint32_t K, uint32_t C, uint32_t T, uint32_t wmax) {
  const uint32_t per = 64 / T, chunks = (K + C - 1) / C, w = (chunks + per - 1) / per;
  return w < wmax ? w : wmax;
}

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_quorum_epochs(
    const JrqQuorumArgs* args, uint32_t K, uint64_t match_eld, uint64_t la_eld, int num_cus,
    hipStream_t stream) {
  // a batch with 2048+ groups per CU (C3K: 1M groups): two groups per lane through every epoch
  // in order (quorum_epochs_pair_kernel), when the arrays allow its 16-B accesses
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  const JrqQuorumArgs& q = *args;
  const bool pair = q.G % 2 == 0 && static_cast<uint64_t>(q.G) >= 2048ull * static_cast<uint64_t>(num_cus) &&
                    (q.match_ld & 1u) == 0 && (match_eld & 1u) == 0 && (la_eld & 1u) == 0 &&
                    al16(q.match) && al16(q.pending_index) && al16(q.last_appended) &&
                    al16(q.last_committed) && al16(q.conf) && al16(q.committed) &&
                    (reinterpret_cast<uintptr_t>(q.status) & 1u) == 0;
  if (pair || q.ts) {  // (tiled inputs: always the pair kernel, G >= 2 and aligned: the caller checks)
    constexpr unsigned kB = JRQ_EPOCHS_PAIR_BLOCK;
    const dim3 grid(static_cast<unsigned>((q.G / 2 + 1 + kB - 1) / kB)), blk(kB);  // + the odd tail's lane
    switch (q.num_peers) {
#define JRQ_LAUNCH(P, R, T) \
  hipLaunchKernelGGL((jrq::quorum_epochs_pair_kernel<P, R, T>), grid, blk, 0, stream, q, K, match_eld, la_eld)
#define JRQ_CASE(P)                                                                            \
  case P:                                                                                      \
    if (q.ts) {                                                                                \
      if (q.run_off) JRQ_LAUNCH(P, true, true); else JRQ_LAUNCH(P, false, true);               \
    } else {                                                                                   \
      if (q.run_off) JRQ_LAUNCH(P, true, false); else JRQ_LAUNCH(P, false, false);             \
    }                                                                                          \
    break;
      JRQ_CASE(1) JRQ_CASE(2) JRQ_CASE(3) JRQ_CASE(4) JRQ_CASE(5) JRQ_CASE(6) JRQ_CASE(7)
      JRQ_CASE(8) JRQ_CASE(9) JRQ_CASE(10) JRQ_CASE(11) JRQ_CASE(12) JRQ_CASE(13) JRQ_CASE(14)
      JRQ_CASE(15) JRQ_CASE(16)
#undef JRQ_CASE
#undef JRQ_LAUNCH
      default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  // otherwise one workgroup per tile of groups; chunks of C epochs (four per wave), at most W
  // waves, super-chunks beyond that
  const bool deep = K >= jrq::kEpochsDeepK;
  switch (args->num_peers) {
#define JRQ_LAUNCH(P, D)                                                                      \
  {                                                                                           \
    using E = jrq::EpochChunk<P, D>;                                                          \
    const dim3 grid(static_cast<unsigned>((static_cast<uint64_t>(args->G) + E::kTile - 1) /   \
                                          E::kTile));                                         \
    const uint32_t w = jrq_epochs_waves(K, E::kC, E::kTile, E::kMaxWaves);                    \
    hipLaunchKernelGGL((jrq::quorum_epochs_kernel<P, E::kC, E::kTile, E::kMaxWaves>), grid,   \
                       dim3(64u * w), 0, stream, *args, K, match_eld, la_eld);                \
  }
#define JRQ_CASE(P)                                                                           \
  case P:                                                                                     \
    if (deep) JRQ_LAUNCH(P, true) else JRQ_LAUNCH(P, false)                                   \
    break;
    JRQ_CASE(1) JRQ_CASE(2) JRQ_CASE(3) JRQ_CASE(4) JRQ_CASE(5) JRQ_CASE(6) JRQ_CASE(7)
    JRQ_CASE(8) JRQ_CASE(9) JRQ_CASE(10) JRQ_CASE(11) JRQ_CASE(12) JRQ_CASE(13) JRQ_CASE(14)
    JRQ_CASE(15) JRQ_CASE(16)
#undef JRQ_CASE
#undef JRQ_LAUNCH
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
