// quorum_core.h -- the per-group quorum arithmetic shared by the stateless epoch kernels
// (quorum.hip) and the resident-table kernels (table.hip).  See quorum.hip for the
// formulation and its references (BallotBox.java:96-139, Ballot.java:63-140).
#pragma once

#include "jrq_device.h"

namespace jrq {

constexpr int64_t kI64Min = INT64_MIN;
constexpr int64_t kI64Max = INT64_MAX;
constexpr uint64_t kConfRuns = 1ull << 63;  // include/jrq.h JRQ_CONF_RUNS

// Lane exchanges of the run walks (table.hip, quorum.hip) as DPP moves (a VALU operand
// modifier, no LDS round trip; __shfl_xor compiles to ds_bpermute, and the walks' reductions
// were a chain of them):
//   kDppXor1 / kDppXor2  quad_perm [1,0,3,2] / [2,3,0,1]: the partner lane 1 / 2 apart
//   kDppHalfMirror       row_half_mirror: lane i of each 8-lane half row gets lane 7 - i, so
//                        lane 0 of an 8-lane group sees lane 7 (the group's other quad)
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141;
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), kCtrl, 0xF, 0xF, false));
}
template <int kCtrl>
__device__ __forceinline__ int64_t dpp64(int64_t x) {
  const uint32_t lo = dpp32<kCtrl>(static_cast<uint32_t>(x));
  const uint32_t hi = dpp32<kCtrl>(static_cast<uint32_t>(static_cast<uint64_t>(x) >> 32));
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}

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

// The same decision in 32-bit arithmetic relative to pendingIndex, for every group whose
// pending window [pi, la] holds fewer than 2^32 - 1 entries (every real group).  Only match
// values inside the window can grant a pending entry, so each peer maps to r = m - pi + 1 in
// [1, W] (W = la - pi + 1, 0 when nothing is pending) or to 0 (below the window, or past
// lastAppended: out of range).  The map is monotone, so it commutes with the q-th-largest and
// the min of the conf words' bounds, and "candidate >= pendingIndex" becomes r >= 1.  The q-th
// largest member: the members' r (others 0) sorted by an odd-even transposition network of u32
// max / min, then element q - 1 (0 when fewer than q members: nothing granted).  Per pair of
// groups ~300 VALU instead of ~540 for kth_largest's P^2 64-bit compares (round 3's tools/pair_probe.hip).
template <int P>
__device__ __forceinline__ uint32_t kth_largest_rel(const uint32_t (&r)[P], uint32_t mask, uint32_t q) {
  uint32_t s[P];
#pragma unroll
  for (int p = 0; p < P; ++p) s[p] = ((mask >> p) & 1u) ? r[p] : 0u;
#pragma unroll
  for (int round = 0; round < P; ++round) {
#pragma unroll
    for (int i = round & 1; i + 1 < P; i += 2) {
      const uint32_t hi = s[i] > s[i + 1] ? s[i] : s[i + 1];
      const uint32_t lo = s[i] > s[i + 1] ? s[i + 1] : s[i];
      s[i] = hi;
      s[i + 1] = lo;
    }
  }
  uint32_t out = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) out = q == static_cast<uint32_t>(p + 1) ? s[p] : out;
  return out;
}

// decide_single inside rel_domain (pi = 0: not the leader; la < pi: nothing pending, W = 0).
// With pi < 2^62 a match below the window (negative ones included) wraps to d >= 2^62 > W:
// no false grant from any int64 match value.  Two steps, so a caller deciding several groups
// can map all of them first and let their 64-bit match words die before the sorting networks.
template <int P>
struct RelGroup {
  uint32_t r[P];  // per slot: m - pi + 1 inside the window, else 0
  uint32_t W;     // pending entries
  uint8_t st;     // out-of-range flags
};

template <int P>
__device__ __forceinline__ void rel_map(int64_t pi, int64_t la, const int64_t (&m)[P], RelGroup<P>& g) {
  g.W = la >= pi ? static_cast<uint32_t>(la - pi) + 1u : 0u;
  g.st = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const uint64_t d = static_cast<uint64_t>(m[p]) - static_cast<uint64_t>(pi);
    g.st |= m[p] > la ? kStOutOfRange : 0;
    g.r[p] = d < g.W ? static_cast<uint32_t>(d) + 1u : 0u;
  }
}

// The single conf word's bound in the relative domain: the largest r in [0, W] every entry up
// to which is granted (0: none), and the status bits (out-of-range acks, empty conf).  The
// commit is pi - 1 + r when pi != 0, r >= 1 and that exceeds lastCommitted.
template <int P>
__device__ __forceinline__ uint32_t rel_cand(uint64_t cw, const RelGroup<P>& g, uint8_t& st) {
  st = g.st;
  if ((cw & 0xFFFFu) == 0 && g.W != 0) st |= kStEmptyConf;
  const uint32_t nmask = static_cast<uint32_t>(cw & 0xFFFFu);
  const uint32_t omask = static_cast<uint32_t>((cw >> 16) & 0xFFFFu);
  const uint32_t nq = static_cast<uint32_t>((cw >> 32) & 0xFFu);
  const uint32_t oq = static_cast<uint32_t>((cw >> 40) & 0xFFu);
  const uint32_t kn = nq == 0 ? g.W : kth_largest_rel<P>(g.r, nmask, nq);
  const uint32_t ko = oq == 0 ? g.W : kth_largest_rel<P>(g.r, omask, oq);
  const uint32_t cand = kn < ko ? kn : ko;
  return cand < g.W ? cand : g.W;
}

template <int P>
__device__ __forceinline__ void rel_decide(int64_t pi, int64_t lc, uint64_t cw, const RelGroup<P>& g,
                                           int64_t& out, uint8_t& st_out) {
  uint8_t st = g.st;
  if ((cw & 0xFFFFu) == 0 && g.W != 0) st |= kStEmptyConf;
  const uint32_t nmask = static_cast<uint32_t>(cw & 0xFFFFu);
  const uint32_t omask = static_cast<uint32_t>((cw >> 16) & 0xFFFFu);
  const uint32_t nq = static_cast<uint32_t>((cw >> 32) & 0xFFu);
  const uint32_t oq = static_cast<uint32_t>((cw >> 40) & 0xFFu);
  const uint32_t kn = nq == 0 ? g.W : kth_largest_rel<P>(g.r, nmask, nq);
  const uint32_t ko = oq == 0 ? g.W : kth_largest_rel<P>(g.r, omask, oq);
  uint32_t cand = kn < ko ? kn : ko;
  cand = cand < g.W ? cand : g.W;
  const int64_t c = pi - 1 + static_cast<int64_t>(cand);
  // commitAt returns false when not the leader (BallotBox.java:101-103): state unchanged
  out = (pi != 0 && cand >= 1u && c > lc) ? c : lc;
  st_out = pi == 0 ? kStNotLeader : st;
}

template <int P>
__device__ __forceinline__ void decide_single_rel(int64_t pi, int64_t la, int64_t lc, uint64_t cw,
                                                  const int64_t (&m)[P], int64_t& out, uint8_t& st_out) {
  RelGroup<P> g;
  rel_map<P>(pi, la, m, g);
  rel_decide<P>(pi, lc, cw, g, out, st_out);
}

// The domain of decide_single_rel: not the leader (pi = 0), or a leader with pendingIndex
// below 2^62 and a window of at most 2^32 - 1 entries -- every real group.  Callers route the rest (negative
// or huge indexes, 4-billion-entry windows) through the 64-bit decide_single, outside their
// fast path: the pair kernel in a second pass, the table by flagging them for its run walk.
__device__ __forceinline__ bool rel_domain(int64_t pi, int64_t la) {
  return pi == 0 ||  // not the leader: lastCommitted, whatever the window
         (pi > 0 && pi < (int64_t{1} << 62) &&
          (la < pi || static_cast<uint64_t>(la - pi) <= 0xFFFFFFFEull));
}

// Runs of one group, in order: run r covers [start(r), start(r+1)) (the last run ends at
// lastAppended, the first starts at or before pendingIndex; a start past lastAppended makes a
// run empty).  best is max(lc, the largest granted index over the runs); each run is
// evaluated on its own, which reproduces the reference's non-monotone commit when an
// even-size conf shrinks (BallotBox.java:124-129).  `Runs` supplies start(r) / conf(r).
// One run: the largest index it grants inside [s, ee] (kI64Min when none, or when the run is
// empty: ee < s); an empty conf on a non-empty run sets kStEmptyConf.
template <int P>
__device__ __forceinline__ int64_t run_candidate(const int64_t (&m)[P], uint64_t cw, int64_t s,
                                                 int64_t ee, uint8_t& st) {
  if (ee < s) return kI64Min;  // run entirely committed already (or empty)
  if ((cw & 0xFFFFu) == 0) st |= kStEmptyConf;
  int64_t cand = run_bound<P>(m, cw);
  cand = cand < ee ? cand : ee;
  return cand >= s ? cand : kI64Min;
}

// run_candidate inside rel_domain, on a group mapped by rel_map: [s, ee] lies inside the
// window [pi, la] (s >= pi by construction, ee <= la), so both ends map to [1, W] and the run
// grants r in [s_rel, e_rel].  Same result and status as run_candidate.
template <int P>
__device__ __forceinline__ int64_t run_candidate_rel(const RelGroup<P>& g, uint64_t cw, int64_t pi,
                                                     int64_t s, int64_t ee, uint8_t& st) {
  if (ee < s) return kI64Min;
  if ((cw & 0xFFFFu) == 0) st |= kStEmptyConf;
  const uint32_t sr = static_cast<uint32_t>(s - pi) + 1u;
  const uint32_t er = static_cast<uint32_t>(ee - pi) + 1u;
  const uint32_t nmask = static_cast<uint32_t>(cw & 0xFFFFu);
  const uint32_t omask = static_cast<uint32_t>((cw >> 16) & 0xFFFFu);
  const uint32_t nq = static_cast<uint32_t>((cw >> 32) & 0xFFu);
  const uint32_t oq = static_cast<uint32_t>((cw >> 40) & 0xFFu);
  const uint32_t kn = nq == 0 ? g.W : kth_largest_rel<P>(g.r, nmask, nq);
  const uint32_t ko = oq == 0 ? g.W : kth_largest_rel<P>(g.r, omask, oq);
  uint32_t c = kn < ko ? kn : ko;
  c = c < er ? c : er;
  return c >= sr ? pi - 1 + static_cast<int64_t>(c) : kI64Min;
}

template <int P, class Runs>
__device__ __forceinline__ int64_t runs_best(const Runs& R, uint32_t nruns, int64_t pi, int64_t la,
                                             int64_t lc, const int64_t (&m)[P], uint8_t& st) {
  int64_t best = lc;
#pragma unroll 1
  for (uint32_t r = 0; r < nruns; ++r) {
    const int64_t rs = R.start(r);
    const int64_t s = (r == 0) ? pi : (rs > pi ? rs : pi);
    const int64_t e = (r + 1 < nruns) ? R.start(r + 1) - 1 : la;
    const int64_t ee = e < la ? e : la;
    if (ee < s) continue;
    const int64_t cand = run_candidate<P>(m, R.conf(r), s, ee, st);
    best = cand > best ? cand : best;
  }
  return best;
}

}  // namespace jrq
