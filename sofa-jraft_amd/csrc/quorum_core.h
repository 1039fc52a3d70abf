// quorum_core.h -- the per-group quorum arithmetic shared by the stateless epoch kernels
// (quorum.hip) and the resident-table kernels (table.hip).  See quorum.hip for the
// formulation and its references (BallotBox.java:96-139, Ballot.java:63-140).
#pragma once

#include "jrq_device.h"

namespace jrq {

constexpr int64_t kI64Min = INT64_MIN;
constexpr int64_t kI64Max = INT64_MAX;
constexpr uint64_t kConfRuns = 1ull << 63;  // include/jrq.h JRQ_CONF_RUNS

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
