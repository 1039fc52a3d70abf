// table_probe.hip -- where the resident-table epoch spends its time (tools only; not part of
// libjrq).  Times, on a C3-shaped table (1M groups x 5 peers, joint conf, every group
// commits), the product kernel against variants that drop one piece at a time:
//   product      table_epoch_kernel<5> as in libjrq (in place + compacted list, 1 atomic / WG)
//   no_atomic    same, each workgroup writes its entries at its own fixed slice (no atomic)
//   no_list      in-place writes only (lastCommitted / pendingIndex), no list at all
//   pair         the stateless quorum_epoch_pair_kernel<5> on the same arrays (committed to a
//                separate array, status bytes)
// Each launch starts from the same pristine lastCommitted / pendingIndex (restored by a copy
// outside the event pair).
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/table_probe tools/table_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../sofa-jraft_amd/csrc/quorum.hip"
#include "../sofa-jraft_amd/csrc/table.hip"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      std::exit(1);                                                                          \
    }                                                                                        \
  } while (0)

namespace probe {

using namespace jrq;

// kMode 1: fixed per-workgroup slices, 2: no list
template <int P, int kMode>
__global__ __launch_bounds__(kTableBlock) void variant(JrqTableArgs t) {
  constexpr uint32_t kWaves = kTableBlock / 64;
  __shared__ uint32_t wave_cnt[kWaves];
  const uint32_t pairs = (t.G + 1) >> 1;
  const uint32_t tt = blockIdx.x * kTableBlock + threadIdx.x;
  const uint32_t g = tt << 1;
  bool c0 = false, c1 = false;
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
    c0 = o0 > lc.x;
    c1 = o1 > lc.y;
    if (c0 || c1) {
      i64x2 o;
      o.x = o0;
      o.y = o1;
      __builtin_nontemporal_store(o, reinterpret_cast<i64x2*>(t.lc + g));
      if (c0 && pr.x != kPiFollowsLc) t.pi[g] = kPiFollowsLc;
      if (c1 && pr.y != kPiFollowsLc) t.pi[g + 1] = kPiFollowsLc;
    }
    e0 = (static_cast<uint64_t>(o0 - pi0 + 1) << 32) | g;
    e1 = (static_cast<uint64_t>(o1 - pi1 + 1) << 32) | (g + 1);
  }
  if (kMode == 2) return;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t b0 = __ballot(c0), b1 = __ballot(c1);
  const uint64_t below = (1ull << lane) - 1ull;
  const uint32_t pre = __popcll(b0 & below) + __popcll(b1 & below);
  if (lane == 0) wave_cnt[w] = __popcll(b0) + __popcll(b1);
  __syncthreads();
  uint32_t pos = blockIdx.x * 2 * kTableBlock + pre;
  for (uint32_t u = 0; u < w; ++u) pos += wave_cnt[u];
  if (c0) t.changed[pos++] = e0;
  if (c1) t.changed[pos] = e1;
}

// the product's structure with pieces switched: kAtomic (segment counter; else fixed slices),
// kPhase2 (deferred list + second phase + its sync), kWaveAtomic (one atomic per wave, no
// workgroup-wide sync around it)
template <int P, bool kAtomic, bool kPhase2, bool kWaveAtomic>
__global__ __launch_bounds__(kTableBlock) void variant2(JrqTableArgs t) {
  constexpr uint32_t kWaves = kTableBlock / 64;
  __shared__ uint32_t wave_cnt[kWaves];
  __shared__ uint32_t blk_base;
  __shared__ uint32_t n_deferred;
  __shared__ uint32_t deferred[2 * kTableBlock];
  const uint32_t pairs = (t.G + 1) >> 1;
  const uint32_t tt = blockIdx.x * kTableBlock + threadIdx.x;
  const uint32_t g = tt << 1;
  if (kPhase2) {
    if (threadIdx.x == 0) n_deferred = 0;
    __syncthreads();
  }
  bool c0 = false, c1 = false;
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
    const bool f0 = static_cast<uint64_t>(cw.x) >> 63, f1 = static_cast<uint64_t>(cw.y) >> 63;
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
    c0 = !f0 && o0 > lc.x;
    c1 = !f1 && o1 > lc.y;
    if (c0 && c1) {
      i64x2 o;
      o.x = o0;
      o.y = o1;
      __builtin_nontemporal_store(o, reinterpret_cast<i64x2*>(t.lc + g));
      if (pr.x != kPiFollowsLc) t.pi[g] = kPiFollowsLc;
      if (pr.y != kPiFollowsLc) t.pi[g + 1] = kPiFollowsLc;
    } else {
      if (c0) table_commit_one(t, g, pr.x, o0);
      if (c1) table_commit_one(t, g + 1, pr.y, o1);
    }
    e0 = (static_cast<uint64_t>(o0 - pi0 + 1) << 32) | g;
    e1 = (static_cast<uint64_t>(o1 - pi1 + 1) << 32) | (g + 1);
    if (kPhase2) {
      if (f0) deferred[atomicAdd(&n_deferred, 1u)] = g;
      if (f1) deferred[atomicAdd(&n_deferred, 1u)] = g + 1;
    }
  }
  bool cd[2] = {false, false};
  uint64_t ed[2] = {0, 0};
  if (kPhase2) {
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < 2; ++j) {
      const uint32_t i = threadIdx.x + kTableBlock * j;
      if (i >= n_deferred) break;
      const uint32_t h = deferred[i];
      const int64_t pr = t.pi[h], lc = t.lc[h], la = t.la[h];
      const uint64_t cw = t.conf[h];
      int64_t m[P];
#pragma unroll
      for (int p = 0; p < P; ++p) m[p] = t.match[static_cast<size_t>(p) * t.ld + h];
      const int64_t pi = pr == kPiFollowsLc ? lc + 1 : pr;
      int64_t out = lc;
      uint8_t st = kStNotLeader;
      if (pi != 0) {
        st = mask_out_of_range<P>(m, la);
        const TableRuns R{&t, h, cw & ~kConfRuns};
        out = runs_best<P>(R, kTableMaxRuns, pi, la, lc, m, st);
      }
      cd[j] = out > lc;
      if (cd[j]) table_commit_one(t, h, pr, out);
      ed[j] = (static_cast<uint64_t>(out - pi + 1) << 32) | h;
    }
  }
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t b0 = __ballot(c0), b1 = __ballot(c1), b2 = __ballot(cd[0]), b3 = __ballot(cd[1]);
  const uint64_t below = (1ull << lane) - 1ull;
  const uint32_t pre = __popcll(b0 & below) + __popcll(b1 & below) + __popcll(b2 & below) +
                       __popcll(b3 & below);
  const uint32_t wc = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
  const uint32_t seg = blockIdx.x % kTableSegments;
  uint32_t pos;
  if (kWaveAtomic) {
    uint32_t base = 0;
    if (lane == 0 && wc) base = static_cast<uint32_t>(atomicAdd(t.ctr + seg, wc));
    base = __shfl(base, 0);
    pos = seg * t.seg_cap * 16 + base + pre;  // counts only: the probe ignores n_changed here
  } else {
    if (lane == 0) wave_cnt[w] = wc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tot = 0;
      for (uint32_t u = 0; u < kWaves; ++u) tot += wave_cnt[u];
      if (kAtomic) {
        const unsigned long long old = atomicAdd(t.ctr + seg, (1ull << 32) | tot);
        blk_base = seg * t.seg_cap + static_cast<uint32_t>(old);
        const uint32_t seg_blocks = (gridDim.x - seg + kTableSegments - 1) / kTableSegments;
        if (static_cast<uint32_t>(old >> 32) + 1u == seg_blocks) {
          t.n_changed[seg] = static_cast<uint32_t>(old) + tot;
          atomicExch(t.ctr + seg, 0ull);
        }
      } else {
        blk_base = blockIdx.x * kTableBlockGroups;
      }
    }
    __syncthreads();
    pos = blk_base + pre;
    for (uint32_t u = 0; u < w; ++u) pos += wave_cnt[u];
  }
  if (c0) t.changed[pos++] = e0;
  if (c1) t.changed[pos++] = e1;
  if (cd[0]) t.changed[pos++] = ed[0];
  if (cd[1]) t.changed[pos] = ed[1];
}

// a copy of the product kernel with pieces switched off: kStatus (status stores), kRuns (run walk)
template <int P, bool kStatus, bool kRuns>
__global__ __launch_bounds__(kTableBlock) void variant3(JrqTableArgs t) {
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
    if (kStatus && t.status) {  // a flagged group's status is written by the run walk
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
  if (kRuns && __builtin_expect(f0, 0)) {
    int64_t pi;
    uint8_t st;
    const int64_t d = table_runs_one<P>(t, g, pi, st);
    if (t.status) t.status[g] = st;
    c0 = d > 0;
    e0 = (static_cast<uint64_t>(t.lc[g] - pi + 1) << 32) | g;
  }
  if (kRuns && __builtin_expect(f1, 0)) {
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

__global__ void zero_ctr(JrqTableArgs t) {
  if (threadIdx.x < kTableSegments) t.ctr[threadIdx.x] = 0;
}

__global__ void init(JrqTableArgs t, uint64_t seed) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  if (g >= t.G) return;
  auto rnd = [&](uint64_t k) {
    uint64_t z = seed + (static_cast<uint64_t>(g) * 8 + k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  const int64_t pi = 1 + static_cast<int64_t>(rnd(0) % (1ull << 40));
  t.pi[g] = kPiFollowsLc;
  t.lc[g] = pi - 1;
  t.la[g] = pi + 1023;
  t.conf[g] = 0x1Full | (0x07ull << 16) | (3ull << 32) | (2ull << 40);  // new 5 + old 3
  t.match[g] = pi + 1023;
  for (uint32_t p = 1; p < t.P; ++p) t.match[p * t.ld + g] = pi - 1 + static_cast<int64_t>(rnd(p) % 1025);
}

}  // namespace probe

int main() {
  const uint32_t G = 1u << 20, P = 5;
  const uint64_t ld = G;
  JrqTableArgs a{};
  int64_t* mem;
  const size_t words = ld * (P + 4 + 6);
  CK(hipMalloc(&mem, words * 8 + 256));
  CK(hipMemset(mem, 0, words * 8 + 256));
  a.match = mem;
  a.pi = mem + ld * P;
  a.la = a.pi + ld;
  a.lc = a.la + ld;
  a.conf = reinterpret_cast<uint64_t*>(a.lc + ld);
  a.xstart = reinterpret_cast<int64_t*>(a.conf + ld);
  a.xconf = reinterpret_cast<uint64_t*>(a.xstart + ld * 3);
  a.ctr = reinterpret_cast<unsigned long long*>(a.xconf + ld * 3);
  a.invalid = reinterpret_cast<uint32_t*>(a.ctr + 16);
  a.ld = ld;
  a.G = G;
  a.P = P;
  CK(hipMalloc(&a.changed, static_cast<size_t>(G) * 8 * 17 + 8 * 65536));
  CK(hipMalloc(&a.n_changed, 64));
  a.seg_cap = jrq_table_seg_cap(G);
  hipLaunchKernelGGL(probe::init, dim3(G / 256), dim3(256), 0, 0, a, 12345ull);
  int64_t *pi0, *lc0;
  CK(hipMalloc(&pi0, G * 8));
  CK(hipMalloc(&lc0, G * 8));
  CK(hipMemcpy(pi0, a.pi, G * 8, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(lc0, a.lc, G * 8, hipMemcpyDeviceToDevice));
  const dim3 grid(((G + 1) / 2 + jrq::kTableBlock - 1) / jrq::kTableBlock), blk(jrq::kTableBlock);
  auto run = [&](const char* name, auto launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int i = 0; i < 25; ++i) {
      CK(hipMemcpyAsync(a.pi, pi0, G * 8, hipMemcpyDeviceToDevice, 0));
      CK(hipMemcpyAsync(a.lc, lc0, G * 8, hipMemcpyDeviceToDevice, 0));
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (i >= 5) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    uint32_t cnt[16] = {}, n = 0;
    CK(hipMemcpy(cnt, a.n_changed, 64, hipMemcpyDeviceToHost));
    for (uint32_t c : cnt) n += c;
    std::printf("%-12s median %.2f us  min %.2f us  (n_changed word %u)\n", name,
                ms[ms.size() / 2] * 1e3, ms[0] * 1e3, n);
  };
  run("product", [&] { hipLaunchKernelGGL(jrq::table_epoch_kernel<5>, grid, blk, 0, 0, a); });
  run("no_atomic", [&] { hipLaunchKernelGGL((probe::variant<5, 1>), grid, blk, 0, 0, a); });
  run("v2_full", [&] { hipLaunchKernelGGL((probe::variant2<5, true, true, false>), grid, blk, 0, 0, a); });
  run("v2_noatomic", [&] { hipLaunchKernelGGL((probe::variant2<5, false, true, false>), grid, blk, 0, 0, a); });
  run("v2_nophase2", [&] { hipLaunchKernelGGL((probe::variant2<5, true, false, false>), grid, blk, 0, 0, a); });
  run("v2_bare", [&] { hipLaunchKernelGGL((probe::variant2<5, false, false, false>), grid, blk, 0, 0, a); });
  run("v3_full", [&] { hipLaunchKernelGGL((probe::variant3<5, true, true>), grid, blk, 0, 0, a); });
  run("v3_nostatus", [&] { hipLaunchKernelGGL((probe::variant3<5, false, true>), grid, blk, 0, 0, a); });
  run("v3_noruns", [&] { hipLaunchKernelGGL((probe::variant3<5, true, false>), grid, blk, 0, 0, a); });
  run("v3_neither", [&] { hipLaunchKernelGGL((probe::variant3<5, false, false>), grid, blk, 0, 0, a); });
  run("v2_waveatom", [&] {
    hipLaunchKernelGGL(probe::zero_ctr, dim3(1), dim3(64), 0, 0, a);
    hipLaunchKernelGGL((probe::variant2<5, true, true, true>), grid, blk, 0, 0, a);
  });
  run("v2_waveatom_np2", [&] {
    hipLaunchKernelGGL(probe::zero_ctr, dim3(1), dim3(64), 0, 0, a);
    hipLaunchKernelGGL((probe::variant2<5, true, false, true>), grid, blk, 0, 0, a);
  });
  run("no_list", [&] { hipLaunchKernelGGL((probe::variant<5, 2>), grid, blk, 0, 0, a); });
  JrqQuorumArgs q{};
  int64_t* committed;
  uint8_t* status;
  CK(hipMalloc(&committed, G * 8));
  CK(hipMalloc(&status, G));
  CK(hipMemcpy(a.pi, lc0, G * 8, hipMemcpyDeviceToDevice));  // pendingIndex = lc + 1 below
  q.match = a.match;
  q.pending_index = a.la;  // any valid pendingIndex <= la: the pair kernel's reads are what count
  q.last_appended = a.la;
  q.last_committed = a.lc;
  q.conf = a.conf;
  q.num_peers = P;
  q.match_ld = ld;
  q.committed = committed;
  q.status = status;
  q.G = G;
  const dim3 pgrid(G / 2 / 256), pblk(256);
  run("pair", [&] { hipLaunchKernelGGL(jrq::quorum_epoch_pair_kernel<5>, pgrid, pblk, 0, 0, q); });
  run("product2", [&] { hipLaunchKernelGGL(jrq::table_epoch_kernel<5>, grid, blk, 0, 0, a); });
  CK(hipDeviceSynchronize());
  return 0;
}
