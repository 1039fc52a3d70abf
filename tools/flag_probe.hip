// flag_probe.hip -- the resident-table epoch with 1 % of the groups flagged (a conf change in
// the pending window): where do the flagged groups cost time?  (tools only; not part of libjrq)
// A C3-shaped table (1M groups x 5 peers, joint 5/3, every group commits); the flagged groups
// have two conf runs.  Variants, each launch from the same pristine lastCommitted/pendingIndex:
//   noflag     the product kernel on the same table with no group flagged (the baseline)
//   product    table_epoch_kernel<5> (each wave walks its own flagged entries after its fast path)
//   r02        the round-2 kernel (flagged groups deferred to an LDS list behind a barrier)
//   fast_only  the fast path with the flagged groups skipped (no walk: the floor)
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/flag_probe tools/flag_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../sofa-jraft_amd/csrc/table.hip"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      std::exit(1);                                                                          \
    }                                                                                        \
  } while (0)

namespace jrq {
template <int P>
__global__ __launch_bounds__(kTableBlock, 8) JRQ_SGPRS_8WAVES void r02_epoch(JrqTableArgs t) {
  constexpr uint32_t kWaves = kTableBlock / 64;
  __shared__ uint32_t wave_cnt[kWaves];   // fast-path commits per wave
  __shared__ uint32_t wave_def[kWaves];   // flagged groups per wave
  __shared__ uint32_t deferred[kWaves][128];
  __shared__ uint64_t staged[kWaves][128];  // fast-path list entries, wave-compacted
  __shared__ uint64_t walk_staged[kTableBlockGroups];  // run-walk list entries
  __shared__ uint32_t walk_n;
  __shared__ uint32_t blk_base, blk_walk;
  const uint32_t pairs = (t.G + 1) >> 1;  // ld covers the pad group of an odd G (not a leader)
  const uint32_t tt = blockIdx.x * kTableBlock + threadIdx.x;
  const uint32_t g = tt << 1;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
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
    // in the second phase with its runs; its single-conf result here is discarded
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
  // list entries and flagged groups -> the wave's slices of LDS (ballot prefixes, no atomics)
  const uint64_t b0 = __ballot(c0), b1 = __ballot(c1);
  const uint64_t bf0 = __ballot(f0), bf1 = __ballot(f1);
  if (c0) staged[w][__popcll(b0 & below)] = e0;
  if (c1) staged[w][__popcll(b0) + __popcll(b1 & below)] = e1;
  if (f0) deferred[w][__popcll(bf0 & below)] = g;
  if (f1) deferred[w][__popcll(bf0) + __popcll(bf1 & below)] = g + 1;
  if (lane == 0) {
    wave_cnt[w] = __popcll(b0) + __popcll(b1);
    wave_def[w] = __popcll(bf0) + __popcll(bf1);
  }
  if (threadIdx.x == 0) walk_n = 0;
  __syncthreads();
  // second phase: the workgroup's flagged groups, packed four lanes each (one per conf run)
  // onto the first lanes, walk their runs -- ~1% of groups flagged then costs one short pass
  // of one or two waves per workgroup (the walk is VALU-heavy: one per wave, or one per
  // lane with the runs in a loop, measured +8..+12 us per 1M-group epoch)
  uint32_t nd = 0;
#pragma unroll
  for (uint32_t u = 0; u < kWaves; ++u) nd += wave_def[u];
  if (__builtin_expect(nd != 0, 0)) {
    for (uint32_t base = 0; base < nd * kTableMaxRuns; base += kTableBlock) {
      const uint32_t q = base + threadIdx.x, i = q / kTableMaxRuns, r = q % kTableMaxRuns;
      const bool act = i < nd;
      int64_t cand = kI64Min, pr = 0, lc = 0, pi = 0;
      uint8_t st = 0;
      uint32_t h = 0;
      if (act) {
        uint32_t k = i, u = 0;
        while (k >= wave_def[u]) k -= wave_def[u++];
        h = deferred[u][k];
        cand = table_run_lane<P>(t, h, r, pr, lc, pi, st);
      }
      cand = max(cand, static_cast<int64_t>(__shfl_xor(static_cast<long long>(cand), 1)));
      cand = max(cand, static_cast<int64_t>(__shfl_xor(static_cast<long long>(cand), 2)));
      uint32_t s32 = st;
      s32 |= __shfl_xor(s32, 1);
      s32 |= __shfl_xor(s32, 2);
      if (act && r == 0) {
        if (t.status) t.status[h] = static_cast<uint8_t>(s32);
        if (cand > lc) {  // pi == 0 (not the leader) returned kI64Min
          table_commit_one(t, h, pr, cand);
          walk_staged[atomicAdd(&walk_n, 1u)] = (static_cast<uint64_t>(cand - pi + 1) << 32) | h;
        }
      }
    }
    __syncthreads();
  }
  // compaction: fast-path entries in (wave, lane) order, then the run walk's; one
  // 64-bit atomic per workgroup ({workgroups done << 32 | entries}) on its segment's counter
  // reserves the workgroup's slice, and the last workgroup of a segment publishes its count
  // and re-zeroes the counter
  const uint32_t seg = blockIdx.x % kTableSegments;
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (uint32_t u = 0; u < kWaves; ++u) tot += wave_cnt[u];
    blk_walk = tot;
    tot += walk_n;
    const unsigned long long old = atomicAdd(t.ctr + seg, (1ull << 32) | tot);
    blk_base = seg * t.seg_cap + static_cast<uint32_t>(old);
    blk_walk += blk_base;
    const uint32_t seg_blocks = (gridDim.x - seg + kTableSegments - 1) / kTableSegments;
    if (static_cast<uint32_t>(old >> 32) + 1u == seg_blocks) {  // the segment is complete
      t.n_changed[seg] = static_cast<uint32_t>(old) + tot;
      atomicExch(t.ctr + seg, 0ull);
    }
  }
  __syncthreads();
  uint32_t pos = blk_base;
  for (uint32_t u = 0; u < w; ++u) pos += wave_cnt[u];
  const uint32_t nw = wave_cnt[w];
  if (lane < nw) t.changed[pos + lane] = staged[w][lane];
  if (lane + 64 < nw) t.changed[pos + lane + 64] = staged[w][lane + 64];
  if (__builtin_expect(nd != 0, 0))
    for (uint32_t i = threadIdx.x; i < walk_n; i += kTableBlock) t.changed[blk_walk + i] = walk_staged[i];
}

}  // namespace jrq

namespace probe {
using namespace jrq;

// the fast path only: flagged groups skipped, no walk (the floor the walk is measured against)
template <int P>
__global__ __launch_bounds__(kTableBlock, 8) JRQ_SGPRS_8WAVES void fast_only(JrqTableArgs t) {
  constexpr uint32_t kWaves = kTableBlock / 64;
  __shared__ uint32_t wave_cnt[kWaves];
  __shared__ uint64_t staged[kWaves][128];
  __shared__ uint32_t blk_base;
  const uint32_t pairs = (t.G + 1) >> 1;
  const uint32_t tt = blockIdx.x * kTableBlock + threadIdx.x;
  const uint32_t g = tt << 1;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
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
    const bool f0 = static_cast<uint64_t>(cw.x) >> 63;
    const bool f1 = static_cast<uint64_t>(cw.y) >> 63;
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
  }
  const uint64_t b0 = __ballot(c0), b1 = __ballot(c1);
  if (c0) staged[w][__popcll(b0 & below)] = e0;
  if (c1) staged[w][__popcll(b0) + __popcll(b1 & below)] = e1;
  const uint32_t cnt = __popcll(b0) + __popcll(b1);
  if (lane == 0) wave_cnt[w] = cnt;
  lds_barrier();
  const uint32_t seg = blockIdx.x % kTableSegments;
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (uint32_t u = 0; u < kWaves; ++u) tot += wave_cnt[u];
    const unsigned long long old = atomicAdd(t.ctr + seg, (1ull << 32) | tot);
    blk_base = seg * t.seg_cap + static_cast<uint32_t>(old);
    const uint32_t seg_blocks = (gridDim.x - seg + kTableSegments - 1) / kTableSegments;
    if (static_cast<uint32_t>(old >> 32) + 1u == seg_blocks) {
      t.n_changed[seg] = static_cast<uint32_t>(old) + tot;
      atomicExch(t.ctr + seg, 0ull);
    }
  }
  lds_barrier();
  uint32_t pos = blk_base;
  for (uint32_t u = 0; u < w; ++u) pos += wave_cnt[u];
  for (uint32_t i = lane; i < cnt; i += 64) t.changed[pos + i] = staged[w][i];
}

__global__ void init(JrqTableArgs t, uint64_t seed, uint32_t flag_ppm) {
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
  const uint64_t joint = 0x1Full | (0x07ull << 16) | (3ull << 32) | (2ull << 40);  // new 5 + old 3
  const bool flagged = rnd(7) % 1000000 < flag_ppm;
  t.conf[g] = joint | (flagged ? kConfRuns : 0ull);
  for (int k = 0; k < 3; ++k) {
    t.xstart[k * t.ld + g] = (flagged && k == 0) ? pi + 1 + static_cast<int64_t>(rnd(6) % 1000) : kI64Max;
    t.xconf[k * t.ld + g] = (flagged && k == 0) ? (0x1Full | (3ull << 32)) : 0ull;
  }
  t.match[g] = pi + 1023;
  for (uint32_t p = 1; p < t.P; ++p) t.match[p * t.ld + g] = pi - 1 + static_cast<int64_t>(rnd(p) % 1025);
}

}  // namespace probe

using jrq::kTableBlockGroups;
int main() {
  const uint32_t G = 1u << 20, P = 5;
  const uint64_t ld = G;
  const uint32_t blocks = (G + kTableBlockGroups - 1) / kTableBlockGroups;
  JrqTableArgs a{};
  int64_t* mem;
  const size_t words = ld * (P + 4 + 6) + static_cast<size_t>(blocks) * 16 * (jrq::kFlagSlots * 8 + 1);
  CK(hipMalloc(&mem, words * 8 + 256));
  CK(hipMemset(mem, 0, words * 8 + 256));
  a.match = mem;
  a.pi = mem + ld * P;
  a.la = a.pi + ld;
  a.lc = a.la + ld;
  a.conf = reinterpret_cast<uint64_t*>(a.lc + ld);
  a.xstart = reinterpret_cast<int64_t*>(a.conf + ld);
  a.xconf = reinterpret_cast<uint64_t*>(a.xstart + ld * 3);
  a.flag_ent = reinterpret_cast<uint64_t*>(a.xconf + ld * 3);
  a.flag_wcnt = reinterpret_cast<uint32_t*>(a.flag_ent + static_cast<size_t>(blocks) * 16 * jrq::kFlagSlots * 8);
  a.ctr = reinterpret_cast<unsigned long long*>(mem + words);
  a.invalid = reinterpret_cast<uint32_t*>(a.ctr + 16);
  a.ld = ld;
  a.G = G;
  a.P = P;
  CK(hipMalloc(&a.changed, static_cast<size_t>(G) * 8 * 17 + 8 * 65536));
  CK(hipMalloc(&a.n_changed, 64));
  a.seg_cap = jrq_table_seg_cap(G);
  unsigned long long* wctr;
  CK(hipMalloc(&wctr, 8));
  int64_t *pi0, *lc0;
  CK(hipMalloc(&pi0, G * 8));
  CK(hipMalloc(&lc0, G * 8));
  const dim3 grid(((G + 1) / 2 + jrq::kTableBlock - 1) / jrq::kTableBlock), blk(jrq::kTableBlock);
  hipStream_t sa;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  auto setup = [&](uint32_t ppm) {
    hipLaunchKernelGGL(probe::init, dim3(G / 256), dim3(256), 0, sa, a, 12345ull, ppm);
    hipLaunchKernelGGL(jrq::table_flags_kernel, dim3(blocks), dim3(jrq::kFlagBlock), 0, sa, a);
    CK(hipMemcpyAsync(pi0, a.pi, G * 8, hipMemcpyDeviceToDevice, sa));
    CK(hipMemcpyAsync(lc0, a.lc, G * 8, hipMemcpyDeviceToDevice, sa));
    CK(hipStreamSynchronize(sa));
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    std::vector<float> ms;
    for (int i = 0; i < 45; ++i) {
      CK(hipMemcpyAsync(a.pi, pi0, G * 8, hipMemcpyDeviceToDevice, sa));
      CK(hipMemcpyAsync(a.lc, lc0, G * 8, hipMemcpyDeviceToDevice, sa));
      CK(hipMemsetAsync(wctr, 0, 8, sa));
      CK(hipEventRecord(e0, sa));
      launch();
      CK(hipEventRecord(e1, sa));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (i >= 5) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    uint32_t cnt[16] = {}, n = 0;
    unsigned long long wn = 0;
    CK(hipMemcpy(cnt, a.n_changed, 64, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&wn, wctr, 8, hipMemcpyDeviceToHost));
    for (uint32_t c : cnt) n += c;
    std::printf("%-14s median %.2f us  min %.2f us  (listed %u + walker %llu)\n", name,
                ms[ms.size() / 2] * 1e3, ms[0] * 1e3, n, wn);
  };
  for (uint32_t ppm : {0u, 10000u}) {
    setup(ppm);
    std::printf("-- %u ppm flagged\n", ppm);
    run("product", [&] { hipLaunchKernelGGL(jrq::table_epoch_kernel<5>, grid, blk, 0, sa, a); });
    if (!ppm) continue;
    run("r02", [&] { hipLaunchKernelGGL(jrq::r02_epoch<5>, grid, blk, 0, sa, a); });
    run("fast_only", [&] { hipLaunchKernelGGL(probe::fast_only<5>, grid, blk, 0, sa, a); });
    run("product_again", [&] { hipLaunchKernelGGL(jrq::table_epoch_kernel<5>, grid, blk, 0, sa, a); });
  }
  CK(hipDeviceSynchronize());
  return 0;
}
