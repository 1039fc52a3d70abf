// table_probe.hip -- where the resident-table epoch spends its time (tools only; not part of
// libjrq).  Times, on a C3-shaped table (1M groups x 5 peers, joint conf, every group
// commits), the product kernel against variants that drop one piece at a time:
//   product      table_epoch_kernel<5> as in libjrq (in place + compacted list, 1 atomic / WG)
//   no_atomic    the fast path alone, each workgroup writing its entries at its own fixed
//                slice (no atomic, no run-walk phase)
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


// the headline pair kernel's fast path (no run tables) with other launch shapes: kBlock threads
// per workgroup, kU pairs per lane (kU pairs kBlock*gridDim apart, all loads issued first)
template <int P, int kBlock, int kU>
__global__ __launch_bounds__(kBlock) JRQ_SGPRS_8WAVES void pair_variant(JrqQuorumArgs a) {
  const uint32_t pairs = a.G >> 1;
  const uint32_t stride = gridDim.x * kBlock;
  const uint32_t t0 = blockIdx.x * kBlock + threadIdx.x;
  i64x2 pi[kU], lc[kU], la[kU], cw[kU], m[kU][P];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const uint32_t t = t0 + u * stride;
    const uint32_t g = (t < pairs ? t : 0u) << 1;
    pi[u] = ld2nt(a.pending_index + g);
    lc[u] = ld2nt(a.last_committed + g);
    la[u] = ld2nt(a.last_appended + g);
    cw[u] = ld2nt(reinterpret_cast<const int64_t*>(a.conf) + g);
#pragma unroll
    for (int p = 0; p < P; ++p) m[u][p] = ld2nt(a.match + static_cast<size_t>(p) * a.match_ld + g);
  }
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const uint32_t t = t0 + u * stride;
    if (t >= pairs) continue;
    const uint32_t g = t << 1;
    int64_t m0[P], m1[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      m0[p] = m[u][p].x;
      m1[p] = m[u][p].y;
    }
    int64_t o0, o1;
    uint8_t s0, s1;
    decide_single<P>(pi[u].x, la[u].x, lc[u].x, static_cast<uint64_t>(cw[u].x), m0, o0, s0);
    decide_single<P>(pi[u].y, la[u].y, lc[u].y, static_cast<uint64_t>(cw[u].y), m1, o1, s1);
    i64x2 out;
    out.x = o0;
    out.y = o1;
    __builtin_nontemporal_store(out, reinterpret_cast<i64x2*>(a.committed + g));
    __builtin_nontemporal_store(static_cast<uint16_t>(s0 | (s1 << 8)),
                                reinterpret_cast<uint16_t*>(a.status + g));
  }
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
  // the flagged-entry slots the product kernel reads (no group flagged here: all zero), laid
  // out as jrq_table_create lays them out
  {
    const size_t waves = static_cast<size_t>((G + jrq::kTableBlockGroups - 1) / jrq::kTableBlockGroups) *
                         (jrq::kTableBlockGroups / 128);
    const size_t fbytes = waves * jrq::kFlagSlots * 64 + waves * 4 + 64;
    CK(hipMalloc(&a.flag_ent, fbytes));
    CK(hipMemset(a.flag_ent, 0, fbytes));
    a.flag_wcnt = reinterpret_cast<uint32_t*>(a.flag_ent + waves * jrq::kFlagSlots * 8);
  }
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
  const dim3 pgrid(G / 2 / jrq::kPairBlock), pblk(jrq::kPairBlock);
  run("pair", [&] { hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<5, false>), pgrid, pblk, 0, 0, q); });
  const uint32_t np = G / 2;
  run("pv_256_u1", [&] { hipLaunchKernelGGL((probe::pair_variant<5, 256, 1>), dim3(np / 256), dim3(256), 0, 0, q); });
  run("pv_512_u1", [&] { hipLaunchKernelGGL((probe::pair_variant<5, 512, 1>), dim3(np / 512), dim3(512), 0, 0, q); });
  run("pv_1024_u1", [&] { hipLaunchKernelGGL((probe::pair_variant<5, 1024, 1>), dim3(np / 1024), dim3(1024), 0, 0, q); });
  run("pv_256_u2", [&] { hipLaunchKernelGGL((probe::pair_variant<5, 256, 2>), dim3(np / 512), dim3(256), 0, 0, q); });
  run("pv_256_u4", [&] { hipLaunchKernelGGL((probe::pair_variant<5, 256, 4>), dim3(np / 1024), dim3(256), 0, 0, q); });
  run("pv_512_u2", [&] { hipLaunchKernelGGL((probe::pair_variant<5, 512, 2>), dim3(np / 1024), dim3(512), 0, 0, q); });
  run("pair_again", [&] { hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<5, false>), pgrid, pblk, 0, 0, q); });
  run("product2", [&] { hipLaunchKernelGGL(jrq::table_epoch_kernel<5>, grid, blk, 0, 0, a); });
  CK(hipDeviceSynchronize());
  return 0;
}
