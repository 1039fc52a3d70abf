// crc_timeline.hip -- per-wave timeline of the CRC64 rounds kernel (tools only; diagnostics).
//
// Launches crc64_rounds_kernel (csrc/crc64.hip) on a C5-shaped batch (64k x 16 KiB entries,
// 1 GiB) with JrqCrcArgs::timeline set, and prints when each wave started and ended
// (s_memrealtime, 100 MHz) by XCC, plus the spread of start times: shows whether every
// workgroup runs concurrently and how evenly the waves finish.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/crc_timeline tools/crc_timeline.hip
//   run:   tools/crc_timeline [grid] [seg_bytes] [seg_map] [prio_steps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "../sofa-jraft_amd/csrc/crc64.hip"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

static uint64_t mulmod(uint64_t a, uint64_t b) {
  uint64_t r = 0;
  for (int i = 63; i >= 0; --i) {
    r = (r & 0x8000000000000000ULL) ? (r << 1) ^ jrq::kCrcPoly : (r << 1);
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = argc > 1 ? std::atoi(argv[1]) : prop.multiProcessorCount;
  const uint64_t seg_bytes = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 0;
  const uint32_t seg_map = argc > 3 ? std::atoi(argv[3]) : 0;
  const uint32_t n = 64 << 10, L = 16 << 10;
  const uint64_t total = (uint64_t)n * L;
  // tables (engine.hip build_tables): slice R_j = bswap(T_j); shift[t][k][i]
  uint64_t t[8][256], T0[256];
  for (int i = 0; i < 256; ++i) {
    uint64_t c = (uint64_t)i << 56;
    for (int k = 0; k < 8; ++k) c = (c & 0x8000000000000000ULL) ? (c << 1) ^ jrq::kCrcPoly : (c << 1);
    t[0][i] = T0[i] = c;
  }
  for (int j = 1; j < 8; ++j)
    for (int i = 0; i < 256; ++i) t[j][i] = t[0][t[j - 1][i] >> 56] ^ (t[j - 1][i] << 8);
  std::vector<uint64_t> slice(8 * 256), shift((size_t)jrq::kShiftTables * 8 * 256);
  for (int j = 0; j < 8; ++j)
    for (int i = 0; i < 256; ++i) slice[j * 256 + i] = __builtin_bswap64(t[j][i]);
  uint64_t K = 0x100;
  for (int tt = 0; tt < jrq::kShiftTables; ++tt) {
    for (int k = 0; k < 8; ++k)
      for (int i = 0; i < 256; ++i) shift[((size_t)tt * 8 + k) * 256 + i] = mulmod((uint64_t)i << (8 * k), K);
    K = mulmod(K, K);
  }
  std::vector<uint8_t> h(total);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < total / 8; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    std::memcpy(&h[i * 8], &x, 8);
  }
  std::vector<uint64_t> offs(n + 1);
  for (uint32_t e = 0; e <= n; ++e) offs[e] = (uint64_t)e * L;
  uint8_t* d_pay;
  uint64_t *d_off, *d_out, *d_slice, *d_shift, *d_acc, *d_pieces, *d_tl;
  uint32_t* d_cnt;
  const uint32_t lanes = grid * jrq::kCrcBlock, scratch = 2 * lanes + 2;
  const size_t nwaves = (size_t)grid * (jrq::kCrcBlock / 64);
  CK(hipMalloc(&d_pay, total));
  CK(hipMemcpy(d_pay, h.data(), total, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_off, offs.size() * 8));
  CK(hipMemcpy(d_off, offs.data(), offs.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_out, (size_t)n * 8));
  CK(hipMalloc(&d_slice, slice.size() * 8));
  CK(hipMemcpy(d_slice, slice.data(), slice.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_shift, shift.size() * 8));
  CK(hipMemcpy(d_shift, shift.data(), shift.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_acc, (size_t)scratch * 8));
  CK(hipMemset(d_acc, 0, (size_t)scratch * 8));
  CK(hipMalloc(&d_cnt, (size_t)scratch * 4));
  CK(hipMemset(d_cnt, 0, (size_t)scratch * 4));
  CK(hipMalloc(&d_pieces, (size_t)scratch * 16));
  CK(hipMalloc(&d_tl, nwaves * 32));
  JrqCrcArgs a{};
  a.payload = d_pay;
  a.offsets = d_off;
  a.n = n;
  a.out = d_out;
  a.slice = d_slice;
  a.shift = d_shift;
  a.acc = d_acc;
  a.cnt = d_cnt;
  a.piece_cont = d_pieces;
  a.piece_tail = d_pieces + scratch;
  a.scratch_len = scratch;
  a.seg_bytes = seg_bytes;
  a.seg_map = seg_map;
  a.timeline = d_tl;
  a.prio_steps = argc > 4 ? std::atoi(argv[4]) : 1;
  hipEvent_t ev0, ev1;
  CK(hipEventCreate(&ev0));
  CK(hipEventCreate(&ev1));
  float best = 1e9f;
  for (int rep = 0; rep < 6; ++rep) {
    CK(hipEventRecord(ev0));
    CK(jrq_launch_crc64(&a, 0, grid, 0));
    CK(hipEventRecord(ev1));
    CK(hipEventSynchronize(ev1));
    float ms;
    CK(hipEventElapsedTime(&ms, ev0, ev1));
    best = std::min(best, ms);
  }
  // correctness spot check (a few whole entries)
  std::vector<uint64_t> out(n);
  CK(hipMemcpy(out.data(), d_out, (size_t)n * 8, hipMemcpyDeviceToHost));
  int bad = 0;
  for (uint32_t e = 0; e < n; e += 4099) {
    uint64_t c = 0;
    for (uint64_t i = offs[e]; i < offs[e + 1]; ++i) c = T0[((c >> 56) ^ h[i]) & 0xFF] ^ (c << 8);
    bad += c != out[e];
  }
  std::vector<uint64_t> tl(nwaves * 4);
  CK(hipMemcpy(tl.data(), d_tl, tl.size() * 8, hipMemcpyDeviceToHost));
  uint64_t s_min = ~0ull, e_max = 0;
  for (size_t w = 0; w < nwaves; ++w) {
    s_min = std::min(s_min, tl[4 * w]);
    e_max = std::max(e_max, tl[4 * w + 1]);
  }
  std::printf("grid %d seg_bytes %llu map %u: best %.4f ms (%.0f GB/s incl. finish kernel), %s\n", grid,
              (unsigned long long)seg_bytes, seg_map, best, total / (best * 1e-3) / 1e9,
              bad ? "MISMATCH" : "spot-check ok");
  std::printf("last launch: first start -> last end %.1f us\n", (e_max - s_min) / 100.0);
  // per XCC: waves, distinct CUs, start spread, end spread, mean duration (us)
  std::map<int, std::vector<size_t>> by_xcc;
  for (size_t w = 0; w < nwaves; ++w) by_xcc[(int)(tl[4 * w + 3] & 0xF)].push_back(w);
  for (auto& kv : by_xcc) {
    std::map<uint64_t, int> cus;
    double s_lo = 1e18, s_hi = 0, e_lo = 1e18, e_hi = 0, dur = 0;
    for (size_t w : kv.second) {
      const uint64_t hw = tl[4 * w + 2];
      cus[(hw >> 8) & 0xFF]++;  // CU_ID | SH_ID | SE_ID
      const double s = (tl[4 * w] - s_min) / 100.0, e = (tl[4 * w + 1] - s_min) / 100.0;
      s_lo = std::min(s_lo, s); s_hi = std::max(s_hi, s);
      e_lo = std::min(e_lo, e); e_hi = std::max(e_hi, e);
      dur += e - s;
    }
    std::printf("xcc %d: waves %zu cus %zu  start %.1f..%.1f  end %.1f..%.1f  mean dur %.1f us\n",
                kv.first, kv.second.size(), cus.size(), s_lo, s_hi, e_lo, e_hi,
                dur / kv.second.size());
  }
  // within-workgroup vs across-workgroup spread of wave end times; per-SIMD order
  {
    const int wpb = jrq::kCrcBlock / 64;
    double in_spread = 0, wg_lo = 1e18, wg_hi = 0;
    std::vector<double> simd_mean(4, 0.0), slot_mean(wpb, 0.0);
    for (int b = 0; b < grid; ++b) {
      double lo = 1e18, hi = 0, mean = 0;
      for (int v = 0; v < wpb; ++v) {
        const size_t w = (size_t)b * wpb + v;
        const double e = (tl[4 * w + 1] - s_min) / 100.0;
        lo = std::min(lo, e); hi = std::max(hi, e); mean += e / wpb;
        simd_mean[(tl[4 * w + 2] >> 4) & 3] += e / (grid * (double)wpb / 4);
        slot_mean[v] += e / grid;
      }
      in_spread += (hi - lo) / grid;
      wg_lo = std::min(wg_lo, mean); wg_hi = std::max(wg_hi, mean);
    }
    std::printf("wave end: mean within-WG spread %.1f us; WG mean end %.1f..%.1f us\n", in_spread,
                wg_lo, wg_hi);
    std::printf("mean end by SIMD:");
    for (double m : simd_mean) std::printf(" %.1f", m);
    std::printf("\nmean end by wave slot:");
    for (double m : slot_mean) std::printf(" %.0f", m);
    std::printf("\n");
  }
  // histogram of wave start times (us, 10 bins)
  std::vector<int> hist(10, 0);
  const double span_us = (e_max - s_min) / 100.0;
  for (size_t w = 0; w < nwaves; ++w) {
    const double s = (tl[4 * w] - s_min) / 100.0;
    hist[std::min(9, (int)(s / span_us * 10))]++;
  }
  std::printf("start-time histogram (10 bins over the launch):");
  for (int c : hist) std::printf(" %d", c);
  std::printf("\n");
  return 0;
}
