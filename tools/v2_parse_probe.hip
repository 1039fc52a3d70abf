// v2_parse_probe.hip -- where v2_parse's time goes (tools only; not part of libjrq).
// 64k V2 records as bench.py's v2 leg stores them (header, type, term, index, 16 KiB data,
// checksum field); each variant launched 20 times between one event pair after a warm-up:
//   product   v2_parse (record parse + the fixed-size path's gate)
//   record    the record parse alone (no block summary, no gate)
//   windows   the offsets and the LDS windows alone (no parse)
//   gate      the block summaries and a one-level gate alone (no parse; round 3 first form)
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/v2_parse_probe tools/v2_parse_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../sofa-jraft_amd/csrc/v2_decode.hip"

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

__global__ __launch_bounds__(256) void record_only(JrqV2Args a) {
  __shared__ uint64_t T[256];
  __shared__ __attribute__((aligned(16))) uint8_t win[256 * kWinSlot];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) T[i] = bswap64(a.slice[i]);
  __syncthreads();
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  uint8_t st;
  uint64_t d, dl;
  v2_parse_record(a, r, T, win + threadIdx.x * kWinSlot, st, d, dl);
}

__global__ __launch_bounds__(256) void windows_only(JrqV2Args a) {
  __shared__ __attribute__((aligned(16))) uint8_t win[256 * kWinSlot];
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  const uint64_t b0 = a.off[r];
  const int64_t L = static_cast<int64_t>(a.off[r + 1] - b0);
  WindowReader rd(a.rec + b0, L, win + threadIdx.x * kWinSlot);
  a.status[r] = static_cast<uint8_t>(rd.at(0) ^ rd.at(L - 1));
}

__global__ __launch_bounds__(256) void gate_only(JrqV2Args a) {
  __shared__ uint64_t s_doff[256];
  __shared__ uint64_t s_len0;
  __shared__ uint32_t s_last;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = r < a.n;
  const uint64_t d = live ? a.off[r] + 30 : 0, dl = 16384;
  const uint8_t st = kV2Ok;
  s_doff[threadIdx.x] = d;
  if (threadIdx.x == 0) s_len0 = dl;
  __syncthreads();
  const uint64_t lb = s_len0;
  const bool bad = live && (st != kV2Ok || dl != lb || (threadIdx.x > 0 && d < s_doff[threadIdx.x - 1] + lb));
  const bool any_bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    const uint32_t nb = a.n - blockIdx.x * blockDim.x;
    uint64_t* sm = a.blk + 4ull * blockIdx.x;
    sm[0] = s_doff[0];
    sm[1] = s_doff[(nb < blockDim.x ? nb : blockDim.x) - 1];
    sm[2] = lb;
    sm[3] = any_bad ? 1u : 0u;
    __threadfence();
    const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long*>(a.gate + 4), 1ull);
    s_last = old + 1 == gridDim.x;
    __threadfence();
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) a.gate[4] = 0;
}
}  // namespace probe

static void varint(std::vector<uint8_t>& v, uint64_t x) {
  while (x >= 0x80) {
    v.push_back(static_cast<uint8_t>(x | 0x80));
    x >>= 7;
  }
  v.push_back(static_cast<uint8_t>(x));
}

int main() {
  const uint32_t N = 65536, L = 16384;
  std::vector<uint8_t> rec;
  std::vector<uint64_t> off(N + 1, 0);
  uint64_t z = 12345;
  auto rnd = [&] {
    z += 0x9E3779B97F4A7C15ull;
    uint64_t x = z;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
  };
  rec.reserve(static_cast<size_t>(N) * (L + 48));
  for (uint32_t i = 0; i < N; ++i) {
    const uint8_t h[6] = {0xBB, 0xD2, 0x01, 0, 0, 0};
    rec.insert(rec.end(), h, h + 6);
    rec.push_back(0x08);
    varint(rec, 0);
    rec.push_back(0x10);
    varint(rec, 1 + rnd() % 100000);
    rec.push_back(0x18);
    varint(rec, 1 + i + (rnd() % (1ull << 40)));
    rec.push_back(0x32);
    varint(rec, L);
    for (uint32_t b = 0; b < L; b += 8) {
      const uint64_t w = rnd();
      for (int k = 0; k < 8; ++k) rec.push_back(static_cast<uint8_t>(w >> (8 * k)));
    }
    rec.push_back(0x38);
    varint(rec, rnd());
    off[i + 1] = rec.size();
  }
  JrqV2Args a{};
  uint8_t* drec;
  CK(hipMalloc(&drec, rec.size() + 64));
  CK(hipMemcpy(drec, rec.data(), rec.size(), hipMemcpyHostToDevice));
  uint64_t* doff;
  CK(hipMalloc(&doff, off.size() * 8));
  CK(hipMemcpy(doff, off.data(), off.size() * 8, hipMemcpyHostToDevice));
  auto alloc = [](size_t b) {
    void* p;
    CK(hipMalloc(&p, b));
    CK(hipMemset(p, 0, b));
    return p;
  };
  a.rec = drec;
  a.off = doff;
  a.n = N;
  a.slice = static_cast<uint64_t*>(alloc(8 * 256 * 8));
  a.xinv = static_cast<uint64_t*>(alloc(8 * 256 * 8));
  a.status = static_cast<uint8_t*>(alloc(N));
  a.type = static_cast<uint8_t*>(alloc(N));
  a.index = static_cast<int64_t*>(alloc(N * 8));
  a.term = static_cast<int64_t*>(alloc(N * 8));
  a.stored = static_cast<uint64_t*>(alloc(N * 8));
  a.has_checksum = static_cast<uint8_t*>(alloc(N));
  a.data_off = static_cast<uint64_t*>(alloc(N * 8));
  a.data_len = static_cast<uint64_t*>(alloc(N * 8));
  a.computed = static_cast<uint64_t*>(alloc(N * 8));
  a.corrupt = static_cast<uint8_t*>(alloc(N));
  a.partial = static_cast<uint64_t*>(alloc(N * 8));
  a.off2 = static_cast<uint64_t*>(alloc((N + 2) * 8));
  a.crc2 = static_cast<uint64_t*>(alloc((N + 1) * 8));
  a.lens = static_cast<uint64_t*>(alloc(N * 8));
  a.gate = static_cast<uint64_t*>(alloc(8 * 24));
  a.blk = static_cast<uint64_t*>(alloc((N / 256 + 1) * 32));
  a.lanes = 256 * 512;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid(N / 256), blk(256);
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 200; ++i) launch();
    CK(hipDeviceSynchronize());
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    std::printf("%-10s %.2f us/launch\n", name, best * 1e3 / 20);
  };
  time("product", [&] { hipLaunchKernelGGL(jrq::v2_parse, grid, blk, 0, 0, a); });
  time("record", [&] { hipLaunchKernelGGL(probe::record_only, grid, blk, 0, 0, a); });
  time("windows", [&] { hipLaunchKernelGGL(probe::windows_only, grid, blk, 0, 0, a); });
  time("gate", [&] { hipLaunchKernelGGL(probe::gate_only, grid, blk, 0, 0, a); });
  time("product2", [&] { hipLaunchKernelGGL(jrq::v2_parse, grid, blk, 0, 0, a); });
  uint8_t st[4];
  CK(hipMemcpy(st, a.status, 4, hipMemcpyDeviceToHost));
  std::printf("status of records 0-3 after the last product launch: %u %u %u %u\n", st[0], st[1], st[2], st[3]);
  return 0;
}
