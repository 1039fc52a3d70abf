// crc_v3_probe.hip -- design probe for the next CRC64 kernel (tools only; not part of libjrq).
//
// Question: how much of the gap between the table hash alone (~7.6-8.8 TB/s on 1 GiB) and the
// HBM stream (~6 TB/s coalesced) does the production kernel (~3.3 TB/s) lose to (a) the
// per-lane scattered access pattern and (b) too little prefetch (one 128-B block in flight,
// drained by a vmcnt(0) at the loop head)?
//
// Every lane owns one S-byte segment and outputs its CRC (checked against a host table walk).
// A "round" is 64 B per lane = 4 x 16-B loads, issued DEPTH-1 rounds ahead into a register
// ring (buffer loads: per-lane voffset constant, the round moves the scalar soffset, so no
// address VGPR is rewritten inside the loop).  G selects who loads what:
//   G=1  lane loads its own 64 B (scattered: 64 lines per wave instruction)
//   G=2  lane pairs load 32 contiguous bytes of one owner per instruction; one DPP stage
//        (quad_perm xor 1 + select) hands each lane its own pieces
//   G=4  quads load 64 contiguous bytes of one owner per instruction; two DPP stages
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/crc_v3_probe tools/crc_v3_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
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

// optional per-wave timeline {start, end, HW_ID, XCC_ID} (set with hipMemcpyToSymbol)
__device__ uint64_t* g_tl = nullptr;
using jrq::u32x4;

__device__ __forceinline__ uint32_t dpp_xor1(uint32_t v) {
  return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t v) {
  return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
}

// One butterfly stage on lane bit b for the register pair (lo: reg bit b = 0, hi: bit b = 1):
// an element stays when its lane bit equals its register bit, else it swaps with the
// partner lane's other register.
template <int B>
__device__ __forceinline__ void stage(u32x4& lo, u32x4& hi, bool bit) {
  u32x4 nlo, nhi;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint32_t plo = B == 0 ? dpp_xor1(lo[c]) : dpp_xor2(lo[c]);
    const uint32_t phi = B == 0 ? dpp_xor1(hi[c]) : dpp_xor2(hi[c]);
    nhi[c] = bit ? hi[c] : plo;
    nlo[c] = bit ? phi : lo[c];
  }
  lo = nlo;
  hi = nhi;
}

// Tab4 image, conflict-free order: lanes with bit 4 set swap the table order of each
// instruction pair (R3<->R2, R1<->R0), so in every ds_read_b64 the lanes l and l+16 that
// share a 16-B slot read its two different halves (bank pairs 2(l&15) and 2(l&15)+1).
struct Tab4x {
  uint32_t lc[4], sel[4], lc0;
  __device__ explicit Tab4x(uint32_t lane) {
    const uint32_t sw = (lane >> 4) & 1u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t j = i ^ sw;  // data byte of instruction i
      const uint32_t k = 3 - j;   // table indexed by byte j
      lc[i] = ((lane & 15u) << 4) | ((k & 1u) << 3) | ((k >> 1) << 16);
      sel[i] = 0x0C060004u | (j << 8);
    }
    lc0 = (lane & 15u) << 4;
  }
  __device__ static uint32_t src_index(uint32_t w) { return jrq::Tab4::src_index(w); }
  __device__ __forceinline__ void step4(jrq::RState& r, const char* lds) const {
    const uint2 t0 = jrq::lds_u2(lds, __builtin_amdgcn_perm(lc[0], r.lo, sel[0]));
    const uint2 t1 = jrq::lds_u2(lds, __builtin_amdgcn_perm(lc[1], r.lo, sel[1]));
    const uint2 t2 = jrq::lds_u2(lds, __builtin_amdgcn_perm(lc[2], r.lo, sel[2]));
    const uint2 t3 = jrq::lds_u2(lds, __builtin_amdgcn_perm(lc[3], r.lo, sel[3]));
    r.lo = jrq::xor3(jrq::xor3(r.hi, t0.x, t1.x), t2.x, t3.x);
    r.hi = jrq::xor3(t0.y, t1.y, t2.y) ^ t3.y;
  }
  __device__ __forceinline__ void step8(jrq::RState& r, uint32_t dlo, uint32_t dhi, const char* lds) const {
    r.lo ^= dlo;
    r.hi ^= dhi;
    step4(r, lds);
    step4(r, lds);
  }
};

template <class Tab>
__device__ __forceinline__ void hash16(const Tab& tb, jrq::RState& r, const u32x4& v, const char* lds) {
  tb.step8(r, v[0], v[1], lds);
  tb.step8(r, v[2], v[3], lds);
}

template <class Tab, int G, int DEPTH, int NL = 4, int AUX = 0, bool MEMONLY = false>
__global__ __launch_bounds__(1024) void v3(const uint8_t* __restrict__ p, const uint64_t* __restrict__ slice,
                                          uint32_t S, uint64_t* __restrict__ out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  __shared__ __attribute__((aligned(16))) uint64_t lds_tab[jrq::kCrcLdsBytes / 8];
  for (uint32_t w = threadIdx.x; w < jrq::kCrcLdsBytes / 8; w += blockDim.x)
    lds_tab[w] = slice[Tab::src_index(w)];
  __syncthreads();
  const char* lds = reinterpret_cast<const char*>(lds_tab);
  const Tab tb(threadIdx.x & 63u);
  const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t m = gl & (G - 1);
  const uint32_t grp = gl - m;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, 0x7fffffff, 0x00020000);
  constexpr uint32_t kRound = 16u * NL;  // bytes per lane per round
  // voff[k]: byte offset (within the round) read by this lane in load k
  uint32_t voff[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const uint32_t q = k & 3, h = k >> 2;  // 4-load quartet h covers 64 B of every owner
    if (G == 1) voff[k] = gl * S + 16u * k;
    if (G == 2) voff[k] = (grp + (q & 1)) * S + 64u * h + 16u * ((q >> 1) * 2 + m);
    if (G == 4) voff[k] = (grp + q) * S + 64u * h + 16u * m;
  }
  const uint32_t rounds = S / kRound;
  u32x4 ring[DEPTH][NL];
#define LOADR(slot, rnd)                                                                    \
  do {                                                                                      \
    const uint32_t rr = (rnd) < rounds ? (rnd) : rounds - 1;                                \
    _Pragma("unroll") for (int k = 0; k < NL; ++k) ring[slot][k] =                          \
        __builtin_amdgcn_raw_buffer_load_b128(rs, voff[k], rr * kRound, AUX);               \
    asm volatile("" ::: "memory");                                                          \
  } while (0)
#pragma unroll
  for (int s = 0; s < DEPTH - 1; ++s) LOADR(s, (uint32_t)s);
  jrq::RState r{0u, 0u};
  for (uint32_t r0 = 0; r0 < rounds; r0 += DEPTH) {
#pragma unroll
    for (int s = 0; s < DEPTH; ++s) {
      LOADR((s + DEPTH - 1) % DEPTH, r0 + s + DEPTH - 1);
#pragma unroll
      for (int h = 0; h < NL / 4; ++h) {
        u32x4 a0 = ring[s][4 * h], a1 = ring[s][4 * h + 1], a2 = ring[s][4 * h + 2], a3 = ring[s][4 * h + 3];
        // pin the slot's first use below this round's loads: without it the scheduler hoists
        // the (memory-free) DPP transposes of every slot to the loop head and waits vmcnt(0)
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        if (G == 2) {  // regs (2h + o): owner o piece 2h + m  ->  own piece 2h + o
          stage<0>(a0, a1, m & 1);
          stage<0>(a2, a3, m & 1);
        }
        if (G == 4) {  // reg o: owner o piece m  ->  reg j: own piece j
          stage<0>(a0, a1, m & 1);
          stage<0>(a2, a3, m & 1);
          stage<1>(a0, a2, (m >> 1) & 1);
          stage<1>(a1, a3, (m >> 1) & 1);
        }
        if (MEMONLY) {
          r.lo ^= a0[0] ^ a1[1] ^ a2[2] ^ a3[3];
          r.hi ^= a0[1] ^ a1[2] ^ a2[3] ^ a3[0];
        } else {
          hash16(tb, r, a0, lds);
          hash16(tb, r, a1, lds);
          hash16(tb, r, a2, lds);
          hash16(tb, r, a3, lds);
        }
      }
    }
  }
#undef LOADR
  out[gl] = jrq::crc_value(r);
  if (g_tl && (threadIdx.x & 63u) == 0) {
    uint64_t* t = g_tl + 4 * (gl >> 6);
    t[0] = t0;
    t[1] = __builtin_amdgcn_s_memrealtime();
    t[2] = __builtin_amdgcn_s_getreg((23 << 11) | (0 << 6) | 4);
    t[3] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
  }
}

// Compute-only ceiling: same LDS image and steps, data synthesised in registers.
template <class Tab>
__global__ __launch_bounds__(1024) void hash_only(const uint64_t* __restrict__ slice, uint32_t S,
                                                 uint64_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint64_t lds_tab[jrq::kCrcLdsBytes / 8];
  for (uint32_t w = threadIdx.x; w < jrq::kCrcLdsBytes / 8; w += blockDim.x)
    lds_tab[w] = slice[Tab::src_index(w)];
  __syncthreads();
  const char* lds = reinterpret_cast<const char*>(lds_tab);
  const Tab tb(threadIdx.x & 63u);
  jrq::RState r{threadIdx.x, blockIdx.x};
  uint32_t x = threadIdx.x * 0x9E3779B9u;
  for (uint32_t i = 0; i < S / 16; ++i) {
    x += 0x6D2B79F5u;
    u32x4 v;
    v[0] = x; v[1] = x ^ 0x55u; v[2] = x + 7u; v[3] = x ^ 0xAAu;
    hash16(tb, r, v, lds);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = jrq::crc_value(r);
}

static uint64_t g_t[256];
static uint64_t host_crc(const uint8_t* q, size_t n) {
  uint64_t c = 0;
  for (size_t i = 0; i < n; ++i) c = g_t[((c >> 56) ^ q[i]) & 0xFF] ^ (c << 8);
  return c;
}

int main() {
  const uint64_t total = 1ull << 30;
  // tables: T0..T3 (T_j = T_{j-1} advanced by a zero byte), slice = bswap(T_j)
  uint64_t t[4][256];
  for (int i = 0; i < 256; ++i) {
    uint64_t c = static_cast<uint64_t>(i) << 56;
    for (int k = 0; k < 8; ++k) c = (c & 0x8000000000000000ULL) ? (c << 1) ^ jrq::kCrcPoly : (c << 1);
    t[0][i] = g_t[i] = c;
  }
  for (int j = 1; j < 4; ++j)
    for (int i = 0; i < 256; ++i) t[j][i] = t[0][t[j - 1][i] >> 56] ^ (t[j - 1][i] << 8);
  std::vector<uint64_t> slice(4 * 256);
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 256; ++i) slice[j * 256 + i] = __builtin_bswap64(t[j][i]);
  std::vector<uint8_t> h(total);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < total / 8; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    std::memcpy(&h[i * 8], &x, 8);
  }
  uint8_t* d;
  uint64_t *ds, *out;
  CK(hipMalloc(&d, total));
  CK(hipMemcpy(d, h.data(), total, hipMemcpyHostToDevice));
  CK(hipMalloc(&ds, slice.size() * 8));
  CK(hipMemcpy(ds, slice.data(), slice.size() * 8, hipMemcpyHostToDevice));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const uint32_t lanes = cus * 1024;
  const uint32_t S = static_cast<uint32_t>(total / lanes);  // 4 KiB on 256 CUs
  CK(hipMalloc(&out, (size_t)lanes * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<uint64_t> o(lanes);
  auto run = [&](const char* name, auto kern) {
    auto launch = [&] { hipLaunchKernelGGL(kern, dim3(cus), dim3(1024), 0, 0, d, ds, S, out); };
    launch();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o.data(), out, (size_t)lanes * 8, hipMemcpyDeviceToHost));
    int bad = 0;
    for (uint32_t k = 0; k < lanes; k += 997)
      bad += o[k] != host_crc(h.data() + (size_t)k * S, S);
    float best = 1e9f, sum = 0;
    const int reps = 10;
    for (int rep = 0; rep < reps; ++rep) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
      sum += ms;
    }
    std::printf("%-28s best %.4f ms %5.0f GB/s  mean %.4f ms  %s\n", name, best,
                (S * (double)lanes) / (best * 1e-3) / 1e9, sum / reps, bad ? "MISMATCH" : "ok");
    std::fflush(stdout);
  };
  auto hrun = [&](const char* name, auto kern) {
    hipLaunchKernelGGL(kern, dim3(cus), dim3(1024), 0, 0, ds, S, out);
    CK(hipDeviceSynchronize());
    float best = 1e9f;
    for (int rep = 0; rep < 10; ++rep) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(kern, dim3(cus), dim3(1024), 0, 0, ds, S, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
    }
    std::printf("%-28s best %.4f ms %5.0f GB/s equiv\n", name, best, (S * (double)lanes) / (best * 1e-3) / 1e9);
  };
  hrun("hash_only Tab4", hash_only<jrq::Tab4>);
  run("G4 D2 R128 Tab4", v3<jrq::Tab4, 4, 2, 8>);
  run("G4 D4 Tab4", v3<jrq::Tab4, 4, 4>);
  // timeline of the R128 variant
  uint64_t* d_tl;
  const size_t nwaves = lanes / 64;
  CK(hipMalloc(&d_tl, nwaves * 32));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tl), &d_tl, sizeof(d_tl)));
  hipLaunchKernelGGL((v3<jrq::Tab4, 4, 2, 8>), dim3(cus), dim3(1024), 0, 0, d, ds, S, out);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> tl(nwaves * 4);
  CK(hipMemcpy(tl.data(), d_tl, tl.size() * 8, hipMemcpyDeviceToHost));
  uint64_t s_min = ~0ull, e_max = 0;
  for (size_t w = 0; w < nwaves; ++w) {
    s_min = std::min(s_min, tl[4 * w]);
    e_max = std::max(e_max, tl[4 * w + 1]);
  }
  std::printf("timeline G4 D2 R128: first start -> last end %.1f us\n", (e_max - s_min) / 100.0);
  for (int x = 0; x < 8; ++x) {
    double e_lo = 1e18, e_hi = 0, dur = 0;
    int cnt = 0;
    for (size_t w = 0; w < nwaves; ++w) {
      if ((int)(tl[4 * w + 3] & 0xF) != x) continue;
      const double st = (tl[4 * w] - s_min) / 100.0, en = (tl[4 * w + 1] - s_min) / 100.0;
      e_lo = std::min(e_lo, en);
      e_hi = std::max(e_hi, en);
      dur += en - st;
      ++cnt;
    }
    if (cnt) std::printf("xcc %d: waves %d end %.1f..%.1f mean dur %.1f us\n", x, cnt, e_lo, e_hi, dur / cnt);
  }
  return 0;
}
