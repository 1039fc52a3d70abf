// loadpat_probe.hip -- the CRC kernels' load pattern alone (tools only; not part of libjrq).
// 1 GiB, 2048 waves (256 workgroups of 512 threads, as crc64_fixed_kernel runs C5), each lane
// owning one 8 KiB piece and XOR-folding it (no table lookups), through
//   p16x64  16 owners x 64 B per instruction, 4 instructions per 64-B half, two halves of a line
//           issued back to back (the product's shape)
//   p8x128  8 owners x 128 B per instruction (full lines), 8 instructions per 128-B round
//   contig  each instruction 1 KiB contiguous (64 lanes x 16 B; the plain-read floor)
//   p16x64r8  the product's shape with an 8-slot ring (512 B per lane in flight)
//   ldsdma  contig order through LDS: global_load_lds_dwordx4 into an 8-slot ring of 1 KiB per
//           wave (8 KiB in flight per wave, 64 KiB per CU), each slot read back with ds_read_b128;
//           ldsdmant the same with nt loads, ldsdma16[nt] with 16 slots (128 KiB per CU)
//   contignt, p16x64nt, p8x128nt  those shapes with nt loads (aux 2)
// Ring: 256 B per lane in flight in the first three.  Reports the median of 20 launches.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/loadpat_probe tools/loadpat_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      std::exit(1);                                                                          \
    }                                                                                        \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kPS = 8192;     // piece bytes per lane
constexpr uint32_t kBlock = 512;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), static_cast<short>(0),
                                           static_cast<int>(n), 0x00020000);
}

__device__ __forceinline__ uint32_t fold(const u32x4& v) { return v.x ^ v.y ^ v.z ^ v.w; }

// mode 0: p16x64, 1: p8x128, 2: contig
template <int kMode>
__global__ __launch_bounds__(kBlock) void probe(const uint8_t* buf, uint32_t* out) {
  const uint32_t L = threadIdx.x & 63u;
  const uint32_t wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const uint8_t* wb = buf + static_cast<size_t>(wave) * 64u * kPS;  // the wave's 64 pieces
  const __amdgpu_buffer_rsrc_t r = rsrc(wb, 64u * kPS);
  uint32_t acc = 0;
  if constexpr (kMode == 0 || kMode == 9) {
    const uint32_t qb = (L & 15u) * kPS + 16u * (L >> 4);
    u32x4 h[4][4];
    auto ld = [&](u32x4 (&H)[4], uint32_t half) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (kMode == 9) H[j] = __builtin_amdgcn_raw_buffer_load_b128(r, qb + j * 16u * kPS + half * 64u, 0, 2);
        else H[j] = __builtin_amdgcn_raw_buffer_load_b128(r, qb + j * 16u * kPS + half * 64u, 0, 0);
      }
    };
    ld(h[0], 0); ld(h[1], 1); ld(h[2], 2); ld(h[3], 3);
    for (uint32_t t = 0; t < kPS / 256; ++t) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc ^= fold(h[0][j]) ^ fold(h[1][j]);
      ld(h[0], 4 * t + 4); ld(h[1], 4 * t + 5);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc ^= fold(h[2][j]) ^ fold(h[3][j]);
      ld(h[2], 4 * t + 6); ld(h[3], 4 * t + 7);
    }
  } else if constexpr (kMode == 3) {  // p16x64 with an 8-slot ring (512 B per lane in flight)
    const uint32_t qb = (L & 15u) * kPS + 16u * (L >> 4);
    u32x4 h[8][4];
    auto ld = [&](u32x4 (&H)[4], uint32_t half) {
#pragma unroll
      for (int j = 0; j < 4; ++j) H[j] = __builtin_amdgcn_raw_buffer_load_b128(r, qb + j * 16u * kPS + half * 64u, 0, 0);
    };
#pragma unroll
    for (int s = 0; s < 8; ++s) ld(h[s], s);
    for (uint32_t t = 0; t < kPS / 512; ++t) {
#pragma unroll
      for (int s = 0; s < 8; s += 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc ^= fold(h[s][j]) ^ fold(h[s + 1][j]);
        ld(h[s], 8 * t + 8 + s);
        ld(h[s + 1], 8 * t + 9 + s);
      }
    }
  } else if constexpr (kMode == 1 || kMode == 10) {
    const uint32_t qb = (L & 7u) * kPS + 16u * (L >> 3);
    u32x4 h[2][8];
    auto ld = [&](u32x4 (&H)[8], uint32_t round) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (kMode == 10) H[j] = __builtin_amdgcn_raw_buffer_load_b128(r, qb + j * 8u * kPS + round * 128u, 0, 2);
        else H[j] = __builtin_amdgcn_raw_buffer_load_b128(r, qb + j * 8u * kPS + round * 128u, 0, 0);
      }
    };
    ld(h[0], 0); ld(h[1], 1);
    for (uint32_t t = 0; t < kPS / 256; ++t) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc ^= fold(h[0][j]);
      ld(h[0], 2 * t + 2);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc ^= fold(h[1][j]);
      ld(h[1], 2 * t + 3);
    }
  } else if constexpr (kMode >= 4 && kMode <= 7) {  // LDS-DMA ring: 4 = 8 slots, 5 = 8 nt, 6 = 16, 7 = 16 nt
    constexpr int kS = kMode >= 6 ? 16 : 8;
    // (the aux operand must be a literal: a template-dependent constant drops the kernel)
    auto dma = [&](const uint8_t* g, uint32_t* l) {
      if constexpr (kMode & 1) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g), l, 16, 0, 2);
      else __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g), l, 16, 0, 0);
    };
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn_lds[];  // [waves][kS][256]
    uint32_t(*ring)[kS][256] = reinterpret_cast<uint32_t(*)[kS][256]>(dyn_lds);
    const uint32_t w = threadIdx.x >> 6;
    const uint8_t* src = wb + L * 16u;
#pragma unroll
    for (int s = 0; s < kS; ++s)
      dma(src + s * 1024u, &ring[w][s][0]);
    for (uint32_t t = 0; t < 64u * kPS / 1024u; t += kS) {
#pragma unroll
      for (int s = 0; s < kS; ++s) {
        // slot s landed: the kS - 1 loads issued after it may still be out (the compiler does
        // not track LDS-DMA landings; the surplus loads of the last round read the slack)
        if (kS == 16) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        const u32x4 v = *reinterpret_cast<const u32x4*>(&ring[w][s][L * 4u]);
        acc ^= fold(v);
        dma(src + (t + kS + s) * 1024u, &ring[w][s][0]);
      }
    }
  } else {
    // each instruction 1 KiB contiguous: the wave's 512 KiB in order
    u32x4 h[2][8];
    auto ld = [&](u32x4 (&H)[8], uint32_t blk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (kMode == 8) H[j] = __builtin_amdgcn_raw_buffer_load_b128(r, (blk * 8u + j) * 1024u + L * 16u, 0, 2);
        else H[j] = __builtin_amdgcn_raw_buffer_load_b128(r, (blk * 8u + j) * 1024u + L * 16u, 0, 0);
      }
    };
    ld(h[0], 0); ld(h[1], 1);
    for (uint32_t t = 0; t < kPS / 256; ++t) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc ^= fold(h[0][j]);
      ld(h[0], 2 * t + 2);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc ^= fold(h[1][j]);
      ld(h[1], 2 * t + 3);
    }
  }
  out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

int main() {
  const size_t bytes = size_t(1) << 30;
  const uint32_t waves = static_cast<uint32_t>(bytes / (64ull * kPS));  // 2048
  const uint32_t grid = waves / (kBlock / 64);
  uint8_t* buf;
  uint32_t* out;
  // room for the surplus loads past the last piece (up to two rounds)
  CK(hipMalloc(&buf, bytes + (1 << 20)));
  CK(hipMemset(buf, 0x5A, bytes + (1 << 20)));
  CK(hipMalloc(&out, static_cast<size_t>(grid) * kBlock * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    std::vector<float> ms;
    for (int i = 0; i < 25; ++i) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (i >= 5) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("%-10s median %7.1f us  min %7.1f us  %6.2f TB/s\n", name, ms[ms.size() / 2] * 1e3,
                ms[0] * 1e3, bytes / (ms[ms.size() / 2] * 1e-3) / 1e12);
  };
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(probe<6>), hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(probe<7>), hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  for (int rep = 0; rep < 2; ++rep) {
    run("p16x64", [&] { hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(kBlock), 0, 0, buf, out); });
    run("p8x128", [&] { hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(kBlock), 0, 0, buf, out); });
    run("contig", [&] { hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(kBlock), 0, 0, buf, out); });
    run("p16x64r8", [&] { hipLaunchKernelGGL(probe<3>, dim3(grid), dim3(kBlock), 0, 0, buf, out); });
    run("ldsdma", [&] { hipLaunchKernelGGL(probe<4>, dim3(grid), dim3(kBlock), 8 * 8 * 1024, 0, buf, out); });
    run("ldsdmant", [&] { hipLaunchKernelGGL(probe<5>, dim3(grid), dim3(kBlock), 8 * 8 * 1024, 0, buf, out); });
    run("ldsdma16", [&] { hipLaunchKernelGGL(probe<6>, dim3(grid), dim3(kBlock), 16 * 8 * 1024, 0, buf, out); });
    run("ldsdma16nt", [&] { hipLaunchKernelGGL(probe<7>, dim3(grid), dim3(kBlock), 16 * 8 * 1024, 0, buf, out); });
    run("p16x64nt", [&] { hipLaunchKernelGGL(probe<9>, dim3(grid), dim3(kBlock), 0, 0, buf, out); });
    run("p8x128nt", [&] { hipLaunchKernelGGL(probe<10>, dim3(grid), dim3(kBlock), 0, 0, buf, out); });
    run("contignt", [&] { hipLaunchKernelGGL(probe<8>, dim3(grid), dim3(kBlock), 0, 0, buf, out); });
  }
  CK(hipDeviceSynchronize());
  return 0;
}
