// inflight_probe.hip -- how much HBM bandwidth the CRC kernel's load pattern gets as a
// function of the bytes each wave keeps in flight and of the VALU work between loads
// (tools only).  Same layout as crc64_rounds_kernel: per-lane segments of S bytes, 64-B
// half-rounds, row group {c, c+16, c+32, c+48} reading 64 contiguous bytes of one owner per
// instruction; a ring of D half-rounds (D-1 in flight while one is consumed); W dependent
// VALU ops per consumed half stand in for the hashing.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/inflight_probe tools/inflight_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int D, int W, int BLOCK, int CH = 1, int SPLIT = 0>
__global__ __launch_bounds__(BLOCK) void ring(const uint8_t* __restrict__ p, uint32_t S,
                                              uint32_t* out) {
  const uint32_t L = threadIdx.x;
  const uint32_t L0 = __builtin_amdgcn_readfirstlane(L & ~63u);
  const uint64_t wave = (uint64_t)blockIdx.x * (BLOCK / 64) + (L0 >> 6);
  const uint8_t* wbase = p + wave * 64ull * S;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(wbase), (short)0, 64u * S, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_none =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(wbase), (short)0, 0u, 0x00020000);
  // SPLIT: rows 0-1 read 32 B of the segment's first half, rows 2-3 32 B of its second half
  const uint32_t row = (L >> 4) & 3u;
  const uint32_t qbase = SPLIT ? (L & 15u) * S + 16u * (row & 1u) + (row >> 1) * (S / 2)
                               : (L & 15u) * S + 16u * row;
  const uint32_t ustep = SPLIT ? 32u : 64u;
  const uint32_t halves = S / 64;
  u32x4 ring[D][4];
  uint32_t acc = L, ch[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) ch[c] = L * (c + 1);
#pragma unroll
  for (int d = 0; d < D - 1; ++d) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      ring[d][q] = __builtin_amdgcn_raw_buffer_load_b128(rs, qbase + q * 16u * S + d * ustep, 0, 0);
  }
  asm volatile("" ::: "memory");
  for (uint32_t h = 0; h < halves; h += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const uint32_t nh = h + d + D - 1;
      const int slot = (d + D - 1) % D;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        ring[slot][q] = __builtin_amdgcn_raw_buffer_load_b128(nh < halves ? rs : rs_none,
                                                              qbase + q * 16u * S + nh * ustep, 0, 0);
      asm volatile("" ::: "memory");
      asm volatile("" : "+v"(ring[d][0]), "+v"(ring[d][1]), "+v"(ring[d][2]), "+v"(ring[d][3]));
#pragma unroll
      for (int q = 0; q < 4; ++q) acc ^= ring[d][q].x ^ ring[d][q].y ^ ring[d][q].z ^ ring[d][q].w;
#pragma unroll
      for (int w = 0; w < W; w += CH) {
#pragma unroll
        for (int c = 0; c < CH; ++c) ch[c] = __builtin_amdgcn_perm(ch[c], acc, 0x01020304u + w);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CH; ++c) acc ^= ch[c];
  out[(uint64_t)blockIdx.x * BLOCK + L] = acc;
}

int main(int argc, char** argv) {
  const uint64_t total = 1ull << 30;
  uint8_t* d;
  uint32_t* out;
  CK(hipMalloc(&d, total));
  CK(hipMemset(d, 0x5a, total));
  CK(hipMalloc(&out, (size_t)256 * 1024 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e9f;
    for (int r = 0; r < 8; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
    }
    std::printf("%-36s best %.4f ms  %.0f GB/s\n", name, best, total / (best * 1e-3) / 1e9);
  };
#define RUNC(D, W, BLOCK, CH)                                                                  \
  {                                                                                            \
    const uint32_t lanes = 256u * BLOCK, S = (uint32_t)(total / lanes) & ~63u;                 \
    time("D=" #D " W=" #W " block=" #BLOCK " chains=" #CH, [&] {                               \
      hipLaunchKernelGGL((ring<D, W, BLOCK, CH>), dim3(256), dim3(BLOCK), 0, 0, d, S, out);    \
    });                                                                                        \
  }
#define RUNS(D, W, CH)                                                                         \
  {                                                                                            \
    const uint32_t lanes = 256u * 1024, S = (uint32_t)(total / lanes) & ~63u;                  \
    time("split32 D=" #D " W=" #W " chains=" #CH, [&] {                                        \
      hipLaunchKernelGGL((ring<D, W, 1024, CH, 1>), dim3(256), dim3(1024), 0, 0, d, S, out);   \
    });                                                                                        \
  }
#define RUN(D, W, BLOCK)                                                                       \
  {                                                                                            \
    const uint32_t lanes = 256u * BLOCK, S = (uint32_t)(total / lanes) & ~63u;                      \
    time("D=" #D " W=" #W " block=" #BLOCK, [&] {                                              \
      hipLaunchKernelGGL((ring<D, W, BLOCK>), dim3(256), dim3(BLOCK), 0, 0, d, S, out);        \
    });                                                                                        \
  }
  if (argc > 1) {  // block-size sweep at W = 0: the rounds kernel's load shape per workgroup size
    RUN(3, 0, 1024) RUN(3, 0, 768) RUN(3, 0, 512) RUN(4, 0, 512) RUN(6, 0, 512) RUN(8, 0, 512)
    RUN(3, 0, 256) RUN(6, 0, 256) RUN(3, 192, 512) RUN(6, 192, 512)
    return 0;
  }
  RUN(3, 0, 1024) RUNS(3, 0, 1) RUNS(4, 0, 1) RUNS(3, 192, 2) RUNS(3, 192, 4) RUNS(3, 160, 2)
  RUN(3, 192, 1024)
  RUNC(3, 192, 1024, 1) RUNC(3, 192, 1024, 2) RUNC(3, 192, 1024, 4) RUNC(3, 192, 1024, 8)
  RUNC(3, 128, 1024, 4) RUNC(3, 96, 1024, 4) RUNC(3, 256, 1024, 4) RUNC(3, 384, 1024, 8)
  RUNC(6, 192, 1024, 4) RUNC(8, 192, 512, 4) RUNC(8, 256, 512, 8)
  return 0;
}
