// unal_probe.hip -- read rate of 16-B buffer loads at a byte misalignment (tools only).
// Each wave streams a contiguous 1 MiB slice of a 1 GiB buffer with raw_buffer_load_b128 at
// base + m (m = 0, 1, 4, 8, 13), XOR-folds what it read and stores one word per lane; prints
// GB/s per m.  Question: does the V2 fixed-size data CRC path (record data at any byte
// alignment) pay for unaligned loads?
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/unal_probe tools/unal_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      std::exit(1);                                                                          \
    }                                                                                        \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void rd(const uint8_t* buf, uint32_t m, uint32_t slice,
                                          uint32_t* out) {
  const uint32_t w = blockIdx.x * 8 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  const uint8_t* base = buf + static_cast<size_t>(w) * slice + m;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(base), static_cast<short>(0), static_cast<int>(slice), 0x00020000);
  u32x4 acc = {0, 0, 0, 0};
  for (uint32_t o = lane * 16u; o < slice; o += 4096u) {
    u32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 1024u * i, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= v[i];
  }
  out[w * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

int main() {
  const size_t bytes = 1ull << 30;
  const uint32_t slice = 1u << 20, waves = static_cast<uint32_t>(bytes / slice) - 1;
  uint8_t* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 0x3C, bytes));
  CK(hipMalloc(&out, static_cast<size_t>(waves + 8) * 64 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid(waves / 8);
  for (int pass = 0; pass < 2; ++pass)
    for (uint32_t m : {0u, 1u, 4u, 8u, 13u, 0u}) {
      for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(rd, grid, dim3(512), 0, 0, buf, m, slice, out);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(rd, grid, dim3(512), 0, 0, buf, m, slice, out);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (pass) std::printf("m=%2u  %.0f GB/s\n", m, static_cast<double>(grid.x) * 8 * slice * 10 / (ms * 1e6));
    }
  return 0;
}
