// mem_probe.hip -- standalone HBM access-pattern probe for the CRC64 kernel design
// (tools only; not part of libjrq).  Reads 1 GiB with several lane->address mappings,
// XOR-folds the data (so no load is dead) and reports GB/s per pattern.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/mem_probe tools/mem_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../sofa-jraft_amd/csrc/crc64.hip"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

// Pattern 0: per-lane segments of S bytes (lane k owns [k*S, (k+1)*S)), 128-B blocks,
// 2-deep register ring (the CRC kernel's access pattern).
template <int BV>
__global__ __launch_bounds__(1024) void per_lane(const uint4* __restrict__ p, uint64_t S,
                                                 uint64_t nseg, uint32_t* out) {
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nseg; k += lanes) {
    const uint4* q = p + k * (S / 16);
    const uint64_t nblk = S / (16 * BV);
    uint4 A[BV], B[BV];
    for (int v = 0; v < BV; ++v) A[v] = q[v];
    asm volatile("" ::: "memory");
    for (uint64_t i = 0; i < nblk; i += 2) {
      const uint64_t b1 = i + 1 < nblk ? i + 1 : nblk - 1;
      for (int v = 0; v < BV; ++v) B[v] = q[b1 * BV + v];
      asm volatile("" ::: "memory");
      for (int v = 0; v < BV; ++v) acc ^= A[v].x ^ A[v].y ^ A[v].z ^ A[v].w;
      const uint64_t b2 = i + 2 < nblk ? i + 2 : nblk - 1;
      for (int v = 0; v < BV; ++v) A[v] = q[b2 * BV + v];
      asm volatile("" ::: "memory");
      for (int v = 0; v < BV; ++v) acc ^= B[v].x ^ B[v].y ^ B[v].z ^ B[v].w;
    }
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// Pattern 2: group-coalesced per-lane segments.  Within each 128-B block, G consecutive
// lanes read G*16 contiguous bytes of ONE owner's block per instruction (G owners share 8
// instructions); a register transpose would hand each owner its own block.
template <int G>
__global__ __launch_bounds__(1024) void per_lane_grp(const uint4* __restrict__ p, uint64_t S,
                                                     uint64_t nseg, uint32_t* out) {
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t m = threadIdx.x % G;
  uint32_t acc = 0;
  for (uint64_t k0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x - m; k0 < nseg; k0 += lanes) {
    const uint64_t nblk = S / 128;
    const uint4* q[8];
    for (int k = 0; k < 8; ++k)
      q[k] = p + (k0 + (k % G)) * (S / 16) + (k / G) * G + m;
    uint4 A[8], B[8];
    for (int v = 0; v < 8; ++v) A[v] = q[v][0];
    asm volatile("" ::: "memory");
    for (uint64_t i = 0; i < nblk; i += 2) {
      const uint64_t b1 = i + 1 < nblk ? i + 1 : nblk - 1;
      for (int v = 0; v < 8; ++v) B[v] = q[v][b1 * 8];
      asm volatile("" ::: "memory");
      for (int v = 0; v < 8; ++v) acc ^= A[v].x ^ A[v].y ^ A[v].z ^ A[v].w;
      const uint64_t b2 = i + 2 < nblk ? i + 2 : nblk - 1;
      for (int v = 0; v < 8; ++v) A[v] = q[v][b2 * 8];
      asm volatile("" ::: "memory");
      for (int v = 0; v < 8; ++v) acc ^= B[v].x ^ B[v].y ^ B[v].z ^ B[v].w;
    }
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// Pattern 1: fully coalesced grid-stride float4 stream.
__global__ __launch_bounds__(1024) void coalesced(const uint4* __restrict__ p, uint64_t n16,
                                                  uint32_t* out) {
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * lanes < n16; i += 4 * lanes) {
    const uint4 a = p[i], b = p[i + lanes], c = p[i + 2 * lanes], d = p[i + 3 * lanes];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  for (; i < n16; i += lanes) acc ^= p[i].x;
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const uint64_t total = 1ull << 30;
  uint4* d;
  uint32_t* out;
  CK(hipMalloc(&d, total));
  CK(hipMemset(d, 0x5a, total));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  CK(hipMalloc(&out, (size_t)cus * 8 * 1024 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e9f, sum = 0;
    const int reps = 10;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
      sum += ms;
    }
    std::printf("%-44s best %.4f ms  %.0f GB/s   mean %.4f ms\n", name, best,
                total / (best * 1e-3) / 1e9, sum / reps);
  };
  if (argc > 1) return 0;
  for (int wg_per_cu : {1, 2}) {
    const int grid = cus * wg_per_cu;
    const uint64_t lanes = (uint64_t)grid * 1024;
    char nm[128];
    std::snprintf(nm, sizeof nm, "coalesced x4 (%d WG/CU)", wg_per_cu);
    time(nm, [&] { hipLaunchKernelGGL(coalesced, dim3(grid), dim3(1024), 0, 0, d, total / 16, out); });
    for (uint64_t S : {1024ull, 4096ull}) {
      const uint64_t nseg = total / S;
      std::snprintf(nm, sizeof nm, "grp2 S=%llu (%d WG/CU)", (unsigned long long)S, wg_per_cu);
      time(nm, [&] { hipLaunchKernelGGL(per_lane_grp<2>, dim3(grid), dim3(1024), 0, 0, d, S, nseg, out); });
      std::snprintf(nm, sizeof nm, "grp4 S=%llu (%d WG/CU)", (unsigned long long)S, wg_per_cu);
      time(nm, [&] { hipLaunchKernelGGL(per_lane_grp<4>, dim3(grid), dim3(1024), 0, 0, d, S, nseg, out); });
      std::snprintf(nm, sizeof nm, "grp8 S=%llu (%d WG/CU)", (unsigned long long)S, wg_per_cu);
      time(nm, [&] { hipLaunchKernelGGL(per_lane_grp<8>, dim3(grid), dim3(1024), 0, 0, d, S, nseg, out); });
    }
    if (wg_per_cu == 2) continue;
    for (uint64_t S : {256ull, 1024ull, 4096ull}) {
      const uint64_t nseg = total / S;
      std::snprintf(nm, sizeof nm, "per-lane S=%llu B128 (%d WG/CU, %.1f seg/lane)",
                    (unsigned long long)S, wg_per_cu, (double)nseg / lanes);
      time(nm, [&] {
        hipLaunchKernelGGL(per_lane<8>, dim3(grid), dim3(1024), 0, 0, d, S, nseg, out);
      });
      std::snprintf(nm, sizeof nm, "per-lane S=%llu B64 (%d WG/CU)", (unsigned long long)S,
                    wg_per_cu);
      time(nm, [&] {
        hipLaunchKernelGGL(per_lane<4>, dim3(grid), dim3(1024), 0, 0, d, S, nseg, out);
      });
    }
  }
  return 0;
}
