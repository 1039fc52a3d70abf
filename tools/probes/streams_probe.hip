// Read bandwidth of S parallel SoA streams against one AoS stream of the same bytes, with the
// quorum pair kernel's load shape (16-B nt loads, one pair of 8-B words per lane per stream).
// Question it answers: how much of the headline kernel's gap to the copy ceiling is the number
// of streams a wave reads at once.  hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef long long i64x2 __attribute__((ext_vector_type(2)));

template <int S>
__global__ __launch_bounds__(256) void soa(const long long* __restrict__ base, size_t ld, uint32_t pairs,
                                          long long* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= pairs) return;
  i64x2 acc = {0, 0};
#pragma unroll
  for (int s = 0; s < S; ++s)
    acc ^= __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(base + s * ld) + i);
  out[i] = acc.x ^ acc.y;
}

// SoA, each wave walking R consecutive 64-pair chunks of every stream (R KiB per stream)
template <int S, int R>
__global__ __launch_bounds__(256) void soa_long(const long long* __restrict__ base, size_t ld, uint32_t pairs,
                                                long long* __restrict__ out) {
  const uint32_t w = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (static_cast<size_t>(w) * 64 * R >= pairs) return;
  i64x2 acc = {0, 0};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = (w * R + r) * 64 + lane;
#pragma unroll
    for (int s = 0; s < S; ++s)
      acc ^= __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(base + s * ld) + i);
  }
  out[w * 64 + lane] = acc.x ^ acc.y;
}

template <int S>
__global__ __launch_bounds__(256) void aos(const long long* __restrict__ base, uint32_t pairs,
                                          long long* __restrict__ out) {
  // each wave reads its 64 pairs' records (S x 16 B each) as one contiguous block, lane-strided
  const uint32_t w = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const i64x2* blk = reinterpret_cast<const i64x2*>(base) + static_cast<size_t>(w) * 64 * S;
  if (static_cast<size_t>(w) * 64 >= pairs) return;
  i64x2 acc = {0, 0};
#pragma unroll
  for (int s = 0; s < S; ++s) acc ^= __builtin_nontemporal_load(blk + s * 64 + lane);
  out[w * 64 + lane] = acc.x ^ acc.y;
}

int main() {
  constexpr int S = 10;            // 5 match + pi + la + lc + conf + (committed-sized) pad
  const uint32_t G = 1u << 20, pairs = G / 2;
  const size_t ld = G;             // words per stream
  long long *d, *o;
  hipMalloc(&d, S * ld * 8 * 4);   // 4 rotating inputs (no cache reuse between launches)
  hipMalloc(&o, pairs * 8);
  hipMemset(d, 1, S * ld * 8 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const dim3 grid((pairs + 255) / 256);
  auto launch = [&](int mode, const long long* in) {
    if (mode == 0) soa<S><<<grid, 256>>>(in, ld, pairs, o);
    else if (mode == 1) aos<S><<<grid, 256>>>(in, pairs, o);
    else if (mode == 2) soa_long<S, 4><<<dim3((pairs / 4 + 255) / 256), 256>>>(in, ld, pairs, o);
    else soa_long<S, 16><<<dim3((pairs / 16 + 255) / 256), 256>>>(in, ld, pairs, o);
  };
  const char* names[] = {"soa", "aos", "soa_long4", "soa_long16"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      const int K = 200;
      for (int k = 0; k < 20; ++k) {
        const long long* in = d + (k & 3) * S * ld;
        launch(mode, in);
      }
      hipEventRecord(a);
      for (int k = 0; k < K; ++k) {
        const long long* in = d + (k & 3) * S * ld;
        launch(mode, in);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double us = ms * 1e3 / K, bytes = double(S) * G * 8 + pairs * 8.0;
      printf("%s S=%d: %.2f us per launch, %.0f GB/s\n", names[mode], S, us, bytes / us / 1e3);
    }
  }
  return 0;
}
