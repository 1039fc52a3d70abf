// The resident table epoch's memory pattern without its decision: 1M groups in
// 256-group tiles of F = P + 4 fields (match[P], pendingIndex, lastAppended, lastCommitted,
// conf), every field of a tile 256 consecutive words.  Per group: read all F words; write one
// 8-B result either to a separate row (the headline pair kernel's committed[]) or in place into
// the tile's lastCommitted field (the table); optionally an 8-B list entry per group into the
// wave's slice.  Two lane shapes: one pair of groups per lane (512-thread workgroups, a wave =
// half a tile) and two pairs per lane (256-thread workgroups, a wave = a whole tile).
// Question it answers: is the table epoch's gap to the pair kernel its lane shape or its
// in-place stores.   hipcc -O3 --offload-arch=gfx950 table_shape_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef long long i64x2 __attribute__((ext_vector_type(2)));
constexpr int P = 5, F = P + 4, LC = P + 2;

template <bool kInPlace, bool kList>
__global__ __launch_bounds__(512) void one_pair(long long* __restrict__ tiles, long long* __restrict__ row,
                                               long long* __restrict__ list, unsigned G) {
  const unsigned i = blockIdx.x * 512 + threadIdx.x;  // pair index
  const unsigned g = 2 * i;
  if (g >= G) return;
  long long* tile = tiles + static_cast<size_t>(g >> 8) * F * 256;
  const unsigned o = g & 255u;
  i64x2 acc = {0, 0};
#pragma unroll
  for (int f = 0; f < F; ++f) acc ^= __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(tile + f * 256 + o));
  if (kInPlace)
    __builtin_nontemporal_store(acc, reinterpret_cast<i64x2*>(tile + LC * 256 + o));
  else
    *reinterpret_cast<i64x2*>(row + g) = acc;
  if (kList) {
    i64x2 e = {static_cast<long long>(g), static_cast<long long>(g + 1)};
    *reinterpret_cast<i64x2*>(list + g) = e;
  }
}

template <bool kInPlace, bool kList>
__global__ __launch_bounds__(256) void two_pairs(long long* __restrict__ tiles, long long* __restrict__ row,
                                                long long* __restrict__ list, unsigned G) {
  const unsigned w = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const unsigned gA = w * 256 + 2 * lane;
  if (gA >= G) return;
  long long* tile = tiles + static_cast<size_t>(w) * F * 256;
  i64x2 acc[2] = {{0, 0}, {0, 0}};
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int f = 0; f < F; ++f)
      acc[h] ^= __builtin_nontemporal_load(reinterpret_cast<const i64x2*>(tile + f * 256 + 2 * lane + 128 * h));
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const unsigned o = 2 * lane + 128 * h;
    if (kInPlace)
      __builtin_nontemporal_store(acc[h], reinterpret_cast<i64x2*>(tile + LC * 256 + o));
    else
      *reinterpret_cast<i64x2*>(row + gA + 128 * h) = acc[h];
    if (kList) {
      i64x2 e = {static_cast<long long>(gA + 128 * h), static_cast<long long>(gA + 128 * h + 1)};
      *reinterpret_cast<i64x2*>(list + w * 256 + o) = e;
    }
  }
}

int main() {
  const unsigned G = 1u << 20;
  constexpr int NB = 6;  // rotating tables: 6 x 72 MB, more than the 256 MB Infinity Cache
  const size_t words = static_cast<size_t>(G) * F;
  long long *d, *row, *list;
  hipMalloc(&d, words * 8 * NB);
  hipMalloc(&row, G * 8ull);
  hipMalloc(&list, G * 8ull);
  hipMemset(d, 1, words * 8 * NB);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto launch = [&](int mode, long long* t) {
    const dim3 g1((G / 2 + 511) / 512), g2((G / 256 * 64 + 255) / 256);
    switch (mode) {
      case 0: one_pair<false, false><<<g1, 512>>>(t, row, list, G); break;
      case 1: one_pair<true, false><<<g1, 512>>>(t, row, list, G); break;
      case 2: one_pair<true, true><<<g1, 512>>>(t, row, list, G); break;
      case 3: two_pairs<false, false><<<g2, 256>>>(t, row, list, G); break;
      case 4: two_pairs<true, false><<<g2, 256>>>(t, row, list, G); break;
      case 5: two_pairs<true, true><<<g2, 256>>>(t, row, list, G); break;
    }
  };
  const char* names[] = {"one_pair_row", "one_pair_inplace", "one_pair_inplace_list",
                         "two_pairs_row", "two_pairs_inplace", "two_pairs_inplace_list"};
  for (int rep = 0; rep < 3; ++rep)
    for (int mode = 0; mode < 6; ++mode) {
      const int K = 240;
      for (int k = 0; k < 60; ++k) launch(mode, d + (k % NB) * words);
      hipEventRecord(a);
      for (int k = 0; k < K; ++k) launch(mode, d + (k % NB) * words);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double us = ms * 1e3 / K;
      const double bytes = double(G) * (F * 8 + 8 + ((mode % 3) == 2 ? 8 : 0));
      printf("%-24s %.2f us per launch, %.0f GB/s\n", names[mode], us, bytes / us / 1e3);
    }
  return 0;
}
