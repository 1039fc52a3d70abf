// pair_probe.hip -- launch shapes of the headline quorum epoch (tools only; not part of libjrq).
// C3-shaped stateless epochs (1M groups x 5 peers, joint conf words, no run tables), 6 rotating
// input buffers (486 MB, past the Infinity Cache, as bench.py's headline leg), back-to-back
// launches between one event pair after a warm-up.  Variants (round 2 also measured grid-stride
// shapes and 4 groups per lane: DESIGN.md §4.1):
//   product   quorum_epoch_pair_kernel<5, false>
//   single64  the product's shape and decision (decide_single: P^2 64-bit compares per conf mask)
//   rel32     the same with decide_single_rel (32-bit relative values, u32 sorting network)
//   floor     the same loads and stores, no decision (words XOR-folded): what the loads cost
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/pair_probe tools/pair_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../sofa-jraft_amd/csrc/quorum.hip"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      std::exit(1);                                                                          \
    }                                                                                        \
  } while (0)

namespace probe {
using jrq::i64x2;

// kMode 0: decide_single (the 64-bit P^2 kth); 1: decide_single_rel (32-bit relative, sorting
// network); 2: no decision (every loaded word folded into the outputs by XOR: the load floor)
template <int P, int kMode>
__global__ __launch_bounds__(512) void variant(JrqQuorumArgs a) {
  const uint32_t t = blockIdx.x * 512 + threadIdx.x;
  if (t >= (a.G >> 1)) return;
  const uint32_t g = t << 1;
  const i64x2 pi = jrq::ld2nt(a.pending_index + g);
  const i64x2 lc = jrq::ld2nt(a.last_committed + g);
  const i64x2 la = jrq::ld2nt(a.last_appended + g);
  const i64x2 cw = jrq::ld2nt(reinterpret_cast<const int64_t*>(a.conf) + g);
  i64x2 m[P];
#pragma unroll
  for (int p = 0; p < P; ++p) m[p] = jrq::ld2nt(a.match + static_cast<size_t>(p) * a.match_ld + g);
  int64_t m0[P], m1[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    m0[p] = m[p].x;
    m1[p] = m[p].y;
  }
  int64_t o0, o1;
  uint8_t s0, s1;
  if (kMode == 0) {
    jrq::decide_single<P>(pi.x, la.x, lc.x, static_cast<uint64_t>(cw.x), m0, o0, s0);
    jrq::decide_single<P>(pi.y, la.y, lc.y, static_cast<uint64_t>(cw.y), m1, o1, s1);
  } else if (kMode == 1) {
    jrq::decide_single_rel<P>(pi.x, la.x, lc.x, static_cast<uint64_t>(cw.x), m0, o0, s0);
    jrq::decide_single_rel<P>(pi.y, la.y, lc.y, static_cast<uint64_t>(cw.y), m1, o1, s1);
  } else {
    o0 = pi.x ^ lc.x ^ la.x ^ cw.x;
    o1 = pi.y ^ lc.y ^ la.y ^ cw.y;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      o0 ^= m0[p];
      o1 ^= m1[p];
    }
    s0 = static_cast<uint8_t>(o0);
    s1 = static_cast<uint8_t>(o1);
  }
  i64x2 out;
  out.x = o0;
  out.y = o1;
  __builtin_nontemporal_store(out, reinterpret_cast<i64x2*>(a.committed + g));
  __builtin_nontemporal_store(static_cast<uint16_t>(s0 | (s1 << 8)),
                              reinterpret_cast<uint16_t*>(a.status + g));
}
}  // namespace probe

static uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main() {
  const uint32_t G = 1u << 20, P = 5, NB = 6;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::vector<JrqQuorumArgs> args(NB);
  for (uint32_t b = 0; b < NB; ++b) {
    std::vector<int64_t> h(static_cast<size_t>(G) * (P + 4));
    for (uint32_t g = 0; g < G; ++g) {
      const int64_t pi = 1 + static_cast<int64_t>(mix(g * 7 + b) & 0xFFFFFFFFFFull);
      const int64_t la = pi + 1023;
      for (uint32_t p = 0; p < P; ++p)
        h[static_cast<size_t>(p) * G + g] = pi - 1 + static_cast<int64_t>(mix(g * 31 + p + b * 977) % 1025);
      h[static_cast<size_t>(P) * G + g] = pi;
      h[static_cast<size_t>(P + 1) * G + g] = la;
      h[static_cast<size_t>(P + 2) * G + g] = pi - 1;
      h[static_cast<size_t>(P + 3) * G + g] =
          static_cast<int64_t>(0x1Full | (0x7ull << 16) | (3ull << 32) | (2ull << 40));
    }
    int64_t* d;
    CK(hipMalloc(&d, h.size() * 8));
    CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    JrqQuorumArgs& a = args[b];
    a = JrqQuorumArgs{};
    a.match = d;
    a.pending_index = d + static_cast<size_t>(P) * G;
    a.last_appended = d + static_cast<size_t>(P + 1) * G;
    a.last_committed = d + static_cast<size_t>(P + 2) * G;
    a.conf = reinterpret_cast<const uint64_t*>(d + static_cast<size_t>(P + 3) * G);
    a.num_peers = P;
    a.match_ld = G;
    a.G = G;
  }
  int64_t* committed;
  uint8_t* status;
  CK(hipMalloc(&committed, static_cast<size_t>(G) * 8));
  CK(hipMalloc(&status, G));
  for (auto& a : args) {
    a.committed = committed;
    a.status = status;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 3000; ++i) launch(args[i % NB]);  // ~50 ms warm-up
    CK(hipDeviceSynchronize());
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 60; ++i) launch(args[i % NB]);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    const double us = best * 1e3 / 60;
    std::printf("%-10s %.2f us/epoch  %.0f GB/s (81 B/group)\n", name, us, 81.0 * G / (us * 1e3));
  };
  const uint32_t pairs = G / 2;
  time("product", [&](const JrqQuorumArgs& a) {
    hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<5, false>), dim3((pairs + 511) / 512), dim3(512), 0, 0, a);
  });
  time("single64", [&](const JrqQuorumArgs& a) {
    hipLaunchKernelGGL((probe::variant<5, 0>), dim3((pairs + 511) / 512), dim3(512), 0, 0, a);
  });
  time("rel32", [&](const JrqQuorumArgs& a) {
    hipLaunchKernelGGL((probe::variant<5, 1>), dim3((pairs + 511) / 512), dim3(512), 0, 0, a);
  });
  time("floor", [&](const JrqQuorumArgs& a) {
    hipLaunchKernelGGL((probe::variant<5, 2>), dim3((pairs + 511) / 512), dim3(512), 0, 0, a);
  });
  time("product2", [&](const JrqQuorumArgs& a) {
    hipLaunchKernelGGL((jrq::quorum_epoch_pair_kernel<5, false>), dim3((pairs + 511) / 512), dim3(512), 0, 0, a);
  });
  return 0;
}
