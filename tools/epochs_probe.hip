// epochs_probe.hip -- chunk shapes of the K-epoch scan kernel (tools only; not part of libjrq).
// Times quorum_epochs_kernel<3, C, T, W> on the C2 shape (10k groups x 3 peers x 64 epochs,
// epoch-major inputs as bench.py's C2 leg lays them out) for several (C epochs per chunk,
// T groups per chunk, W max waves), and checks every variant's output bytes against the first.
// (Earlier variants of this probe isolated the costs of the product kernel: no status stores
// -0.65 us, no stores at all -1.2 us, no LDS scan -1.2 us, XCD-contiguous tile order -0.4 us,
// status packed 4 per dword +0.3 us; and found its epoch loads issued one epoch per round
// trip behind per-lane conditions: 9.0 -> 8.1 us once every load was unconditional.  Chaining
// the chunks through LDS flags instead of the barrier, so early chunks store sooner: 8.3 us.)
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/epochs_probe tools/epochs_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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


static uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main() {
  const uint32_t G = 10000, P = 3, K = 64;
  std::vector<int64_t> match(static_cast<size_t>(K) * P * G), la(static_cast<size_t>(K) * G);
  std::vector<int64_t> pi(G), lc(G);
  std::vector<uint64_t> conf(G, 0x7ull | (2ull << 32));  // 3 voters, quorum 2
  for (uint32_t g = 0; g < G; ++g) {
    lc[g] = 1000 + static_cast<int64_t>(mix(g) % 100000);
    pi[g] = lc[g] + 1;
  }
  for (uint32_t k = 0; k < K; ++k)
    for (uint32_t g = 0; g < G; ++g) {
      la[static_cast<size_t>(k) * G + g] = lc[g] + 16 * (k + 1);
      for (uint32_t p = 0; p < P; ++p)
        match[(static_cast<size_t>(k) * P + p) * G + g] =
            lc[g] + static_cast<int64_t>(mix((static_cast<uint64_t>(k) * P + p) * G + g) % (16 * (k + 1) + 1));
    }
  int64_t *d_match, *d_la, *d_pi, *d_lc, *d_out;
  uint64_t* d_conf;
  uint8_t* d_st;
  CK(hipMalloc(&d_match, match.size() * 8));
  CK(hipMalloc(&d_la, la.size() * 8));
  CK(hipMalloc(&d_pi, G * 8));
  CK(hipMalloc(&d_lc, G * 8));
  CK(hipMalloc(&d_conf, G * 8));
  CK(hipMalloc(&d_out, static_cast<size_t>(K) * G * 8));
  CK(hipMalloc(&d_st, static_cast<size_t>(K) * G));
  CK(hipMemcpy(d_match, match.data(), match.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_la, la.data(), la.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pi, pi.data(), G * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_lc, lc.data(), G * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_conf, conf.data(), G * 8, hipMemcpyHostToDevice));
  JrqQuorumArgs a{};
  a.match = d_match;
  a.pending_index = d_pi;
  a.last_appended = d_la;
  a.last_committed = d_lc;
  a.conf = d_conf;
  a.num_peers = P;
  a.match_ld = G;
  a.committed = d_out;
  a.status = d_st;
  a.G = G;
  const uint64_t meld = static_cast<uint64_t>(P) * G, leld = G;
  const double bytes = static_cast<double>(K) * G * (8.0 * (P + 1) + 9.0);
  std::vector<int64_t> ref_out, out(static_cast<size_t>(K) * G);
  std::vector<uint8_t> ref_st, st(static_cast<size_t>(K) * G);
  auto run = [&](const char* name, auto kern, uint32_t C, uint32_t T, uint32_t W) {
    const dim3 grid((G + T - 1) / T), blk(64 * jrq_epochs_waves(K, C, T, W));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms;
    CK(hipMemset(d_out, 0, static_cast<size_t>(K) * G * 8));
    for (int i = 0; i < 40; ++i) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(kern, grid, blk, 0, 0, a, K, meld, leld);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (i >= 10) ms.push_back(t);
    }
    // back-to-back launches between one event pair (bench.py's timing)
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kern, grid, blk, 0, 0, a, K, meld, leld);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float tb = 0;
    CK(hipEventElapsedTime(&tb, e0, e1));
    tb /= 20;
    std::sort(ms.begin(), ms.end());
    CK(hipMemcpy(out.data(), d_out, out.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(st.data(), d_st, st.size(), hipMemcpyDeviceToHost));
    if (ref_out.empty()) {
      ref_out = out;
      ref_st = st;
    }
    const bool same = out == ref_out && st == ref_st;
    std::printf("%-16s grid %5u x %4u  median %6.2f us  b2b %6.2f us  %5.0f GB/s  %s\n", name, grid.x,
                blk.x, ms[ms.size() / 2] * 1e3, tb * 1e3, bytes / (tb * 1e-3) / 1e9,
                same ? "same" : "DIFFERENT");
  };
#define V(C, T, W) run("C" #C "_T" #T "_W" #W, jrq::quorum_epochs_kernel<3, C, T, W>, C, T, W)
  V(4, 32, 8);   // the product shape for P = 3
  V(4, 32, 16);
  V(2, 32, 16);
  V(8, 32, 4);
  V(8, 32, 8);
  V(4, 64, 16);
  V(8, 64, 8);
  V(2, 64, 16);
  V(4, 32, 8);
  CK(hipDeviceSynchronize());
  return 0;
}
