// append_entries.hip -- follower-side batched verify of AppendEntries requests.
//
// Reference: NodeImpl.handleAppendEntriesRequest (jraft-core/.../core/NodeImpl.java:1766-1792)
// walks the request's EntryMeta list with index = prevLogIndex + 1 + i, slices each entry's
// bytes out of the request's concatenated `data` by data_len (logEntryFromMeta :1809-1823:
// ENTRY_TYPE_UNKNOWN entries are skipped and consume no bytes), and answers EINVAL at the
// first entry whose stored checksum differs from LogEntry.checksum() (:1777-1789).
// Wire format: raft.proto EntryMeta {term, type, data_len, checksum, ...},
// rpc.proto AppendEntriesRequest {prev_log_index, entries, data}.
//
// Batched over R requests / N entries:
//   1. ae_block_sums  + ae_scan_sums + ae_meta: exclusive scan of the effective data_len
//      (0 for UNKNOWN) -> payload offsets[N+1]; per-entry index from the request's
//      prevLogIndex; has_eff = hasChecksum && type != UNKNOWN.
//   2. the fused LogEntry checksum + verify kernel (crc64.hip).
//   3. ae_first_corrupt: per request, the position of the first corrupt entry (or -1),
//      i.e. the entry the reference reports in its EINVAL response.
#include "jrq_device.h"

namespace jrq {

constexpr int kScanBlock = 1024;
constexpr int kScanPerThread = 4;
constexpr int kScanTile = kScanBlock * kScanPerThread;  // entries per tile

__device__ __forceinline__ uint64_t eff_len(const JrqAeArgs& a, uint32_t e) {
  return a.type[e] == 0 ? 0ull : static_cast<uint64_t>(a.data_len[e]);
}

// Phase 1: per-tile sums of effective lengths.
__global__ __launch_bounds__(kScanBlock) void ae_block_sums(JrqAeArgs a) {
  __shared__ uint64_t w[kScanBlock / 64];
  const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanPerThread;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPerThread; ++k)
    if (base + k < a.n) s += eff_len(a, base + k);
  uint64_t total;
  (void)block_exclusive_scan(s, w, &total);
  if (threadIdx.x == 0) a.tile_sums[blockIdx.x] = total;
}

// Phase 2: one block scans the tile sums in place (exclusive), looping over chunks.
__global__ __launch_bounds__(kScanBlock) void ae_scan_sums(JrqAeArgs a, uint32_t ntiles) {
  __shared__ uint64_t w[kScanBlock / 64];
  uint64_t carry = 0;
  for (uint32_t c = 0; c < ntiles; c += kScanBlock) {
    const uint32_t i = c + threadIdx.x;
    const uint64_t v = i < ntiles ? a.tile_sums[i] : 0;
    uint64_t total;
    const uint64_t ex = block_exclusive_scan(v, w, &total);
    if (i < ntiles) a.tile_sums[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) a.offsets[a.n] = carry;  // payload bytes consumed by the batch
}

// Phase 3: offsets, indexes, effective has-checksum flags.
__global__ __launch_bounds__(kScanBlock) void ae_meta(JrqAeArgs a) {
  __shared__ uint64_t w[kScanBlock / 64];
  const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanPerThread;
  uint64_t len[kScanPerThread];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPerThread; ++k) {
    len[k] = base + k < a.n ? eff_len(a, base + k) : 0;
    s += len[k];
  }
  uint64_t total;
  uint64_t off = a.tile_sums[blockIdx.x] + block_exclusive_scan(s, w, &total);
#pragma unroll
  for (int k = 0; k < kScanPerThread; ++k) {
    const uint32_t e = base + k;
    if (e >= a.n) break;
    a.offsets[e] = off;
    off += len[k];
    // request of entry e: last r with req_off[r] <= e
    uint32_t lo = 0, hi = a.r;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (a.req_off[mid] <= e) lo = mid;
      else hi = mid;
    }
    a.index[e] = a.prev_log_index[lo] + 1 + static_cast<int64_t>(e - a.req_off[lo]);
    const bool has = a.has_checksum == nullptr || a.has_checksum[e];
    a.has_eff[e] = static_cast<uint8_t>(has && a.type[e] != 0);
  }
}

// Phase 4: one wave per request finds its first corrupt entry.
__global__ __launch_bounds__(256) void ae_first_corrupt(JrqAeArgs a) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (wave >= a.r) return;
  const uint32_t b = a.req_off[wave], e = a.req_off[wave + 1];
  int32_t first = -1;
  for (uint32_t i = b; i < e; i += 64) {
    const bool bad = (i + lane < e) && a.corrupt[i + lane] != 0;
    const uint64_t m = __ballot(bad);
    if (m) {
      first = static_cast<int32_t>(i - b) + __builtin_ctzll(m);
      break;
    }
  }
  if (lane == 0) a.first_corrupt[wave] = first;
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_ae_meta(
    const JrqAeArgs* a, hipStream_t stream) {
  const uint32_t ntiles = (a->n + jrq::kScanTile - 1) / jrq::kScanTile;
  hipLaunchKernelGGL(jrq::ae_block_sums, dim3(ntiles), dim3(jrq::kScanBlock), 0, stream, *a);
  hipLaunchKernelGGL(jrq::ae_scan_sums, dim3(1), dim3(jrq::kScanBlock), 0, stream, *a, ntiles);
  hipLaunchKernelGGL(jrq::ae_meta, dim3(ntiles), dim3(jrq::kScanBlock), 0, stream, *a);
  return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_ae_first_corrupt(
    const JrqAeArgs* a, hipStream_t stream) {
  const uint32_t blocks = (a->r + 3) / 4;  // 4 waves (requests) per 256-thread block
  hipLaunchKernelGGL(jrq::ae_first_corrupt, dim3(blocks ? blocks : 1), dim3(256), 0, stream, *a);
  return hipGetLastError();
}
