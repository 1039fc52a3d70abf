// engine.hip -- the C ABI of libjrq.so (include/jrq.h): engine lifetime, constant
// tables, staging for host-pointer calls, kernel dispatch and RCCL publication.
//
// Host-side code only; the kernels live in crc64.hip and quorum.hip.  Nothing here
// computes a result on the CPU: every jrq_* entry point runs its work on the GPU
// and fails (negative return) when no gfx950 device is usable.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/jrq.h"
#include "jrq_device.h"

extern "C" hipError_t jrq_launch_crc64(JrqCrcArgs* args, int log_entry, int grid,
                                       hipStream_t stream);
extern "C" hipError_t jrq_launch_crc64_fixed(JrqCrcArgs* args, int log_entry, int grid,
                                             hipStream_t stream);
extern "C" hipError_t jrq_launch_quorum(const JrqQuorumArgs* args, int num_cus, hipStream_t stream);
extern "C" hipError_t jrq_launch_quorum_epochs(const JrqQuorumArgs* args, uint32_t K,
                                               uint64_t match_eld, uint64_t la_eld,
                                               int num_cus, hipStream_t stream);
extern "C" hipError_t jrq_launch_ae_meta(const JrqAeArgs* a, hipStream_t stream);
extern "C" hipError_t jrq_launch_lease(const JrqLeaseArgs* a, int num_cus, hipStream_t stream);
extern "C" hipError_t jrq_launch_readindex(const JrqReadIndexArgs* a, int num_cus, hipStream_t stream);
extern "C" hipError_t jrq_launch_fanout(const JrqFanoutArgs* a, hipStream_t stream);
extern "C" hipError_t jrq_launch_v2_parse(const JrqV2Args* a, hipStream_t stream);
extern "C" hipError_t jrq_launch_v2_finish(const JrqV2Args* a, const JrqCrcArgs* walk, int num_cus,
                                           hipStream_t stream);
extern "C" hipError_t jrq_launch_ae_first_corrupt(const JrqAeArgs* a, hipStream_t stream);
extern "C" hipError_t jrq_launch_table_update(const JrqTableArgs* a, const JrqGroupState* states,
                                              uint32_t n_states, const uint64_t* recs,
                                              uint32_t n_recs, hipStream_t stream);
extern "C" hipError_t jrq_launch_table_epoch(const JrqTableArgs* a, hipStream_t stream);
extern "C" hipError_t jrq_launch_table_fsm(const JrqTableArgs* a, const uint32_t* groups, const int64_t* applied,
                                           const int64_t* first, const int64_t* size, uint32_t n,
                                           hipStream_t stream);
extern "C" hipError_t jrq_launch_table_fan_gather(const int64_t* ff, const uint8_t* fs, const uint32_t* n,
                                                  const uint32_t* off, uint32_t slices, int64_t* out_first,
                                                  uint8_t* out_status, hipStream_t stream);
extern "C" hipError_t jrq_launch_table_acks(const JrqTableArgs* a, const uint64_t* const* seg_ptr, uint32_t n,
                                            const uint32_t* seg_off, const uint64_t* seg_stamp,
                                            uint32_t nseg, hipStream_t stream);
extern "C" hipError_t jrq_launch_table_list_gather(const uint64_t* changed, const uint32_t* n,
                                                   uint32_t slices, uint32_t* off, uint32_t* total,
                                                   uint64_t* out, hipStream_t stream);

static_assert(sizeof(jrq_group_state) == sizeof(JrqGroupState), "jrq_group_state layout");
static_assert(JRQ_TABLE_MAX_RUNS == jrq::kTableMaxRuns, "table runs");
static_assert(JRQ_TABLE_SLICE == jrq::kListSlice, "table list slices");

namespace {

thread_local std::string g_create_error;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

}  // namespace

struct jrq_engine {
  int device = -1;
  int num_cus = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  uint64_t* slice = nullptr;  // [kSliceTables][256]
  uint64_t* xinv = nullptr;   // [8][256] TI[i][b] = b * x^(8i - 64) mod P (v2_decode.hip)
  uint64_t* shift = nullptr;  // [kShiftTables][8][256]
  uint64_t* acc = nullptr;    // straddler accumulators
  uint32_t* cnt = nullptr;    // straddler counters
  uint64_t* pieces = nullptr; // per-segment straddler pieces: [2][scratch_len]
  uint32_t* fan_ctr = nullptr; // commit fan-out {listed sum, blocks done}, zero between launches
  uint64_t* v2_gate = nullptr; // V2 decode gate {k, L, bad, end, arrivals, -, -, -, segment arrivals[16]}; arrivals zero between launches
  uint32_t scratch_len = 0;
  int crc_grid = 0;
  // Test / A-B overrides, set only through jrq_debug_set (never from the environment):
  // JRQ_DBG_CRC_SEG_BYTES: fixed CRC segment size (0 = automatic, ~payload / lanes); tests use
  // it to force many straddling entries
  uint64_t crc_seg_bytes = 0;
  int crc_regs = -1;         // JRQ_DBG_CRC_REGS: force the boundary path (-1: per call site)
  uint32_t regs_hint = 0;    // set by host variants around their _dev call (unaligned_bounds)
  uint32_t crc_prio = 1;     // JRQ_DBG_CRC_PRIO: progress-stepped wave priority (A/B knob)
  uint32_t crc_seg_map = 1;  // JRQ_DBG_CRC_SEG_MAP: 1 = per-workgroup contiguous chunks (faster on C5), 0 = interleaved
  bool upload_pageable = false;  // JRQ_DBG_UPLOAD_PAGEABLE: hand caller pages to HIP's own copy
  uint32_t max_groups = 0;
  uint8_t max_peers = 0;
  DevBuf stage[27];  // 0-13 host-variant staging, 14 stream-update chunk CRCs, 15 fixed-size offsets, 16-19 AppendEntries scratch, 20 jrq_table_read de-tiling, 21-26 V2 decode scratch
  // pinned bounce buffers for the host variants' uploads (stage_in): two chunks, each
  // reusable once the copy recorded after it has run
  uint8_t* bounce[2] = {nullptr, nullptr};
  hipEvent_t bounce_done[2] = {nullptr, nullptr};
  bool bounce_busy[2] = {false, false};
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = -1;
  std::string err;
};

namespace {

// --------------------------------------------------------------- helpers ---

struct DeviceGuard {  // (no set / restore when the caller is on the engine's device already:
  int prev = -1;       //  a launch-sized call should cost the launch, ~17 us epochs are host-bound)
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev == dev) {
      prev = -1;
      ok = true;
      return;
    }
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int fail(jrq_engine* e, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (e) e->err = buf;
  else g_create_error = buf;
  return code;
}

#define JRQ_HIP(e, call)                                                                    \
  do {                                                                                      \
    hipError_t _s = (call);                                                                 \
    if (_s != hipSuccess)                                                                   \
      return fail((e), JRQ_E_HIP, "%s failed: %s", #call, hipGetErrorString(_s));          \
  } while (0)

// GF(2)[x] / (x^64 + poly): a * b mod G, MSB-first representation as in CRC64.java.
uint64_t mulmod(uint64_t a, uint64_t b) {
  uint64_t r = 0;
  for (int i = 63; i >= 0; --i) {
    r = (r & 0x8000000000000000ULL) ? (r << 1) ^ jrq::kCrcPoly : (r << 1);
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
}

// Constant tables (see crc64.hip):
//   T0[i]  = CRC64 table entry (jraft-core/.../util/CRC64.java:41-92, generated from the poly)
//   T1[i]  = T0[i] advanced by one zero byte
//   slice  = { bswap(T0) .. bswap(T7) }  (reversed-domain slice-by-8)
//   shift[t][k][i] = (i * x^(8k)) * x^(8 * 2^t) mod G
//   xinv[k][i]     = i * x^(8k - 64) mod G   (x^-1 = x^63 + (p + 1) / x for G = x^64 + p)
void build_tables(std::vector<uint64_t>& slice, std::vector<uint64_t>& shift,
                  std::vector<uint64_t>& xinv) {
  uint64_t t[jrq::kSliceTables][256];
  for (int i = 0; i < 256; ++i) {
    uint64_t c = static_cast<uint64_t>(i) << 56;
    for (int k = 0; k < 8; ++k) c = (c & 0x8000000000000000ULL) ? (c << 1) ^ jrq::kCrcPoly : (c << 1);
    t[0][i] = c;
  }
  for (int j = 1; j < jrq::kSliceTables; ++j)  // T_j = T_{j-1} advanced by one zero byte
    for (int i = 0; i < 256; ++i) t[j][i] = t[0][t[j - 1][i] >> 56] ^ (t[j - 1][i] << 8);
  slice.resize(jrq::kSliceTables * 256);
  for (int j = 0; j < jrq::kSliceTables; ++j)
    for (int i = 0; i < 256; ++i) slice[j * 256 + i] = __builtin_bswap64(t[j][i]);
  shift.resize(static_cast<size_t>(jrq::kShiftTables) * 8 * 256);
  uint64_t K = 0x100;  // x^8
  for (int t = 0; t < jrq::kShiftTables; ++t) {
    for (int k = 0; k < 8; ++k)
      for (int i = 0; i < 256; ++i)
        shift[(static_cast<size_t>(t) * 8 + k) * 256 + i] = mulmod(static_cast<uint64_t>(i) << (8 * k), K);
    K = mulmod(K, K);  // x^(8 * 2^(t+1))
  }
  const uint64_t xm1 = (1ull << 63) | ((jrq::kCrcPoly ^ 1ull) >> 1);
  xinv.resize(8 * 256);
  for (int k = 0; k < 8; ++k)
    for (int i = 0; i < 256; ++i) {
      uint64_t v = static_cast<uint64_t>(i);
      for (int b = 0; b < 64 - 8 * k; ++b) v = (v >> 1) ^ ((v & 1ull) ? xm1 : 0ull);
      xinv[k * 256 + i] = v;
    }
}

int ensure_stage(jrq_engine* e, int slot, size_t bytes, void** out) {
  DevBuf& b = e->stage[slot];
  if (bytes == 0) bytes = 16;
  if (b.cap < bytes) {
    if (b.p) {
      JRQ_HIP(e, hipStreamSynchronize(e->stream));
      JRQ_HIP(e, hipFree(b.p));
      b.p = nullptr;
      b.cap = 0;
    }
    size_t cap = bytes + bytes / 4;
    JRQ_HIP(e, hipMalloc(&b.p, cap));
    b.cap = cap;
  }
  *out = b.p;
  return JRQ_OK;
}

// Host -> device upload of caller memory through the engine's pinned bounce chunks: a CPU
// copy into a pinned chunk, then an async DMA from it on the engine stream, two chunks in
// flight.  (Round 2 moved here from HIP's own pageable copy after that copy failed with
// "illegal memory access"; round 3 found the trigger elsewhere -- concurrent host
// registrations, now serialised in jrq_host_register -- and kept the bounce path: it needs no
// pinning of caller pages at all.  JRQ_DBG_UPLOAD_PAGEABLE selects HIP's copy for A/B runs.)
constexpr size_t kBounceChunk = size_t(8) << 20;

int ensure_bounce(jrq_engine* e) {
  for (int i = 0; i < 2; ++i)
    if (!e->bounce[i]) {
      JRQ_HIP(e, hipHostMalloc(reinterpret_cast<void**>(&e->bounce[i]), kBounceChunk, hipHostMallocDefault));
      JRQ_HIP(e, hipEventCreateWithFlags(&e->bounce_done[i], hipEventDisableTiming));
    }
  return JRQ_OK;
}

int upload(jrq_engine* e, void* dst, const void* src, size_t bytes) {
  if (int rc = ensure_bounce(e)) return rc;
  int i = 0;
  for (size_t off = 0; off < bytes; off += kBounceChunk, i ^= 1) {
    const size_t n = bytes - off < kBounceChunk ? bytes - off : kBounceChunk;
    if (e->bounce_busy[i]) JRQ_HIP(e, hipEventSynchronize(e->bounce_done[i]));
    std::memcpy(e->bounce[i], static_cast<const uint8_t*>(src) + off, n);
    JRQ_HIP(e, hipMemcpyAsync(static_cast<uint8_t*>(dst) + off, e->bounce[i], n,
                              hipMemcpyHostToDevice, e->stream));
    JRQ_HIP(e, hipEventRecord(e->bounce_done[i], e->stream));
    e->bounce_busy[i] = true;
  }
  return JRQ_OK;
}

// Device -> host into caller memory that is not page-locked: through the same bounce chunks
// (the DMA into one chunk overlaps the CPU copy out of the other), so that no HIP copy ever
// touches pageable memory.  HIP's pageable copies lock the caller's pages themselves and may
// keep them locked after the copy returns; a buffer the caller frees and the allocator later
// hands out again at the same address then meets a lock over pages that no longer exist.  Two
// bench runs (rounds 4 and 5) ended in "illegal memory access" at a pageable result copy after
// large pageable transfers of since-freed arrays.  Synchronous: the data is in
// `dst` when it returns.
int download(jrq_engine* e, void* dst, const void* src, size_t bytes) {
  if (int rc = ensure_bounce(e)) return rc;
  int prev = -1, i = 0;
  size_t prev_off = 0, prev_n = 0;
  auto drain = [&](int k, size_t off, size_t n) -> int {
    JRQ_HIP(e, hipEventSynchronize(e->bounce_done[k]));
    std::memcpy(static_cast<uint8_t*>(dst) + off, e->bounce[k], n);
    e->bounce_busy[k] = false;
    return JRQ_OK;
  };
  for (size_t off = 0; off < bytes; off += kBounceChunk, i ^= 1) {
    const size_t n = bytes - off < kBounceChunk ? bytes - off : kBounceChunk;
    if (e->bounce_busy[i]) JRQ_HIP(e, hipEventSynchronize(e->bounce_done[i]));  // an upload's DMA
    JRQ_HIP(e, hipMemcpyAsync(e->bounce[i], static_cast<const uint8_t*>(src) + off, n,
                              hipMemcpyDeviceToHost, e->stream));
    JRQ_HIP(e, hipEventRecord(e->bounce_done[i], e->stream));
    e->bounce_busy[i] = true;
    if (prev >= 0)
      if (int rc = drain(prev, prev_off, prev_n)) return rc;
    prev = i;
    prev_off = off;
    prev_n = n;
  }
  if (prev >= 0) return drain(prev, prev_off, prev_n);
  return JRQ_OK;
}

// Caller memory registered with HIP (jrq_host_register, hipHostMalloc) goes straight to the
// DMA engine; anything else through the bounce chunks.
// Page-locked ranges libjrq made itself (jrq_host_alloc / jrq_host_register), base -> range:
// an upload from one of them needs no HIP pointer query (a flush stages ~30 parts), and a
// registration whose pages overlap a live one is refused (jrq_host_register).
struct PinnedRange {
  size_t bytes;
  bool owned;  // jrq_host_alloc (freed with jrq_host_free), else a caller registration
};
std::mutex g_pinned_mu;
std::map<uintptr_t, PinnedRange> g_pinned;
constexpr uintptr_t kPage = 4096;

bool known_pinned(const void* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> lk(g_pinned_mu);
  auto it = g_pinned.upper_bound(a);
  if (it == g_pinned.begin()) return false;
  --it;
  return a < it->first + it->second.bytes;
}

// Does [p, p + bytes), widened to whole pages, share a page with a live range?  The driver pins
// and maps whole pages, so two registrations sharing one would each hold a mapping of it.
bool overlaps_live_pages(uintptr_t p, size_t bytes) {
  const uintptr_t lo = p & ~(kPage - 1), hi = (p + bytes + kPage - 1) & ~(kPage - 1);
  std::lock_guard<std::mutex> lk(g_pinned_mu);
  auto it = g_pinned.lower_bound(hi);  // first range starting at or past hi: no overlap
  while (it != g_pinned.begin()) {
    --it;
    const uintptr_t rlo = it->first & ~(kPage - 1);
    const uintptr_t rhi = (it->first + it->second.bytes + kPage - 1) & ~(kPage - 1);
    if (rlo < hi && lo < rhi) return true;
    if (rhi <= lo) break;  // ranges are disjoint in pages, so ordered by end as by start
  }
  return false;
}

void note_pinned(const void* p, size_t bytes, bool owned) {
  std::lock_guard<std::mutex> lk(g_pinned_mu);
  g_pinned[reinterpret_cast<uintptr_t>(p)] = PinnedRange{bytes, owned};
}

// The live range starting exactly at p: 1 caller registration, 2 jrq_host_alloc, 0 none.
int pinned_kind(const void* p) {
  std::lock_guard<std::mutex> lk(g_pinned_mu);
  auto it = g_pinned.find(reinterpret_cast<uintptr_t>(p));
  return it == g_pinned.end() ? 0 : (it->second.owned ? 2 : 1);
}

void forget_pinned(const void* p) {
  std::lock_guard<std::mutex> lk(g_pinned_mu);
  g_pinned.erase(reinterpret_cast<uintptr_t>(p));
}

bool host_pinned(const void* p) {
  if (known_pinned(p)) return true;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // an unregistered pointer reports an error: not sticky
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

int download_any(jrq_engine* e, void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return JRQ_OK;
  if (e->upload_pageable || host_pinned(dst)) {
    JRQ_HIP(e, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, e->stream));
    return JRQ_OK;
  }
  return download(e, dst, src, bytes);
}
#define JRQ_DOWN(e, dst, src, bytes)                        \
  do {                                                      \
    const int _rc = download_any((e), (dst), (src), (bytes)); \
    if (_rc) return _rc;                                    \
  } while (0)

int upload_any(jrq_engine* e, void* dst, const void* src, size_t bytes) {
  if (e->upload_pageable || host_pinned(src)) {
    JRQ_HIP(e, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e->stream));
    return JRQ_OK;
  }
  return upload(e, dst, src, bytes);
}

template <typename T>
int stage_in(jrq_engine* e, int slot, const T* host, size_t count, const T** dev) {
  if (host == nullptr) {
    *dev = nullptr;
    return JRQ_OK;
  }
  void* p = nullptr;
  int rc = ensure_stage(e, slot, count * sizeof(T), &p);
  if (rc) return rc;
  if (count && (rc = upload_any(e, p, host, count * sizeof(T)))) return rc;
  *dev = static_cast<const T*>(p);
  return JRQ_OK;
}

// offsets[0..n] must be monotone: the CRC kernels' segment walk and lower-bound search assume
// it, and an interior offset below offsets[0] would wrap in the host variants' rebase and send
// the kernels past the staged window.
int check_monotone(jrq_engine* e, const uint64_t* off, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return fail(e, JRQ_E_INVALID, "offsets not monotone at entry %u", i);
  return JRQ_OK;
}

// offsets[i] = i * entry_bytes: the segment walk's view of a fixed-size batch the fixed kernel
// cannot take (crc_fixed_k)
__global__ void iota_offsets_kernel(uint64_t* off, uint32_t n, uint64_t entry_bytes) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += gridDim.x * blockDim.x)
    off[i] = static_cast<uint64_t>(i) * entry_bytes;
}

// crc64_fixed_kernel (crc64.hip) takes a batch of N entries of entry_bytes each, k lanes per
// entry (k pieces): the fewest k (a power of two <= 64) that gives every lane of the grid a
// piece, with pieces of whole 256-B multiples (4-half-round turns) whose 64-lane rows fit the
// u32 lane offsets, on a 16-B aligned payload.  0 = not applicable (the offsets path).
// C1: 1M x 256 B -> k = 1; C5: 64k x 16 KiB -> k = 2.
uint32_t crc_fixed_k(const jrq_engine* e, const void* payload, uint64_t entry_bytes, uint32_t N) {
  if (entry_bytes < 256 || entry_bytes % 256 != 0 || (reinterpret_cast<uintptr_t>(payload) & 15u))
    return 0;
  const uint64_t lanes = static_cast<uint64_t>(e->crc_grid) * jrq::kCrcFixedBlock;
  uint32_t k = 1;
  while (static_cast<uint64_t>(N) * k < lanes && k < 64 && (entry_bytes / (2 * k)) % 256 == 0) k *= 2;
  if (static_cast<uint64_t>(N) * k < lanes || entry_bytes / k >= (1ull << 26)) return 0;
  return k;
}

// All N ranges of a host offsets array the same length (0 if not).
uint64_t uniform_length(const uint64_t* off, uint32_t n) {
  const uint64_t L = off[1] - off[0];
  for (uint32_t i = 1; i < n; ++i)
    if (off[i + 1] - off[i] != L) return 0;
  return L;
}

int crc_fixed_dispatch(jrq_engine* e, JrqCrcArgs& a, int log_entry) {
  a.slice = e->slice;
  a.shift = e->shift;
  JRQ_HIP(e, jrq_launch_crc64_fixed(&a, log_entry, e->crc_grid, e->stream));
  return JRQ_OK;
}

// Entry boundaries off the 64-B half-round grid make the CRC kernel's boundary path frequent:
// host variants then pick the register boundary path (crc64_rounds_kernel<true>).
uint32_t unaligned_bounds(const uint64_t* off, uint32_t n) {
  for (uint32_t i = 1; i <= n; ++i)
    if ((off[i] - off[0]) & 63u) return 1;
  return 0;
}

int crc_dispatch(jrq_engine* e, JrqCrcArgs& a, int log_entry) {
  if (a.n == 0) return JRQ_OK;
  a.slice = e->slice;
  a.shift = e->shift;
  a.acc = e->acc;
  a.cnt = e->cnt;
  a.piece_cont = e->pieces;
  a.piece_tail = e->pieces + e->scratch_len;
  a.scratch_len = e->scratch_len;
  a.seg_bytes = e->crc_seg_bytes;
  a.seg_map = e->crc_seg_map;
  a.prio_steps = e->crc_prio;
  if (e->crc_regs >= 0) a.regs_slowpath = static_cast<uint32_t>(e->crc_regs);
  else a.regs_slowpath |= e->regs_hint;
  JRQ_HIP(e, jrq_launch_crc64(&a, log_entry, e->crc_grid, e->stream));
  return JRQ_OK;
}

}  // namespace

// ================================================================ C ABI ====

extern "C" {

int jrq_abi_version(void) { return JRQ_ABI_VERSION; }

const char* jrq_last_error(const jrq_engine* e) {
  return e ? e->err.c_str() : g_create_error.c_str();
}

jrq_engine* jrq_create(int device, uint32_t max_groups, uint8_t max_peers, int* err) {
  auto set = [&](int c) {
    if (err) *err = c;
  };
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    fail(nullptr, JRQ_E_NODEV, "no HIP device visible");
    set(JRQ_E_NODEV);
    return nullptr;
  }
  if (device < 0 || device >= ndev || max_peers == 0 || max_peers > JRQ_MAX_PEERS) {
    fail(nullptr, JRQ_E_INVALID, "bad device %d or max_peers %u", device, max_peers);
    set(JRQ_E_INVALID);
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess ||
      std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    fail(nullptr, JRQ_E_NODEV, "device %d is not gfx950 (%s)", device, prop.gcnArchName);
    set(JRQ_E_NODEV);
    return nullptr;
  }
  DeviceGuard guard(device);
  auto* e = new jrq_engine();
  e->device = device;
  e->num_cus = prop.multiProcessorCount;
  e->max_groups = max_groups;
  e->max_peers = max_peers;
  e->crc_grid = e->num_cus;  // persistent: one 1024-thread workgroup per CU (128 KiB LDS)
  e->scratch_len = static_cast<uint32_t>(2ull * e->crc_grid * jrq::kCrcRegsBlock + 2);  // >= 2 slots per lane
  int rc = JRQ_OK;
  std::vector<uint64_t> slice, shift, xinv;
  build_tables(slice, shift, xinv);
  auto try_hip = [&](hipError_t s, const char* what) {
    if (s != hipSuccess && rc == JRQ_OK) rc = fail(nullptr, JRQ_E_HIP, "%s: %s", what, hipGetErrorString(s));
  };
  try_hip(hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking), "hipStreamCreate");
  e->stream = e->own_stream;
  try_hip(hipMalloc(&e->slice, slice.size() * 8), "hipMalloc(slice)");
  try_hip(hipMalloc(&e->shift, shift.size() * 8), "hipMalloc(shift)");
  try_hip(hipMalloc(&e->xinv, xinv.size() * 8), "hipMalloc(xinv)");
  // acc/cnt: [scratch_len] entry slots + [2 * (scratch_len / 64 + 2)] 64-segment group slots
  // + [2 * (scratch_len / 4096 + 2)] 64-group supergroup slots (crc64.hip straddle_piece)
  const size_t slots = e->scratch_len + 2 * (e->scratch_len / 64 + 2) + 2 * (e->scratch_len / 4096 + 2);
  try_hip(hipMalloc(&e->acc, slots * 8), "hipMalloc(acc)");
  try_hip(hipMalloc(&e->cnt, slots * 4), "hipMalloc(cnt)");
  try_hip(hipMalloc(&e->pieces, static_cast<size_t>(e->scratch_len) * 16), "hipMalloc(pieces)");
  try_hip(hipMalloc(&e->fan_ctr, 16), "hipMalloc(fan_ctr)");
  try_hip(hipMalloc(&e->v2_gate, 8 * (8 + 16)), "hipMalloc(v2_gate)");
  if (rc == JRQ_OK) {
    try_hip(hipMemset(e->fan_ctr, 0, 16), "zero fan_ctr");
    try_hip(hipMemset(e->v2_gate, 0, 8 * (8 + 16)), "zero v2_gate");
    try_hip(hipMemcpy(e->slice, slice.data(), slice.size() * 8, hipMemcpyHostToDevice), "upload slice");
    try_hip(hipMemcpy(e->shift, shift.data(), shift.size() * 8, hipMemcpyHostToDevice), "upload shift");
    try_hip(hipMemcpy(e->xinv, xinv.data(), xinv.size() * 8, hipMemcpyHostToDevice), "upload xinv");
    try_hip(hipMemset(e->acc, 0, slots * 8), "zero acc");
    try_hip(hipMemset(e->cnt, 0, slots * 4), "zero cnt");
  }
  if (rc != JRQ_OK) {
    set(rc);
    jrq_destroy(e);
    return nullptr;
  }
  set(JRQ_OK);
  return e;
}

void jrq_destroy(jrq_engine* e) {
  if (!e) return;
  DeviceGuard guard(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->comm) (void)ncclCommDestroy(e->comm);
  for (auto& b : e->stage)
    if (b.p) (void)hipFree(b.p);
  for (int i = 0; i < 2; ++i) {
    if (e->bounce[i]) (void)hipHostFree(e->bounce[i]);
    if (e->bounce_done[i]) (void)hipEventDestroy(e->bounce_done[i]);
  }
  if (e->slice) (void)hipFree(e->slice);
  if (e->shift) (void)hipFree(e->shift);
  if (e->xinv) (void)hipFree(e->xinv);
  if (e->acc) (void)hipFree(e->acc);
  if (e->cnt) (void)hipFree(e->cnt);
  if (e->pieces) (void)hipFree(e->pieces);
  if (e->fan_ctr) (void)hipFree(e->fan_ctr);
  if (e->v2_gate) (void)hipFree(e->v2_gate);
  if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
  delete e;
}

void* jrq_get_stream(jrq_engine* e) { return e ? static_cast<void*>(e->stream) : nullptr; }

int jrq_set_stream(jrq_engine* e, void* s) {
  if (!e) return JRQ_E_INVALID;
  e->stream = s ? static_cast<hipStream_t>(s) : e->own_stream;
  return JRQ_OK;
}

int jrq_synchronize(jrq_engine* e) {
  if (!e) return JRQ_E_INVALID;
  DeviceGuard guard(e->device);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

int jrq_debug_set(jrq_engine* e, int option, int64_t value) {
  if (!e) return JRQ_E_INVALID;
  switch (option) {
    case JRQ_DBG_CRC_SEG_BYTES:  // rounded up to 256 B by the kernel
      if (value < 0) break;
      e->crc_seg_bytes = static_cast<uint64_t>(value);
      return JRQ_OK;
    case JRQ_DBG_CRC_REGS:
      if (value < -1 || value > 1) break;
      e->crc_regs = static_cast<int>(value);
      return JRQ_OK;
    case JRQ_DBG_CRC_PRIO:
      if (value < 0 || value > 3) break;
      e->crc_prio = static_cast<uint32_t>(value);
      return JRQ_OK;
    case JRQ_DBG_CRC_SEG_MAP:
      if (value < 0 || value > 1) break;
      e->crc_seg_map = static_cast<uint32_t>(value);
      return JRQ_OK;
    case JRQ_DBG_UPLOAD_PAGEABLE:
      if (value < 0 || value > 1) break;
      e->upload_pageable = value != 0;
      return JRQ_OK;
    default:
      return fail(e, JRQ_E_INVALID, "unknown debug option %d", option);
  }
  return fail(e, JRQ_E_INVALID, "debug option %d: value %lld out of range", option,
              static_cast<long long>(value));
}

// Registration, unregistration and driver-owned page-locked allocations go through one
// process-wide lock.  Round 3 traced the round-2/3 "illegal memory access" of a later pageable
// copy to hipHostRegister / hipHostUnregister called from several threads at once (the C++
// mirror's pack workers each registering their own staging buffer): with the same buffers
// registered from one thread, or allocated with hipHostMalloc, the failing test passed
// (DESIGN.md §4.10).  A JNI host may pin DirectByteBuffers from any thread, so the library
// serialises the calls itself; they are rare (setup, buffer growth), never per epoch.
//
// Round 4 saw one more "illegal memory access" from a pageable device-to-host copy after a clean
// synchronisation, in a bench run whose previous leg had registered numpy arrays that share
// heap pages with their neighbours, ignored the unregister return codes and freed the arrays
// (DESIGN.md §4.10).  The driver pins and maps whole pages: a page shared by two registrations
// is mapped twice, and a registration that outlives its memory leaves HIP treating whatever the
// allocator later puts at that address as registered -- a copy to or from it then DMAs through
// a mapping of pages the process no longer has.  So the registry is kept at page granularity:
// a registration whose pages touch a live one is refused (the buffer then travels through the
// bounce chunks), an unregistration forgets its range only once HIP has dropped it, and only
// ranges this library registered can be unregistered.
namespace {
std::mutex g_pin_mu;
}  // namespace

int jrq_host_register(void* ptr, size_t bytes) {
  if (!ptr || !bytes) return JRQ_E_INVALID;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  if (overlaps_live_pages(reinterpret_cast<uintptr_t>(ptr), bytes)) return JRQ_E_STATE;
  if (hipHostRegister(ptr, bytes, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return JRQ_E_HIP;
  }
  note_pinned(ptr, bytes, false);
  return JRQ_OK;
}

int jrq_host_unregister(void* ptr) {
  if (!ptr) return JRQ_E_INVALID;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  if (pinned_kind(ptr) != 1) return JRQ_E_INVALID;  // not a live jrq_host_register range
  if (hipHostUnregister(ptr) != hipSuccess) {
    (void)hipGetLastError();
    return JRQ_E_HIP;  // still registered: still known, so no later registration overlaps it
  }
  forget_pinned(ptr);
  return JRQ_OK;
}

int jrq_host_registered_bytes(const void* ptr, size_t* bytes) {
  if (!bytes) return JRQ_E_INVALID;
  std::lock_guard<std::mutex> lk(g_pinned_mu);
  *bytes = 0;
  if (!ptr) {  // NULL: the total over every live range (a leak check for hosts and tests)
    for (auto& r : g_pinned) *bytes += r.second.bytes;
    return static_cast<int>(g_pinned.size());
  }
  auto it = g_pinned.find(reinterpret_cast<uintptr_t>(ptr));
  if (it == g_pinned.end()) return 0;
  *bytes = it->second.bytes;
  return 1;
}

int jrq_host_alloc(size_t bytes, void** out) {
  if (!out) return JRQ_E_INVALID;
  *out = nullptr;
  if (!bytes) return JRQ_E_INVALID;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return JRQ_E_NOMEM;
  }
  note_pinned(*out, bytes, true);
  return JRQ_OK;
}

int jrq_host_free(void* ptr) {
  if (!ptr) return JRQ_E_INVALID;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  if (pinned_kind(ptr) != 2) return JRQ_E_INVALID;  // not a live jrq_host_alloc block
  if (hipHostFree(ptr) != hipSuccess) {
    (void)hipGetLastError();
    return JRQ_E_HIP;
  }
  forget_pinned(ptr);
  return JRQ_OK;
}

// ----------------------------------------------------------------- quorum ---

int jrq_quorum_epoch_dev(jrq_engine* e, const jrq_group_batch* in, int64_t* committed_out,
                         uint8_t* status_out, uint32_t G) {
  if (!e || !in) return e ? fail(e, JRQ_E_INVALID, "null batch") : JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (in->num_peers == 0 || in->num_peers > JRQ_MAX_PEERS)
    return fail(e, JRQ_E_INVALID, "num_peers %u outside 1..%d", in->num_peers, JRQ_MAX_PEERS);
  if (!in->match || !in->pending_index || !in->last_appended || !in->last_committed ||
      !committed_out || !status_out || !in->conf ||
      (in->run_off && (!in->run_start || !in->run_conf)) || in->match_ld < G)
    return fail(e, JRQ_E_INVALID, "missing array or match_ld < G");
  DeviceGuard guard(e->device);
  JrqQuorumArgs a{};
  a.match = in->match;
  a.pending_index = in->pending_index;
  a.last_appended = in->last_appended;
  a.last_committed = in->last_committed;
  a.conf = in->conf;
  a.run_off = in->run_off;
  a.run_start = in->run_start;
  a.run_conf = in->run_conf;
  a.num_peers = in->num_peers;
  a.match_ld = in->match_ld;
  a.committed = committed_out;
  a.status = status_out;
  a.G = G;
  // enough 256-thread blocks for ~8 per CU, grid-stride beyond
  JRQ_HIP(e, jrq_launch_quorum(&a, e->num_cus, e->stream));
  return JRQ_OK;
}

int jrq_quorum_epoch_tiles_dev(jrq_engine* e, const jrq_group_tiles* in, int64_t* committed_out,
                               uint8_t* status_out, uint32_t G) {
  if (!e || !in) return e ? fail(e, JRQ_E_INVALID, "null batch") : JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (in->num_peers == 0 || in->num_peers > JRQ_MAX_PEERS)
    return fail(e, JRQ_E_INVALID, "num_peers %u outside 1..%d", in->num_peers, JRQ_MAX_PEERS);
  if (!in->tiles || !committed_out || !status_out || (in->run_off && (!in->run_start || !in->run_conf)))
    return fail(e, JRQ_E_INVALID, "missing array");
  if (G < 2 || (reinterpret_cast<uintptr_t>(in->tiles) & 15u) || (reinterpret_cast<uintptr_t>(committed_out) & 15u) ||
      (reinterpret_cast<uintptr_t>(status_out) & 1u))
    return fail(e, JRQ_E_INVALID, "tiles / committed_out not 16-B aligned, status_out odd or G < 2");
  DeviceGuard guard(e->device);
  const uint32_t P = in->num_peers;
  JrqQuorumArgs a{};
  a.match = in->tiles;
  a.pending_index = in->tiles + 256u * P;
  a.last_appended = a.pending_index + 256;
  a.last_committed = a.last_appended + 256;
  a.conf = reinterpret_cast<const uint64_t*>(a.last_committed + 256);
  a.ts = 256ull * (P + 4);
  a.run_off = in->run_off;
  a.run_start = in->run_start;
  a.run_conf = in->run_conf;
  a.num_peers = P;
  a.match_ld = 0;
  a.committed = committed_out;
  a.status = status_out;
  a.G = G;
  JRQ_HIP(e, jrq_launch_quorum(&a, e->num_cus, e->stream));
  return JRQ_OK;
}

int jrq_quorum_epoch_tiles(jrq_engine* e, const jrq_group_tiles* in, int64_t* committed_out,
                           uint8_t* status_out, uint32_t G) {
  if (!e || !in) return e ? fail(e, JRQ_E_INVALID, "null batch") : JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (!committed_out || !status_out || !in->tiles || in->num_peers == 0 || in->num_peers > JRQ_MAX_PEERS ||
      (in->run_off && (!in->run_start || !in->run_conf)))
    return fail(e, JRQ_E_INVALID, "missing array or bad num_peers");
  DeviceGuard guard(e->device);
  jrq_group_tiles d = *in;
  int rc;
  const size_t words = (static_cast<size_t>(G) + 255) / 256 * 256 * (in->num_peers + 4);
  if ((rc = stage_in(e, 0, in->tiles, words, &d.tiles))) return rc;
  if (in->run_off) {  // host memory: the CSR is checked before a kernel indexes with it
    const uint32_t* ro = in->run_off;
    if (ro[0] != 0) return fail(e, JRQ_E_INVALID, "run_off must start at 0");
    for (uint32_t g = 0; g < G; ++g)
      if (ro[g + 1] < ro[g]) return fail(e, JRQ_E_INVALID, "run_off not monotone at group %u", g);
    if ((rc = stage_in(e, 5, in->run_off, static_cast<size_t>(G) + 1, &d.run_off))) return rc;
    if ((rc = stage_in(e, 6, in->run_start, ro[G], &d.run_start))) return rc;
    if ((rc = stage_in(e, 7, in->run_conf, ro[G], &d.run_conf))) return rc;
  }
  void *dc = nullptr, *ds = nullptr;
  if ((rc = ensure_stage(e, 8, static_cast<size_t>(G) * 8, &dc))) return rc;
  if ((rc = ensure_stage(e, 9, G, &ds))) return rc;
  if ((rc = jrq_quorum_epoch_tiles_dev(e, &d, static_cast<int64_t*>(dc), static_cast<uint8_t*>(ds), G)))
    return rc;
  JRQ_DOWN(e, committed_out, dc, static_cast<size_t>(G) * 8);
  JRQ_DOWN(e, status_out, ds, G);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

int jrq_quorum_epoch(jrq_engine* e, const jrq_group_batch* in, int64_t* committed_out,
                     uint8_t* status_out, uint32_t G) {
  if (!e || !in) return e ? fail(e, JRQ_E_INVALID, "null batch") : JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (!committed_out || !status_out) return fail(e, JRQ_E_INVALID, "null output");
  if (in->num_peers == 0 || in->num_peers > JRQ_MAX_PEERS || in->match_ld < G || !in->match)
    return fail(e, JRQ_E_INVALID, "bad num_peers / match_ld");
  if (!in->pending_index || !in->last_appended || !in->last_committed ||
      (!in->run_off && !in->conf) || (in->run_off && (!in->run_start || !in->run_conf)))
    return fail(e, JRQ_E_INVALID, "missing group array");
  DeviceGuard guard(e->device);
  jrq_group_batch d = *in;
  int rc;
  const size_t P = in->num_peers;
  std::vector<uint64_t> cw;  // flagged conf words (outlives the asynchronous staging copy)
  if ((rc = stage_in(e, 0, in->match, (P - 1) * in->match_ld + G, &d.match))) return rc;
  if ((rc = stage_in(e, 1, in->pending_index, G, &d.pending_index))) return rc;
  if ((rc = stage_in(e, 2, in->last_appended, G, &d.last_appended))) return rc;
  if ((rc = stage_in(e, 3, in->last_committed, G, &d.last_committed))) return rc;
  if (in->run_off) {
    // the CSR is host memory here: check it before any kernel indexes with it
    const uint32_t* ro = in->run_off;
    if (ro[0] != 0 || ro[G] > in->num_runs)
      return fail(e, JRQ_E_INVALID, "run_off must start at 0 and end <= num_runs");
    // conf words with JRQ_CONF_RUNS on exactly the groups whose runs the kernels must walk:
    // a group with one run is an ordinary single-conf group (the fast path)
    cw.resize(G);
    for (uint32_t g = 0; g < G; ++g) {
      if (ro[g + 1] < ro[g]) return fail(e, JRQ_E_INVALID, "run_off not monotone at group %u", g);
      const uint32_t n = ro[g + 1] - ro[g];
      cw[g] = n == 1 ? (in->run_conf[ro[g]] & ~JRQ_CONF_RUNS)
                     : (JRQ_CONF_RUNS | (in->conf ? in->conf[g] : 0));
    }
    if ((rc = stage_in(e, 4, cw.data(), G, &d.conf))) return rc;
    if ((rc = stage_in(e, 5, in->run_off, static_cast<size_t>(G) + 1, &d.run_off))) return rc;
    if ((rc = stage_in(e, 6, in->run_start, in->num_runs, &d.run_start))) return rc;
    if ((rc = stage_in(e, 7, in->run_conf, in->num_runs, &d.run_conf))) return rc;
  } else {
    if ((rc = stage_in(e, 4, in->conf, G, &d.conf))) return rc;
  }
  void *dc = nullptr, *ds = nullptr;
  if ((rc = ensure_stage(e, 8, static_cast<size_t>(G) * 8, &dc))) return rc;
  if ((rc = ensure_stage(e, 9, G, &ds))) return rc;
  if ((rc = jrq_quorum_epoch_dev(e, &d, static_cast<int64_t*>(dc), static_cast<uint8_t*>(ds), G)))
    return rc;
  JRQ_DOWN(e, committed_out, dc, static_cast<size_t>(G) * 8);
  JRQ_DOWN(e, status_out, ds, G);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

// --------------------------------------------------------------- checksum ---

int jrq_quorum_epochs_dev(jrq_engine* e, const jrq_group_batch* in, uint32_t K,
                          uint64_t match_eld, uint64_t la_eld, int64_t* committed_out,
                          uint8_t* status_out, uint32_t G) {
  if (!e || !in) return e ? fail(e, JRQ_E_INVALID, "null batch") : JRQ_E_INVALID;
  if (G == 0 || K == 0) return JRQ_OK;
  if (!committed_out || !status_out) return fail(e, JRQ_E_INVALID, "null output");
  if (in->num_peers == 0 || in->num_peers > JRQ_MAX_PEERS || in->match_ld < G || !in->match ||
      !in->pending_index || !in->last_appended || !in->last_committed || !in->conf)
    return fail(e, JRQ_E_INVALID, "bad num_peers / match_ld / null array");
  if (in->run_off && (!in->run_start || !in->run_conf))
    return fail(e, JRQ_E_INVALID, "run_off without run_start / run_conf");
  if (K > 1 && (match_eld < static_cast<uint64_t>(in->num_peers) * in->match_ld || la_eld < G))
    return fail(e, JRQ_E_INVALID, "epoch strides overlap");
  DeviceGuard guard(e->device);
  JrqQuorumArgs a{};
  a.match = in->match;
  a.pending_index = in->pending_index;
  a.last_appended = in->last_appended;
  a.last_committed = in->last_committed;
  a.conf = in->conf;
  a.run_off = in->run_off;
  a.run_start = in->run_start;
  a.run_conf = in->run_conf;
  a.num_peers = in->num_peers;
  a.match_ld = in->match_ld;
  a.committed = committed_out;
  a.status = status_out;
  a.G = G;
  JRQ_HIP(e, jrq_launch_quorum_epochs(&a, K, match_eld, la_eld, e->num_cus, e->stream));
  return JRQ_OK;
}

int jrq_quorum_epochs_tiles_dev(jrq_engine* e, const jrq_group_tiles* in, uint32_t K,
                                uint64_t epoch_ld, int64_t* committed_out, uint8_t* status_out,
                                uint32_t G) {
  if (!e || !in) return e ? fail(e, JRQ_E_INVALID, "null batch") : JRQ_E_INVALID;
  if (G == 0 || K == 0) return JRQ_OK;
  if (in->num_peers == 0 || in->num_peers > JRQ_MAX_PEERS)
    return fail(e, JRQ_E_INVALID, "num_peers %u outside 1..%d", in->num_peers, JRQ_MAX_PEERS);
  if (!in->tiles || !committed_out || !status_out || (in->run_off && (!in->run_start || !in->run_conf)))
    return fail(e, JRQ_E_INVALID, "missing array");
  const uint32_t P = in->num_peers;
  const uint64_t extent = (static_cast<uint64_t>(G) + 255) / 256 * 256 * (P + 4);
  if (K > 1 && epoch_ld < extent) return fail(e, JRQ_E_INVALID, "epoch_ld below the tiles' extent");
  if (G < 2 || (epoch_ld & 1u) || (reinterpret_cast<uintptr_t>(in->tiles) & 15u) ||
      (reinterpret_cast<uintptr_t>(committed_out) & 15u) || (G & 1u && K > 1) ||
      (reinterpret_cast<uintptr_t>(status_out) & 1u))
    return fail(e, JRQ_E_INVALID, "tiles / committed_out not 16-B aligned, epoch_ld odd, status_out odd, "
                                  "G < 2, or G odd with K > 1");
  DeviceGuard guard(e->device);
  JrqQuorumArgs a{};
  a.match = in->tiles;
  a.pending_index = in->tiles + 256u * P;
  a.last_appended = a.pending_index + 256;
  a.last_committed = a.last_appended + 256;
  a.conf = reinterpret_cast<const uint64_t*>(a.last_committed + 256);
  a.ts = 256ull * (P + 4);
  a.run_off = in->run_off;
  a.run_start = in->run_start;
  a.run_conf = in->run_conf;
  a.num_peers = P;
  a.committed = committed_out;
  a.status = status_out;
  a.G = G;
  JRQ_HIP(e, jrq_launch_quorum_epochs(&a, K, epoch_ld, epoch_ld, e->num_cus, e->stream));
  return JRQ_OK;
}

int jrq_crc64_batch_dev(jrq_engine* e, const uint8_t* payload, const uint64_t* offsets, uint32_t N,
                        uint64_t* crc_out) {
  if (!e) return JRQ_E_INVALID;
  if (N == 0) return JRQ_OK;
  if (!payload || !offsets || !crc_out) return fail(e, JRQ_E_INVALID, "null pointer");
  DeviceGuard guard(e->device);
  JrqCrcArgs a{};
  a.payload = payload;
  a.offsets = offsets;
  a.n = N;
  a.out = crc_out;
  return crc_dispatch(e, a, 0);
}

// The segment walk over generated offsets (stage 15), for fixed-size batches the fixed kernel
// cannot take.
int fixed_offsets(jrq_engine* e, uint64_t entry_bytes, uint32_t N, const uint64_t** off) {
  void* d = nullptr;
  int rc;
  if ((rc = ensure_stage(e, 15, (static_cast<size_t>(N) + 1) * 8, &d))) return rc;
  const uint32_t blocks = (N + 1 + 255) / 256;
  hipLaunchKernelGGL(iota_offsets_kernel, dim3(blocks < 1024 ? blocks : 1024), dim3(256), 0,
                     e->stream, static_cast<uint64_t*>(d), N, entry_bytes);
  JRQ_HIP(e, hipGetLastError());
  *off = static_cast<const uint64_t*>(d);
  return JRQ_OK;
}

int jrq_crc64_fixed_dev(jrq_engine* e, const uint8_t* payload, uint64_t entry_bytes, uint32_t N,
                        uint64_t* crc_out) {
  if (!e) return JRQ_E_INVALID;
  if (N == 0) return JRQ_OK;
  if (!payload || !crc_out) return fail(e, JRQ_E_INVALID, "null pointer");
  DeviceGuard guard(e->device);
  const uint32_t k = crc_fixed_k(e, payload, entry_bytes, N);
  if (k == 0) {
    const uint64_t* off;
    int rc;
    if ((rc = fixed_offsets(e, entry_bytes, N, &off))) return rc;
    return jrq_crc64_batch_dev(e, payload, off, N, crc_out);
  }
  JrqCrcArgs a{};
  a.payload = payload;
  a.n = N;
  a.out = crc_out;
  a.entry_bytes = entry_bytes;
  a.fixed_k = k;
  return crc_fixed_dispatch(e, a, 0);
}

int jrq_crc64_batch(jrq_engine* e, const uint8_t* payload, const uint64_t* offsets, uint32_t N,
                    uint64_t* crc_out) {
  if (!e) return JRQ_E_INVALID;
  if (N == 0) return JRQ_OK;
  if (!payload || !offsets || !crc_out) return fail(e, JRQ_E_INVALID, "null pointer");
  DeviceGuard guard(e->device);
  int rc;
  if ((rc = check_monotone(e, offsets, N))) return rc;
  const uint64_t lo = offsets[0], hi = offsets[N];
  // stage only the referenced payload window and rebase the offsets onto it
  const uint8_t* dp;
  const uint64_t* doff;
  if ((rc = stage_in(e, 10, payload + lo, hi - lo, &dp))) return rc;
  std::vector<uint64_t> rebased(offsets, offsets + N + 1);
  for (auto& o : rebased) o -= lo;
  if ((rc = stage_in(e, 11, rebased.data(), rebased.size(), &doff))) return rc;
  void* dout = nullptr;
  if ((rc = ensure_stage(e, 12, static_cast<size_t>(N) * 8, &dout))) return rc;
  JrqCrcArgs a{};
  a.payload = dp;
  a.offsets = doff;
  a.n = N;
  a.out = static_cast<uint64_t*>(dout);
  a.regs_slowpath = unaligned_bounds(offsets, N);
  const uint64_t ul = uniform_length(offsets, N);
  if (const uint32_t k = crc_fixed_k(e, dp, ul, N)) {
    a.entry_bytes = ul;
    a.fixed_k = k;
    rc = crc_fixed_dispatch(e, a, 0);
  } else {
    rc = crc_dispatch(e, a, 0);
  }
  if (rc) return rc;
  JRQ_DOWN(e, crc_out, dout, static_cast<size_t>(N) * 8);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

int jrq_crc64_stream_update_dev(jrq_engine* e, uint64_t* state, const uint8_t* payload,
                                const uint64_t* offsets, uint32_t S) {
  if (!e) return JRQ_E_INVALID;
  if (S == 0) return JRQ_OK;
  if (!state || !payload || !offsets) return fail(e, JRQ_E_INVALID, "null pointer");
  DeviceGuard guard(e->device);
  void* chunk = nullptr;
  int rc;
  if ((rc = ensure_stage(e, 14, static_cast<size_t>(S) * 8, &chunk))) return rc;
  JrqCrcArgs a{};
  a.payload = payload;
  a.offsets = offsets;
  a.n = S;
  a.out = static_cast<uint64_t*>(chunk);
  a.stream_state = state;  // folded into the registers by crc64_finish_kernel
  return crc_dispatch(e, a, 0);
}

int jrq_crc64_stream_update(jrq_engine* e, uint64_t* state, const uint8_t* payload,
                            const uint64_t* offsets, uint32_t S) {
  if (!e) return JRQ_E_INVALID;
  if (S == 0) return JRQ_OK;
  if (!state || !payload || !offsets) return fail(e, JRQ_E_INVALID, "null pointer");
  DeviceGuard guard(e->device);
  int rc;
  if ((rc = check_monotone(e, offsets, S))) return rc;
  const uint64_t lo = offsets[0], hi = offsets[S];
  const uint8_t* dp;
  const uint64_t* doff;
  const uint64_t* dstate;
  if ((rc = stage_in(e, 10, payload + lo, hi - lo, &dp))) return rc;
  std::vector<uint64_t> rebased(offsets, offsets + S + 1);
  for (auto& o : rebased) o -= lo;
  if ((rc = stage_in(e, 11, rebased.data(), rebased.size(), &doff))) return rc;
  if ((rc = stage_in(e, 13, static_cast<const uint64_t*>(state), S, &dstate))) return rc;
  uint64_t* ds = const_cast<uint64_t*>(dstate);
  e->regs_hint = unaligned_bounds(offsets, S);
  rc = jrq_crc64_stream_update_dev(e, ds, dp, doff, S);
  e->regs_hint = 0;
  if (rc) return rc;
  JRQ_DOWN(e, state, ds, static_cast<size_t>(S) * 8);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

int jrq_logentry_checksum_batch_dev(jrq_engine* e, const uint8_t* type, const int64_t* index,
                                    const int64_t* term, const uint64_t* peer_xor,
                                    const uint8_t* payload, const uint64_t* offsets, uint32_t N,
                                    uint64_t* out, const uint64_t* expected, const uint8_t* has,
                                    uint8_t* corrupt_out) {
  if (!e) return JRQ_E_INVALID;
  if (N == 0) return JRQ_OK;
  if (!type || !index || !term || !payload || !offsets || !out)
    return fail(e, JRQ_E_INVALID, "null pointer");
  if ((expected == nullptr) != (corrupt_out == nullptr))
    return fail(e, JRQ_E_INVALID, "expected and corrupt_out go together");
  DeviceGuard guard(e->device);
  JrqCrcArgs a{};
  a.payload = payload;
  a.offsets = offsets;
  a.n = N;
  a.out = out;
  a.type = type;
  a.index = index;
  a.term = term;
  a.peer_xor = peer_xor;
  a.expected = expected;
  a.has = has;
  a.corrupt = corrupt_out;
  return crc_dispatch(e, a, 1);
}

int jrq_logentry_checksum_fixed_dev(jrq_engine* e, const uint8_t* type, const int64_t* index,
                                    const int64_t* term, const uint64_t* peer_xor,
                                    const uint8_t* payload, uint64_t entry_bytes, uint32_t N,
                                    uint64_t* out, const uint64_t* expected, const uint8_t* has,
                                    uint8_t* corrupt_out) {
  if (!e) return JRQ_E_INVALID;
  if (N == 0) return JRQ_OK;
  if (!type || !index || !term || !payload || !out)
    return fail(e, JRQ_E_INVALID, "null pointer");
  if ((expected == nullptr) != (corrupt_out == nullptr))
    return fail(e, JRQ_E_INVALID, "expected and corrupt_out go together");
  DeviceGuard guard(e->device);
  const uint32_t k = crc_fixed_k(e, payload, entry_bytes, N);
  if (k == 0) {
    const uint64_t* off;
    int rc;
    if ((rc = fixed_offsets(e, entry_bytes, N, &off))) return rc;
    return jrq_logentry_checksum_batch_dev(e, type, index, term, peer_xor, payload, off, N, out,
                                           expected, has, corrupt_out);
  }
  JrqCrcArgs a{};
  a.payload = payload;
  a.n = N;
  a.out = out;
  a.type = type;
  a.index = index;
  a.term = term;
  a.peer_xor = peer_xor;
  a.expected = expected;
  a.has = has;
  a.corrupt = corrupt_out;
  a.entry_bytes = entry_bytes;
  a.fixed_k = k;
  return crc_fixed_dispatch(e, a, 1);
}

int jrq_logentry_checksum_batch(jrq_engine* e, const uint8_t* type, const int64_t* index,
                                const int64_t* term, const uint64_t* peer_xor,
                                const uint8_t* payload, const uint64_t* offsets, uint32_t N,
                                uint64_t* out, const uint64_t* expected, const uint8_t* has,
                                uint8_t* corrupt_out) {
  if (!e) return JRQ_E_INVALID;
  if (N == 0) return JRQ_OK;
  if (!type || !index || !term || !payload || !offsets || !out)
    return fail(e, JRQ_E_INVALID, "null pointer");
  if ((expected == nullptr) != (corrupt_out == nullptr))
    return fail(e, JRQ_E_INVALID, "expected and corrupt_out go together");
  DeviceGuard guard(e->device);
  int rc;
  if ((rc = check_monotone(e, offsets, N))) return rc;
  const uint64_t lo = offsets[0], hi = offsets[N];
  const uint8_t *dp, *dt, *dh;
  const uint64_t *doff, *dpx, *dex;
  const int64_t *di, *dtm;
  if ((rc = stage_in(e, 10, payload + lo, hi - lo, &dp))) return rc;
  std::vector<uint64_t> rebased(offsets, offsets + N + 1);
  for (auto& o : rebased) o -= lo;
  if ((rc = stage_in(e, 11, rebased.data(), rebased.size(), &doff))) return rc;
  if ((rc = stage_in(e, 1, type, N, &dt))) return rc;
  if ((rc = stage_in(e, 2, index, N, &di))) return rc;
  if ((rc = stage_in(e, 3, term, N, &dtm))) return rc;
  if ((rc = stage_in(e, 4, peer_xor, N, &dpx))) return rc;
  if ((rc = stage_in(e, 5, expected, N, &dex))) return rc;
  if ((rc = stage_in(e, 6, has, N, &dh))) return rc;
  void *dout = nullptr, *dcor = nullptr;
  if ((rc = ensure_stage(e, 12, static_cast<size_t>(N) * 8, &dout))) return rc;
  if (corrupt_out && (rc = ensure_stage(e, 13, N, &dcor))) return rc;
  const uint64_t ul = uniform_length(offsets, N);
  if (crc_fixed_k(e, dp, ul, N)) {  // equal entries: the fixed-size kernel (one launch)
    rc = jrq_logentry_checksum_fixed_dev(e, dt, di, dtm, dpx, dp, ul, N, static_cast<uint64_t*>(dout),
                                         dex, dh, static_cast<uint8_t*>(dcor));
  } else {
    e->regs_hint = unaligned_bounds(offsets, N);
    rc = jrq_logentry_checksum_batch_dev(e, dt, di, dtm, dpx, dp, doff, N, static_cast<uint64_t*>(dout),
                                         dex, dh, static_cast<uint8_t*>(dcor));
    e->regs_hint = 0;
  }
  if (rc) return rc;
  JRQ_DOWN(e, out, dout, static_cast<size_t>(N) * 8);
  if (corrupt_out) JRQ_DOWN(e, corrupt_out, dcor, N);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

// --------------------------------------------------------------- lease -----

int jrq_lease_check_dev(jrq_engine* e, const int64_t* ts, uint64_t ld, uint32_t num_peers,
                        const uint64_t* conf, const uint8_t* self_slot, uint32_t G, int64_t now_ms,
                        int64_t lease_timeout_ms, uint8_t* ok_out, int64_t* lease_start,
                        uint16_t* dead_out) {
  if (!e) return JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (!ts || !conf || !self_slot || !ok_out || !lease_start || ld < G || num_peers == 0 ||
      num_peers > JRQ_MAX_PEERS)
    return fail(e, JRQ_E_INVALID, "bad lease batch");
  DeviceGuard guard(e->device);
  JrqLeaseArgs a{};
  a.last_rpc_ts = ts;
  a.ld = ld;
  a.conf = conf;
  a.self_slot = self_slot;
  a.now_ms = now_ms;
  a.lease_timeout_ms = lease_timeout_ms;
  a.num_peers = num_peers;
  a.G = G;
  a.ok = ok_out;
  a.lease_start = lease_start;
  a.dead = dead_out;
  JRQ_HIP(e, jrq_launch_lease(&a, e->num_cus, e->stream));
  return JRQ_OK;
}

int jrq_lease_check(jrq_engine* e, const int64_t* ts, uint64_t ld, uint32_t num_peers,
                    const uint64_t* conf, const uint8_t* self_slot, uint32_t G, int64_t now_ms,
                    int64_t lease_timeout_ms, uint8_t* ok_out, int64_t* lease_start,
                    uint16_t* dead_out) {
  if (!e) return JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (!ts || !conf || !self_slot || !ok_out || !lease_start || ld < G || num_peers == 0 ||
      num_peers > JRQ_MAX_PEERS)
    return fail(e, JRQ_E_INVALID, "bad lease batch");
  DeviceGuard guard(e->device);
  int rc;
  const int64_t* dts;
  const uint64_t* dconf;
  const uint8_t* dself;
  const int64_t* dlead;
  if ((rc = stage_in(e, 0, ts, (num_peers - 1) * ld + G, &dts))) return rc;
  if ((rc = stage_in(e, 1, conf, G, &dconf))) return rc;
  if ((rc = stage_in(e, 2, self_slot, G, &dself))) return rc;
  if ((rc = stage_in(e, 3, lease_start, G, &dlead))) return rc;
  void *dok, *ddead;
  if ((rc = ensure_stage(e, 8, G, &dok))) return rc;
  if ((rc = ensure_stage(e, 9, static_cast<size_t>(G) * 2, &ddead))) return rc;
  if ((rc = jrq_lease_check_dev(e, dts, ld, num_peers, dconf, dself, G, now_ms, lease_timeout_ms,
                                static_cast<uint8_t*>(dok), const_cast<int64_t*>(dlead),
                                static_cast<uint16_t*>(ddead))))
    return rc;
  JRQ_DOWN(e, ok_out, dok, G);
  JRQ_DOWN(e, lease_start, dlead, static_cast<size_t>(G) * 8);
  if (dead_out) JRQ_DOWN(e, dead_out, ddead, static_cast<size_t>(G) * 2);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

// ------------------------------------------------------------ ReadIndex -----

static_assert(JRQ_READINDEX_PENDING == jrq::kRiPending && JRQ_READINDEX_SUCCESS == jrq::kRiSuccess &&
                  JRQ_READINDEX_FAILURE == jrq::kRiFailure && JRQ_READINDEX_INVALID == jrq::kRiInvalid,
              "ReadIndex verdicts");

int jrq_readindex_quorum_dev(jrq_engine* e, const uint64_t* conf, const uint8_t* self_slot,
                             const uint64_t* order, const uint16_t* ok_mask, uint32_t num_peers,
                             uint32_t G, uint8_t* result_out) {
  if (!e) return JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (!conf || !self_slot || !order || !ok_mask || !result_out || num_peers == 0 ||
      num_peers > JRQ_MAX_PEERS)
    return fail(e, JRQ_E_INVALID, "bad ReadIndex batch");
  DeviceGuard guard(e->device);
  JrqReadIndexArgs a{};
  a.conf = conf;
  a.self_slot = self_slot;
  a.order = order;
  a.ok_mask = ok_mask;
  a.num_peers = num_peers;
  a.G = G;
  a.result = result_out;
  JRQ_HIP(e, jrq_launch_readindex(&a, e->num_cus, e->stream));
  return JRQ_OK;
}

int jrq_readindex_quorum(jrq_engine* e, const uint64_t* conf, const uint8_t* self_slot,
                         const uint64_t* order, const uint16_t* ok_mask, uint32_t num_peers,
                         uint32_t G, uint8_t* result_out) {
  if (!e) return JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (!conf || !self_slot || !order || !ok_mask || !result_out || num_peers == 0 ||
      num_peers > JRQ_MAX_PEERS)
    return fail(e, JRQ_E_INVALID, "bad ReadIndex batch");
  DeviceGuard guard(e->device);
  int rc;
  const uint64_t* dconf;
  const uint8_t* dself;
  const uint64_t* dord;
  const uint16_t* dok;
  if ((rc = stage_in(e, 0, conf, G, &dconf))) return rc;
  if ((rc = stage_in(e, 1, self_slot, G, &dself))) return rc;
  if ((rc = stage_in(e, 2, order, G, &dord))) return rc;
  if ((rc = stage_in(e, 3, ok_mask, G, &dok))) return rc;
  void* dres;
  if ((rc = ensure_stage(e, 8, G, &dres))) return rc;
  if ((rc = jrq_readindex_quorum_dev(e, dconf, dself, dord, dok, num_peers, G,
                                     static_cast<uint8_t*>(dres))))
    return rc;
  JRQ_DOWN(e, result_out, dres, G);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

// ------------------------------------------------------------ leader tick ---

int jrq_leader_tick_dev(jrq_engine* e, const int64_t* ts, uint64_t ld, uint32_t num_peers,
                        const uint64_t* conf, const uint8_t* self_slot, uint32_t G, int64_t now_ms,
                        int64_t lease_timeout_ms, uint8_t* ok_out, int64_t* lease_start,
                        uint16_t* dead_out, const uint64_t* order, const uint16_t* ok_mask,
                        uint8_t* ri_result) {
  if (!e) return JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (!ts || !conf || !self_slot || !ok_out || !lease_start || ld < G || num_peers == 0 ||
      num_peers > JRQ_MAX_PEERS)
    return fail(e, JRQ_E_INVALID, "bad leader-tick batch");
  if ((order != nullptr) != (ok_mask != nullptr) || (order != nullptr) != (ri_result != nullptr))
    return fail(e, JRQ_E_INVALID, "order, ok_mask and ri_result: all three or none");
  DeviceGuard guard(e->device);
  JrqLeaseArgs a{};
  a.last_rpc_ts = ts;
  a.ld = ld;
  a.conf = conf;
  a.self_slot = self_slot;
  a.now_ms = now_ms;
  a.lease_timeout_ms = lease_timeout_ms;
  a.num_peers = num_peers;
  a.G = G;
  a.ok = ok_out;
  a.lease_start = lease_start;
  a.dead = dead_out;
  a.order = order;
  a.ri_ok_mask = ok_mask;
  a.ri_result = ri_result;
  JRQ_HIP(e, jrq_launch_lease(&a, e->num_cus, e->stream));
  return JRQ_OK;
}

int jrq_leader_tick(jrq_engine* e, const int64_t* ts, uint64_t ld, uint32_t num_peers,
                    const uint64_t* conf, const uint8_t* self_slot, uint32_t G, int64_t now_ms,
                    int64_t lease_timeout_ms, uint8_t* ok_out, int64_t* lease_start,
                    uint16_t* dead_out, const uint64_t* order, const uint16_t* ok_mask,
                    uint8_t* ri_result) {
  if (!e) return JRQ_E_INVALID;
  if (G == 0) return JRQ_OK;
  if (!ts || !conf || !self_slot || !ok_out || !lease_start || ld < G || num_peers == 0 ||
      num_peers > JRQ_MAX_PEERS)
    return fail(e, JRQ_E_INVALID, "bad leader-tick batch");
  if ((order != nullptr) != (ok_mask != nullptr) || (order != nullptr) != (ri_result != nullptr))
    return fail(e, JRQ_E_INVALID, "order, ok_mask and ri_result: all three or none");
  DeviceGuard guard(e->device);
  int rc;
  const int64_t* dts;
  const uint64_t *dconf, *dord = nullptr;
  const uint8_t* dself;
  const int64_t* dlead;
  const uint16_t* dokm = nullptr;
  if ((rc = stage_in(e, 0, ts, (num_peers - 1) * ld + G, &dts))) return rc;
  if ((rc = stage_in(e, 1, conf, G, &dconf))) return rc;
  if ((rc = stage_in(e, 2, self_slot, G, &dself))) return rc;
  if ((rc = stage_in(e, 3, lease_start, G, &dlead))) return rc;
  if (order && (rc = stage_in(e, 4, order, G, &dord))) return rc;
  if (ok_mask && (rc = stage_in(e, 5, ok_mask, G, &dokm))) return rc;
  void *dok, *ddead, *dres = nullptr;
  if ((rc = ensure_stage(e, 8, G, &dok))) return rc;
  if ((rc = ensure_stage(e, 9, static_cast<size_t>(G) * 2, &ddead))) return rc;
  if (ri_result && (rc = ensure_stage(e, 10, G, &dres))) return rc;
  if ((rc = jrq_leader_tick_dev(e, dts, ld, num_peers, dconf, dself, G, now_ms, lease_timeout_ms,
                                static_cast<uint8_t*>(dok), const_cast<int64_t*>(dlead),
                                static_cast<uint16_t*>(ddead), dord, dokm,
                                static_cast<uint8_t*>(dres))))
    return rc;
  JRQ_DOWN(e, ok_out, dok, G);
  JRQ_DOWN(e, lease_start, dlead, static_cast<size_t>(G) * 8);
  if (dead_out) JRQ_DOWN(e, dead_out, ddead, static_cast<size_t>(G) * 2);
  if (ri_result) JRQ_DOWN(e, ri_result, dres, G);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

// ------------------------------------------------------- AppendEntries -----

int jrq_append_entries_verify_dev(jrq_engine* e, uint32_t R, const uint32_t* req_off,
                                  const int64_t* prev_log_index, uint32_t N, const int64_t* term,
                                  const uint8_t* type, const int64_t* data_len,
                                  const uint64_t* peer_xor, const uint64_t* checksum,
                                  const uint8_t* has_checksum, const uint8_t* data,
                                  uint64_t* checksum_out, uint8_t* corrupt_out,
                                  int32_t* first_corrupt_out) {
  if (!e) return JRQ_E_INVALID;
  if (R == 0) return JRQ_OK;
  if (!req_off || !prev_log_index || !first_corrupt_out)
    return fail(e, JRQ_E_INVALID, "null request array");
  if (N > 0 && (!term || !type || !data_len || !checksum || !data || !checksum_out || !corrupt_out))
    return fail(e, JRQ_E_INVALID, "null entry array");
  DeviceGuard guard(e->device);
  int rc;
  void *offs, *idx, *has, *tiles;
  const size_t ntiles = (static_cast<size_t>(N) + 4095) / 4096 + 1;
  if ((rc = ensure_stage(e, 16, (static_cast<size_t>(N) + 1) * 8, &offs))) return rc;
  if ((rc = ensure_stage(e, 17, static_cast<size_t>(N) * 8 + 8, &idx))) return rc;
  if ((rc = ensure_stage(e, 18, static_cast<size_t>(N) + 1, &has))) return rc;
  if ((rc = ensure_stage(e, 19, ntiles * 8, &tiles))) return rc;
  JrqAeArgs ae{};
  ae.r = R;
  ae.req_off = req_off;
  ae.prev_log_index = prev_log_index;
  ae.n = N;
  ae.type = type;
  ae.data_len = data_len;
  ae.has_checksum = has_checksum;
  ae.offsets = static_cast<uint64_t*>(offs);
  ae.index = static_cast<int64_t*>(idx);
  ae.has_eff = static_cast<uint8_t*>(has);
  ae.tile_sums = static_cast<uint64_t*>(tiles);
  ae.corrupt = corrupt_out;
  ae.first_corrupt = first_corrupt_out;
  if (N > 0) {
    JRQ_HIP(e, jrq_launch_ae_meta(&ae, e->stream));
    JrqCrcArgs a{};
    a.payload = data;
    a.offsets = ae.offsets;
    a.n = N;
    a.out = checksum_out;
    a.type = type;
    a.index = ae.index;
    a.term = term;
    a.peer_xor = peer_xor;
    a.expected = checksum;
    a.has = ae.has_eff;
    a.corrupt = corrupt_out;
    if ((rc = crc_dispatch(e, a, 1))) return rc;
  }
  JRQ_HIP(e, jrq_launch_ae_first_corrupt(&ae, e->stream));
  return JRQ_OK;
}

int jrq_append_entries_verify(jrq_engine* e, uint32_t R, const uint32_t* req_off,
                              const int64_t* prev_log_index, uint32_t N, const int64_t* term,
                              const uint8_t* type, const int64_t* data_len,
                              const uint64_t* peer_xor, const uint64_t* checksum,
                              const uint8_t* has_checksum, const uint8_t* data,
                              uint64_t* checksum_out, uint8_t* corrupt_out,
                              int32_t* first_corrupt_out) {
  if (!e) return JRQ_E_INVALID;
  if (R == 0) return JRQ_OK;
  if (!req_off || !prev_log_index || !first_corrupt_out)
    return fail(e, JRQ_E_INVALID, "null request array");
  if (req_off[0] != 0 || req_off[R] != N) return fail(e, JRQ_E_INVALID, "req_off must span [0, N]");
  if (N > 0 && (!term || !type || !data_len || !checksum || !checksum_out || !corrupt_out))
    return fail(e, JRQ_E_INVALID, "null entry array");
  DeviceGuard guard(e->device);
  uint64_t bytes = 0;  // consumed payload bytes (host arrays are readable here)
  for (uint32_t i = 0; i < N; ++i) {
    if (data_len[i] < 0) return fail(e, JRQ_E_INVALID, "negative data_len");
    if (type[i] != 0) bytes += static_cast<uint64_t>(data_len[i]);
  }
  if (bytes && !data) return fail(e, JRQ_E_INVALID, "null data");
  int rc;
  const uint32_t *dro;
  const int64_t *dpli, *dterm, *dlen;
  const uint8_t *dtype, *dhas, *ddata;
  const uint64_t *dpx, *dck;
  if ((rc = stage_in(e, 0, req_off, static_cast<size_t>(R) + 1, &dro))) return rc;
  if ((rc = stage_in(e, 1, prev_log_index, R, &dpli))) return rc;
  if ((rc = stage_in(e, 2, term, N, &dterm))) return rc;
  if ((rc = stage_in(e, 3, type, N, &dtype))) return rc;
  if ((rc = stage_in(e, 4, data_len, N, &dlen))) return rc;
  if ((rc = stage_in(e, 5, peer_xor, N, &dpx))) return rc;
  if ((rc = stage_in(e, 6, checksum, N, &dck))) return rc;
  if ((rc = stage_in(e, 7, has_checksum, N, &dhas))) return rc;
  if ((rc = stage_in(e, 10, data ? data : reinterpret_cast<const uint8_t*>(&bytes), bytes, &ddata)))
    return rc;
  void *dout, *dcor, *dfirst;
  if ((rc = ensure_stage(e, 12, static_cast<size_t>(N) * 8 + 8, &dout))) return rc;
  if ((rc = ensure_stage(e, 13, static_cast<size_t>(N) + 1, &dcor))) return rc;
  if ((rc = ensure_stage(e, 9, static_cast<size_t>(R) * 4, &dfirst))) return rc;
  if ((rc = jrq_append_entries_verify_dev(e, R, dro, dpli, N, dterm, dtype, dlen, dpx, dck, dhas,
                                          ddata, static_cast<uint64_t*>(dout),
                                          static_cast<uint8_t*>(dcor), static_cast<int32_t*>(dfirst))))
    return rc;
  if (N) {
    JRQ_DOWN(e, checksum_out, dout, static_cast<size_t>(N) * 8);
    JRQ_DOWN(e, corrupt_out, dcor, N);
  }
  JRQ_DOWN(e, first_corrupt_out, dfirst, static_cast<size_t>(R) * 4);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

// ------------------------------------------------------ commit fan-out -----

int jrq_commit_fanout_dev(jrq_engine* e, uint32_t G, const int64_t* prev_committed,
                          const int64_t* committed, const int64_t* last_applied,
                          int64_t* cq_first, int64_t* cq_size, int64_t* first_closure_out,
                          uint8_t* status_out, uint64_t* listed_out, uint32_t* num_listed_out) {
  if (!e) return JRQ_E_INVALID;
  if (!num_listed_out) return fail(e, JRQ_E_INVALID, "null num_listed_out");
  if (G > 0 && (!prev_committed || !committed || !last_applied || !cq_first || !cq_size ||
                !first_closure_out || !status_out || !listed_out))
    return fail(e, JRQ_E_INVALID, "null fan-out array");
  DeviceGuard guard(e->device);
  if (G == 0) {
    JRQ_HIP(e, hipMemsetAsync(num_listed_out, 0, 4, e->stream));
    return JRQ_OK;
  }
  JrqFanoutArgs a{};
  a.G = G;
  a.prev_committed = prev_committed;
  a.committed = committed;
  a.last_applied = last_applied;
  a.cq_first = cq_first;
  a.cq_size = cq_size;
  a.first_closure = first_closure_out;
  a.status = status_out;
  a.listed = listed_out;
  a.num_listed = num_listed_out;
  a.ctr = e->fan_ctr;
  JRQ_HIP(e, jrq_launch_fanout(&a, e->stream));
  return JRQ_OK;
}

int jrq_commit_fanout(jrq_engine* e, uint32_t G, const int64_t* prev_committed,
                      const int64_t* committed, const int64_t* last_applied, int64_t* cq_first,
                      int64_t* cq_size, int64_t* first_closure_out, uint8_t* status_out,
                      uint64_t* listed_out, uint32_t* num_listed_out) {
  if (!e) return JRQ_E_INVALID;
  if (!num_listed_out) return fail(e, JRQ_E_INVALID, "null num_listed_out");
  if (G == 0) {
    *num_listed_out = 0;
    return JRQ_OK;
  }
  if (!prev_committed || !committed || !last_applied || !cq_first || !cq_size ||
      !first_closure_out || !status_out || !listed_out)
    return fail(e, JRQ_E_INVALID, "null fan-out array");
  DeviceGuard guard(e->device);
  int rc;
  const int64_t *dprev, *dcom, *dla, *dcf0, *dcs0;
  if ((rc = stage_in(e, 0, prev_committed, G, &dprev))) return rc;
  if ((rc = stage_in(e, 1, committed, G, &dcom))) return rc;
  if ((rc = stage_in(e, 2, last_applied, G, &dla))) return rc;
  if ((rc = stage_in(e, 3, cq_first, G, &dcf0))) return rc;
  if ((rc = stage_in(e, 4, cq_size, G, &dcs0))) return rc;
  void *dfc, *dst, *dlist, *dnum;
  if ((rc = ensure_stage(e, 8, static_cast<size_t>(G) * 8, &dfc))) return rc;
  if ((rc = ensure_stage(e, 9, G, &dst))) return rc;
  const size_t words = (static_cast<size_t>(G) + 63) / 64;
  if ((rc = ensure_stage(e, 12, words * 8, &dlist))) return rc;
  if ((rc = ensure_stage(e, 13, 16, &dnum))) return rc;
  int64_t* dcf = const_cast<int64_t*>(dcf0);
  int64_t* dcs = const_cast<int64_t*>(dcs0);
  if ((rc = jrq_commit_fanout_dev(e, G, dprev, dcom, dla, dcf, dcs, static_cast<int64_t*>(dfc),
                                  static_cast<uint8_t*>(dst), static_cast<uint64_t*>(dlist),
                                  static_cast<uint32_t*>(dnum))))
    return rc;
  const size_t b8 = static_cast<size_t>(G) * 8;
  JRQ_DOWN(e, cq_first, dcf, b8);
  JRQ_DOWN(e, cq_size, dcs, b8);
  JRQ_DOWN(e, first_closure_out, dfc, b8);
  JRQ_DOWN(e, status_out, dst, G);
  JRQ_DOWN(e, num_listed_out, dnum, 4);
  JRQ_DOWN(e, listed_out, dlist, words * 8);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

// ------------------------------------------------------- V2 decode -----

int jrq_v2_decode_verify_dev(jrq_engine* e, const uint8_t* rec, const uint64_t* off, uint32_t N,
                             uint8_t* status, uint8_t* type, int64_t* index, int64_t* term,
                             uint64_t* stored, uint8_t* has_checksum, uint64_t* data_off,
                             uint64_t* data_len, uint32_t* peer_counts, uint64_t* computed,
                             uint8_t* corrupt) {
  if (!e) return JRQ_E_INVALID;
  if (N == 0) return JRQ_OK;
  if (N >= 0x7FFFFFFFu) return fail(e, JRQ_E_INVALID, "N too large");
  if (!rec || !off || !status || !type || !index || !term || !stored || !has_checksum ||
      !data_off || !data_len || !computed || !corrupt)
    return fail(e, JRQ_E_INVALID, "null V2 decode array");
  DeviceGuard guard(e->device);
  int rc;
  void *partial, *off2, *crc2;
  if ((rc = ensure_stage(e, 21, static_cast<size_t>(N) * 8, &partial))) return rc;
  if ((rc = ensure_stage(e, 22, (static_cast<size_t>(N) + 2) * 8, &off2))) return rc;
  if ((rc = ensure_stage(e, 23, (static_cast<size_t>(N) + 1) * 8, &crc2))) return rc;
  void *lens, *blk;  // per record: header / trailer lengths; per 256 records: parse summaries
  if ((rc = ensure_stage(e, 24, static_cast<size_t>(N) * 8, &lens))) return rc;
  if ((rc = ensure_stage(e, 25, (static_cast<size_t>(N) + 255) / 256 * 32, &blk))) return rc;
  JrqV2Args v{};
  v.rec = rec;
  v.off = off;
  v.n = N;
  v.slice = e->slice;
  v.xinv = e->xinv;
  v.status = status;
  v.type = type;
  v.index = index;
  v.term = term;
  v.stored = stored;
  v.has_checksum = has_checksum;
  v.data_off = data_off;
  v.data_len = data_len;
  v.peer_counts = peer_counts;
  v.computed = computed;
  v.corrupt = corrupt;
  v.partial = static_cast<uint64_t*>(partial);
  v.off2 = static_cast<uint64_t*>(off2);
  v.crc2 = static_cast<const uint64_t*>(crc2);
  v.lens = static_cast<uint64_t*>(lens);
  v.gate = e->v2_gate;
  v.blk = static_cast<uint64_t*>(blk);
  // (the fixed-size path hashes from the 128-B line of each data start: records 128-B aligned)
  v.lanes = (reinterpret_cast<uintptr_t>(rec) & 127u) ? ~0ull
                                                     : static_cast<uint64_t>(e->crc_grid) * jrq::kCrcFixedBlock;
  JRQ_HIP(e, jrq_launch_v2_parse(&v, e->stream));  // (its last block writes the gate)
  // every record with the same data length (the common case: fixed-size commands): the data
  // ranges alone, k lanes per record (crc64_fixed_kernel at the data starts), finished in place
  // (computed = partial ^ crc(data), corrupt); the gate words on the device pick this or the
  // segment walk below, each kernel of the other path returns at once
  {
    JrqCrcArgs f{};
    f.payload = rec;
    f.starts = v.data_off;
    f.gate = v.gate;
    f.n = N;
    f.out = computed;
    f.peer_xor = v.partial;  // type ^ crc(LogId) ^ peers, from v2_parse
    f.expected = stored;
    f.has = has_checksum;
    f.corrupt = corrupt;
    if ((rc = crc_fixed_dispatch(e, f, 1))) return rc;
  }
  // otherwise one range per record from its data start (the leading header first): one
  // streaming pass over the records, one entry boundary per record; v2_finish assembles each
  // range from its pieces and recovers the data CRCs.  Two launches, which return at once when
  // the fixed-size path took the batch: ~5 us each then (launch and kernel-boundary cost,
  // tools/trace_gaps.py), so the walk's own finish kernel was folded into v2_finish.  (On a
  // second stream beside the fixed-size kernel they still ran after it -- the rounds kernel's
  // 160 KiB of LDS waits for the fixed kernel's workgroups to leave -- and the call took 262
  // instead of 257 us.)
  JrqCrcArgs a{};
  a.gate = v.gate;
  a.payload = rec;
  a.offsets = v.off2;
  a.n = N + 1;
  a.out = static_cast<uint64_t*>(crc2);
  a.regs_slowpath = 1;  // an unaligned boundary per record
  a.no_finish = 1;
  if ((rc = crc_dispatch(e, a, 0))) return rc;  // (sets a.lanes and the scratch pointers)
  JRQ_HIP(e, jrq_launch_v2_finish(&v, &a, e->num_cus, e->stream));
  return JRQ_OK;
}

int jrq_v2_decode_verify(jrq_engine* e, const uint8_t* rec, const uint64_t* off, uint32_t N,
                         uint8_t* status, uint8_t* type, int64_t* index, int64_t* term,
                         uint64_t* stored, uint8_t* has_checksum, uint64_t* data_off,
                         uint64_t* data_len, uint32_t* peer_counts, uint64_t* computed,
                         uint8_t* corrupt) {
  if (!e) return JRQ_E_INVALID;
  if (N == 0) return JRQ_OK;
  if (!off || !status || !type || !index || !term || !stored || !has_checksum || !data_off ||
      !data_len || !computed || !corrupt)
    return fail(e, JRQ_E_INVALID, "null V2 decode array");
  int rc;
  if ((rc = check_monotone(e, off, N))) return rc;
  const uint64_t lo = off[0], hi = off[N];
  if (hi > lo && !rec) return fail(e, JRQ_E_INVALID, "null records");
  DeviceGuard guard(e->device);
  const uint8_t* drec;
  const uint64_t* doff;
  uint8_t dummy = 0;
  if ((rc = stage_in(e, 10, hi > lo ? rec + lo : &dummy, hi > lo ? hi - lo : 1, &drec))) return rc;
  std::vector<uint64_t> rebased(off, off + N + 1);
  for (auto& o : rebased) o -= lo;
  if ((rc = stage_in(e, 11, rebased.data(), rebased.size(), &doff))) return rc;
  const size_t n8 = static_cast<size_t>(N) * 8;
  void *dst, *dty, *didx, *dtm, *dsto, *dhas, *ddo, *ddl, *dpc, *dcmp, *dcor;
  if ((rc = ensure_stage(e, 0, N, &dst)) || (rc = ensure_stage(e, 1, N, &dty)) ||
      (rc = ensure_stage(e, 2, n8, &didx)) || (rc = ensure_stage(e, 3, n8, &dtm)) ||
      (rc = ensure_stage(e, 4, n8, &dsto)) || (rc = ensure_stage(e, 5, N, &dhas)) ||
      (rc = ensure_stage(e, 6, n8, &ddo)) || (rc = ensure_stage(e, 7, n8, &ddl)) ||
      (rc = ensure_stage(e, 8, static_cast<size_t>(N) * 4, &dpc)) ||
      (rc = ensure_stage(e, 9, n8, &dcmp)) || (rc = ensure_stage(e, 12, N, &dcor)))
    return rc;
  if ((rc = jrq_v2_decode_verify_dev(
           e, drec, doff, N, static_cast<uint8_t*>(dst), static_cast<uint8_t*>(dty),
           static_cast<int64_t*>(didx), static_cast<int64_t*>(dtm), static_cast<uint64_t*>(dsto),
           static_cast<uint8_t*>(dhas), static_cast<uint64_t*>(ddo), static_cast<uint64_t*>(ddl),
           peer_counts ? static_cast<uint32_t*>(dpc) : nullptr, static_cast<uint64_t*>(dcmp),
           static_cast<uint8_t*>(dcor))))
    return rc;
  JRQ_DOWN(e, status, dst, N);
  JRQ_DOWN(e, type, dty, N);
  JRQ_DOWN(e, index, didx, n8);
  JRQ_DOWN(e, term, dtm, n8);
  JRQ_DOWN(e, stored, dsto, n8);
  JRQ_DOWN(e, has_checksum, dhas, N);
  JRQ_DOWN(e, data_off, ddo, n8);
  JRQ_DOWN(e, data_len, ddl, n8);
  if (peer_counts)
    JRQ_DOWN(e, peer_counts, dpc, static_cast<size_t>(N) * 4);
  JRQ_DOWN(e, computed, dcmp, n8);
  JRQ_DOWN(e, corrupt, dcor, N);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  for (uint32_t i = 0; i < N; ++i) data_off[i] += lo;  // back to the caller's base
  return JRQ_OK;
}

// -------------------------------------------------- resident group table -----

struct jrq_table {
  jrq_engine* e = nullptr;
  void* mem = nullptr;        // every device array of the table, one allocation
  JrqTableArgs a{};           // device pointers (changed / n_changed / status set per epoch)
  DevBuf st_stage, rec_stage, changed_stage;  // staging of the host variants
  uint32_t* n_dev = nullptr;  // host-variant epoch: slice counts [slices], offsets [slices], total
  uint32_t* n_host = nullptr; // pinned: the total
  uint32_t slices = 0;        // JRQ_TABLE_SLICE-group slices of the changed list
  uint64_t stage_cap_s = 0, stage_cap_r = 0;  // jrq_table_stage: reserved capacity
  uint64_t staged_s = 0, staged_r = 0;        // headers / records staged since the last apply
  DevBuf ack_stage, seg_stage;                // order-free ack records (jrq_table_stage_acks)
  DevBuf fsm_stage;                           // jrq_table_fsm_update (host variant)
  uint64_t stage_cap_a = 0, staged_a = 0;    // records copied into ack_stage
  uint64_t ack_total = 0;                     // records of every staged segment
  uint32_t stage_cap_seg = 0;
  std::vector<uint32_t> seg_off;              // staged segments: first record (over all), stamp,
  std::vector<uint64_t> seg_stamp;            // where its records are (ack_stage or a region)
  std::vector<uint64_t> seg_ptr;
  uint64_t seg_last_n = 0;                    // the last segment's record count (merging)
  std::vector<void*> regions;                 // jrq_table_ack_region allocations
  std::mutex regions_mu;
  size_t state_bytes = 0;     // the rows at the start of mem (jrq_table_copy)
};

namespace {

static int table_check(jrq_table* t) {
  if (!t || !t->e) return JRQ_E_INVALID;
  return JRQ_OK;
}

static int stage_buf(jrq_engine* e, DevBuf& b, size_t bytes, void** out) {
  if (bytes == 0) bytes = 16;
  if (b.cap < bytes) {
    if (b.p) {
      JRQ_HIP(e, hipStreamSynchronize(e->stream));
      JRQ_HIP(e, hipFree(b.p));
      b.p = nullptr;
      b.cap = 0;
    }
    const size_t cap = bytes + bytes / 4;
    JRQ_HIP(e, hipMalloc(&b.p, cap));
    b.cap = cap;
  }
  *out = b.p;
  return JRQ_OK;
}

}  // namespace

jrq_table* jrq_table_create(jrq_engine* e, uint32_t G, uint32_t P, int* err) {
  auto set = [&](int c) {
    if (err) *err = c;
  };
  if (!e || G == 0 || G > JRQ_TABLE_MAX_GROUPS || P == 0 || P > JRQ_MAX_PEERS) {
    if (e) fail(e, JRQ_E_INVALID, "table: bad G %u or num_peers %u", G, P);
    set(JRQ_E_INVALID);
    return nullptr;
  }
  DeviceGuard guard(e->device);
  auto* t = new jrq_table();
  t->e = e;
  const uint64_t ld = (static_cast<uint64_t>(G) + 63) & ~63ull;  // pairs + 512-B rows
  // the state jrq_table_copy copies: the hot tiles (256 groups each: match[P] as 256-u32 rows,
  // pi, la, lc, conf as 256-word rows, JrqTableArgs), the cold rows xstart[3], xconf[3], the
  // flagged-entry slots flag_ent[waves][128][8] + flag_wcnt[waves] (u32); then the control word
  // `invalid`.  Epoch waves decide 128 groups (half a tile); the grid is whole workgroups of
  // kTableBlockWaves waves, and every wave of it reads its tile and its slots: tiles and slots
  // are allocated for the whole grid
  // (units of 128 groups, allocated for whole workgroups of two units per wave, which covers
  // the one-unit grid too)
  const uint64_t kUnitAlign = 2 * jrq::kTableBlockWaves;
  const uint64_t waves = ((G + jrq::kListSlice - 1) / jrq::kListSlice + kUnitAlign - 1) / kUnitAlign * kUnitAlign;
  const uint64_t tiles = (waves + 1) / 2;
  const uint64_t flag_words = waves * jrq::kFlagSlots * 8 + (waves + 1) / 2;
  const uint64_t ts = static_cast<uint64_t>(P) * (jrq::kTableSlice / 2) + 4 * jrq::kTableSlice;  // words per tile
  // + rstamp[ld], + fsm[3][ld] (lastAppliedIndex, ClosureQueue firstIndex and size)
  const uint64_t words = tiles * ts + ld * 2 * (jrq::kTableMaxRuns - 1) + flag_words + ld + 3 * ld;
  const size_t bytes = words * 8 + 64;
  t->slices = (G + JRQ_TABLE_SLICE - 1) / JRQ_TABLE_SLICE;
  if (hipMalloc(&t->mem, bytes) != hipSuccess || hipMemset(t->mem, 0, bytes) != hipSuccess ||
      hipMalloc(&t->n_dev, 4 * (2 * static_cast<size_t>(t->slices) + 1)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&t->n_host), 64, hipHostMallocDefault) != hipSuccess) {
    fail(e, JRQ_E_NOMEM, "table: allocation of %zu bytes failed", bytes);
    jrq_table_destroy(t);
    set(JRQ_E_NOMEM);
    return nullptr;
  }
  int64_t* w = static_cast<int64_t*>(t->mem);
  JrqTableArgs& a = t->a;
  a.match = reinterpret_cast<uint32_t*>(w);
  a.pi = w + (jrq::kTableSlice / 2) * P;
  a.la = a.pi + jrq::kTableSlice;
  a.lc = a.la + jrq::kTableSlice;
  a.conf = reinterpret_cast<uint64_t*>(a.lc + jrq::kTableSlice);
  a.ts = ts;
  a.xstart = w + tiles * ts;
  a.xconf = reinterpret_cast<uint64_t*>(a.xstart + ld * (jrq::kTableMaxRuns - 1));
  a.flag_ent = reinterpret_cast<uint64_t*>(a.xconf + ld * (jrq::kTableMaxRuns - 1));
  a.flag_wcnt = reinterpret_cast<uint32_t*>(a.flag_ent + waves * jrq::kFlagSlots * 8);
  a.rstamp = reinterpret_cast<uint64_t*>(a.flag_ent + waves * jrq::kFlagSlots * 8 + (waves + 1) / 2);
  a.fsm = reinterpret_cast<int64_t*>(a.rstamp + ld);
  a.invalid = reinterpret_cast<uint32_t*>(w + words);
  t->state_bytes = words * 8;
  a.ld = ld;
  a.G = G;
  a.P = P;
  set(JRQ_OK);
  return t;
}

void jrq_table_destroy(jrq_table* t) {
  if (!t) return;
  if (t->e) {
    DeviceGuard guard(t->e->device);
    (void)hipStreamSynchronize(t->e->stream);
    for (DevBuf* b : {&t->st_stage, &t->rec_stage, &t->changed_stage, &t->ack_stage, &t->seg_stage, &t->fsm_stage})
      if (b->p) (void)hipFree(b->p);
    for (void* r : t->regions) (void)hipFree(r);
    if (t->mem) (void)hipFree(t->mem);
    if (t->n_dev) (void)hipFree(t->n_dev);
    if (t->n_host) (void)hipHostFree(t->n_host);
  }
  delete t;
}

int jrq_table_update_dev(jrq_table* t, const jrq_group_state* states, uint32_t n_states,
                         const uint64_t* recs, uint32_t n_recs) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if ((n_states && !states) || (n_recs && !recs)) return fail(e, JRQ_E_INVALID, "null update array");
  DeviceGuard guard(e->device);
  JRQ_HIP(e, jrq_launch_table_update(&t->a, reinterpret_cast<const JrqGroupState*>(states),
                                     n_states, recs, n_recs, e->stream));
  return JRQ_OK;
}

int jrq_table_update(jrq_table* t, const jrq_group_state* states, uint32_t n_states,
                     const uint64_t* recs, uint32_t n_recs) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if ((n_states && !states) || (n_recs && !recs)) return fail(e, JRQ_E_INVALID, "null update array");
  // no host pass over the records (it would cost as much as their PCIe transfer): the
  // kernels skip and count invalid ones, reported by jrq_table_check
  DeviceGuard guard(e->device);
  int rc;
  void *ds = nullptr, *dr = nullptr;
  if (n_states) {
    if ((rc = stage_buf(e, t->st_stage, static_cast<size_t>(n_states) * sizeof(jrq_group_state), &ds))) return rc;
    if ((rc = upload_any(e, ds, states, static_cast<size_t>(n_states) * sizeof(jrq_group_state)))) return rc;
  }
  if (n_recs) {
    if ((rc = stage_buf(e, t->rec_stage, static_cast<size_t>(n_recs) * 8, &dr))) return rc;
    if ((rc = upload_any(e, dr, recs, static_cast<size_t>(n_recs) * 8))) return rc;
  }
  return jrq_table_update_dev(t, static_cast<const jrq_group_state*>(ds), n_states,
                              static_cast<const uint64_t*>(dr), n_recs);
}

int jrq_table_update_gather(jrq_table* t, uint32_t parts, const jrq_group_state* const* states,
                            const uint32_t* n_states, const uint64_t* const* recs,
                            const uint32_t* n_recs) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if (parts && (!states || !n_states || !recs || !n_recs)) return fail(e, JRQ_E_INVALID, "null part arrays");
  uint64_t ns = 0, nr = 0;
  for (uint32_t i = 0; i < parts; ++i) {
    if ((n_states[i] && !states[i]) || (n_recs[i] && !recs[i])) return fail(e, JRQ_E_INVALID, "null part %u", i);
    ns += n_states[i];
    nr += n_recs[i];
  }
  if (ns > UINT32_MAX || nr > UINT32_MAX) return fail(e, JRQ_E_INVALID, "update larger than 2^32 items");
  DeviceGuard guard(e->device);
  int rc;
  void *ds = nullptr, *dr = nullptr;
  if (ns && (rc = stage_buf(e, t->st_stage, ns * sizeof(jrq_group_state), &ds))) return rc;
  if (nr && (rc = stage_buf(e, t->rec_stage, nr * 8, &dr))) return rc;
  uint64_t os = 0, orr = 0;
  for (uint32_t i = 0; i < parts; ++i) {  // the parts back to back: headers, then records
    if (n_states[i] && (rc = upload_any(e, static_cast<jrq_group_state*>(ds) + os, states[i],
                                        static_cast<size_t>(n_states[i]) * sizeof(jrq_group_state))))
      return rc;
    if (n_recs[i] && (rc = upload_any(e, static_cast<uint64_t*>(dr) + orr, recs[i],
                                      static_cast<size_t>(n_recs[i]) * 8)))
      return rc;
    os += n_states[i];
    orr += n_recs[i];
  }
  return jrq_table_update_dev(t, static_cast<const jrq_group_state*>(ds), static_cast<uint32_t>(ns),
                              static_cast<const uint64_t*>(dr), static_cast<uint32_t>(nr));
}

int jrq_table_stage_reserve(jrq_table* t, uint32_t max_states, uint32_t max_recs) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  t->staged_s = t->staged_r = 0;  // parts staged and never applied (a failed flush) are dropped
  DeviceGuard guard(e->device);
  int rc;
  void* p = nullptr;
  if ((rc = stage_buf(e, t->st_stage, static_cast<size_t>(max_states) * sizeof(jrq_group_state), &p))) return rc;
  if ((rc = stage_buf(e, t->rec_stage, static_cast<size_t>(max_recs) * 8, &p))) return rc;
  t->stage_cap_s = t->st_stage.cap / sizeof(jrq_group_state);
  t->stage_cap_r = t->rec_stage.cap / 8;
  return JRQ_OK;
}

int jrq_table_stage(jrq_table* t, const jrq_group_state* states, uint32_t n_states,
                    const uint64_t* recs, uint32_t n_recs) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if ((n_states && !states) || (n_recs && !recs)) return fail(e, JRQ_E_INVALID, "null update array");
  if (t->staged_s + n_states > t->stage_cap_s || t->staged_r + n_recs > t->stage_cap_r)
    return fail(e, JRQ_E_STATE, "table: staging beyond jrq_table_stage_reserve");
  DeviceGuard guard(e->device);
  int rc;
  if (n_states && (rc = upload_any(e, static_cast<jrq_group_state*>(t->st_stage.p) + t->staged_s, states,
                                   static_cast<size_t>(n_states) * sizeof(jrq_group_state))))
    return rc;
  if (n_recs && (rc = upload_any(e, static_cast<uint64_t*>(t->rec_stage.p) + t->staged_r, recs,
                                 static_cast<size_t>(n_recs) * 8)))
    return rc;
  t->staged_s += n_states;
  t->staged_r += n_recs;
  return JRQ_OK;
}

int jrq_table_stage_apply(jrq_table* t) {
  if (table_check(t)) return JRQ_E_INVALID;
  const uint64_t ns = t->staged_s, nr = t->staged_r, na = t->ack_total;
  t->staged_s = t->staged_r = t->staged_a = t->ack_total = 0;
  int rc;
  if ((ns || nr) &&
      (rc = jrq_table_update_dev(t, static_cast<const jrq_group_state*>(t->st_stage.p), static_cast<uint32_t>(ns),
                                 static_cast<const uint64_t*>(t->rec_stage.p), static_cast<uint32_t>(nr))))
    return rc;
  if (na) {  // the ack segments' stamps, places and starts, then one launch over every record
    jrq_engine* e = t->e;
    DeviceGuard guard(e->device);
    const uint32_t nseg = static_cast<uint32_t>(t->seg_off.size());
    uint64_t* ds = static_cast<uint64_t*>(t->seg_stage.p);
    uint64_t* dp = ds + t->stage_cap_seg;
    uint32_t* doff = reinterpret_cast<uint32_t*>(dp + t->stage_cap_seg);
    if ((rc = upload_any(e, ds, t->seg_stamp.data(), nseg * 8))) return rc;
    if ((rc = upload_any(e, dp, t->seg_ptr.data(), nseg * 8))) return rc;
    if ((rc = upload_any(e, doff, t->seg_off.data(), nseg * 4))) return rc;
    JRQ_HIP(e, jrq_launch_table_acks(&t->a, reinterpret_cast<const uint64_t* const*>(dp), static_cast<uint32_t>(na),
                                     doff, ds, nseg, e->stream));
  }
  t->seg_off.clear();
  t->seg_stamp.clear();
  t->seg_ptr.clear();
  return JRQ_OK;
}

namespace {
// One staged segment of order-free records at device address p: merged into the last one when it
// has the same stamp and continues it in memory.
int add_ack_segment(jrq_table* t, uint64_t stamp, const uint64_t* p, uint32_t n) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  if (!t->seg_stamp.empty() && t->seg_stamp.back() == stamp && t->seg_ptr.back() + 8 * t->seg_last_n == a) {
    t->seg_last_n += n;
  } else {
    if (t->seg_off.size() + 1 > t->stage_cap_seg)
      return fail(t->e, JRQ_E_STATE, "table: ack segments beyond jrq_table_stage_reserve_acks");
    if (t->ack_total + n > 0xFFFFFFFFull) return fail(t->e, JRQ_E_STATE, "table: more than 2^32 ack records");
    t->seg_off.push_back(static_cast<uint32_t>(t->ack_total));
    t->seg_stamp.push_back(stamp);
    t->seg_ptr.push_back(a);
    t->seg_last_n = n;
  }
  t->ack_total += n;
  return JRQ_OK;
}
}  // namespace

int jrq_table_stage_reserve_acks(jrq_table* t, uint32_t max_acks, uint32_t max_segments) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  t->staged_a = t->ack_total = 0;  // acks staged and never applied (a failed flush) are dropped
  t->seg_off.clear();
  t->seg_stamp.clear();
  t->seg_ptr.clear();
  if (max_segments == 0) max_segments = 1;
  DeviceGuard guard(e->device);
  int rc;
  void* p = nullptr;
  if ((rc = stage_buf(e, t->ack_stage, static_cast<size_t>(max_acks) * 8, &p))) return rc;
  if ((rc = stage_buf(e, t->seg_stage, static_cast<size_t>(max_segments) * 20, &p))) return rc;
  t->stage_cap_a = t->ack_stage.cap / 8;
  t->stage_cap_seg = static_cast<uint32_t>(t->seg_stage.cap / 20);
  return JRQ_OK;
}

int jrq_table_stage_acks(jrq_table* t, uint64_t stamp, const uint64_t* acks, uint32_t n) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if (n && !acks) return fail(e, JRQ_E_INVALID, "null ack array");
  if (n == 0) return JRQ_OK;
  if (t->staged_a + n > t->stage_cap_a)
    return fail(e, JRQ_E_STATE, "table: ack staging beyond jrq_table_stage_reserve_acks");
  DeviceGuard guard(e->device);
  int rc;
  uint64_t* dst = static_cast<uint64_t*>(t->ack_stage.p) + t->staged_a;
  if ((rc = add_ack_segment(t, stamp, dst, n))) return rc;
  if ((rc = upload_any(e, dst, acks, static_cast<size_t>(n) * 8))) return rc;
  t->staged_a += n;
  return JRQ_OK;
}

int jrq_table_stage_acks_dev(jrq_table* t, uint64_t stamp, const uint64_t* acks_dev, uint32_t n) {
  if (table_check(t)) return JRQ_E_INVALID;
  if (n && !acks_dev) return fail(t->e, JRQ_E_INVALID, "null ack array");
  if (n == 0) return JRQ_OK;
  return add_ack_segment(t, stamp, acks_dev, n);
}

int jrq_table_ack_region(jrq_table* t, uint64_t capacity, uint64_t** region_out) {
  if (table_check(t)) return JRQ_E_INVALID;
  if (!region_out || capacity == 0) return fail(t->e, JRQ_E_INVALID, "ack region: null output or zero capacity");
  DeviceGuard guard(t->e->device);
  void* p = nullptr;
  if (hipMalloc(&p, capacity * 8) != hipSuccess) {
    (void)hipGetLastError();
    return fail(t->e, JRQ_E_NOMEM, "ack region of %llu records", static_cast<unsigned long long>(capacity));
  }
  {
    std::lock_guard<std::mutex> l(t->regions_mu);
    t->regions.push_back(p);
  }
  *region_out = static_cast<uint64_t*>(p);
  return JRQ_OK;
}

int jrq_table_ack_region_free(jrq_table* t, uint64_t* region) {
  if (table_check(t)) return JRQ_E_INVALID;
  {
    std::lock_guard<std::mutex> l(t->regions_mu);
    auto it = std::find(t->regions.begin(), t->regions.end(), static_cast<void*>(region));
    if (it == t->regions.end()) return fail(t->e, JRQ_E_INVALID, "not an ack region of this table");
    t->regions.erase(it);
  }
  DeviceGuard guard(t->e->device);
  JRQ_HIP(t->e, hipStreamSynchronize(t->e->stream));  // (copies into it or reads of it may be queued)
  JRQ_HIP(t->e, hipFree(region));
  return JRQ_OK;
}

int jrq_table_ack_push(jrq_table* t, uint64_t* region_dst, const uint64_t* host_src, uint32_t n) {
  // callable from any thread, concurrently with the table's other calls: it only queues a copy
  // on the engine's stream, and reports errors by code alone (no shared error text)
  if (!t || !t->e || (n && (!region_dst || !host_src))) return JRQ_E_INVALID;
  if (n == 0) return JRQ_OK;
  if (!t->e->upload_pageable && !host_pinned(host_src)) return JRQ_E_INVALID;
  DeviceGuard guard(t->e->device);
  if (hipMemcpyAsync(region_dst, host_src, static_cast<size_t>(n) * 8, hipMemcpyHostToDevice, t->e->stream) !=
      hipSuccess) {
    (void)hipGetLastError();
    return JRQ_E_HIP;
  }
  return JRQ_OK;
}

int jrq_table_epoch_dev(jrq_table* t, uint64_t* changed_out, uint32_t* n_changed, uint8_t* status_out) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if (!changed_out || !n_changed) return fail(e, JRQ_E_INVALID, "null changed output");
  DeviceGuard guard(e->device);
  JrqTableArgs a = t->a;
  a.changed = changed_out;
  a.n_changed = n_changed;
  a.status = status_out;
  JRQ_HIP(e, jrq_launch_table_epoch(&a, e->stream));
  return JRQ_OK;
}

int jrq_table_epoch(jrq_table* t, uint64_t* changed_out, uint32_t* n_changed, uint8_t* status_out) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if (!changed_out || !n_changed) return fail(e, JRQ_E_INVALID, "null changed output");
  DeviceGuard guard(e->device);
  const uint32_t G = t->a.G;
  const size_t cap = static_cast<size_t>(t->slices) * JRQ_TABLE_SLICE;
  int rc;
  void* dch = nullptr;
  // staging: the slices, the gathered list, the status bytes
  if ((rc = stage_buf(e, t->changed_stage, 2 * cap * 8 + G, &dch))) return rc;
  uint64_t* slices = static_cast<uint64_t*>(dch);
  uint64_t* list = slices + cap;
  uint8_t* dst = status_out ? reinterpret_cast<uint8_t*>(list + cap) : nullptr;
  if ((rc = jrq_table_epoch_dev(t, slices, t->n_dev, dst))) return rc;
  // the slices back to back on the device, then only the entries cross PCIe
  uint32_t* off = t->n_dev + t->slices;
  uint32_t* total = off + t->slices;
  JRQ_HIP(e, jrq_launch_table_list_gather(slices, t->n_dev, t->slices, off, total, list, e->stream));
  JRQ_DOWN(e, t->n_host, total, 4);
  if (status_out) JRQ_DOWN(e, status_out, dst, G);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  const uint32_t n = t->n_host[0];
  if (n > G) return fail(e, JRQ_E_STATE, "table list overflow (%u entries)", n);
  if (n) {
    JRQ_DOWN(e, changed_out, list, static_cast<size_t>(n) * 8);
    JRQ_HIP(e, hipStreamSynchronize(e->stream));
  }
  *n_changed = n;
  return JRQ_OK;
}

int jrq_table_fsm_update_dev(jrq_table* t, const uint32_t* groups_dev, const int64_t* last_applied_dev,
                             const int64_t* cq_first_dev, const int64_t* cq_size_dev, uint32_t n) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if (n && (!groups_dev || !last_applied_dev || !cq_first_dev || !cq_size_dev))
    return fail(e, JRQ_E_INVALID, "null fsm update array");
  DeviceGuard guard(e->device);
  JRQ_HIP(e, jrq_launch_table_fsm(&t->a, groups_dev, last_applied_dev, cq_first_dev, cq_size_dev, n, e->stream));
  return JRQ_OK;
}

int jrq_table_fsm_update(jrq_table* t, const uint32_t* groups, const int64_t* last_applied,
                         const int64_t* cq_first, const int64_t* cq_size, uint32_t n) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if (n && (!groups || !last_applied || !cq_first || !cq_size)) return fail(e, JRQ_E_INVALID, "null fsm update array");
  if (n == 0) return JRQ_OK;
  DeviceGuard guard(e->device);
  // one staging block: the three int64 arrays, then the group ids
  void* d = nullptr;
  int rc;
  if ((rc = stage_buf(e, t->fsm_stage, static_cast<size_t>(n) * 28, &d))) return rc;
  int64_t* da = static_cast<int64_t*>(d);
  uint32_t* dg = reinterpret_cast<uint32_t*>(da + 3ull * n);
  if ((rc = upload_any(e, da, last_applied, static_cast<size_t>(n) * 8)) ||
      (rc = upload_any(e, da + n, cq_first, static_cast<size_t>(n) * 8)) ||
      (rc = upload_any(e, da + 2ull * n, cq_size, static_cast<size_t>(n) * 8)) ||
      (rc = upload_any(e, dg, groups, static_cast<size_t>(n) * 4)))
    return rc;
  return jrq_table_fsm_update_dev(t, dg, da, da + n, da + 2ull * n, n);
}

int jrq_table_fsm_read(jrq_table* t, int64_t* last_applied, int64_t* cq_first, int64_t* cq_size) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  DeviceGuard guard(e->device);
  const size_t G = t->a.G;
  if (last_applied) JRQ_DOWN(e, last_applied, t->a.fsm, G * 8);
  if (cq_first) JRQ_DOWN(e, cq_first, t->a.fsm + t->a.ld, G * 8);
  if (cq_size) JRQ_DOWN(e, cq_size, t->a.fsm + 2 * t->a.ld, G * 8);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  return JRQ_OK;
}

int jrq_table_epoch_fanout_dev(jrq_table* t, uint64_t* slices_out, uint32_t* n_changed_out,
                               int64_t* fan_first_out, uint8_t* fan_status_out) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if (!slices_out || !n_changed_out || !fan_first_out || !fan_status_out)
    return fail(e, JRQ_E_INVALID, "null fan-out epoch output");
  DeviceGuard guard(e->device);
  JrqTableArgs a = t->a;
  a.changed = slices_out;
  a.n_changed = n_changed_out;
  a.status = nullptr;
  a.fan_first = fan_first_out;
  a.fan_status = fan_status_out;
  JRQ_HIP(e, jrq_launch_table_epoch(&a, e->stream));
  return JRQ_OK;
}

int jrq_table_epoch_fanout(jrq_table* t, uint64_t* changed_out, uint32_t* n_changed, int64_t* fan_first_out,
                           uint8_t* fan_status_out) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if (!changed_out || !n_changed || !fan_first_out || !fan_status_out)
    return fail(e, JRQ_E_INVALID, "null fan-out epoch output");
  DeviceGuard guard(e->device);
  const uint32_t S = t->slices;
  const size_t cap = static_cast<size_t>(S) * JRQ_TABLE_SLICE;
  int rc;
  void* dch = nullptr;
  // staging: the slices and their gathered list, the slice-shaped fan results and their gathered
  // copies (first closures, then statuses)
  if ((rc = stage_buf(e, t->changed_stage, 2 * cap * 8 + 2 * cap * 8 + 2 * cap, &dch))) return rc;
  uint64_t* slices = static_cast<uint64_t*>(dch);
  uint64_t* list = slices + cap;
  int64_t* ff = reinterpret_cast<int64_t*>(list + cap);
  int64_t* lf = ff + cap;
  uint8_t* fs = reinterpret_cast<uint8_t*>(lf + cap);
  uint8_t* ls = fs + cap;
  if ((rc = jrq_table_epoch_fanout_dev(t, slices, t->n_dev, ff, fs))) return rc;
  uint32_t* off = t->n_dev + S;
  uint32_t* total = off + S;
  JRQ_HIP(e, jrq_launch_table_list_gather(slices, t->n_dev, S, off, total, list, e->stream));
  JRQ_HIP(e, jrq_launch_table_fan_gather(ff, fs, t->n_dev, off, S, lf, ls, e->stream));
  JRQ_DOWN(e, t->n_host, total, 4);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  const uint32_t n = t->n_host[0];
  if (n > t->a.G) return fail(e, JRQ_E_STATE, "table list overflow (%u entries)", n);
  if (n) {
    JRQ_DOWN(e, changed_out, list, static_cast<size_t>(n) * 8);
    JRQ_DOWN(e, fan_first_out, lf, static_cast<size_t>(n) * 8);
    JRQ_DOWN(e, fan_status_out, ls, n);
    JRQ_HIP(e, hipStreamSynchronize(e->stream));
  }
  *n_changed = n;
  return JRQ_OK;
}

uint32_t jrq_table_slices(const jrq_table* t) { return t ? t->slices : 0; }

int jrq_table_committed_dev(jrq_table* t, int64_t* out_dev) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  if (!out_dev) return fail(e, JRQ_E_INVALID, "null committed output");
  DeviceGuard guard(e->device);
  const size_t G = t->a.G, full = G / jrq::kTableSlice, rest = G % jrq::kTableSlice;
  const size_t tb = jrq::kTableSlice * 8;  // the lc rows, tile by tile (lastCommitted is never
                                            // encoded: only pendingIndex follows it)
  if (full)
    JRQ_HIP(e, hipMemcpy2DAsync(out_dev, tb, t->a.lc, t->a.ts * 8, tb, full, hipMemcpyDeviceToDevice, e->stream));
  if (rest)
    JRQ_HIP(e, hipMemcpyAsync(out_dev + full * jrq::kTableSlice, t->a.lc + full * t->a.ts, rest * 8,
                              hipMemcpyDeviceToDevice, e->stream));
  return JRQ_OK;
}

int jrq_table_read(jrq_table* t, int64_t* pending_index, int64_t* last_appended,
                   int64_t* last_committed, int64_t* match) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  DeviceGuard guard(e->device);
  const size_t G = t->a.G;
  const size_t tiles = (G + jrq::kTableSlice - 1) / jrq::kTableSlice;
  const size_t rb = static_cast<size_t>(t->a.P) * jrq::kTableSlice * 4;  // a tile's u32 match rows
  // de-tiled on the device into staging (one 2-D copy per field: the whole tiles, 256 words
  // each, tile stride apart; then the last partial tile), then one download of it all
  void* stage = nullptr;
  int rc;
  if ((rc = ensure_stage(e, 20, 3 * G * 8 + (match ? tiles * rb : 0), &stage))) return rc;
  int64_t* d_lc = static_cast<int64_t*>(stage);
  int64_t* d_pi = d_lc + G;
  int64_t* d_la = d_pi + G;
  uint32_t* d_mw = reinterpret_cast<uint32_t*>(d_la + G);
  auto field = [&](int64_t* dst, const int64_t* row) -> hipError_t {
    const size_t full = G / jrq::kTableSlice, rest = G % jrq::kTableSlice;
    const size_t tb = jrq::kTableSlice * 8;
    hipError_t r = hipSuccess;
    if (full) r = hipMemcpy2DAsync(dst, tb, row, t->a.ts * 8, tb, full, hipMemcpyDeviceToDevice, e->stream);
    if (r == hipSuccess && rest)
      r = hipMemcpyAsync(dst + full * jrq::kTableSlice, row + full * t->a.ts, rest * 8,
                         hipMemcpyDeviceToDevice, e->stream);
    return r;
  };
  JRQ_HIP(e, field(d_lc, t->a.lc));
  JRQ_HIP(e, field(d_pi, t->a.pi));
  JRQ_HIP(e, field(d_la, t->a.la));
  if (match)  // the u32 match words: every tile's P rows (P KiB at the tile's start)
    JRQ_HIP(e, hipMemcpy2DAsync(d_mw, rb, t->a.match, t->a.ts * 8, rb, tiles, hipMemcpyDeviceToDevice,
                                e->stream));
  std::vector<int64_t> host(3 * G);
  std::vector<uint32_t> mw(match ? tiles * rb / 4 : 0);
  JRQ_DOWN(e, host.data(), stage, 3 * G * 8);
  if (match) JRQ_DOWN(e, mw.data(), d_mw, tiles * rb);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  const int64_t* lc = host.data();
  int64_t* pw = host.data() + G;
  for (size_t g = 0; g < G; ++g)
    if (pw[g] == JRQ_PI_FOLLOWS_LC) pw[g] = lc[g] + 1;
  if (match)  // absolute: the group's match base + its word (group order within the tile)
    for (size_t g = 0; g < G; ++g) {
      const int64_t b = jrq::mbase(pw[g]);
      const uint32_t* row = mw.data() + (g / jrq::kTableSlice) * t->a.P * jrq::kTableSlice;
      for (uint32_t p = 0; p < t->a.P; ++p)
        match[p * G + g] = b + static_cast<int64_t>(row[p * jrq::kTableSlice + g % jrq::kTableSlice]);
    }
  if (pending_index) std::memcpy(pending_index, pw, G * 8);
  if (last_committed) std::memcpy(last_committed, lc, G * 8);
  if (last_appended) std::memcpy(last_appended, host.data() + 2 * G, G * 8);
  return JRQ_OK;
}

int jrq_table_check(jrq_table* t) {
  if (table_check(t)) return JRQ_E_INVALID;
  jrq_engine* e = t->e;
  DeviceGuard guard(e->device);
  JRQ_DOWN(e, t->n_host + 1, t->a.invalid, 4);
  JRQ_HIP(e, hipMemsetAsync(t->a.invalid, 0, 4, e->stream));
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  if (t->n_host[1])
    return fail(e, JRQ_E_INVALID, "%u group headers / records skipped: group >= G, field or num_runs out of range",
                t->n_host[1]);
  return JRQ_OK;
}

int jrq_table_copy(jrq_table* dst, const jrq_table* src) {
  if (table_check(dst) || !src || !src->e) return JRQ_E_INVALID;
  jrq_engine* e = dst->e;
  if (src->a.G != dst->a.G || src->a.P != dst->a.P || src->a.ld != dst->a.ld)
    return fail(e, JRQ_E_INVALID, "table shapes differ");
  DeviceGuard guard(e->device);
  JRQ_HIP(e, hipMemcpyAsync(dst->mem, src->mem, dst->state_bytes, hipMemcpyDeviceToDevice, e->stream));
  return JRQ_OK;
}

int jrq_table_view_get(jrq_table* t, jrq_table_view* v) {
  if (table_check(t) || !v) return JRQ_E_INVALID;
  v->match = t->a.match;
  v->pending_index = t->a.pi;
  v->last_appended = t->a.la;
  v->last_committed = t->a.lc;
  v->conf = t->a.conf;
  v->ld = t->a.ld;
  v->tile_groups = jrq::kTableSlice;
  v->tile_stride = t->a.ts;
  v->G = t->a.G;
  v->num_peers = t->a.P;
  return JRQ_OK;
}

// ---------------------------------------------------------------- RCCL -----

int jrq_rccl_get_unique_id(uint8_t id_out[128]) {
  if (!id_out) return JRQ_E_INVALID;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return JRQ_E_RCCL;
  static_assert(sizeof(id.internal) == 128, "ncclUniqueId is 128 bytes");
  std::memcpy(id_out, id.internal, 128);
  return JRQ_OK;
}

int jrq_rccl_init(jrq_engine* e, int nranks, int rank, const uint8_t id_in[128]) {
  if (!e || !id_in || nranks <= 0 || rank < 0 || rank >= nranks) return JRQ_E_INVALID;
  DeviceGuard guard(e->device);
  ncclUniqueId id;
  std::memcpy(id.internal, id_in, 128);
  if (e->comm) {
    (void)ncclCommDestroy(e->comm);
    e->comm = nullptr;
  }
  ncclResult_t r = ncclCommInitRank(&e->comm, nranks, id, rank);
  if (r != ncclSuccess) return fail(e, JRQ_E_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
  e->nranks = nranks;
  e->rank = rank;
  return JRQ_OK;
}

int jrq_rccl_nranks(jrq_engine* e) {
  if (!e) return JRQ_E_INVALID;
  if (!e->comm) return 0;
  int n = 0;
  ncclResult_t r = ncclCommCount(e->comm, &n);
  if (r != ncclSuccess) return fail(e, JRQ_E_RCCL, "ncclCommCount: %s", ncclGetErrorString(r));
  return n;
}

int jrq_publish_committed_dev(jrq_engine* e, const int64_t* local, int64_t* global,
                              uint64_t count_per_rank) {
  if (!e || !local || !global) return JRQ_E_INVALID;
  if (!e->comm) return fail(e, JRQ_E_STATE, "jrq_rccl_init not called");
  DeviceGuard guard(e->device);
  ncclResult_t r = ncclAllGather(local, global, count_per_rank, ncclInt64, e->comm, e->stream);
  if (r != ncclSuccess) return fail(e, JRQ_E_RCCL, "ncclAllGather: %s", ncclGetErrorString(r));
  return JRQ_OK;
}

}  // extern "C"

struct jrq_snapshot {
  std::vector<jrq_table*> t;
  std::vector<jrq_engine*> e;
  std::vector<int64_t*> local, global;
  std::vector<uint32_t> G;
  uint64_t k = 0;
  int via = 0;
};

extern "C" {

jrq_snapshot* jrq_snapshot_create(jrq_table* const* tables, int n, int* err) {
  auto set = [&](int c) {
    if (err) *err = c;
  };
  if (!tables || n <= 0) {
    set(JRQ_E_INVALID);
    return nullptr;
  }
  auto* s = new jrq_snapshot();
  for (int i = 0; i < n; ++i) {
    if (!tables[i] || !tables[i]->e) {
      delete s;
      set(JRQ_E_INVALID);
      return nullptr;
    }
    s->t.push_back(tables[i]);
    s->e.push_back(tables[i]->e);
    s->G.push_back(tables[i]->a.G);
  }
  s->k = s->G[0];
  for (int i = 0; i + 1 < n; ++i)
    if (s->G[i] != s->k || s->G[n - 1] > s->k) {
      fail(s->e[0], JRQ_E_INVALID, "snapshot: tables must hold k groups each (the last at most k)");
      delete s;
      set(JRQ_E_INVALID);
      return nullptr;
    }
  if (n == 1 && s->G[0] > s->k) s->k = s->G[0];
  s->local.assign(n, nullptr);
  s->global.assign(n, nullptr);
  for (int i = 0; i < n; ++i) {
    DeviceGuard guard(s->e[i]->device);
    if (hipMalloc(&s->local[i], s->k * 8) != hipSuccess ||
        hipMalloc(&s->global[i], s->k * 8 * n) != hipSuccess ||
        hipMemset(s->local[i], 0xFF, s->k * 8) != hipSuccess) {
      fail(s->e[i], JRQ_E_NOMEM, "snapshot: device buffers");
      jrq_snapshot_destroy(s);
      set(JRQ_E_NOMEM);
      return nullptr;
    }
  }
  bool all = true;
  for (int i = 0; i < n; ++i) all = all && s->e[i]->comm && s->e[i]->nranks == n && s->e[i]->rank == i;
  s->via = all ? 1 : 0;
  set(JRQ_OK);
  return s;
}

void jrq_snapshot_destroy(jrq_snapshot* s) {
  if (!s) return;
  for (size_t i = 0; i < s->e.size(); ++i) {
    DeviceGuard guard(s->e[i]->device);
    (void)hipStreamSynchronize(s->e[i]->stream);
    if (s->local[i]) (void)hipFree(s->local[i]);
    if (s->global[i]) (void)hipFree(s->global[i]);
  }
  delete s;
}

int jrq_snapshot_publish(jrq_snapshot* s) {
  if (!s) return JRQ_E_INVALID;
  const int n = static_cast<int>(s->t.size());
  for (int i = 0; i < n; ++i) {
    const int rc = jrq_table_committed_dev(s->t[i], s->local[i]);
    if (rc) return rc;
  }
  std::vector<const int64_t*> loc(s->local.begin(), s->local.end());
  return jrq_publish_committed_all_dev(s->e.data(), n, loc.data(), s->global.data(), s->k);
}

int jrq_snapshot_read(jrq_snapshot* s, int i, int64_t* host_out) {
  if (!s || i < 0 || i >= static_cast<int>(s->e.size()) || !host_out) return JRQ_E_INVALID;
  jrq_engine* e = s->e[i];
  DeviceGuard guard(e->device);
  const int n = static_cast<int>(s->t.size());
  std::vector<int64_t> all(s->k * n);
  JRQ_DOWN(e, all.data(), s->global[i], all.size() * 8);
  JRQ_HIP(e, hipStreamSynchronize(e->stream));
  uint64_t at = 0;
  for (int j = 0; j < n; ++j) {
    std::memcpy(host_out + at, all.data() + s->k * j, static_cast<size_t>(s->G[j]) * 8);
    at += s->G[j];
  }
  return JRQ_OK;
}

int jrq_snapshot_via(const jrq_snapshot* s) { return s ? s->via : JRQ_E_INVALID; }

int jrq_rccl_init_all(jrq_engine* const* engines, int n) {
  if (!engines || n <= 0) return JRQ_E_INVALID;
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) {
    if (!engines[i]) return JRQ_E_INVALID;
    devs[i] = engines[i]->device;
  }
  for (int i = 0; i < n; ++i)
    if (engines[i]->comm) {
      (void)ncclCommDestroy(engines[i]->comm);
      engines[i]->comm = nullptr;
    }
  std::vector<ncclComm_t> comms(n, nullptr);
  const ncclResult_t r = ncclCommInitAll(comms.data(), n, devs.data());
  if (r != ncclSuccess) {
    for (auto c : comms)
      if (c) (void)ncclCommDestroy(c);
    return fail(engines[0], JRQ_E_RCCL, "ncclCommInitAll: %s", ncclGetErrorString(r));
  }
  for (int i = 0; i < n; ++i) {
    engines[i]->comm = comms[i];
    engines[i]->nranks = n;
    engines[i]->rank = i;
  }
  return JRQ_OK;
}

int jrq_publish_committed_all_dev(jrq_engine* const* engines, int n, const int64_t* const* local,
                                  int64_t* const* global, uint64_t count) {
  if (!engines || n <= 0 || !local || !global) return JRQ_E_INVALID;
  bool rccl = true;
  for (int i = 0; i < n; ++i) {
    if (!engines[i] || !local[i] || !global[i]) return JRQ_E_INVALID;
    rccl = rccl && engines[i]->comm && engines[i]->nranks == n && engines[i]->rank == i;
  }
  if (rccl) {  // one grouped all-gather over the n communicators
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; i < n && r == ncclSuccess; ++i) {
      DeviceGuard guard(engines[i]->device);
      r = ncclAllGather(local[i], global[i], count, ncclInt64, engines[i]->comm, engines[i]->stream);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return fail(engines[0], JRQ_E_RCCL, "grouped ncclAllGather: %s",
                  ncclGetErrorString(r != ncclSuccess ? r : r2));
    return JRQ_OK;
  }
  // device-to-device copies: destination i's stream waits for source j's stream, then copies
  std::vector<hipEvent_t> ev(n, nullptr);
  int rc = JRQ_OK;
  for (int j = 0; j < n && rc == JRQ_OK; ++j) {
    DeviceGuard guard(engines[j]->device);
    if (hipEventCreateWithFlags(&ev[j], hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(ev[j], engines[j]->stream) != hipSuccess)
      rc = fail(engines[j], JRQ_E_HIP, "publish: event on engine %d", j);
  }
  for (int i = 0; i < n && rc == JRQ_OK; ++i) {
    DeviceGuard guard(engines[i]->device);
    for (int j = 0; j < n && rc == JRQ_OK; ++j) {
      if (hipStreamWaitEvent(engines[i]->stream, ev[j], 0) != hipSuccess ||
          hipMemcpyPeerAsync(global[i] + static_cast<size_t>(j) * count, engines[i]->device, local[j],
                             engines[j]->device, count * 8, engines[i]->stream) != hipSuccess)
        rc = fail(engines[i], JRQ_E_HIP, "publish: copy %d -> %d", j, i);
    }
  }
  // and every source stream waits for the copies that read its buffer: its next write of
  // local[j] (the next publish's de-tiled lastCommitted) cannot overtake them
  std::vector<hipEvent_t> done(n, nullptr);
  for (int i = 0; i < n && rc == JRQ_OK; ++i) {
    DeviceGuard guard(engines[i]->device);
    if (hipEventCreateWithFlags(&done[i], hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(done[i], engines[i]->stream) != hipSuccess)
      rc = fail(engines[i], JRQ_E_HIP, "publish: completion event on engine %d", i);
  }
  for (int j = 0; j < n && rc == JRQ_OK; ++j) {
    DeviceGuard guard(engines[j]->device);
    for (int i = 0; i < n && rc == JRQ_OK; ++i)
      if (i != j && hipStreamWaitEvent(engines[j]->stream, done[i], 0) != hipSuccess)
        rc = fail(engines[j], JRQ_E_HIP, "publish: engine %d waiting for engine %d's copies", j, i);
  }
  for (int j = 0; j < n; ++j) {
    DeviceGuard guard(engines[j]->device);
    if (ev[j]) (void)hipEventDestroy(ev[j]);  // (released once the waits it is part of complete)
    if (done[j]) (void)hipEventDestroy(done[j]);
  }
  return rc;
}

}  // extern "C"
