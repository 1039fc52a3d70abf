// jrq_device.h -- shared device-side definitions for the libjrq kernels (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// SGPR budget of a kernel.  Waves per SIMD on gfx950 = min(VGPR bound, 800 / (ceil(sgpr/16)*16
// + 16)): .sgpr_count <= 80 keeps 8, 82..96 gives 7, while the compiler's occupancy model
// (and its `Occupancy` remark) still says 8 -- so a 1024-thread workgroup at 96 SGPRs runs 1
// workgroup per CU, not 2 (table_epoch_kernel<5>: 24.2 -> 20.3 us per 1M groups,
// round 3's tools/table_probe.hip).  amdgpu_num_sgpr(n) yields .sgpr_count = n - 2.
#define JRQ_SGPRS(n) __attribute__((amdgpu_num_sgpr(n)))
#define JRQ_SGPRS_8WAVES JRQ_SGPRS(82)

namespace jrq {

// ----------------------------------------------------------------- CRC64 ---
// CRC-64/ECMA-182, MSB first, poly 0x42F0E1EBA9EA3693, init 0, xorout 0
// (reference: jraft-core/.../util/CRC64.java:27-40).
constexpr uint64_t kCrcPoly = 0x42F0E1EBA9EA3693ULL;

// Device copies of the constant tables (written once by jrq_create):
//   slice[8][256]  "reversed-domain" slice tables R0..R7, see crc64.hip
//   shift[kShiftTables][8][256]  multiply-by-x^(8*2^t) mod P byte tables
constexpr int kShiftTables = 48;  // shifts up to 2^48 - 1 bytes

// LDS image of the slice tables (128 KiB): 8 tables x 8 replicas (crc64.hip Tab8).
constexpr int kSliceTables = 8;
constexpr int kCrcLdsBytes = 8 * 256 * 8 * 8;
constexpr int kCrcBlock = 512;       // threads per workgroup (8 waves, 1 workgroup / CU)
constexpr int kCrcRegsBlock = 768;   // the register boundary path's workgroup (crc64.hip)
#ifndef JRQ_CRC_FIXED_BLOCK          // (A/B knob) the fixed-size kernel's workgroup
#define JRQ_CRC_FIXED_BLOCK 512
#endif
constexpr int kCrcFixedBlock = JRQ_CRC_FIXED_BLOCK;
#ifndef JRQ_CRC_FIXED_WIDE_BLOCK     // (A/B knob) its workgroup when one lane takes a whole entry
#define JRQ_CRC_FIXED_WIDE_BLOCK 1024
#endif
constexpr int kCrcFixedWideBlock = JRQ_CRC_FIXED_WIDE_BLOCK;
static_assert(kCrcLdsBytes / 8 % kCrcFixedBlock == 0 && kCrcLdsBytes / 8 % kCrcFixedWideBlock == 0,
              "the table image splits evenly over the fixed kernel's threads");

// Status flags, identical to include/jrq.h jrq_group_status.
constexpr uint8_t kStNotLeader = 1, kStOutOfRange = 2, kStEmptyConf = 4;
// ReadIndex heartbeat round verdicts (include/jrq.h JRQ_READINDEX_*)
constexpr uint8_t kRiPending = 0, kRiSuccess = 1, kRiFailure = 2, kRiInvalid = 3;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint64_t bswap64(uint64_t v) { return __builtin_bswap64(v); }

// Workgroup barrier for a hand-off through LDS only: waits for the wave's own LDS operations,
// not for its global stores.  __syncthreads() also waits vmcnt(0) -- on gfx9 stores count there
// too -- so a wave that has just stored its results would sit out their round trip to memory
// before the barrier (the memory clobber keeps the compiler from moving memory accesses across).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Block-wide exclusive scan of one value per thread (wave shuffles + LDS).
__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* lds_warp,
                                                         uint64_t* total) {
  using u64 = unsigned long long;  // the __shfl_* overloads take (unsigned) long long
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  u64 x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u64 y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) lds_warp[wave] = x;
  __syncthreads();
  if (wave == 0) {
    const int nw = blockDim.x >> 6;
    u64 s = lane < nw ? lds_warp[lane] : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const u64 y = __shfl_up(s, d, 64);
      if (lane >= d) s += y;
    }
    if (lane < nw) lds_warp[lane] = s;  // inclusive wave totals
  }
  __syncthreads();
  const uint64_t before = wave ? lds_warp[wave - 1] : 0;
  *total = lds_warp[(blockDim.x >> 6) - 1];
  __syncthreads();
  return before + x - v;
}

}  // namespace jrq

// Host-visible launch parameter blocks (plain structs, passed by value).
struct JrqCrcArgs {
  const uint8_t* payload;
  const uint64_t* offsets;  // N+1
  uint32_t n;
  uint64_t* out;
  // LogEntry fields (all null for the plain crc64 batch)
  const uint8_t* type;
  const int64_t* index;
  const int64_t* term;
  const uint64_t* peer_xor;
  const uint64_t* expected;
  const uint8_t* has;
  uint8_t* corrupt;
  // engine constants / scratch
  const uint64_t* slice;   // [8][256] reversed-domain slice tables R0..R7
  const uint64_t* shift;   // [kShiftTables][8][256]
  uint64_t* acc;           // straddler accumulators, zero between launches
  uint32_t* cnt;           // straddler arrival counters, zero between launches
  uint64_t* piece_cont;    // per segment: its head/middle piece of a straddling entry
  uint64_t* piece_tail;    // per segment: its tail piece of a straddling entry
  uint32_t scratch_len;    // entries in acc/cnt/piece_*
  uint32_t lanes;          // lanes of the rounds grid (set by the launcher)
  uint32_t seg_map;        // 0: 64-segment chunks round-robin over workgroups; 1: per workgroup
  uint64_t seg_bytes;      // nonzero: segment size (rounded up to 256 B; tests / tuning)
  uint32_t prio_steps;     // 1: waves lower their priority as they progress (crc64.hip)
  uint32_t regs_slowpath;  // 1: boundary half-rounds hash from registers (crc64_rounds_kernel<true>)
  uint64_t* stream_state;  // nullable: streaming Checksum registers folded by the finish kernel
  uint64_t entry_bytes;    // crc64_fixed_kernel: every entry this long, back to back (no offsets)
  uint32_t fixed_k;        // crc64_fixed_kernel: lanes per entry (power of two, 1..64)
  const uint64_t* starts;  // crc64_fixed_kernel<., true>: entry i starts at payload + starts[i]
  const uint64_t* gate;    // nullable device words {k, entry_bytes} (V2 decode): the starts
                           // kernel runs iff k != 0, the segment walk (rounds + finish) iff k == 0
  uint32_t no_finish;      // 1: launch the rounds kernel only; the caller's kernel assembles the
                           // straddling entries (crc_pieces) -- V2's v2_finish does
};

// Segment walk geometry shared by crc64_rounds_kernel / crc64_finish_kernel (crc64.hip) and
// v2_finish (v2_decode.hip).  Entries spanning at most kMaxSlotParts segments hand their pieces
// over through per-segment slots (plain stores) XOR-ed by whoever finishes the entry; longer
// ones through the atomic slot (their out[] is final after the rounds kernel).
constexpr uint64_t kMaxSlotParts = 64;

// Segment size (bytes; identical in every kernel of one walk): a multiple of 256 (two 128-B
// rounds), ~span / lanes of the rounds grid, never more segments than straddler slots.
__device__ __forceinline__ uint64_t seg_size(const JrqCrcArgs& a, uint64_t span) {
  auto up256 = [](uint64_t x) { return (x + 255) & ~255ull; };
  const uint64_t lanes = a.lanes;
  uint64_t S = a.seg_bytes ? up256(a.seg_bytes) : up256((span + lanes - 1) / lanes);
  if (S < 256) S = 256;
  const uint64_t s_min = up256((span + a.scratch_len - 3) / (a.scratch_len - 2));
  return S < s_min ? s_min : S;
}

// An entry [o0, o1) of the walk (stream base, misalignment D, segment size S) that straddles
// 2..kMaxSlotParts segments: *v = the XOR of its pieces (true); otherwise false and its out[]
// entry holds the CRC.
__device__ __forceinline__ bool crc_pieces(const JrqCrcArgs& a, uint64_t o0, uint64_t o1, uint64_t base,
                                           uint64_t D, uint64_t S, uint64_t& v) {
  const uint64_t first = (o0 - base + D) / S, last = o1 > o0 ? (o1 - 1 - base + D) / S : first;
  if (last == first || last - first + 1 > kMaxSlotParts) return false;
  v = a.piece_tail[last];
  for (uint64_t g = first; g < last; ++g) v ^= a.piece_cont[g];
  return true;
}

// Leader lease / alive-quorum check (quorum.hip, lease kernel).
struct JrqLeaseArgs {
  const int64_t* last_rpc_ts;   // [P][ld] lastRpcSendTimestamp per peer slot
  uint64_t ld;
  const uint64_t* conf;         // [G] packed conf word (masks + quorums)
  const uint8_t* self_slot;     // [G] the leader's own slot (always alive)
  int64_t now_ms;
  int64_t lease_timeout_ms;
  uint32_t num_peers;
  uint32_t G;
  uint8_t* ok;                  // [G] bit0 conf quorum alive, bit1 old-conf quorum alive (or no old conf)
  int64_t* lease_start;         // [G] lastLeaderTimestamp after the checks (in/out)
  uint16_t* dead;               // [G] peer slots found dead (new | old conf), nullable
  // the leader tick (jrq_leader_tick*): the ReadIndex round of the same groups, fused; null
  // for the lease check alone
  const uint64_t* order;        // [G] nibble p = arrival position of slot p's response, 0 = none
  const uint16_t* ri_ok_mask;   // [G] bit p = slot p's response succeeded
  uint8_t* ri_result;           // [G] kRiPending / kRiSuccess / kRiFailure / kRiInvalid
};

// ReadIndex heartbeat quorum (quorum.hip): one heartbeat round per group.
struct JrqReadIndexArgs {
  const uint64_t* conf;         // [G] packed conf word (new mask + quorum are read)
  const uint8_t* self_slot;     // [G] the leader's own slot (no heartbeat sent to it)
  const uint64_t* order;        // [G] nibble p = arrival position of slot p's response, 0 = none
  const uint16_t* ok_mask;      // [G] bit p = slot p's response succeeded
  uint32_t num_peers;
  uint32_t G;
  uint8_t* result;              // [G] kRiPending / kRiSuccess / kRiFailure / kRiInvalid
};

// AppendEntries batch verify (append_entries.hip): inputs + engine scratch.
struct JrqAeArgs {
  uint32_t r;                      // requests
  const uint32_t* req_off;         // [r+1] entry ranges per request
  const int64_t* prev_log_index;   // [r]
  uint32_t n;                      // entries
  const uint8_t* type;             // [n] EntryType number
  const int64_t* data_len;         // [n]
  const uint8_t* has_checksum;     // [n] nullable (= all have one)
  uint64_t* offsets;               // scratch [n+1] payload offsets
  int64_t* index;                  // scratch [n] log indexes
  uint8_t* has_eff;                // scratch [n] has && type != UNKNOWN
  uint64_t* tile_sums;             // scratch [ceil(n/4096)]
  const uint8_t* corrupt;          // [n] verify flags (from the checksum kernel)
  int32_t* first_corrupt;          // [r] out
};

// Commit fan-out after an epoch (commit_fanout.hip).
struct JrqFanoutArgs {
  uint32_t G;
  const int64_t* prev_committed;  // [G] BallotBox.lastCommittedIndex before the epoch
  const int64_t* committed;       // [G] after the epoch
  const int64_t* last_applied;    // [G] FSMCaller.lastAppliedIndex
  int64_t* cq_first;              // [G] ClosureQueue.firstIndex (in/out)
  int64_t* cq_size;               // [G] ClosureQueue size (in/out)
  int64_t* first_closure;         // [G] out: popClosureUntil result
  uint8_t* status;                // [G] out: jrq_fanout_status
  uint64_t* listed;               // [ceil(G/64)] out: bitmap of APPLY / INVALID groups
  uint32_t* num_listed;           // [1] out
  uint32_t* ctr;                  // engine scratch: u64 {blocks done << 32 | sum}, zero between launches
};

// V2 log-entry decode + verify (v2_decode.hip).
struct JrqV2Args {
  const uint8_t* rec;
  const uint64_t* off;     // [n+1]
  uint32_t n;
  const uint64_t* slice;   // engine slice tables (R_j = bswap of T_j = i * x^(64 + 8j))
  const uint64_t* xinv;    // engine [8][256]: i * x^(8k - 64) mod P
  uint8_t* status;
  uint8_t* type;
  int64_t* index;
  int64_t* term;
  uint64_t* stored;
  uint8_t* has_checksum;
  uint64_t* data_off;
  uint64_t* data_len;
  uint32_t* peer_counts;   // nullable
  uint64_t* computed;
  uint8_t* corrupt;
  uint64_t* partial;       // scratch [n]
  uint64_t* off2;          // scratch [n+2]: record i's range = [off2[i+1], off2[i+2])
  const uint64_t* crc2;    // scratch [n+1] (CRC of the ranges; range 0 = the leading header)
  uint64_t* lens;          // scratch [n] header length << 32 | trailer length
  uint64_t* gate;          // engine words [24]: {k, L, bad, end, arrivals, -, -, -, segment
                           // arrivals [16]} -- the data CRCs by
                           // crc64_fixed_kernel (k lanes per record) when every record decoded with
                           // data length L; arrivals is zero between launches
  uint64_t* blk;           // scratch [4 * ceil(n / 256)]: v2_parse's per-block summaries
  uint64_t lanes;          // lanes of the CRC grid (crc64_fixed_kernel)
};

// Lanes per entry of crc64_fixed_kernel for N entries of L bytes on `lanes` lanes: the fewest
// power of two (<= 64) giving every lane a piece of whole 256-B multiples; 0 = not applicable.
__host__ __device__ inline uint32_t jrq_fixed_k(uint64_t L, uint32_t n, uint64_t lanes) {
  if (L < 256 || L % 256 != 0) return 0;
  uint32_t k = 1;
  while (static_cast<uint64_t>(n) * k < lanes && k < 64 && (L / (2 * k)) % 256 == 0) k *= 2;
  if (static_cast<uint64_t>(n) * k < lanes || L / k > (1ull << 25)) return 0;
  return k;
}

struct JrqQuorumArgs {
  const int64_t* match;
  const int64_t* pending_index;
  const int64_t* last_appended;
  const int64_t* last_committed;
  const uint64_t* conf;
  const uint32_t* run_off;
  const int64_t* run_start;
  const uint64_t* run_conf;
  uint32_t num_peers;
  uint64_t match_ld;
  int64_t* committed;
  uint8_t* status;
  uint32_t G;
  uint64_t ts;  // 0: the inputs are rows; else words per 256-group tile (the fields' rows in
                // tile 0 above, match[p] at match + 256 p: jrq_quorum_epoch_tiles_dev)
};

// Resident group table (table.hip; include/jrq.h jrq_table).
namespace jrq {
constexpr int kTableMaxRuns = 4;                   // JRQ_TABLE_MAX_RUNS
constexpr uint32_t kTableSlice = 256;              // groups per tile (jrq_table_view.tile_groups)
constexpr uint32_t kListSlice = 128;               // JRQ_TABLE_SLICE: groups per epoch wave and
                                                   // per slice of its changed list (half a tile)
constexpr uint32_t kTableBlockWaves = 4;           // waves per epoch / flags workgroup
constexpr int64_t kPiFollowsLc = INT64_MIN;        // JRQ_PI_FOLLOWS_LC
constexpr uint32_t kFlagSlots = kListSlice;        // flagged-entry slots per epoch wave
}  // namespace jrq
// The hot fields live in tiles of kTableSlice (256) groups, two epoch waves per tile: tile i
// holds match[0..P-1], pendingIndex, lastAppended, lastCommitted, conf of groups [256 i,
// 256 i + 256), so a tile is one contiguous (4P + 32) * 256-B block (field-major
// rows over all groups ran 20 % slower: tools/probes/streams_probe.hip).  pendingIndex,
// lastAppended, lastCommitted and conf are 256 consecutive int64 words each; element g of such
// a field is row[(g >> 8) * ts + (g & 255)] (tf()).  The match of a slot is a u32 relative to
// the group's match base (mbase(pendingIndex): pendingIndex - 1 rounded down to a multiple of
// 2^30, fixed for a billion entries), saturated at 0 below it -- a match below the pending
// window grants nothing whatever its value -- so a slot costs 4 B instead of 8 (r05); the 256
// u32 of a slot's row sit in group order (r06: the epoch's lane l of half h reads groups
// 128 h + 2 l, + 1 as one 8-B load).
struct JrqTableArgs {
  uint32_t* match;       // match[0] row of tile 0 (u32); match[p] at match + 256 p, tile stride 2 ts
  int64_t* pi;           // pendingIndex, or kPiFollowsLc
  int64_t* la;
  int64_t* lc;
  uint64_t* conf;        // run 0 conf word | JRQ_CONF_RUNS
  uint64_t ts;           // int64 words per tile: 128 P + 1024
  int64_t* xstart;       // [jrq::kTableMaxRuns - 1][ld] extra run starts (INT64_MAX = unused)
  uint64_t* xconf;       // [kTableMaxRuns - 1][ld]
  uint64_t ld;           // row stride of xstart / xconf (cold fields: group-major rows)
  uint32_t G;            // groups (ld >= G rounded up to pairs; pad groups are not leaders)
  uint32_t P;
  uint32_t* invalid;     // records / headers skipped as invalid since the last jrq_table_check
  uint64_t* changed;     // [slices][JRQ_TABLE_SLICE] out: epoch wave w's slice at changed[128 w ..]
  uint32_t* n_changed;   // [slices] out
  uint8_t* status;       // [G] out, nullable
  uint64_t* flag_ent;    // [waves][kFlagSlots][8] per 128-group epoch wave: its groups flagged
                         // JRQ_CONF_RUNS as 64-B entries {group, run starts 1-3, conf words 0-3}
  uint32_t* flag_wcnt;   // [waves] how many
  uint64_t* rstamp;      // [ld] reset stamp of each group (JRQ_STATE_STAMP headers): order-free
                         // ack records from segments stamped earlier are dropped
  int64_t* fsm;          // [3][ld] FSMCaller state of each group (r06): lastAppliedIndex, then the
                         // ClosureQueue's firstIndex and size (jrq_table_fsm_update)
  int64_t* fan_first;    // [slices][JRQ_TABLE_SLICE] out, fused fan-out epochs only: popClosureUntil's
                         // result of the slice's committing groups, at their delta ranks
  uint8_t* fan_status;   // [slices][JRQ_TABLE_SLICE] out: their jrq_fanout_status
};

// Element g of a tiled int64 field (its row in tile 0: t.pi, t.la, t.lc, t.conf).
template <class T>
__host__ __device__ __forceinline__ T& tf(T* row, const JrqTableArgs& t, uint32_t g) {
  return row[static_cast<size_t>(g >> 8) * t.ts + (g & 255u)];
}

namespace jrq {
// include/jrq.h jrq_fanout_status
constexpr uint8_t kFanNone = 0, kFanApply = 1, kFanSkip = 2, kFanInvalid = 3;

// One group's FSMCallerImpl.doCommitted gate and ClosureQueueImpl.popClosureUntil for the epoch's
// last committed index c (FSMCallerImpl.java:462-482, ClosureQueueImpl.java:113-142; the closed
// form of commit_fanout.hip): the status, the first popped closure's index (c + 1 when none is
// popped, -1 for INVALID) and the queue (f, n) after the pops.
__device__ __forceinline__ uint8_t fan_one(int64_t prev, int64_t c, int64_t applied, int64_t& f,
                                           int64_t& n, int64_t& first_closure) {
  first_closure = 0;
  if (c <= prev) return kFanNone;  // onCommitted was not called for this group
  if (applied >= c) return kFanSkip;
  if (n == 0 || c < f) {
    first_closure = c + 1;
    return kFanApply;
  }
  if (c > f + n - 1) {
    first_closure = -1;
    return kFanInvalid;
  }
  first_closure = f;
  n -= c - f + 1;
  f = c + 1;
  return kFanApply;
}

constexpr int kMatchPageBits = 30;  // match base granularity (JRQ_TABLE_MATCH_PAGE)
// The match base of a group whose (resolved) pendingIndex is pi; 0 when not the leader.
__host__ __device__ __forceinline__ int64_t mbase(int64_t pi) {
  return pi > 0 ? ((pi - 1) & ~((int64_t{1} << kMatchPageBits) - 1)) : 0;
}
}  // namespace jrq

// The u32 match word of slot p of group g.
__host__ __device__ __forceinline__ uint32_t& tm(const JrqTableArgs& t, uint32_t p, uint32_t g) {
  return t.match[static_cast<size_t>(g >> 8) * (2 * t.ts) + p * 256u + (g & 255u)];
}

// One group header as the ABI carries it (include/jrq.h jrq_group_state).
struct JrqGroupState {
  uint32_t group;
  uint16_t num_runs;
  uint16_t flags;
  int64_t pending_index;
  int64_t last_appended;
  int64_t last_committed;
  uint64_t run_conf[jrq::kTableMaxRuns];
  int64_t run_start[jrq::kTableMaxRuns];
};
static_assert(sizeof(JrqGroupState) == 96, "jrq_group_state layout");
