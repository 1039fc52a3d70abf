// crc64.hip -- batched CRC-64/ECMA-182 and fused LogEntry.checksum for gfx950.
//
// Replaces, for a whole batch of log entries at once:
//   CrcUtil.crc64(...)      jraft-core/.../util/CrcUtil.java:36-80
//   CRC64.update(...)       jraft-core/.../util/CRC64.java:100-110
//   LogEntry.checksum()     jraft-core/.../entity/LogEntry.java:88-108
//   LogEntry.isCorrupted()  jraft-core/.../entity/LogEntry.java:156-158
//
// Design (DESIGN.md §CRC64 has the roofline):
//  * The payload is cut into equal flat SEGMENTS of S = 2^s bytes (S from the
//    batch size so that every lane of the persistent grid gets ~1 segment); each
//    lane walks its segment entry by entry with a serial table CRC.  Work per
//    lane is the same whatever the entry-length distribution.
//  * The CRC is linear over GF(2) with init 0, so a piece of an entry that ends
//    n bytes before the entry's end contributes crc(piece) * x^(8n) mod P, and
//    the entry's CRC is the XOR of its pieces.  Pieces of entries that straddle a
//    segment boundary are XOR-combined in a scratch slot with agent-scope
//    atomics; the last arriving piece (arrival counter) writes the result and
//    re-zeroes the slot.
//  * Byte-serial update in the "reversed domain": with r = bswap64(crc), one
//    2-byte step is r = (r >> 16) ^ R1[r & 0xFF] ^ R0[(r >> 8) & 0xFF], and a
//    little-endian 8-byte load XORs straight into r (no byte swaps).  R0/R1 live
//    in LDS replicated 32x so that lane l only touches bank slot l&31: every
//    ds_read_b64 is conflict-free.  One step = 2 v_perm (LDS address), 2 LDS
//    reads, 1 v_alignbit + 1 shift, 2 v_bitop3 (XOR3).
//  * The x^(8n) multiplications use byte tables in global memory (one per power
//    of two, L2-resident); they run at most once per piece that does not end its
//    entry, i.e. at most once per segment.
#include "jrq_device.h"

namespace jrq {

// LDS address selectors for v_perm_b32 (S0 = lane constant, S1 = r.lo):
//   lane constant: byte0 = (l&31)<<3, byte2 = 1 (table R1 at +64 KiB)
//   R1 index = r byte 0 -> address byte1; R0 index = r byte 1 -> address byte1.
constexpr uint32_t kSelR1 = 0x0C060004u;  // {lc.b0, lo.b0, lc.b2, 0}
constexpr uint32_t kSelR0 = 0x0C0C0104u;  // {lc.b0, lo.b1, 0, 0}

struct RState {
  uint32_t lo, hi;
};

__device__ __forceinline__ void step2(RState& r, const char* lds, uint32_t lc) {
  const uint32_t a1 = __builtin_amdgcn_perm(lc, r.lo, kSelR1);
  const uint32_t a0 = __builtin_amdgcn_perm(lc, r.lo, kSelR0);
  const uint2 t1 = *reinterpret_cast<const uint2*>(lds + a1);
  const uint2 t0 = *reinterpret_cast<const uint2*>(lds + a0);
  const uint32_t nlo = __builtin_amdgcn_alignbit(r.hi, r.lo, 16);
  const uint32_t nhi = r.hi >> 16;
  r.lo = xor3(nlo, t1.x, t0.x);
  r.hi = xor3(nhi, t1.y, t0.y);
}

// One byte: r = R0[(r ^ b) & 0xFF] ^ (r >> 8)   (CRC64.update(byte), CRC64.java:100-103)
__device__ __forceinline__ void step1(RState& r, uint32_t b, const char* lds, uint32_t lc) {
  const uint32_t a0 = __builtin_amdgcn_perm(lc, r.lo ^ b, 0x0C0C0004u);
  const uint2 t0 = *reinterpret_cast<const uint2*>(lds + a0);
  const uint32_t nlo = __builtin_amdgcn_alignbit(r.hi, r.lo, 8);
  r.lo = nlo ^ t0.x;
  r.hi = (r.hi >> 8) ^ t0.y;
}

// Eight bytes given as a little-endian (lo, hi) dword pair.
__device__ __forceinline__ void step8(RState& r, uint32_t dlo, uint32_t dhi, const char* lds,
                                      uint32_t lc) {
  r.lo ^= dlo;
  r.hi ^= dhi;
  step2(r, lds, lc);
  step2(r, lds, lc);
  step2(r, lds, lc);
  step2(r, lds, lc);
}

__device__ __forceinline__ void step16(RState& r, const uint4& v, const char* lds, uint32_t lc) {
  step8(r, v.x, v.y, lds, lc);
  step8(r, v.z, v.w, lds, lc);
}

__device__ __forceinline__ uint64_t crc_value(const RState& r) {
  // crc = bswap64(r)
  return (static_cast<uint64_t>(__builtin_bswap32(r.lo)) << 32) | __builtin_bswap32(r.hi);
}

// CRC of payload[a, b) from a zero register.
template <int BV>
__device__ __forceinline__ uint64_t crc_range(const uint8_t* __restrict__ payload, uint64_t a,
                                              uint64_t b, const char* lds, uint32_t lc) {
  RState r{0u, 0u};
  uint64_t p = a;
  const uint64_t mis = reinterpret_cast<uintptr_t>(payload) & 15u;
  while (p < b && ((p + mis) & 15u)) {  // unaligned head (by address), byte-serial
    step1(r, payload[p], lds, lc);
    ++p;
  }
  // Blocks of 16*BV bytes through a 2-deep register ring: block i+1's loads are issued
  // before block i is hashed, unconditionally (address clamped to the last block), so
  // the compiler's wait before block i is a counted vmcnt(BV), not vmcnt(0).  Unrolled
  // by two with fixed buffer roles: a loaded register is never copied (a copy would
  // force the wait early).  The empty asm after each load group is a compiler memory
  // barrier: the loads may not be re-issued (rematerialised) at their use a block
  // later; it implies no hardware wait.  BV = 8 reads whole 128-B lines per lane.
  constexpr uint32_t kBlkBytes = 16u * BV;
  const uint64_t nblk = (b - p) / kBlkBytes;
  if (nblk != 0) {
    const uint4* q = reinterpret_cast<const uint4*>(payload + p);
    const uint64_t last = nblk - 1;
    uint4 A[BV], B[BV];
#define JRQ_LOAD(X, blk)                                 \
  do {                                                   \
    const uint64_t bb = (blk) < last ? (blk) : last;     \
    const uint4* qq = q + BV * bb;                       \
    _Pragma("unroll") for (int v = 0; v < BV; ++v) X[v] = qq[v]; \
    asm volatile("" ::: "memory");                       \
  } while (0)
#define JRQ_HASH(X)                                                          \
  do {                                                                       \
    _Pragma("unroll") for (int v = 0; v < BV; ++v) step16(r, X[v], lds, lc); \
  } while (0)
    JRQ_LOAD(A, 0);
    for (uint64_t i = 0;;) {
      JRQ_LOAD(B, i + 1);
      JRQ_HASH(A);
      if (++i == nblk) break;
      JRQ_LOAD(A, i + 1);
      JRQ_HASH(B);
      if (++i == nblk) break;
    }
#undef JRQ_LOAD
#undef JRQ_HASH
    p += nblk * kBlkBytes;
  }
  while (p + 16 <= b) {
    const uint4 v = *reinterpret_cast<const uint4*>(payload + p);
    step16(r, v, lds, lc);
    p += 16;
  }
  while (p + 2 <= b) {  // tail
    const uint32_t w = payload[p] | (static_cast<uint32_t>(payload[p + 1]) << 8);
    r.lo ^= w;
    step2(r, lds, lc);
    p += 2;
  }
  if (p < b) step1(r, payload[p], lds, lc);
  return crc_value(r);
}

// LogId.checksum(): crc64(BE64(index) || BE64(term))  (LogId.java:45-50, Bits.java:71-80).
// The big-endian bytes, read as a little-endian u64, are bswap64(v).
__device__ __forceinline__ uint64_t logid_crc(int64_t index, int64_t term, const char* lds,
                                              uint32_t lc) {
  RState r{0u, 0u};
  const uint64_t bi = bswap64(static_cast<uint64_t>(index));
  const uint64_t bt = bswap64(static_cast<uint64_t>(term));
  step8(r, static_cast<uint32_t>(bi), static_cast<uint32_t>(bi >> 32), lds, lc);
  step8(r, static_cast<uint32_t>(bt), static_cast<uint32_t>(bt >> 32), lds, lc);
  return crc_value(r);
}

// c * x^(8n) mod P via the global power tables: one 8-lookup pass per set bit of n.
__device__ __forceinline__ uint64_t crc_shift(uint64_t c, uint64_t n,
                                              const uint64_t* __restrict__ shift) {
  for (int t = 0; n != 0 && t < kShiftTables; ++t, n >>= 1) {
    if (!(n & 1u)) continue;
    const uint64_t* tb = shift + static_cast<size_t>(t) * 8 * 256;
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) v ^= tb[k * 256 + ((c >> (8 * k)) & 0xFF)];
    c = v;
  }
  return c;
}

// Two independent chains per lane: [a, b) is cut at m into halves that are hashed in
// lockstep (their 2-byte steps interleave, so one chain's LDS latency hides under the
// other's), then crc = crc(X) * x^(8|Y|) ^ crc(Y).  Both halves move through 64-B
// blocks with a 2-deep register ring each; X takes the unaligned head first, Y the tail
// last.  Short ranges fall back to one chain.
__device__ __forceinline__ uint64_t crc_range2(const uint8_t* __restrict__ payload, uint64_t a,
                                               uint64_t b, const char* lds, uint32_t lc,
                                               const uint64_t* __restrict__ shift) {
  constexpr uint64_t kBB = 64;  // block bytes per chain
  if (b - a < 4 * kBB) return crc_range<4>(payload, a, b, lds, lc);
  RState x{0u, 0u}, y{0u, 0u};
  uint64_t p = a;
  const uint64_t mis = reinterpret_cast<uintptr_t>(payload) & 15u;
  while (p < b && ((p + mis) & 15u)) {
    step1(x, payload[p], lds, lc);
    ++p;
  }
  const uint64_t nb = (b - p) / (2 * kBB);  // blocks per chain (>= 1 here)
  const uint64_t m = p + nb * kBB;
  const uint4* qx = reinterpret_cast<const uint4*>(payload + p);
  const uint4* qy = reinterpret_cast<const uint4*>(payload + m);
  const uint64_t last = nb - 1;
  uint4 XA[4], XB[4], YA[4], YB[4];
#define JRQ_LOAD2(X, Y, blk)                                            \
  do {                                                                  \
    const uint64_t bb = (blk) < last ? (blk) : last;                    \
    _Pragma("unroll") for (int v = 0; v < 4; ++v) X[v] = qx[4 * bb + v]; \
    _Pragma("unroll") for (int v = 0; v < 4; ++v) Y[v] = qy[4 * bb + v]; \
    asm volatile("" ::: "memory");                                      \
  } while (0)
#define JRQ_HASH2(X, Y)                          \
  do {                                           \
    _Pragma("unroll") for (int v = 0; v < 4; ++v) { \
      x.lo ^= X[v].x;                            \
      x.hi ^= X[v].y;                            \
      y.lo ^= Y[v].x;                            \
      y.hi ^= Y[v].y;                            \
      _Pragma("unroll") for (int s = 0; s < 4; ++s) { \
        step2(x, lds, lc);                       \
        step2(y, lds, lc);                       \
      }                                          \
      x.lo ^= X[v].z;                            \
      x.hi ^= X[v].w;                            \
      y.lo ^= Y[v].z;                            \
      y.hi ^= Y[v].w;                            \
      _Pragma("unroll") for (int s = 0; s < 4; ++s) { \
        step2(x, lds, lc);                       \
        step2(y, lds, lc);                       \
      }                                          \
    }                                            \
  } while (0)
  JRQ_LOAD2(XA, YA, 0);
  for (uint64_t i = 0;;) {
    JRQ_LOAD2(XB, YB, i + 1);
    JRQ_HASH2(XA, YA);
    if (++i == nb) break;
    JRQ_LOAD2(XA, YA, i + 1);
    JRQ_HASH2(XB, YB);
    if (++i == nb) break;
  }
#undef JRQ_LOAD2
#undef JRQ_HASH2
  // Y continues over the tail [m + nb*kBB, b)
  uint64_t q = m + nb * kBB;
  while (q + 16 <= b) {
    step16(y, *reinterpret_cast<const uint4*>(payload + q), lds, lc);
    q += 16;
  }
  while (q + 2 <= b) {
    y.lo ^= payload[q] | (static_cast<uint32_t>(payload[q + 1]) << 8);
    step2(y, lds, lc);
    q += 2;
  }
  if (q < b) step1(y, payload[q], lds, lc);
  return crc_shift(crc_value(x), b - m, shift) ^ crc_value(y);
}

template <bool kLogEntry>
__device__ __forceinline__ uint64_t entry_fields(const JrqCrcArgs& a, uint32_t e, const char* lds,
                                                 uint32_t lc) {
  if (!kLogEntry) return 0;
  // LogEntry.checksum: type.getNumber() ^ id.checksum() ^ peers' checksums (LogEntry.java:89-94)
  uint64_t f = static_cast<uint64_t>(a.type[e]) ^ logid_crc(a.index[e], a.term[e], lds, lc);
  if (a.peer_xor) f ^= a.peer_xor[e];
  return f;
}

template <bool kLogEntry>
__device__ __forceinline__ void emit(const JrqCrcArgs& a, uint32_t e, uint64_t v) {
  a.out[e] = v;
  if (kLogEntry && a.expected != nullptr && a.corrupt != nullptr) {
    const bool has = (a.has == nullptr) || a.has[e];
    a.corrupt[e] = static_cast<uint8_t>(has && a.expected[e] != v);
  }
}

// One piece of an entry that spans `parts` segments: XOR its (already shifted) CRC into
// the entry's scratch slot; the last of the `parts` arrivals publishes and re-zeroes it.
// Hand-off = 8-byte agent-scope atomics on both sides (MI355X_MICROARCH.md, visibility
// "valid forms"): the XOR is drained (s_waitcnt vmcnt(0)) before the arrival add, the last
// arriver reads the slot with an atomic after its add returned.  No release/acquire
// fences: those would write back the XCD's L2 / invalidate L1 on every piece.
template <bool kLogEntry>
__device__ __forceinline__ void straddle_piece(const JrqCrcArgs& a, uint32_t e, uint32_t slot,
                                               uint32_t parts, uint64_t c) {
  __hip_atomic_fetch_xor(&a.acc[slot], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t arrived =
      __hip_atomic_fetch_add(&a.cnt[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (arrived + 1 == parts) {
    // read-and-zero in one memory-side RMW (an xor-with-0 would be folded into a load)
    const uint64_t v =
        __hip_atomic_exchange(&a.acc[slot], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    emit<kLogEntry>(a, e, v);
    __hip_atomic_store(&a.cnt[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// First e in [0, n] with offsets[e] >= x (offsets[n] >= x is guaranteed by the caller).
__device__ __forceinline__ uint32_t lower_bound_off(const uint64_t* __restrict__ off, uint32_t n,
                                                    uint64_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    if (off[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Hash one piece: kVariant 4 / 8 = one chain with 64-B / 128-B blocks, 2 = two chains.
template <int kVariant>
__device__ __forceinline__ uint64_t crc_piece(const JrqCrcArgs& a, uint64_t lo, uint64_t hi,
                                              const char* lds, uint32_t lc) {
  if (kVariant == 2) return crc_range2(a.payload, lo, hi, lds, lc, a.shift);
  return crc_range<kVariant == 8 ? 8 : 4>(a.payload, lo, hi, lds, lc);
}

template <bool kLogEntry, int kVariant>
__global__ __launch_bounds__(kCrcBlock) void crc64_segments_kernel(JrqCrcArgs a) {
  __shared__ __attribute__((aligned(16))) uint64_t lds_tab[kCrcLdsBytes / 8];
  const char* lds = reinterpret_cast<const char*>(lds_tab);

  // Replicate R0/R1 into the lane-private bank image: word w = table<<13 | idx<<5 | slot.
  for (uint32_t w = threadIdx.x; w < kCrcLdsBytes / 8; w += blockDim.x) {
    const uint32_t table = w >> 13, idx = (w >> 5) & 255u;
    lds_tab[w] = a.slice[table * 256 + idx];
  }
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lc = ((lane & 31u) << 3) | (1u << 16);

  const uint64_t base = a.offsets[0];
  const uint64_t total = a.offsets[a.n] - base;
  const uint64_t lanes = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  // Segment size S ~ total/lanes (>= 2^min_seg_log2).  All lanes walk their segments in
  // lockstep, so lane l reads near l*S at any moment: S is an ODD multiple of 64 B so
  // that those addresses spread over the memory channels (a power-of-two stride piles
  // a whole wave onto a few of them).  seg_mode 0 keeps the power-of-two size (A/B).
  uint64_t S;
  if (a.seg_bytes != 0) {
    S = a.seg_bytes;
  } else if (a.seg_mode == 0) {
    uint32_t s = a.min_seg_log2;
    while (s < 40 && (total >> (s + 1)) >= lanes) ++s;
    S = 1ull << s;
  } else {
    uint64_t t = (total + lanes - 1) / lanes;
    const uint64_t floor_bytes = 1ull << a.min_seg_log2;
    if (t < floor_bytes) t = floor_bytes;
    S = (((t + 63) >> 6) | 1u) << 6;
  }
  // never more segments than straddler slots (scratch_len - 2)
  const uint64_t s_min = (total + a.scratch_len - 3) / (a.scratch_len - 2);
  if (S < s_min) S = s_min;
  uint64_t nseg = (total + S - 1) / S;
  if (nseg == 0) nseg = 1;

  for (uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k < nseg;
       k += lanes) {
    const uint64_t s0 = base + k * S;
    const uint64_t s1 = (k + 1 == nseg) ? base + total : s0 + S;
    const bool last_seg = (k + 1 == nseg);
    uint32_t e = lower_bound_off(a.offsets, a.n, s0);
    uint64_t oe = a.offsets[e];

    // piece of the entry that began in an earlier segment
    if (e > 0 && oe > s0) {
      const uint32_t t = e - 1;
      const uint64_t pe = oe < s1 ? oe : s1;
      uint64_t c = crc_piece<kVariant>(a, s0, pe, lds, lc);
      c = crc_shift(c, oe - pe, a.shift);
      const uint64_t ot = a.offsets[t];
      const uint64_t first = (ot - base) / S, lastseg = (oe - 1 - base) / S;
      straddle_piece<kLogEntry>(a, t, static_cast<uint32_t>(first),
                                static_cast<uint32_t>(lastseg - first + 1), c);
    }

    // entries that begin inside this segment (zero-length ones at the very end go to the last)
    while (e < a.n && (oe < s1 || (last_seg && oe == s1))) {
      const uint64_t oe1 = a.offsets[e + 1];
      const uint64_t pe = oe1 < s1 ? oe1 : s1;
      const uint64_t fields = entry_fields<kLogEntry>(a, e, lds, lc);
      uint64_t c = crc_piece<kVariant>(a, oe, pe, lds, lc);
      if (oe1 <= s1) {
        emit<kLogEntry>(a, e, c ^ fields);  // whole entry inside the segment
      } else {
        // head piece of a straddling entry: shift its data CRC to the entry end, add the fields
        c = crc_shift(c, oe1 - pe, a.shift) ^ fields;
        const uint64_t lastseg = (oe1 - 1 - base) / S;
        straddle_piece<kLogEntry>(a, e, static_cast<uint32_t>(k),
                                  static_cast<uint32_t>(lastseg - k + 1), c);
      }
      ++e;
      oe = oe1;
    }
  }
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_crc64(const JrqCrcArgs* args, int log_entry, int grid,
                                       hipStream_t stream) {
  const dim3 g(grid), blk(jrq::kCrcBlock);
  // variant: two chains per lane, or one chain with 128-B / 64-B per-lane load blocks
  const int v = args->chains >= 2 ? 2 : (args->block_bytes >= 128 ? 8 : 4);
#define JRQ_LAUNCH(LE, V) \
  hipLaunchKernelGGL((jrq::crc64_segments_kernel<LE, V>), g, blk, 0, stream, *args)
  if (log_entry) {
    if (v == 2) JRQ_LAUNCH(true, 2);
    else if (v == 8) JRQ_LAUNCH(true, 8);
    else JRQ_LAUNCH(true, 4);
  } else {
    if (v == 2) JRQ_LAUNCH(false, 2);
    else if (v == 8) JRQ_LAUNCH(false, 8);
    else JRQ_LAUNCH(false, 4);
  }
#undef JRQ_LAUNCH
  return hipGetLastError();
}
