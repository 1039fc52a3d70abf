// crc64.hip -- batched CRC-64/ECMA-182 and fused LogEntry.checksum for gfx950.
//
// Replaces, for a whole batch of log entries at once:
//   CrcUtil.crc64(...)      jraft-core/.../util/CrcUtil.java:36-80
//   CRC64.update(...)       jraft-core/.../util/CRC64.java:100-110
//   LogEntry.checksum()     jraft-core/.../entity/LogEntry.java:88-108
//   LogEntry.isCorrupted()  jraft-core/.../entity/LogEntry.java:156-158
//
// Design (DESIGN.md §4.2 has the roofline):
//  * The payload is cut into equal flat SEGMENTS of S bytes (S from the batch size so
//    that every lane of the persistent grid gets ~1 segment); each lane walks its
//    segment entry by entry with a serial table CRC.  Work per lane is the same
//    whatever the entry-length distribution.
//  * The CRC is linear over GF(2) with init 0, so a piece of an entry that ends n bytes
//    before the entry's end contributes crc(piece) * x^(8n) mod P, and the entry's CRC is
//    the XOR of its pieces.  Pieces of entries that straddle a segment boundary are
//    XOR-combined in a scratch slot with agent-scope atomics; the last arriving piece
//    (arrival counter) writes the result and re-zeroes the slot.
//  * Table CRC in the "reversed domain" r = bswap64(crc): a little-endian 8-byte load
//    XORs straight into r (no byte swaps), and one k-byte step is
//      r = (r >> 8k) ^ R_{k-1}[byte 0 of r] ^ ... ^ R_0[byte k-1 of r],
//    R_j = bswap(T_j), T_j[i] = i * x^(64 + 8j) mod P.  Two LDS table flavours:
//      Tab2: slice-by-2, R0/R1 replicated 32x so lane l only touches bank pair l&31
//            (conflict-free): per 2 bytes 2 v_perm + 2 ds_read_b64 + 2 shifts + 2 XOR3.
//      Tab4: slice-by-4, R0..R3 replicated 16x, two tables interleaved per 16-B slot:
//            per 4 bytes 4 v_perm + 4 ds_read_b64 (2-way bank conflicts) + 4 XOR3/XOR,
//            the 32-bit shift is free (register rename); half the dependent LDS round
//            trips per byte of Tab2.
//    Either way an LDS address is one v_perm of a data byte and a lane constant.
//  * The x^(8n) multiplications use byte tables in global memory (one per power of two,
//    L2-resident); they run at most once per piece that does not end its entry.
#include "jrq_device.h"

namespace jrq {

struct RState {
  uint32_t lo, hi;
};

__device__ __forceinline__ uint64_t crc_value(const RState& r) {
  // crc = bswap64(r)
  return (static_cast<uint64_t>(__builtin_bswap32(r.lo)) << 32) | __builtin_bswap32(r.hi);
}

__device__ __forceinline__ uint2 lds_u2(const char* lds, uint32_t addr) {
  return *reinterpret_cast<const uint2*>(lds + addr);
}

// ------------------------------------------------------------ slice-by-2 ---
// LDS image: byte address = table<<16 | index<<8 | (lane&31)<<3 (R0 at 0, R1 at 64 KiB).
struct Tab2 {
  static constexpr uint32_t kSelR1 = 0x0C060004u;  // {lc.b0, lo.b0, lc.b2, 0}
  static constexpr uint32_t kSelR0 = 0x0C0C0104u;  // {lc.b0, lo.b1, 0, 0}
  uint32_t lc;  // byte0 = (lane&31)<<3, byte2 = 1
  __device__ explicit Tab2(uint32_t lane) : lc(((lane & 31u) << 3) | (1u << 16)) {}

  // word w of the image holds R_{w>>13}[(w>>5)&255]
  __device__ static uint32_t src_index(uint32_t w) { return (w >> 13) * 256 + ((w >> 5) & 255u); }

  __device__ __forceinline__ void step2(RState& r, const char* lds) const {
    const uint2 t1 = lds_u2(lds, __builtin_amdgcn_perm(lc, r.lo, kSelR1));
    const uint2 t0 = lds_u2(lds, __builtin_amdgcn_perm(lc, r.lo, kSelR0));
    const uint32_t nlo = __builtin_amdgcn_alignbit(r.hi, r.lo, 16);
    const uint32_t nhi = r.hi >> 16;
    r.lo = xor3(nlo, t1.x, t0.x);
    r.hi = xor3(nhi, t1.y, t0.y);
  }
  // one byte: r = R0[(r ^ b) & 0xFF] ^ (r >> 8)   (CRC64.update(byte), CRC64.java:100-103)
  __device__ __forceinline__ void step1(RState& r, uint32_t b, const char* lds) const {
    const uint2 t0 = lds_u2(lds, __builtin_amdgcn_perm(lc, r.lo ^ b, 0x0C0C0004u));
    const uint32_t nlo = __builtin_amdgcn_alignbit(r.hi, r.lo, 8);
    r.lo = nlo ^ t0.x;
    r.hi = (r.hi >> 8) ^ t0.y;
  }
  // eight bytes as a little-endian (lo, hi) dword pair
  __device__ __forceinline__ void step8(RState& r, uint32_t dlo, uint32_t dhi,
                                        const char* lds) const {
    r.lo ^= dlo;
    r.hi ^= dhi;
    step2(r, lds);
    step2(r, lds);
    step2(r, lds);
    step2(r, lds);
  }
};

// ------------------------------------------------------------ slice-by-4 ---
// LDS image: byte address = (k>>1)<<16 | index<<8 | (lane&15)<<4 | (k&1)<<3 for table R_k
// (16 replicas; R0/R1 share the 16-B slots of the first 64 KiB, R2/R3 of the second).
struct Tab4 {
  uint32_t lc0, lc1, lc2, lc3;  // byte0 = (lane&15)<<4 | (k&1)<<3, byte2 = k>>1
  __device__ explicit Tab4(uint32_t lane)
      : lc0(((lane & 15u) << 4)),
        lc1(((lane & 15u) << 4) | 8u),
        lc2(((lane & 15u) << 4) | (1u << 16)),
        lc3(((lane & 15u) << 4) | 8u | (1u << 16)) {}

  // word w = (k>>1)<<13 | index<<5 | replica<<1 | (k&1)
  __device__ static uint32_t src_index(uint32_t w) {
    return (((w >> 13) << 1) | (w & 1u)) * 256 + ((w >> 5) & 255u);
  }

  // four bytes already XORed into r.lo: r = (r >> 32) ^ R3[b0] ^ R2[b1] ^ R1[b2] ^ R0[b3]
  __device__ __forceinline__ void step4(RState& r, const char* lds) const {
    const uint2 t3 = lds_u2(lds, __builtin_amdgcn_perm(lc3, r.lo, 0x0C060004u));
    const uint2 t2 = lds_u2(lds, __builtin_amdgcn_perm(lc2, r.lo, 0x0C060104u));
    const uint2 t1 = lds_u2(lds, __builtin_amdgcn_perm(lc1, r.lo, 0x0C060204u));
    const uint2 t0 = lds_u2(lds, __builtin_amdgcn_perm(lc0, r.lo, 0x0C060304u));
    r.lo = xor3(xor3(r.hi, t3.x, t2.x), t1.x, t0.x);
    r.hi = xor3(t3.y, t2.y, t1.y) ^ t0.y;
  }
  __device__ __forceinline__ void step1(RState& r, uint32_t b, const char* lds) const {
    const uint2 t0 = lds_u2(lds, __builtin_amdgcn_perm(lc0, r.lo ^ b, 0x0C060004u));
    const uint32_t nlo = __builtin_amdgcn_alignbit(r.hi, r.lo, 8);
    r.lo = nlo ^ t0.x;
    r.hi = (r.hi >> 8) ^ t0.y;
  }
  __device__ __forceinline__ void step8(RState& r, uint32_t dlo, uint32_t dhi,
                                        const char* lds) const {
    r.lo ^= dlo;
    r.hi ^= dhi;
    step4(r, lds);
    step4(r, lds);
  }
};

template <class Tab>
__device__ __forceinline__ void step16(const Tab& tb, RState& r, const uint4& v, const char* lds) {
  tb.step8(r, v.x, v.y, lds);
  tb.step8(r, v.z, v.w, lds);
}

// CRC of payload[a, b) from a zero register, one chain.
// Blocks of 16*BV bytes go through a 2-deep register ring: block i+1's loads are issued
// before block i is hashed, unconditionally (address clamped to the last block), so the
// compiler's wait before block i is a counted vmcnt(BV), not vmcnt(0).  Unrolled by two
// with fixed buffer roles: a loaded register is never copied (a copy would force the wait
// early).  The empty asm after each load group is a compiler memory barrier: the loads
// may not be re-issued (rematerialised) at their use a block later; it implies no
// hardware wait.  BV = 8 reads whole 128-B lines per lane.
template <class Tab, int BV>
__device__ __forceinline__ uint64_t crc_range(const Tab& tb, const uint8_t* __restrict__ payload,
                                              uint64_t a, uint64_t b, const char* lds) {
  RState r{0u, 0u};
  uint64_t p = a;
  const uint64_t mis = reinterpret_cast<uintptr_t>(payload) & 15u;
  while (p < b && ((p + mis) & 15u)) {  // unaligned head (by address), byte-serial
    tb.step1(r, payload[p], lds);
    ++p;
  }
  constexpr uint32_t kBlkBytes = 16u * BV;
  const uint64_t nblk = (b - p) / kBlkBytes;
  if (nblk != 0) {
    const uint4* q = reinterpret_cast<const uint4*>(payload + p);
    const uint64_t last = nblk - 1;
    uint4 A[BV], B[BV];
#define JRQ_LOAD(X, blk)                                             \
  do {                                                               \
    const uint64_t bb = (blk) < last ? (blk) : last;                 \
    const uint4* qq = q + BV * bb;                                   \
    _Pragma("unroll") for (int v = 0; v < BV; ++v) X[v] = qq[v];     \
    asm volatile("" ::: "memory");                                   \
  } while (0)
#define JRQ_HASH(X)                                                             \
  do {                                                                          \
    _Pragma("unroll") for (int v = 0; v < BV; ++v) step16(tb, r, X[v], lds);    \
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
    step16(tb, r, *reinterpret_cast<const uint4*>(payload + p), lds);
    p += 16;
  }
  while (p < b) {  // tail, byte-serial
    tb.step1(r, payload[p], lds);
    ++p;
  }
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

// Two independent chains per lane: [a, b) is cut at m into halves hashed in lockstep
// (one chain's LDS latency hides under the other's), then crc = crc(X) * x^(8|Y|) ^ crc(Y).
// 64-B blocks with a 2-deep register ring per chain; X takes the unaligned head first, Y
// the tail last.  Short ranges fall back to one chain.
template <class Tab>
__device__ __forceinline__ uint64_t crc_range2(const Tab& tb, const uint8_t* __restrict__ payload,
                                               uint64_t a, uint64_t b, const char* lds,
                                               const uint64_t* __restrict__ shift) {
  constexpr uint64_t kBB = 64;
  if (b - a < 4 * kBB) return crc_range<Tab, 4>(tb, payload, a, b, lds);
  RState x{0u, 0u}, y{0u, 0u};
  uint64_t p = a;
  const uint64_t mis = reinterpret_cast<uintptr_t>(payload) & 15u;
  while (p < b && ((p + mis) & 15u)) {
    tb.step1(x, payload[p], lds);
    ++p;
  }
  const uint64_t nb = (b - p) / (2 * kBB);  // blocks per chain (>= 1 here)
  const uint64_t m = p + nb * kBB;
  const uint4* qx = reinterpret_cast<const uint4*>(payload + p);
  const uint4* qy = reinterpret_cast<const uint4*>(payload + m);
  const uint64_t last = nb - 1;
  uint4 XA[4], XB[4], YA[4], YB[4];
#define JRQ_LOAD2(X, Y, blk)                                             \
  do {                                                                   \
    const uint64_t bb = (blk) < last ? (blk) : last;                     \
    _Pragma("unroll") for (int v = 0; v < 4; ++v) X[v] = qx[4 * bb + v]; \
    _Pragma("unroll") for (int v = 0; v < 4; ++v) Y[v] = qy[4 * bb + v]; \
    asm volatile("" ::: "memory");                                       \
  } while (0)
#define JRQ_HASH2(X, Y)                           \
  do {                                            \
    _Pragma("unroll") for (int v = 0; v < 4; ++v) { \
      tb.step8(x, X[v].x, X[v].y, lds);           \
      tb.step8(y, Y[v].x, Y[v].y, lds);           \
      tb.step8(x, X[v].z, X[v].w, lds);           \
      tb.step8(y, Y[v].z, Y[v].w, lds);           \
    }                                             \
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
  uint64_t q = m + nb * kBB;  // Y continues over the tail
  while (q + 16 <= b) {
    step16(tb, y, *reinterpret_cast<const uint4*>(payload + q), lds);
    q += 16;
  }
  while (q < b) {
    tb.step1(y, payload[q], lds);
    ++q;
  }
  return crc_shift(crc_value(x), b - m, shift) ^ crc_value(y);
}

// LogId.checksum(): crc64(BE64(index) || BE64(term))  (LogId.java:45-50, Bits.java:71-80).
// The big-endian bytes, read as a little-endian u64, are bswap64(v).
template <class Tab>
__device__ __forceinline__ uint64_t logid_crc(const Tab& tb, int64_t index, int64_t term,
                                              const char* lds) {
  RState r{0u, 0u};
  const uint64_t bi = bswap64(static_cast<uint64_t>(index));
  const uint64_t bt = bswap64(static_cast<uint64_t>(term));
  tb.step8(r, static_cast<uint32_t>(bi), static_cast<uint32_t>(bi >> 32), lds);
  tb.step8(r, static_cast<uint32_t>(bt), static_cast<uint32_t>(bt >> 32), lds);
  return crc_value(r);
}

template <bool kLogEntry, class Tab>
__device__ __forceinline__ uint64_t entry_fields(const Tab& tb, const JrqCrcArgs& a, uint32_t e,
                                                 const char* lds) {
  if (!kLogEntry) return 0;
  // LogEntry.checksum: type.getNumber() ^ id.checksum() ^ peers' checksums (LogEntry.java:89-94)
  uint64_t f = static_cast<uint64_t>(a.type[e]) ^ logid_crc(tb, a.index[e], a.term[e], lds);
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

// Kernel variants (A/B knobs, include/jrq.h engine notes):
//   kV2B4  Tab2, one chain, 64-B blocks      kV2B8  Tab2, one chain, 128-B blocks
//   kV2C2  Tab2, two chains                  kV4B8  Tab4, one chain, 128-B blocks
//   kV4C2  Tab4, two chains
enum : int { kV2B4 = 0, kV2B8 = 1, kV2C2 = 2, kV4B8 = 3, kV4C2 = 4 };

template <int kVariant>
struct VariantTab {
  using type = Tab2;
};
template <>
struct VariantTab<kV4B8> {
  using type = Tab4;
};
template <>
struct VariantTab<kV4C2> {
  using type = Tab4;
};

template <int kVariant, class Tab>
__device__ __forceinline__ uint64_t crc_piece(const Tab& tb, const JrqCrcArgs& a, uint64_t lo,
                                              uint64_t hi, const char* lds) {
  if (kVariant == kV2C2 || kVariant == kV4C2) return crc_range2(tb, a.payload, lo, hi, lds, a.shift);
  if (kVariant == kV2B4) return crc_range<Tab, 4>(tb, a.payload, lo, hi, lds);
  return crc_range<Tab, 8>(tb, a.payload, lo, hi, lds);
}

template <bool kLogEntry, int kVariant>
__global__ __launch_bounds__(kCrcBlock) void crc64_segments_kernel(JrqCrcArgs a) {
  using Tab = typename VariantTab<kVariant>::type;
  __shared__ __attribute__((aligned(16))) uint64_t lds_tab[kCrcLdsBytes / 8];
  const char* lds = reinterpret_cast<const char*>(lds_tab);

  // Build the replicated LDS image of the slice tables (a.slice = R0, R1, R2, R3).
  for (uint32_t w = threadIdx.x; w < kCrcLdsBytes / 8; w += blockDim.x)
    lds_tab[w] = a.slice[Tab::src_index(w)];
  __syncthreads();

  const Tab tb(threadIdx.x & 63u);

  const uint64_t base = a.offsets[0];
  const uint64_t total = a.offsets[a.n] - base;
  const uint64_t lanes = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  // Segment size S ~ total/lanes (>= 2^min_seg_log2).  seg_mode 0: a power of two (the
  // measured best); 1: an odd multiple of 64 B (A/B alternative); seg_bytes: fixed.
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
      uint64_t c = crc_piece<kVariant>(tb, a, s0, pe, lds);
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
      const uint64_t fields = entry_fields<kLogEntry>(tb, a, e, lds);
      uint64_t c = crc_piece<kVariant>(tb, a, oe, pe, lds);
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

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_crc64(
    const JrqCrcArgs* args, int log_entry, int grid, hipStream_t stream) {
  const dim3 g(grid), blk(jrq::kCrcBlock);
  using namespace jrq;
  const bool t4 = args->tables >= 4;
  const int v = args->chains >= 2 ? (t4 ? kV4C2 : kV2C2)
                                  : (t4 ? kV4B8 : (args->block_bytes >= 128 ? kV2B8 : kV2B4));
#define JRQ_LAUNCH(LE, V) \
  hipLaunchKernelGGL((crc64_segments_kernel<LE, V>), g, blk, 0, stream, *args)
#define JRQ_VARIANTS(LE)                 \
  switch (v) {                           \
    case kV2B4: JRQ_LAUNCH(LE, kV2B4); break; \
    case kV2B8: JRQ_LAUNCH(LE, kV2B8); break; \
    case kV2C2: JRQ_LAUNCH(LE, kV2C2); break; \
    case kV4B8: JRQ_LAUNCH(LE, kV4B8); break; \
    default: JRQ_LAUNCH(LE, kV4C2); break;    \
  }
  if (log_entry) {
    JRQ_VARIANTS(true)
  } else {
    JRQ_VARIANTS(false)
  }
#undef JRQ_VARIANTS
#undef JRQ_LAUNCH
  return hipGetLastError();
}
