// crc64.hip -- batched CRC-64/ECMA-182 and fused LogEntry.checksum for gfx950.
//
// Replaces, for a whole batch of log entries at once:
//   CrcUtil.crc64(...)      jraft-core/.../util/CrcUtil.java:36-80
//   CRC64.update(...)       jraft-core/.../util/CRC64.java:100-110
//   LogEntry.checksum()     jraft-core/.../entity/LogEntry.java:88-108
//   LogEntry.isCorrupted()  jraft-core/.../entity/LogEntry.java:156-158
//
// Design (DESIGN.md §4.2 has the roofline and the probe numbers behind each choice):
//  * Flat segments.  The payload window is cut into equal SEGMENTS of S bytes (a multiple of
//    256, S ~ total / lanes of the persistent grid); each lane owns one segment and walks the
//    entries inside it in order, so the work per lane does not depend on the entry lengths.
//    CRC64 here is linear over GF(2) (init 0, xorout 0): a piece of an entry that ends n bytes
//    before the entry's end contributes crc(piece) * x^(8n) mod P, and the entry's CRC is the
//    XOR of its pieces.  Pieces of entries that span segments meet in a scratch slot through
//    agent-scope atomics; the last arriving piece writes the result and re-zeroes the slot.
//  * Coalesced row-group loads + row-swap transpose.  A lane reading only its own segment
//    touches 64 different cache lines per wave instruction and streams at ~4.8 TB/s at best;
//    instead the 4 lanes {c, c+16, c+32, c+48} read 64 contiguous bytes of ONE owner per
//    instruction (4 loads = 64 B per lane per half-round, every owner's 64 B in full), and a
//    2-stage butterfly of v_permlane16_swap / v_permlane32_swap (16 swaps per half-round,
//    no selects) hands every lane its own 4 pieces.  Half-rounds run through a 3-deep
//    register ring; buffer loads with a per-wave descriptor clamp reads past the data to 0.
//  * Table CRC in the "reversed domain" r = bswap64(crc): a little-endian load XORs straight
//    into r, and 8 bytes are one step  r = R7[b0] ^ R6[b1] ^ ... ^ R0[b7] (slice-by-8, Tab8),
//    R_j = bswap(T_j),
//    T_j[i] = i * x^(64 + 8j) mod P.  The tables live in LDS, replicated 8x, and the 4 lanes
//    sharing a replica visit its tables in 4 rotations, so every ds_read_b64 is bank-conflict
//    free.  An LDS address is one v_perm of a data byte and a per-lane constant.
//  * Entry boundaries are events: a round that lies inside one entry is hashed from the
//    registers; a round holding a boundary or the data edge is finished from global memory
//    (L2-hot) byte/16-B wise, then the entry is emitted (or its piece handed off).
//  * The x^(8n) multiplications use byte tables in global memory (one per power of two,
//    L2-resident); they run at most once per piece that does not end its entry.
#include "jrq_device.h"

#ifndef JRQ_CRC_LOAD_AUX
#define JRQ_CRC_LOAD_AUX 0  // cache-policy bits of the half-line ring loads (2 = nt on gfx950)
#endif
#ifndef JRQ_CRC_LINE_AUX
// cache-policy bits of the full-line ring loads: every instruction reads whole 128-B lines, so
// nothing else wants the line afterwards and `nt` streams it (DESIGN.md §4.2 "Cache policy")
#define JRQ_CRC_LINE_AUX 2
#endif


namespace jrq {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

// ------------------------------------------------------------ slice-by-8 ---
// 8 bytes per step: r = R7[b0] ^ R6[b1] ^ R5[b2] ^ R4[b3] ^ R3[b4] ^ R2[b5] ^ R1[b6] ^ R0[b7]
// (b0..b3 = r.lo, b4..b7 = r.hi after the data XOR).  Half as many dependent LDS round
// trips per byte as slice-by-4 at the same VALU count per byte.
// LDS image, 8 replicas: byte address = g<<16 | index<<8 | replica<<5 | p<<3 holds R_{4g+p}
// (g = 1: tables R4..R7, used with r.lo; g = 0: R0..R3, used with r.hi; p = 3 - byte).
// Conflict-free ds_read_b64: in a 32-lane group the 4 lanes sharing a replica (lane & 7) are
// its 4 rotations rot = (lane >> 3) & 3, and instruction i reads table position
// p = (i + rot) & 3 -- all 32 lanes on distinct bank pairs.  The rotation is one v_perm of
// each state word (swz), so the address v_perm's byte selector stays an immediate.
struct Tab8 {
  uint32_t lc[4];  // instruction i: b0 = replica<<5 | p_i<<3, b1 = 1 (g = 1), b2 = 0 (g = 0)
  uint32_t swz;    // v_perm selector: byte i of x = byte 3 - p_i of the word
  __device__ explicit Tab8(uint32_t lane) {
    const uint32_t rep = lane & 7u, rot = (lane >> 3) & 3u;
    swz = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t p = (static_cast<uint32_t>(i) + rot) & 3u;
      lc[i] = (rep << 5) | (p << 3) | (1u << 8);
      swz |= (3u - p) << (8 * i);
    }
  }

  // word w = g<<13 | index<<5 | replica<<2 | p  ->  R_{4g+p}[index]
  __device__ static uint32_t src_index(uint32_t w) {
    return (((w >> 13) << 2) | (w & 3u)) * 256 + ((w >> 5) & 255u);
  }

  // eight bytes already XORed into r; the new r.lo / r.hi also take the words wl / wh (the
  // next step's data, folded into the XOR trees)
  __device__ __forceinline__ void step8w(RState& r, uint32_t wl, uint32_t wh,
                                         const char* lds) const {
    const uint32_t xl = __builtin_amdgcn_perm(r.lo, r.lo, swz);
    const uint32_t xh = __builtin_amdgcn_perm(r.hi, r.hi, swz);
    const uint2 t0 = lds_u2(lds, __builtin_amdgcn_perm(lc[0], xl, 0x0C050004u));
    const uint2 t1 = lds_u2(lds, __builtin_amdgcn_perm(lc[1], xl, 0x0C050104u));
    const uint2 t2 = lds_u2(lds, __builtin_amdgcn_perm(lc[2], xl, 0x0C050204u));
    const uint2 t3 = lds_u2(lds, __builtin_amdgcn_perm(lc[3], xl, 0x0C050304u));
    const uint2 u0 = lds_u2(lds, __builtin_amdgcn_perm(lc[0], xh, 0x0C060004u));
    const uint2 u1 = lds_u2(lds, __builtin_amdgcn_perm(lc[1], xh, 0x0C060104u));
    const uint2 u2 = lds_u2(lds, __builtin_amdgcn_perm(lc[2], xh, 0x0C060204u));
    const uint2 u3 = lds_u2(lds, __builtin_amdgcn_perm(lc[3], xh, 0x0C060304u));
    r.lo = xor3(xor3(xor3(t0.x, t1.x, t2.x), t3.x, u0.x), xor3(u1.x, u2.x, u3.x), wl);
    r.hi = xor3(xor3(xor3(t0.y, t1.y, t2.y), t3.y, u0.y), xor3(u1.y, u2.y, u3.y), wh);
  }
  __device__ __forceinline__ void step8(RState& r, uint32_t dlo, uint32_t dhi,
                                        const char* lds) const {
    r.lo ^= dlo;
    r.hi ^= dhi;
    step8w(r, 0u, 0u, lds);
  }
  // one byte: r = R0[(r ^ b) & 0xFF] ^ (r >> 8)   (CRC64.update(byte), CRC64.java:100-103)
  __device__ __forceinline__ void step1(RState& r, uint32_t b, const char* lds) const {
    const uint32_t lc0 = lc[0] & 0xE0u;  // this lane's replica of R0 (g = 0, p = 0)
    const uint2 t0 = lds_u2(lds, __builtin_amdgcn_perm(lc0, r.lo ^ b, 0x0C060004u));
    const uint32_t nlo = __builtin_amdgcn_alignbit(r.hi, r.lo, 8);
    r.lo = nlo ^ t0.x;
    r.hi = (r.hi >> 8) ^ t0.y;
  }
  // 64 bytes = 8 steps; words 2s+2, 2s+3 ride step s's XOR trees
  __device__ __forceinline__ void step64(RState& r, const u32x4 (&v)[4], const char* lds) const {
    r.lo ^= v[0][0];
    r.hi ^= v[0][1];
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int wl = 2 * s + 2, wh = 2 * s + 3;
      step8w(r, v[wl >> 2][wl & 3], v[wh >> 2][wh & 3], lds);
    }
    step8w(r, 0u, 0u, lds);
  }
};

using CrcTab = Tab8;

// -------------------------------------------------------- row transpose ---
// The four lanes {c, c+16, c+32, c+48} of a wave (one per 16-lane row) read the 64
// contiguous bytes of one owner segment per load instruction: load q of the lane in row i
// holds piece i (16 B at 16i) of owner lane 16q + c.  Two butterfly stages of gfx950's
// row-swap instructions turn that back into "register j = piece j of this lane's own
// segment"; each swap exchanges one register pair in place, no lane selects.
//   stage 1 (row bit 0): v_permlane16_swap  -- odd rows of a <-> even rows of b
//   stage 2 (row bit 1): v_permlane32_swap  -- rows 2,3 of a <-> rows 0,1 of b
__device__ __forceinline__ void swap16(u32x4& a, u32x4& b) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const auto r = __builtin_amdgcn_permlane16_swap(a[c], b[c], false, false);
    a[c] = r[0];
    b[c] = r[1];
  }
}
__device__ __forceinline__ void swap32(u32x4& a, u32x4& b) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const auto r = __builtin_amdgcn_permlane32_swap(a[c], b[c], false, false);
    a[c] = r[0];
    b[c] = r[1];
  }
}
// Must run with the whole wave active (the swaps read the partner rows).
__device__ __forceinline__ void row_transpose(u32x4& a0, u32x4& a1, u32x4& a2, u32x4& a3) {
  swap16(a0, a1);
  swap16(a2, a3);
  swap32(a0, a2);
  swap32(a1, a3);
}

// The same, pinned below the loads issued before it (the asm keeps the scheduler from
// hoisting the memory-free swaps and draining the prefetch with vmcnt(0)).
__device__ __forceinline__ void transpose_ring(u32x4 (&v)[4]) {
  asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
  row_transpose(v[0], v[1], v[2], v[3]);
}

// ------------------------------------------------------- line transpose ---
// Full-line shape: load q (0..7) of lane L = 8p + c reads 16-B piece p of the 128-B line of
// owner lane c + 8q, so each instruction reads 8 owners x 128 B, whole lines (no line is
// split across instructions; with `nt` loads a line read half by one instruction and half by
// the next was evicted in between).  Loads 0..3 land in a[0..3], 4..7 in
// b[0..3].  Three butterfly stages swap lane bit 5 / 4 / 3 with register bit 2 / 1 / 0, after
// which lane o holds its own line: a = bytes 0..63, b = bytes 64..127.
//   lane bit 5: v_permlane32_swap   (a[i] <-> b[i])
//   lane bit 4: v_permlane16_swap   (x[0] <-> x[2], x[1] <-> x[3])
//   lane bit 3: two DPP row_ror:8 moves with bank masks (x[0] <-> x[1], x[2] <-> x[3]): lanes
//               with bit 3 clear take their partner's even register into their odd one, lanes
//               with bit 3 set their partner's odd register into their even one.
__device__ __forceinline__ void swap8(uint32_t& a, uint32_t& b) {
  const uint32_t a0 = a, b0 = b;
  b = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(b0), static_cast<int>(a0),
                                                        0x128 /* row_ror:8 */, 0xF, 0x3, false));
  a = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(a0), static_cast<int>(b0),
                                                        0x128, 0xF, 0xC, false));
}
__device__ __forceinline__ void swap8v(u32x4& a, u32x4& b) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    uint32_t x = a[c], y = b[c];
    swap8(x, y);
    a[c] = x;
    b[c] = y;
  }
}
// Must run with the whole wave active.  The asm pin keeps the swaps below the loads issued
// before them (the scheduler would otherwise hoist them and drain the ring with vmcnt(0)).
__device__ __forceinline__ void transpose_line(u32x4 (&a)[4], u32x4 (&b)[4]) {
  asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]),
               "+v"(b[2]), "+v"(b[3]));
#pragma unroll
  for (int i = 0; i < 4; ++i) swap32(a[i], b[i]);
  swap16(a[0], a[2]);
  swap16(a[1], a[3]);
  swap16(b[0], b[2]);
  swap16(b[1], b[3]);
  swap8v(a[0], a[1]);
  swap8v(a[2], a[3]);
  swap8v(b[0], b[1]);
  swap8v(b[2], b[3]);
}

// --------------------------------------------------------------- helpers ---

// Continue r over virtual bytes [p, q) read from global memory (A = address of virtual byte
// 0, 16-B aligned).  Slow path: rounds that hold an entry boundary or the data edge.
__device__ __forceinline__ void hash_global(const CrcTab& tb, RState& r, const uint8_t* __restrict__ A,
                                            uint64_t p, uint64_t q, const char* lds) {
  while (p < q && (p & 15u)) {
    tb.step1(r, A[p], lds);
    ++p;
  }
  while (p + 16 <= q) {
    const uint4 v = *reinterpret_cast<const uint4*>(A + p);
    tb.step8(r, v.x, v.y, lds);
    tb.step8(r, v.z, v.w, lds);
    p += 16;
  }
  while (p < q) {
    tb.step1(r, A[p], lds);
    ++p;
  }
}

// Bytes [p, q) (0 <= p < q <= 64) of the lane's current half-round, from its registers (the
// transposed ring slot: dword w of the half = v[w >> 2][w & 3]).  Whole 8-byte words inside
// the range take one slice-by-8 step, the partial words at the range's ends go byte by byte.
__device__ __forceinline__ void hash_regs(const CrcTab& tb, RState& r, const u32x4 (&v)[4],
                                          uint32_t p, uint32_t q, const char* lds) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t w0 = v[k >> 1][(k & 1) * 2], w1 = v[k >> 1][(k & 1) * 2 + 1];
    const uint32_t b = 8u * k, e = b + 8u;
    if (p <= b && e <= q) {
      tb.step8(r, w0, w1, lds);
    } else if (p < e && b < q) {
      const uint32_t lo = p > b ? p : b, hi = q < e ? q : e;
      for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t sh = (i - b) * 8u;
        tb.step1(r, (sh < 32 ? (w0 >> sh) : (w1 >> (sh - 32))) & 0xFFu, lds);
      }
    }
  }
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

// Data CRC of entry e is final: plain batches are done; LogEntry batches get their fields
// from logentry_fields_kernel afterwards (in place).
__device__ __forceinline__ void emit(const JrqCrcArgs& a, uint32_t e, uint64_t v) { a.out[e] = v; }

// Read-XOR-arrive on one accumulator slot: XOR c into acc, then count the arrival; the
// arrival that completes `parts` gets the accumulated value back (and re-zeroes the slot).
// Hand-off = 8-byte agent-scope atomics on both sides (MI355X_MICROARCH.md, visibility
// "valid forms"): the XOR is drained (s_waitcnt vmcnt(0)) before the arrival add, the last
// arriver reads the slot with an atomic after its add returned.  No release/acquire
// fences: those would write back the XCD's L2 / invalidate L1 on every piece.
__device__ __forceinline__ bool arrive_xor(uint64_t* acc, uint32_t* cnt, uint32_t parts,
                                           uint64_t c, uint64_t* v, uint32_t n = 1) {
  __hip_atomic_fetch_xor(acc, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t arrived = __hip_atomic_fetch_add(cnt, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (arrived + n != parts) return false;
  // read-and-zero in one memory-side RMW (an xor-with-0 would be folded into a load)
  *v = __hip_atomic_exchange(acc, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // settle the exchange here: its result is consumed on some paths only, and a returning
  // load still pending where those paths join the ring loop made the compiler guard every
  // later write of its register (a step temp) with a vmcnt wait on the payload ring
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  return true;
}

// One piece (segment k) of an entry spanning segments [first, first + parts) with parts >
// kMaxSlotParts.  Two levels, so no slot sees more than 64 arrivals: the pieces of one
// 64-segment group meet in a group slot (acc/cnt + scratch_len; key 2*group + 1 for the
// entry's first group, 2*group otherwise -- a group is touched by at most one long entry
// ending in it and one starting in it), and each group's last arriver carries the group XOR
// to the entry slot acc[first] -- through a third, supergroup level (64 groups, same keying)
// when the entry spans more than 64 groups.  A single 1 GiB entry (a snapshot archive) otherwise put
// every segment's atomics on one address: 3.5 ms instead of ~0.2 ms.
__device__ __forceinline__ void straddle_piece(const JrqCrcArgs& a, uint32_t e, uint64_t first,
                                               uint64_t parts, uint64_t k, uint64_t c) {
  const uint64_t last = first + parts - 1;
  const uint64_t grp = k >> 6, fg = first >> 6, lg = last >> 6;
  const uint64_t lo = first > (grp << 6) ? first : (grp << 6);
  const uint64_t hi = last < (grp << 6) + 63 ? last : (grp << 6) + 63;
  const uint64_t key = 2 * grp + (grp == fg ? 1 : 0);
  // A whole wave handing off pieces of one entry (the wave's 64 segments are one group, as
  // chunks start on 64-segment boundaries): XOR them across lanes and arrive once with 64.
  // A snapshot archive hits this at every wave's end; 64 same-address atomics per wave
  // instruction otherwise serialize at the memory-side atomic unit.
  uint32_t n = 1;
  if (__builtin_amdgcn_read_exec() == ~0ull &&
      __ballot(e == __builtin_amdgcn_readfirstlane(e)) == ~0ull) {
    uint32_t clo = static_cast<uint32_t>(c), chi = static_cast<uint32_t>(c >> 32);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      clo ^= __shfl_xor(clo, o);
      chi ^= __shfl_xor(chi, o);
    }
    if (__lane_id() != 0) return;
    c = (static_cast<uint64_t>(chi) << 32) | clo;
    n = 64;
  }
  uint64_t v;
  if (!arrive_xor(a.acc + a.scratch_len + key, a.cnt + a.scratch_len + key,
                  static_cast<uint32_t>(hi - lo + 1), c, &v, n))
    return;
  uint64_t entry_parts = lg - fg + 1;
  if (entry_parts > 64) {  // > 64 groups (a GiB-scale archive): 64-group supergroup level
    const uint64_t l1 = 2 * (static_cast<uint64_t>(a.scratch_len) / 64 + 2);
    const uint64_t sg = grp >> 6, fsg = fg >> 6, lsg = lg >> 6;
    const uint64_t glo = fg > (sg << 6) ? fg : (sg << 6);
    const uint64_t ghi = lg < (sg << 6) + 63 ? lg : (sg << 6) + 63;
    const uint64_t key2 = a.scratch_len + l1 + 2 * sg + (sg == fsg ? 1 : 0);
    if (!arrive_xor(a.acc + key2, a.cnt + key2, static_cast<uint32_t>(ghi - glo + 1), v, &v))
      return;
    entry_parts = lsg - fsg + 1;
  }
  if (arrive_xor(a.acc + first, a.cnt + first, static_cast<uint32_t>(entry_parts), v, &v))
    emit(a, e, v);
}

// First e in [0, n] with off[e] >= x, given off[0] <= x <= off[n].  Probes off[g-1 .. g+1]
// around the interpolated guess g (one round trip when entries are evenly sized), then
// bisects the side that holds the answer.
__device__ __forceinline__ uint32_t interp_lower_bound(const uint64_t* __restrict__ off, uint32_t n,
                                                       uint64_t base, uint64_t total, uint64_t x) {
  if (x <= base) return 0;
  double f = static_cast<double>(x - base) / static_cast<double>(total) * static_cast<double>(n);
  uint32_t g = f >= static_cast<double>(n) ? n : static_cast<uint32_t>(f);
  if (g == 0) g = 1;
  const uint64_t a0 = off[g - 1], a1 = off[g];
  const uint64_t a2 = g < n ? off[g + 1] : ~0ull;
  if (a0 < x && x <= a1) return g;
  if (a1 < x && x <= a2) return g + 1;
  uint32_t lo, hi;
  if (x <= a0) {
    lo = 0;
    hi = g - 1;
  } else {
    lo = g + 2;
    hi = n;
  }
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    if (off[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Per-lane walk of one segment.  Positions are VIRTUAL: byte v of the stream is payload
// offset base - D + v (D = misalignment of payload + base), so segment k = [kS, (k+1)S) and
// virtual 0 is 16-B aligned.  E(e) = virtual start of entry e.  The walk keeps positions
// relative to the segment start in 32 bits (S < 2^31; boundaries past 2^32 clamp).
struct SegWalk {
  uint32_t pos;      // next byte to hash
  uint32_t next;     // next event: min(cur_end, hi)
  uint32_t hi;       // min(S, data end)
  uint32_t cur;      // entry being hashed (or next to start)
  uint32_t cur_end;  // E(cur + 1)
  uint32_t flags;
  static constexpr uint32_t kStarted = 1, kLastSeg = 2, kDone = 4;
};

// kRegs: a half-round holding an entry boundary hashes its bytes from the ring registers
// (hash_regs) instead of re-reading them from L2 (hash_global).  Faster when boundaries are
// frequent and unaligned (V2 records, ragged batches), but the extra live ranges spill a few
// VGPRs at a 128-VGPR budget (1024-thread workgroups), ~9 % on boundary-free aligned batches.
// Entry boundaries of a wave's window, cached in LDS (the rest of the 160 KiB next to the
// 128 KiB of tables): offsets[eb .. eb + kOffWin) of the window's first entry eb, as u32
// bytes from the window start (0xFFFFFFFF: 4 GiB or more past it).  An event then looks its
// next boundary up in LDS instead of global memory: a global load there made every entry end
// wait for the wave's whole in-flight prefetch ring (vmcnt is in order) -- small entries
// (C1, V2 ranges) are all events.
constexpr uint32_t kOffWin = 512;
static_assert(kCrcLdsBytes + (kCrcRegsBlock / 64) * kOffWin * 4 <= 160 * 1024, "LDS budget");

// Workgroup size kBlock (one workgroup per CU: the LDS tables fill it).  The boundary-free
// path runs kCrcBlock = 512 (2 waves per SIMD, 256 VGPRs each), which also holds its share of
// the table image over the first loads (below); 1024 threads (128 VGPRs) spilled the ring and
// the step trees: C1 0.087 -> 0.080 ms at 512 (tools/ab_inproc.py).  The register boundary path
// (V2 records) runs 768 threads (168 VGPRs, no spill; 512 measured 2-3 % slower there).
template <uint32_t kBlock, bool kRegs>
__global__ __launch_bounds__(kBlock) void crc64_rounds_kernel(JrqCrcArgs a) {
  __shared__ __attribute__((aligned(16))) uint64_t lds_tab[kCrcLdsBytes / 8];
  __shared__ uint32_t offwin[kBlock / 64][kOffWin];
  if (a.gate != nullptr && a.gate[0] != 0) return;  // V2: the fixed-size path took the batch
  const char* lds = reinterpret_cast<const char*>(lds_tab);

  // The replicated LDS image of the slice tables: its L2 reads go out first, the LDS writes
  // and the barrier follow once the first chunk's ring loads are out too, so the first
  // payload round trip overlaps the table build instead of waiting behind it (a wave
  // without a first chunk writes its share before leaving; every wave meets the one barrier).
  // (512 threads: 32 words per thread, held in registers over the first loads; the 768-thread
  // shape has no registers to spare and builds the image up front)
  constexpr bool kTabEarly = kBlock == 512;
  constexpr uint32_t kTabWords = kCrcLdsBytes / 8, kTabPer = kTabEarly ? kTabWords / kBlock : 1;
  static_assert(!kTabEarly || kTabWords % kBlock == 0, "table share");
  uint64_t tab_v[kTabPer];
  if (kTabEarly) {
#pragma unroll
    for (uint32_t i = 0; i < kTabPer; ++i)
      tab_v[i] = a.slice[CrcTab::src_index(threadIdx.x + i * kBlock)];
  } else {
    for (uint32_t w = threadIdx.x; w < kTabWords; w += kBlock) lds_tab[w] = a.slice[CrcTab::src_index(w)];
    __syncthreads();
  }
  auto build_tables = [&]() {
    if (!kTabEarly) return;
#pragma unroll
    for (uint32_t i = 0; i < kTabPer; ++i) lds_tab[threadIdx.x + i * kBlock] = tab_v[i];
    __syncthreads();
  };

  const CrcTab tb(threadIdx.x & 63u);
  const uint32_t n = a.n;
  const uint64_t* __restrict__ off = a.offsets;
  const uint64_t base = off[0];
  const uint64_t total = off[n] - base;
  const uintptr_t addr0 = reinterpret_cast<uintptr_t>(a.payload + base);
  const uint64_t D = addr0 & 15u;
  // virtual byte 0 (up to 15 bytes before payload + base, inside the same 16-B granule)
  const uint8_t* A = reinterpret_cast<const uint8_t*>(addr0 - D);
  const uint64_t span = D + total;
  const uint64_t grid = gridDim.x;

  // Lane->segment map: every wave owns 64 CONTIGUOUS segments (its window, 64*S bytes: few
  // DRAM pages and TLB entries per wave), and consecutive 64-segment chunks go round-robin
  // over the workgroups, so small batches still spread over all CUs.
  const uint64_t S = seg_size(a, span);
  const uint64_t nseg = span == 0 ? 1 : (span + S - 1) / S;
  const uint32_t rounds = static_cast<uint32_t>(S / 128);

  // L0 (first lane of the wave) through readfirstlane: the compiler then knows the wave's
  // window and descriptor are uniform (SGPRs; no waterfall loop around each buffer load)
  const uint32_t L = threadIdx.x;
  const uint32_t L0 = __builtin_amdgcn_readfirstlane(L & ~63u);
  const uint32_t WS = static_cast<uint32_t>(S);  // lane-to-lane segment step (window < 2^31)
  const uint32_t lane_off = (L - L0) * WS;       // this lane's segment, relative to the wave's
  // load q of half-round h reads 16 B of owner lane 16q + c at offset 64h + 16*row, so the
  // lanes {c, c+16, c+32, c+48} read 64 contiguous bytes per instruction
  const uint32_t qbase = (L & 15u) * WS + 16u * ((L >> 4) & 3u);
  const uint64_t waves = blockDim.x / 64;
  // Wave priority by progress: the SIMD arbiter otherwise serves its 4 waves oldest-first,
  // so equal shares of work finish at 4 distinct times and the last quarter of the launch
  // runs with few waves in flight.  Waves start at priority 3 and step down at 1/2, 3/4 and
  // 7/8 of their own work (chunk c = j * G + g over all G waves of the grid), letting the
  // waves behind them catch up.
  // (all of it wave-uniform, kept in SGPRs through readfirstlane: VALU temporaries here
  // collided with the prefetch ring's registers and cost a vmcnt(0) per iteration)
  uint32_t prio_lvl = 0, pt0 = ~0u, pt1 = ~0u, pt2 = ~0u;
  if (a.prio_steps) {
    const uint64_t G = grid * waves, C = (nseg + 63) / 64;
    const uint64_t g = a.seg_map ? blockIdx.x * waves + (L0 >> 6) : (L0 >> 6) * grid + blockIdx.x;
    const uint64_t w64 = (g < C ? (C - g + G - 1) / G : 0) * rounds * 2;
    const uint32_t work = __builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(w64 > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : w64));
    pt0 = work / 2;
    pt1 = work - work / 4;
    pt2 = work - work / 8;
    __builtin_amdgcn_s_setprio(3);
  }
  for (uint64_t j = 0;; ++j) {
    const uint64_t kw = a.seg_map ? ((j * grid + blockIdx.x) * waves + (L0 >> 6)) * 64
                                  : ((j * waves + (L0 >> 6)) * grid + blockIdx.x) * 64;
    if (kw >= nseg) {  // wave-uniform
      if (j == 0) build_tables();
      break;
    }
    const uint64_t wbase = kw * S;  // the wave's window starts at its first segment
    const uint64_t k = kw + (L - L0);
    const uint64_t s0 = wbase + lane_off;
    auto E = [&](uint32_t e) -> uint64_t { return off[e] - base + D; };
    auto rel = [&](uint64_t v) -> uint32_t {  // future boundary relative to s0, clamped
      const uint64_t d = v - s0;
      return d > 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(d);
    };
    uint32_t* const win = offwin[L0 >> 6];
    uint32_t eb = 0, wcnt = 0;  // the LDS window: entries [eb, eb + wcnt)
    // rel(E(e)) / E(e) through the window when it holds e
    auto relE = [&](uint32_t e) -> uint32_t {
      const uint32_t i = e - eb;
      if (i < wcnt) {
        const uint32_t v = win[i];
        return v == 0xFFFFFFFFu ? v : v - lane_off;
      }
      return rel(E(e));
    };
    auto absE = [&](uint32_t e) -> uint64_t {
      const uint32_t i = e - eb;
      if (i < wcnt) {
        const uint32_t v = win[i];
        if (v != 0xFFFFFFFFu) return wbase + v;
      }
      return E(e);
    };

    // buffer descriptor: from the wave's first segment to the data end (loads past it
    // return zero).  Its words pass through readfirstlane: the compiler then keeps it in
    // SGPRs (otherwise it may hold it in VGPRs and wrap each load in a waterfall loop).
    const uint64_t nrec = span - wbase;
    const uintptr_t wptr = reinterpret_cast<uintptr_t>(A + wbase);
    const uint32_t wlo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(wptr));
    const uint32_t whi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(wptr >> 32));
    const uint32_t nr = __builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(nrec > 0x7FFFFFFFull ? 0x7FFFFFFFull : nrec));

    // Ring of three half-rounds (64 B per lane each, 16 VGPRs): two in flight while one is
    // hashed.  Half-round h: load q reads 16 B of owner lane 16q + c at segment offset
    // 64h + 16*row, so each row group reads 64 contiguous bytes of one owner per instruction.
    // The boundary-free shape (!kRegs, 512 threads) runs a ring of four, the two halves of a
    // 128-B line loaded back to back (see the loop); the register boundary path (768 threads,
    // 168 VGPRs) keeps three.
    constexpr bool kRing4 = !kRegs;
    u32x4 h0[4], h1[4], h2[4], h3[4];
    // Each half-round's loads use a descriptor whose base is advanced by the half's offset
    // (scalar adds), so the per-lane voffsets stay loop-invariant: no VALU address temps
    // that the register allocator could place on a ring slot still being loaded (such a
    // write-after-write made the compiler wait for the whole ring, vmcnt(0)).
    const uint32_t qa0 = qbase, qa1 = qbase + 16u * WS, qa2 = qbase + 32u * WS,
                   qa3 = qbase + 48u * WS;
    // full-line shape (kRing4): load q reads 16-B piece L >> 3 of owner (L & 7) + 8q's line
    const uint32_t lb = (L & 7u) * WS + 16u * ((L >> 3) & 7u);
    const uint64_t wptr_u = (static_cast<uint64_t>(whi) << 32) | wlo;
#define JRQ_LOAD_HALF(H, hh)                                                             \
  do {                                                                                   \
    const uint32_t ho = __builtin_amdgcn_readfirstlane((hh) * 64u);                      \
    const uint64_t hp = wptr_u + ho;                                                     \
    const uint32_t hlo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(hp));      \
    const uint32_t hhi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(hp >> 32)); \
    uint32_t hn; /* nr - min(ho, nr) on the scalar unit (no VALU temp; see above) */     \
    asm("s_min_u32 %0, %1, %2\n\ts_sub_u32 %0, %2, %0" : "=&s"(hn) : "s"(ho), "s"(nr));   \
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(                 \
        reinterpret_cast<uint8_t*>((static_cast<uint64_t>(hhi) << 32) | hlo),            \
        static_cast<short>(0), static_cast<int>(hn), 0x00020000);                        \
    H[0] = __builtin_amdgcn_raw_buffer_load_b128(rh, qa0, 0, JRQ_CRC_LOAD_AUX);                         \
    H[1] = __builtin_amdgcn_raw_buffer_load_b128(rh, qa1, 0, JRQ_CRC_LOAD_AUX);                         \
    H[2] = __builtin_amdgcn_raw_buffer_load_b128(rh, qa2, 0, JRQ_CRC_LOAD_AUX);                         \
    H[3] = __builtin_amdgcn_raw_buffer_load_b128(rh, qa3, 0, JRQ_CRC_LOAD_AUX);                         \
    asm volatile("" ::: "memory");                                                       \
  } while (0)
#define JRQ_LOAD_LINE(HA, HB, ll)                                                        \
  do {                                                                                   \
    const uint32_t ho = __builtin_amdgcn_readfirstlane((ll) * 128u);                     \
    const uint64_t hp = wptr_u + ho;                                                     \
    const uint32_t hlo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(hp));      \
    const uint32_t hhi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(hp >> 32)); \
    uint32_t hn;                                                                         \
    asm("s_min_u32 %0, %1, %2\n\ts_sub_u32 %0, %2, %0" : "=&s"(hn) : "s"(ho), "s"(nr));   \
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(                 \
        reinterpret_cast<uint8_t*>((static_cast<uint64_t>(hhi) << 32) | hlo),            \
        static_cast<short>(0), static_cast<int>(hn), 0x00020000);                        \
    HA[0] = __builtin_amdgcn_raw_buffer_load_b128(rh, lb, 0, JRQ_CRC_LINE_AUX);          \
    HA[1] = __builtin_amdgcn_raw_buffer_load_b128(rh, lb + 8u * WS, 0, JRQ_CRC_LINE_AUX); \
    HA[2] = __builtin_amdgcn_raw_buffer_load_b128(rh, lb + 16u * WS, 0, JRQ_CRC_LINE_AUX); \
    HA[3] = __builtin_amdgcn_raw_buffer_load_b128(rh, lb + 24u * WS, 0, JRQ_CRC_LINE_AUX); \
    HB[0] = __builtin_amdgcn_raw_buffer_load_b128(rh, lb + 32u * WS, 0, JRQ_CRC_LINE_AUX); \
    HB[1] = __builtin_amdgcn_raw_buffer_load_b128(rh, lb + 40u * WS, 0, JRQ_CRC_LINE_AUX); \
    HB[2] = __builtin_amdgcn_raw_buffer_load_b128(rh, lb + 48u * WS, 0, JRQ_CRC_LINE_AUX); \
    HB[3] = __builtin_amdgcn_raw_buffer_load_b128(rh, lb + 56u * WS, 0, JRQ_CRC_LINE_AUX); \
    asm volatile("" ::: "memory");                                                       \
  } while (0)
    // the ring's first two half-rounds go out before the segment setup: the setup's dependent
    // lookups (entry search, boundary window) then overlap the payload fetch instead of
    // leaving HBM idle at the start of every chunk (short segments: C1, V2)
    if constexpr (kRing4) {
      JRQ_LOAD_LINE(h0, h1, 0u);
    } else {
      JRQ_LOAD_HALF(h0, 0u);
      JRQ_LOAD_HALF(h1, 1u);
    }
    if (j == 0) build_tables();

    // ---- segment setup ----
    SegWalk sw;
    RState r{0u, 0u};
    sw.flags = SegWalk::kStarted | (k + 1 == nseg ? SegWalk::kLastSeg : 0u) |
               (k < nseg ? 0u : SegWalk::kDone);
    sw.hi = static_cast<uint32_t>(span - s0 < S ? span - s0 : S);
    sw.pos = static_cast<uint32_t>(s0 < D ? D - s0 : 0);
    sw.cur = 0;
    sw.next = 0;
    sw.cur_end = 0;
    // entry cur starts at pos: skip (emit) zero-length entries there -- they belong to the
    // segment holding pos, the last segment also owning those at the data end -- then arm
    // the next event.  The boundary is loaded here, not prefetched an entry ahead: a load
    // still in flight across ring iterations made the compiler drain the whole prefetch
    // ring (vmcnt(0)) at the top of every iteration.
    auto start_entry = [&]() {
      while (sw.cur < n) {
        sw.cur_end = relE(sw.cur + 1);
        if (sw.cur_end != sw.pos || !(sw.pos < S || (sw.flags & SegWalk::kLastSeg))) break;
        emit(a, sw.cur, 0);  // crc64 of no bytes
        ++sw.cur;
      }
      if (sw.cur >= n || sw.pos >= sw.hi) {
        sw.flags |= SegWalk::kDone;
      } else {
        sw.next = sw.cur_end < sw.hi ? sw.cur_end : sw.hi;
      }
    };
    uint32_t e0 = 0;
    if (!(sw.flags & SegWalk::kDone))
      e0 = interp_lower_bound(off, n, base, total, s0 + sw.pos - D + base);
    // fill the wave's LDS window from its first lane's entry (lane 0 is never done here: the
    // chunk's first segment exists), one coalesced pass of up to kOffWin offsets -- as many as
    // the window's 64 segments hold at the batch's mean entry size, plus a wave of margin
    // (boundaries past the window fall back to global loads: slower, same result)
    eb = __builtin_amdgcn_readfirstlane(e0);  // wave-uniform (SGPRs): every lane is active
    {
      const double est = static_cast<double>(64 * S) / static_cast<double>(total ? total : 1) *
                         static_cast<double>(n) + 65.0;
      uint32_t c = n + 1 - eb < kOffWin ? n + 1 - eb : kOffWin;
      if (est < static_cast<double>(c)) c = static_cast<uint32_t>(est);
      wcnt = __builtin_amdgcn_readfirstlane(c);
    }
    for (uint32_t i = L - L0; i < wcnt; i += 64) {
      const uint64_t d = E(eb + i) - wbase;
      win[i] = d > 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(d);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!(sw.flags & SegWalk::kDone)) {
      const uint32_t e = e0;
      if (e > 0 && absE(e) > s0 + sw.pos) {  // entry e-1 began in an earlier segment
        sw.cur = e - 1;
        sw.flags &= ~SegWalk::kStarted;
        sw.cur_end = relE(e);
        sw.next = sw.cur_end < sw.hi ? sw.cur_end : sw.hi;
      } else {
        sw.cur = e;
        start_entry();
      }
    }

    // An event at pos == next: the entry ends (emit / hand off its tail piece), or the
    // segment ends inside the entry (hand off a shifted head/middle piece).  `mem` records
    // that the walk read global memory (see process()).
    bool mem = false;
    auto event = [&]() {
      const bool started = sw.flags & SegWalk::kStarted;
      if (sw.pos == sw.cur_end) {
        const uint64_t v = crc_value(r);
        if (started) {
          emit(a, sw.cur, v);
        } else {  // tail piece: this segment is the entry's last
          mem = true;
          const uint64_t first = absE(sw.cur) / S;
          if (k - first + 1 <= kMaxSlotParts)
            a.piece_tail[k] = v;
          else
            straddle_piece(a, sw.cur, first, k - first + 1, k, v);
        }
        r = RState{0u, 0u};
        sw.flags |= SegWalk::kStarted;
        ++sw.cur;
        start_entry();
      } else {  // pos == hi < entry end
        mem = true;
        const uint64_t ce = absE(sw.cur + 1);
        const uint64_t c = crc_shift(crc_value(r), ce - (s0 + sw.hi), a.shift);
        const uint64_t first = started ? k : absE(sw.cur) / S;
        const uint64_t last = (ce - 1) / S;
        if (last - first + 1 <= kMaxSlotParts)  // head / middle piece
          a.piece_cont[k] = c;
        else
          straddle_piece(a, sw.cur, first, last - first + 1, k, c);
        sw.flags |= SegWalk::kDone;
      }
    };

    const uint32_t halves = __builtin_amdgcn_readfirstlane(rounds * 2);
    const uint32_t prog0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(j * halves));
    // prefetches past the chunk's last half-round re-read that half (L2-hot): the half
    // index stays wave-uniform and the descriptor a single SGPR quad -- selecting an empty
    // descriptor instead put it in VGPRs and wrapped every load in a waterfall loop.
    // The ring loop has no exit but its header: the last iteration's surplus stages load and
    // transpose (L2-hot) and skip process().  A `break` between stages joined ring states
    // with different halves in flight at the loop header, and the compiler then waited for
    // two halves (vmcnt(4)) before hashing the oldest one: the ring ran one half deep.
    auto last_half = [&](uint32_t h) -> uint32_t { return h < halves ? h : halves - 1u; };
    // settle the setup's loads first (e.g. an unused interpolation probe): a load the
    // compiler still counts as in flight when the ring starts costs a vmcnt(0) at the top
    // of every ring iteration
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

    auto process = [&](uint32_t hh, const u32x4 (&v)[4]) {
      if (sw.flags & SegWalk::kDone) return;
      const uint32_t hs = hh * 64u, he = hs + 64u;
      if (sw.pos == hs && he <= sw.next) {  // fast path: the half lies inside entry cur
        tb.step64(r, v, lds);
        sw.pos = he;
      }
      if (sw.flags & SegWalk::kDone) return;
      if (sw.pos == sw.next || sw.pos < he) {  // slow path: events / partial halves
        mem = false;
        while (!(sw.flags & SegWalk::kDone)) {
          if (sw.pos == sw.next) {
            event();
            continue;
          }
          if (sw.pos >= he) break;
          if (sw.pos == hs && he <= sw.next) {
            tb.step64(r, v, lds);
            sw.pos = he;
            continue;
          }
          const uint32_t lim = he < sw.next ? he : sw.next;
          if (kRegs && sw.pos >= hs && s0 + he <= span) {
            hash_regs(tb, r, v, sw.pos - hs, lim - hs, lds);
          } else {
            hash_global(tb, r, A, s0 + sw.pos, s0 + lim, lds);
            mem = true;
          }
          sw.pos = lim;
        }
        if (__builtin_amdgcn_ballot_w64(mem)) __builtin_amdgcn_s_waitcnt(0x0F70);
      }
    };

    // transposes run with the whole wave active (row swaps), before any per-lane branch; the
    // asm pin keeps the half's first use below the loads issued before it (otherwise the
    // scheduler hoists the memory-free transposes and drains the prefetch with vmcnt(0))
    auto transpose_half = [&](u32x4 (&v)[4]) {
      asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
      row_transpose(v[0], v[1], v[2], v[3]);
    };

    if constexpr (kRing4) {
      // 4-slot ring, the two halves of a 128-B line loaded back to back: the line's second
      // half then meets its first half's fill in L2.  With the halves issued one step apart,
      // 15-19 % of the lines were fetched twice (rocprofv3 TCC_EA0_RDREQ_128B, DESIGN.md
      // §4.2): the waves of an XCD walk segments 2^k bytes apart in step, so they contend for
      // the same L2 sets, and a line could be evicted between its two halves.
      // (lines, not halves: last_half(2 l) / 2 is the clamped line)
      JRQ_LOAD_LINE(h2, h3, last_half(2u) >> 1);
      for (uint32_t hh0 = 0; hh0 < halves; hh0 += 4) {
        const uint32_t hh = __builtin_amdgcn_readfirstlane(hh0);  // keep the counter in SGPRs
        if (a.prio_steps) {  // wave-uniform: lower this wave's priority as it gets ahead
          const uint32_t prog = prog0 + hh;
          const uint32_t lvl = __builtin_amdgcn_readfirstlane(
              static_cast<uint32_t>(prog >= pt0) + (prog >= pt1) + (prog >= pt2));
          if (lvl != prio_lvl) {
            prio_lvl = lvl;
            if (lvl == 1) __builtin_amdgcn_s_setprio(2);
            else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
          }
        }
        transpose_line(h0, h1);
        process(hh, h0);
        if (hh + 1 < halves) process(hh + 1, h1);  // wave-uniform
        JRQ_LOAD_LINE(h0, h1, last_half(hh + 4) >> 1);
        transpose_line(h2, h3);
        if (hh + 2 < halves) process(hh + 2, h2);
        if (hh + 3 < halves) process(hh + 3, h3);
        JRQ_LOAD_LINE(h2, h3, last_half(hh + 6) >> 1);
      }
    } else {
      for (uint32_t hh0 = 0; hh0 < halves; hh0 += 3) {
        const uint32_t hh = __builtin_amdgcn_readfirstlane(hh0);  // keep the counter in SGPRs
        if (a.prio_steps) {  // wave-uniform: lower this wave's priority as it gets ahead
          const uint32_t prog = prog0 + hh;
          const uint32_t lvl = __builtin_amdgcn_readfirstlane(
              static_cast<uint32_t>(prog >= pt0) + (prog >= pt1) + (prog >= pt2));
          if (lvl != prio_lvl) {
            prio_lvl = lvl;
            if (lvl == 1) __builtin_amdgcn_s_setprio(2);
            else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
          }
        }
        JRQ_LOAD_HALF(h2, last_half(hh + 2));
        transpose_half(h0);
        process(hh, h0);
        JRQ_LOAD_HALF(h0, last_half(hh + 3));
        transpose_half(h1);
        if (hh + 1 < halves) process(hh + 1, h1);  // wave-uniform
        JRQ_LOAD_HALF(h1, last_half(hh + 4));
        transpose_half(h2);
        if (hh + 2 < halves) process(hh + 2, h2);
      }
    }
#undef JRQ_LOAD_HALF
#undef JRQ_LOAD_LINE
  }
}

// Per entry, after the rounds kernel:
//  * an entry that spans 2..kMaxSlotParts segments: data CRC = XOR of its pieces, the head /
//    middle pieces in piece_cont[first .. last-1] (already shifted to the entry end), the tail
//    in piece_tail[last]; every other entry's data CRC is already in out[e];
//  * LogEntry batches: LogEntry.checksum() = type.getNumber() ^ LogId.checksum() ^ peers'
//    checksums ^ crc64(data) (LogEntry.java:88-108), LogId.checksum() = crc64(BE64(index) ||
//    BE64(term)) (LogId.java:45-50, Bits.java:71-80), then isCorrupted() (:156-158).
// One lane per entry over coalesced streams; the 16 LogId bytes go through table R0 in LDS
// byte by byte (CRC64.update(byte), CRC64.java:100-103).
template <bool kLogEntry>
__global__ __launch_bounds__(256) void crc64_finish_kernel(JrqCrcArgs a) {
  __shared__ uint64_t r0[256];
  if (a.gate != nullptr && a.gate[0] != 0) return;  // V2: the fixed-size path took the batch
  if (kLogEntry) r0[threadIdx.x] = a.slice[threadIdx.x];  // R0 = bswap(T0) (blockDim == 256)
  __syncthreads();
  const uint64_t* __restrict__ off = a.offsets;
  const uint64_t base = off[0];
  const uint64_t D = reinterpret_cast<uintptr_t>(a.payload + base) & 15u;
  const uint64_t span = D + (off[a.n] - base);
  const uint64_t S = seg_size(a, span);
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < a.n; e += stride) {
    const uint64_t o0 = off[e], o1 = off[e + 1];
    uint64_t v;
    if (!crc_pieces(a, o0, o1, base, D, S, v)) {
      // whole entry (or atomic hand-off): out[e] is final
      if (!kLogEntry && a.stream_state == nullptr) continue;
      v = a.out[e];
    }
    if (!kLogEntry && a.stream_state != nullptr) {
      // streaming Checksum (CRC64.update, CRC64.java:106-110): register * x^(8 len) ^ crc(chunk);
      // init 0 and xorout 0 make CRC64 linear
      const uint64_t len = o1 - o0;
      a.stream_state[e] = crc_shift(a.stream_state[e], len, a.shift) ^ (len ? v : 0);
    }
    if (kLogEntry) {
      uint64_t r = 0;
      // the big-endian bytes of index then term, in stream order = little-endian bswap64(v)
      const uint64_t bi = bswap64(static_cast<uint64_t>(a.index[e]));
      const uint64_t bt = bswap64(static_cast<uint64_t>(a.term[e]));
#pragma unroll
      for (int q = 0; q < 8; ++q) r = r0[(r ^ (bi >> (8 * q))) & 0xFF] ^ (r >> 8);
#pragma unroll
      for (int q = 0; q < 8; ++q) r = r0[(r ^ (bt >> (8 * q))) & 0xFF] ^ (r >> 8);
      v ^= static_cast<uint64_t>(a.type[e]) ^ bswap64(r);
      if (a.peer_xor) v ^= a.peer_xor[e];
      if (a.expected != nullptr && a.corrupt != nullptr) {
        const bool has = (a.has == nullptr) || a.has[e];
        a.corrupt[e] = static_cast<uint8_t>(has && a.expected[e] != v);
      }
    }
    a.out[e] = v;
  }
}

// ------------------------------------------------------ fixed-size entries ---
// N entries of EL bytes each, back to back: no segments, no offsets.  An entry is hashed by
// k = fixed_k consecutive lanes (a power of two, k pieces of PS = EL / k bytes, PS a multiple of
// 256; k > 1 only when N < lanes, e.g. C5's 64k x 16 KiB on 128k lanes), lane c of a wave takes
// piece c of row r (64 pieces), so every piece ends in the same half-round on all lanes.  The k
// piece CRCs meet by linearity in log2(k) butterfly levels, crc(A || B) = crc(A) x^(8|B|) ^
// crc(B), and the last lane of the entry applies the LogEntry fields (coalesced, loaded when
// the row starts) and stores the result: one launch, no finish kernel.  The loads are the rounds kernel's transposed row-group shape with
// lane stride EL; a ring of four half-rounds turns 4 halves per step, an entry = EL / 256 turns,
// so the field loads of a row sit at least 16 ring loads before their use (the compiler never
// waits for the ring on their account).  C1 (1M x 256 B): the segment walk wrote 6.5x its 8 MB
// of results as scattered 8-B stores and re-read them in the finish kernel.
// kStarts (V2 decode): entry i starts at payload + starts[i] (non-decreasing, any byte
// alignment: each piece is hashed from its 128-B line, below), k and EL come from the device words
// gate[0..1] written by v2_parse (gate[3]: the payload's end offset); k == 0 means the
// segment walk takes the batch instead.  With kLogEntry the record's partial checksum (type ^
// crc(LogId) ^ peers, from v2_parse) arrives in peer_xor: out = partial ^ crc(data) and the
// verify compare, as v2_finish does on the segment-walk path.
template <bool kLogEntry, bool kStarts, int kBlock>
__global__ __launch_bounds__(kBlock) void crc64_fixed_kernel(JrqCrcArgs a) {
  __shared__ __attribute__((aligned(16))) uint64_t lds_tab[kCrcLdsBytes / 8];
  if (kStarts && a.gate[0] == 0) return;
  const char* lds = reinterpret_cast<const char*>(lds_tab);
  constexpr uint32_t kTabPer = kCrcLdsBytes / 8 / kBlock;
  uint64_t tab_v[kTabPer];  // this thread's share of the table image (written after the first loads)
#pragma unroll
  for (uint32_t i = 0; i < kTabPer; ++i)
    tab_v[i] = a.slice[CrcTab::src_index(threadIdx.x + i * kBlock)];
  auto build_tables = [&]() {
#pragma unroll
    for (uint32_t i = 0; i < kTabPer; ++i) lds_tab[threadIdx.x + i * kBlock] = tab_v[i];
    __syncthreads();
  };
  const CrcTab tb(threadIdx.x & 63u);
  const uint32_t L = threadIdx.x;
  const uint32_t L0 = __builtin_amdgcn_readfirstlane(L & ~63u);
  const uint32_t lane = L - L0;
  const uint32_t n = a.n;
  const uint32_t K = kStarts ? static_cast<uint32_t>(a.gate[0]) : a.fixed_k;
  const uint64_t EL = kStarts ? a.gate[1] : a.entry_bytes;
  const uint32_t kl = 31u - __builtin_clz(K);  // lanes per entry, log2
  const uint64_t PS = EL >> kl;                // piece bytes
  const uint32_t EPR = 64u >> kl;                              // entries per row
  const uint32_t rows = (n + EPR - 1) / EPR;
  // contiguous rows per wave (a wave streams 64 * EL * rows bytes in order)
  const uint32_t W = gridDim.x * (kBlock / 64);
  const uint32_t w = blockIdx.x * (kBlock / 64) + (L0 >> 6);
  const uint32_t per = rows / W, extra = rows % W;
  const uint32_t r0 = __builtin_amdgcn_readfirstlane(w * per + (w < extra ? w : extra));
  const uint32_t r1 = __builtin_amdgcn_readfirstlane(r0 + per + (w < extra ? 1u : 0u));
  if (r0 >= r1) {  // no rows: write the table share (every wave meets the one barrier)
    build_tables();
    return;
  }
  const uint32_t HE = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(PS >> 6));  // halves per piece
  const uint32_t turns = HE >> 2;
  // load window end (read once: the loads' memory clobber would re-read it in the ring)
  const uint64_t total = kStarts ? a.gate[3] : static_cast<uint64_t>(n) * EL;
  const uint32_t WS = static_cast<uint32_t>(PS);  // lane-to-lane stride (64 * PS < 2^32)
  // full-line shape: load q reads 16-B piece L >> 3 of owner (L & 7) + 8q's line
  // (transpose_line); qa[q] = that owner's offset + 16 (L >> 3)
  const uint32_t qb = (L & 7u) * WS + 16u * ((L >> 3) & 7u);
  uint32_t qa[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) qa[q] = qb + 8u * static_cast<uint32_t>(q) * WS;
  const uintptr_t pbase = reinterpret_cast<uintptr_t>(a.payload);
  // kStarts: the row's base (its first piece) and each owner's offset from it, through
  // __shfl (the load of lane 16q + c reads owner 16q + c's piece); a new row costs a load
  // Byte-misaligned 16-B loads stream at ~60 % of the aligned rate (round 3's tools/unal_probe.hip),
  // and lines split between two loads cannot be `nt`: a piece starting at byte b of a 128-B
  // line is hashed over [start - b, start - b + PS) -- whole lines, the ring's own loads --
  // with the b bytes before it zeroed in the row's first line (leading zeros leave the raw CRC
  // unchanged), and the b bytes it missed are hashed after the loop; the payload is 128-B
  // aligned (the host checks).  b_next: the b of the row whose first line went out last.
  uint64_t row_base = 0;
  uint32_t b_next = 0;
  auto set_row = [&](uint32_t row) {
    const uint32_t er = row * EPR + (lane >> kl);
    const uint64_t psu = a.starts[er < n ? er : n - 1u] + static_cast<uint64_t>(lane & (K - 1u)) * PS;
    b_next = static_cast<uint32_t>(psu & 127u);
    const uint64_t ps = psu & ~127ull;
    const uint32_t rb_lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(ps));
    const uint32_t rb_hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(ps >> 32));
    row_base = (static_cast<uint64_t>(rb_hi) << 32) | rb_lo;
    const uint32_t rel = static_cast<uint32_t>(ps - row_base);
    const uint32_t c = L & 7u, ro = 16u * ((L >> 3) & 7u);
#pragma unroll
    for (int q = 0; q < 8; ++q) qa[q] = __shfl(rel, static_cast<int>(c + 8u * q)) + ro;
  };
  // load cursor (row, line of the piece) of the next 128-B line to issue, scalar; past the
  // wave's last line its loads get an empty descriptor (zeros, no memory request: re-reading
  // that line cost up to 3 % of the bytes when it had left L2)
  uint32_t crow = r0, cline = 0, cur_live = 1u;
  const uint32_t LE = HE >> 1;  // lines per piece
  auto load_line = [&](u32x4 (&HA)[4], u32x4 (&HB)[4]) {
    // kStarts: a row's offsets are set when its first line goes out, so at the top of row r the
    // last row set is r (its first line leaves during row r - 1, row r + 1's during row r)
    if (kStarts && cline == 0 && cur_live) set_row(crow);
    const uint64_t o = kStarts ? row_base + static_cast<uint64_t>(cline) * 128u
                               : static_cast<uint64_t>(crow) * 64u * PS + static_cast<uint64_t>(cline) * 128u;
    const uint64_t hp = pbase + o;
    const uint32_t hlo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(hp));
    const uint32_t hhi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(hp >> 32));
    // lanes past entry n-1 read zeros; kStarts: the dword past the last chunk of the batch may
    // lie past the payload (gate[3] = its end): zeros too
    const uint64_t left = total - o;
    const uint32_t hn = cur_live ? __builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(left > 0x7FFFFFFFull ? 0x7FFFFFFFull : left)) : 0u;
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint8_t*>((static_cast<uint64_t>(hhi) << 32) | hlo),
        static_cast<short>(0), static_cast<int>(hn), 0x00020000);
    constexpr int kAux = JRQ_CRC_LINE_AUX;
#pragma unroll
    for (int q = 0; q < 4; ++q) HA[q] = __builtin_amdgcn_raw_buffer_load_b128(rh, qa[q], 0, kAux);
#pragma unroll
    for (int q = 0; q < 4; ++q) HB[q] = __builtin_amdgcn_raw_buffer_load_b128(rh, qa[4 + q], 0, kAux);
    asm volatile("" ::: "memory");
    if (cline + 1 < LE) {
      ++cline;
    } else if (crow + 1 < r1) {
      ++crow;
      cline = 0;
    } else {
      cur_live = 0u;
    }
  };
  u32x4 h0[4], h1[4], h2[4], h3[4];
  load_line(h0, h1);
  load_line(h2, h3);
  build_tables();
  // LogEntry fields: absent arrays read word 0 of the slice table (R0[0] = 0), masked below
  const uint64_t* const z = a.slice;
  const bool ver = kLogEntry && a.expected != nullptr && a.corrupt != nullptr;
  const uint64_t* const p_peer = kLogEntry && a.peer_xor ? a.peer_xor : z;
  const uint64_t* const p_exp = ver ? a.expected : z;
  const uint8_t* const p_has = ver && a.has ? a.has : reinterpret_cast<const uint8_t*>(z);
  const uint32_t m_peer = a.peer_xor ? ~0u : 0u, m_exp = ver ? ~0u : 0u, m_has = ver && a.has ? ~0u : 0u;
  const uint32_t piece = lane & (K - 1u);
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t e0 = r * EPR + (lane >> kl);
    const bool live = e0 < n;
    const uint32_t e = live ? e0 : n - 1u;
    uint32_t f_type = 0, f_has = 0;
    uint64_t f_index = 0, f_term = 0, f_peer = 0, f_exp = 0;
    if (kLogEntry) {
      if (!kStarts) {
        f_type = a.type[e];
        f_index = static_cast<uint64_t>(a.index[e]);
        f_term = static_cast<uint64_t>(a.term[e]);
      }
      f_peer = p_peer[e & m_peer];
      f_exp = p_exp[e & m_exp];
      f_has = p_has[e & m_has];
    }
    RState s{0u, 0u};
    uint32_t q = 0;
    const uint32_t bh = kStarts ? b_next : 0u;  // this row's piece offset in its first line
    // a ring of two 128-B lines per lane (slots h0 + h1, h2 + h3), each line read whole by
    // its load instructions (8 owners x 128 B each): with half-lines per instruction 15 % of
    // the lines were fetched twice, and `nt` loads could not be used
    do {
      transpose_line(h0, h1);
      if (kStarts && q == 0) {  // the bytes before the piece: zeros (wave-uniform branch)
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const int sh = static_cast<int>(bh) - 4 * j;
          const uint32_t keep = sh <= 0 ? ~0u : sh >= 4 ? 0u : (~0u << (8 * sh));
          if (j < 16) h0[j >> 2][j & 3] &= keep;
          else h1[(j - 16) >> 2][j & 3] &= keep;
        }
      }
      tb.step64(s, h0, lds);
      tb.step64(s, h1, lds);
      load_line(h0, h1);
      transpose_line(h2, h3);
      tb.step64(s, h2, lds);
      tb.step64(s, h3, lds);
      load_line(h2, h3);
    } while (++q < turns);
    uint64_t c = crc_value(s);
    if (kStarts) {  // hashed [ps - b, ps - b + PS) with its first b bytes zeroed: add the b missed
      // T = the first b bytes of the 128-B line at tl (the line may run past the records' end:
      // then byte loads)
      const uint64_t tl = ((a.starts[e] + static_cast<uint64_t>(piece) * PS) & ~127ull) + PS;
      const uint32_t b = bh;
      if (tl + 128u <= total) {
        uint4 tw[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) tw[i] = reinterpret_cast<const uint4*>(a.payload + tl)[i];
        // whole 8-B words, then the last b & 7 bytes one by one: at most 15 + 7 dependent
        // table steps (byte by byte it was up to 127)
#pragma unroll
        for (int w = 0; w < 16; ++w) {
          if (8u * w + 8u <= b) {
            const uint4 v = tw[w >> 1];
            tb.step8(s, (w & 1) ? v.z : v.x, (w & 1) ? v.w : v.y, lds);
          }
        }
        const uint32_t wi = b >> 3, rem = b & 7u;
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
          const uint4 v = tw[w >> 1];
          lo = wi == static_cast<uint32_t>(w) ? ((w & 1) ? v.z : v.x) : lo;
          hi = wi == static_cast<uint32_t>(w) ? ((w & 1) ? v.w : v.y) : hi;
        }
#pragma unroll
        for (uint32_t t = 0; t < 7; ++t)
          if (t < rem) tb.step1(s, ((t < 4 ? lo : hi) >> (8 * (t & 3u))) & 0xFFu, lds);
      } else {
        for (uint32_t t = 0; t < b; ++t) tb.step1(s, a.payload[tl + t], lds);
      }
      c = crc_value(s);
    }
    // pieces -> entry: at level l, the group of 2^l lanes holding the earlier bytes is shifted
    // past the 2^l * PS bytes of its partner group (x^(8 * 2^l * PS), global power tables)
    for (uint32_t l = 0; l < kl; ++l) {
      const uint64_t sh = (piece >> l) & 1u ? c : crc_shift(c, PS << l, a.shift);
      const uint32_t lo = __shfl_xor(static_cast<uint32_t>(sh), 1 << l);
      const uint32_t hi = __shfl_xor(static_cast<uint32_t>(sh >> 32), 1 << l);
      const uint64_t other = (static_cast<uint64_t>(hi) << 32) | lo;
      if ((piece >> l) & 1u) c ^= other;  // the later group accumulates
    }
    const bool last = piece == K - 1u;  // the lane holding the entry's CRC
    if (kLogEntry) {  // LogEntry.checksum(): type ^ LogId.checksum() ^ peers ^ crc64(data)
      if (!kStarts) {
        RState lid{0u, 0u};
        const uint64_t bi = bswap64(f_index), bt = bswap64(f_term);
        tb.step8(lid, static_cast<uint32_t>(bi), static_cast<uint32_t>(bi >> 32), lds);
        tb.step8(lid, static_cast<uint32_t>(bt), static_cast<uint32_t>(bt >> 32), lds);
        c ^= static_cast<uint64_t>(f_type) ^ crc_value(lid);
      }
      c ^= f_peer;
      if (ver && live && last) a.corrupt[e] = static_cast<uint8_t>((m_has ? f_has != 0 : true) && f_exp != c);
    }
    if (live && last) a.out[e] = c;
  }
}

}  // namespace jrq

// Fixed-size entries (crc64_fixed_kernel): fixed_k lanes per entry, 64 * (entry_bytes / fixed_k)
// < 2^32, (entry_bytes / fixed_k) % 256 == 0.
extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_crc64_fixed(
    JrqCrcArgs* args, int log_entry, int grid, hipStream_t stream) {
  // one lane per entry (C1-like batches, several rows per wave): 1024-thread workgroups (118
  // VGPRs, 4 waves per SIMD); pieces of larger entries: 512 (r06 A/B, profiles/r06_experiments.json)
  const bool wide = args->starts == nullptr && args->fixed_k == 1;
  if (args->starts != nullptr && log_entry)  // V2 decode: partial ^ crc(data), gated on the device
    hipLaunchKernelGGL((jrq::crc64_fixed_kernel<true, true, jrq::kCrcFixedBlock>), dim3(grid),
                       dim3(jrq::kCrcFixedBlock), 0, stream, *args);
  else if (args->starts != nullptr)  // plain CRCs at given starts, gated on the device
    hipLaunchKernelGGL((jrq::crc64_fixed_kernel<false, true, jrq::kCrcFixedBlock>), dim3(grid),
                       dim3(jrq::kCrcFixedBlock), 0, stream, *args);
  else if (log_entry && wide)
    hipLaunchKernelGGL((jrq::crc64_fixed_kernel<true, false, jrq::kCrcFixedWideBlock>), dim3(grid),
                       dim3(jrq::kCrcFixedWideBlock), 0, stream, *args);
  else if (log_entry)
    hipLaunchKernelGGL((jrq::crc64_fixed_kernel<true, false, jrq::kCrcFixedBlock>), dim3(grid),
                       dim3(jrq::kCrcFixedBlock), 0, stream, *args);
  else if (wide)
    hipLaunchKernelGGL((jrq::crc64_fixed_kernel<false, false, jrq::kCrcFixedWideBlock>), dim3(grid),
                       dim3(jrq::kCrcFixedWideBlock), 0, stream, *args);
  else
    hipLaunchKernelGGL((jrq::crc64_fixed_kernel<false, false, jrq::kCrcFixedBlock>), dim3(grid),
                       dim3(jrq::kCrcFixedBlock), 0, stream, *args);
  return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_crc64(
    JrqCrcArgs* args, int log_entry, int grid, hipStream_t stream) {
  if (args->regs_slowpath) {
    args->lanes = static_cast<uint32_t>(grid) * jrq::kCrcRegsBlock;
    hipLaunchKernelGGL((jrq::crc64_rounds_kernel<jrq::kCrcRegsBlock, true>), dim3(grid),
                       dim3(jrq::kCrcRegsBlock), 0, stream, *args);
  } else {
    args->lanes = static_cast<uint32_t>(grid) * jrq::kCrcBlock;
    hipLaunchKernelGGL((jrq::crc64_rounds_kernel<jrq::kCrcBlock, false>), dim3(grid),
                       dim3(jrq::kCrcBlock), 0, stream, *args);
  }
  if (args->no_finish) return hipGetLastError();  // (the caller's own kernel assembles the pieces)
  const uint32_t blocks = (args->n + 255) / 256;
  const uint32_t cap = static_cast<uint32_t>(grid) * 8;
  const dim3 fg(blocks < cap ? blocks : cap);
  if (log_entry)
    hipLaunchKernelGGL(jrq::crc64_finish_kernel<true>, fg, dim3(256), 0, stream, *args);
  else
    hipLaunchKernelGGL(jrq::crc64_finish_kernel<false>, fg, dim3(256), 0, stream, *args);
  return hipGetLastError();
}
