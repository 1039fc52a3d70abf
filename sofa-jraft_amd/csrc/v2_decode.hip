// v2_decode.hip -- batched V2 log-entry decode + checksum verify on read.
//
// Reference, per record a LogStorage returns for one log index:
//   AutoDetectDecoder.decode   jraft-core/.../entity/codec/AutoDetectDecoder.java:41-52
//   V2Decoder.decode           jraft-core/.../entity/codec/v2/V2Decoder.java:46-110
//   PBLogEntry parsing         jraft-core/.../entity/codec/v2/LogOutter.java:185-275 (protobuf
//                              3.5.1 CodedInputStream, pom.xml:74), log.proto:10-20
//   LogEntry.isCorrupted       jraft-core/.../entity/LogEntry.java:88-108,156-158, checked on
//                              read by LogManagerImpl (core/LogManagerImpl.java:733-745)
//
// Record layout (V2Encoder.java:76-130, LogEntryV2CodecFactory.java:52-60):
//   0xBB 0xD2 0x01 <3 reserved> PBLogEntry{type 1, term 2, index 3, peers 4*, old_peers 5*,
//   data 6, checksum 7?, learners 8*, old_learners 9*}
//
// Design: the records are one flat buffer with offsets[N+1] (the batch a segment / RocksDB
// scan hands over).
//   v2_parse   one lane per record walks the protobuf fields through a 16-B aligned chunk
//              cache (a handful of dependent loads per record: the header fields, then a jump
//              over `data` to the trailing checksum / learner fields).  Peer strings are hashed
//              byte-wise from an LDS copy of the CRC table while their canonical form is
//              checked; type ^ crc(LogId) ^ peers goes to a partial word.  It also writes one
//              CRC range per record, [data start, next data start), and its last block to
//              arrive writes the gate of the fixed-size data path (every record decoded, one
//              data length).
//   fixed path crc64_fixed_kernel at the data starts (k lanes per record), finishing in place:
//              computed = partial ^ crc(data), corrupt = has_checksum && stored != computed.
//   otherwise  the batched segment walk (crc64.hip) over the ranges -- one pass over the
//              record bytes at streaming bandwidth -- then v2_finish: the data CRC recovered
//              from its range's CRC by linearity (see v2_finish), computed, corrupt.
//   The kernels of the path not taken return at their first instruction (gate on the device,
//   so the _dev entry point stays free of host synchronisation).
//
// A peer string is hashed as stored when it is already what PeerId.toString() would render
// from it (V2Encoder always writes toString(), so this is every record it produced).  A
// record with any other peer string -- which the reference re-renders or rejects with
// IllegalArgumentException -- or with unknown-field groups nested deeper than 2 gets status
// HOST: the host decodes it with the reference decoder.
#include "jrq_device.h"

namespace jrq {

typedef uint32_t v2u32x4 __attribute__((ext_vector_type(4)));

// include/jrq.h jrq_v2_status
constexpr uint8_t kV2Ok = 0, kV2Null = 1, kV2V1 = 2, kV2Host = 3;

// A record's bytes through a one-line cache: a miss loads the whole aligned 64-B line (four
// independent 16-B loads, one round trip) -- a V2 header (magic, type, term, index, the data
// tag and length) mostly fits one line, where 16-B chunks cost one dependent round trip each.
struct ChunkReader {
  const uint8_t* rec;  // record start
  int64_t limit;       // record length
  uintptr_t line_addr;
  v2u32x4 c0, c1, c2, c3;
  bool err;
  __device__ explicit ChunkReader(const uint8_t* r, int64_t len)
      : rec(r), limit(len), line_addr(~static_cast<uintptr_t>(0)), err(false) {}
  // byte at record position pos (< limit): its 64-B line holds a valid byte and lies in one
  // 4 KiB page with it, so the aligned loads never leave the mapped buffer
  __device__ __forceinline__ uint32_t at(int64_t pos) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(rec) + static_cast<uintptr_t>(pos);
    const uintptr_t la = a & ~static_cast<uintptr_t>(63);
    if (la != line_addr) {
      const v2u32x4* p = reinterpret_cast<const v2u32x4*>(la);
      c0 = p[0];
      c1 = p[1];
      c2 = p[2];
      c3 = p[3];
      line_addr = la;
    }
    // (selects on scalars: a dynamically indexed vector would live in scratch memory)
    const uint32_t o = static_cast<uint32_t>(a & 63u), d = o >> 2, q = d & 3u, h = d >> 2;
    auto sel4 = [q](v2u32x4 v) { return q < 2 ? (q == 0 ? v.x : v.y) : (q == 2 ? v.z : v.w); };
    const uint32_t w0 = sel4(c0), w1 = sel4(c1), w2 = sel4(c2), w3 = sel4(c3);
    const uint32_t w = h < 2 ? (h == 0 ? w0 : w1) : (h == 2 ? w2 : w3);
    return (w >> (8 * (o & 3u))) & 0xFFu;
  }
};

// A record's bytes for the parse, one lane per record: the 128 B from the 64-B line of its first
// byte and the 128 B ending with the line of its last byte, loaded together (one round trip)
// and staged into the lane's slice of LDS; any other byte is a single global load.  A V2
// header (magic, type, term, index, peers, the data tag and length) and its trailer (checksum,
// learners) fit the two windows.  With a one-line cache per lane instead (ChunkReader), a
// wave went to memory whenever any of its 64 lanes crossed a line -- nearly every header byte,
// the lanes' records starting at unrelated offsets: 29-30 us for 64k records.
constexpr uint32_t kWinSlot = 272;  // LDS bytes per lane (256 + 16: 16-B aligned slots starting in different banks)

struct WindowReader {
  const uint8_t* rec;
  int64_t limit;
  uintptr_t head, tail;  // the windows' 64-B aligned starts
  const uint8_t* slot;   // the lane's LDS copy: [0, 128) head window, [128, 256) tail window
  bool err;
  __device__ WindowReader(const uint8_t* r, int64_t len, uint8_t* lds) : rec(r), limit(len), slot(lds), err(false) {
    // len >= 1.  A line is loaded only when it holds a byte of the record (so it lies in a
    // mapped page); the line at `tail` always does (tail >= head, tail <= the last byte's line).
    const uintptr_t s = reinterpret_cast<uintptr_t>(r), e = s + static_cast<uintptr_t>(len);
    head = s & ~static_cast<uintptr_t>(63);
    const uintptr_t last = (e - 1) & ~static_cast<uintptr_t>(63);
    tail = last >= head + 64 ? last - 64 : head;
    const uintptr_t lines[4] = {head, head + 64, tail, tail + 64};
    v2u32x4 v[16];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      if (lines[l] <= e - 1) {
        const v2u32x4* p = reinterpret_cast<const v2u32x4*>(lines[l]);
#pragma unroll
        for (int c = 0; c < 4; ++c) v[4 * l + c] = p[c];
      }
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      if (lines[l] <= e - 1) {
#pragma unroll
        for (int c = 0; c < 4; ++c) *reinterpret_cast<v2u32x4*>(lds + 64 * l + 16 * c) = v[4 * l + c];
      }
    }
  }
  __device__ __forceinline__ uint32_t at(int64_t pos) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(rec) + static_cast<uintptr_t>(pos);
    if (a - head < 128) return slot[a - head];
    if (a - tail < 128) return slot[128 + (a - tail)];
    return rec[pos];
  }
};

// A varint from 10 bytes of a window (independent LDS reads, no per-byte branch): its value
// accumulated as readRawVarint64 does (readRawVarint32 = the low 32 bits: bytes 5..9 only
// carry bits >= 35), *n = the bytes it takes, 11 if all ten continue (malformed).
__device__ __forceinline__ uint64_t lds_varint(const uint8_t* w, uint32_t* n) {
  uint32_t b[10], cont = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    b[i] = w[i];
    cont |= ((b[i] >> 7) & 1u) << i;
  }
  const uint32_t k = static_cast<uint32_t>(__builtin_ctz(~cont)) + 1u;
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) v |= i < static_cast<int>(k) ? static_cast<uint64_t>(b[i] & 0x7Fu) << (7 * i) : 0ull;
  *n = k;
  return v;
}

// The record as V2Encoder writes a data entry (V2Encoder.java:76-130; generated writeTo order,
// LogOutter.java:518-546): type, term, index, data, an optional checksum, nothing else, each
// varint inside the LDS windows.  Decodes it with a fixed sequence of window reads (a handful
// of dependent LDS round trips per record); false on anything else -- peers, learners, unknown
// fields, other orders, a field outside the windows -- and the general parser decodes the
// record from its start.  One lane per record runs a wave's records in lockstep: the general
// parser's per-byte loop and field switch were 29 us for 64k records (round 3's tools/v2_parse_probe.hip).
struct V2Fast {
  uint32_t etype;
  int64_t term, index, doff, dlen;
  uint64_t ck;
  bool have_ck;
};

__device__ __forceinline__ bool v2_fast_fields(const WindowReader& rd, int64_t L, V2Fast& f) {
  const uintptr_t base = reinterpret_cast<uintptr_t>(rd.rec);
  int64_t p = 6;
  // the window bytes from record position q on (nullptr: its record bytes up to q + 10 are not
  // all inside one window).  Reads may run up to 9 bytes past a window: past the head window
  // that is the tail window's copy (so the record must end first), past the tail window the
  // lane slot's padding (the tail window ends with the record's last line)
  auto win = [&](int64_t q) -> const uint8_t* {
    const uintptr_t a = base + static_cast<uintptr_t>(q);
    const uintptr_t need = static_cast<uintptr_t>(L - q < 10 ? L - q : 10);
    if (a - rd.head < 128 && a - rd.head + need <= 128) return rd.slot + (a - rd.head);
    if (a - rd.tail < 128) return rd.slot + 128 + (a - rd.tail);
    return nullptr;
  };
  // tag, then a varint value: false unless the tag is `want` and both fit the record
  auto field = [&](uint32_t want, uint64_t* v) -> bool {
    if (p + 1 >= L) return false;
    const uint8_t* w = win(p);
    if (!w || w[0] != want) return false;
    const uint8_t* x = win(p + 1);
    if (!x) return false;
    uint32_t n;
    *v = lds_varint(x, &n);
    if (n > 10 || p + 1 + static_cast<int64_t>(n) > L) return false;
    p += 1 + n;
    return true;
  };
  uint64_t v;
  if (!field(0x08, &v) || static_cast<uint32_t>(v) > 3u) return false;  // type: an EntryType
  f.etype = static_cast<uint32_t>(v);
  if (!field(0x10, &v)) return false;
  f.term = static_cast<int64_t>(v);
  if (!field(0x18, &v)) return false;
  f.index = static_cast<int64_t>(v);
  if (!field(0x32, &v)) return false;  // data: a length-delimited field
  const int32_t size = static_cast<int32_t>(static_cast<uint32_t>(v));
  if (size < 0 || size > L - p) return false;
  f.doff = p;
  f.dlen = size;
  p += size;
  f.have_ck = false;
  f.ck = 0;
  if (p == L) return true;
  if (!field(0x38, &v)) return false;
  f.ck = v;
  f.have_ck = true;
  return p == L;
}

struct PbIn {
  WindowReader rd;
  int64_t pos;
  uint32_t last_tag;
  __device__ PbIn(const uint8_t* r, int64_t len, uint8_t* lds) : rd(r, len, lds), pos(6), last_tag(0) {}
  __device__ __forceinline__ uint32_t byte() {
    if (pos >= rd.limit) {
      rd.err = true;  // truncatedMessage
      return 0;
    }
    return rd.at(pos++);
  }
  // readRawVarint32 (5 value bytes + up to 5 discarded)
  __device__ uint32_t varint32() {
    uint32_t r = 0;
    for (int i = 0; i < 5; ++i) {
      const uint32_t x = byte();
      if (rd.err) return 0;
      r |= (x & 0x7Fu) << (7 * i);
      if (!(x & 0x80u)) return r;
    }
    for (int i = 0; i < 5; ++i) {
      const uint32_t x = byte();
      if (rd.err) return 0;
      if (!(x & 0x80u)) return r;
    }
    rd.err = true;  // malformedVarint
    return 0;
  }
  __device__ uint64_t varint64() {
    uint64_t r = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      const uint32_t x = byte();
      if (rd.err) return 0;
      r |= static_cast<uint64_t>(x & 0x7Fu) << shift;
      if (!(x & 0x80u)) return r;
    }
    rd.err = true;
    return 0;
  }
  __device__ uint32_t tag() {
    if (pos >= rd.limit) {
      last_tag = 0;
      return 0;
    }
    last_tag = varint32();
    if (!rd.err && (last_tag >> 3) == 0) rd.err = true;  // invalidTag
    return rd.err ? 0 : last_tag;
  }
  // length-delimited field: offset of its payload, *len its size
  __device__ int64_t bytes(int64_t* len) {
    const int32_t size = static_cast<int32_t>(varint32());
    if (rd.err) return 0;
    if (size < 0 || size > rd.limit - pos) {
      rd.err = true;
      return 0;
    }
    const int64_t at = pos;
    pos += size;
    *len = size;
    return at;
  }
  __device__ void skip(int64_t n) {
    if (n > rd.limit - pos) {
      rd.err = true;
      pos = rd.limit;
    } else {
      pos += n;
    }
  }
};

// Integer.toString canonical decimal of an int32 (sign only for negatives, no leading zeros)
struct CanonInt {
  int64_t v = 0;
  uint32_t n = 0;
  bool neg = false, ok = true;
  __device__ __forceinline__ void push(uint32_t c) {
    if (n == 0 && c == '-') {
      neg = true;
    } else if (c >= '0' && c <= '9') {
      const uint32_t digits = n - (neg ? 1u : 0u);
      if (digits == 1 && v == 0) ok = false;  // leading zero
      v = v * 10 + (c - '0');
      if (v > 2147483648LL) ok = false;
    } else {
      ok = false;
    }
    ++n;
  }
  __device__ __forceinline__ bool canonical() const {
    const uint32_t digits = n - (neg ? 1u : 0u);
    if (!ok || digits == 0) return false;
    if (neg && v == 0) return false;  // "-0"
    return neg ? v <= 2147483648LL : v <= 2147483647LL;
  }
};

// crc64 of the peer string at [at, at+len) (MSB-first byte table in LDS); *canon = the
// bytes are exactly PeerId.toString() of what they parse to: ip ":" port [":" idx != 0]
__device__ uint64_t peer_crc(PbIn& in, int64_t at, int64_t len, const uint64_t* T, bool* canon) {
  uint64_t crc = 0;
  uint32_t colons = 0, tok_len = 0;
  bool ok = true;
  CanonInt port, idx;
  for (int64_t i = 0; i < len; ++i) {
    const uint32_t c = in.rd.at(at + i);
    crc = T[((crc >> 56) ^ c) & 0xFFu] ^ (crc << 8);
    if (c == ':') {
      ok = ok && tok_len > 0;
      ++colons;
      tok_len = 0;
      continue;
    }
    ++tok_len;
    if (colons == 1) port.push(c);
    else if (colons == 2) idx.push(c);
  }
  ok = ok && tok_len > 0 && (colons == 1 || colons == 2) && port.canonical();
  if (colons == 2) ok = ok && idx.canonical() && idx.v != 0;
  *canon = ok;
  return crc;
}

__device__ __forceinline__ uint64_t crc_bytes_be(uint64_t crc, uint64_t v, const uint64_t* T) {
#pragma unroll
  for (int s = 56; s >= 0; s -= 8) crc = T[((crc >> 56) ^ (v >> s)) & 0xFFu] ^ (crc << 8);
  return crc;
}

constexpr uint32_t kV2Segments = 16;  // first-level arrival counters of v2_parse (gate[8..23])

// One lane per record; then the block's summary for the fixed-size data path's gate (below).
__device__ void v2_parse_record(const JrqV2Args& a, uint32_t r, const uint64_t* T, uint8_t* win,
                                uint8_t& st_out, uint64_t& d_out, uint64_t& dl_out);

__global__ __launch_bounds__(256) void v2_parse(JrqV2Args a) {
  __shared__ uint64_t T[256];
  __shared__ uint64_t s_doff[256];
  __shared__ uint64_t s_len0;
  __shared__ uint32_t s_last;
  __shared__ __attribute__((aligned(16))) uint8_t win[256 * kWinSlot];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) T[i] = bswap64(a.slice[i]);
  __syncthreads();
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r == 0) {
    a.off2[0] = a.off[0];
    a.off2[a.n + 1] = a.off[a.n];
  }
  const bool live = r < a.n;
  uint8_t st = kV2Null;
  uint64_t d = 0, dl = 0;
  if (live) v2_parse_record(a, r, T, win + threadIdx.x * kWinSlot, st, d, dl);
  // The gate of the fixed-size data path (crc64_fixed_kernel at the data starts): every record
  // decoded, all with the data length L0 of record 0, data ranges in order, and each 64
  // consecutive ones within 1 GiB (the fixed kernel reads a row of records through one buffer
  // descriptor at u32 offsets from its first start; checked per pair of adjacent blocks of 256,
  // a sufficient condition).  Each block summarises its records {first start, last start, its
  // first length, broken}; the last block to arrive combines the summaries and writes
  // gate = {k, L0, broken, end}: k lanes per record for crc64_fixed_kernel, 0 = the segment walk.
  s_doff[threadIdx.x] = d;
  if (threadIdx.x == 0) s_len0 = dl;
  __syncthreads();
  const uint64_t lb = s_len0;
  const bool bad = live && (st != kV2Ok || dl != lb ||
                            (threadIdx.x > 0 && d < s_doff[threadIdx.x - 1] + lb));
  const bool any_bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    const uint32_t nb = a.n - blockIdx.x * blockDim.x;
    uint64_t* sm = a.blk + 4ull * blockIdx.x;
    // The hand-off to the last block uses agent-scope relaxed atomics (stores and loads that
    // go to the coherence point, past the XCDs' own L2s) and one explicit wait for the
    // summary's stores before the arrival: __threadfence() here is buffer_wbl2 + buffer_inv,
    // an L2 writeback per workgroup (twice), ~10 us for the 256 workgroups of 64k records
    // (round 3's tools/v2_parse_probe.hip "gate").
    auto st_agent = [](uint64_t* q, uint64_t v) { __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    auto add_agent = [](uint64_t* q) { return __hip_atomic_fetch_add(q, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    st_agent(sm + 0, s_doff[0]);
    st_agent(sm + 1, s_doff[(nb < blockDim.x ? nb : blockDim.x) - 1]);
    st_agent(sm + 2, lb);
    st_agent(sm + 3, any_bad ? 1u : 0u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the summary is at the coherence point
    // arrival in two levels (block b -> segment counter b % 16, the last of each segment ->
    // gate[4]): same-address atomics serialise
    const uint32_t seg = blockIdx.x % kV2Segments;
    const uint32_t in_seg = (gridDim.x - seg + kV2Segments - 1) / kV2Segments;
    bool last = false;
    if (add_agent(a.gate + 8 + seg) + 1 == in_seg) {
      st_agent(a.gate + 8 + seg, 0);  // (no other arrival on it in this launch)
      const uint32_t segs = gridDim.x < kV2Segments ? gridDim.x : kV2Segments;
      last = add_agent(a.gate + 4) + 1 == segs;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  auto ld_agent = [](const uint64_t* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const uint64_t L0 = ld_agent(a.blk + 2);
  bool broken = false;
  for (uint32_t b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
    const uint64_t* sm = a.blk + 4ull * b;
    const uint64_t s0 = ld_agent(sm), s1 = ld_agent(sm + 1), s2 = ld_agent(sm + 2), s3 = ld_agent(sm + 3);
    broken = broken || s3 != 0 || s2 != L0;
    const uint64_t first_prev = b ? ld_agent(sm - 4) : s0;
    if (b) broken = broken || s0 < ld_agent(sm - 3) + L0;
    broken = broken || s1 + L0 - first_prev >= (1ull << 30);
  }
  broken = __syncthreads_or(broken);
  if (threadIdx.x == 0) {
    const uint32_t k = broken ? 0u : jrq_fixed_k(L0, a.n, a.lanes);
    a.gate[0] = L0 / (k ? k : 1u) <= (1ull << 23) ? k : 0u;
    a.gate[1] = L0;
    a.gate[2] = broken ? 1u : 0u;
    a.gate[3] = a.off[a.n];  // the records' end: crc64_fixed_kernel's load window
    __hip_atomic_store(a.gate + 4, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the arrival
    // count, zero for the next launch (the segment counters were re-zeroed by their last arrivers)
  }
}

__device__ void v2_parse_record(const JrqV2Args& a, uint32_t r, const uint64_t* T, uint8_t* win,
                                uint8_t& st_out, uint64_t& d_out, uint64_t& dl_out) {
  const uint64_t b0 = a.off[r];
  const int64_t L = static_cast<int64_t>(a.off[r + 1] - b0);
  const uint8_t* rec = a.rec + b0;
  uint8_t st = kV2Ok;
  int64_t idx = 0, tm = 0, doff = 0, dlen = 0;
  uint64_t ck = 0, pxor = 0;
  bool have_type = false, have_term = false, have_index = false, have_data = false,
       have_ck = false, host = false, deep = false;
  uint32_t etype = 0, counts = 0;
  if (L < 1) {
    st = kV2Null;
  } else {
    PbIn in(rec, L, win);
    const uint32_t m0 = in.rd.at(0);
    if (m0 != 0xBBu) {
      st = kV2V1;
    } else if (L < 6 || in.rd.at(1) != 0xD2u || in.rd.at(2) != 1u) {
      st = kV2Null;
    } else if (V2Fast f; v2_fast_fields(in.rd, L, f)) {  // the common encoding
      etype = f.etype;
      tm = f.term;
      idx = f.index;
      doff = f.doff;
      dlen = f.dlen;
      ck = f.ck;
      have_ck = f.have_ck;
    } else {
      uint32_t grp[2] = {0, 0};  // open unknown-field groups (field numbers)
      int depth = 0;
      bool stop = false;  // END_GROUP at top level
      while (!in.rd.err && !deep && !stop) {
        const uint32_t t = in.tag();
        if (in.rd.err) break;
        if (t == 0) {
          if (depth) in.rd.err = true;  // input ended inside a group
          break;
        }
        int64_t len = 0, at;
        if (depth == 0) {
          switch (t) {
            case 8: {  // type (enum): numbers outside EntryType stay unknown
              const int32_t v = static_cast<int32_t>(in.varint32());
              if (!in.rd.err && v >= 0 && v <= 3) {
                etype = static_cast<uint32_t>(v);
                have_type = true;
              }
              continue;
            }
            case 16: tm = static_cast<int64_t>(in.varint64()); have_term = true; continue;
            case 24: idx = static_cast<int64_t>(in.varint64()); have_index = true; continue;
            case 34: case 42: case 66: case 74: {
              at = in.bytes(&len);
              if (in.rd.err) continue;
              bool canon;
              pxor ^= peer_crc(in, at, len, T, &canon);
              host = host || !canon;
              const uint32_t sh = t == 34 ? 0 : t == 42 ? 8 : t == 66 ? 16 : 24;
              if (((counts >> sh) & 0xFFu) != 0xFFu) counts += 1u << sh;
              continue;
            }
            case 50:  // data: the last occurrence wins
              at = in.bytes(&len);
              if (!in.rd.err) {
                doff = at;
                dlen = len;
                have_data = true;
              }
              continue;
            case 56: ck = in.varint64(); have_ck = true; continue;
            default: break;
          }
        }
        // unknown field (any number / wire-type mismatch), inside a group or not
        switch (t & 7u) {
          case 0: (void)in.varint64(); break;
          case 1: in.skip(8); break;
          case 2: (void)in.bytes(&len); break;
          case 3:
            if (depth == 2) deep = true;  // deeper nesting: stop, decode on the host
            else grp[depth++] = t >> 3;
            break;
          case 4:
            if (depth == 0) stop = true;  // checkLastTagWas(0) fails below
            else if (grp[--depth] != (t >> 3)) in.rd.err = true;
            break;
          case 5: in.skip(4); break;
          default: in.rd.err = true;  // invalidWireType
        }
      }
      if (deep) st = kV2Host;
      else if (in.rd.err || stop || !have_type || !have_term || !have_index || !have_data) st = kV2Null;
      else if (host) st = kV2Host;
    }
  }
  if (st != kV2Ok) {
    etype = 0;
    idx = tm = 0;
    ck = 0;
    have_ck = false;
    doff = 0;
    dlen = 0;
    counts = 0;
    pxor = 0;
  }
  const uint64_t logid = crc_bytes_be(crc_bytes_be(0, static_cast<uint64_t>(idx), T),
                                      static_cast<uint64_t>(tm), T);
  a.partial[r] = st == kV2Ok ? (static_cast<uint64_t>(etype) ^ logid ^ pxor) : 0;
  a.status[r] = st;
  a.type[r] = static_cast<uint8_t>(etype);
  a.index[r] = idx;
  a.term[r] = tm;
  a.stored[r] = ck;
  a.has_checksum[r] = have_ck ? 1 : 0;
  a.data_off[r] = b0 + static_cast<uint64_t>(doff);
  a.data_len[r] = static_cast<uint64_t>(dlen);
  if (a.peer_counts) a.peer_counts[r] = counts;
  a.off2[r + 1] = b0 + static_cast<uint64_t>(doff);  // a failed record: its start
  // the lengths of the bytes around the data (v2_finish hashes and removes them from the
  // range CRCs when the segment walk runs)
  const uint64_t hl = st == kV2Ok ? static_cast<uint64_t>(doff) : 0;
  const uint64_t tl = st == kV2Ok ? static_cast<uint64_t>(L - doff - dlen) : 0;
  a.lens[r] = (hl << 32) | tl;
  st_out = st;
  d_out = b0 + static_cast<uint64_t>(doff);
  dl_out = static_cast<uint64_t>(dlen);
}

// The CRC pass hashes one range per record, [data start, next record's data start): the data,
// then a suffix of k bytes -- the record's trailer (checksum / learner fields) and the next
// record's header.  CRC64 here is linear (init 0, xorout 0) and x is invertible mod P
// (P(0) = 1), so
//   crc(suffix) = crc(trailer) * x^(8 |next header|) ^ crc(next header)
//   crc(data)   = (crc(range) ^ crc(suffix)) * x^(-8k)
// with the trailer / header CRCs hashed here from the record bytes.  A multiply by
// x^(+-64) is one lookup per register byte: T_i[b] = b x^(64 + 8i) (the engine's slice tables,
// un-swapped), TI_i[b] = b x^(8i - 64) (engine xinv); single bytes use T_0 / TI_7.  One entry
// boundary per record instead of two: the CRC pass takes 310 instead of 330 us on 64k x 16 KiB
// records (round 3's tools/v2_boundary_probe.py).
// (The fixed-size data path -- gate[0] != 0 -- finishes inside crc64_fixed_kernel: this kernel
// then returns at once.)
__global__ __launch_bounds__(256) void v2_finish(JrqV2Args a, JrqCrcArgs w) {
  __shared__ uint64_t Tf[8][256], Ti[8][256];
  if (a.gate[0] != 0) return;  // (grid-uniform)
  // the walk's geometry (w: the rounds kernel's arguments): a range's CRC is its out[] entry
  // or the XOR of its pieces -- assembled here, so the walk needs no crc64_finish_kernel
  const uint64_t* const off2 = w.offsets;
  const uint64_t wbase = off2[0];
  const uint64_t wD = reinterpret_cast<uintptr_t>(w.payload + wbase) & 15u;
  const uint64_t wS = seg_size(w, wD + (off2[w.n] - wbase));
  for (uint32_t e = threadIdx.x; e < 8 * 256; e += blockDim.x) {
    Tf[e >> 8][e & 255u] = bswap64(a.slice[e]);
    Ti[e >> 8][e & 255u] = a.xinv[e];
  }
  __syncthreads();
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += stride) {
    const bool ok = a.status[r] == kV2Ok;
    uint64_t c = 0;
    if (ok) {
      const bool more = r + 1 < a.n;
      uint64_t h = more ? a.lens[r + 1] >> 32 : 0;  // next record's header (0 if it failed)
      const uint64_t tl = a.lens[r] & 0xFFFFFFFFull, k = tl + h;
      // the CRCs of this record's trailer and the next record's header, from their bytes
      uint64_t s = 0, hc = 0;
      {
        const uint64_t e = a.off[r + 1];
        ChunkReader rd(a.rec + e - tl, static_cast<int64_t>(tl));
        for (uint64_t p = 0; p < tl; ++p) s = Tf[0][((s >> 56) ^ rd.at(static_cast<int64_t>(p))) & 0xFFu] ^ (s << 8);
        ChunkReader rn(a.rec + e, static_cast<int64_t>(h));
        for (uint64_t p = 0; p < h; ++p) hc = Tf[0][((hc >> 56) ^ rn.at(static_cast<int64_t>(p))) & 0xFFu] ^ (hc << 8);
      }
      for (; h >= 8; h -= 8) {  // s * x^64
        uint64_t t = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) t ^= Tf[i][(s >> (8 * i)) & 0xFFu];
        s = t;
      }
      for (; h > 0; --h) s = (s << 8) ^ Tf[0][s >> 56];
      s ^= hc;
      uint64_t range;
      if (!crc_pieces(w, off2[r + 1], off2[r + 2], wbase, wD, wS, range)) range = a.crc2[r + 1];
      uint64_t d = range ^ s, m = k;
      for (; m >= 8; m -= 8) {  // d * x^-64
        uint64_t t = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) t ^= Ti[i][(d >> (8 * i)) & 0xFFu];
        d = t;
      }
      for (; m > 0; --m) d = (d >> 8) ^ Ti[7][d & 0xFFu];
      c = a.partial[r] ^ d;  // d = crc(data)
    }
    a.computed[r] = c;
    a.corrupt[r] = (ok && a.has_checksum[r] && a.stored[r] != c) ? 1 : 0;
  }
}

}  // namespace jrq

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_v2_parse(
    const JrqV2Args* a, hipStream_t stream) {
  const uint32_t blocks = (a->n + 255) / 256;
  hipLaunchKernelGGL(jrq::v2_parse, dim3(blocks ? blocks : 1), dim3(256), 0, stream, *a);
  return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t jrq_launch_v2_finish(
    const JrqV2Args* a, const JrqCrcArgs* walk, int num_cus, hipStream_t stream) {
  // each workgroup stages 32 KiB of tables in LDS: one record per lane, at most 2 workgroups
  // per CU (a grid of 8 per CU re-read 64 MiB of tables from L2 for 64k records)
  uint32_t blocks = (a->n + 255) / 256;
  const uint32_t cap = static_cast<uint32_t>(num_cus) * 2u;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(jrq::v2_finish, dim3(blocks ? blocks : 1), dim3(256), 0, stream, *a, *walk);
  return hipGetLastError();
}
