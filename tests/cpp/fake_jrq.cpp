// fake_jrq.cpp -- TEST DOUBLE of libjrq.so for CPU-only sanitizer builds of the host mirror.
//
// TEST INFRASTRUCTURE ONLY.  ThreadSanitizer and AddressSanitizer cannot instrument the GPU
// side, and this container has no GPU, so the sanitizer binaries (tests/cpp/Makefile:
// host_test_tsan, host_test_asan) link the host mirror (sofa-jraft_amd/host/jraft_host.cpp)
// against this stand-in instead of libjrq.so.  It implements the few entry points the mirror
// calls with the CPU oracle (oracle/jraft_oracle.c: the Java-faithful BallotBox replay and the
// byte-at-a-time CRC), so that every concurrent host-side path -- locks, dirty lists, packing,
// gathering, delivery, the flusher -- runs under the sanitizers with real epoch results.  It is
// never built into libjrq.so, libjraft_host.so or anything bench.py or smoke() loads; the GPU
// build of the same tests (tests/_build/host_test) links the real library.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_set>
#include <string>
#include <vector>

#include "../../include/jrq.h"
#include "../../oracle/jraft_oracle.h"

struct jrq_engine {
  std::string err;
};

namespace {
thread_local std::string g_err;
}

struct jrq_table {
  jrq_engine* e;
  uint32_t G, P;
  std::vector<int64_t> pi, la, lc, match;  // pi resolved (never JRQ_PI_FOLLOWS_LC)
  std::vector<uint8_t> nr;
  std::vector<int64_t> start;   // [G][JRQ_TABLE_MAX_RUNS]
  std::vector<uint64_t> conf;   // [G][JRQ_TABLE_MAX_RUNS]
  uint32_t invalid = 0;
  std::mutex mu;  // the real table orders calls on the engine stream
  std::vector<jrq_group_state> staged_s;  // jrq_table_stage: copied at once (the real one DMAs)
  std::vector<uint64_t> staged_r;
  std::vector<uint64_t> rstamp;           // JRQ_STATE_STAMP per group
  std::vector<uint64_t> staged_a;         // jrq_table_stage_acks: records, segments
  std::vector<uint64_t*> regions;         // jrq_table_ack_region (freed with the table)
  std::vector<std::pair<size_t, uint64_t>> segs;
};

extern "C" {

jrq_engine* jrq_create(int, uint32_t, uint8_t, int* err) {
  if (err) *err = JRQ_OK;
  return new jrq_engine();
}
void jrq_destroy(jrq_engine* e) { delete e; }
const char* jrq_last_error(const jrq_engine* e) { return e ? e->err.c_str() : g_err.c_str(); }
int jrq_synchronize(jrq_engine* e) { return e ? JRQ_OK : JRQ_E_INVALID; }  // (calls complete at once)
int jrq_host_register(void* p, size_t n) { return p && n ? JRQ_OK : JRQ_E_INVALID; }
int jrq_host_unregister(void* p) { return p ? JRQ_OK : JRQ_E_INVALID; }
int jrq_host_alloc(size_t n, void** out) {
  if (!out) return JRQ_E_INVALID;
  *out = n ? std::aligned_alloc(4096, (n + 4095) & ~size_t(4095)) : nullptr;
  return *out ? JRQ_OK : (n ? JRQ_E_NOMEM : JRQ_E_INVALID);
}
int jrq_host_free(void* p) {
  if (!p) return JRQ_E_INVALID;
  std::free(p);
  return JRQ_OK;
}

int jrq_crc64_batch(jrq_engine*, const uint8_t* payload, const uint64_t* offsets, uint32_t N,
                    uint64_t* crc_out) {
  std::vector<uint64_t> off(offsets, offsets + N + 1);
  for (auto& o : off) o -= offsets[0];
  jo_crc64_batch(payload + offsets[0], off.data(), N, crc_out);
  return JRQ_OK;
}

int jrq_crc64_stream_update(jrq_engine*, uint64_t* state, const uint8_t* payload,
                            const uint64_t* offsets, uint32_t S) {
  for (uint32_t s = 0; s < S; ++s)
    state[s] = jo_crc64_update(state[s], payload + offsets[s], offsets[s + 1] - offsets[s]);
  return JRQ_OK;
}

int jrq_logentry_checksum_batch(jrq_engine*, const uint8_t* type, const int64_t* index,
                                const int64_t* term, const uint64_t* peer_xor,
                                const uint8_t* payload, const uint64_t* offsets, uint32_t N,
                                uint64_t* out, const uint64_t* expected, const uint8_t* has,
                                uint8_t* corrupt_out) {
  std::vector<uint64_t> off(offsets, offsets + N + 1);
  for (auto& o : off) o -= offsets[0];
  jo_logentry_checksum_batch(type, index, term, peer_xor, payload + offsets[0], off.data(), N, out,
                             expected, has, corrupt_out);
  return JRQ_OK;
}

jrq_table* jrq_table_create(jrq_engine* e, uint32_t G, uint32_t P, int* err) {
  auto* t = new jrq_table();
  t->e = e;
  t->G = G;
  t->P = P;
  t->pi.assign(G, 0);
  t->la.assign(G, 0);
  t->lc.assign(G, 0);
  t->match.assign(static_cast<size_t>(G) * P, 0);
  t->nr.assign(G, 0);
  t->start.assign(static_cast<size_t>(G) * JRQ_TABLE_MAX_RUNS, 0);
  t->conf.assign(static_cast<size_t>(G) * JRQ_TABLE_MAX_RUNS, 0);
  t->rstamp.assign(G, 0);
  if (err) *err = JRQ_OK;
  return t;
}
void jrq_table_destroy(jrq_table* t) {
  if (!t) return;
  for (uint64_t* r : t->regions) delete[] r;
  delete t;
}

// Failure injection for the host tests (tests/cpp/host_test.cpp testFlushFailureRelists): the
// next `n` update calls fail as a lost device would, after applying nothing.
static std::atomic<int> g_fail_updates{0};
void fake_jrq_fail_updates(int n) { g_fail_updates.store(n); }
// Records of one upload naming the same (group, field) twice: the device applies an upload's
// records in parallel, so which of the two lands is not defined -- the host must never send
// them (the double applies records last to first, so the older value wins, and counts them).
static std::atomic<uint64_t> g_dup_records{0};
uint64_t fake_jrq_dup_records() { return g_dup_records.load(); }

int jrq_table_update_gather(jrq_table* t, uint32_t parts, const jrq_group_state* const* states,
                            const uint32_t* n_states, const uint64_t* const* recs,
                            const uint32_t* n_recs) {
  if (g_fail_updates.load() > 0) {
    g_fail_updates.fetch_sub(1);
    t->e->err = "injected update failure";
    return JRQ_E_HIP;
  }
  std::lock_guard<std::mutex> l(t->mu);
  for (uint32_t i = 0; i < parts; ++i)  // headers of every part first (include/jrq.h)
    for (uint32_t k = 0; k < n_states[i]; ++k) {
      const jrq_group_state& s = states[i][k];
      const int64_t pi = s.pending_index == JRQ_PI_FOLLOWS_LC ? s.last_committed + 1 : s.pending_index;
      if (s.group >= t->G || s.num_runs > JRQ_TABLE_MAX_RUNS ||
          (s.num_runs == 0 && pi != 0 && s.last_appended >= pi)) {
        ++t->invalid;
        continue;
      }
      const uint32_t g = s.group;
      t->pi[g] = pi;
      t->la[g] = s.last_appended;
      t->lc[g] = s.last_committed;
      t->nr[g] = static_cast<uint8_t>(s.num_runs);
      for (uint32_t r = 0; r < JRQ_TABLE_MAX_RUNS; ++r) {
        t->start[g * JRQ_TABLE_MAX_RUNS + r] = s.run_start[r];
        t->conf[g * JRQ_TABLE_MAX_RUNS + r] = s.run_conf[r] & ~JRQ_CONF_RUNS;
      }
      if (s.flags & JRQ_STATE_STAMP) {  // run_start[0] carries the reset stamp (run 0 has none)
        t->rstamp[g] = static_cast<uint64_t>(s.run_start[0]);
        t->start[g * JRQ_TABLE_MAX_RUNS] = 0;
      }
      if (s.flags & JRQ_STATE_RESET_MATCH)
        for (uint32_t p = 0; p < t->P; ++p) t->match[static_cast<size_t>(g) * t->P + p] = pi - 1;
    }
  {
    std::unordered_set<uint64_t> seen;
    for (uint32_t i = 0; i < parts; ++i)
      for (uint32_t k = 0; k < n_recs[i]; ++k)
        if (!seen.insert(recs[i][k] & 0xFFFFFFFFull).second) g_dup_records.fetch_add(1);
  }
  for (uint32_t i = parts; i-- > 0;)
    for (uint32_t k = n_recs[i]; k-- > 0;) {
      const uint64_t r = recs[i][k];
      const uint32_t f = static_cast<uint32_t>(r & 31u), g = static_cast<uint32_t>(r >> 5) & ((1u << 27) - 1u);
      const int64_t v = static_cast<int64_t>(static_cast<uint32_t>(r >> 32));
      if (g >= t->G || f > 16u || (f < 16u && f >= t->P)) {
        ++t->invalid;
        continue;
      }
      const int64_t val = t->pi[g] - 1 + v;
      if (f == 16u) {
        if (t->nr[g] == 0 && t->pi[g] != 0 && val >= t->pi[g]) {
          ++t->invalid;
          continue;
        }
        t->la[g] = val;
      } else {
        t->match[static_cast<size_t>(g) * t->P + f] = val;
      }
    }
  return JRQ_OK;
}

int jrq_table_stage_reserve(jrq_table* t, uint32_t, uint32_t) {
  std::lock_guard<std::mutex> l(t->mu);
  t->staged_s.clear();
  t->staged_r.clear();
  return JRQ_OK;
}

int jrq_table_stage(jrq_table* t, const jrq_group_state* states, uint32_t n_states,
                    const uint64_t* recs, uint32_t n_recs) {
  std::lock_guard<std::mutex> l(t->mu);
  t->staged_s.insert(t->staged_s.end(), states, states + n_states);
  t->staged_r.insert(t->staged_r.end(), recs, recs + n_recs);
  return JRQ_OK;
}

int jrq_table_stage_reserve_acks(jrq_table* t, uint32_t, uint32_t) {
  std::lock_guard<std::mutex> l(t->mu);
  t->staged_a.clear();
  t->segs.clear();
  return JRQ_OK;
}

int jrq_table_stage_acks(jrq_table* t, uint64_t stamp, const uint64_t* acks, uint32_t n) {
  std::lock_guard<std::mutex> l(t->mu);
  if (!n) return JRQ_OK;
  t->segs.emplace_back(t->staged_a.size(), stamp);
  t->staged_a.insert(t->staged_a.end(), acks, acks + n);
  return JRQ_OK;
}

// Streamed records (jrq_table_ack_region / _push / jrq_table_stage_acks_dev): regions are host
// memory here and a push copies at once (it touches no table state: callable from any thread).
int jrq_table_ack_region(jrq_table* t, uint64_t capacity, uint64_t** region_out) {
  std::lock_guard<std::mutex> l(t->mu);
  *region_out = new uint64_t[capacity];
  t->regions.push_back(*region_out);
  return JRQ_OK;
}
int jrq_table_ack_region_free(jrq_table* t, uint64_t* region) {
  std::lock_guard<std::mutex> l(t->mu);
  auto it = std::find(t->regions.begin(), t->regions.end(), region);
  if (it == t->regions.end()) return JRQ_E_INVALID;
  t->regions.erase(it);
  delete[] region;
  return JRQ_OK;
}
int jrq_table_ack_push(jrq_table*, uint64_t* dst, const uint64_t* src, uint32_t n) {
  std::memcpy(dst, src, static_cast<size_t>(n) * 8);
  return JRQ_OK;
}
int jrq_table_stage_acks_dev(jrq_table* t, uint64_t stamp, const uint64_t* acks, uint32_t n) {
  return jrq_table_stage_acks(t, stamp, acks, n);
}

int jrq_table_stage_apply(jrq_table* t) {
  std::vector<jrq_group_state> s;
  std::vector<uint64_t> r, a;
  std::vector<std::pair<size_t, uint64_t>> segs;
  {
    std::lock_guard<std::mutex> l(t->mu);
    std::swap(s, t->staged_s);
    std::swap(r, t->staged_r);
    std::swap(a, t->staged_a);
    std::swap(segs, t->segs);
  }
  const jrq_group_state* sp = s.data();  // (update_gather carries the failure injection)
  const uint64_t* rp = r.data();
  const uint32_t ns = static_cast<uint32_t>(s.size()), nr = static_cast<uint32_t>(r.size());
  const int rc = jrq_table_update_gather(t, 1, &sp, &ns, &rp, &nr);
  if (rc) return rc;
  // the order-free ack records (include/jrq.h JRQ_ACK): after the headers and records, a max,
  // records stamped before their group's last reset dropped
  std::lock_guard<std::mutex> l(t->mu);
  for (size_t k = 0; k < segs.size(); ++k) {
    const size_t e = k + 1 < segs.size() ? segs[k + 1].first : a.size();
    for (size_t i = segs[k].first; i < e; ++i) {
      const uint64_t w = a[i];
      const uint32_t f = static_cast<uint32_t>(w & 31u), g = static_cast<uint32_t>(w >> 5) & ((1u << 27) - 1u);
      if (g >= t->G || f > 16u || (f < 16u && f >= t->P)) {
        ++t->invalid;
        continue;
      }
      if (segs[k].second < t->rstamp[g] || t->pi[g] <= 0) continue;
      const int64_t b = t->pi[g] - 1;
      const int64_t v = b + static_cast<int32_t>(static_cast<uint32_t>(w >> 32) - static_cast<uint32_t>(b));
      if (f == 16u) {
        if (v - t->pi[g] >= 0x7FFFFFFF || (t->nr[g] == 0 && v >= t->pi[g])) {
          ++t->invalid;
          continue;
        }
        t->la[g] = std::max(t->la[g], v);
      } else {
        int64_t& m = t->match[static_cast<size_t>(g) * t->P + f];
        m = std::max(m, v);
      }
    }
  }
  return JRQ_OK;
}

// The single-process snapshot (include/jrq.h jrq_snapshot): "device" memory is host memory
// here; RCCL is never available, so it publishes by copies, as two engines on one GPU do.
int jrq_rccl_init_all(jrq_engine* const* engines, int n) {
  if (!engines || n <= 0) return JRQ_E_INVALID;
  engines[0]->err = "ncclCommInitAll: not in the test double";
  return JRQ_E_RCCL;
}
int jrq_table_committed_dev(jrq_table* t, int64_t* out) {
  std::lock_guard<std::mutex> l(t->mu);
  std::copy(t->lc.begin(), t->lc.end(), out);
  return JRQ_OK;
}
int jrq_publish_committed_all_dev(jrq_engine* const*, int n, const int64_t* const* local,
                                  int64_t* const* global, uint64_t count) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) std::copy(local[j], local[j] + count, global[i] + static_cast<size_t>(j) * count);
  return JRQ_OK;
}
struct jrq_snapshot {
  std::vector<jrq_table*> t;
  uint64_t k = 0;
  std::vector<std::vector<int64_t>> local, global;
};
jrq_snapshot* jrq_snapshot_create(jrq_table* const* tables, int n, int* err) {
  auto* s = new jrq_snapshot();
  s->t.assign(tables, tables + n);
  s->k = tables[0]->G;
  s->local.assign(n, std::vector<int64_t>(s->k, -1));
  s->global.assign(n, std::vector<int64_t>(s->k * n, -1));
  if (err) *err = JRQ_OK;
  return s;
}
void jrq_snapshot_destroy(jrq_snapshot* s) { delete s; }
int jrq_snapshot_publish(jrq_snapshot* s) {
  const int n = static_cast<int>(s->t.size());
  std::vector<const int64_t*> loc;
  std::vector<int64_t*> glob;
  for (int i = 0; i < n; ++i) {
    jrq_table_committed_dev(s->t[i], s->local[i].data());
    loc.push_back(s->local[i].data());
    glob.push_back(s->global[i].data());
  }
  return jrq_publish_committed_all_dev(nullptr, n, loc.data(), glob.data(), s->k);
}
int jrq_snapshot_read(jrq_snapshot* s, int i, int64_t* out) {
  uint64_t at = 0;
  for (size_t j = 0; j < s->t.size(); ++j) {
    std::copy(s->global[i].begin() + s->k * j, s->global[i].begin() + s->k * j + s->t[j]->G, out + at);
    at += s->t[j]->G;
  }
  return JRQ_OK;
}
int jrq_snapshot_via(const jrq_snapshot*) { return 0; }

#ifdef FAKE_JRQ_CLOSED_FORM
// The host-API cost probe (tools/api_probe.py) needs 1M-group epochs in milliseconds, not the
// replay's seconds: the closed form of DESIGN.md §1 (a run [s, e] commits min(e, k_new, k_old)
// when that is >= max(s, pendingIndex)), status left 0.
static int64_t kth(const int64_t* m, uint32_t P, uint32_t mask, uint32_t q) {
  if (q == 0) return INT64_MAX;
  int64_t v[16];
  uint32_t n = 0;
  for (uint32_t p = 0; p < P; ++p)
    if ((mask >> p) & 1u) v[n++] = m[p];
  if (n < q) return INT64_MIN;
  std::partial_sort(v, v + q, v + n, [](int64_t a, int64_t b) { return a > b; });
  return v[q - 1];
}
#endif

// One epoch, group by group through the oracle's BallotBox replay (jo_quorum_epoch_replay).
int jrq_table_epoch(jrq_table* t, uint64_t* changed_out, uint32_t* n_changed, uint8_t* status_out) {
  std::lock_guard<std::mutex> l(t->mu);
  uint32_t n = 0;
  std::vector<int64_t> m(t->P);
  for (uint32_t g = 0; g < t->G; ++g) {
    if (status_out) status_out[g] = JO_ST_NOT_LEADER;
    if (t->pi[g] == 0 || t->nr[g] == 0) continue;
    for (uint32_t p = 0; p < t->P; ++p) m[p] = t->match[static_cast<size_t>(g) * t->P + p];
    int64_t c = t->lc[g];
    uint8_t st = 0;
#ifdef FAKE_JRQ_CLOSED_FORM
    for (uint32_t r = 0; r < t->nr[g]; ++r) {
      const uint64_t cw = t->conf[g * JRQ_TABLE_MAX_RUNS + r];
      const int64_t s = std::max(r == 0 ? t->pi[g] : t->start[g * JRQ_TABLE_MAX_RUNS + r], t->pi[g]);
      const int64_t e = r + 1 < t->nr[g] ? t->start[g * JRQ_TABLE_MAX_RUNS + r + 1] - 1 : t->la[g];
      const int64_t k = std::min({e, kth(m.data(), t->P, cw & 0xFFFFu, (cw >> 32) & 0xFFu),
                                  kth(m.data(), t->P, (cw >> 16) & 0xFFFFu, (cw >> 40) & 0xFFu)});
      if (k >= s && k > c) c = k;
    }
#else
    const uint32_t ro[2] = {0, t->nr[g]};
    jo_quorum_epoch_replay(1, t->P, m.data(), &t->pi[g], &t->la[g], &t->lc[g],
                           &t->conf[g * JRQ_TABLE_MAX_RUNS], ro, &t->start[g * JRQ_TABLE_MAX_RUNS],
                           &t->conf[g * JRQ_TABLE_MAX_RUNS], 64, &c, &st);
#endif
    if (status_out) status_out[g] = st;
    if (c > t->lc[g]) {
      changed_out[n++] = (static_cast<uint64_t>(c - t->pi[g] + 1) << 32) | g;
      t->lc[g] = c;
      t->pi[g] = c + 1;
    }
  }
  *n_changed = n;
  return JRQ_OK;
}

// the follower / reader / leader-tick paths of the host mirror, decided by the oracle
int jrq_append_entries_verify(jrq_engine*, uint32_t R, const uint32_t* req_off, const int64_t* prev,
                              uint32_t, const int64_t* term, const uint8_t* type,
                              const int64_t* data_len, const uint64_t* peer_xor,
                              const uint64_t* checksum, const uint8_t* has, const uint8_t* data,
                              uint64_t* checksum_out, uint8_t* corrupt_out, int32_t* first_out) {
  jo_append_entries_verify(R, req_off, prev, term, type, data_len, peer_xor, checksum, has, data,
                           checksum_out, corrupt_out, first_out);
  return JRQ_OK;
}

int jrq_v2_decode_verify(jrq_engine*, const uint8_t* rec, const uint64_t* off, uint32_t N,
                         uint8_t* status, uint8_t* type, int64_t* index, int64_t* term,
                         uint64_t* stored, uint8_t* has, uint64_t* doff, uint64_t* dlen,
                         uint32_t* pc, uint64_t* sum, uint8_t* corrupt) {
  jo_v2_decode_batch(rec, off, N, status, type, index, term, stored, has, doff, dlen, pc, sum, corrupt);
  return JRQ_OK;
}

int jrq_leader_tick(jrq_engine*, const int64_t* ts, uint64_t ld, uint32_t P, const uint64_t* conf,
                    const uint8_t* self, uint32_t G, int64_t now, int64_t timeout, uint8_t* ok,
                    int64_t* lease, uint16_t* dead, const uint64_t* order, const uint16_t* okm,
                    uint8_t* ri) {
  if (ld != G) return JRQ_E_INVALID;  // (the mirror's rows are G apart)
  jo_lease_check(G, P, ts, conf, self, now, timeout, ok, lease, dead);
  if (order) jo_readindex_quorum(G, P, conf, self, order, okm, ri);
  return JRQ_OK;
}

int jrq_commit_fanout(jrq_engine*, uint32_t G, const int64_t* prev, const int64_t* committed,
                      const int64_t* last_applied, int64_t* cq_first, int64_t* cq_size,
                      int64_t* first_out, uint8_t* status, uint64_t* listed, uint32_t* num_listed) {
  std::vector<uint64_t> off(G + 1, 0);
  std::vector<int64_t> seq;
  for (uint32_t g = 0; g < G; ++g) {
    if (committed[g] > prev[g]) seq.push_back(committed[g]);  // one onCommitted per moved group
    off[g + 1] = seq.size();
  }
  std::vector<int64_t> la(last_applied, last_applied + G);
  jo_commit_fanout_replay(G, off.data(), seq.data(), la.data(), cq_first, cq_size, first_out, status);
  uint32_t n = 0;
  for (uint32_t w = 0; w < (G + 63) / 64; ++w) listed[w] = 0;
  for (uint32_t g = 0; g < G; ++g)
    if (status[g] == JRQ_FAN_APPLY || status[g] == JRQ_FAN_INVALID) {
      listed[g >> 6] |= 1ull << (g & 63);
      ++n;
    }
  *num_listed = n;
  return JRQ_OK;
}

}  // extern "C"
