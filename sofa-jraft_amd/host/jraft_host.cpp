// jraft_host.cpp -- C++ host mirror of BallotBox / LogEntry / CrcUtil over libjrq.so.
// See jraft_host.h.  No checksum or quorum arithmetic happens here: it is all
// delegated to the GPU through include/jrq.h.
#include "jraft_host.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <sstream>
#include <thread>

namespace jraft {

namespace {

void throwIfError(int rc, jrq_engine* e, const char* what) {
  if (rc != JRQ_OK) {
    std::string msg = std::string(what) + " failed (" + std::to_string(rc) + "): ";
    const char* t = jrq_last_error(e);
    if (t) msg += t;
    throw std::runtime_error(msg);
  }
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

}  // namespace

// ------------------------------------------------------------------ entities

std::string PeerId::toString() const {
  std::string s = ip + ":" + std::to_string(port);  // Endpoint.toString (Endpoint.java:60-65)
  if (idx != 0) s += ":" + std::to_string(idx);    // PeerId.toString (PeerId.java:135-144)
  return s;
}

bool PeerId::parse(const std::string& s, PeerId* out) {
  auto t = split(s, ':');
  if (t.size() != 2 && t.size() != 3) return false;
  try {
    out->ip = t[0];
    out->port = std::stoi(t[1]);
    out->idx = t.size() == 3 ? std::stoi(t[2]) : 0;
  } catch (...) {
    return false;
  }
  return true;
}

Configuration Configuration::parse(const std::string& s) {
  Configuration c;
  for (auto& item : split(s, ',')) {
    std::string p = item;
    bool learner = false;
    auto pos = p.find("/learner");  // LEARNER_POSTFIX (Configuration.java:45)
    if (pos != std::string::npos && pos > 0) {
      p = p.substr(0, pos);
      learner = true;
    }
    PeerId id;
    if (PeerId::parse(p, &id)) (learner ? c.learners : c.peers).push_back(id);
  }
  return c;
}

uint64_t LogEntry::checksum(Engine& eng) const { return eng.checksum({this})[0]; }

bool LogEntry::isCorrupted(Engine& eng) const { return eng.verify({this})[0] != 0; }

// ------------------------------------------------------------------- engine

Engine::Engine(int device, uint32_t max_groups, uint8_t max_peers) {
  int err = 0;
  e_ = jrq_create(device, max_groups, max_peers, &err);
  if (!e_) throw std::runtime_error(std::string("jrq_create: ") + jrq_last_error(nullptr));
}

Engine::~Engine() { jrq_destroy(e_); }

std::vector<uint64_t> Engine::crc64(const std::vector<std::vector<uint8_t>>& items) {
  std::vector<uint64_t> offs(items.size() + 1, 0);
  for (size_t i = 0; i < items.size(); ++i) offs[i + 1] = offs[i] + items[i].size();
  std::vector<uint8_t> payload(std::max<uint64_t>(offs.back(), 1));
  for (size_t i = 0; i < items.size(); ++i)
    if (!items[i].empty()) std::memcpy(payload.data() + offs[i], items[i].data(), items[i].size());
  std::vector<uint64_t> out(items.size());
  if (!items.empty())
    throwIfError(jrq_crc64_batch(e_, payload.data(), offs.data(), (uint32_t)items.size(), out.data()),
                 e_, "jrq_crc64_batch");
  return out;
}

uint64_t Engine::peerXor(const LogEntry& e, std::map<std::string, uint64_t>& cache) {
  // LogEntry.checksumPeers over peers, oldPeers, learners, oldLearners (LogEntry.java:101-108)
  uint64_t x = 0;
  for (auto* list : {&e.peers, &e.oldPeers, &e.learners, &e.oldLearners})
    for (auto& p : *list) x ^= cache.at(p.toString());
  return x;
}

std::vector<uint64_t> Engine::checksum(const std::vector<const LogEntry*>& entries) {
  // PeerId.checksum of every distinct peer string: one GPU CRC batch (PeerId.java:60-65)
  std::map<std::string, uint64_t> cache;
  for (auto* e : entries)
    for (auto* list : {&e->peers, &e->oldPeers, &e->learners, &e->oldLearners})
      for (auto& p : *list) cache.emplace(p.toString(), 0);
  if (!cache.empty()) {
    std::vector<std::vector<uint8_t>> strs;
    for (auto& kv : cache) strs.emplace_back(kv.first.begin(), kv.first.end());
    auto crcs = crc64(strs);
    size_t i = 0;
    for (auto& kv : cache) kv.second = crcs[i++];
  }
  const uint32_t n = (uint32_t)entries.size();
  std::vector<uint8_t> type(n);
  std::vector<int64_t> index(n), term(n);
  std::vector<uint64_t> px(n), offs(n + 1, 0), out(n);
  for (uint32_t i = 0; i < n; ++i) {
    type[i] = (uint8_t)entries[i]->type;
    index[i] = entries[i]->id.index;
    term[i] = entries[i]->id.term;
    px[i] = peerXor(*entries[i], cache);
    offs[i + 1] = offs[i] + entries[i]->data.size();
  }
  std::vector<uint8_t> payload(std::max<uint64_t>(offs[n], 1));
  for (uint32_t i = 0; i < n; ++i)
    if (!entries[i]->data.empty())
      std::memcpy(payload.data() + offs[i], entries[i]->data.data(), entries[i]->data.size());
  if (n)
    throwIfError(jrq_logentry_checksum_batch(e_, type.data(), index.data(), term.data(), px.data(),
                                             payload.data(), offs.data(), n, out.data(), nullptr,
                                             nullptr, nullptr),
                 e_, "jrq_logentry_checksum_batch");
  return out;
}

std::vector<uint8_t> Engine::verify(const std::vector<const LogEntry*>& entries) {
  auto sums = checksum(entries);
  // the GPU also provides the fused compare (jrq_logentry_checksum_batch verify mode);
  // here the stored checksums travel with the entries, so compare the returned values.
  std::vector<uint8_t> bad(entries.size());
  for (size_t i = 0; i < entries.size(); ++i)
    bad[i] = entries[i]->hasChecksum_ && entries[i]->checksum_ != sums[i];
  return bad;
}

uint64_t CrcUtil::crc64(Engine& eng, const uint8_t* array, size_t offset, size_t length) {
  if (array == nullptr) return 0;  // CrcUtil.crc64(null) -> 0
  std::vector<std::vector<uint8_t>> one(1);
  one[0].assign(array + offset, array + offset + length);
  return eng.crc64(one)[0];
}

void CRC64::update(const uint8_t* b, size_t off, size_t len) {
  if (len == 0) return;
  if (b == nullptr) throw std::invalid_argument("null buffer");  // Java: NullPointerException
  buf_.insert(buf_.end(), b + off, b + off + len);
  maybeFlush();
}

void CRC64::flush() {
  if (buf_.empty()) return;
  const uint64_t offs[2] = {0, buf_.size()};
  throwIfError(jrq_crc64_stream_update(eng_->raw(), &crc_, buf_.data(), offs, 1), eng_->raw(),
               "jrq_crc64_stream_update");
  buf_.clear();
}

uint64_t CRC64::getValue() {
  flush();
  return crc_;
}

// --------------------------------------------------------------- ballot box

// Persistent workers for flush()'s pack and deliver passes (spawning threads per flush cost
// ~2 ms on the GPU box): run(f) calls f(part, parts) on every worker and on the caller, and
// returns when all have finished; the first exception thrown by any part is rethrown.
struct GroupBatch::Pool {
  explicit Pool(unsigned n) {
    for (unsigned i = 1; i < n; ++i) th.emplace_back([this, i] { loop(i); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  unsigned size() const { return static_cast<unsigned>(th.size()) + 1; }
  void run(const std::function<void(unsigned, unsigned)>& f) {
    const unsigned n = size();
    err.assign(n, nullptr);
    {
      std::lock_guard<std::mutex> l(mu);
      job = &f;
      pending = n - 1;
      ++gen;
    }
    cv.notify_all();
    call(f, 0, n);
    std::unique_lock<std::mutex> l(mu);
    done.wait(l, [this] { return pending == 0; });
    job = nullptr;
    for (auto& e : err)
      if (e) std::rethrow_exception(e);
  }

 private:
  void call(const std::function<void(unsigned, unsigned)>& f, unsigned i, unsigned n) {
    try {
      f(i, n);
    } catch (...) {
      err[i] = std::current_exception();
    }
  }
  void loop(unsigned i) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(unsigned, unsigned)>* f;
      {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
        f = job;
      }
      call(*f, i, size());
      std::lock_guard<std::mutex> l(mu);
      if (--pending == 0) done.notify_one();
    }
  }
  std::vector<std::thread> th;
  std::vector<std::exception_ptr> err;
  std::mutex mu;
  std::condition_variable cv, done;
  const std::function<void(unsigned, unsigned)>* job = nullptr;
  uint64_t gen = 0;
  unsigned pending = 0;
  bool stop = false;
};

// f(begin, end) over [0, n) on the pool, only when each part gets at least `grain` items.
template <class F>
void GroupBatch::parallelFor(size_t n, size_t grain, F&& f) {
  if (n < 2 * grain) {
    f(size_t(0), n);
    return;
  }
  if (!pool_) {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    pool_.reset(new Pool(std::min(16u, hw)));  // the box's CPU share per GPU
  }
  const size_t parts = std::min<size_t>(pool_->size(), n / grain);
  pool_->run([&](unsigned i, unsigned) {
    if (i < parts) f(n * i / parts, n * (i + 1) / parts);
  });
}

template <class T>
void GroupBatch::PinnedBuf<T>::reserve(size_t n) {
  if (n <= cap) return;
  const size_t want = std::max(n, 2 * cap);
  const size_t bytes = ((want * sizeof(T)) + 4095) & ~size_t(4095);
  release();
  p = static_cast<T*>(std::aligned_alloc(4096, bytes));
  if (!p) throw std::bad_alloc();
  registered = jrq_host_register(p, bytes) == JRQ_OK;  // DMA straight from these pages
  cap = bytes / sizeof(T);
}

template <class T>
void GroupBatch::PinnedBuf<T>::release() {
  if (p) {
    if (registered) jrq_host_unregister(p);
    std::free(p);
  }
  p = nullptr;
  cap = 0;
  registered = false;
}

GroupBatch::GroupBatch(Engine* eng, uint32_t groups, uint32_t peers)
    : eng_(eng), G_(groups), P_(peers) {
  if (peers == 0 || peers > JRQ_MAX_PEERS) throw std::invalid_argument("peers must be 1..16");
  if (groups == 0 || groups > JRQ_TABLE_MAX_GROUPS) throw std::invalid_argument("groups must be 1..2^27");
  const size_t GP = static_cast<size_t>(G_) * P_;
  pi_.assign(G_, 0);
  lc_.assign(G_, 0);
  la_.assign(G_, -1);
  runs_.assign(static_cast<size_t>(G_) * JRQ_TABLE_MAX_RUNS, Run{0, 0});
  nruns_.assign(G_, 0);
  slotPeer_.assign(GP, kNoPeer);
  slotUse_.assign(GP, 0);
  match_.assign(GP, 0);
  dirty_.assign(G_, 0);
  waiter_.resize(G_);
  inited_.assign(G_, 0);
  closures_.resize(G_);
}

GroupBatch::~GroupBatch() {
  if (table_) jrq_table_destroy(table_);
}

uint32_t GroupBatch::internPeer(const PeerId& p) {
  auto it = peerIds_.find(p);
  if (it != peerIds_.end()) return it->second;
  const uint32_t id = static_cast<uint32_t>(peerIds_.size());
  peerIds_.emplace(p, id);
  return id;
}

// Slots named by the masks of the group's live conf runs: their peers vote on pending entries.
uint32_t GroupBatch::liveMask(uint32_t g) const {
  uint32_t m = 0;
  for (uint32_t r = 0; r < nruns_[g]; ++r) {
    const uint64_t cw = runs_[static_cast<size_t>(g) * JRQ_TABLE_MAX_RUNS + r].conf;
    m |= static_cast<uint32_t>(cw & 0xFFFFu) | static_cast<uint32_t>((cw >> 16) & 0xFFFFu);
  }
  return m;
}

// The slot of `peer` in group g.  create: a free slot, else the least recently acked slot that
// no live conf run names (and that is not in `reserved`), its match reset (its peer's acks no
// longer matter to any pending ballot).  Throws std::length_error when every slot is live.
int GroupBatch::slotOf(uint32_t g, uint32_t peer, bool create, uint32_t reserved) {
  const size_t base = static_cast<size_t>(g) * P_;
  int victim = -1;
  for (uint32_t s = 0; s < P_; ++s) {
    if (slotPeer_[base + s] == peer) return static_cast<int>(s);
    if (victim < 0 && slotPeer_[base + s] == kNoPeer) victim = static_cast<int>(s);
  }
  if (!create) return -1;
  if (victim < 0) {
    const uint32_t busy = liveMask(g) | reserved;
    for (uint32_t s = 0; s < P_; ++s)
      if (!((busy >> s) & 1u) && (victim < 0 || slotUse_[base + s] < slotUse_[base + victim]))
        victim = static_cast<int>(s);
    if (victim < 0)
      throw std::length_error("more distinct live peers in group " + std::to_string(g) +
                              " than the " + std::to_string(P_) + " peer slots");
  }
  slotPeer_[base + victim] = peer;
  slotUse_[base + victim] = flushes_;
  if (match_[base + victim] != 0) {
    match_[base + victim] = 0;
    markDirty(g, 1u << victim);
  }
  return victim;
}

uint64_t GroupBatch::confWord(uint32_t g, const Configuration& conf, const Configuration* old) {
  // Ballot.init (Ballot.java:63-85): peers only, quorum = size/2+1, oldQuorum 0 if null
  uint32_t nm = 0, om = 0;
  for (auto& p : conf.peers) nm |= 1u << slotOf(g, internPeer(p), true, nm | om);
  uint32_t nq = static_cast<uint32_t>(conf.peers.size()) / 2 + 1, oq = 0;
  if (old) {
    for (auto& p : old->peers) om |= 1u << slotOf(g, internPeer(p), true, nm | om);
    oq = static_cast<uint32_t>(old->peers.size()) / 2 + 1;
  }
  return JRQ_CONF(nm, om, nq, oq);
}

// Would a gap [lo, hi] in `slot`'s acks skip a pending entry whose ballot counts that slot?
bool GroupBatch::gapCountsPeer(uint32_t g, int slot, int64_t lo, int64_t hi) const {
  const Run* R = &runs_[static_cast<size_t>(g) * JRQ_TABLE_MAX_RUNS];
  const uint32_t n = nruns_[g];
  for (uint32_t r = 0; r < n; ++r) {
    const int64_t s = r == 0 ? pi_[g] : R[r].start;
    const int64_t e = r + 1 < n ? R[r + 1].start - 1 : la_[g];
    const uint64_t cw = R[r].conf;
    const uint32_t m = static_cast<uint32_t>(cw & 0xFFFFu) | static_cast<uint32_t>((cw >> 16) & 0xFFFFu);
    if (std::max(s, lo) <= std::min(e, hi) && ((m >> slot) & 1u)) return true;
  }
  return false;
}

// Drop runs wholly below pendingIndex (pendingMetaQueue.removeRange, BallotBox.java:130).
void GroupBatch::dropDeadRuns(uint32_t g) {
  Run* R = &runs_[static_cast<size_t>(g) * JRQ_TABLE_MAX_RUNS];
  uint32_t n = nruns_[g], k = 0;
  while (k + 1 < n && R[k + 1].start <= pi_[g]) ++k;
  if (k) {
    for (uint32_t r = k; r < n; ++r) R[r - k] = R[r];
    nruns_[g] = static_cast<uint8_t>(n - k);
  }
}

// BallotBox.commitAt's commit, after the epoch (:130-137): drop the ballots up to c, run their
// closures (ClosureQueue.popClosureUntil -> done.run(OK)), then waiter.onCommitted(c).
void GroupBatch::commitTo(uint32_t g, int64_t c) {
  if (auto& q = closures_[g]) {
    while (!q->empty() && q->front().first <= c) {
      auto done = std::move(q->front().second);
      q->pop_front();
      done(true);
    }
  }
  pi_[g] = c + 1;
  lc_[g] = c;
  dropDeadRuns(g);
  if (waiter_[g]) waiter_[g](c);
}

uint32_t GroupBatch::flush() {
  if (!eng_) throw std::logic_error("GroupBatch::flush needs an Engine");
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  stats_ = FlushStats{};
  if (!table_) {  // first flush: the device table starts empty, ship every group's state
    int err = 0;
    table_ = jrq_table_create(eng_->raw(), G_, P_, &err);
    if (!table_) throwIfError(err ? err : JRQ_E_NOMEM, eng_->raw(), "jrq_table_create");
    for (uint32_t g = 0; g < G_; ++g) {
      uint32_t bits = 0;
      if (pi_[g] != 0 || lc_[g] != 0 || nruns_[g] != 0) bits |= kDirtyHeader;
      for (uint32_t s = 0; s < P_; ++s)
        if (match_[static_cast<size_t>(g) * P_ + s] != 0) bits |= 1u << s;
      if (bits) markDirty(g, bits);
    }
  }
  // pack the changes: one header per group whose header changed, else 8-B records -- two
  // passes over the dirty groups (count, then fill at per-chunk offsets), split across threads
  const size_t nd = dirtyList_.size();
  const size_t kChunk = 1u << 12;
  const size_t nchunks = (nd + kChunk - 1) / kChunk;
  std::vector<uint32_t> cs(nchunks + 1, 0), cr(nchunks + 1, 0);
  parallelFor(nchunks, 1, [&](size_t c0, size_t c1) {
    for (size_t c = c0; c < c1; ++c) {
      uint32_t ns = 0, nr = 0;
      for (size_t i = c * kChunk, e = std::min(nd, (c + 1) * kChunk); i < e; ++i) {
        const uint32_t g = dirtyList_[i], d = dirty_[g];
        if (d & kDirtyHeader) ++ns;
        else if ((d & kDirtyLa) && pi_[g] != 0) ++nr;
        if (pi_[g] != 0) nr += static_cast<uint32_t>(__builtin_popcount(d & 0xFFFFu));
      }
      cs[c + 1] = ns;
      cr[c + 1] = nr;
    }
  });
  for (size_t c = 0; c < nchunks; ++c) {
    cs[c + 1] += cs[c];
    cr[c + 1] += cr[c];
  }
  const uint32_t ns = cs[nchunks], nr = cr[nchunks];
  states_.reserve(ns + 1);
  recs_.reserve(nr + 1);
  parallelFor(nchunks, 1, [&](size_t c0, size_t c1) {
    for (size_t c = c0; c < c1; ++c) {
      uint32_t si = cs[c], ri = cr[c];
      for (size_t i = c * kChunk, e = std::min(nd, (c + 1) * kChunk); i < e; ++i) {
        const uint32_t g = dirtyList_[i], d = dirty_[g];
        dirty_[g] = 0;
        const int64_t pi = pi_[g], base = pi - 1;
        if (d & kDirtyHeader) {
          jrq_group_state& st = states_.p[si++];
          std::memset(&st, 0, sizeof st);
          st.group = g;
          st.num_runs = nruns_[g];
          st.flags = (d & kDirtyReset) ? JRQ_STATE_RESET_MATCH : 0;
          // the table's steady-state encoding of pendingIndex = lastCommittedIndex + 1: the
          // group's next commit then writes lastCommitted only
          st.pending_index = (pi != 0 && pi == lc_[g] + 1) ? JRQ_PI_FOLLOWS_LC : pi;
          st.last_appended = la_[g];
          st.last_committed = lc_[g];
          const Run* R = &runs_[static_cast<size_t>(g) * JRQ_TABLE_MAX_RUNS];
          for (uint32_t r = 0; r < nruns_[g]; ++r) {
            st.run_conf[r] = R[r].conf;
            st.run_start[r] = R[r].start;
          }
        } else if ((d & kDirtyLa) && pi != 0) {
          recs_.p[ri++] = JRQ_REC(g, JRQ_REC_LAST_APPENDED, la_[g] - base);
        }
        if (pi == 0) continue;  // not the leader: its acks are refused (commitAt returns false)
        for (uint32_t m = d & 0xFFFFu; m; m &= m - 1) {
          const uint32_t s = static_cast<uint32_t>(__builtin_ctz(m));
          const int64_t v = match_[static_cast<size_t>(g) * P_ + s] - base;
          recs_.p[ri++] = JRQ_REC(g, s, v > 0 ? v : 0);
        }
      }
    }
  });
  dirtyList_.clear();
  changed_.reserve(G_);
  const auto t1 = clk::now();
  throwIfError(jrq_table_update(table_, states_.p, ns, recs_.p, nr), eng_->raw(), "jrq_table_update");
  uint32_t n = 0;
  throwIfError(jrq_table_epoch(table_, changed_.p, &n, nullptr), eng_->raw(), "jrq_table_epoch");
  const auto t2 = clk::now();
  // deliver: groups are independent, so their commits (closures, then onCommitted) run split
  // across threads; one group's callbacks run on one thread, in order.  A commit touches the
  // group in several host arrays at random places: prefetch a few groups ahead.
  parallelFor(n, 1u << 12, [&](size_t i0, size_t i1) {
    constexpr size_t kAhead = 8;
    for (size_t i = i0; i < i1; ++i) {
      if (i + kAhead < i1) {
        const uint32_t h = static_cast<uint32_t>(changed_.p[i + kAhead]);
        __builtin_prefetch(&pi_[h], 1);
        __builtin_prefetch(&lc_[h], 1);
        __builtin_prefetch(&nruns_[h], 0);
        __builtin_prefetch(&closures_[h], 0);
        __builtin_prefetch(&waiter_[h], 0);
      }
      const uint64_t w = changed_.p[i];
      const uint32_t g = static_cast<uint32_t>(w);
      commitTo(g, pi_[g] - 1 + static_cast<int64_t>(w >> 32));
    }
  });
  ++flushes_;
  const auto t3 = clk::now();
  auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
  stats_.states = ns;
  stats_.records = nr;
  stats_.changed = n;
  stats_.h2d_bytes = static_cast<uint64_t>(ns) * sizeof(jrq_group_state) + static_cast<uint64_t>(nr) * 8;
  stats_.d2h_bytes = 4 * JRQ_TABLE_SEGMENTS + static_cast<uint64_t>(n) * 8;
  stats_.pack_ms = ms(t1 - t0);
  stats_.device_ms = ms(t2 - t1);
  stats_.deliver_ms = ms(t3 - t2);
  return n;
}

BallotBox::BallotBox(std::shared_ptr<GroupBatch> batch, uint32_t group) : batch_(std::move(batch)), g_(group) {
  if (g_ >= batch_->groups()) throw std::out_of_range("group id");
}

bool BallotBox::init(const BallotBoxOptions& opts) {
  if (!opts.waiter || !opts.closureQueue) return false;  // "waiter or closure queue is null."
  batch_->waiter_[g_] = opts.waiter;
  batch_->inited_[g_] = 1;
  return true;
}

bool BallotBox::commitAt(int64_t first, int64_t last, const PeerId& peer) {
  GroupBatch& b = *batch_;
  const int64_t pi = b.pi_[g_];
  if (pi == 0) return false;                                     // :101-103
  if (last < pi) return true;                                    // :104-106
  if (last > b.la_[g_]) throw std::out_of_range("ArrayIndexOutOfBoundsException");  // :107-109
  const int s = b.slotOf(g_, b.internPeer(peer), true);
  const size_t k = static_cast<size_t>(g_) * b.P_ + s;
  int64_t& m = b.match_[k];
  const int64_t lo = std::max(m + 1, pi);
  if (first > lo && b.gapCountsPeer(g_, s, lo, first - 1))
    throw std::logic_error("non-contiguous ack: the Replicator never skips entries");
  if (last > m) {
    m = last;
    b.markDirty(g_, 1u << s);
  }
  b.slotUse_[k] = b.flushes_;
  return true;
}

void BallotBox::clearPendingTasks() {
  GroupBatch& b = *batch_;
  // Acks recorded since the last epoch would have committed at once in the reference
  // (BallotBox.commitAt decides synchronously): decide them before the queue is dropped.
  if ((b.dirty_[g_] & 0xFFFFu) && b.pi_[g_] != 0 && b.eng_) b.flush();
  if (auto& q = b.closures_[g_]) {
    for (auto& c : *q) c.second(false);  // ClosureQueue.clear runs closures with EPERM
    q->clear();
  }
  b.nruns_[g_] = 0;
  b.pi_[g_] = 0;
  b.la_[g_] = -1;
  b.markDirty(g_, GroupBatch::kDirtyHeader);
}

bool BallotBox::resetPendingIndex(int64_t n) {
  GroupBatch& b = *batch_;
  if (!(b.pi_[g_] == 0 && b.la_[g_] < b.pi_[g_])) return false;
  if (n <= b.lc_[g_]) return false;
  b.pi_[g_] = n;
  b.la_[g_] = n - 1;
  b.nruns_[g_] = 0;
  // a new leader's replicators start over
  std::fill(b.match_.begin() + static_cast<size_t>(g_) * b.P_,
            b.match_.begin() + static_cast<size_t>(g_ + 1) * b.P_, 0);
  b.markDirty(g_, GroupBatch::kDirtyHeader | GroupBatch::kDirtyReset);
  return true;
}

bool BallotBox::appendPendingTasks(const Configuration& conf, const Configuration* oldConf,
                                   int64_t count) {
  GroupBatch& b = *batch_;
  if (b.pi_[g_] <= 0) return false;  // :204-207
  if (count <= 0) return true;
  if (b.la_[g_] + count - b.pi_[g_] + 1 > INT32_MAX)  // pendingMetaQueue is a Java ArrayList
    throw std::length_error("pending queue larger than an ArrayList");
  const uint64_t cw = b.confWord(g_, conf, oldConf);
  GroupBatch::Run* R = &b.runs_[static_cast<size_t>(g_) * JRQ_TABLE_MAX_RUNS];
  uint8_t& n = b.nruns_[g_];
  const int64_t idx = b.la_[g_] + 1;
  if (n == 0 || R[n - 1].conf != cw) {  // Ballot.init with a new conf: a new conf run
    if (n == JRQ_TABLE_MAX_RUNS) {
      if (idx > b.pi_[g_])  // NodeImpl never has more than 2 (joint, then stable) pending
        throw std::length_error("more conf runs pending than JRQ_TABLE_MAX_RUNS");
      n = 0;  // the queue is empty: every earlier run is dead
    }
    R[n++] = GroupBatch::Run{idx, cw};
    b.dropDeadRuns(g_);
    b.markDirty(g_, GroupBatch::kDirtyHeader);
  }
  b.la_[g_] = idx + count - 1;
  b.markDirty(g_, GroupBatch::kDirtyLa);
  return true;
}

bool BallotBox::appendPendingTask(const Configuration& conf, const Configuration* oldConf,
                                  std::function<void(bool)> done) {
  GroupBatch& b = *batch_;
  if (b.pi_[g_] <= 0) return false;  // :204-207
  if (!appendPendingTasks(conf, oldConf, 1)) return false;
  if (done) {
    auto& q = b.closures_[g_];
    if (!q) q.reset(new std::deque<std::pair<int64_t, std::function<void(bool)>>>());
    q->emplace_back(b.la_[g_], std::move(done));
  }
  return true;
}

bool BallotBox::setLastCommittedIndex(int64_t c) {
  GroupBatch& b = *batch_;
  if (b.pi_[g_] != 0 || b.la_[g_] >= b.pi_[g_]) {
    if (!(c < b.pi_[g_]))  // Requires.requireTrue (:229-231)
      throw std::invalid_argument("Node changes to leader, pendingIndex=" +
                                  std::to_string(b.pi_[g_]) +
                                  ", param lastCommittedIndex=" + std::to_string(c));
    return false;
  }
  if (c < b.lc_[g_]) return false;
  if (c > b.lc_[g_]) {
    b.lc_[g_] = c;
    b.markDirty(g_, GroupBatch::kDirtyHeader);
    if (b.waiter_[g_]) b.waiter_[g_](c);
  }
  return true;
}

int64_t BallotBox::getLastCommittedIndex() const { return batch_->lc_[g_]; }
int64_t BallotBox::getPendingIndex() const { return batch_->pi_[g_]; }
int64_t BallotBox::getPendingMetaQueueSize() const {
  const GroupBatch& b = *batch_;
  return b.pi_[g_] == 0 ? 0 : b.la_[g_] - b.pi_[g_] + 1;
}

std::string BallotBox::describe() const {
  std::ostringstream o;
  o << "  lastCommittedIndex: " << getLastCommittedIndex() << "\n"
    << "  pendingIndex: " << getPendingIndex() << "\n"
    << "  pendingMetaQueueSize: " << getPendingMetaQueueSize() << "\n";
  return o.str();
}

}  // namespace jraft
