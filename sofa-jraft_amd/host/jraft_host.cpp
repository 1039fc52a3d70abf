// jraft_host.cpp -- C++ host mirror of BallotBox / LogEntry / CrcUtil over libjrq.so.
// See jraft_host.h.  No checksum or quorum arithmetic happens here: it is all
// delegated to the GPU through include/jrq.h.
#include "jraft_host.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <sstream>
#include <thread>

#include <linux/membarrier.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace jraft {

namespace testing {
void (*fastPathHook)() = nullptr;
void (*slotAssignHook)() = nullptr;
std::atomic<uint32_t> ackChunkRecords{GroupBatch::kAckChunk};
}  // namespace testing

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
  std::string s = ip_ + ":" + std::to_string(port_);  // Endpoint.toString (Endpoint.java:60-65)
  if (idx_ != 0) s += ":" + std::to_string(idx_);    // PeerId.toString (PeerId.java:135-144)
  return s;
}

bool PeerId::parse(const std::string& s, PeerId* out) {
  auto t = split(s, ':');
  if (t.size() != 2 && t.size() != 3) return false;
  try {
    const int32_t port = std::stoi(t[1]);
    const int32_t idx = t.size() == 3 ? std::stoi(t[2]) : 0;
    out->ip_ = t[0];
    out->port_ = port;
    out->idx_ = idx;
  } catch (...) {
    return false;
  }
  out->internId.store(0, std::memory_order_relaxed);  // new contents: look the id up again
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

std::vector<uint64_t> Engine::peerChecksums(const std::vector<const LogEntry*>& entries) {
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
  std::vector<uint64_t> px(entries.size());
  for (size_t i = 0; i < entries.size(); ++i) px[i] = peerXor(*entries[i], cache);
  return px;
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

// ------------------------------------------------------------ peer interning

namespace {

// Process-wide PeerId -> id table (ids from 1; PeerId::internId 0 = not looked up).  A PeerId
// only changes through PeerId::parse, which clears its cached id, so a cached id is current
// and a lookup is one load; Java compares PeerIds by value (PeerId.equals -> Endpoint.equals ->
// String.equals, PeerId.java:180-199), and equal PeerIds intern to the same id.
class PeerRegistry {
 public:
  static PeerRegistry& get() {
    static PeerRegistry r;
    return r;
  }
  uint32_t id(const PeerId& p) {
    const uint32_t c = p.internId.load(std::memory_order_relaxed);
    if (c != 0) return c;
    uint32_t i;
    {
      std::lock_guard<std::mutex> l(mu_);
      auto it = map_.find(p);
      if (it != map_.end()) {
        i = it->second;
      } else {
        if (next_ >= (1u << 24)) throw std::length_error("more than 2^24 distinct PeerIds");
        i = next_++;
        map_.emplace(p, i);
      }
    }
    p.internId.store(i, std::memory_order_relaxed);
    return i;
  }

 private:
  struct Hash {
    size_t operator()(const PeerId& p) const {
      return std::hash<std::string>()(p.getIp()) ^ (static_cast<size_t>(p.getPort()) << 20) ^
             (static_cast<size_t>(p.getIdx()) << 40);
    }
  };
  std::mutex mu_;
  std::unordered_map<PeerId, uint32_t, Hash> map_;
  uint32_t next_ = 1;
};

inline uint32_t peerId(const PeerId& p) { return PeerRegistry::get().id(p); }

std::atomic<uint64_t> g_batchSerial{1};
// the batch whose commits this thread is delivering (flush / clearPendingTasks must not re-enter)
thread_local const GroupBatch* tl_delivering = nullptr;

int64_t nowNs() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Relaxed atomic access to record fields that commitAt's fast path reads or writes without
// the group's lock (plain moves on x86; they keep the concurrent accesses well defined).
template <class T>
inline T ald(const T& x) {
  return __atomic_load_n(&x, __ATOMIC_RELAXED);
}
template <class T>
inline void ast(T& x, T v) {
  __atomic_store_n(&x, v, __ATOMIC_RELAXED);
}

// Slot stamps (slotUse): the generation of the slot's last raising ack in 15 bits, bit 15 set
// when that ack changed the match (the pack ships the slot) -- a slot assignment stamps without
// it.  older(a, b): a's generation precedes b's (circularly, in 15 bits).
constexpr uint16_t kStampChanged = 0x8000u;
inline uint16_t stampOf(uint32_t gen, bool changed) {
  return static_cast<uint16_t>((gen & 0x7FFFu) | (changed ? kStampChanged : 0u));
}
inline bool stampOlder(uint16_t a, uint16_t b) { return ((a - b) & 0x7FFFu) >= 0x4000u; }
inline bool stampChangedIn(uint16_t u, uint32_t gen) {
  return (u & kStampChanged) && (u & 0x7FFFu) == (gen & 0x7FFFu);
}

// The asymmetric barrier pair behind the call regions: a caller's region entry is a plain
// store and a compiler barrier; the rare side (flush, quiesce) runs membarrier(2), which puts a
// full barrier on every thread of the process, before it reads the callers' counters.  Without
// membarrier the callers' entry becomes a full barrier (a locked store) instead.
bool registerMembarrier() {
  const long q = syscall(__NR_membarrier, MEMBARRIER_CMD_QUERY, 0, 0);
  if (q < 0 || !(q & MEMBARRIER_CMD_PRIVATE_EXPEDITED)) return false;
  return syscall(__NR_membarrier, MEMBARRIER_CMD_REGISTER_PRIVATE_EXPEDITED, 0, 0) == 0;
}
const bool g_membarrier = registerMembarrier();

// Callers that entered their regions with the cheap entry (g_membarrier) rely on this barrier
// for the store->load order quiesce and flush need; a local fence cannot give it, so a failing
// membarrier after a successful registration is fatal rather than a silent downgrade.
void heavyBarrier() {
  if (!g_membarrier) {
    std::atomic_thread_fence(std::memory_order_seq_cst);
    return;
  }
  if (syscall(__NR_membarrier, MEMBARRIER_CMD_PRIVATE_EXPEDITED, 0, 0) != 0) {
    std::fprintf(stderr, "jraft_host: membarrier(PRIVATE_EXPEDITED) failed after registration\n");
    std::abort();
  }
}

// a one-byte spin lock (calls hold it for a few hundred ns at most)
inline void spinLock(std::atomic<uint8_t>& l) {
  for (unsigned n = 0; l.exchange(1, std::memory_order_acquire) != 0; ++n) {
    if (n < 64) {
      __builtin_ia32_pause();
    } else {
      std::this_thread::yield();
    }
  }
}

}  // namespace

// --------------------------------------------------------------- ballot box

// One calling thread's state in a batch (cache-line aligned: the lists of different threads are
// written concurrently, each by its own thread): the groups it listed in generation t, in
// v[t & 1] (written only by the thread, inside its call regions; flush() takes v[t & 1] once
// generation t has ended and its regions have drained), and the region counter (odd inside).
struct alignas(128) GroupBatch::DirtyList {
  std::atomic<uint32_t> seq{0};
  std::vector<uint32_t> v[2];
  std::atomic<size_t> n[2] = {};          // v[i].size(), for the flusher's policy
  std::atomic<int64_t> firstNs[2] = {};   // when v[i] got its first group
  // the order-free records (JRQ_ACK) the thread wrote in generation t, in ack[t & 1]: page-locked
  // (jrq_host_alloc, sized by the flushing thread between uses), DMA-ed as they are; nack[i]
  // records, in segments (first record, reset stamp) of seg[i]
  PinnedBuf<uint64_t> ack[2];
  uint32_t nack[2] = {};
  // ack[i]'s device region (jrq_table_ack_region, as many records as ack[i].cap; set before the
  // capacity is published) and how many of its records the thread has pushed there so far: full
  // chunks go up while the thread writes (jrq_table_ack_push), the flush pushes the rest
  uint64_t* dack[2] = {};
  size_t dcap[2] = {};
  uint32_t shipped[2] = {};
  std::vector<std::pair<uint32_t, uint64_t>> seg[2];
};

namespace {
// One call region of the calling thread (see GroupBatch's threading note): the accesses between
// entry and exit that the flush or a quiescing writer must see complete.  No lock is taken and
// no thread is waited for inside one.
struct Region {
  std::atomic<uint32_t>& seq;
  uint32_t s;
  explicit Region(std::atomic<uint32_t>& q) : seq(q), s(q.load(std::memory_order_relaxed)) {
    if (g_membarrier) {
      seq.store(s + 1, std::memory_order_relaxed);
      std::atomic_signal_fence(std::memory_order_seq_cst);
    } else {
      // without membarrier the entry itself must order this store before the region's loads
      // (of the gate byte, the slot ids): a seq_cst store alone does not, in the C++ model
      seq.store(s + 1, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_seq_cst);
    }
  }
  ~Region() { seq.store(s + 2, std::memory_order_release); }
};
}  // namespace

struct alignas(128) GroupBatch::Part {  // one pack part's headers and records (page-locked)
  PinnedBuf<jrq_group_state> st;
  PinnedBuf<uint64_t> rec;
  uint32_t ns = 0, nr = 0;
};

// One deliver worker's share of an epoch: the commits it applied (group, index, waiter) and
// the closures it popped, run after every group of the share has moved.
struct alignas(128) GroupBatch::Delivery {  // (one per worker: no false sharing of its vectors)
  struct Commit {
    int64_t c;
    const CommitWaiter* waiter;  // the group's (set once by BallotBox::init, before its first ack)
  };
  std::vector<Commit> commits;
  std::vector<std::function<void(bool)>> done;  // in commit order
  std::vector<uint32_t> ndone;                  // closures per commit
};

struct GroupBatch::Flusher {
  std::thread th;
  std::atomic<bool> stop{false};
};

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

// CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota (a container
// sees every CPU of the host in hardware_concurrency()).
static unsigned usableCpus() {
  unsigned n = std::max(1u, std::thread::hardware_concurrency());
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = std::max(1, CPU_COUNT(&set));
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
      n = std::min<unsigned>(n, std::max<long long>(1, std::atoll(q) / period));
    std::fclose(f);
  }
  return n;
}

void GroupBatch::setFlushThreads(unsigned n) {
  std::lock_guard<std::mutex> fl(flushMu_);
  pool_.reset();
  poolSize_ = std::max(1u, std::min(n, 64u));
}

// f(part, begin, end) over [0, n) on the pool, only when each part gets at least `grain` items.
// How many parts parallelFor(n, grain, f) cuts [0, n) into; part i is [n i / parts, n (i+1) / parts).
size_t GroupBatch::partsFor(size_t n, size_t grain) {
  if (n < 2 * grain) return 1;
  if (!pool_) {  // default: the box's CPU share per GPU, at most 16
    pool_.reset(new Pool(poolSize_ ? poolSize_ : std::min(16u, usableCpus())));
  }
  return std::min<size_t>(pool_->size(), n / grain);
}

template <class F>
void GroupBatch::parallelFor(size_t n, size_t grain, F&& f) {
  const size_t parts = partsFor(n, grain);
  if (parts == 1) {
    f(0u, size_t(0), n);
    return;
  }
  pool_->run([&](unsigned i, unsigned) {
    if (i < parts) f(i, n * i / parts, n * (i + 1) / parts);
  });
}

// Driver-owned page-locked memory (jrq_host_alloc), not heap pages registered with HIP: a
// registered heap range that is later freed and reused by the process for other memory is
// exactly what a device mapping must not outlive ("Staging memory").  Called
// only from the flushing thread, never from pack workers.
template <class T>
void GroupBatch::PinnedBuf<T>::reserve(size_t n) {
  if (n <= cap) return;
  const size_t want = std::max(n, 2 * cap);
  const size_t bytes = ((want * sizeof(T)) + 4095) & ~size_t(4095);
  release();
  void* q = nullptr;
  if (jrq_host_alloc(bytes, &q) != JRQ_OK || !q) throw std::bad_alloc();
  p = static_cast<T*>(q);
  cap = bytes / sizeof(T);
}

template <class T>
void GroupBatch::PinnedBuf<T>::release() {
  if (p) jrq_host_free(p);
  p = nullptr;
  cap = 0;
}

GroupBatch::GroupBatch(Engine* eng, uint32_t groups, uint32_t peers)
    : eng_(eng), G_(groups), P_(peers), serial_(g_batchSerial.fetch_add(1)) {
  if (peers == 0 || peers > JRQ_MAX_PEERS) throw std::invalid_argument("peers must be 1..16");
  if (groups == 0 || groups > JRQ_TABLE_MAX_GROUPS) throw std::invalid_argument("groups must be 1..2^27");
  static_assert(sizeof(Hot) == 56, "group record header");
  stride_ = (sizeof(Hot) + 14 * static_cast<size_t>(P_) + 63) & ~size_t(63);
  // 2 MiB-aligned and advised for transparent huge pages: the calls walk 128 MB of records at
  // C3, 32 records per 4 KiB page
  const size_t kHuge = size_t(2) << 20;
  const size_t bytes = (stride_ * G_ + kHuge - 1) & ~(kHuge - 1);
  rec_ = static_cast<unsigned char*>(std::aligned_alloc(kHuge, bytes));
  if (!rec_) throw std::bad_alloc();
  (void)madvise(rec_, bytes, MADV_HUGEPAGE);
  std::memset(rec_, 0, bytes);
  for (uint32_t g = 0; g < G_; ++g) {
    Hot* h = new (rec_ + static_cast<size_t>(g) * stride_) Hot();
    h->lock.store(0, std::memory_order_relaxed);
    h->gate.store(0, std::memory_order_relaxed);
    h->listed = 0;
    h->nruns = 0;
    h->lastN = 0xFF;
    h->lastO = 0xFF;
    h->dirty = 0;
    h->pi = 0;
    h->lc = 0;
    h->la = -1;
    h->lastConf = 0;
    h->lastSlots = 0;
    uint32_t* sp = slotPeerOf(g);
    for (uint32_t s = 0; s < P_; ++s) sp[s] = kNoPeer;
  }
  runs_.assign(static_cast<size_t>(G_) * JRQ_TABLE_MAX_RUNS, Run{0, 0});
  packedIn_.reset(new uint64_t[G_]());
  rstamp_.reset(new uint64_t[G_]());
  waiter_.resize(G_);
  closures_.resize(G_);
}

GroupBatch::~GroupBatch() {
  try {
    stopFlusher();
  } catch (...) {
  }
  if (table_) jrq_table_destroy(table_);
  std::free(rec_);
}

void GroupBatch::lock(uint32_t g) const { spinLock(hot(g).lock); }

// This thread's dirty list for this batch: a thread-local cache of 4 (batch, list) pairs, and on
// a miss the batch's own per-thread map -- one list per (thread, batch) however many batches a
// thread alternates between (a miss costs a mutex, never a new list).
namespace {
struct ListSlot {
  const void* b;
  uint64_t serial;
  void* l;
};
// initial-exec: one fs-relative load per call (the default model of a shared library calls
// __tls_get_addr, and commitAt's fast path looks its list up on every call)
thread_local ListSlot tl_lists[4] __attribute__((tls_model("initial-exec"))) = {};
thread_local unsigned tl_next __attribute__((tls_model("initial-exec"))) = 0;
}  // namespace

inline GroupBatch::DirtyList* GroupBatch::myDirtyList() {
  for (const ListSlot& s : tl_lists)
    if (s.b == this && s.serial == serial_) return static_cast<DirtyList*>(s.l);
  return myDirtyListSlow();
}

GroupBatch::DirtyList* GroupBatch::myDirtyListSlow() {
  DirtyList* l;
  {
    std::lock_guard<std::mutex> g(listsMu_);
    DirtyList*& mine = byThread_[std::this_thread::get_id()];
    if (!mine) {
      lists_.emplace_back(new DirtyList());
      mine = lists_.back().get();
    }
    l = mine;
  }
  tl_lists[tl_next++ & 3u] = ListSlot{this, serial_, l};
  return l;
}

// Under the group's lock: the bits say what to pack; the group goes on the calling thread's
// list of the current generation unless it is on one already.
void GroupBatch::markDirty(uint32_t g, uint32_t bits) {
  Hot& h = hot(g);
  h.dirty |= bits;
  // on this generation's list already: its pack takes the lock after us and sees the bits
  if (ald(h.listed) == gen_.load(std::memory_order_acquire)) return;
  DirtyList* l = myDirtyList();
  Region rg(l->seq);
  listIn(l, h, g, gen_.load(std::memory_order_acquire));
}

// commitAt's common case without the lock (see the threading note in jraft_host.h): a peer
// with a slot, acks contiguous with its last one.  Everything else -- a peer without a slot, a
// gap to check against the conf runs, an index past lastAppended (the exception), a group
// being quiesced -- goes to the locked path, which decides it as before.
int GroupBatch::ackFast(uint32_t g, int64_t first, int64_t last, uint32_t peer) {
  DirtyList* l = myDirtyList();
  Region rg(l->seq);
  Hot& h = hot(g);
  if (h.gate.load(std::memory_order_acquire)) return -1;
  const int64_t pi = ald(h.pi);
  if (pi == 0) return 0;     // BallotBox.java:101-103
  if (last < pi) return 1;   // :104-106
  if (last > ald(h.la)) return -1;
  const uint32_t* sp = slotPeerOf(g);
  uint32_t s = 0;
  while (s < P_ && __atomic_load_n(&sp[s], __ATOMIC_ACQUIRE) != peer) ++s;
  if (s == P_) return -1;
  int64_t* mp = matchOf(g) + s;
  const int64_t m = ald(*mp);
  if (first > std::max(m + 1, pi)) return -1;
  if (__builtin_expect(testing::fastPathHook != nullptr, 0)) testing::fastPathHook();
  if (last > m) {
    const uint32_t t = gen_.load(std::memory_order_acquire);
    ast(*mp, last);
    // after the match (the pack reads the stamp, then the match)
    ast(slotUseOf(g)[s], stampOf(t, true));
    // the ack itself goes up as an order-free record; the group is listed for the pack only
    // when this thread's record buffer is full
    if (!appendAck(l, t, JRQ_ACK(g, s, last))) listIn(l, h, g, t);
  }
  return 1;
}

bool GroupBatch::appendAck(DirtyList* l, uint32_t t, uint64_t rec) {
  const uint32_t i = t & 1u;
  const uint32_t n = l->nack[i];
  // (acquire: the flushing thread publishes a first buffer of the generation in use, below)
  if (n >= __atomic_load_n(&l->ack[i].cap, __ATOMIC_ACQUIRE)) return false;
  // the counter of resets so far (a reset of this group happened-before this call saw its gate
  // open, so the record is stamped at or after it)
  const uint64_t R = resetSeq_.load(std::memory_order_acquire);
  auto& sg = l->seg[i];
  if (sg.empty() || sg.back().second != R) sg.emplace_back(n, R);
  l->ack[i].p[n] = rec;
  l->nack[i] = n + 1;
  // a full chunk goes up now, on the engine's stream, while the thread goes on writing: the
  // flush then has only the last partial chunk to copy (a failed push leaves it to the flush)
  if (l->dack[i] && n + 1 - l->shipped[i] >= testing::ackChunkRecords.load(std::memory_order_relaxed) &&
      jrq_table_ack_push(table_, l->dack[i] + l->shipped[i], l->ack[i].p + l->shipped[i],
                         n + 1 - l->shipped[i]) == JRQ_OK)
    l->shipped[i] = n + 1;
  return true;
}

// The device region behind a thread's record buffer of parity i, as large as the buffer (on the
// flushing thread, between the buffer's uses).
void GroupBatch::ensureRegion(DirtyList& l, uint32_t i, size_t cap) {
  if (!table_ || cap == 0 || l.dcap[i] >= cap) return;
  if (l.dack[i]) {
    (void)jrq_table_ack_region_free(table_, l.dack[i]);
    l.dack[i] = nullptr;
    l.dcap[i] = 0;
  }
  uint64_t* r = nullptr;
  if (jrq_table_ack_region(table_, cap, &r) == JRQ_OK && r) {  // else the staging copy path
    l.dack[i] = r;
    l.dcap[i] = cap;
  }
}

void GroupBatch::stampReset(uint32_t g) {
  rstamp_[g] = resetSeq_.fetch_add(1, std::memory_order_acq_rel) + 1;
  markDirty(g, kDirtyHeader);
}

// In a call region: g on this thread's list of generation t, unless it is on one already.
void GroupBatch::listIn(DirtyList* l, Hot& h, uint32_t g, uint32_t t) {
  if (ald(h.listed) == t) return;
  std::vector<uint32_t>& v = l->v[t & 1u];
  if (v.empty()) l->firstNs[t & 1u].store(nowNs(), std::memory_order_relaxed);
  v.push_back(g);
  l->n[t & 1u].store(v.size(), std::memory_order_relaxed);
  ast(h.listed, t);
}

void GroupBatch::waitRegions() {
  heavyBarrier();
  std::lock_guard<std::mutex> lg(listsMu_);
  for (auto& l : lists_) {
    const uint32_t s = l->seq.load(std::memory_order_acquire);
    if (!(s & 1u)) continue;
    for (unsigned n = 0; l->seq.load(std::memory_order_acquire) == s; ++n) {
      if (n < 256) __builtin_ia32_pause();
      else std::this_thread::yield();
    }
  }
}

void GroupBatch::quiesce(uint32_t g) {
  Hot& h = hot(g);
  if (h.gate.load(std::memory_order_relaxed)) return;
  h.gate.store(1, std::memory_order_relaxed);
  waitRegions();
}

// Slots named by the masks of the group's live conf runs: their peers vote on pending entries.
uint32_t GroupBatch::liveMask(uint32_t g) const {
  uint32_t m = 0;
  const uint32_t n = hot(g).nruns;
  for (uint32_t r = 0; r < n; ++r) {
    const uint64_t cw = runs_[static_cast<size_t>(g) * JRQ_TABLE_MAX_RUNS + r].conf;
    m |= static_cast<uint32_t>(cw & 0xFFFFu) | static_cast<uint32_t>((cw >> 16) & 0xFFFFu);
  }
  return m;
}

// The slot of `peer` in group g.  create: a free slot, else the least recently acked slot that
// no live conf run names (and that is not in `reserved`), its match reset (its peer's acks no
// longer matter to any pending ballot).  -1 when there is none (every slot is live).
int GroupBatch::slotOf(uint32_t g, uint32_t peer, bool create, uint32_t reserved) {
  uint32_t* sp = slotPeerOf(g);
  int victim = -1;
  for (uint32_t s = 0; s < P_; ++s) {
    if (sp[s] == peer) return static_cast<int>(s);
    if (victim < 0 && sp[s] == kNoPeer) victim = static_cast<int>(s);
  }
  if (!create) return -1;
  uint16_t* su = slotUseOf(g);
  if (victim < 0) {
    const uint32_t busy = liveMask(g) | reserved;
    for (uint32_t s = 0; s < P_; ++s)
      if (!((busy >> s) & 1u) &&  // least recently acked, in the 16-bit stamps' circular order
          (victim < 0 || stampOlder(ald(su[s]), ald(su[victim]))))
        victim = static_cast<int>(s);
    if (victim < 0) return -1;
    quiesce(g);  // the slot's peer may be acking on the fast path
    // its records (and every other record of the group written so far) are dropped by the
    // reset stamp; the live slots' current matches go up again as pack records
    stampReset(g);
    markDirty(g, (1u << P_) - 1u);
  }
  // The slot's stamp and match first, its peer last (a release store the fast path's acquire
  // load of the slot ids pairs with): an ack of `peer` that finds the slot on the fast path --
  // possible for a free slot, which is not quiesced -- then finds it fully set up, and nothing
  // here overwrites what that ack writes (the reverse order could reset its match).
  ast(su[victim], stampOf(gen_.load(std::memory_order_acquire), false));
  int64_t* m = matchOf(g);
  if (ald(m[victim]) != 0) {
    ast(m[victim], int64_t(0));
    markDirty(g, 1u << victim);
  }
  __atomic_store_n(&sp[victim], peer, __ATOMIC_RELEASE);
  if (__builtin_expect(testing::slotAssignHook != nullptr, 0)) testing::slotAssignHook();
  return victim;
}

uint64_t GroupBatch::confWord(uint32_t g, const uint32_t* ids, uint32_t nn, uint32_t no, bool hasOld,
                              uint64_t* slots) {
  // Ballot.init (Ballot.java:63-85): peers only, quorum = size/2+1, oldQuorum 0 if null
  uint32_t nm = 0, om = 0;
  uint64_t sl = 0;
  for (uint32_t i = 0; i < nn + no; ++i) {
    const int s = slotOf(g, ids[i], true, nm | om);
    if (s < 0)
      throw std::length_error("more distinct live peers in group " + std::to_string(g) +
                              " than the " + std::to_string(P_) + " peer slots");
    (i < nn ? nm : om) |= 1u << s;
    if (i < 16) sl |= static_cast<uint64_t>(s) << (4 * i);
  }
  if (slots) *slots = sl;
  return JRQ_CONF(nm, om, nn / 2 + 1, hasOld ? no / 2 + 1 : 0);
}

// Would a gap [lo, hi] in `slot`'s acks skip a pending entry whose ballot counts that slot?
bool GroupBatch::gapCountsPeer(uint32_t g, int slot, int64_t lo, int64_t hi) const {
  const Run* R = &runs_[static_cast<size_t>(g) * JRQ_TABLE_MAX_RUNS];
  const Hot& h = hot(g);
  const uint32_t n = h.nruns;
  for (uint32_t r = 0; r < n; ++r) {
    const int64_t s = r == 0 ? h.pi : R[r].start;
    const int64_t e = r + 1 < n ? R[r + 1].start - 1 : h.la;
    const uint64_t cw = R[r].conf;
    const uint32_t m = static_cast<uint32_t>(cw & 0xFFFFu) | static_cast<uint32_t>((cw >> 16) & 0xFFFFu);
    if (std::max(s, lo) <= std::min(e, hi) && ((m >> slot) & 1u)) return true;
  }
  return false;
}

// Drop runs wholly below pendingIndex (pendingMetaQueue.removeRange, BallotBox.java:130).
void GroupBatch::dropDeadRuns(uint32_t g) {
  Hot& h = hot(g);
  const uint32_t n = h.nruns;
  if (n < 2) return;
  Run* R = &runs_[static_cast<size_t>(g) * JRQ_TABLE_MAX_RUNS];
  uint32_t k = 0;
  while (k + 1 < n && R[k + 1].start <= h.pi) ++k;
  if (k) {
    for (uint32_t r = k; r < n; ++r) R[r - k] = R[r];
    h.nruns = static_cast<uint8_t>(n - k);
  }
}

// Append groups[0..n) to `part` (reserved for them): per group, under its lock, the dirty bits
// are taken and the header or records written from the group's current state.
#ifndef JRAFT_PACK_AHEAD
#define JRAFT_PACK_AHEAD 4
#endif
#ifndef JRAFT_DELIVER_AHEAD
#define JRAFT_DELIVER_AHEAD 8
#endif
#ifndef JRAFT_PREFETCH_LINES
#define JRAFT_PREFETCH_LINES 1
#endif
// Prefetch (for writing) the first `JRAFT_PREFETCH_LINES` 64-B lines of group g's record.
inline void prefetchRecord(const uint8_t* rec, size_t stride, uint32_t g) {
  const uint8_t* r = rec + static_cast<size_t>(g) * stride;
  for (size_t l = 0; l < JRAFT_PREFETCH_LINES && l * 64 < stride; ++l) __builtin_prefetch(r + 64 * l, 1);
}

void GroupBatch::packRange(Part& part, const uint32_t* groups, size_t n) {
  uint32_t si = part.ns, ri = part.nr;
  constexpr size_t kAhead = JRAFT_PACK_AHEAD;
  for (size_t i = 0; i < n; ++i) {
    if (i + kAhead < n) prefetchRecord(rec_, stride_, groups[i + kAhead]);
    const uint32_t g = groups[i];
    Guard lk(*this, g);
    // A group can sit on two threads' lists of one generation (two fast-path acks of different
    // peers listing it at once): pack it once -- a second pass would ship the slots again, and
    // the device applies an upload's records in parallel, so an older value could land last.
    if (packedIn_[g] == packSerial_) continue;
    packedIn_[g] = packSerial_;
    Hot& h = hot(g);
    uint32_t d = h.dirty;
    h.dirty = 0;
    {  // slots the fast path acked in this generation or the next (stamp, then match)
      const uint16_t* su = slotUseOf(g);
      for (uint32_t s = 0; s < P_; ++s) {
        const uint16_t u = ald(su[s]);
        if (stampChangedIn(u, packGen_) || stampChangedIn(u, packGen_ + 1)) d |= 1u << s;
      }
    }
    const int64_t pi = h.pi, base = pi - 1;
    if (d & kDirtyHeader) {
      jrq_group_state& st = part.st.p[si++];
      std::memset(&st, 0, sizeof st);
      st.group = g;
      st.num_runs = h.nruns;
      st.flags = (d & kDirtyReset) ? JRQ_STATE_RESET_MATCH : 0;
      // the table's steady-state encoding of pendingIndex = lastCommittedIndex + 1: the
      // group's next commit then writes lastCommitted only
      st.pending_index = (pi != 0 && pi == h.lc + 1) ? JRQ_PI_FOLLOWS_LC : pi;
      st.last_appended = h.la;
      st.last_committed = h.lc;
      const Run* R = &runs_[static_cast<size_t>(g) * JRQ_TABLE_MAX_RUNS];
      for (uint32_t r = 0; r < h.nruns; ++r) {
        st.run_conf[r] = R[r].conf;
        st.run_start[r] = R[r].start;
      }
      // the group's reset stamp rides in run_start[0] (which a header otherwise ignores):
      // order-free records written before its last reset are dropped
      st.flags |= JRQ_STATE_STAMP;
      st.run_start[0] = static_cast<int64_t>(rstamp_[g]);
    } else if ((d & kDirtyLa) && pi != 0) {
      part.rec.p[ri++] = JRQ_REC(g, JRQ_REC_LAST_APPENDED, h.la - base);
    }
    if (pi == 0) continue;  // not the leader: its acks are refused (commitAt returns false)
    const int64_t* m = matchOf(g);
    for (uint32_t b = d & 0xFFFFu; b; b &= b - 1) {
      const uint32_t s = static_cast<uint32_t>(__builtin_ctz(b));
      const int64_t v = ald(m[s]) - base;
      part.rec.p[ri++] = JRQ_REC(g, s, v > 0 ? v : 0);
    }
  }
  part.ns = si;
  part.nr = ri;
}

// After a failed upload or epoch: every group this flush swapped out goes back on a live list
// with its whole state marked (header, every slot, queue size), so the next flush re-syncs the
// device's copy -- whatever part of this one reached it -- from the host's.  The pack cleared
// the dirty bits of the groups it had packed; without this they were listed nowhere and never
// shipped again.
void GroupBatch::relistAfterFailure() {
  const uint32_t all = kDirtyHeader | kDirtyLa | ((1u << P_) - 1u);
  for (auto& v : work_) {
    for (uint32_t g : v) {
      Guard lk(*this, g);
      Hot& h = hot(g);
      const uint32_t d = h.dirty & kDirtyReset;
      h.dirty = 0;  // not on any list: markDirty lists it again
      markDirty(g, all | d);
    }
    v.clear();
  }
}

uint32_t GroupBatch::flush() {
  if (tl_delivering == this)
    throw std::logic_error("GroupBatch::flush from inside a commit callback of the same batch");
  {
    std::lock_guard<std::mutex> el(errMu_);
    if (!flusherError_.empty()) {
      const std::string err = flusherError_;
      flusherError_.clear();
      throw std::runtime_error("GroupBatch flusher: " + err);
    }
  }
  std::lock_guard<std::mutex> fl(flushMu_);
  return flushLocked();
}

uint32_t GroupBatch::flushLocked() {
  if (!eng_) throw std::logic_error("GroupBatch::flush needs an Engine");
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  FlushStats stats;
  if (!table_) {  // first flush: the device table starts empty, ship every group's state
    int err = 0;
    table_ = jrq_table_create(eng_->raw(), G_, P_, &err);
    if (!table_) throwIfError(err ? err : JRQ_E_NOMEM, eng_->raw(), "jrq_table_create");
    for (uint32_t g = 0; g < G_; ++g) {
      Guard lk(*this, g);
      const Hot& h = hot(g);
      uint32_t bits = 0;
      if (h.pi != 0 || h.lc != 0 || h.nruns != 0) bits |= kDirtyHeader;
      const int64_t* m = matchOf(g);
      for (uint32_t s = 0; s < P_; ++s)
        if (ald(m[s]) != 0) bits |= 1u << s;
      if (bits) markDirty(g, bits);
    }
  }
  // end the generation and take its lists once its call regions have drained: callers go on
  // listing groups (and the fast path stamping acks) in the next one
  const uint32_t t = gen_.load(std::memory_order_acquire);
  ++packSerial_;
  gen_.store(t + 1, std::memory_order_release);  // (orders the last swap of v[t & 1] before
                                                 // its reuse in generation t + 2)
  packGen_ = t;
  waitRegions();
  const auto tw = clk::now();
  size_t nl;
  std::vector<DirtyList*> taken;  // the lists whose generation-t records this flush ships
  {
    std::lock_guard<std::mutex> g(listsMu_);
    nl = lists_.size();
    if (work_.size() < nl) work_.resize(nl);
    for (size_t i = 0; i < nl; ++i) {
      DirtyList& l = *lists_[i];
      work_[i].clear();
      std::swap(l.v[t & 1u], work_[i]);
      l.n[t & 1u].store(0, std::memory_order_relaxed);
      taken.push_back(&l);
    }
  }
  const uint32_t ti = t & 1u;
  size_t nacks = 0, nsegs = 0;
  for (DirtyList* l : taken) {
    nacks += l->nack[ti];
    nsegs += l->seg[ti].size();
  }
  // the record buffers of generation t are consumed once the epoch has synchronised: emptied
  // and sized for their next use (generation t + 2) from what this one held -- on this thread,
  // as every page-locked allocation of the batch is
  auto recycleAcks = [&] {
    for (size_t i = 0; i < taken.size(); ++i) {
      DirtyList* l = taken[i];
      // what the thread wrote this generation: its records, or -- while it had no buffer --
      // the groups it listed, each a queue size and P acks at most
      const size_t used = std::max<size_t>(l->nack[ti], work_[i].size() * (P_ + 1));
      l->nack[ti] = 0;
      l->shipped[ti] = 0;
      l->seg[ti].clear();
      l->ack[ti].reserve(std::max<size_t>(used + used / 2, 1u << 14));
      ensureRegion(*l, ti, l->ack[ti].cap);
      // a thread's first buffer of the generation now in use (t + 1): nothing writes a buffer
      // of capacity 0, so it can be published now -- pointer first, capacity last (release)
      PinnedBuf<uint64_t>& nx = l->ack[ti ^ 1u];
      if (__atomic_load_n(&nx.cap, __ATOMIC_RELAXED) == 0) {
        const size_t want = l->ack[ti].cap;
        void* q = nullptr;
        if (jrq_host_alloc(want * sizeof(uint64_t), &q) == JRQ_OK && q) {
          nx.p = static_cast<uint64_t*>(q);
          ensureRegion(*l, ti ^ 1u, want);  // (before the capacity is published)
          __atomic_store_n(&nx.cap, want, __ATOMIC_RELEASE);
        }
      }
    }
  };
  std::vector<size_t> pre(nl + 1, 0);
  for (size_t i = 0; i < nl; ++i) pre[i + 1] = pre[i] + work_[i].size();
  const size_t nd = pre[nl];
  uint32_t n = 0;
  auto t1 = t0;
  try {
    // pack: the dirty groups cut into K contiguous ranges ("parts") of the concatenated
    // lists, claimed in order by the pool's workers, each packed under the groups' locks into
    // its own page-locked buffers; the flushing thread stages a part's upload (an asynchronous
    // DMA, jrq_table_stage) as soon as it is packed, so the DMA of the early parts overlaps the
    // packing of the later ones -- the update's H2D (36 MB at C3) is the PCIe-bound part of a
    // flush.  All HIP calls stay on the flushing thread.  A group's header and records sit in
    // one part.
    const size_t kGrain = 1u << 12;
    const size_t workers = partsFor(nd, kGrain);  // (1 below 2 * kGrain groups)
    const size_t K = workers <= 1 ? 1 : std::min<size_t>(4 * workers, nd / kGrain);
    if (parts_.size() < K) parts_.resize(K);
    changed_.reserve(G_);
    // staging grows here, on this thread: allocation and release of page-locked memory stay
    // out of the pack workers
    for (size_t k = 0; k < K; ++k) {
      const size_t len = nd * (k + 1) / K - nd * k / K;
      Part& P = parts_[k];
      P.ns = P.nr = 0;
      P.st.reserve(len + 1);
      P.rec.reserve(len * (P_ + 1) + 1);
    }
    throwIfError(jrq_table_stage_reserve(table_, static_cast<uint32_t>(nd + 1),
                                         static_cast<uint32_t>(nd * (P_ + 1) + 1)),
                 eng_->raw(), "jrq_table_stage_reserve");
    // the order-free records first: the threads streamed their full chunks to their device
    // regions while writing them (on the engine's stream, ahead of everything below); the rest
    // goes up now, and every segment is registered where it lies.  A thread without a region
    // (its first generation) has its records copied through the staging buffer.
    size_t ncopy = 0;
    for (DirtyList* l : taken)
      if (!l->dack[ti]) ncopy += l->nack[ti];
    throwIfError(jrq_table_stage_reserve_acks(table_, static_cast<uint32_t>(ncopy), static_cast<uint32_t>(nsegs + 1)),
                 eng_->raw(), "jrq_table_stage_reserve_acks");
    for (DirtyList* l : taken) {
      const uint32_t na = l->nack[ti];
      uint64_t* const dr = l->dack[ti];
      stats.acks_streamed += dr ? l->shipped[ti] : 0u;
      if (dr && na > l->shipped[ti]) {
        throwIfError(jrq_table_ack_push(table_, dr + l->shipped[ti], l->ack[ti].p + l->shipped[ti], na - l->shipped[ti]),
                     eng_->raw(), "jrq_table_ack_push");
        l->shipped[ti] = na;
      }
      const auto& sg = l->seg[ti];
      for (size_t k = 0; k < sg.size(); ++k) {
        const uint32_t b = sg[k].first, e = k + 1 < sg.size() ? sg[k + 1].first : na;
        if (dr)
          throwIfError(jrq_table_stage_acks_dev(table_, sg[k].second, dr + b, e - b), eng_->raw(),
                       "jrq_table_stage_acks_dev");
        else
          throwIfError(jrq_table_stage_acks(table_, sg[k].second, l->ack[ti].p + b, e - b), eng_->raw(),
                       "jrq_table_stage_acks");
      }
    }
    stats.acks = static_cast<uint32_t>(nacks);
    auto packPart = [&](size_t k) {
      Part& P = parts_[k];
      const size_t b0 = nd * k / K, e0 = nd * (k + 1) / K;
      size_t li = static_cast<size_t>(std::upper_bound(pre.begin(), pre.end(), b0) - pre.begin()) - 1;
      for (size_t pos = b0; pos < e0; ++li) {  // the pieces of the lists inside [b0, e0)
        const size_t l0 = pos - pre[li], hi = std::min(e0, pre[li + 1]) - pre[li];
        if (hi <= l0) continue;
        packRange(P, work_[li].data() + l0, hi - l0);
        pos = pre[li] + hi;
      }
    };
    auto stagePart = [&](size_t k) {
      const Part& P = parts_[k];
      stats.states += P.ns;
      stats.records += P.nr;
      throwIfError(jrq_table_stage(table_, P.st.p, P.ns, P.rec.p, P.nr), eng_->raw(), "jrq_table_stage");
    };
    if (K == 1) {
      packPart(0);
      stagePart(0);
    } else {
      std::unique_ptr<std::atomic<uint8_t>[]> done(new std::atomic<uint8_t>[K]);
      for (size_t k = 0; k < K; ++k) done[k].store(0, std::memory_order_relaxed);
      std::atomic<size_t> next{0};
      std::atomic<bool> abort{false};
      pool_->run([&](unsigned i, unsigned) {
        if (i == 0) {  // the flushing thread: stage the parts in order as they complete
          try {
            for (size_t k = 0; k < K; ++k) {
              uint8_t st;
              for (unsigned spin = 0; (st = done[k].load(std::memory_order_acquire)) == 0; ++spin) {
                if (spin < 256) __builtin_ia32_pause();
                else std::this_thread::yield();
              }
              if (st == 2) return;  // the worker's exception comes back from run()
              stagePart(k);
            }
          } catch (...) {
            abort.store(true, std::memory_order_relaxed);
            throw;
          }
          return;
        }
        for (;;) {
          const size_t k = next.fetch_add(1, std::memory_order_relaxed);
          if (k >= K) return;
          if (abort.load(std::memory_order_relaxed)) {
            done[k].store(2, std::memory_order_release);
            continue;
          }
          try {
            packPart(k);
          } catch (...) {
            done[k].store(2, std::memory_order_release);
            abort.store(true, std::memory_order_relaxed);
            throw;
          }
          done[k].store(1, std::memory_order_release);
        }
      });
    }
    const auto ta0 = clk::now();
    throwIfError(jrq_table_stage_apply(table_), eng_->raw(), "jrq_table_stage_apply");
    stats.pack_wait_ms = std::chrono::duration<double, std::milli>(tw - t0).count();
    stats.pack_apply_ms = std::chrono::duration<double, std::milli>(clk::now() - ta0).count();
    t1 = clk::now();
    throwIfError(jrq_table_epoch(table_, changed_.p, &n, nullptr), eng_->raw(), "jrq_table_epoch");
    recycleAcks();
  } catch (...) {
    // the groups of the generation's records go back on a list in full, like the listed ones
    // (whatever part of this update reached the device, the next one re-syncs them)
    (void)jrq_synchronize(eng_->raw());  // (no DMA may still read the buffers)
    const uint32_t all = kDirtyHeader | kDirtyLa | ((1u << P_) - 1u);
    for (DirtyList* l : taken)
      for (uint32_t k = 0; k < l->nack[ti]; ++k) {
        const uint32_t g = static_cast<uint32_t>(l->ack[ti].p[k] >> 5) & ((1u << 27) - 1u);
        Guard lk(*this, g);
        markDirty(g, all);
      }
    recycleAcks();
    relistAfterFailure();
    throw;
  }
  const auto t2 = clk::now();
  // deliver: per changed group, under its lock, the commit BallotBox.commitAt makes
  // (:130-134: drop ballots up to c, pendingIndex = c + 1, lastCommittedIndex = c) -- for
  // every group of a worker's share first -- then, without the locks, its closures
  // (ClosureQueue.popClosureUntil -> done.run(OK)) and waiter.onCommitted(c) (:137), group by
  // group in order.  A callback that throws cannot leave a group half-applied: the host state
  // then stays what the device table already holds (its pendingIndex follows lastCommitted),
  // and the first exception is rethrown after every callback ran.  A commit touches one group
  // record at a random place: prefetch a few groups ahead.  The workers claim the list in
  // kDeliverChunks chunks each, in order, rather than one fixed range each: a worker the OS
  // deschedules then holds up one chunk, not a sixteenth of the flush (r06 A/B, one process
  // per run: deliver 1.93 -> 1.58 ms median at 16 API threads).  A worker's
  // groups still come in list order, so its callbacks run group by group in order.
  const size_t dparts = partsFor(n, 1u << 12);
  if (deliveries_.size() < dparts) deliveries_.resize(dparts);
  std::vector<std::exception_ptr> errs(dparts);
  std::vector<double> apply_ms(dparts, 0.0), cb_ms(dparts, 0.0);
  constexpr size_t kDeliverChunks = 4;
  const size_t chunk = (n + dparts * kDeliverChunks - 1) / (dparts * kDeliverChunks);
  std::atomic<size_t> nextChunk{0};
  auto deliverPart = [&](unsigned part) {
    const auto d0 = clk::now();
    Delivery& D = deliveries_[part];
    D.commits.clear();
    D.done.clear();
    D.ndone.clear();
    constexpr size_t kAhead = JRAFT_DELIVER_AHEAD;
    for (;;) {
    const size_t i0 = nextChunk.fetch_add(1, std::memory_order_relaxed) * chunk;
    if (i0 >= n) break;
    const size_t i1 = std::min<size_t>(n, i0 + chunk);
    for (size_t i = i0; i < i1; ++i) {
      if (i + kAhead < i1) {
        const uint32_t a = static_cast<uint32_t>(changed_.p[i + kAhead]);
        prefetchRecord(rec_, stride_, a);
        __builtin_prefetch(&closures_[a], 0);
        __builtin_prefetch(&waiter_[a], 0);
      }
      const uint64_t w = changed_.p[i];
      const uint32_t g = static_cast<uint32_t>(w);
      Guard lk(*this, g);
      Hot& h = hot(g);
      const int64_t c = h.pi - 1 + static_cast<int64_t>(w >> 32);
      uint32_t nd0 = 0;
      if (auto& q = closures_[g]) {
        while (!q->empty() && q->front().first <= c) {
          D.done.push_back(std::move(q->front().second));
          q->pop_front();
          ++nd0;
        }
      }
      ast(h.pi, c + 1);
      h.lc = c;
      dropDeadRuns(g);
      D.commits.push_back(Delivery::Commit{c, &waiter_[g]});
      D.ndone.push_back(nd0);
    }
    }
    const auto d1 = clk::now();
    struct Scope {
      const GroupBatch* prev;
      explicit Scope(const GroupBatch* b) : prev(tl_delivering) { tl_delivering = b; }
      ~Scope() { tl_delivering = prev; }
    } scope(this);
    size_t k = 0;
    for (size_t j = 0; j < D.commits.size(); ++j) {
      for (uint32_t u = 0; u < D.ndone[j]; ++u, ++k) {
        try {
          D.done[k](true);
        } catch (...) {
          if (!errs[part]) errs[part] = std::current_exception();
        }
      }
      try {
        if (*D.commits[j].waiter) (*D.commits[j].waiter)(D.commits[j].c);
      } catch (...) {
        if (!errs[part]) errs[part] = std::current_exception();
      }
    }
    D.commits.clear();
    D.done.clear();
    apply_ms[part] = std::chrono::duration<double, std::milli>(d1 - d0).count();
    cb_ms[part] = std::chrono::duration<double, std::milli>(clk::now() - d1).count();
  };
  if (dparts == 1) {
    deliverPart(0u);
  } else {
    pool_->run([&](unsigned i, unsigned) {
      if (i < dparts) deliverPart(i);
    });
  }
  flushes_.fetch_add(1, std::memory_order_relaxed);
  const auto t3 = clk::now();
  auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
  stats.changed = n;
  stats.h2d_bytes = static_cast<uint64_t>(stats.states) * sizeof(jrq_group_state) +
                    static_cast<uint64_t>(stats.records) * 8 + static_cast<uint64_t>(stats.acks) * 8;
  stats.d2h_bytes = 4 + static_cast<uint64_t>(n) * 8;
  stats.pack_ms = ms(t1 - t0);
  stats.device_ms = ms(t2 - t1);
  stats.deliver_ms = ms(t3 - t2);
  for (size_t i = 0; i < dparts; ++i) {
    stats.deliver_apply_ms = std::max(stats.deliver_apply_ms, apply_ms[i]);
    stats.deliver_callbacks_ms = std::max(stats.deliver_callbacks_ms, cb_ms[i]);
  }
  stats_ = stats;
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
  return n;
}

void GroupBatch::startFlusher(const FlushPolicy& policy) {
  stopFlusher();
  flusher_.reset(new Flusher());
  Flusher* f = flusher_.get();
  f->th = std::thread([this, f, policy] {
    const int64_t delayNs = static_cast<int64_t>(policy.maxDelayUs) * 1000;
    const auto nap = std::chrono::microseconds(std::max<uint32_t>(10, std::min<uint32_t>(100, policy.maxDelayUs / 8)));
    try {
      while (!f->stop.load(std::memory_order_acquire)) {
        size_t pending = 0;
        int64_t oldest = INT64_MAX;
        {
          std::lock_guard<std::mutex> g(listsMu_);
          const uint32_t t = gen_.load(std::memory_order_acquire) & 1u;
          for (auto& l : lists_) {
            const size_t k = l->n[t].load(std::memory_order_relaxed);
            if (k) {
              pending += k;
              oldest = std::min(oldest, l->firstNs[t].load(std::memory_order_relaxed));
            }
          }
        }
        if (pending && (pending >= policy.maxDirtyGroups || nowNs() - oldest >= delayNs)) {
          std::lock_guard<std::mutex> fl(flushMu_);
          flushLocked();
        } else {
          std::this_thread::sleep_for(nap);
        }
      }
    } catch (const std::exception& ex) {
      // the flusher stops; the error is rethrown by the next flush() or stopFlusher()
      std::lock_guard<std::mutex> el(errMu_);
      if (flusherError_.empty()) flusherError_ = ex.what();
    }
  });
}

void GroupBatch::stopFlusher() {
  if (flusher_) {
    flusher_->stop.store(true, std::memory_order_release);
    if (flusher_->th.joinable()) flusher_->th.join();
    flusher_.reset();
  }
  std::string err;
  {
    std::lock_guard<std::mutex> el(errMu_);
    std::swap(err, flusherError_);
  }
  if (!err.empty()) throw std::runtime_error("GroupBatch flusher: " + err);
}

BallotBox::BallotBox(std::shared_ptr<GroupBatch> batch, uint32_t group) : batch_(std::move(batch)), g_(group) {
  if (g_ >= batch_->groups()) throw std::out_of_range("group id");
}

bool BallotBox::init(const BallotBoxOptions& opts) {
  if (!opts.waiter || !opts.closureQueue) return false;  // "waiter or closure queue is null."
  GroupBatch& b = *batch_;
  GroupBatch::Guard lk(b, g_);
  b.waiter_[g_] = opts.waiter;
  return true;
}

bool BallotBox::commitAt(int64_t first, int64_t last, const PeerId& peer) {
  GroupBatch& b = *batch_;
  const uint32_t id = peerId(peer);
  const int r = b.ackFast(g_, first, last, id);
  if (r >= 0) return r != 0;
  GroupBatch::Guard lk(b, g_);
  GroupBatch::Hot& h = b.hot(g_);
  const int64_t pi = h.pi;
  if (pi == 0) return false;                                     // :101-103
  if (last < pi) return true;                                    // :104-106
  if (last > h.la) throw std::out_of_range("ArrayIndexOutOfBoundsException");  // :107-109
  const int s = b.slotOf(g_, id, true);
  // every slot is named by a live conf run and this peer by none: no pending ballot counts
  // it, so Ballot.grant finds nothing (Ballot.java:100-127) and commitAt returns true
  if (s < 0) return true;
  int64_t& m = b.matchOf(g_)[s];
  const int64_t mv = ald(m);
  const int64_t lo = std::max(mv + 1, pi);
  if (first > lo && b.gapCountsPeer(g_, s, lo, first - 1))
    throw std::logic_error("non-contiguous ack: the Replicator never skips entries");
  if (last > mv) {
    ast(m, last);
    b.markDirty(g_, 1u << s);
    ast(b.slotUseOf(g_)[s], stampOf(b.gen_.load(std::memory_order_acquire), false));
  }
  return true;
}

void BallotBox::clearPendingTasks() {
  GroupBatch& b = *batch_;
  if (tl_delivering == batch_.get())
    throw std::logic_error("BallotBox.clearPendingTasks from inside a commit callback of its batch");
  // waits for a flush in progress (it may hold this group's acks)
  std::lock_guard<std::mutex> fl(b.flushMu_);
  // Acks recorded since the last epoch would have committed at once in the reference
  // (BallotBox.commitAt decides synchronously): decide them before the queue is dropped.
  bool decide;
  {
    GroupBatch::Guard lk(b, g_);
    const GroupBatch::Hot& h = b.hot(g_);
    // acks of the current generation (the locked path's dirty bits, the fast path's stamps)
    bool acks = (h.dirty & 0xFFFFu) != 0;
    const uint32_t t = b.gen_.load(std::memory_order_acquire);
    for (uint32_t s = 0; s < b.P_; ++s) acks = acks || stampChangedIn(ald(b.slotUseOf(g_)[s]), t);
    decide = acks && h.pi != 0 && b.eng_;
  }
  if (decide) b.flushLocked();
  std::unique_ptr<std::deque<std::pair<int64_t, std::function<void(bool)>>>> q;
  {
    GroupBatch::Guard lk(b, g_);
    GroupBatch::Hot& h = b.hot(g_);
    // an ack of this leadership may still be on the fast path: it completes before pendingIndex
    // drops to 0, and none starts after (resetPendingIndex relies on it)
    if (h.pi != 0) {
      b.quiesce(g_);
      b.stampReset(g_);  // this leadership's records not yet applied are dropped
    }
    q = std::move(b.closures_[g_]);
    h.nruns = 0;
    h.lastConf = 0;
    ast(h.pi, int64_t(0));
    ast(h.la, int64_t(-1));
    b.markDirty(g_, GroupBatch::kDirtyHeader);
  }
  if (q)
    for (auto& c : *q) c.second(false);  // ClosureQueue.clear runs closures with EPERM
}

bool BallotBox::resetPendingIndex(int64_t n) {
  GroupBatch& b = *batch_;
  GroupBatch::Guard lk(b, g_);
  GroupBatch::Hot& h = b.hot(g_);
  if (!(h.pi == 0 && h.la < h.pi)) return false;
  if (n <= h.lc) return false;
  // (no fast-path ack can be in flight: pendingIndex is 0 -- never a leader, or stepped down
  // through clearPendingTasks, which quiesced the group -- and the fast path writes nothing then)
  ast(h.pi, n);
  ast(h.la, n - 1);
  h.nruns = 0;
  h.lastConf = 0;
  // a new leader's replicators start over
  for (uint32_t s = 0; s < b.P_; ++s) ast(b.matchOf(g_)[s], int64_t(0));
  b.markDirty(g_, GroupBatch::kDirtyHeader | GroupBatch::kDirtyReset);
  return true;
}

bool BallotBox::appendPendingTasks(const Configuration& conf, const Configuration* oldConf,
                                   int64_t count) {
  return append(conf, oldConf, count, nullptr);
}

bool BallotBox::appendPendingTask(const Configuration& conf, const Configuration* oldConf,
                                  std::function<void(bool)> done) {
  return append(conf, oldConf, 1, done ? &done : nullptr);
}

// The ballots and (for one entry) the closure under one hold of the group's lock, as the
// reference appends both under its write lock (BallotBox.java:203-214).
bool BallotBox::append(const Configuration& conf, const Configuration* oldConf, int64_t count,
                       std::function<void(bool)>* done) {
  GroupBatch& b = *batch_;
  // the peers' ids, interned outside the group's lock
  const size_t nn = conf.peers.size(), no = oldConf ? oldConf->peers.size() : 0;
  uint32_t small[32];
  std::vector<uint32_t> big;
  uint32_t* ids = small;
  if (nn + no > 32) {
    big.resize(nn + no);
    ids = big.data();
  }
  for (size_t i = 0; i < nn; ++i) ids[i] = peerId(conf.peers[i]);
  for (size_t i = 0; i < no; ++i) ids[nn + i] = peerId(oldConf->peers[i]);
  GroupBatch::Guard lk(b, g_);
  GroupBatch::Hot& h = b.hot(g_);
  if (h.pi <= 0) return false;  // :204-207
  if (count <= 0) return true;
  if (h.la + count - h.pi + 1 > INT32_MAX)  // pendingMetaQueue is a Java ArrayList
    throw std::length_error("pending queue larger than an ArrayList");
  // the conf word: the group's last conf again (the common case: NodeImpl passes its current
  // conf with every task) when the same ids sit in the cached slots, else Ballot.init's walk
  const uint32_t tot = static_cast<uint32_t>(nn + no);
  const uint8_t oTag = oldConf ? static_cast<uint8_t>(no) : 0xFF;
  uint64_t cw;
  if (h.nruns != 0 && h.lastN == nn && h.lastO == oTag && tot <= 16 && no < 0xFF &&
      b.sameSlots(g_, ids, tot, h.lastSlots)) {
    cw = h.lastConf;
  } else {
    uint64_t sl = 0;
    cw = b.confWord(g_, ids, static_cast<uint32_t>(nn), static_cast<uint32_t>(no), oldConf != nullptr, &sl);
    const bool cache = tot <= 16 && nn < 0xFF && no < 0xFF;
    h.lastN = cache ? static_cast<uint8_t>(nn) : 0xFF;
    h.lastO = oTag;
    h.lastSlots = sl;
  }
  const int64_t idx = h.la + 1;
  if (h.nruns == 0 || h.lastConf != cw) {  // Ballot.init with a new conf: a new conf run
    GroupBatch::Run* R = &b.runs_[static_cast<size_t>(g_) * JRQ_TABLE_MAX_RUNS];
    uint8_t& n = h.nruns;
    if (n == JRQ_TABLE_MAX_RUNS) {
      if (idx > h.pi)  // NodeImpl never has more than 2 (joint, then stable) pending
        throw std::length_error("more conf runs pending than JRQ_TABLE_MAX_RUNS");
      n = 0;  // the queue is empty: every earlier run is dead
    }
    R[n++] = GroupBatch::Run{idx, cw};
    h.lastConf = cw;
    b.dropDeadRuns(g_);
    b.markDirty(g_, GroupBatch::kDirtyHeader);
  }
  ast(h.la, idx + count - 1);
  {  // the new queue end as an order-free record (else the pack ships it)
    GroupBatch::DirtyList* l = b.myDirtyList();
    Region rg(l->seq);
    const uint32_t t = b.gen_.load(std::memory_order_acquire);
    if (!b.appendAck(l, t, JRQ_ACK(g_, JRQ_REC_LAST_APPENDED, h.la))) {
      h.dirty |= GroupBatch::kDirtyLa;
      b.listIn(l, h, g_, t);
    }
  }
  if (done) {  // ClosureQueue.appendPendingClosure (ClosureQueueImpl.java:98-105)
    auto& q = b.closures_[g_];
    if (!q) q.reset(new std::deque<std::pair<int64_t, std::function<void(bool)>>>());
    q->emplace_back(h.la, std::move(*done));
  }
  return true;
}

bool BallotBox::setLastCommittedIndex(int64_t c) {
  GroupBatch& b = *batch_;
  CommitWaiter w;
  {
    GroupBatch::Guard lk(b, g_);
    GroupBatch::Hot& h = b.hot(g_);
    if (h.pi != 0 || h.la >= h.pi) {
      if (!(c < h.pi))  // Requires.requireTrue (:229-231)
        throw std::invalid_argument("Node changes to leader, pendingIndex=" +
                                    std::to_string(h.pi) +
                                    ", param lastCommittedIndex=" + std::to_string(c));
      return false;
    }
    if (c < h.lc) return false;
    if (c == h.lc) return true;
    h.lc = c;
    b.markDirty(g_, GroupBatch::kDirtyHeader);
    w = b.waiter_[g_];
  }
  if (w) w(c);  // onCommitted after unlocking (:244-246)
  return true;
}

int64_t BallotBox::getLastCommittedIndex() const {
  GroupBatch::Guard lk(*batch_, g_);
  return batch_->hot(g_).lc;
}
int64_t BallotBox::getPendingIndex() const {
  GroupBatch::Guard lk(*batch_, g_);
  return batch_->hot(g_).pi;
}
int64_t BallotBox::getPendingMetaQueueSize() const {
  const GroupBatch& b = *batch_;
  GroupBatch::Guard lk(b, g_);
  const GroupBatch::Hot& h = b.hot(g_);
  return h.pi == 0 ? 0 : h.la - h.pi + 1;
}

std::string BallotBox::describe() const {
  int64_t lc, pi, q;
  {
    const GroupBatch& b = *batch_;
    GroupBatch::Guard lk(b, g_);
    const GroupBatch::Hot& h = b.hot(g_);
    lc = h.lc;
    pi = h.pi;
    q = pi == 0 ? 0 : h.la - pi + 1;
  }
  std::ostringstream o;
  o << "  lastCommittedIndex: " << lc << "\n"
    << "  pendingIndex: " << pi << "\n"
    << "  pendingMetaQueueSize: " << q << "\n";
  return o.str();
}

// -------------------------------------------------------- follower / reader

std::vector<int32_t> FollowerVerifier::verify(const std::vector<const AppendEntriesRequest*>& reqs,
                                              std::vector<uint64_t>* checksums) {
  const uint32_t R = static_cast<uint32_t>(reqs.size());
  std::vector<uint32_t> reqOff(R + 1, 0);
  std::vector<int64_t> prev(R);
  std::vector<const LogEntry*> metas;
  for (uint32_t r = 0; r < R; ++r) {
    const AppendEntriesRequest& q = *reqs[r];
    if (q.dataLen.size() != q.entries.size()) throw std::invalid_argument("dataLen per entry");
    prev[r] = q.prevLogIndex;
    reqOff[r + 1] = reqOff[r] + static_cast<uint32_t>(q.entries.size());
    for (auto& e : q.entries) metas.push_back(&e);
  }
  const uint32_t N = reqOff[R];
  std::vector<int32_t> first(R, -1);
  if (R == 0) return first;
  // the PeerId checksums of configuration entries (one GPU CRC batch), then every request's
  // entries in one launch sequence (scan -> CRC -> first corrupt)
  const std::vector<uint64_t> px = eng_->peerChecksums(metas);
  std::vector<int64_t> term(N), dlen(N);
  std::vector<uint8_t> type(N), has(N);
  std::vector<uint64_t> stored(N), out(N);
  std::vector<uint8_t> corrupt(N);
  std::vector<uint8_t> data;
  uint32_t i = 0;
  for (uint32_t r = 0; r < R; ++r) {
    const AppendEntriesRequest& q = *reqs[r];
    for (size_t k = 0; k < q.entries.size(); ++k, ++i) {
      const LogEntry& e = q.entries[k];
      term[i] = e.id.term;
      type[i] = static_cast<uint8_t>(e.type);
      dlen[i] = q.dataLen[k];
      has[i] = e.hasChecksum();
      stored[i] = e.getChecksum();
    }
    data.insert(data.end(), q.data.begin(), q.data.end());
  }
  if (data.empty()) data.push_back(0);
  throwIfError(jrq_append_entries_verify(eng_->raw(), R, reqOff.data(), prev.data(), N, term.data(),
                                         type.data(), dlen.data(), px.data(), stored.data(),
                                         has.data(), data.data(), out.data(), corrupt.data(),
                                         first.data()),
               eng_->raw(), "jrq_append_entries_verify");
  if (checksums) *checksums = std::move(out);
  return first;
}

std::vector<DecodedEntry> LogReader::decode(const std::vector<std::vector<uint8_t>>& records) {
  const uint32_t N = static_cast<uint32_t>(records.size());
  std::vector<DecodedEntry> outv(N);
  if (N == 0) return outv;
  std::vector<uint64_t> off(N + 1, 0);
  for (uint32_t i = 0; i < N; ++i) off[i + 1] = off[i] + records[i].size();
  std::vector<uint8_t> buf(std::max<uint64_t>(off[N], 1));
  for (uint32_t i = 0; i < N; ++i)
    if (!records[i].empty()) std::memcpy(buf.data() + off[i], records[i].data(), records[i].size());
  std::vector<uint8_t> status(N), type(N), has(N), corrupt(N);
  std::vector<int64_t> index(N), term(N);
  std::vector<uint64_t> stored(N), doff(N), dlen(N), sum(N);
  std::vector<uint32_t> pc(N);
  throwIfError(jrq_v2_decode_verify(eng_->raw(), buf.data(), off.data(), N, status.data(), type.data(),
                                    index.data(), term.data(), stored.data(), has.data(), doff.data(),
                                    dlen.data(), pc.data(), sum.data(), corrupt.data()),
               eng_->raw(), "jrq_v2_decode_verify");
  for (uint32_t i = 0; i < N; ++i) {
    DecodedEntry& d = outv[i];
    d.status = status[i];
    if (d.status != JRQ_V2_OK) continue;
    d.entry.type = static_cast<EntryType>(type[i]);
    d.entry.id = LogId{index[i], term[i]};
    if (has[i]) d.entry.setChecksum(stored[i]);
    d.entry.data.assign(buf.begin() + static_cast<std::ptrdiff_t>(doff[i]),
                        buf.begin() + static_cast<std::ptrdiff_t>(doff[i] + dlen[i]));
    d.peerCount = pc[i];
    d.corrupt = corrupt[i] != 0;
  }
  return outv;
}

// --------------------------------------------------------------- FSM caller

FSMCallerBatch::FSMCallerBatch(Engine& eng, uint32_t groups) : eng_(&eng), G_(groups) {
  prev_.assign(G_, 0);
  committed_.assign(G_, 0);
  lastApplied_.assign(G_, 0);
  cqFirst_.assign(G_, 0);
  cqSize_.assign(G_, 0);
  closures_.resize(G_);
}

void FSMCallerBatch::resetFirstIndex(uint32_t g, int64_t firstIndex) {
  std::lock_guard<std::mutex> l(mu_);
  if (!closures_[g].empty()) throw std::logic_error("resetFirstIndex on a non-empty ClosureQueue");  // :85-87
  cqFirst_[g] = firstIndex;
  cqSize_[g] = 0;
}

void FSMCallerBatch::appendPendingClosure(uint32_t g, std::function<void(bool)> done) {
  std::lock_guard<std::mutex> l(mu_);
  closures_[g].push_back(std::move(done));
  cqSize_[g] = static_cast<int64_t>(closures_[g].size());
}

void FSMCallerBatch::setLastApplied(uint32_t g, int64_t lastApplied) {
  std::lock_guard<std::mutex> l(mu_);
  lastApplied_[g] = lastApplied;
  prev_[g] = committed_[g] = std::max(committed_[g], lastApplied);
}

void FSMCallerBatch::onCommitted(uint32_t g, int64_t committedIndex) {
  std::lock_guard<std::mutex> l(mu_);
  if (committedIndex > committed_[g]) committed_[g] = committedIndex;
}

uint32_t FSMCallerBatch::doCommitted(const Apply& onApply, const std::function<void(uint32_t)>& onInvalid) {
  struct Job {
    uint32_t g;
    int64_t first, last;
    std::vector<std::function<void(bool)>> done;
  };
  std::vector<Job> jobs;
  std::vector<uint32_t> invalid;
  {
    std::lock_guard<std::mutex> l(mu_);
    std::vector<int64_t> first(G_), oldSize = cqSize_;
    std::vector<uint8_t> status(G_);
    std::vector<uint64_t> listed((G_ + 63) / 64);
    uint32_t n = 0;
    throwIfError(jrq_commit_fanout(eng_->raw(), G_, prev_.data(), committed_.data(), lastApplied_.data(),
                                   cqFirst_.data(), cqSize_.data(), first.data(), status.data(),
                                   listed.data(), &n),
                 eng_->raw(), "jrq_commit_fanout");
    for (size_t w = 0; w < listed.size(); ++w)
      for (uint64_t b = listed[w]; b; b &= b - 1) {
        const uint32_t g = static_cast<uint32_t>(w * 64 + static_cast<uint64_t>(__builtin_ctzll(b)));
        if (status[g] == JRQ_FAN_INVALID) {
          invalid.push_back(g);
          continue;
        }
        Job j{g, lastApplied_[g] + 1, committed_[g], {}};
        const int64_t popped = oldSize[g] - cqSize_[g];  // the kernel's pop, from the queue's front
        for (int64_t k = 0; k < popped; ++k) {
          j.done.push_back(std::move(closures_[g].front()));
          closures_[g].pop_front();
        }
        lastApplied_[g] = committed_[g];
        jobs.push_back(std::move(j));
      }
    prev_ = committed_;
  }
  for (auto& j : jobs) onApply(j.g, j.first, j.last, j.done);
  if (onInvalid)
    for (uint32_t g : invalid) onInvalid(g);
  return static_cast<uint32_t>(jobs.size());
}

// ---------------------------------------------------------- sharded batch

ShardedGroupBatch::ShardedGroupBatch(const std::vector<Engine*>& engines, uint32_t groups, uint32_t peers)
    : eng_(engines), G_(groups) {
  if (engines.empty()) throw std::invalid_argument("ShardedGroupBatch needs at least one engine");
  for (Engine* e : engines)
    if (!e) throw std::invalid_argument("ShardedGroupBatch: null engine");
  const uint32_t n = static_cast<uint32_t>(engines.size());
  if (groups < n) throw std::invalid_argument("ShardedGroupBatch: fewer groups than engines");
  k_ = static_cast<uint32_t>((static_cast<uint64_t>(groups) + n - 1) / n);
  if (static_cast<uint64_t>(k_) * (n - 1) >= groups)
    throw std::invalid_argument("ShardedGroupBatch: the last engine would hold no group");
  const unsigned per = std::max(1u, std::min(16u, usableCpus()) / n);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t lo = i * k_, hi = std::min(groups, lo + k_);
    shard_.push_back(std::make_shared<GroupBatch>(engines[i], hi - lo, peers));
    shard_.back()->setFlushThreads(per);
  }
}

ShardedGroupBatch::~ShardedGroupBatch() {
  if (snap_) jrq_snapshot_destroy(snap_);
}

const std::shared_ptr<GroupBatch>& ShardedGroupBatch::shardOf(uint32_t g, uint32_t* local) const {
  if (g >= G_) throw std::out_of_range("group id");
  const uint32_t s = g / k_;
  if (local) *local = g - s * k_;
  return shard_[s];
}

BallotBox ShardedGroupBatch::box(uint32_t g) const {
  uint32_t l = 0;
  const auto& b = shardOf(g, &l);
  return BallotBox(b, l);
}

void ShardedGroupBatch::setFlushThreads(unsigned n) {
  for (auto& b : shard_) b->setFlushThreads(n);
}

uint32_t ShardedGroupBatch::flush() {
  const size_t n = shard_.size();
  std::vector<uint32_t> changed(n, 0);
  std::vector<std::exception_ptr> err(n);
  auto one = [&](size_t i) {
    try {
      changed[i] = shard_[i]->flush();
    } catch (...) {
      err[i] = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  for (size_t i = 1; i < n; ++i) th.emplace_back(one, i);
  one(0);
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
  uint32_t total = 0;
  for (uint32_t c : changed) total += c;
  return total;
}

bool ShardedGroupBatch::rcclInitAll() {
  std::vector<jrq_engine*> raw;
  for (Engine* e : eng_) raw.push_back(e->raw());
  rccl_ = jrq_rccl_init_all(raw.data(), static_cast<int>(raw.size())) == JRQ_OK;
  if (snap_) {  // (the snapshot object records how it publishes when it is made)
    jrq_snapshot_destroy(snap_);
    snap_ = nullptr;
  }
  return rccl_;
}

void ShardedGroupBatch::publish() {
  if (!snap_) {
    std::vector<jrq_table*> tabs;
    for (auto& b : shard_) {
      if (!b->table_) throw std::logic_error("ShardedGroupBatch::publish before the first flush");
      tabs.push_back(b->table_);
    }
    int err = 0;
    snap_ = jrq_snapshot_create(tabs.data(), static_cast<int>(tabs.size()), &err);
    if (!snap_) throwIfError(err ? err : JRQ_E_NOMEM, eng_[0]->raw(), "jrq_snapshot_create");
  }
  throwIfError(jrq_snapshot_publish(snap_), eng_[0]->raw(), "jrq_snapshot_publish");
}

void ShardedGroupBatch::readSnapshot(uint32_t i, int64_t* out) {
  if (!snap_) throw std::logic_error("ShardedGroupBatch::readSnapshot before publish");
  throwIfError(jrq_snapshot_read(snap_, static_cast<int>(i), out), eng_[i]->raw(), "jrq_snapshot_read");
}

bool ShardedGroupBatch::publishedOverRccl() const { return snap_ && jrq_snapshot_via(snap_) == 1; }

// ------------------------------------------------------------- leader tick

LeaderTicker::LeaderTicker(Engine& eng, uint32_t groups, uint32_t peers)
    : eng_(&eng), G_(groups), P_(peers) {
  if (peers == 0 || peers > JRQ_MAX_PEERS) throw std::invalid_argument("peers outside 1..16");
  ts_.assign(static_cast<size_t>(P_) * G_, 0);
  conf_.assign(G_, 0);
  self_.assign(G_, 0);
  lease_.assign(G_, 0);
  order_.assign(G_, 0);
  okMask_.assign(G_, 0);
  arrivals_.assign(G_, 0);
  peers_.resize(G_);
  reads_.resize(G_);
  waiting_.resize(G_);
  round_.assign(G_, 0);
}

int LeaderTicker::slot(uint32_t g, const PeerId& peer) const {
  const uint32_t id = peerId(peer);
  const auto& v = peers_[g];
  for (size_t s = 0; s < v.size(); ++s)
    if (v[s] == id) return static_cast<int>(s);
  return -1;
}

void LeaderTicker::becomeLeader(uint32_t g, const Configuration& conf, const Configuration* oldConf,
                                const PeerId& self, int64_t nowMs) {
  if (g >= G_) throw std::out_of_range("group id");
  std::vector<std::function<void(bool)>> failed;
  {
    std::lock_guard<std::mutex> l(mu_);
    auto& v = peers_[g];
    v.clear();
    auto slotOf = [&](const PeerId& p) {
      const uint32_t id = peerId(p);
      for (size_t s = 0; s < v.size(); ++s)
        if (v[s] == id) return static_cast<uint32_t>(s);
      if (v.size() >= P_) throw std::length_error("more distinct peers than slots");
      v.push_back(id);
      return static_cast<uint32_t>(v.size() - 1);
    };
    uint32_t nm = 0, om = 0;
    for (auto& p : conf.peers) nm |= 1u << slotOf(p);
    if (oldConf)
      for (auto& p : oldConf->peers) om |= 1u << slotOf(p);
    self_[g] = static_cast<uint8_t>(slotOf(self));
    // quorums as getQuorum / checkDeadNodes count them: peers.size() / 2 + 1 (distinct ids)
    const uint32_t nn = static_cast<uint32_t>(__builtin_popcount(nm)), no = static_cast<uint32_t>(__builtin_popcount(om));
    conf_[g] = JRQ_CONF(nm, om, nn / 2 + 1, no ? no / 2 + 1 : 0);
    for (uint32_t s = 0; s < P_; ++s) ts_[static_cast<size_t>(s) * G_ + g] = nowMs;
    lease_[g] = nowMs;
    closeRound(g, failed);
  }
  for (auto& f : failed) f(false);
}

// the group's open round and queued reads end (their closures go to `out`)
void LeaderTicker::closeRound(uint32_t g, std::vector<std::function<void(bool)>>& out) {
  for (auto& f : reads_[g]) out.push_back(std::move(f));
  for (auto& f : waiting_[g]) out.push_back(std::move(f));
  reads_[g].clear();
  waiting_[g].clear();
  round_[g] = 0;
  order_[g] = 0;
  okMask_[g] = 0;
  arrivals_[g] = 0;
}

void LeaderTicker::stepDown(uint32_t g) {
  std::vector<std::function<void(bool)>> failed;
  {
    std::lock_guard<std::mutex> l(mu_);
    conf_[g] = 0;
    closeRound(g, failed);
  }
  for (auto& f : failed) f(false);
}

void LeaderTicker::onRpcSent(uint32_t g, const PeerId& peer, int64_t nowMs) {
  std::lock_guard<std::mutex> l(mu_);
  const int s = slot(g, peer);
  if (s >= 0) ts_[static_cast<size_t>(s) * G_ + g] = nowMs;
}

void LeaderTicker::readIndex(uint32_t g, std::function<void(bool)> done) {
  int answer = -1;  // -1 queued, 0 false, 1 true
  {
    std::lock_guard<std::mutex> l(mu_);
    if (g >= G_ || conf_[g] == 0) answer = 0;                    // not the leader (EPERM)
    else if (((conf_[g] >> 32) & 0xFFu) <= 1) answer = 1;        // quorum <= 1: fast path
    else waiting_[g].push_back(std::move(done));
  }
  if (answer >= 0) done(answer == 1);
}

uint64_t LeaderTicker::startReadRound(uint32_t g) {
  std::lock_guard<std::mutex> l(mu_);
  if (g >= G_ || conf_[g] == 0 || round_[g] != 0 || waiting_[g].empty()) return 0;
  reads_[g].swap(waiting_[g]);
  order_[g] = 0;
  okMask_[g] = 0;
  arrivals_[g] = 0;
  round_[g] = ++roundSeq_;
  return round_[g];
}

void LeaderTicker::onHeartbeatResponse(uint32_t g, uint64_t round, const PeerId& peer, bool success) {
  std::lock_guard<std::mutex> l(mu_);
  if (g >= G_ || round == 0 || round != round_[g]) return;  // another round's response
  const int s = slot(g, peer);
  if (s < 0 || ((order_[g] >> (4 * s)) & 0xFu) != 0) return;  // one response per peer
  const uint32_t pos = arrivals_[g] < 15 ? ++arrivals_[g] : 15u;
  order_[g] |= static_cast<uint64_t>(pos) << (4 * s);
  if (success) okMask_[g] |= static_cast<uint16_t>(1u << s);
}

uint32_t LeaderTicker::tick(int64_t nowMs, int64_t leaseTimeoutMs, const StepDown& onStepDown) {
  std::vector<uint8_t> ok(G_), ri(G_);
  std::vector<uint16_t> dead(G_);
  std::vector<std::pair<uint32_t, uint16_t>> downs;
  std::vector<std::pair<std::function<void(bool)>, bool>> done;
  {
    std::lock_guard<std::mutex> l(mu_);
    throwIfError(jrq_leader_tick(eng_->raw(), ts_.data(), G_, P_, conf_.data(), self_.data(), G_, nowMs,
                                 leaseTimeoutMs, ok.data(), lease_.data(), dead.data(), order_.data(),
                                 okMask_.data(), ri.data()),
                 eng_->raw(), "jrq_leader_tick");
    for (uint32_t g = 0; g < G_; ++g) {
      if (conf_[g] == 0) continue;  // not a leader
      if (round_[g] != 0 && ri[g] != JRQ_READINDEX_PENDING) {  // the open round is decided
        const bool good = ri[g] == JRQ_READINDEX_SUCCESS;
        for (auto& f : reads_[g]) done.emplace_back(std::move(f), good);
        reads_[g].clear();
        round_[g] = 0;  // its late responses are dropped from now on
        order_[g] = 0;
        okMask_[g] = 0;
        arrivals_[g] = 0;
      }
      if (ok[g] != 3) {  // "Majority of the group dies": step down
        downs.emplace_back(g, dead[g]);
        conf_[g] = 0;
        std::vector<std::function<void(bool)>> failed;
        closeRound(g, failed);
        for (auto& f : failed) done.emplace_back(std::move(f), false);
      }
    }
  }
  for (auto& d : done) d.first(d.second);
  if (onStepDown)
    for (auto& d : downs) onStepDown(d.first, d.second);
  return static_cast<uint32_t>(downs.size());
}

int64_t LeaderTicker::lastLeaderTimestamp(uint32_t g) const {
  std::lock_guard<std::mutex> l(mu_);
  return lease_[g];
}

bool LeaderTicker::isLeader(uint32_t g) const {
  std::lock_guard<std::mutex> l(mu_);
  return conf_[g] != 0;
}

}  // namespace jraft
