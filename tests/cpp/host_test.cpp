// host_test.cpp -- the reference's hot-path unit tests, re-expressed against the C++ host
// mirror (sofa-jraft_amd/host) over libjrq.so.  Run by tests/test_host_cpp.py:
//   host_test cpu   -> tests that need no GPU (synchronous BallotBox semantics)
//   host_test gpu   -> everything, decisions and checksums computed on the GPU
// The differential tests replay the same calls through the oracle's Java-faithful BallotBox
// (oracle/jraft_oracle.c, test infrastructure) and compare the state after every flush.
// Sources restated (jraft-core/src/test/java/com/alipay/sofa/jraft/...):
//   core/BallotBoxTest.java:62-154, entity/BallotTest.java:37-50,
//   entity/LogEntryTest.java:95-125, util/CrcUtilTest.java:27-42
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include <random>
#include <set>

#include "../../oracle/jraft_oracle.h"
#include "../../sofa-jraft_amd/host/jraft_host.h"

using namespace jraft;

static int g_fail = 0, g_pass = 0;
#define CHECK(c)                                                               \
  do {                                                                         \
    if (!(c)) {                                                                \
      std::fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
      ++g_fail;                                                                \
      return;                                                                  \
    }                                                                          \
  } while (0)

template <typename E, typename F>
static bool throws(F f) {
  try {
    f();
  } catch (const E&) {
    return true;
  } catch (...) {
    return false;
  }
  return false;
}

struct Waiter {  // the Mockito FSMCaller of BallotBoxTest
  std::vector<int64_t> calls;
  CommitWaiter fn() {
    return [this](int64_t i) { calls.push_back(i); };
  }
};

static Configuration conf(const char* s) { return Configuration::parse(s); }

// --------------------------------------------------------- CPU (no engine)

static void testResetPendingIndex() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(box.getPendingIndex() == 0);
  CHECK(box.resetPendingIndex(1));
  CHECK(box.getPendingIndex() == 1);
}

static void testAppendPendingTask() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  Configuration c = conf("localhost:8081,localhost:8082,localhost:8083");
  Configuration o = conf("localhost:8081");
  CHECK(box.getPendingMetaQueueSize() == 0);
  CHECK(!box.appendPendingTask(c, &o));
  CHECK(box.resetPendingIndex(1));
  CHECK(box.appendPendingTask(c, &o));
  CHECK(box.getPendingMetaQueueSize() == 1);
}

static void testClearPendingTasks() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  Configuration c = conf("localhost:8081,localhost:8082,localhost:8083");
  CHECK(box.resetPendingIndex(1));
  bool ran = false, ok = true;
  CHECK(box.appendPendingTask(c, nullptr, [&](bool st) { ran = true; ok = st; }));
  box.clearPendingTasks();
  CHECK(box.getPendingMetaQueueSize() == 0 && box.getPendingIndex() == 0);
  CHECK(ran && !ok);  // closures fail when the leader steps down
}

static void testCommitAtChecks() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(!box.commitAt(1, 3, PeerId("localhost", 8081)));  // not leader
  CHECK(box.resetPendingIndex(1));
  Configuration c = conf("localhost:8081,localhost:8082,localhost:8083");
  Configuration o = conf("localhost:8081");
  CHECK(box.appendPendingTask(c, &o));
  CHECK(box.getLastCommittedIndex() == 0);
  CHECK(throws<std::out_of_range>([&] { box.commitAt(1, 3, PeerId("localhost", 8081)); }));
  CHECK(box.commitAt(1, 1, PeerId("localhost", 8081)));
  CHECK(box.commitAt(1, 1, PeerId("localhost", 8084)));  // unknown peer: no-op, true
}

static void testSetLastCommittedIndexHasPending() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(box.resetPendingIndex(1));
  CHECK(throws<std::invalid_argument>([&] { box.setLastCommittedIndex(1); }));
}

static void testSetLastCommittedIndexLessThan() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(!box.setLastCommittedIndex(-1));
}

static void testSetLastCommittedIndex() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(box.getLastCommittedIndex() == 0);
  CHECK(box.setLastCommittedIndex(1));
  CHECK(box.getLastCommittedIndex() == 1);
  CHECK(w.calls.size() == 1 && w.calls[0] == 1);  // verify(waiter, only()).onCommitted(1)
}

static void testInitRequiresWaiter() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 8);
  BallotBox box(batch, 0);
  CHECK(!box.init({}));
}

static void testNonContiguousAckRejected() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(box.resetPendingIndex(10));
  Configuration c = conf("a:1,b:2,c:3");
  for (int i = 0; i < 10; ++i) CHECK(box.appendPendingTask(c, nullptr));
  CHECK(box.commitAt(10, 12, PeerId("b", 2)));
  CHECK(box.commitAt(13, 15, PeerId("b", 2)));
  CHECK(throws<std::logic_error>([&] { box.commitAt(17, 18, PeerId("b", 2)); }));
}

// --------------------------------------------------------------- GPU tests

static void testCommitAtOnGpu(Engine& eng) {
  auto batch = std::make_shared<GroupBatch>(&eng, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(!box.commitAt(1, 3, PeerId("localhost", 8081)));
  CHECK(box.resetPendingIndex(1));
  Configuration c = conf("localhost:8081,localhost:8082,localhost:8083");
  Configuration o = conf("localhost:8081");
  CHECK(box.appendPendingTask(c, &o));
  CHECK(throws<std::out_of_range>([&] { box.commitAt(1, 3, PeerId("localhost", 8081)); }));
  CHECK(box.commitAt(1, 1, PeerId("localhost", 8081)));
  batch->flush();
  CHECK(box.getLastCommittedIndex() == 0);
  CHECK(box.getPendingIndex() == 1);
  CHECK(box.commitAt(1, 1, PeerId("localhost", 8082)));
  batch->flush();
  CHECK(box.getLastCommittedIndex() == 1);
  CHECK(box.getPendingIndex() == 2);
  CHECK(w.calls.size() == 1 && w.calls[0] == 1);  // verify(waiter, only()).onCommitted(1)
}

static void testBallotGrantOnGpu(Engine& eng) {
  // BallotTest.testGrant: conf {8081,8082,8083}; 8081 -> not granted; unknown 8084 -> not;
  // 8082 -> granted.
  auto batch = std::make_shared<GroupBatch>(&eng, 1, 8);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(box.resetPendingIndex(1));
  CHECK(box.appendPendingTask(conf("localhost:8081,localhost:8082,localhost:8083"), nullptr));
  box.commitAt(1, 1, PeerId("localhost", 8081));
  batch->flush();
  CHECK(box.getLastCommittedIndex() == 0);
  box.commitAt(1, 1, PeerId("localhost", 8084));
  batch->flush();
  CHECK(box.getLastCommittedIndex() == 0);
  box.commitAt(1, 1, PeerId("localhost", 8082));
  batch->flush();
  CHECK(box.getLastCommittedIndex() == 1);
}

static void testManyGroupsJointConsensusOnGpu(Engine& eng) {
  // 1000 groups; group g: stable 3-peer conf for 5 entries, then a joint stretch
  // (new 5 peers, old 3) for 5 entries; peers ack different depths.
  const uint32_t G = 1000;
  auto batch = std::make_shared<GroupBatch>(&eng, G, 8);
  std::vector<BallotBox> boxes;
  std::vector<Waiter> ws(G);
  Configuration c3 = conf("p:1,p:2,p:3"), c5 = conf("p:1,p:2,p:3,p:4,p:5");
  for (uint32_t g = 0; g < G; ++g) {
    boxes.emplace_back(batch, g);
    CHECK(boxes[g].init({ws[g].fn()}));
    CHECK(boxes[g].resetPendingIndex(100));
    for (int i = 0; i < 5; ++i) CHECK(boxes[g].appendPendingTask(c3, nullptr));
    for (int i = 0; i < 5; ++i) CHECK(boxes[g].appendPendingTask(c5, &c3));
  }
  for (uint32_t g = 0; g < G; ++g) {
    // leader p:1 acks all; p:2 acks up to 100 + g % 10; p:4 acks up to 100 + (g / 10) % 10
    boxes[g].commitAt(100, 109, PeerId("p", 1));
    boxes[g].commitAt(100, 100 + g % 10, PeerId("p", 2));
    boxes[g].commitAt(100, 100 + (g / 10) % 10, PeerId("p", 4));
  }
  batch->flush();
  for (uint32_t g = 0; g < G; ++g) {
    const int64_t a = 100 + g % 10, b = 100 + (g / 10) % 10;
    // entries 100..104 (c3): need 2 of {1,2,3}: 1 + (2 if idx<=a) -> commit up to min(104, a)
    // entries 105..109 (joint): new needs 3 of {1..5} = {1, 2 if <=a, 4 if <=b};
    // old needs 2 of {1,2,3} -> needs 2 (idx <= a)  => granted iff idx <= a and idx <= b
    int64_t exp = 99;
    for (int64_t i = 100; i <= 109; ++i) {
      bool gr = i <= 104 ? (i <= a) : (i <= a && i <= b);
      if (gr) exp = i;
    }
    CHECK(boxes[g].getLastCommittedIndex() == exp);
    if (exp > 99) CHECK(ws[g].calls.size() == 1 && ws[g].calls[0] == exp);
  }
}

static void testLogEntryChecksumOnGpu(Engine& eng) {
  // LogEntryTest.testChecksum (LogEntryTest.java:95-125)
  LogEntry entry;
  entry.type = EntryType::NO_OP;
  entry.id = {100, 3};
  entry.data.assign({'h', 'e', 'l', 'l', 'o'});
  entry.peers = {PeerId("localhost", 99, 1), PeerId("localhost", 100, 2)};
  const uint64_t c = entry.checksum(eng);
  CHECK(c != 0);
  CHECK(c == 0x670396DD526CA3BDull);  // tests/golden/entity_vectors.json
  CHECK(c == entry.checksum(eng));
  CHECK(!entry.isCorrupted(eng));
  CHECK(!entry.hasChecksum());
  entry.setChecksum(c);
  CHECK(entry.hasChecksum());
  CHECK(!entry.isCorrupted(eng));
  entry.id.index = 1;
  CHECK(entry.checksum(eng) != c);
  CHECK(entry.isCorrupted(eng));
  entry.id.index = 100;
  CHECK(!entry.isCorrupted(eng));
  entry.data.assign({'h', 'E', 'l', 'l', 'o'});
  CHECK(entry.checksum(eng) != c);
  CHECK(entry.isCorrupted(eng));
}

static void testCrcUtilOnGpu(Engine& eng) {
  // CrcUtilTest: byte[] and (byte[], off, len) agree; catalogue check value
  const char* s = "123456789";
  std::vector<uint8_t> v(s, s + 9);
  CHECK(CrcUtil::crc64(eng, v) == 0x6C40DF5F0B497347ull);
  std::vector<uint8_t> w = {'x', 'y'};
  w.insert(w.end(), v.begin(), v.end());
  CHECK(CrcUtil::crc64(eng, w.data(), 2, 9) == 0x6C40DF5F0B497347ull);
  CHECK(CrcUtil::crc64(eng, nullptr, 0, 0) == 0);
}

static void testCRC64ChecksumOnGpu(Engine& eng) {
  // java.util.zip.Checksum use by RheaKV snapshots: update(byte), update(byte[],off,len) in
  // pieces, getValue mid-stream, reset; small flush threshold forces many GPU folds.
  const char* s = "123456789";
  CRC64 c(eng, 4);
  c.update(s[0]);
  c.update(reinterpret_cast<const uint8_t*>(s), 1, 3);
  CHECK(c.getValue() == CrcUtil::crc64(eng, reinterpret_cast<const uint8_t*>(s), 0, 4));
  c.update(reinterpret_cast<const uint8_t*>(s), 4, 5);
  CHECK(c.getValue() == 0x6C40DF5F0B497347ull);
  c.update(reinterpret_cast<const uint8_t*>(s), 0, 0);
  CHECK(c.getValue() == 0x6C40DF5F0B497347ull);
  c.reset();
  CHECK(c.getValue() == 0);
  std::vector<uint8_t> big(1 << 20);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto& b : big) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; b = (uint8_t)x; }
  CRC64 d(eng, 100000);
  for (size_t o = 0; o < big.size(); o += 77777) d.update(big.data(), o, std::min<size_t>(77777, big.size() - o));
  CHECK(d.getValue() == CrcUtil::crc64(eng, big));
}

// ------------------------------------------------------- differential tests

// One group driven identically through the host mirror and the oracle's BallotBox; peers are
// PeerId("p", id) on the mirror side and `id` on the oracle side.
struct Twin {
  BallotBox box;
  jo_ballot_box* bb;
  Waiter w;
  Twin(std::shared_ptr<GroupBatch> b, uint32_t g) : box(std::move(b), g), bb(jo_bb_new()) {
    box.init({w.fn()});
  }
  Twin(Twin&& o) noexcept : box(o.box), bb(o.bb), w(std::move(o.w)) {
    o.bb = nullptr;
    box.init({w.fn()});
  }
  ~Twin() {
    if (bb) jo_bb_free(bb);
  }
  static Configuration confOf(const std::vector<int32_t>& ids) {
    Configuration c;
    for (int32_t i : ids) c.peers.emplace_back("p", i);
    return c;
  }
  bool append(const std::vector<int32_t>& cur, const std::vector<int32_t>* old, int64_t n) {
    const Configuration c = confOf(cur);
    const Configuration o = old ? confOf(*old) : Configuration();
    bool ok = true;
    for (int64_t i = 0; i < n; ++i) {
      ok = box.appendPendingTask(c, old ? &o : nullptr) && ok;
      jo_bb_append_pending_task(bb, cur.data(), (int32_t)cur.size(), old ? old->data() : nullptr,
                                old ? (int32_t)old->size() : -1);
    }
    return ok;
  }
  void ack(int64_t first, int64_t last, int32_t peer) {
    box.commitAt(first, last, PeerId("p", peer));
    jo_bb_commit_at(bb, first, last, peer);
  }
  bool same() const {
    return box.getLastCommittedIndex() == jo_bb_last_committed_index(bb) &&
           box.getPendingIndex() == jo_bb_pending_index(bb) &&
           box.getPendingMetaQueueSize() == jo_bb_queue_size(bb) &&
           (w.calls.empty() ? jo_bb_on_committed_calls(bb) == 0
                            : w.calls.back() == jo_bb_on_committed_last(bb));
  }
};

static void testAddPeerCatchUpOnGpu(Engine& eng) {
  // A peer being added is acked by its catch-up replicator before any conf names it
  // (Replicator.java:1387-1392); the joint conf entry then counts it, and its next, contiguous
  // ack must be accepted (pendingIndex 100, the new peer caught up to 105, joint conf at 111).
  auto batch = std::make_shared<GroupBatch>(&eng, 1, 8);
  Twin t(batch, 0);
  CHECK(t.box.resetPendingIndex(100) && jo_bb_reset_pending_index(t.bb, 100) == JO_TRUE);
  const std::vector<int32_t> c3 = {1, 2, 3}, c4 = {1, 2, 3, 4};
  CHECK(t.append(c3, nullptr, 11));  // 100..110
  t.ack(100, 105, 4);                // not in any conf yet
  CHECK(t.append(c4, &c3, 1));       // 111: joint {1,2,3,4} / {1,2,3}
  t.ack(106, 111, 4);
  t.ack(100, 111, 1);
  t.ack(100, 108, 2);
  batch->flush();
  CHECK(t.same());
  CHECK(t.box.getLastCommittedIndex() == 108);  // 111 needs 3 of 4 and 2 of 3: {1, 4} only
  t.ack(109, 111, 2);
  batch->flush();
  CHECK(t.same() && t.box.getLastCommittedIndex() == 111);
}

// Random call sequences (appends under stable and joint confs, conf changes that replace
// peers, contiguous acks from members and catch-up peers, step-downs and new terms) through
// the mirror and the oracle; the state must agree after every flush.  More distinct peers
// than slots pass through each group over time, so slots are recycled.
static void testRandomDifferentialOnGpu(Engine& eng) {
  const uint32_t G = 96, P = 8;
  auto batch = std::make_shared<GroupBatch>(&eng, G, P);
  std::vector<Twin> tw;
  tw.reserve(G);
  std::mt19937_64 rng(20240611);
  auto R = [&](int64_t n) { return static_cast<int64_t>(rng() % static_cast<uint64_t>(n)); };
  struct S {
    std::vector<int32_t> cur, old;
    bool joint = false;
    std::map<int32_t, int64_t> m;  // peer -> highest acked index (the Replicator's view)
    int64_t la = 0;
    int64_t confEntry = 0;  // index of the last conf entry appended
  };
  std::vector<S> st(G);
  auto pickConf = [&](std::vector<int32_t> keep) {
    std::set<int32_t> s(keep.begin(), keep.end());
    const size_t n = 1 + R(3);
    while (s.size() < n) s.insert(1 + static_cast<int32_t>(R(12)));
    while (s.size() > n) s.erase(std::next(s.begin(), R(s.size())));
    return std::vector<int32_t>(s.begin(), s.end());
  };
  for (uint32_t g = 0; g < G; ++g) {
    tw.emplace_back(batch, g);
    Twin& t = tw.back();
    const int64_t lc = R(50);
    t.box.setLastCommittedIndex(lc);
    jo_bb_set_last_committed_index(t.bb, lc);
    const int64_t pi = lc + 1 + R(5);
    CHECK(t.box.resetPendingIndex(pi) && jo_bb_reset_pending_index(t.bb, pi) == JO_TRUE);
    st[g].cur = pickConf({});
    st[g].la = pi - 1;
    for (int32_t p = 1; p <= 12; ++p) st[g].m[p] = pi - 1 - R(3);
  }
  int flushes = 0;
  for (int step = 0; step < 6000; ++step) {
    const uint32_t g = static_cast<uint32_t>(R(G));
    Twin& t = tw[g];
    S& s = st[g];
    const int64_t a = R(100);
    if (t.box.getPendingIndex() == 0) {  // stepped down: a new term later
      if (a < 20) {
        const int64_t pi = std::max(s.la + 1, t.box.getLastCommittedIndex() + 1) + R(3);
        CHECK(t.box.resetPendingIndex(pi) && jo_bb_reset_pending_index(t.bb, pi) == JO_TRUE);
        s.la = pi - 1;
        s.joint = false;
        s.confEntry = 0;
        for (auto& kv : s.m) kv.second = pi - 1 - R(3);
      }
    } else if (a < 35) {  // appendPendingTask x k under the current conf
      const int64_t k = 1 + R(4);
      CHECK(t.append(s.cur, s.joint ? &s.old : nullptr, k));
      s.la += k;
    } else if (a < 40) {  // conf change: stable -> joint (replacing peers), joint -> stable
      // NodeImpl starts the next stage only once the previous conf entry is committed
      // (ConfigurationCtx.nextStage on onConfigurationChangeDone, NodeImpl.java:457-487)
      if (t.box.getLastCommittedIndex() < s.confEntry) continue;
      if (!s.joint) {
        s.old = s.cur;
        s.cur = pickConf(std::vector<int32_t>(s.old.begin(), s.old.begin() + R(s.old.size() + 1)));
        s.joint = true;
      } else {
        s.joint = false;
      }
      CHECK(t.append(s.cur, s.joint ? &s.old : nullptr, 1));
      s.la += 1;
      s.confEntry = s.la;
    } else if (a < 94) {  // an ack, contiguous per peer: members mostly, any peer sometimes
      int32_t p;
      if (R(10) < 8) {
        const auto& pool = (s.joint && R(2)) ? s.old : s.cur;
        p = pool[R(pool.size())];
      } else {
        p = 1 + static_cast<int32_t>(R(12));
      }
      const int64_t first = s.m[p] + 1;
      const int64_t last = std::min(s.la, first + R(6));
      if (last >= first) {
        t.ack(first, last, p);
        s.m[p] = last;
      }
    } else if (a < 96) {  // the leader steps down
      t.box.clearPendingTasks();
      jo_bb_clear_pending_tasks(t.bb);
    } else {
      batch->flush();
      ++flushes;
      for (uint32_t h = 0; h < G; ++h) {
        if (!tw[h].same()) {
          std::fprintf(stderr, "  group %u: mirror lc %lld pi %lld q %lld | oracle lc %lld pi %lld q %lld\n", h,
                       (long long)tw[h].box.getLastCommittedIndex(), (long long)tw[h].box.getPendingIndex(),
                       (long long)tw[h].box.getPendingMetaQueueSize(),
                       (long long)jo_bb_last_committed_index(tw[h].bb), (long long)jo_bb_pending_index(tw[h].bb),
                       (long long)jo_bb_queue_size(tw[h].bb));
          CHECK(false);
        }
      }
    }
  }
  CHECK(flushes > 10);
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  struct T {
    const char* name;
    std::function<void()> fn;
  };
  std::vector<T> tests = {
      {"testResetPendingIndex", testResetPendingIndex},
      {"testAppendPendingTask", testAppendPendingTask},
      {"testClearPendingTasks", testClearPendingTasks},
      {"testCommitAtChecks", testCommitAtChecks},
      {"testSetLastCommittedIndexHasPending", testSetLastCommittedIndexHasPending},
      {"testSetLastCommittedIndexLessThan", testSetLastCommittedIndexLessThan},
      {"testSetLastCommittedIndex", testSetLastCommittedIndex},
      {"testInitRequiresWaiter", testInitRequiresWaiter},
      {"testNonContiguousAckRejected", testNonContiguousAckRejected},
  };
  std::unique_ptr<Engine> eng;
  if (gpu) {
    eng.reset(new Engine(0));
    Engine& e = *eng;
    tests.push_back({"testCommitAtOnGpu", [&] { testCommitAtOnGpu(e); }});
    tests.push_back({"testAddPeerCatchUpOnGpu", [&] { testAddPeerCatchUpOnGpu(e); }});
    tests.push_back({"testRandomDifferentialOnGpu", [&] { testRandomDifferentialOnGpu(e); }});
    tests.push_back({"testBallotGrantOnGpu", [&] { testBallotGrantOnGpu(e); }});
    tests.push_back({"testManyGroupsJointConsensusOnGpu", [&] { testManyGroupsJointConsensusOnGpu(e); }});
    tests.push_back({"testLogEntryChecksumOnGpu", [&] { testLogEntryChecksumOnGpu(e); }});
    tests.push_back({"testCrcUtilOnGpu", [&] { testCrcUtilOnGpu(e); }});
    tests.push_back({"testCRC64ChecksumOnGpu", [&] { testCRC64ChecksumOnGpu(e); }});
  }
  for (auto& t : tests) {
    const int before = g_fail;
    t.fn();
    if (g_fail == before) {
      ++g_pass;
      std::printf("PASS %s\n", t.name);
    } else {
      std::printf("FAIL %s\n", t.name);
    }
  }
  std::printf("%d passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
