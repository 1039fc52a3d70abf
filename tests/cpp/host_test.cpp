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
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include <random>
#include <set>

#include "../../oracle/jraft_oracle.h"
#include "../../sofa-jraft_amd/host/jraft_host.h"

using namespace jraft;

// Failure injection, present only in the sanitizer builds' test double (tests/cpp/fake_jrq.cpp):
// the next n jrq_table_update_gather calls fail.  Null against the real libjrq.so.
extern "C" void fake_jrq_fail_updates(int n) __attribute__((weak));
// Records of one upload that named the same (group, field) twice (the double counts them).
extern "C" uint64_t fake_jrq_dup_records() __attribute__((weak));

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

// The order-free records (JRQ_ACK, r06): acks and queue growth written at call time, applied on
// the device as a max.  A slot given to another peer resets the group's stamp, which drops every
// record of the group written before it -- the live peers' acks among them -- so the pack must
// ship their current matches again: the commit below needs them (3 slots: peers 1, 2 in the
// conf, 3 a catch-up peer; peer 4 then takes peer 3's slot in the same epoch).
static void testResetStampKeepsLiveAcks(Engine& eng) {
  auto batch = std::make_shared<GroupBatch>(&eng, 2, 3);
  Twin t(batch, 1);
  CHECK(t.box.resetPendingIndex(1) && jo_bb_reset_pending_index(t.bb, 1) == JO_TRUE);
  const std::vector<int32_t> c12 = {1, 2}, c124 = {1, 2, 4};
  CHECK(t.append(c12, nullptr, 10));  // 1..10
  t.ack(1, 2, 3);                     // peer 3 takes the free third slot
  batch->flush();                     // (sizes this thread's record buffers)
  CHECK(t.same() && batch->lastFlush().acks == 0);
  t.ack(1, 10, 1);                    // records (JRQ_ACK), not pack records
  t.ack(1, 6, 2);
  CHECK(t.append(c124, &c12, 1));     // 11: peer 4 needs a slot: peer 3's (no live conf names it)
  batch->flush();
  CHECK(batch->lastFlush().acks >= 3);
  CHECK(t.same() && t.box.getLastCommittedIndex() == 6);  // peers 1, 2 acked 1..6
  t.ack(7, 11, 2);
  t.ack(1, 11, 4);
  batch->flush();  // 11 is joint: {1, 2, 4} has 2 and 4, but {1, 2} only 2
  CHECK(t.same());
  CHECK(t.box.getLastCommittedIndex() == 10);
  t.ack(11, 11, 1);
  batch->flush();
  CHECK(t.same());
  CHECK(t.box.getLastCommittedIndex() == 11);
}

// The node's groups over three engines in one process (ShardedGroupBatch, r06): every group's
// commits against its oracle BallotBox after each concurrent flush of the shards, and the
// published node-wide snapshot (device copies: RCCL refuses three engines on one GPU) equal to
// every group's getLastCommittedIndex.
static void testShardedBatchOnGpu(Engine& eng) {
  Engine e1(0, 1u << 12, 16), e2(0, 1u << 12, 16);
  const uint32_t G = 1001, P = 5;
  ShardedGroupBatch sb({&eng, &e1, &e2}, G, P);
  CHECK(sb.shards() == 3 && sb.groupsPerShard() == 334);
  CHECK(!sb.rcclInitAll());  // one GPU (or the test double): copies
  std::vector<Twin> tw;
  tw.reserve(G);
  for (uint32_t g = 0; g < G; ++g) {
    uint32_t l = 0;
    tw.emplace_back(sb.shardOf(g, &l), l);
  }
  std::mt19937_64 rng(91);
  const std::vector<int32_t> c5 = {1, 2, 3, 4, 5};
  for (uint32_t g = 0; g < G; ++g) {
    const int64_t pi = 1 + static_cast<int64_t>(rng() % 1000);
    CHECK(tw[g].box.resetPendingIndex(pi) && jo_bb_reset_pending_index(tw[g].bb, pi) == JO_TRUE);
  }
  std::vector<std::array<int64_t, 5>> m(G);
  for (uint32_t g = 0; g < G; ++g) m[g].fill(tw[g].box.getPendingIndex() - 1);
  std::vector<int64_t> snap(G);
  for (int epoch = 0; epoch < 4; ++epoch) {
    for (uint32_t g = 0; g < G; ++g) {
      CHECK(tw[g].append(c5, nullptr, 1 + static_cast<int64_t>(rng() % 20)));
      const int64_t la = tw[g].box.getPendingIndex() + tw[g].box.getPendingMetaQueueSize() - 1;
      for (int p = 0; p < 5; ++p) {
        const int64_t to = std::min(la, m[g][p] + static_cast<int64_t>(rng() % 25));
        if (to > m[g][p]) {
          tw[g].ack(m[g][p] + 1, to, p + 1);
          m[g][p] = to;
        }
      }
    }
    sb.flush();
    sb.publish();
    for (uint32_t g = 0; g < G; ++g) CHECK(tw[g].same());
    for (uint32_t i = 0; i < sb.shards(); ++i) {
      sb.readSnapshot(i, snap.data());
      for (uint32_t g = 0; g < G; ++g) CHECK(snap[g] == tw[g].box.getLastCommittedIndex());
    }
  }
  CHECK(!sb.publishedOverRccl());
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

// ------------------------------------------------------- concurrent callers

// The reference's callers of one BallotBox run concurrently (BallotBox is @ThreadSafe,
// BallotBox.java:45, a StampedLock per call, :98): the NodeImpl disruptor appends
// (NodeImpl.java:1195-1196), the LogManager thread self-acks (NodeImpl.java:1156), one Bolt
// callback thread per replicator acks its peer (Replicator.java:1391).  Here one thread per
// role works over every group of the batch while a background flusher decides epochs, and a
// second stage steps down a quarter of the groups from several threads at once.  The final
// state of every group must equal the oracle's BallotBox fed the same calls in one order (the
// post-epoch state is order-independent, BallotBox.java:96-139), every closure must run
// exactly once, and onCommitted must see increasing indices ending at lastCommittedIndex.
static void testConcurrentCallers(Engine& eng, uint32_t G, int64_t kEntries) {
  const uint32_t P = 5, kAcks = 4;  // peers 0 (leader) .. 4
  auto batch = std::make_shared<GroupBatch>(&eng, G, 8);
  std::vector<BallotBox> boxes;
  boxes.reserve(G);
  struct Obs {
    std::atomic<int64_t> last{-1};
    std::atomic<int64_t> calls{0};
    std::atomic<bool> monotone{true};
    std::atomic<int64_t> closuresOk{0}, closuresFailed{0};
  };
  std::vector<Obs> obs(G);
  std::vector<int64_t> pi0(G);
  std::vector<int64_t> jointAt(G, 0);  // index of the joint conf entry (0: stays stable)
  std::vector<std::atomic<int64_t>> published(G);  // highest appended index, for the ackers
  std::mt19937_64 rng(77);
  for (uint32_t g = 0; g < G; ++g) {
    boxes.emplace_back(batch, g);
    Obs* o = &obs[g];
    boxes[g].init({[o](int64_t c) {
      const int64_t prev = o->last.exchange(c);
      if (c <= prev) o->monotone = false;
      o->calls.fetch_add(1);
    }});
    pi0[g] = 1 + static_cast<int64_t>(rng() % 1000);
    CHECK(boxes[g].resetPendingIndex(pi0[g]));
    published[g].store(pi0[g] - 1);
    if (g % 4 == 1) jointAt[g] = pi0[g] + kEntries / 3 + static_cast<int64_t>(rng() % (kEntries / 4));
  }
  auto confOf = [](int n) {
    Configuration c;
    for (int p = 0; p < n; ++p) c.peers.emplace_back("10.0.0.1", 9000 + p);
    return c;
  };
  const Configuration c3 = confOf(3), c5 = confOf(5);
  std::vector<PeerId> peers;
  for (int p = 0; p < 5; ++p) peers.emplace_back("10.0.0.1", 9000 + p);
  batch->startFlusher(FlushPolicy{200, 4096});
  std::atomic<bool> failed{false};
  std::vector<std::thread> th;
  // the NodeImpl disruptor: batches of appends per group, every 3rd entry with a closure
  th.emplace_back([&] {
    try {
      for (int64_t k = 0; k < kEntries; k += 8) {
        // halfway, hold the appends until the background flusher has flushed at least once:
        // the flusher then provably ran concurrently with the callers, whatever the timing
        if (k == (kEntries / 16) * 8) {
          const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(60);
          while (batch->flushCount() < 1 && std::chrono::steady_clock::now() < until)
            std::this_thread::sleep_for(std::chrono::microseconds(100));
          if (batch->flushCount() < 1) failed = true;
        }
        for (uint32_t g = 0; g < G; ++g) {
          for (int64_t i = 0; i < 8; ++i) {
            const int64_t idx = pi0[g] + k + i;
            const bool joint = jointAt[g] && idx >= jointAt[g];
            const Configuration& c = joint ? c5 : c3;
            const Configuration* old = joint ? &c3 : nullptr;
            Obs* o = &obs[g];
            const bool ok = idx % 3 == 0
                                ? boxes[g].appendPendingTask(c, old, [o](bool st) {
                                    (st ? o->closuresOk : o->closuresFailed).fetch_add(1);
                                  })
                                : boxes[g].appendPendingTask(c, old);
            if (!ok) failed = true;
          }
          published[g].store(pi0[g] + k + 7, std::memory_order_release);
        }
      }
    } catch (...) {
      failed = true;
    }
  });
  // the LogManager self-ack (peer 0) and one replicator thread per follower: contiguous acks
  // up to what has been appended, peer p lagging p entries behind; peers 3 and 4 (named only
  // by the joint conf) ack every group, as catch-up replicators would
  for (uint32_t p = 0; p < P; ++p)
    th.emplace_back([&, p] {
      try {
        std::vector<int64_t> m(G);
        for (uint32_t g = 0; g < G; ++g) m[g] = pi0[g] - 1;
        for (;;) {
          bool more = false;
          for (uint32_t g = 0; g < G; ++g) {
            const int64_t top = std::min(published[g].load(std::memory_order_acquire) - static_cast<int64_t>(p),
                                         pi0[g] + kEntries - 1 - static_cast<int64_t>(p));
            if (m[g] < pi0[g] + kEntries - 1 - static_cast<int64_t>(p)) more = true;
            if (top > m[g]) {
              const int64_t last = std::min(top, m[g] + static_cast<int64_t>(kAcks));
              boxes[g].commitAt(m[g] + 1, last, peers[p]);
              m[g] = last;
            }
          }
          if (!more) break;
        }
      } catch (...) {
        failed = true;
      }
    });
  // readers: getLastCommittedIndex never goes backwards
  th.emplace_back([&] {
    std::vector<int64_t> seen(G, 0);
    for (int r = 0; r < 200; ++r)
      for (uint32_t g = 0; g < G; ++g) {
        const int64_t c = boxes[g].getLastCommittedIndex();
        if (c < seen[g]) failed = true;
        seen[g] = c;
      }
  });
  for (auto& t : th) t.join();
  batch->stopFlusher();
  batch->flush();
  CHECK(!failed);
  if (fake_jrq_dup_records) CHECK(fake_jrq_dup_records() == 0);
  std::vector<jo_ballot_box*> ob(G);
  auto same = [&](uint32_t g) {
    const int64_t lc = jo_bb_last_committed_index(ob[g]);
    if (boxes[g].getLastCommittedIndex() == lc && boxes[g].getPendingIndex() == jo_bb_pending_index(ob[g]) &&
        boxes[g].getPendingMetaQueueSize() == jo_bb_queue_size(ob[g]))
      return true;
    std::fprintf(stderr, "  group %u: mirror lc %lld pi %lld q %lld, oracle lc %lld pi %lld q %lld\n", g,
                 (long long)boxes[g].getLastCommittedIndex(), (long long)boxes[g].getPendingIndex(),
                 (long long)boxes[g].getPendingMetaQueueSize(), (long long)lc,
                 (long long)jo_bb_pending_index(ob[g]), (long long)jo_bb_queue_size(ob[g]));
    return false;
  };
  for (uint32_t g = 0; g < G; ++g) {
    jo_ballot_box* bb = ob[g] = jo_bb_new();
    CHECK(jo_bb_reset_pending_index(bb, pi0[g]) == JO_TRUE);
    const int32_t i3[] = {0, 1, 2}, i5[] = {0, 1, 2, 3, 4};
    for (int64_t idx = pi0[g]; idx < pi0[g] + kEntries; ++idx) {
      const bool joint = jointAt[g] && idx >= jointAt[g];
      jo_bb_append_pending_task(bb, joint ? i5 : i3, joint ? 5 : 3, joint ? i3 : nullptr, joint ? 3 : -1);
    }
    for (int32_t p = 0; p < static_cast<int32_t>(P); ++p) jo_bb_commit_at(bb, pi0[g], pi0[g] + kEntries - 1 - p, p);
    CHECK(same(g));
    const int64_t lc = jo_bb_last_committed_index(bb);
    CHECK(obs[g].monotone && obs[g].last == lc);
    // closures of entries <= lc ran once with OK; the rest are still queued
    int64_t exp = 0;
    for (int64_t idx = pi0[g]; idx <= lc; ++idx) exp += idx % 3 == 0;
    CHECK(obs[g].closuresOk == exp && obs[g].closuresFailed == 0);
  }
  // >= 1 background flush (waited for mid-run above) + the explicit one after stopFlusher
  CHECK(batch->flushCount() >= 2);
  // step-downs from several threads at once (groups g % 16 < 4), concurrent with acks of the
  // other groups by peer 4 up to the last entry
  std::vector<std::thread> th2;
  for (uint32_t t = 0; t < 4; ++t)
    th2.emplace_back([&, t] {
      for (uint32_t g = t; g < G; g += 16) boxes[g].clearPendingTasks();
    });
  th2.emplace_back([&] {
    for (uint32_t g = 0; g < G; ++g)
      if (g % 16 >= 4) boxes[g].commitAt(pi0[g], pi0[g] + kEntries - 1, peers[4]);
  });
  for (auto& t : th2) t.join();
  batch->flush();
  for (uint32_t g = 0; g < G; ++g) {
    if (g % 16 < 4) {
      jo_bb_clear_pending_tasks(ob[g]);
      int64_t queued = 0;  // entries above lc with closures: failed by the step-down
      for (int64_t idx = boxes[g].getLastCommittedIndex() + 1; idx < pi0[g] + kEntries; ++idx) queued += idx % 3 == 0;
      CHECK(obs[g].closuresFailed == queued);
    } else {
      jo_bb_commit_at(ob[g], pi0[g], pi0[g] + kEntries - 1, 4);
    }
    CHECK(same(g));
    CHECK(obs[g].last == jo_bb_last_committed_index(ob[g]));
  }
  for (auto* bb : ob) jo_bb_free(bb);
}

// Every slot of the group named by a live conf run, and a peer in none of them acks: no pending
// ballot counts it (Ballot.grant finds nothing, Ballot.java:100-127), commitAt returns true.
static void testAckFromPeerWithoutSlot() {
  auto batch = std::make_shared<GroupBatch>(nullptr, 1, 3);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(box.resetPendingIndex(5));
  CHECK(box.appendPendingTask(conf("a:1,b:2,c:3"), nullptr));
  CHECK(box.commitAt(5, 5, PeerId("d", 4)));
  CHECK(box.commitAt(5, 5, PeerId("a", 1)));
  CHECK(box.getPendingMetaQueueSize() == 1);
}

// flush() and clearPendingTasks() from inside a commit callback of the same batch are refused.
static void testReentrantFlushRefused(Engine& eng) {
  auto batch = std::make_shared<GroupBatch>(&eng, 2, 3);
  BallotBox a(batch, 0), b(batch, 1);
  bool refusedFlush = false, refusedClear = false, appended = false;
  CHECK(a.init({[&](int64_t) {
    try {
      batch->flush();
    } catch (const std::logic_error&) {
      refusedFlush = true;
    }
    try {
      b.clearPendingTasks();
    } catch (const std::logic_error&) {
      refusedClear = true;
    }
    appended = b.appendPendingTask(conf("a:1,b:2,c:3"), nullptr);  // recording calls are fine
  }}));
  Waiter w;
  CHECK(b.init({w.fn()}));
  CHECK(a.resetPendingIndex(1) && b.resetPendingIndex(1));
  CHECK(a.appendPendingTask(conf("a:1,b:2,c:3"), nullptr));
  a.commitAt(1, 1, PeerId("a", 1));
  a.commitAt(1, 1, PeerId("b", 2));
  batch->flush();
  CHECK(a.getLastCommittedIndex() == 1);
  CHECK(refusedFlush && refusedClear && appended);
  CHECK(b.getPendingMetaQueueSize() == 1);
}

// an upload that fails after flush() swapped the dirty lists out must not strand
// the groups it carried -- the pack had cleared their dirty bits.  The next flush ships them
// again and every group commits.
static void testFlushFailureRelists(Engine& eng) {
  if (!fake_jrq_fail_updates) return;  // (the real library has no failure injection)
  const uint32_t G = 300;
  auto batch = std::make_shared<GroupBatch>(&eng, G, 3);
  std::vector<BallotBox> boxes;
  std::vector<Waiter> ws(G);
  for (uint32_t g = 0; g < G; ++g) {
    boxes.emplace_back(batch, g);
    CHECK(boxes[g].init({ws[g].fn()}));
    CHECK(boxes[g].resetPendingIndex(1));
    CHECK(boxes[g].appendPendingTasks(conf("a:1,b:2,c:3"), nullptr, 4));
  }
  batch->flush();  // the headers
  for (uint32_t g = 0; g < G; ++g) {
    boxes[g].commitAt(1, 3, PeerId("a", 1));
    boxes[g].commitAt(1, 2 + g % 2, PeerId("b", 2));
  }
  fake_jrq_fail_updates(1);
  CHECK(throws<std::runtime_error>([&] { batch->flush(); }));
  for (uint32_t g = 0; g < G; ++g) CHECK(boxes[g].getLastCommittedIndex() == 0);
  CHECK(batch->flush() == G);  // re-shipped in full: every group commits
  for (uint32_t g = 0; g < G; ++g) {
    CHECK(boxes[g].getLastCommittedIndex() == 2 + g % 2);
    CHECK(ws[g].calls.size() == 1 && ws[g].calls[0] == 2 + g % 2);
  }
  // and the state stays in step: a further ack commits exactly once more
  for (uint32_t g = 0; g < G; ++g) boxes[g].commitAt(3 + g % 2, 4, PeerId("b", 2));
  boxes[0].commitAt(4, 4, PeerId("a", 1));
  batch->flush();
  CHECK(boxes[0].getLastCommittedIndex() == 4);
  for (uint32_t g = 1; g < G; ++g) CHECK(boxes[g].getLastCommittedIndex() == 3);
}

// a callback that throws must not leave the other groups of the epoch half
// delivered.  Every group's commit is applied before any callback runs, the exception comes
// back from flush() after all of them ran, and the next epoch decides from the right state
// (no false commit from a stale pendingIndex).
static void testThrowingCallback(Engine& eng) {
  const uint32_t G = 64;
  auto batch = std::make_shared<GroupBatch>(&eng, G, 3);
  std::vector<BallotBox> boxes;
  std::vector<Waiter> ws(G);
  for (uint32_t g = 0; g < G; ++g) {
    boxes.emplace_back(batch, g);
    if (g == 7)
      CHECK(boxes[g].init({[](int64_t) { throw std::runtime_error("callback failed"); }}));
    else
      CHECK(boxes[g].init({ws[g].fn()}));
    CHECK(boxes[g].resetPendingIndex(1));
    CHECK(boxes[g].appendPendingTasks(conf("a:1,b:2,c:3"), nullptr, 10));
  }
  int closures = 0;
  CHECK(boxes[9].appendPendingTask(conf("a:1,b:2,c:3"), nullptr, [&](bool ok) {
    if (ok) ++closures;
    throw std::logic_error("closure failed");
  }));
  for (uint32_t g = 0; g < G; ++g) {
    boxes[g].commitAt(1, 5, PeerId("a", 1));
    boxes[g].commitAt(1, 5, PeerId("b", 2));
  }
  bool threw = false;
  try {
    batch->flush();
  } catch (const std::exception&) {
    threw = true;  // the first of the callbacks' exceptions, after all of them ran
  }
  CHECK(threw);
  for (uint32_t g = 0; g < G; ++g) {
    CHECK(boxes[g].getLastCommittedIndex() == 5);
    CHECK(boxes[g].getPendingIndex() == 6);
    if (g != 7) CHECK(ws[g].calls.size() == 1 && ws[g].calls[0] == 5);
  }
  // entry 11 of group 9 (its closure) is not committed yet: nothing popped
  CHECK(closures == 0);
  for (uint32_t g = 0; g < G; ++g) boxes[g].commitAt(6, 7, PeerId("a", 1));
  boxes[3].commitAt(6, 6, PeerId("c", 3));
  try {
    batch->flush();
  } catch (const std::exception&) {
  }
  CHECK(boxes[3].getLastCommittedIndex() == 6);
  for (uint32_t g = 0; g < G; ++g)
    if (g != 3) CHECK(boxes[g].getLastCommittedIndex() == 5);
}

// commitAt's fast path against a step-down: peer 1's ack of entries 2..15 is held inside the
// fast path (between its reads and its write, through the test hook) while another thread
// steps the leader down.  clearPendingTasks must wait for it (quiesce): otherwise, as this
// node becomes leader again with a shorter log (resetPendingIndex(10), entries 10..19 of the
// new term), the held write lands on the new leadership's slot and counts as peer 1's ack of
// entries it never received -- a commit of 10..19 with the leader's ack alone.
namespace {
std::atomic<int> g_hold{0};  // 1: the next fast-path ack parks (2 while parked) until 0
}
static void testFastPathStepDown(Engine& eng) {
  auto batch = std::make_shared<GroupBatch>(&eng, 4, 3);
  BallotBox box(batch, 2);
  box.init({[](int64_t) {}});
  Configuration c;
  for (int p = 0; p < 3; ++p) c.peers.emplace_back("10.0.0.4", 6000 + p);
  const PeerId p0("10.0.0.4", 6000), p1("10.0.0.4", 6001);
  CHECK(box.resetPendingIndex(1));
  CHECK(box.appendPendingTasks(c, nullptr, 100));
  CHECK(box.commitAt(1, 1, p1));  // peer 1's slot exists: its next ack takes the fast path
  batch->flush();
  testing::fastPathHook = [] {
    int one = 1;
    if (g_hold.compare_exchange_strong(one, 2))
      while (g_hold.load() == 2) std::this_thread::yield();
  };
  g_hold.store(1);
  std::thread acker([&] { box.commitAt(2, 15, p1); });
  while (g_hold.load() != 2) std::this_thread::yield();
  std::atomic<bool> cleared{false};
  std::thread stepDown([&] {
    box.clearPendingTasks();
    cleared.store(true);
  });
  const auto t0 = std::chrono::steady_clock::now();
  while (!cleared.load() && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(200))
    std::this_thread::yield();
  const bool waited = !cleared.load();  // the step-down waited for the held ack
  if (!waited) {  // (no quiesce) the new leadership starts while the old ack is still held
    CHECK(box.resetPendingIndex(10));
    CHECK(box.appendPendingTasks(c, nullptr, 10));
    CHECK(box.commitAt(10, 19, p0));
  }
  g_hold.store(0);
  acker.join();
  stepDown.join();
  testing::fastPathHook = nullptr;
  if (waited) {
    CHECK(box.resetPendingIndex(10));
    CHECK(box.appendPendingTasks(c, nullptr, 10));
    CHECK(box.commitAt(10, 19, p0));
  }
  batch->flush();
  CHECK(waited);
  CHECK(box.getLastCommittedIndex() == 0);  // 10..19 have the leader's ack only (a held ack
                                            // landing late would commit 10..15)
}

// a free slot is given to a peer (append names a new peer) while that peer's
// replicator acks.  The ack can find the slot on the fast path as soon as the peer id is
// published (a free slot is not quiesced), so slotOf must have written the slot's stamp and
// match before publishing, and nothing after: here the ack runs, to completion, at the instant
// the id is published (the test hook), and must survive -- c's next contiguous ack then takes
// the fast path again (its match is 4, not reset to 0), and entry 5 ({a, c}) commits.
namespace {
std::atomic<int> g_assignArm{0};
std::atomic<bool> g_assignAckDone{false};
std::function<void()> g_assignAck;
std::thread g_assignThread;
std::atomic<int> g_fastCount{0};
}  // namespace
static void testFreeSlotAckDuringAssign(Engine& eng) {
  auto batch = std::make_shared<GroupBatch>(&eng, 2, 3);
  BallotBox box(batch, 1);
  Waiter w;
  CHECK(box.init({w.fn()}));
  const PeerId a("10.0.0.5", 7000), b("10.0.0.5", 7001), c("10.0.0.5", 7002);
  CHECK(box.resetPendingIndex(1));
  CHECK(box.appendPendingTasks(conf("10.0.0.5:7000,10.0.0.5:7001"), nullptr, 4));
  CHECK(box.commitAt(1, 4, a));
  batch->flush();
  CHECK(box.getLastCommittedIndex() == 0);
  g_assignAck = [&] { box.commitAt(1, 4, c); };  // c catches up on 1..4 (no ballot counts it)
  testing::slotAssignHook = [] {
    int one = 1;
    if (!g_assignArm.compare_exchange_strong(one, 0)) return;
    g_assignThread = std::thread([] {
      g_assignAck();
      g_assignAckDone.store(true);
    });
    // the fast path takes no lock: it completes while this thread holds the group's lock
    const auto t0 = std::chrono::steady_clock::now();
    while (!g_assignAckDone.load() && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5))
      std::this_thread::yield();
  };
  g_assignArm.store(1);
  CHECK(box.appendPendingTask(conf("10.0.0.5:7000,10.0.0.5:7002"), nullptr));  // entry 5: c's slot
  testing::slotAssignHook = nullptr;
  if (g_assignThread.joinable()) g_assignThread.join();
  CHECK(g_assignAckDone.load());
  testing::fastPathHook = [] { g_fastCount.fetch_add(1); };
  CHECK(box.commitAt(5, 5, c));
  testing::fastPathHook = nullptr;
  CHECK(g_fastCount.load() == 1);  // contiguous with the kept ack of 1..4
  CHECK(box.commitAt(5, 5, a));
  CHECK(box.commitAt(1, 5, b));
  batch->flush();
  CHECK(box.getLastCommittedIndex() == 5);
  CHECK(!w.calls.empty() && w.calls.back() == 5);
}

// The append fast path reuses the group's last conf word only for the same peers in the same
// split between conf and old conf: {a,b,c} then {a,b} + old {c} is a new run (Ballot.init with
// oldQuorum 1), and entry 2 needs c's ack.
static void testConfCacheSplit(Engine& eng) {
  auto batch = std::make_shared<GroupBatch>(&eng, 1, 4);
  BallotBox box(batch, 0);
  Waiter w;
  CHECK(box.init({w.fn()}));
  CHECK(box.resetPendingIndex(1));
  Configuration abc = conf("a:1,b:2,c:3"), ab = conf("a:1,b:2"), c = conf("c:3");
  CHECK(box.appendPendingTask(abc, nullptr));
  CHECK(box.appendPendingTask(abc, nullptr));   // same conf: the cached word, no new run
  CHECK(box.appendPendingTask(ab, &c));         // same ids, another split: a new run
  CHECK(box.appendPendingTask(ab, &c));
  box.commitAt(1, 4, PeerId("a", 1));
  box.commitAt(1, 4, PeerId("b", 2));
  batch->flush();
  CHECK(box.getLastCommittedIndex() == 2);
  box.commitAt(1, 4, PeerId("c", 3));
  batch->flush();
  CHECK(box.getLastCommittedIndex() == 4);
  CHECK(w.calls.size() == 2 && w.calls[0] == 2 && w.calls[1] == 4);
}

// a thread alternating between many batches keeps one dirty list per batch.
static void testManyBatchesOneThread(Engine& eng) {
  std::vector<std::shared_ptr<GroupBatch>> batches;
  std::vector<BallotBox> boxes;
  for (int i = 0; i < 9; ++i) {
    batches.push_back(std::make_shared<GroupBatch>(&eng, 4, 3));
    for (uint32_t g = 0; g < 4; ++g) {
      boxes.emplace_back(batches.back(), g);
      Waiter w;
      CHECK(boxes.back().init({[](int64_t) {}}));
      CHECK(boxes.back().resetPendingIndex(1));
    }
  }
  for (int round = 0; round < 50; ++round)
    for (auto& b : boxes) CHECK(b.appendPendingTasks(conf("a:1,b:2,c:3"), nullptr, 1));
  for (auto& b : batches) CHECK(b->dirtyLists() == 1);
}

// ------------------------------------------------ follower / reader / leader tick

// NodeImpl.handleAppendEntriesRequest's verify loop through FollowerVerifier (one GPU batch of
// requests) against the oracle's loop: DATA entries of ragged sizes, UNKNOWN metas that consume
// no data, a CONFIGURATION entry with peers, some stored checksums corrupted.
static void testFollowerVerifierOnGpu(Engine& eng) {
  std::mt19937_64 rng(41);
  std::vector<AppendEntriesRequest> reqs(40);
  const PeerId pa("10.1.1.1", 8081), pb("10.1.1.2", 8082, 1);
  const uint64_t pxab = jo_peerid_checksum("10.1.1.1", 8081, 0) ^ jo_peerid_checksum("10.1.1.2", 8082, 1);
  std::vector<uint32_t> reqOff(1, 0);
  std::vector<int64_t> prev, term, dlen;
  std::vector<uint8_t> type, has, data;
  std::vector<uint64_t> px, stored;
  for (size_t r = 0; r < reqs.size(); ++r) {
    AppendEntriesRequest& q = reqs[r];
    q.prevLogIndex = 1000 * static_cast<int64_t>(r);
    const int n = static_cast<int>(rng() % 12);
    for (int k = 0; k < n; ++k) {
      LogEntry e;
      const int kind = static_cast<int>(rng() % 10);
      e.type = kind == 0 ? EntryType::UNKNOWN : kind == 1 ? EntryType::CONFIGURATION : EntryType::DATA;
      e.id = LogId{q.prevLogIndex + 1 + k, 3};
      const int64_t len = e.type == EntryType::UNKNOWN ? 0 : static_cast<int64_t>(rng() % 3000);
      std::vector<uint8_t> bytes(static_cast<size_t>(len));
      for (auto& b : bytes) b = static_cast<uint8_t>(rng());
      uint64_t pxe = 0;
      if (e.type == EntryType::CONFIGURATION) {
        e.peers = {pa, pb};
        pxe = pxab;
      }
      uint64_t c = jo_logentry_checksum(static_cast<int32_t>(e.type), e.id.index, e.id.term, pxe,
                                        bytes.data(), bytes.size());
      if (rng() % 7 == 0) c ^= 1;  // corrupted in transit
      if (rng() % 9 != 0) e.setChecksum(c);  // some metas carry no checksum
      q.entries.push_back(e);
      q.dataLen.push_back(len);
      q.data.insert(q.data.end(), bytes.begin(), bytes.end());
      term.push_back(e.id.term);
      type.push_back(static_cast<uint8_t>(e.type));
      dlen.push_back(len);
      px.push_back(pxe);
      stored.push_back(e.getChecksum());
      has.push_back(e.hasChecksum());
    }
    prev.push_back(q.prevLogIndex);
    reqOff.push_back(reqOff.back() + static_cast<uint32_t>(n));
    data.insert(data.end(), q.data.begin(), q.data.end());
  }
  std::vector<const AppendEntriesRequest*> rp;
  for (auto& q : reqs) rp.push_back(&q);
  FollowerVerifier fv(eng);
  std::vector<uint64_t> sums;
  const auto first = fv.verify(rp, &sums);
  const uint32_t N = reqOff.back();
  std::vector<uint64_t> esum(N);
  std::vector<uint8_t> ecor(N);
  std::vector<int32_t> efirst(reqs.size());
  if (data.empty()) data.push_back(0);
  jo_append_entries_verify(static_cast<uint32_t>(reqs.size()), reqOff.data(), prev.data(), term.data(),
                           type.data(), dlen.data(), px.data(), stored.data(), has.data(), data.data(),
                           esum.data(), ecor.data(), efirst.data());
  CHECK(first == efirst);
  CHECK(sums == esum);
  int corrupt_requests = 0;
  for (auto f : first) corrupt_requests += f >= 0;
  CHECK(corrupt_requests > 3);
}

// LogManagerImpl's read path through LogReader: V2 records as V2Encoder writes them
// (header, type 1, term 2, index 3, data 6, checksum 7), one corrupted, one truncated
// (undecodable), one empty (the reference's null).
static void testLogReaderOnGpu(Engine& eng) {
  auto varint = [](std::vector<uint8_t>& o, uint64_t v) {
    while (v >= 0x80) {
      o.push_back(static_cast<uint8_t>(v | 0x80));
      v >>= 7;
    }
    o.push_back(static_cast<uint8_t>(v));
  };
  std::mt19937_64 rng(43);
  std::vector<std::vector<uint8_t>> recs;
  std::vector<uint64_t> sums;
  for (int i = 0; i < 300; ++i) {
    std::vector<uint8_t> data(static_cast<size_t>(rng() % 5000));
    for (auto& b : data) b = static_cast<uint8_t>(rng());
    const int64_t index = 100 + i, term = 7;
    uint64_t c = jo_logentry_checksum(2, index, term, 0, data.data(), data.size());
    sums.push_back(c);
    if (i == 17) c ^= 0x10;  // corrupted
    std::vector<uint8_t> r = {0xBB, 0xD2, 0x01, 0, 0, 0};
    r.push_back(0x08); varint(r, 2);
    r.push_back(0x10); varint(r, static_cast<uint64_t>(term));
    r.push_back(0x18); varint(r, static_cast<uint64_t>(index));
    r.push_back(0x32); varint(r, data.size());
    r.insert(r.end(), data.begin(), data.end());
    r.push_back(0x38); varint(r, c);
    if (i == 23) r.resize(r.size() - 3);  // truncated checksum varint
    if (i == 29) r.clear();               // no bytes: the reference's null
    recs.push_back(std::move(r));
  }
  LogReader rd(eng);
  const auto out = rd.decode(recs);
  CHECK(out.size() == recs.size());
  for (int i = 0; i < 300; ++i) {
    if (i == 23 || i == 29) {
      CHECK(out[i].status != JRQ_V2_OK);
      continue;
    }
    CHECK(out[i].status == JRQ_V2_OK);
    CHECK(out[i].entry.type == EntryType::DATA && out[i].entry.id.index == 100 + i && out[i].entry.id.term == 7);
    CHECK(out[i].corrupt == (i == 17));
    CHECK(out[i].entry.hasChecksum() && (i == 17 || out[i].entry.getChecksum() == sums[i]));
    CHECK(out[i].entry.checksum(eng) == sums[i]);  // the decoded bytes hash to the original
  }
}

// Lease checks and ReadIndex rounds of many leader groups through LeaderTicker (one device
// pass per tick) against the oracle's checkDeadNodes and closure replay on the same inputs.
static void testLeaderTickerOnGpu(Engine& eng) {
  const uint32_t G = 600, P = 5;
  LeaderTicker lt(eng, G, P);
  std::mt19937_64 rng(47);
  std::vector<PeerId> ps;
  for (uint32_t p = 0; p < 7; ++p) ps.emplace_back("10.2.0.1", static_cast<int32_t>(7000 + p));
  const int64_t t0 = 1000000, lease = 900;
  struct Exp { std::vector<int32_t> nids, oids; int32_t self; std::vector<int64_t> ts; std::vector<int> order; uint32_t okm = 0; };
  std::vector<Exp> ex(G);
  std::vector<int> verdict(G, -1);  // callback results: -1 none yet, 0 false, 1 true
  for (uint32_t g = 0; g < G; ++g) {
    Configuration c, o;
    const uint32_t n = rng() % 2 ? 3 : 5;
    for (uint32_t p = 0; p < n; ++p) c.peers.push_back(ps[p]);
    const bool joint = g % 5 == 0;
    if (joint) o.peers = {ps[0], ps[1], ps[2]};
    lt.becomeLeader(g, c, joint ? &o : nullptr, ps[0], t0);
    Exp& e = ex[g];
    for (uint32_t p = 0; p < n; ++p) e.nids.push_back(static_cast<int32_t>(p));
    if (joint) e.oids = {0, 1, 2};
    e.self = 0;
    e.ts.assign(P, t0);
    for (uint32_t p = 1; p < n; ++p) {
      const int64_t t = t0 + 2000 - static_cast<int64_t>(rng() % 2000);
      lt.onRpcSent(g, ps[p], t);
      e.ts[p] = t;
    }
    if (g % 3 == 0) {  // a ReadIndex round with some responses in a random order
      lt.readIndex(g, [&verdict, g](bool ok) { verdict[g] = ok ? 1 : 0; });
      const uint64_t round = lt.startReadRound(g);
      CHECK(round != 0);
      std::vector<int> peers;
      for (uint32_t p = 1; p < n; ++p) if (rng() % 4) peers.push_back(static_cast<int>(p));
      std::shuffle(peers.begin(), peers.end(), rng);
      for (int p : peers) {
        const bool okr = rng() % 10 < 6;
        lt.onHeartbeatResponse(g, round, ps[p], okr);
        e.order.push_back(p);
        if (okr) e.okm |= 1u << p;
      }
    }
  }
  std::vector<std::pair<uint32_t, uint16_t>> downs;
  const int64_t now = t0 + 2000;
  lt.tick(now, lease, [&](uint32_t g, uint16_t dead) { downs.emplace_back(g, dead); });
  std::set<uint32_t> down;
  for (auto& d : downs) down.insert(d.first);
  for (uint32_t g = 0; g < G; ++g) {
    const Exp& e = ex[g];
    int64_t start = t0;
    uint32_t dm = 0;
    bool okn = jo_check_dead_nodes(e.nids.data(), static_cast<int32_t>(e.nids.size()), e.ts.data(), e.self, now, lease, &start, &dm);
    bool oko = e.oids.empty() || jo_check_dead_nodes(e.oids.data(), static_cast<int32_t>(e.oids.size()), e.ts.data(), e.self, now, lease, &start, &dm);
    const bool stepped = !(okn && oko);
    CHECK(stepped == (down.count(g) != 0));
    CHECK(lt.isLeader(g) == !stepped);
    if (!stepped) CHECK(lt.lastLeaderTimestamp(g) == start);
    if (g % 3 == 0) {
      uint64_t order = 0;
      for (size_t k = 0; k < e.order.size(); ++k) order |= static_cast<uint64_t>(k + 1) << (4 * e.order[k]);
      uint32_t mask = 0;
      for (int32_t p : e.nids) mask |= 1u << p;
      const uint8_t r = jo_readindex_round(mask, P, 0, order, e.okm);
      const int want = r == 1 ? 1 : r == 2 ? 0 : (stepped ? 0 : -1);
      CHECK(verdict[g] == want);
    } else {
      CHECK(verdict[g] == -1);
    }
  }
  CHECK(!downs.empty() && downs.size() < G);
  // a second tick: the stepped-down groups are not checked again, the rest keep their lease
  const size_t before = downs.size();
  lt.tick(now, lease, [&](uint32_t g, uint16_t dead) { downs.emplace_back(g, dead); });
  CHECK(downs.size() == before);
}

// every response that confirms a read left its peer after the read arrived,
// as in the reference, where each readLeader call sends its own heartbeat round
// (NodeImpl.java:1386-1394).  A read arriving after its group's round was sent waits for the
// next round; a late response of a decided round never counts toward the next one; a
// single-voter group answers at once (readLeader's quorum <= 1 fast path, :1345-1352).
static void testReadIndexRounds(Engine& eng) {
  const uint32_t G = 4, P = 5;
  LeaderTicker lt(eng, G, P);
  std::vector<PeerId> ps;
  for (uint32_t p = 0; p < 5; ++p) ps.emplace_back("10.3.0.1", static_cast<int32_t>(7100 + p));
  Configuration c5, c1;
  c5.peers.assign(ps.begin(), ps.end());  // quorum 3: the leader + 2 successes
  c1.peers = {ps[0]};
  const int64_t t0 = 1000;
  for (uint32_t g = 0; g < 3; ++g) lt.becomeLeader(g, c5, nullptr, ps[0], t0);
  lt.becomeLeader(3, c1, nullptr, ps[0], t0);
  auto tick = [&] { lt.tick(t0 + 10, 1000, nullptr); };
  // (a) a read joining mid-round waits for the next round
  int first = -1, late = -1;
  lt.readIndex(0, [&](bool ok) { first = ok; });
  const uint64_t r1 = lt.startReadRound(0);
  CHECK(r1 != 0 && lt.startReadRound(0) == 0);  // one round open at a time
  lt.onHeartbeatResponse(0, r1, ps[1], true);
  lt.readIndex(0, [&](bool ok) { late = ok; });  // after r1 was sent and answered once
  lt.onHeartbeatResponse(0, r1, ps[2], true);
  tick();
  CHECK(first == 1 && late == -1);  // r1's responses confirm only the read sent with r1
  const uint64_t r2 = lt.startReadRound(0);
  CHECK(r2 != 0 && r2 != r1);
  tick();
  CHECK(late == -1);  // no response of r2 yet
  lt.onHeartbeatResponse(0, r2, ps[3], true);
  lt.onHeartbeatResponse(0, r2, ps[4], true);
  tick();
  CHECK(late == 1);
  // (b) a late response of a decided round is dropped
  int a = -1, b = -1;
  lt.readIndex(1, [&](bool ok) { a = ok; });
  const uint64_t q1 = lt.startReadRound(1);
  lt.onHeartbeatResponse(1, q1, ps[1], true);
  lt.onHeartbeatResponse(1, q1, ps[2], true);
  tick();
  CHECK(a == 1);
  lt.readIndex(1, [&](bool ok) { b = ok; });
  const uint64_t q2 = lt.startReadRound(1);
  lt.onHeartbeatResponse(1, q1, ps[3], true);  // stale: q1 is decided
  lt.onHeartbeatResponse(1, q1, ps[4], true);
  lt.onHeartbeatResponse(1, q2, ps[1], true);  // one success of q2 only: not a quorum
  tick();
  CHECK(b == -1);
  lt.onHeartbeatResponse(1, q2, ps[2], false);
  lt.onHeartbeatResponse(1, q2, ps[3], false);
  lt.onHeartbeatResponse(1, q2, ps[4], false);
  tick();
  CHECK(b == 0);  // q2 failed: 3 failures >= failPeersThreshold 3
  // (c) a step-down fails the open round and the queued reads
  int o = -1, w = -1;
  lt.readIndex(2, [&](bool ok) { o = ok; });
  const uint64_t s1 = lt.startReadRound(2);
  lt.readIndex(2, [&](bool ok) { w = ok; });
  lt.stepDown(2);
  CHECK(o == 0 && w == 0);
  lt.onHeartbeatResponse(2, s1, ps[1], true);  // after the step-down: ignored
  int x = -1;
  lt.readIndex(2, [&](bool ok) { x = ok; });
  CHECK(x == 0 && lt.startReadRound(2) == 0);
  // (d) quorum <= 1: at once, no round
  int one = -1;
  lt.readIndex(3, [&](bool ok) { one = ok; });
  CHECK(one == 1 && lt.startReadRound(3) == 0);
}

// FSMCallerImpl.doCommitted for many groups through FSMCallerBatch (one jrq_commit_fanout per
// pass) against the oracle's call-by-call ClosureQueue / doCommitted replay: groups whose
// commit did not move (or only a stale one arrived), commits below the queue's first index (no
// closure popped), commits beyond the queue (INVALID), and ordinary pops.
static void testFSMCallerBatchOnGpu(Engine& eng) {
  const uint32_t G = 700;
  FSMCallerBatch fc(eng, G);
  std::mt19937_64 rng(53);
  std::vector<int64_t> first(G), size(G), la(G), prev(G), com(G);
  std::vector<std::vector<int>> ran(G);  // closure results per group, in run order
  for (uint32_t g = 0; g < G; ++g) {
    la[g] = 100 + static_cast<int64_t>(rng() % 50);
    fc.setLastApplied(g, la[g]);
    prev[g] = la[g];
    first[g] = la[g] + 1 + static_cast<int64_t>(rng() % 3);
    size[g] = static_cast<int64_t>(rng() % 20);
    fc.resetFirstIndex(g, first[g]);
    for (int64_t k = 0; k < size[g]; ++k)
      fc.appendPendingClosure(g, [&ran, g, k](bool ok) { ran[g].push_back(ok ? static_cast<int>(k) : -1); });
    const int kind = static_cast<int>(rng() % 6);
    com[g] = kind == 0 ? prev[g]                                   // no commit
             : kind == 1 ? la[g] - 1                              // stale: no onCommitted
             : kind == 2 ? first[g] + size[g] + 5                 // beyond the queue: INVALID
                         : first[g] + static_cast<int64_t>(rng() % (size[g] + 1));  // ordinary
    if (com[g] > prev[g]) fc.onCommitted(g, com[g]);
  }
  std::vector<int> applied(G, 0), invalid(G, 0);
  std::vector<std::pair<int64_t, int64_t>> range(G);
  fc.doCommitted(
      [&](uint32_t g, int64_t a, int64_t b, std::vector<std::function<void(bool)>>& done) {
        applied[g] = 1;
        range[g] = {a, b};
        for (auto& d : done) d(true);
      },
      [&](uint32_t g) { invalid[g] = 1; });
  // the oracle: one onCommitted per moved group, replayed call by call
  std::vector<uint64_t> off(G + 1, 0);
  std::vector<int64_t> seq;
  for (uint32_t g = 0; g < G; ++g) {
    if (com[g] > prev[g]) seq.push_back(com[g]);
    off[g + 1] = seq.size();
  }
  std::vector<int64_t> ola = la, ofirst = first, osize = size, ofc(G);
  std::vector<uint8_t> ost(G);
  jo_commit_fanout_replay(G, off.data(), seq.data(), ola.data(), ofirst.data(), osize.data(), ofc.data(), ost.data());
  int napply = 0, ninvalid = 0;
  for (uint32_t g = 0; g < G; ++g) {
    CHECK(applied[g] == (ost[g] == JRQ_FAN_APPLY));
    CHECK(invalid[g] == (ost[g] == JRQ_FAN_INVALID));
    napply += applied[g];
    ninvalid += invalid[g];
    const int64_t popped = size[g] - osize[g];
    CHECK(static_cast<int64_t>(ran[g].size()) == popped);
    for (int64_t k = 0; k < popped; ++k) CHECK(ran[g][static_cast<size_t>(k)] == static_cast<int>(k));
    if (applied[g]) {
      CHECK(range[g].first == la[g] + 1 && range[g].second == com[g]);
      CHECK(fc.lastApplied(g) == ola[g]);
    }
  }
  CHECK(napply > 100 && ninvalid > 20);
}

int main(int argc, char** argv) {
  // "gpu": with an engine (the real libjrq.so on the GPU box; the sanitizer builds link the
  // test double tests/cpp/fake_jrq.cpp instead and run the same list on the CPU)
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
      {"testAckFromPeerWithoutSlot", testAckFromPeerWithoutSlot},
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
    tests.push_back({"testConcurrentCallers", [&] { testConcurrentCallers(e, 384, 400); }});
    // > 8192 changed groups per epoch: flush() packs and delivers on several threads
    tests.push_back({"testConcurrentCallersWide", [&] { testConcurrentCallers(e, 20000, 48); }});
    // the same with the record chunks streamed every 37 records (jrq_table_ack_push from the
    // calling threads while others call, flush and push tails)
    tests.push_back({"testConcurrentCallersStreamed", [&] {
                       testing::ackChunkRecords.store(37);
                       try {
                         testConcurrentCallers(e, 2000, 120);
                       } catch (...) {
                         testing::ackChunkRecords.store(GroupBatch::kAckChunk);
                         throw;
                       }
                       testing::ackChunkRecords.store(GroupBatch::kAckChunk);
                     }});
    tests.push_back({"testReentrantFlushRefused", [&] { testReentrantFlushRefused(e); }});
    tests.push_back({"testFlushFailureRelists", [&] { testFlushFailureRelists(e); }});
    tests.push_back({"testThrowingCallback", [&] { testThrowingCallback(e); }});
    tests.push_back({"testManyBatchesOneThread", [&] { testManyBatchesOneThread(e); }});
    tests.push_back({"testConfCacheSplit", [&] { testConfCacheSplit(e); }});
    tests.push_back({"testFastPathStepDown", [&] { testFastPathStepDown(e); }});
    tests.push_back({"testFreeSlotAckDuringAssign", [&] { testFreeSlotAckDuringAssign(e); }});
    tests.push_back({"testFollowerVerifierOnGpu", [&] { testFollowerVerifierOnGpu(e); }});
    tests.push_back({"testLogReaderOnGpu", [&] { testLogReaderOnGpu(e); }});
    tests.push_back({"testLeaderTickerOnGpu", [&] { testLeaderTickerOnGpu(e); }});
    tests.push_back({"testReadIndexRounds", [&] { testReadIndexRounds(e); }});
    tests.push_back({"testResetStampKeepsLiveAcks", [&] { testResetStampKeepsLiveAcks(e); }});
    tests.push_back({"testShardedBatchOnGpu", [&] { testShardedBatchOnGpu(e); }});
    tests.push_back({"testFSMCallerBatchOnGpu", [&] { testFSMCallerBatchOnGpu(e); }});
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
