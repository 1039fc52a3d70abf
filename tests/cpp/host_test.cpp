// host_test.cpp -- the reference's hot-path unit tests, re-expressed against the C++ host
// mirror (sofa-jraft_amd/host) over libjrq.so.  Run by tests/test_host_cpp.py:
//   host_test cpu   -> tests that need no GPU (synchronous BallotBox semantics)
//   host_test gpu   -> everything, decisions and checksums computed on the GPU
// Sources restated (jraft-core/src/test/java/com/alipay/sofa/jraft/...):
//   core/BallotBoxTest.java:62-154, entity/BallotTest.java:37-50,
//   entity/LogEntryTest.java:95-125, util/CrcUtilTest.java:27-42
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

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
