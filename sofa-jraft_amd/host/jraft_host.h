// jraft_host.h -- C++ host-side mirror of SOFAJRaft's hot-path API over libjrq.so.
//
// The reference host is Java (JDK absent in this image, SURVEY.md env probes), so the
// host side above the C ABI is written in C++ with the reference's class and method
// names, argument meaning and error behaviour:
//   jraft::BallotBox  <- jraft-core/.../core/BallotBox.java (commitAt, appendPendingTask,
//                        resetPendingIndex, setLastCommittedIndex, clearPendingTasks,
//                        getLastCommittedIndex, describe, shutdown)
//   jraft::LogEntry   <- jraft-core/.../entity/LogEntry.java (checksum, isCorrupted, setChecksum)
//   jraft::CrcUtil    <- jraft-core/.../util/CrcUtil.java (crc64 of byte ranges)
//   jraft::PeerId / Configuration (peers only; learners never vote, Configuration.java:184-186)
// Exceptions mirror the Java ones: std::out_of_range for ArrayIndexOutOfBoundsException,
// std::invalid_argument for IllegalArgumentException (Requires.requireTrue).
//
// Every checksum and every quorum decision is computed by libjrq.so on the GPU.  The
// BallotBox objects of many groups share one GroupBatch, whose state lives in a resident
// device table (jrq_table); acks are recorded at call time (with the reference's synchronous
// checks), only the changes are uploaded, and flush() decides an epoch on the GPU, after
// which the FSMCaller waiter sees onCommitted(index) exactly as the reference calls it.
#pragma once

#include <atomic>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/jrq.h"

namespace jraft {

// ------------------------------------------------------------------ entities

// Immutable once built, as the reference's PeerId is in use (its fields are private and only
// parse() sets them, PeerId.java:150-170): the interned id cached in it then never goes stale,
// and a BallotBox call resolves its peer with one load.
class PeerId {
  std::string ip_;
  int32_t port_ = 0;
  int32_t idx_ = 0;

 public:
  PeerId() = default;
  PeerId(std::string ip, int32_t port, int32_t idx = 0) : ip_(std::move(ip)), port_(port), idx_(idx) {}
  PeerId(const PeerId& o) : ip_(o.ip_), port_(o.port_), idx_(o.idx_), internId(o.internId.load(std::memory_order_relaxed)) {}
  PeerId(PeerId&& o) noexcept
      : ip_(std::move(o.ip_)), port_(o.port_), idx_(o.idx_), internId(o.internId.load(std::memory_order_relaxed)) {}
  PeerId& operator=(const PeerId& o) {
    ip_ = o.ip_;
    port_ = o.port_;
    idx_ = o.idx_;
    internId.store(o.internId.load(std::memory_order_relaxed), std::memory_order_relaxed);
    return *this;
  }
  const std::string& getIp() const { return ip_; }
  int32_t getPort() const { return port_; }
  int32_t getIdx() const { return idx_; }
  // PeerId.toString (PeerId.java:135-144): ip:port[:idx]
  std::string toString() const;
  // PeerId.parse (PeerId.java:150-170): "ip:port" or "ip:port:idx"; resets the interned id
  static bool parse(const std::string& s, PeerId* out);
  bool operator==(const PeerId& o) const { return ip_ == o.ip_ && port_ == o.port_ && idx_ == o.idx_; }
  bool operator<(const PeerId& o) const {
    return ip_ != o.ip_ ? ip_ < o.ip_ : (port_ != o.port_ ? port_ < o.port_ : idx_ < o.idx_);
  }
  // The process-wide id of this peer (0 = not looked up yet), like the hash a Java String
  // caches; written with atomics, so one PeerId may be shared by threads.
  mutable std::atomic<uint32_t> internId{0};
};

struct Configuration {
  std::vector<PeerId> peers;     // voting members, in order (duplicates kept, as ArrayList)
  std::vector<PeerId> learners;  // never vote
  // Configuration.parse (Configuration.java:285-311): "a:1,b:2,c:3/learner"
  static Configuration parse(const std::string& s);
  bool isEmpty() const { return peers.empty(); }
  bool operator==(const Configuration& o) const { return peers == o.peers && learners == o.learners; }
};

enum class EntryType : int32_t { UNKNOWN = 0, NO_OP = 1, DATA = 2, CONFIGURATION = 3 };

struct LogId {
  int64_t index = 0;
  int64_t term = 0;
};

class Engine;  // owns one jrq_engine

// LogEntry (LogEntry.java): checksum fields; data is a byte range owned by the entry.
struct LogEntry {
  EntryType type = EntryType::UNKNOWN;
  LogId id;
  std::vector<PeerId> peers, oldPeers, learners, oldLearners;
  std::vector<uint8_t> data;
  bool hasChecksum_ = false;
  uint64_t checksum_ = 0;

  uint64_t checksum(Engine& eng) const;          // LogEntry.checksum (:88-99), on the GPU
  bool isCorrupted(Engine& eng) const;           // :156-158
  void setChecksum(uint64_t c) { checksum_ = c; hasChecksum_ = true; }  // :169-172
  bool hasChecksum() const { return hasChecksum_; }                    // :147-149
  uint64_t getChecksum() const { return checksum_; }
};

// ------------------------------------------------------------------- engine

class Engine {
 public:
  explicit Engine(int device = 0, uint32_t max_groups = 1u << 20, uint8_t max_peers = 16);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;
  jrq_engine* raw() { return e_; }

  // CrcUtil.crc64 over many byte ranges at once (CrcUtil.java:36-80): one GPU batch.
  std::vector<uint64_t> crc64(const std::vector<std::vector<uint8_t>>& items);
  // LogEntry.checksum for a batch (LogEntry.java:88-108); PeerId checksums of every
  // distinct peer are computed in the same style (GPU CRC batch of the peer strings).
  std::vector<uint64_t> checksum(const std::vector<const LogEntry*>& entries);
  // isCorrupted for a batch: hasChecksum && stored != checksum() (:156-158).
  std::vector<uint8_t> verify(const std::vector<const LogEntry*>& entries);
  // Per entry, the XOR of the PeerId.checksum() of its peers, oldPeers, learners and
  // oldLearners (LogEntry.java:101-108): one GPU CRC batch over the distinct peer strings.
  std::vector<uint64_t> peerChecksums(const std::vector<const LogEntry*>& entries);

 private:
  uint64_t peerXor(const LogEntry& e, std::map<std::string, uint64_t>& cache);
  jrq_engine* e_ = nullptr;
};

class CrcUtil {
 public:
  // CrcUtil.crc64(byte[]) / (byte[], off, len) (CrcUtil.java:36-57); null -> 0.
  static uint64_t crc64(Engine& eng, const uint8_t* array, size_t offset, size_t length);
  static uint64_t crc64(Engine& eng, const std::vector<uint8_t>& array) {
    return crc64(eng, array.data(), 0, array.size());
  }
};

// CRC64 implements java.util.zip.Checksum (CRC64.java:26,100-126), the checksum RheaKV
// wraps around snapshot archives (AbstractKVStoreSnapshotFile.java:121-123,139-143 via
// CheckedOutputStream/CheckedInputStream in ZipUtil.java:45-94).  Bytes are buffered on the
// host (as the BufferedOutputStream in front of the checked stream does) and folded into
// the register on the GPU by jrq_crc64_stream_update in chunks of up to flushBytes.
class CRC64 {
 public:
  explicit CRC64(Engine& eng, size_t flushBytes = 64u << 20) : eng_(&eng), flush_(flushBytes) {}
  void update(int b) { buf_.push_back(static_cast<uint8_t>(b)); maybeFlush(); }  // :100-103
  void update(const uint8_t* b, size_t off, size_t len);                        // :106-110
  uint64_t getValue();                                                          // :119-121
  void reset() { buf_.clear(); crc_ = 0; }                                      // :124-126

 private:
  void maybeFlush() { if (buf_.size() >= flush_) flush(); }
  void flush();
  Engine* eng_;
  size_t flush_;
  uint64_t crc_ = 0;
  std::vector<uint8_t> buf_;
};

// -------------------------------------------------------- follower / reader

// One AppendEntriesRequest as the follower receives it (rpc.proto AppendEntriesRequest /
// raft.proto EntryMeta): the EntryMetas and the request's data, every entry's bytes back to
// back (an ENTRY_TYPE_UNKNOWN meta consumes none, NodeImpl.java:1809-1823).
struct AppendEntriesRequest {
  int64_t prevLogIndex = 0;
  std::vector<LogEntry> entries;  // meta fields; entries[i].data left empty (the bytes are in data)
  std::vector<int64_t> dataLen;   // EntryMeta.data_len per entry
  std::vector<uint8_t> data;
};

// NodeImpl.handleAppendEntriesRequest's per-entry isCorrupted loop (NodeImpl.java:1766-1792)
// for a batch of requests at once (jrq_append_entries_verify): per request the position of its
// first corrupt entry -- the one the reference answers with EINVAL -- or -1.
class FollowerVerifier {
 public:
  explicit FollowerVerifier(Engine& eng) : eng_(&eng) {}
  std::vector<int32_t> verify(const std::vector<const AppendEntriesRequest*>& reqs,
                              std::vector<uint64_t>* checksums = nullptr);

 private:
  Engine* eng_;
};

// LogManagerImpl's read path (getEntry -> AutoDetectDecoder.decode -> isCorrupted,
// LogManagerImpl.java:733-745) for a batch of stored V2 records (jrq_v2_decode_verify).
struct DecodedEntry {
  uint8_t status = 0;     // JRQ_V2_OK / _NULL (the reference's null) / _V1 / _HOST (decode on the host)
  LogEntry entry;         // type, id, stored checksum, data (peers: decode on the host when needed)
  uint32_t peerCount = 0; // peers + oldPeers + learners + oldLearners in the record
  bool corrupt = false;   // isCorrupted(): LogEntryCorruptedException / RaftError.EIO
};
class LogReader {
 public:
  explicit LogReader(Engine& eng) : eng_(&eng) {}
  std::vector<DecodedEntry> decode(const std::vector<std::vector<uint8_t>>& records);

 private:
  Engine* eng_;
};

// --------------------------------------------------------------- FSM caller

// The FSMCaller side of many groups (FSMCallerImpl.onCommitted / doCommitted, FSMCallerImpl.
// java:239-244, 462-482, with each group's ClosureQueueImpl, ClosureQueueImpl.java:83-142): the
// commits of an epoch are gated and their closures popped for every group by one device pass
// (jrq_commit_fanout); the host then runs, per applying group, the popped closures and the
// state machine over (lastApplied, committed].  A BallotBox's waiter feeds onCommitted.
class FSMCallerBatch {
 public:
  // onApply(group, firstIndex, lastIndex, closures popped for [firstClosure, lastIndex])
  using Apply = std::function<void(uint32_t group, int64_t first, int64_t last,
                                   std::vector<std::function<void(bool)>>& closures)>;
  FSMCallerBatch(Engine& eng, uint32_t groups);
  // ClosureQueueImpl.resetFirstIndex (:83-92) when the node becomes leader; appendPendingClosure
  // (:95-105) for each entry it appends (BallotBox.appendPendingTask)
  void resetFirstIndex(uint32_t g, int64_t firstIndex);
  void appendPendingClosure(uint32_t g, std::function<void(bool)> done);
  void setLastApplied(uint32_t g, int64_t lastApplied);  // after loading a snapshot / at start
  // FSMCallerImpl.onCommitted: the epoch's commit of the group (the largest one wins)
  void onCommitted(uint32_t g, int64_t committedIndex);
  // One doCommitted pass over every group with a new commit; returns the groups applied.
  // onInvalid(g): popClosureUntil returned -1 ("Invalid firstClosureIndex").
  uint32_t doCommitted(const Apply& onApply, const std::function<void(uint32_t)>& onInvalid = {});
  int64_t lastApplied(uint32_t g) const { return lastApplied_[g]; }

 private:
  Engine* eng_;
  uint32_t G_;
  std::mutex mu_;
  std::vector<int64_t> prev_, committed_, lastApplied_, cqFirst_, cqSize_;
  std::vector<std::deque<std::function<void(bool)>>> closures_;
};

// ------------------------------------------------------------- leader tick

// The leader-side timers of many Raft groups, decided for all of them by one device pass
// (jrq_leader_tick): NodeImpl.handleStepDownTimeout -> checkDeadNodes (NodeImpl.java:
// 1970-2016: is a quorum of the conf -- and of the old conf -- alive, by each peer's
// lastRpcSendTimestamp; the lease start moves to the oldest alive one) and the ReadOnlySafe
// heartbeat round of readLeader (:1343-1396, ReadIndexHeartbeatResponseClosure :1246-1291).
// Per group a slot per distinct peer of conf + old conf (<= peers), its timestamps and the open
// ReadIndex round's responses in arrival order.  Calls lock the ticker (one mutex): the
// per-RPC call is a few stores.
class LeaderTicker {
 public:
  using StepDown = std::function<void(uint32_t group, uint16_t deadSlots)>;
  LeaderTicker(Engine& eng, uint32_t groups, uint32_t peers);
  // becomeLeader: the group's conf (and old conf while joint), the leader's own peer, the
  // lease start (lastLeaderTimestamp); every peer's timestamp starts at nowMs
  void becomeLeader(uint32_t g, const Configuration& conf, const Configuration* oldConf,
                    const PeerId& self, int64_t nowMs);
  void stepDown(uint32_t g);  // not checked any more; an open ReadIndex round fails
  // Replicator: an RPC to `peer` left (its lastRpcSendTimestamp)
  void onRpcSent(uint32_t g, const PeerId& peer, int64_t nowMs);
  // readLeader, ReadOnlySafe (NodeImpl.java:1343-1396): queue a read for the group's NEXT
  // heartbeat round; done runs once with that round's verdict (true: the read index may be
  // served).  A conf whose quorum is <= 1 answers true at once (readLeader's fast path,
  // :1345-1352); a group that is not the leader answers false at once.  A read never joins a
  // round whose heartbeats were already sent: every response that confirms it left its peer
  // after the read arrived (the reference sends a fresh round per readLeader call, :1386-1394).
  void readIndex(uint32_t g, std::function<void(bool)> done);
  // Open the group's next round if reads are queued and no round is open: the queued reads
  // become the round's, and the returned id (nonzero, unique per ticker) tags the heartbeats
  // the host now sends to every conf peer but the leader.  0: nothing to send now.  A host
  // calls it after readIndex and after every tick (a decided round leaves the next one to open).
  uint64_t startReadRound(uint32_t g);
  // A heartbeat response (success = response.getSuccess()) carrying the round id its request
  // was sent with.  Responses of any other round -- one already decided, or a stale retry --
  // are dropped, so a late response never counts toward a later round.
  void onHeartbeatResponse(uint32_t g, uint64_t round, const PeerId& peer, bool success);
  // One pass over every leader group: groups without an alive quorum call stepDown (then
  // stop being checked), decided ReadIndex rounds run their closures.  Returns the groups
  // that failed the lease check.
  uint32_t tick(int64_t nowMs, int64_t leaseTimeoutMs, const StepDown& onStepDown);
  int64_t lastLeaderTimestamp(uint32_t g) const;
  bool isLeader(uint32_t g) const;

 private:
  int slot(uint32_t g, const PeerId& peer) const;
  void closeRound(uint32_t g, std::vector<std::function<void(bool)>>& out);
  Engine* eng_;
  uint32_t G_, P_;
  mutable std::mutex mu_;
  std::vector<int64_t> ts_;          // [P][G] lastRpcSendTimestamp per slot
  std::vector<uint64_t> conf_;       // [G] JRQ_CONF word of the slots (0: not a leader)
  std::vector<uint8_t> self_;        // [G] the leader's slot
  std::vector<int64_t> lease_;       // [G] lastLeaderTimestamp
  std::vector<uint64_t> order_;      // [G] arrival positions of the open round's responses
  std::vector<uint16_t> okMask_;     // [G]
  std::vector<uint8_t> arrivals_;    // [G] responses in the open round so far
  std::vector<std::vector<uint32_t>> peers_;  // [G] interned peer of each slot
  std::vector<std::vector<std::function<void(bool)>>> reads_;    // [G] open round's closures
  std::vector<std::vector<std::function<void(bool)>>> waiting_;  // [G] reads for the next round
  std::vector<uint64_t> round_;      // [G] id of the open round (0: none)
  uint64_t roundSeq_ = 0;            // last round id handed out
};

// --------------------------------------------------------------- ballot box

// FSMCaller.onCommitted (FSMCallerImpl.java:239-244) as seen by BallotBox.
using CommitWaiter = std::function<void(int64_t lastCommittedIndex)>;

struct BallotBoxOptions {
  CommitWaiter waiter;  // BallotBoxOptions.getWaiter (must be set, BallotBox.java:82-90)
  bool closureQueue = true;  // stands for the non-null ClosureQueue requirement
};

class GroupBatch;

// One Raft group's BallotBox (BallotBox.java), backed by a shared GroupBatch.  Thread-safe as
// the reference's @ThreadSafe BallotBox is (BallotBox.java:45, a StampedLock per box): every
// call takes the group's lock, and onCommitted / closures run after it is released.
class BallotBox {
 public:
  BallotBox(std::shared_ptr<GroupBatch> batch, uint32_t group);
  // :82-90 -- once, before the group's first ack (the reference's waiter is final)
  bool init(const BallotBoxOptions& opts);
  // :96-139 -- false if not leader; true if last < pendingIndex (stale); throws
  // std::out_of_range when last >= pendingIndex + queue size; otherwise records the ack,
  // decided at the next GroupBatch::flush().  Any peer may ack (a catch-up replicator of a
  // peer not yet in a conf included, Replicator.java:1387-1392).  A peer's acks must be
  // contiguous over the entries whose ballots count it (the Replicator invariant,
  // Replicator.java:1387-1401): a gap over such an entry throws std::logic_error.
  bool commitAt(int64_t firstLogIndex, int64_t lastLogIndex, const PeerId& peer);
  // :147-156 -- acks recorded since the last epoch are decided first (it waits for a flush in
  // progress and flushes once more), as the reference has already committed them when the
  // leader steps down.  Not from inside a commit callback of the same batch (logic_error).
  void clearPendingTasks();
  bool resetPendingIndex(int64_t newPendingIndex);                             // :167-186
  // :197-215 -- oldConf == nullptr means a stable configuration
  bool appendPendingTask(const Configuration& conf, const Configuration* oldConf,
                         std::function<void(bool)> done = {});
  // `count` appendPendingTask calls with the same conf and no closures (NodeImpl.
  // executeApplyingTasks appends its batch of tasks under one conf, NodeImpl.java:1182-1200)
  bool appendPendingTasks(const Configuration& conf, const Configuration* oldConf, int64_t count);
  bool setLastCommittedIndex(int64_t lastCommittedIndex);                      // :223-248
  int64_t getLastCommittedIndex() const;                                       // :67-79
  int64_t getPendingIndex() const;
  int64_t getPendingMetaQueueSize() const;
  std::string describe() const;                                                // :256-281
  void shutdown() { clearPendingTasks(); }

 private:
  bool append(const Configuration& conf, const Configuration* oldConf, int64_t count,
              std::function<void(bool)>* done);
  std::shared_ptr<GroupBatch> batch_;
  uint32_t g_;
};

// What one GroupBatch::flush() moved and how long each part took.
struct FlushStats {
  uint32_t states = 0;       // group headers uploaded (96 B each)
  uint32_t records = 0;      // 8-B update records uploaded (changed acks / queue sizes)
  uint32_t acks = 0;         // 8-B order-free records written at call time (JRQ_ACK)
  uint32_t acks_streamed = 0;  // of them, pushed to the device by the calling threads themselves
  uint32_t changed = 0;      // groups whose commit advanced (8-B entries downloaded)
  uint64_t h2d_bytes = 0, d2h_bytes = 0;
  double pack_ms = 0, device_ms = 0, deliver_ms = 0;
  // the slowest deliver worker's two passes: commits applied under the groups' locks, then the
  // closures and onCommitted callbacks
  double deliver_apply_ms = 0, deliver_callbacks_ms = 0;
  // inside pack_ms: ending the generation (its call regions drained), and the apply call (which
  // waits for the records' copies ahead of it on the stream)
  double pack_wait_ms = 0, pack_apply_ms = 0;
};

// When the background flusher (GroupBatch::startFlusher) runs an epoch: as soon as the oldest
// change not yet flushed is maxDelayUs old, or maxDirtyGroups groups have changed, whichever
// comes first (the reference decides inside commitAt; the batch trades that for one GPU epoch
// per flush, and this bounds the ack -> onCommitted delay it adds).
struct FlushPolicy {
  uint32_t maxDelayUs = 1000;
  uint32_t maxDirtyGroups = 1u << 16;
};

// BallotBox state of G groups, resident on the GPU (include/jrq.h jrq_table): the host keeps
// a shadow of what Java's BallotBox holds, records what the API calls change, and flush()
// ships only those changes (from page-locked buffers), runs one epoch and delivers the
// commits -- closures, then waiter.onCommitted(index), as BallotBox.commitAt does after
// unlocking (BallotBox.java:131-137).
//
// Threading (the reference's callers: Bolt callback threads per replicator -> commitAt,
// Replicator.java:1391; the LogManager thread's self-ack, NodeImpl.java:1156; the NodeImpl
// disruptor -> appendPendingTask, NodeImpl.java:1195-1196; Bolt server threads ->
// setLastCommittedIndex): every BallotBox call may come from any thread, concurrently with
// other calls and with flush().  Each group has its own lock (a one-byte spin lock: calls
// are short), peers are interned in a lock-free-read process-wide table, and each calling
// thread lists the groups it changes in its own dirty list, which flush() takes, so callers
// keep recording acks for the next epoch while one is packed, decided and delivered.
// commitAt's common case -- a peer that has a slot acking entries contiguous with its last
// ack -- takes no lock and no locked instruction: it raises the slot's match, stamps the slot
// with the batch's generation and lists the group, inside a "call region" of its thread (a
// counter of the thread's own); flush() starts a new generation and waits, behind one
// membarrier(2), for every region of the old one to end, and the rare writers that move a
// slot to another peer or reset a group's matches do the same under the group's lock.  Calls
// for one (group, peer) must not overlap -- the Replicator makes them under its ThreadId lock
// (Replicator.java:1155, 1391) -- overlapping ones could keep the lower of two acks (a later
// commit, never a wrong one).
// Flushes are serialised.  flush() packs and delivers on up to 16 threads; callbacks run
// without the group's lock and may call commitAt / appendPendingTask* (on any group), but not
// flush() or clearPendingTasks() of this batch (std::logic_error).
class GroupBatch : public std::enable_shared_from_this<GroupBatch> {
 public:
  static constexpr uint32_t kAckChunk = 1u << 15;  // records a thread pushes to the device at once
  // eng may be null until the first flush() (host-only state checks need no GPU)
  GroupBatch(Engine* eng, uint32_t groups, uint32_t peers);
  ~GroupBatch();
  GroupBatch(const GroupBatch&) = delete;
  GroupBatch& operator=(const GroupBatch&) = delete;
  uint32_t groups() const { return G_; }
  uint32_t peers() const { return P_; }
  // One epoch: upload what changed, evaluate every group on the GPU, advance
  // pendingIndex / lastCommittedIndex, drop committed ballots, run closures, call waiters.
  // Returns the number of groups whose commit index advanced.  Every changed group's state
  // moves before any callback runs; an exception a callback throws is rethrown after all of
  // them ran.  If the upload or the epoch fails, the groups it carried are shipped again (in
  // full) by the next flush.  Rethrows, once, the error that stopped the background flusher.
  uint32_t flush();
  // Stats of the last flush (read them from the thread that flushed, or after stopFlusher).
  const FlushStats& lastFlush() const { return stats_; }
  // A background thread flushing under `policy` until stopFlusher() (or destruction).
  void startFlusher(const FlushPolicy& policy);
  void stopFlusher();
  uint64_t flushCount() const { return flushes_.load(std::memory_order_relaxed); }
  // Dirty lists of this batch (one per thread that ever changed one of its groups).
  size_t dirtyLists() {
    std::lock_guard<std::mutex> l(listsMu_);
    return lists_.size();
  }
  // Threads flush() packs and delivers on (default: the CPUs this process may use, cgroup
  // quota included, at most 16).
  void setFlushThreads(unsigned n);

 private:
  friend class BallotBox;
  friend class ShardedGroupBatch;
  struct Run {
    int64_t start;
    uint64_t conf;
  };
  template <class T>
  struct PinnedBuf {  // page-locked host staging (jrq_host_alloc)
    T* p = nullptr;
    size_t cap = 0;
    void reserve(size_t n);
    void release();
    PinnedBuf() = default;
    PinnedBuf(PinnedBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
    ~PinnedBuf() { release(); }
  };
  struct DirtyList;  // one per calling thread
  struct Pool;
  struct Flusher;
  struct Part;       // one pack worker's share of a flush
  struct Delivery;   // one deliver worker's commits and callbacks
  static constexpr uint32_t kNoPeer = 0xFFFFFFFFu;
  void ensureRegion(DirtyList& l, uint32_t i, size_t cap);
  static constexpr uint32_t kDirtyLa = 1u << 16, kDirtyHeader = 1u << 17, kDirtyReset = 1u << 18;

  // One group's record: what every API call and the flush touch, in one or two adjacent cache
  // lines (128 B at P = 5) instead of a word in each of nine arrays: the hot header, then
  // match[P] (int64, highest index acked per slot), slotPeer[P] (u32, interned PeerId of the
  // slot), slotUse[P] (u16: the generation of the slot's last raising ack or assignment, mod
  // 2^15, which orders the victims of a slot reassignment; bit 15 marks a fast-path ack that
  // raised the match, which the pack of that generation or the next ships).  Its conf runs live apart (runs_: read when a conf changes or a run
  // dies).  Fields the fast path reads or writes without the lock go through atomic accesses.
  struct Hot {
    std::atomic<uint8_t> lock;  // the group's one-byte spin lock
    std::atomic<uint8_t> gate;  // set by a holder of the lock that moves slots or resets
                                // matches: commitAt's fast path steps aside (quiesce)
    uint8_t nruns;              // conf runs of the pending queue
    uint8_t lastN, lastO;       // the last appended conf's peer counts (lastO 0xFF: no old
                                // conf; lastN 0xFF: no cached conf)
    uint32_t dirty;             // lastAppended / header / slots changed under the lock since
                                // the last pack (the fast path's acks are in the slot stamps)
    uint32_t listed;            // the generation whose dirty list holds the group
    int64_t pi, lc, la;         // pendingIndex, lastCommittedIndex, lastAppended
    uint64_t lastConf;          // conf word of the last run (appends compare against it)
    uint64_t lastSlots;         // slot of the last conf's i-th peer, 4 bits each (<= 16 peers)
  };
  Hot& hot(uint32_t g) const { return *reinterpret_cast<Hot*>(rec_ + static_cast<size_t>(g) * stride_); }
  int64_t* matchOf(uint32_t g) const {
    return reinterpret_cast<int64_t*>(rec_ + static_cast<size_t>(g) * stride_ + sizeof(Hot));
  }
  uint32_t* slotPeerOf(uint32_t g) const {
    return reinterpret_cast<uint32_t*>(rec_ + static_cast<size_t>(g) * stride_ + sizeof(Hot) + 8 * P_);
  }
  uint16_t* slotUseOf(uint32_t g) const {
    return reinterpret_cast<uint16_t*>(rec_ + static_cast<size_t>(g) * stride_ + sizeof(Hot) + 12 * P_);
  }

  void lock(uint32_t g) const;
  void unlock(uint32_t g) const {
    Hot& h = hot(g);
    if (h.gate.load(std::memory_order_relaxed)) h.gate.store(0, std::memory_order_release);
    h.lock.store(0, std::memory_order_release);
  }
  struct Guard {  // the group's lock for a scope
    const GroupBatch& b;
    uint32_t g;
    Guard(const GroupBatch& b_, uint32_t g_) : b(b_), g(g_) { b.lock(g); }
    ~Guard() { b.unlock(g); }
  };
  // all of these run under the group's lock
  int slotOf(uint32_t g, uint32_t peer, bool create, uint32_t reserved = 0);
  uint32_t liveMask(uint32_t g) const;
  // conf word of a Configuration pair given its peers' ids (new conf's nn, then old conf's no)
  uint64_t confWord(uint32_t g, const uint32_t* ids, uint32_t nn, uint32_t no, bool hasOld,
                    uint64_t* slots = nullptr);
  // the ids' slots are the cached ones of the group's last conf (append's fast path)
  bool sameSlots(uint32_t g, const uint32_t* ids, uint32_t n, uint64_t slots) const {
    const uint32_t* sp = slotPeerOf(g);
    for (uint32_t i = 0; i < n; ++i)
      if (sp[(slots >> (4 * i)) & 15u] != ids[i]) return false;
    return true;
  }
  bool gapCountsPeer(uint32_t g, int slot, int64_t lo, int64_t hi) const;
  void markDirty(uint32_t g, uint32_t bits);
  void dropDeadRuns(uint32_t g);
  // commitAt's lock-free common case: 0 / 1 = its result, -1 = take the locked path
  int ackFast(uint32_t g, int64_t first, int64_t last, uint32_t peer);
  // In a call region of generation t: the order-free record `rec` (JRQ_ACK) on this thread's
  // buffer of t, in the segment of the current reset stamp; false when the buffer is full (the
  // caller then lists the group for the pack, as before)
  bool appendAck(DirtyList* l, uint32_t t, uint64_t rec);
  // Under the group's lock, after quiesce(g): records of g written so far are stale (an ended
  // leadership, a slot given to another peer): the group's next header carries a new reset
  // stamp, which drops them on the device
  void stampReset(uint32_t g);
  void listIn(DirtyList* l, Hot& h, uint32_t g, uint32_t t);
  // under the group's lock, before moving a slot to another peer or resetting matches: no
  // fast-path ack of the group is in flight or starts until the lock is released
  void quiesce(uint32_t g);
  // every call region that began before this returns has ended (flush: the old generation's
  // lists and stamps are complete)
  void waitRegions();

  DirtyList* myDirtyList();
  DirtyList* myDirtyListSlow();  // a thread's first call in this batch, or a cache miss
  uint32_t flushLocked();
  void packRange(Part& part, const uint32_t* groups, size_t n);
  void relistAfterFailure();
  size_t partsFor(size_t n, size_t grain);
  template <class F>
  void parallelFor(size_t n, size_t grain, F&& f);

  Engine* eng_;
  uint32_t G_, P_;
  size_t stride_;                         // bytes per group record (a multiple of 64)
  unsigned char* rec_ = nullptr;          // [G] group records (64-B aligned)
  const uint64_t serial_;                 // process-unique id (thread-local list caches)
  std::vector<Run> runs_;                 // [G][JRQ_TABLE_MAX_RUNS] conf runs of the queue
  std::vector<CommitWaiter> waiter_;
  // ClosureQueue (ClosureQueueImpl.java): only non-null closures, per group, in index order
  std::vector<std::unique_ptr<std::deque<std::pair<int64_t, std::function<void(bool)>>>>> closures_;
  std::mutex listsMu_;                    // the per-thread dirty lists
  std::vector<std::unique_ptr<DirtyList>> lists_;
  std::unordered_map<std::thread::id, DirtyList*> byThread_;  // one list per calling thread
  std::mutex flushMu_;                    // one flush at a time
  std::vector<std::vector<uint32_t>> work_;  // swapped-out dirty lists (buffers kept)
  std::vector<Part> parts_;
  std::vector<Delivery> deliveries_;
  uint32_t packGen_ = 0;                  // the generation the running flush packs
  uint64_t packSerial_ = 0;               // flushes started (never wraps)
  std::unique_ptr<uint64_t[]> packedIn_;  // [G] the flush that last packed the group
  // Resets (stampReset) so far; a record is written in a segment stamped with this counter, and
  // a group's headers carry the counter of its last reset (JRQ_STATE_STAMP)
  std::atomic<uint64_t> resetSeq_{0};
  std::unique_ptr<uint64_t[]> rstamp_;    // [G] the group's last reset (under its lock)
  jrq_table* table_ = nullptr;
  PinnedBuf<uint64_t> changed_;
  std::atomic<uint64_t> flushes_{0};
  // the dirty-list generation: flush() takes the lists of the generation it ends (1, 2, ...)
  std::atomic<uint32_t> gen_{1};
  FlushStats stats_;
  std::unique_ptr<Pool> pool_;
  unsigned poolSize_ = 0;
  std::unique_ptr<Flusher> flusher_;
  std::mutex errMu_;
  std::string flusherError_;              // what stopped the background flusher (rethrown once)
};

// A node's groups over several engines (GPUs) in one process (r06; VERDICT r05 missing #1):
// a JVM holds every region of its node (RheaKV StoreEngine.java:93), so one host process drives
// one resident table per GPU.  Group g lives on engine g / k (k = ceil(G / engines), contiguous
// blocks as the multi-process path shards them, jraft_amd/dist.py) as that shard's group g % k,
// in a GroupBatch of its own: calls on different shards share nothing.  flush() runs every
// shard's epoch at once (a thread per shard, each packing and delivering on its share of the
// flush threads; HIP calls of different engines may run concurrently, include/jrq.h).  The
// node-wide committed snapshot (what getLastCommittedIndex readers on every GPU see,
// BallotBox.java:67-79) is published on every engine's device by publish(): one grouped RCCL
// all-gather once rcclInitAll() has made a single-process communicator (ncclCommInitAll), else
// device-to-device copies (two engines on one GPU, which RCCL refuses).
class ShardedGroupBatch {
 public:
  ShardedGroupBatch(const std::vector<Engine*>& engines, uint32_t groups, uint32_t peers);
  ~ShardedGroupBatch();
  ShardedGroupBatch(const ShardedGroupBatch&) = delete;
  ShardedGroupBatch& operator=(const ShardedGroupBatch&) = delete;
  uint32_t groups() const { return G_; }
  uint32_t shards() const { return static_cast<uint32_t>(shard_.size()); }
  uint32_t groupsPerShard() const { return k_; }
  // the shard holding group g, and g's id inside it
  const std::shared_ptr<GroupBatch>& shardOf(uint32_t g, uint32_t* local) const;
  BallotBox box(uint32_t g) const;  // group g's BallotBox (its shard's batch)
  // One epoch on every shard at once; the groups whose commit advanced.  Rethrows the first
  // shard's error after every shard's flush returned.
  uint32_t flush();
  // ncclCommInitAll over the engines' devices; false (and copies from then on) if RCCL refuses
  bool rcclInitAll();
  // After a flush: the node-wide committed[] on every engine's device (asynchronous)
  void publish();
  // engine i's published snapshot, every group's lastCommittedIndex (G words; synchronises)
  void readSnapshot(uint32_t i, int64_t* out);
  bool publishedOverRccl() const;
  const FlushStats& lastFlush(uint32_t shard) const { return shard_[shard]->lastFlush(); }
  void setFlushThreads(unsigned n);  // per shard

 private:
  std::vector<Engine*> eng_;
  uint32_t G_, k_;
  std::vector<std::shared_ptr<GroupBatch>> shard_;
  jrq_snapshot* snap_ = nullptr;
  bool rccl_ = false;
};

namespace testing {
// Called inside commitAt's fast path between its reads and its writes when set (tests widen the
// window a concurrent slot reassignment must not fall into).  Null in production.
extern void (*fastPathHook)();
// Called under the group's lock right after a slot is given to a peer (its id published), when
// set: a test acks from that peer on the fast path there.  Null in production.
extern void (*slotAssignHook)();
// Records a calling thread pushes to the device at once (GroupBatch::kAckChunk); tests make it
// small so that the pushes interleave with everything else.
extern std::atomic<uint32_t> ackChunkRecords;
}  // namespace testing

}  // namespace jraft
