// jraft_drive.cpp -- a multi-Raft load driver over the C++ host mirror (libjraft_host.so):
// it turns a synthetic epoch series into the BallotBox calls a SOFAJRaft host makes and flushes
// one GroupBatch per epoch, so bench.py and the tests measure and check the drop-in path end
// to end (API calls -> changed records from page-locked buffers -> resident device table ->
// changed commits -> closures / onCommitted).
//
// jraft_drive_epochs -- per group g and epoch k (arrays from the caller, e.g. jraft_amd.workloads):
//   epoch 0: setLastCommittedIndex(lc0) as a follower, resetPendingIndex(pi0) as the new
//            leader (NodeImpl.becomeLeader), then appendPendingTask for [pi0, la[0]]
//   epoch k: appendPendingTask for (la[k-1], la[k]] (NodeImpl.executeApplyingTasks,
//            NodeImpl.java:1182-1200, batched: BallotBox::appendPendingTasks)
//   entries >= switch_at[g] (when nonzero) are appended under conf_b instead of conf_a: a
//   conf change inside the pending window (NodeImpl.java:2065-2086, :1195-1196)
//   every peer slot p whose match moved: commitAt(prev + 1, match[k][p][g], peer p) -- the
//   Replicator's contiguous ack (Replicator.java:1387-1392); p = 0 is the leader's own
//   LeaderStableClosure ack (NodeImpl.java:1147-1163)
//   then GroupBatch::flush(): one epoch on the GPU.
//   The calls of an epoch come from `threads` threads, each owning a contiguous slice of the
//   groups (the reference's callers are concurrent: NodeImpl disruptor, LogManager thread, one
//   Bolt callback thread per replicator).
// jraft_drive_latency -- steady load with the background flusher (GroupBatch::startFlusher):
//   `threads` producers loop over their groups, one entry per group per pass
//   (appendPendingTask, then every peer's commitAt of it); onCommitted(c) measures the time
//   from the quorum-completing ack of entry c to the callback.  flush() packs and delivers on
//   `flush_threads` threads (0: its default), beside the producers.
// Peer p of every group is PeerId("127.0.0.1", 8001 + p); conf words name peer slots by bit.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <exception>
#include <thread>
#include <unordered_map>
#include <vector>

#include "jraft_host.h"

namespace {

thread_local std::string g_err;

struct Confs {
  jraft::Configuration cur, old;
  bool hasOld = false;
};

jraft::Configuration confOfMask(uint32_t mask) {
  jraft::Configuration c;
  for (int p = 0; p < 16; ++p)
    if ((mask >> p) & 1u) c.peers.emplace_back("127.0.0.1", 8001 + p);
  return c;
}

Confs confsOfWord(uint64_t cw) {
  Confs c;
  c.cur = confOfMask(static_cast<uint32_t>(cw & 0xFFFFu));
  c.hasOld = ((cw >> 40) & 0xFFu) != 0;
  if (c.hasOld) c.old = confOfMask(static_cast<uint32_t>((cw >> 16) & 0xFFFFu));
  return c;
}

int64_t nowNs() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// T persistent workers: run(f) calls f(t) for t in [0, T) (t = 0 on the caller) and waits.
class Workers {
 public:
  explicit Workers(unsigned n) {
    for (unsigned i = 1; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~Workers() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(const std::function<void(unsigned)>& f) {
    {
      std::lock_guard<std::mutex> l(mu_);
      job_ = &f;
      pending_ = static_cast<unsigned>(th_.size());
      err_ = nullptr;
      ++gen_;
    }
    cv_.notify_all();
    std::exception_ptr mine;
    try {
      f(0);
    } catch (...) {
      mine = std::current_exception();
    }
    std::unique_lock<std::mutex> l(mu_);
    done_.wait(l, [this] { return pending_ == 0; });
    if (mine) std::rethrow_exception(mine);
    if (err_) std::rethrow_exception(err_);
  }

 private:
  void loop(unsigned i) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(unsigned)>* f;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
      }
      std::exception_ptr e;
      try {
        (*f)(i);
      } catch (...) {
        e = std::current_exception();
      }
      std::lock_guard<std::mutex> l(mu_);
      if (e && !err_) err_ = e;
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(unsigned)>* job_ = nullptr;
  std::exception_ptr err_;
  uint64_t gen_ = 0;
  unsigned pending_ = 0;
  bool stop_ = false;
};

}  // namespace

extern "C" {

const char* jraft_drive_last_error(void) { return g_err.c_str(); }

// stats_out[k * 17 + i]: 0 api_ms, 1 pack_ms, 2 device_ms, 3 deliver_ms, 4 flush_ms,
// 5 h2d_bytes, 6 d2h_bytes, 7 states, 8 records (pack + call-time), 9 changed, 10 api_calls,
// 11 acks (the call-time order-free records among them), 12 deliver_apply_ms, 13
// deliver_callbacks_ms (the slowest deliver worker's two passes), 14 pack_wait_ms, 15
// pack_apply_ms, 16 acks_streamed
//
// jraft_drive_epochs_sharded -- the same over `shards` engines on `device` in one process
// (ShardedGroupBatch: contiguous group blocks, the shards' epochs concurrent on their streams);
// after each flush the node-wide snapshot is published, and committed_out is read from engine
// k % shards's copy of it, checked against every group's getLastCommittedIndex.  stats: pack,
// device and deliver ms are the slowest shard's; bytes, states, records and changed the sums.
int jraft_drive_epochs_sharded(int device, uint32_t shards, uint32_t G, uint32_t P, uint32_t K,
                               uint32_t threads, const int64_t* pi0, const int64_t* lc0,
                               const uint64_t* conf_a, const uint64_t* conf_b,
                               const int64_t* switch_at, const int64_t* la, const int64_t* match,
                               int64_t* committed_out, double* stats_out) {
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
  try {
    const unsigned T = std::max(1u, std::min(threads, G));
    const uint32_t S = std::max(1u, std::min(shards, G));
    const uint32_t per = (G + S - 1) / S;
    std::vector<std::unique_ptr<jraft::Engine>> engs;
    std::vector<jraft::Engine*> ep;
    for (uint32_t i = 0; i < S; ++i) {
      engs.emplace_back(new jraft::Engine(device, S == 1 ? G : per, static_cast<uint8_t>(P)));
      ep.push_back(engs.back().get());
    }
    std::shared_ptr<jraft::GroupBatch> batch;
    std::unique_ptr<jraft::ShardedGroupBatch> sharded;
    std::vector<jraft::BallotBox> boxes;
    boxes.reserve(G);
    // (JRAFT_DRIVE_FLUSH_THREADS: the flush pool's size, for tools/drive_ab.py; unset: the
    // batch's default)
    // (JRAFT_DRIVE_ACK_CHUNK: records a calling thread streams to the device at once, 0 = never
    // during the calls -- every record then goes up at the flush; tools/drive_ab.py A/B only)
    if (const char* ac = std::getenv("JRAFT_DRIVE_ACK_CHUNK"))
      jraft::testing::ackChunkRecords.store(std::atoi(ac) > 0 ? static_cast<uint32_t>(std::atoi(ac)) : 0xFFFFFFFFu);
    const char* ft = std::getenv("JRAFT_DRIVE_FLUSH_THREADS");
    const unsigned fthreads = ft ? static_cast<unsigned>(std::atoi(ft)) : 0u;
    if (S == 1) {
      batch = std::make_shared<jraft::GroupBatch>(ep[0], G, P);
      if (fthreads) batch->setFlushThreads(fthreads);
      for (uint32_t g = 0; g < G; ++g) boxes.emplace_back(batch, g);
    } else {
      sharded.reset(new jraft::ShardedGroupBatch(ep, G, P));
      if (fthreads) sharded->setFlushThreads(fthreads);
      sharded->rcclInitAll();  // one device: refused, copies
      for (uint32_t g = 0; g < G; ++g) boxes.push_back(sharded->box(g));
    }
    std::vector<int64_t> snap(sharded ? G : 0);
    std::vector<jraft::PeerId> peers;
    for (uint32_t p = 0; p < P; ++p) peers.emplace_back("127.0.0.1", 8001 + static_cast<int>(p));
    // every distinct conf word's Configurations, built before the threads start (read-only)
    std::unordered_map<uint64_t, Confs> confs;
    for (uint32_t g = 0; g < G; ++g) {
      if (!confs.count(conf_a[g])) confs.emplace(conf_a[g], confsOfWord(conf_a[g]));
      if (switch_at && switch_at[g] > 0 && !confs.count(conf_b[g])) confs.emplace(conf_b[g], confsOfWord(conf_b[g]));
    }
    // the callers' own state, group-major (a Replicator keeps its peer's matchIndex; here one
    // row per group of the P peers' acks per epoch and of their previous acks), laid out before
    // the timed calls so that the timing is the API's, not a strided walk of the input series
    // (each group's Configurations resolved once: a NodeImpl holds its conf, it does not look it
    // up per task)
    std::vector<const Confs*> ca(G), cb(G, nullptr);
    for (uint32_t g = 0; g < G; ++g) {
      ca[g] = &confs.at(conf_a[g]);
      if (switch_at && switch_at[g] > 0) cb[g] = &confs.at(conf_b[g]);
    }
    std::vector<int64_t> prev(static_cast<size_t>(P) * G, 0);
    std::vector<int64_t> acks(static_cast<size_t>(K) * G * P);
    for (uint32_t k = 0; k < K; ++k)
      for (uint32_t p = 0; p < P; ++p)
        for (uint32_t g = 0; g < G; ++g)
          acks[(static_cast<size_t>(k) * G + g) * P + p] = match[(static_cast<size_t>(k) * P + p) * G + g];
    auto append = [&](uint32_t g, int64_t from, int64_t to) -> uint64_t {  // entries [from, to]
      uint64_t calls = 0;
      const int64_t sw = switch_at ? switch_at[g] : 0;
      auto run = [&](const Confs* cp, int64_t a, int64_t b) {
        if (b < a) return;
        const Confs& c = *cp;
        if (!boxes[g].appendPendingTasks(c.cur, c.hasOld ? &c.old : nullptr, b - a + 1))
          throw std::runtime_error("appendPendingTasks refused");
        ++calls;
      };
      if (sw > 0) {
        run(ca[g], from, std::min(to, sw - 1));
        run(cb[g], std::max(from, sw), to);
      } else {
        run(ca[g], from, to);
      }
      return calls;
    };
    Workers workers(T);
    std::vector<uint64_t> calls(T);
    for (uint32_t k = 0; k < K; ++k) {
      const auto t0 = clk::now();
      const int64_t* lak = la + static_cast<size_t>(k) * G;
      const int64_t* ak = acks.data() + static_cast<size_t>(k) * G * P;
      workers.run([&](unsigned t) {
        uint64_t n = 0;
        const uint32_t g0 = static_cast<uint32_t>(static_cast<uint64_t>(G) * t / T);
        const uint32_t g1 = static_cast<uint32_t>(static_cast<uint64_t>(G) * (t + 1) / T);
        for (uint32_t g = g0; g < g1; ++g) {
          if (k == 0) {
            boxes[g].init({[](int64_t) {}});
            boxes[g].setLastCommittedIndex(lc0[g]);
            if (!boxes[g].resetPendingIndex(pi0[g])) throw std::runtime_error("resetPendingIndex refused");
            n += 3 + append(g, pi0[g], lak[g]);
          } else {
            const int64_t lp = la[static_cast<size_t>(k - 1) * G + g];
            if (lak[g] > lp) n += append(g, lp + 1, lak[g]);
          }
          for (uint32_t p = 0; p < P; ++p) {
            const int64_t m = ak[static_cast<size_t>(g) * P + p];
            int64_t& pv = prev[static_cast<size_t>(g) * P + p];
            if (k == 0) pv = m < pi0[g] ? m : pi0[g] - 1;
            if (m > pv) {
              boxes[g].commitAt(pv + 1, m, peers[p]);
              pv = m;
              ++n;
            }
          }
        }
        calls[t] = n;
      });
      const auto t1 = clk::now();
      if (sharded) {
        sharded->flush();
        sharded->publish();
      } else {
        batch->flush();
      }
      const auto t2 = clk::now();
      int64_t* ck = committed_out + static_cast<size_t>(k) * G;
      for (uint32_t g = 0; g < G; ++g) ck[g] = boxes[g].getLastCommittedIndex();
      if (sharded) {
        sharded->readSnapshot(k % S, snap.data());
        for (uint32_t g = 0; g < G; ++g)
          if (snap[g] != ck[g])
            throw std::runtime_error("published snapshot of group " + std::to_string(g) + " on engine " +
                                     std::to_string(k % S) + " differs from its getLastCommittedIndex");
      }
      double* o = stats_out + static_cast<size_t>(k) * 17;
      std::fill(o, o + 17, 0.0);
      for (uint32_t i = 0; i < S; ++i) {
        const jraft::FlushStats& s = sharded ? sharded->lastFlush(i) : batch->lastFlush();
        o[1] = std::max(o[1], s.pack_ms);
        o[2] = std::max(o[2], s.device_ms);
        o[3] = std::max(o[3], s.deliver_ms);
        o[5] += static_cast<double>(s.h2d_bytes);
        o[6] += static_cast<double>(s.d2h_bytes);
        o[7] += s.states;
        o[8] += static_cast<double>(s.records) + s.acks;
        o[11] += s.acks;
        o[9] += s.changed;
        o[12] = std::max(o[12], s.deliver_apply_ms);
        o[13] = std::max(o[13], s.deliver_callbacks_ms);
        o[14] = std::max(o[14], s.pack_wait_ms);
        o[15] = std::max(o[15], s.pack_apply_ms);
        o[16] += s.acks_streamed;
      }
      o[0] = ms(t1 - t0);
      o[4] = ms(t2 - t1);
      uint64_t nc = 0;
      for (uint64_t c : calls) nc += c;
      o[10] = static_cast<double>(nc);
    }
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int jraft_drive_epochs(int device, uint32_t G, uint32_t P, uint32_t K, uint32_t threads,
                       const int64_t* pi0, const int64_t* lc0, const uint64_t* conf_a,
                       const uint64_t* conf_b, const int64_t* switch_at, const int64_t* la,
                       const int64_t* match, int64_t* committed_out, double* stats_out) {
  return jraft_drive_epochs_sharded(device, 1, G, P, K, threads, pi0, lc0, conf_a, conf_b, switch_at,
                                    la, match, committed_out, stats_out);
}

// out[0] commits (onCommitted calls), 1 entries appended, 2 commitAt calls, 3 seconds,
// 4 flushes, 5 p50 latency us, 6 p90, 7 p99, 8 p99.9, 9 max, 10 latency samples, 11 producer
// duty cycle (busy / wall)
int jraft_drive_latency(int device, uint32_t G, uint32_t P, uint32_t threads, uint32_t flush_threads,
                        double seconds, uint32_t max_delay_us, uint32_t max_dirty, uint32_t pass_us,
                        double* out) {
  try {
    const unsigned T = std::max(1u, std::min(threads, G));
    jraft::Engine eng(device, G, static_cast<uint8_t>(P));
    auto batch = std::make_shared<jraft::GroupBatch>(&eng, G, P);
    if (flush_threads) batch->setFlushThreads(flush_threads);
    std::vector<jraft::BallotBox> boxes;
    boxes.reserve(G);
    std::vector<jraft::PeerId> peers;
    for (uint32_t p = 0; p < P; ++p) peers.emplace_back("127.0.0.1", 8001 + static_cast<int>(p));
    const jraft::Configuration conf = confOfMask((1u << P) - 1u);
    // per group: the entry whose quorum-completing ack was recorded last, and when
    std::unique_ptr<std::atomic<int64_t>[]> ackIdx(new std::atomic<int64_t>[G]);
    std::unique_ptr<std::atomic<int64_t>[]> ackNs(new std::atomic<int64_t>[G]);
    std::mutex latMu;
    std::vector<std::vector<float>*> latLists;
    std::atomic<uint64_t> commits{0};
    static std::atomic<uint64_t> runs{0};
    const uint64_t run = ++runs;
    auto latList = [&]() -> std::vector<float>& {  // one list per callback thread and run
      thread_local std::vector<float>* mine = nullptr;
      thread_local uint64_t owner = 0;
      if (owner != run) {
        mine = new std::vector<float>();
        owner = run;
        std::lock_guard<std::mutex> l(latMu);
        latLists.push_back(mine);
      }
      return *mine;
    };
    for (uint32_t g = 0; g < G; ++g) {
      ackIdx[g].store(-1);
      ackNs[g].store(0);
      boxes.emplace_back(batch, g);
      boxes[g].init({[&, g](int64_t c) {
        commits.fetch_add(1, std::memory_order_relaxed);
        if (ackIdx[g].load(std::memory_order_acquire) == c)
          latList().push_back(static_cast<float>((nowNs() - ackNs[g].load(std::memory_order_relaxed)) * 1e-3));
      }});
      if (!boxes[g].resetPendingIndex(1)) throw std::runtime_error("resetPendingIndex refused");
    }
    batch->flush();  // the first flush ships every group's header
    std::atomic<bool> stop{false};
    std::vector<uint64_t> entries(T, 0);
    std::vector<int64_t> busyNs(T, 0);
    batch->startFlusher(jraft::FlushPolicy{max_delay_us, max_dirty});
    const int64_t t0 = nowNs();
    {
      Workers workers(T);
      std::thread timer([&] {
        std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
        stop.store(true);
      });
      // a producer's exception (rethrown by workers.run) must still stop and join the timer and
      // the flusher before it leaves: a joinable std::thread destroyed would call terminate
      struct Join {
        std::atomic<bool>& stop;
        std::thread& timer;
        jraft::GroupBatch& batch;
        ~Join() {
          stop.store(true);
          if (timer.joinable()) timer.join();
          if (std::uncaught_exceptions() > 0) {  // (the normal path stops it below, rethrowing)
            try {
              batch.stopFlusher();
            } catch (...) {
            }
          }
        }
      } join{stop, timer, *batch};
      workers.run([&](unsigned t) {
        const uint32_t g0 = static_cast<uint32_t>(static_cast<uint64_t>(G) * t / T);
        const uint32_t g1 = static_cast<uint32_t>(static_cast<uint64_t>(G) * (t + 1) / T);
        uint64_t n = 0;
        int64_t busy = 0;
        // paced producers: one pass over the slice per pass_us, spread evenly over it in chunks
        // of 256 groups (the replicators' acks arrive with the network: neither a spinning loop,
        // which also hits the box's cgroup CPU quota, nor a burst per pass, which measured the
        // flush of a burst instead of the steady state)
        const uint32_t kChunk = 256;
        const int64_t passNs = static_cast<int64_t>(pass_us) * 1000;
        for (int64_t idx = 1; !stop.load(std::memory_order_relaxed); ++idx) {
          const int64_t p0 = nowNs();
          for (uint32_t c0 = g0; c0 < g1 && !stop.load(std::memory_order_relaxed); c0 += kChunk) {
            const uint32_t c1 = std::min(g1, c0 + kChunk);
            const int64_t b0 = nowNs();
            for (uint32_t g = c0; g < c1; ++g) {
              if (!boxes[g].appendPendingTasks(conf, nullptr, 1)) throw std::runtime_error("append refused");
              for (uint32_t p = 0; p < P; ++p) boxes[g].commitAt(idx, idx, peers[p]);
              ackNs[g].store(nowNs(), std::memory_order_relaxed);
              ackIdx[g].store(idx, std::memory_order_release);
              ++n;
            }
            const int64_t b1 = nowNs();
            busy += b1 - b0;
            if (passNs) {  // on schedule: this chunk's share of the pass
              const int64_t due = p0 + passNs * static_cast<int64_t>(c1 - g0) / static_cast<int64_t>(g1 - g0);
              if (due > b1) std::this_thread::sleep_for(std::chrono::nanoseconds(due - b1));
            }
          }
        }
        entries[t] = n;
        busyNs[t] = busy;
      });
      timer.join();
    }
    batch->stopFlusher();  // rethrows an error that stopped the flusher
    batch->flush();
    const double secs = (nowNs() - t0) * 1e-9;
    std::vector<float> all;
    for (auto* l : latLists) {
      all.insert(all.end(), l->begin(), l->end());
      delete l;
    }
    std::sort(all.begin(), all.end());
    auto q = [&](double f) { return all.empty() ? 0.0 : static_cast<double>(all[std::min(all.size() - 1, static_cast<size_t>(f * all.size()))]); };
    uint64_t ne = 0;
    for (uint64_t e : entries) ne += e;
    out[0] = static_cast<double>(commits.load());
    out[1] = static_cast<double>(ne);
    out[2] = static_cast<double>(ne) * P;
    out[3] = secs;
    out[4] = static_cast<double>(batch->flushCount());
    out[5] = q(0.5);
    out[6] = q(0.9);
    out[7] = q(0.99);
    out[8] = q(0.999);
    out[9] = all.empty() ? 0.0 : all.back();
    out[10] = static_cast<double>(all.size());
    double busy = 0;
    for (int64_t b : busyNs) busy += static_cast<double>(b);
    out[11] = busy * 1e-9 / (secs * T);  // the producers' duty cycle
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

}  // extern "C"
