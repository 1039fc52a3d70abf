// jraft_drive.cpp -- a multi-Raft load driver over the C++ host mirror (libjraft_host.so):
// it turns a synthetic epoch series into the BallotBox calls a SOFAJRaft host makes and flushes
// one GroupBatch per epoch, so bench.py and the tests measure and check the drop-in path end
// to end (API calls -> changed records from page-locked buffers -> resident device table ->
// changed commits -> closures / onCommitted).
//
// Per group g and epoch k (arrays from the caller, e.g. jraft_amd.workloads):
//   epoch 0: setLastCommittedIndex(lc0) as a follower, resetPendingIndex(pi0) as the new
//            leader (NodeImpl.becomeLeader), then appendPendingTask for [pi0, la[0]]
//   epoch k: appendPendingTask for (la[k-1], la[k]] (NodeImpl.executeApplyingTasks,
//            NodeImpl.java:1182-1200, batched: BallotBox::appendPendingTasks)
//   entries >= switch_at[g] (when nonzero) are appended under conf_b instead of conf_a: a
//   conf change inside the pending window (NodeImpl.java:2065-2086, :1195-1196)
//   every peer slot p whose match moved: commitAt(prev + 1, match[k][p][g], peer p) -- the
//   Replicator's contiguous ack (Replicator.java:1387-1392); p = 0 is the leader's own
//   LeaderStableClosure ack (NodeImpl.java:1147-1163)
//   then GroupBatch::flush(): one epoch on the GPU
// Peer p of every group is PeerId("127.0.0.1", 8001 + p); conf words name peer slots by bit.
#include <chrono>
#include <cstring>
#include <string>
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

}  // namespace

extern "C" {

const char* jraft_drive_last_error(void) { return g_err.c_str(); }

// stats_out[k * 11 + i]: 0 api_ms, 1 pack_ms, 2 device_ms, 3 deliver_ms, 4 flush_ms,
// 5 h2d_bytes, 6 d2h_bytes, 7 states, 8 records, 9 changed, 10 api_calls
int jraft_drive_epochs(int device, uint32_t G, uint32_t P, uint32_t K, const int64_t* pi0,
                       const int64_t* lc0, const uint64_t* conf_a, const uint64_t* conf_b,
                       const int64_t* switch_at, const int64_t* la, const int64_t* match,
                       int64_t* committed_out, double* stats_out) {
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
  try {
    jraft::Engine eng(device, G, static_cast<uint8_t>(P));
    auto batch = std::make_shared<jraft::GroupBatch>(&eng, G, P);
    std::vector<jraft::BallotBox> boxes;
    boxes.reserve(G);
    std::vector<jraft::PeerId> peers;
    for (uint32_t p = 0; p < P; ++p) peers.emplace_back("127.0.0.1", 8001 + static_cast<int>(p));
    std::unordered_map<uint64_t, Confs> confs;
    auto confsOf = [&](uint64_t cw) -> const Confs& {
      auto it = confs.find(cw);
      if (it != confs.end()) return it->second;
      Confs c;
      c.cur = confOfMask(static_cast<uint32_t>(cw & 0xFFFFu));
      c.hasOld = ((cw >> 40) & 0xFFu) != 0;
      if (c.hasOld) c.old = confOfMask(static_cast<uint32_t>((cw >> 16) & 0xFFFFu));
      return confs.emplace(cw, std::move(c)).first->second;
    };
    std::vector<int64_t> prev(static_cast<size_t>(P) * G, 0);
    auto append = [&](uint32_t g, int64_t from, int64_t to) -> uint64_t {  // entries [from, to]
      uint64_t calls = 0;
      const int64_t sw = switch_at ? switch_at[g] : 0;
      auto run = [&](uint64_t cw, int64_t a, int64_t b) {
        if (b < a) return;
        const Confs& c = confsOf(cw);
        if (!boxes[g].appendPendingTasks(c.cur, c.hasOld ? &c.old : nullptr, b - a + 1))
          throw std::runtime_error("appendPendingTasks refused");
        ++calls;
      };
      if (sw > 0) {
        run(conf_a[g], from, std::min(to, sw - 1));
        run(conf_b[g], std::max(from, sw), to);
      } else {
        run(conf_a[g], from, to);
      }
      return calls;
    };
    for (uint32_t k = 0; k < K; ++k) {
      const auto t0 = clk::now();
      uint64_t calls = 0;
      const int64_t* lak = la + static_cast<size_t>(k) * G;
      const int64_t* mk = match + static_cast<size_t>(k) * P * G;
      for (uint32_t g = 0; g < G; ++g) {
        if (k == 0) {
          boxes.emplace_back(batch, g);
          boxes[g].init({[](int64_t) {}});
          boxes[g].setLastCommittedIndex(lc0[g]);
          if (!boxes[g].resetPendingIndex(pi0[g])) throw std::runtime_error("resetPendingIndex refused");
          calls += 3 + append(g, pi0[g], lak[g]);
        } else {
          const int64_t lp = la[static_cast<size_t>(k - 1) * G + g];
          if (lak[g] > lp) calls += append(g, lp + 1, lak[g]);
        }
        for (uint32_t p = 0; p < P; ++p) {
          const int64_t m = mk[static_cast<size_t>(p) * G + g];
          int64_t& pv = prev[static_cast<size_t>(p) * G + g];
          if (k == 0) pv = m < pi0[g] ? m : pi0[g] - 1;
          if (m > pv) {
            boxes[g].commitAt(pv + 1, m, peers[p]);
            pv = m;
            ++calls;
          }
        }
      }
      const auto t1 = clk::now();
      batch->flush();
      const auto t2 = clk::now();
      for (uint32_t g = 0; g < G; ++g)
        committed_out[static_cast<size_t>(k) * G + g] = boxes[g].getLastCommittedIndex();
      const jraft::FlushStats& s = batch->lastFlush();
      double* o = stats_out + static_cast<size_t>(k) * 11;
      o[0] = ms(t1 - t0);
      o[1] = s.pack_ms;
      o[2] = s.device_ms;
      o[3] = s.deliver_ms;
      o[4] = ms(t2 - t1);
      o[5] = static_cast<double>(s.h2d_bytes);
      o[6] = static_cast<double>(s.d2h_bytes);
      o[7] = s.states;
      o[8] = s.records;
      o[9] = s.changed;
      o[10] = static_cast<double>(calls);
    }
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

}  // extern "C"
