// jraft_host.cpp -- C++ host mirror of BallotBox / LogEntry / CrcUtil over libjrq.so.
// See jraft_host.h.  No checksum or quorum arithmetic happens here: it is all
// delegated to the GPU through include/jrq.h.
#include "jraft_host.h"

#include <algorithm>
#include <cstring>
#include <sstream>

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

GroupBatch::GroupBatch(Engine* eng, uint32_t groups, uint32_t peers)
    : eng_(eng), G_(groups), P_(peers), grp_(groups) {
  if (peers == 0 || peers > JRQ_MAX_PEERS) throw std::invalid_argument("peers must be 1..16");
  for (auto& g : grp_) g.match.assign(P_, 0);
}

int GroupBatch::slotOf(Group& g, const PeerId& p, bool create) {
  auto it = g.slot.find(p);
  if (it != g.slot.end()) return it->second;
  if (!create) return -1;
  if ((uint32_t)g.slot.size() >= P_) throw std::length_error("more distinct peers than slots");
  int s = (int)g.slot.size();
  g.slot.emplace(p, s);
  return s;
}

uint64_t GroupBatch::confWord(Group& g, const Configuration& conf, const Configuration* old) {
  // Ballot.init (Ballot.java:63-85): peers only, quorum = size/2+1, oldQuorum 0 if null
  uint32_t nm = 0, om = 0;
  for (auto& p : conf.peers) nm |= 1u << slotOf(g, p, true);
  uint32_t nq = (uint32_t)conf.peers.size() / 2 + 1, oq = 0;
  if (old) {
    for (auto& p : old->peers) om |= 1u << slotOf(g, p, true);
    oq = (uint32_t)old->peers.size() / 2 + 1;
  }
  return JRQ_CONF(nm, om, nq, oq);
}

uint32_t GroupBatch::flush() {
  std::vector<uint32_t> live;
  for (uint32_t i = 0; i < G_; ++i)
    if (grp_[i].pendingIndex != 0 && grp_[i].lastAppended >= grp_[i].pendingIndex) live.push_back(i);
  if (live.empty()) return 0;
  const uint32_t G = (uint32_t)live.size();
  std::vector<int64_t> match((size_t)P_ * G), pi(G), la(G), lc(G), committed(G);
  std::vector<uint64_t> conf(G);
  std::vector<uint32_t> run_off(G + 1, 0);
  std::vector<int64_t> run_start;
  std::vector<uint64_t> run_conf;
  for (uint32_t k = 0; k < G; ++k) {
    Group& g = grp_[live[k]];
    for (uint32_t p = 0; p < P_; ++p) match[(size_t)p * G + k] = g.match[p];
    pi[k] = g.pendingIndex;
    la[k] = g.lastAppended;
    lc[k] = g.lastCommitted;
    conf[k] = g.runs.empty() ? 0 : g.runs.front().conf;
    for (auto& r : g.runs) {
      run_start.push_back(r.start);
      run_conf.push_back(r.conf);
    }
    run_off[k + 1] = (uint32_t)run_start.size();
  }
  std::vector<uint8_t> status(G);
  jrq_group_batch b{};
  b.match = match.data();
  b.pending_index = pi.data();
  b.last_appended = la.data();
  b.last_committed = lc.data();
  b.conf = conf.data();
  b.run_off = run_off.data();
  b.run_start = run_start.data();
  b.run_conf = run_conf.data();
  b.num_peers = P_;
  b.num_runs = (uint32_t)run_start.size();
  b.match_ld = G;
  if (!eng_) throw std::logic_error("GroupBatch::flush needs an Engine");
  throwIfError(jrq_quorum_epoch(eng_->raw(), &b, committed.data(), status.data(), G), eng_->raw(),
               "jrq_quorum_epoch");
  uint32_t advanced = 0;
  for (uint32_t k = 0; k < G; ++k) {
    Group& g = grp_[live[k]];
    const int64_t c = committed[k];
    if (c <= g.lastCommitted) continue;
    // pendingMetaQueue.removeRange(0, c - pendingIndex + 1); pendingIndex = c + 1 (:130-132)
    const int64_t ncommitted = c - g.pendingIndex + 1;
    for (int64_t i = 0; i < ncommitted && i < (int64_t)g.closures.size(); ++i)
      if (g.closures[i]) g.closures[i](true);  // ClosureQueue.popClosureUntil -> done.run(OK)
    g.closures.erase(g.closures.begin(),
                     g.closures.begin() + std::min<int64_t>(ncommitted, (int64_t)g.closures.size()));
    g.pendingIndex = c + 1;
    g.lastCommitted = c;
    while (g.runs.size() > 1 && g.runs[1].start <= g.pendingIndex) g.runs.erase(g.runs.begin());
    ++advanced;
    if (g.waiter) g.waiter(c);  // waiter.onCommitted(lastCommittedIndex), after the "unlock"
  }
  return advanced;
}

BallotBox::BallotBox(std::shared_ptr<GroupBatch> batch, uint32_t group) : batch_(std::move(batch)), g_(group) {
  if (g_ >= batch_->groups()) throw std::out_of_range("group id");
}

bool BallotBox::init(const BallotBoxOptions& opts) {
  if (!opts.waiter || !opts.closureQueue) return false;  // "waiter or closure queue is null."
  auto& g = batch_->grp_[g_];
  g.waiter = opts.waiter;
  g.inited = true;
  return true;
}

bool BallotBox::commitAt(int64_t first, int64_t last, const PeerId& peer) {
  auto& g = batch_->grp_[g_];
  if (g.pendingIndex == 0) return false;                         // :101-103
  if (last < g.pendingIndex) return true;                        // :104-106
  if (last > g.lastAppended) throw std::out_of_range("ArrayIndexOutOfBoundsException");  // :107-109
  const int s = batch_->slotOf(g, peer, false);
  if (s < 0) return true;  // not in any conf of this group: Ballot.grant finds nothing
  int64_t& m = g.match[s];
  if (first > std::max(m + 1, g.pendingIndex))
    throw std::logic_error("non-contiguous ack: the Replicator never skips entries");
  if (last > m) m = last;
  return true;
}

void BallotBox::clearPendingTasks() {
  auto& g = batch_->grp_[g_];
  for (auto& c : g.closures)
    if (c) c(false);  // ClosureQueue.clear runs closures with EPERM
  g.closures.clear();
  g.runs.clear();
  g.pendingIndex = 0;
  g.lastAppended = -1;
}

bool BallotBox::resetPendingIndex(int64_t n) {
  auto& g = batch_->grp_[g_];
  if (!(g.pendingIndex == 0 && g.lastAppended < g.pendingIndex)) return false;
  if (n <= g.lastCommitted) return false;
  g.pendingIndex = n;
  g.lastAppended = n - 1;
  g.runs.clear();
  std::fill(g.match.begin(), g.match.end(), 0);  // a new leader's replicators start over
  return true;
}

bool BallotBox::appendPendingTask(const Configuration& conf, const Configuration* oldConf,
                                  std::function<void(bool)> done) {
  auto& g = batch_->grp_[g_];
  if (g.pendingIndex <= 0) return false;  // :204-207
  const uint64_t cw = batch_->confWord(g, conf, oldConf);
  const int64_t idx = g.lastAppended + 1;
  if (g.runs.empty() || g.runs.back().conf != cw) g.runs.push_back({idx, cw});
  g.lastAppended = idx;
  g.closures.push_back(std::move(done));
  return true;
}

bool BallotBox::setLastCommittedIndex(int64_t c) {
  auto& g = batch_->grp_[g_];
  if (g.pendingIndex != 0 || g.lastAppended >= g.pendingIndex) {
    if (!(c < g.pendingIndex))  // Requires.requireTrue (:229-231)
      throw std::invalid_argument("Node changes to leader, pendingIndex=" +
                                  std::to_string(g.pendingIndex) +
                                  ", param lastCommittedIndex=" + std::to_string(c));
    return false;
  }
  if (c < g.lastCommitted) return false;
  if (c > g.lastCommitted) {
    g.lastCommitted = c;
    if (g.waiter) g.waiter(c);
  }
  return true;
}

int64_t BallotBox::getLastCommittedIndex() const { return batch_->grp_[g_].lastCommitted; }
int64_t BallotBox::getPendingIndex() const { return batch_->grp_[g_].pendingIndex; }
int64_t BallotBox::getPendingMetaQueueSize() const {
  auto& g = batch_->grp_[g_];
  return g.pendingIndex == 0 ? 0 : g.lastAppended - g.pendingIndex + 1;
}

std::string BallotBox::describe() const {
  std::ostringstream o;
  o << "  lastCommittedIndex: " << getLastCommittedIndex() << "\n"
    << "  pendingIndex: " << getPendingIndex() << "\n"
    << "  pendingMetaQueueSize: " << getPendingMetaQueueSize() << "\n";
  return o.str();
}

}  // namespace jraft
