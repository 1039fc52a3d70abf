/*
 * jraft_oracle.h -- CPU restatement of SOFAJRaft's quorum + checksum hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/, the smoke()
 * entry of __graft_entry__.py and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU baseline.  The product path (libjrq.so)
 * never links or calls it.
 *
 * Everything here restates the reference Java loop structure one-for-one
 * (byte-at-a-time CRC table walk, per-entry Ballot objects, per-(entry, ack)
 * grant loop) so that it doubles as the "port" CPU baseline.
 * Citations: JC = jraft-core/src/main/java/com/alipay/sofa/jraft in the
 * reference tree.
 */
#ifndef JRAFT_ORACLE_H
#define JRAFT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- CRC-64/ECMA-182 (JC/util/CRC64.java) ------------------- */

/* The 256-entry table, generated from the polynomial (JC/util/CRC64.java:41-92). */
const uint64_t *jo_crc64_table(void);
/* CRC64.update(byte[],off,len) continuing from `crc` (JC/util/CRC64.java:100-110). */
uint64_t jo_crc64_update(uint64_t crc, const uint8_t *p, size_t n);
/* CrcUtil.crc64(byte[],off,len): fresh state, update, getValue (JC/util/CrcUtil.java:51-57). */
uint64_t jo_crc64(const uint8_t *p, size_t n);
/* Batch of ragged payloads: out[i] = crc64(payload[off[i] .. off[i+1])). */
void jo_crc64_batch(const uint8_t *payload, const uint64_t *offsets, uint32_t n, uint64_t *out);

/* ---------------- checksums (JC/entity) ---------------------------- */

/* LogId.checksum: crc64(BE64(index) || BE64(term)) (JC/entity/LogId.java:45-50, JC/util/Bits.java:71-80). */
uint64_t jo_logid_checksum(int64_t index, int64_t term);
/* PeerId.checksum: crc64(latin1(ip ":" port [":" idx if idx != 0]))
 * (JC/entity/PeerId.java:60-65,135-144; JC/util/Endpoint.java:60-65; JC/util/AsciiStringUtil.java:27-34). */
uint64_t jo_peerid_checksum(const char *ip, int32_t port, int32_t idx);
/* LogEntry.checksum (JC/entity/LogEntry.java:88-108): type ^ LogId ^ (xor of peer checksums) ^ crc64(data).
 * peer_xor is the XOR of every PeerId.checksum() of peers, oldPeers, learners, oldLearners
 * (XOR is order independent: JC/entity/Checksum.java:40-42). */
uint64_t jo_logentry_checksum(int32_t type, int64_t index, int64_t term, uint64_t peer_xor,
                              const uint8_t *data, size_t len);
/* Batch form with optional verify (LogEntry.isCorrupted, JC/entity/LogEntry.java:156-158).
 * expected/has/corrupt may be NULL (then no verify).  has==NULL means "every entry has a checksum". */
void jo_logentry_checksum_batch(const uint8_t *type, const int64_t *index, const int64_t *term,
                                const uint64_t *peer_xor, const uint8_t *payload,
                                const uint64_t *offsets, uint32_t n, uint64_t *out,
                                const uint64_t *expected, const uint8_t *has, uint8_t *corrupt);

/* Follower receive path (JC/core/NodeImpl.java:1766-1792, logEntryFromMeta :1809-1823):
 * per request r, index runs from prev_log_index[r]+1; an entry of type UNKNOWN (0) is
 * skipped and consumes no data; otherwise it takes the next data_len bytes of `data`
 * (requests back to back) and, if has_checksum (NULL = all), is corrupt when the stored
 * checksum differs from LogEntry.checksum().  first_corrupt[r] = position of the first
 * corrupt entry (where the reference returns EINVAL) or -1.  checksum_out gets every
 * entry's computed checksum. */
void jo_append_entries_verify(uint32_t R, const uint32_t *req_off, const int64_t *prev_log_index,
                              const int64_t *term, const uint8_t *type, const int64_t *data_len,
                              const uint64_t *peer_xor, const uint64_t *checksum,
                              const uint8_t *has_checksum, const uint8_t *data,
                              uint64_t *checksum_out, uint8_t *corrupt_out, int32_t *first_corrupt);

/* NodeImpl.checkDeadNodes0 (JC/core/NodeImpl.java:1970-2000) over a peer list (ids),
 * with lastRpcSendTimestamp per id in ts[] and the leader's own id `self`.  Returns 1 when
 * the alive count reaches size/2+1 and then stores the lease start (oldest alive
 * timestamp of a non-self member, INT64_MAX if none) in *lease_start; ORs the dead ids
 * into *dead_mask. */
int jo_check_dead_nodes(const int32_t *peers, int32_t n, const int64_t *ts, int32_t self,
                        int64_t now_ms, int64_t lease_timeout_ms, int64_t *lease_start,
                        uint32_t *dead_mask);
/* handleStepDownTimeout (:2003-2016) for G groups with the engine's packed conf words
 * (peer lists rebuilt from the masks in slot order): ok bit0 conf, bit1 old conf (or none). */
void jo_lease_check(uint32_t G, uint32_t P, const int64_t *ts /* [P][G] */, const uint64_t *conf,
                    const uint8_t *self_slot, int64_t now_ms, int64_t lease_timeout_ms,
                    uint8_t *ok, int64_t *lease_start /* in/out */, uint16_t *dead);

/* NodeImpl.readLeader's ReadOnlySafe heartbeat round (JC/core/NodeImpl.java:1246-1396) for
 * one group: conf peers = the set bits of mask (slot order), heartbeat responses from slots
 * < P other than self in arrival order (order: 4 bits per slot, position 1..15, 0 = none;
 * ties by slot), ok_mask bit = success.  Returns 0 pending, 1 success, 2 failure. */
uint8_t jo_readindex_round(uint32_t mask, uint32_t P, uint32_t self, uint64_t order, uint32_t ok_mask);
void jo_readindex_quorum(uint32_t G, uint32_t P, const uint64_t *conf, const uint8_t *self_slot,
                         const uint64_t *order, const uint16_t *ok_mask, uint8_t *result);

/* ---------------- Ballot (JC/entity/Ballot.java) --------------------------- */

#define JO_MAX_CONF 32 /* peers per Configuration list kept by the oracle */

typedef struct {
    int32_t peer[JO_MAX_CONF];
    uint8_t found[JO_MAX_CONF];
    int32_t n;
} jo_peer_list;

typedef struct {
    jo_peer_list peers;
    int32_t quorum;
    jo_peer_list old_peers;
    int32_t old_quorum;
} jo_ballot;

typedef struct {
    int32_t pos0, pos1;
} jo_pos_hint;

/* Ballot.init(conf, oldConf) (JC/entity/Ballot.java:63-85).  Peers are small integer ids:
 * PeerId.equals == id equality.  nconf < 0 means conf == null, nold < 0 means oldConf == null. */
int jo_ballot_init(jo_ballot *b, const int32_t *conf, int32_t nconf, const int32_t *old, int32_t nold);
/* Ballot.grant(peer, hint) including the PosHint search (JC/entity/Ballot.java:87-127). */
jo_pos_hint jo_ballot_grant_hint(jo_ballot *b, int32_t peer, jo_pos_hint hint);
void jo_ballot_grant(jo_ballot *b, int32_t peer);
/* Ballot.isGranted (JC/entity/Ballot.java:138-140). */
int jo_ballot_is_granted(const jo_ballot *b);

/* ---------------- BallotBox (JC/core/BallotBox.java) ----------------------- */

enum { JO_FALSE = 0, JO_TRUE = 1, JO_AIOOBE = -1 /* ArrayIndexOutOfBoundsException */,
       JO_IAE = -2 /* IllegalArgumentException */ };

typedef struct jo_ballot_box jo_ballot_box;

jo_ballot_box *jo_bb_new(void);
void jo_bb_free(jo_ballot_box *bb);
int64_t jo_bb_last_committed_index(const jo_ballot_box *bb); /* :67-79 */
int64_t jo_bb_pending_index(const jo_ballot_box *bb);
int64_t jo_bb_queue_size(const jo_ballot_box *bb);
/* FSMCaller.onCommitted(idx) calls observed so far (the Mockito waiter of BallotBoxTest). */
int64_t jo_bb_on_committed_calls(const jo_ballot_box *bb);
int64_t jo_bb_on_committed_last(const jo_ballot_box *bb);
int jo_bb_commit_at(jo_ballot_box *bb, int64_t first, int64_t last, int32_t peer); /* :96-139 */
void jo_bb_clear_pending_tasks(jo_ballot_box *bb);                                 /* :147-156 */
int jo_bb_reset_pending_index(jo_ballot_box *bb, int64_t new_pending_index);       /* :167-186 */
int jo_bb_append_pending_task(jo_ballot_box *bb, const int32_t *conf, int32_t nconf,
                              const int32_t *old, int32_t nold);                   /* :197-215 */
int jo_bb_set_last_committed_index(jo_ballot_box *bb, int64_t idx);                /* :223-248 */

/* ---------------- one quorum epoch, replayed as calls ---------------------- */

/* Per-group status codes shared with the engine (include/jrq.h). */
enum { JO_ST_OK = 0, JO_ST_NOT_LEADER = 1, JO_ST_OUT_OF_RANGE = 2, JO_ST_EMPTY_CONF = 4 };

/*
 * Replays one epoch of a group batch through real jo_ballot_box objects:
 *   for each group g: resetPendingIndex(pendingIndex), appendPendingTask for every
 *   index in [pendingIndex, lastAppended] with the conf of the run that covers it,
 *   then, per peer p, the acks a Replicator would send for match[p][g]: contiguous
 *   commitAt(first, last, p) calls of at most `chunk` entries from pendingIndex up to
 *   match (interleaved round-robin across peers, leader first); a peer whose match
 *   exceeds lastAppended sends commitAt(pendingIndex, match) which throws AIOOBE.
 * Runs: run_off[G+1] (NULL => one run per group from conf[]), run_start[R] (first
 * index of the run), run_conf[R] in the same packing as conf[].
 * conf packing (uint64, shared with include/jrq.h): bits 0-15 new-peer mask over
 *   the group's peer slots, 16-31 old-peer mask, 32-39 new quorum, 40-47 old quorum.
 *   The oracle builds Ballots from the masks exactly as Ballot.init does (quorum =
 *   n/2+1, computed here, not read); old quorum byte 0 means oldConf == null, any
 *   other value means an old conf is present (possibly empty).
 * lastCommitted[g] is the state before the epoch.  Outputs committed[g] and status[g].
 * Returns the number of Ballot.grant calls executed (the work the reference does).
 */
int64_t jo_quorum_epoch_replay(uint32_t G, uint32_t P, const int64_t *match /* [P][G] */,
                               const int64_t *pending_index, const int64_t *last_appended,
                               const int64_t *last_committed, const uint64_t *conf,
                               const uint32_t *run_off, const int64_t *run_start,
                               const uint64_t *run_conf, int64_t chunk,
                               int64_t *committed_out, uint8_t *status_out);

/* ---------------- commit fan-out (ClosureQueueImpl, FSMCallerImpl) -------- */
enum { JO_FAN_NONE = 0, JO_FAN_APPLY = 1, JO_FAN_SKIP = 2, JO_FAN_INVALID = 3 };
/*
 * Per group g: a ClosureQueue holding cq_size[g] closures for log indices cq_first[g]..
 * (resetFirstIndex + appendPendingClosure, JC/closure/ClosureQueueImpl.java:83-105), then
 * the epoch's onCommitted calls seq[seq_off[g] .. seq_off[g+1]) (increasing, as BallotBox
 * emits them), each run through FSMCallerImpl.doCommitted (JC/core/FSMCallerImpl.java:
 * 462-482: skip if lastAppliedIndex >= c; popClosureUntil(c), :113-142; a -1 return fails
 * Requires.requireTrue and the call ends; else entries up to c are applied and
 * lastAppliedIndex = c).  Outputs per group: status (NONE: no call; INVALID: some pop
 * returned -1; APPLY: some call popped/applied; SKIP otherwise), first_closure = index of
 * the first closure popped during the epoch, or (last call's c)+1 when none was popped
 * (-1 for INVALID, 0 for NONE/SKIP); cq_first/cq_size/last_applied updated in place.
 * Returns the number of closures popped in total.
 */
int64_t jo_commit_fanout_replay(uint32_t G, const uint64_t *seq_off, const int64_t *seq,
                                int64_t *last_applied, int64_t *cq_first, int64_t *cq_size,
                                int64_t *first_closure, uint8_t *status);

/* ---------------- V2 log entry decode + verify on read ---------------------- */
/* Statuses: OK; NULL = the reference decoder returns null (AutoDetectDecoder on an empty
 * record, V2Decoder on a short header / bad magic / bad version, or protobuf's
 * InvalidProtocolBufferException incl. missing required fields); V1 = first byte is not the
 * V2 magic (routed to V1Decoder, not restated); PEER_NONCANON = decodes, but a peer string
 * re-renders differently through PeerId.parse/toString (the checksum uses the re-rendered
 * string); PEER_THROWS = JRaftUtils.getPeerId throws IllegalArgumentException. */
enum { JO_V2_OK = 0, JO_V2_NULL = 1, JO_V2_V1 = 2, JO_V2_PEER_NONCANON = 3, JO_V2_PEER_THROWS = 4 };
uint64_t jo_v2_peer_checksum(const uint8_t *s, int64_t n, int *kind);
/*
 * Record r = rec[off[r] .. off[r+1]): the bytes a LogStorage holds for one index
 * (LogEntryV2CodecFactory header 0xBB 0xD2 0x01 + 3 reserved, then a PBLogEntry,
 * JC/entity/codec/v2/V2Encoder.java:76-130), decoded as AutoDetectDecoder/V2Decoder do
 * (JC/entity/codec/AutoDetectDecoder.java:41-52, v2/V2Decoder.java:46-110) and verified as
 * LogManagerImpl does on read (JC/core/LogManagerImpl.java:733-745: isCorrupted).
 * peer_counts[r] (nullable) = peers | old_peers<<8 | learners<<16 | old_learners<<24 (each
 * saturating at 255).  data_off is absolute into rec.  Undecodable records get zeros,
 * data_off = off[r], data_len 0.
 */
void jo_v2_decode_batch(const uint8_t *rec, const uint64_t *off, uint32_t n, uint8_t *status,
                        uint8_t *type, int64_t *index, int64_t *term, uint64_t *stored,
                        uint8_t *has_checksum, uint64_t *data_off, uint64_t *data_len,
                        uint32_t *peer_counts, uint64_t *computed, uint8_t *corrupt);

#ifdef __cplusplus
}
#endif
#endif
