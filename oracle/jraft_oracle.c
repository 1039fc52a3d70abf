/*
 * jraft_oracle.c -- CPU restatement of SOFAJRaft's quorum + checksum hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see jraft_oracle.h).  Never linked into libjrq.so.
 * Loop structure deliberately follows the Java reference (JC = jraft-core/src/
 * main/java/com/alipay/sofa/jraft): it is both the parity oracle and the "port"
 * CPU baseline that bench.py times.
 */
#include "jraft_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ======================= CRC64 (JC/util/CRC64.java) ======================= */

/* CRC-64/ECMA-182, MSB first: poly=0x42f0e1eba9ea3693 init=0 refin=false
 * refout=false xorout=0 (JC/util/CRC64.java:27-40).  Entry i is the register
 * after shifting i<<56 through 8 polynomial steps; tests/golden pins every entry
 * against the literal table at JC/util/CRC64.java:41-92. */
#define JO_POLY 0x42F0E1EBA9EA3693ULL
static uint64_t g_table[256];
static int g_table_ready = 0;

static void build_table(void) {
    for (int i = 0; i < 256; ++i) {
        uint64_t c = (uint64_t)i << 56;
        for (int k = 0; k < 8; ++k) c = (c & 0x8000000000000000ULL) ? (c << 1) ^ JO_POLY : (c << 1);
        g_table[i] = c;
    }
    g_table_ready = 1;
}

const uint64_t *jo_crc64_table(void) {
    if (!g_table_ready) build_table();
    return g_table;
}

/* CRC64.update(byte): tab_index = ((int)(crc >> 56) ^ b) & 0xFF;
 * crc = CRC_TABLE[tab_index] ^ (crc << 8)  (JC/util/CRC64.java:100-103).
 * Java's arithmetic >> is masked by & 0xFF, so a logical shift is equivalent. */
uint64_t jo_crc64_update(uint64_t crc, const uint8_t *p, size_t n) {
    const uint64_t *t = jo_crc64_table();
    for (size_t i = 0; i < n; ++i) crc = t[((crc >> 56) ^ p[i]) & 0xFF] ^ (crc << 8);
    return crc;
}

/* CrcUtil.crc64(byte[],off,len): ThreadLocal CRC64 -> update -> getValue -> reset
 * (JC/util/CrcUtil.java:51-57).  A zero-length range returns 0. */
uint64_t jo_crc64(const uint8_t *p, size_t n) { return jo_crc64_update(0, p, n); }

void jo_crc64_batch(const uint8_t *payload, const uint64_t *offsets, uint32_t n, uint64_t *out) {
    for (uint32_t i = 0; i < n; ++i)
        out[i] = jo_crc64(payload + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
}

/* ======================= checksums (JC/entity) ============================ */

/* Bits.putLong big-endian (JC/util/Bits.java:71-80). */
static void put_long_be(uint8_t *b, int64_t v) {
    uint64_t u = (uint64_t)v;
    for (int k = 7; k >= 0; --k) { b[k] = (uint8_t)u; u >>= 8; }
}

/* LogId.checksum (JC/entity/LogId.java:45-50). */
uint64_t jo_logid_checksum(int64_t index, int64_t term) {
    uint8_t bs[16];
    put_long_be(bs, index);
    put_long_be(bs + 8, term);
    return jo_crc64(bs, 16);
}

/* PeerId.checksum over AsciiStringUtil.unsafeEncode(toString()) (JC/entity/PeerId.java:60-65,
 * 135-144; Endpoint.toString JC/util/Endpoint.java:60-65).  Characters are truncated to a byte
 * ((byte) in.charAt(i), JC/util/AsciiStringUtil.java:27-34); C strings are already bytes. */
uint64_t jo_peerid_checksum(const char *ip, int32_t port, int32_t idx) {
    char s[512];
    int n = (idx != 0) ? snprintf(s, sizeof s, "%s:%d:%d", ip, port, idx)
                       : snprintf(s, sizeof s, "%s:%d", ip, port);
    if (n < 0) return 0;
    if ((size_t)n >= sizeof s) n = (int)sizeof s - 1;
    return jo_crc64((const uint8_t *)s, (size_t)n);
}

/* LogEntry.checksum (JC/entity/LogEntry.java:88-99):
 *   c = type.getNumber() ^ id.checksum();  c ^= peer.checksum() for each peer list;
 *   if (data != null && data.hasRemaining()) c ^= CrcUtil.crc64(data).
 * An empty data buffer is skipped by the reference and contributes crc64("") = 0 here:
 * identical result. */
uint64_t jo_logentry_checksum(int32_t type, int64_t index, int64_t term, uint64_t peer_xor,
                              const uint8_t *data, size_t len) {
    uint64_t c = (uint64_t)(int64_t)type ^ jo_logid_checksum(index, term);
    c ^= peer_xor;
    if (data != NULL && len > 0) c ^= jo_crc64(data, len);
    return c;
}

void jo_logentry_checksum_batch(const uint8_t *type, const int64_t *index, const int64_t *term,
                                const uint64_t *peer_xor, const uint8_t *payload,
                                const uint64_t *offsets, uint32_t n, uint64_t *out,
                                const uint64_t *expected, const uint8_t *has, uint8_t *corrupt) {
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t c = jo_logentry_checksum(type[i], index[i], term[i], peer_xor ? peer_xor[i] : 0,
                                          payload + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
        out[i] = c;
        /* LogEntry.isCorrupted: hasChecksum && checksum != checksum() (:156-158). */
        if (expected && corrupt) corrupt[i] = (uint8_t)(((has == NULL) || has[i]) && expected[i] != c);
    }
}

/* ======================= follower receive (JC/core/NodeImpl.java) ========== */

void jo_append_entries_verify(uint32_t R, const uint32_t *req_off, const int64_t *prev_log_index,
                              const int64_t *term, const uint8_t *type, const int64_t *data_len,
                              const uint64_t *peer_xor, const uint64_t *checksum,
                              const uint8_t *has_checksum, const uint8_t *data,
                              uint64_t *checksum_out, uint8_t *corrupt_out, int32_t *first_corrupt) {
    size_t pos = 0; /* allData position: requests are back to back */
    for (uint32_t r = 0; r < R; ++r) {
        int64_t index = prev_log_index[r]; /* long index = prevLogIndex (:1763) */
        first_corrupt[r] = -1;
        for (uint32_t i = req_off[r]; i < req_off[r + 1]; ++i) {
            index++;
            corrupt_out[i] = 0;
            if (type[i] == 0) { /* ENTRY_TYPE_UNKNOWN: logEntryFromMeta returns null */
                checksum_out[i] = jo_logentry_checksum(0, index, term[i], peer_xor ? peer_xor[i] : 0,
                                                       NULL, 0);
                continue;
            }
            const size_t len = (size_t)(data_len[i] > 0 ? data_len[i] : 0);
            const uint64_t c = jo_logentry_checksum(type[i], index, term[i], peer_xor ? peer_xor[i] : 0,
                                                    data + pos, len);
            pos += len;
            checksum_out[i] = c;
            const int has = has_checksum == NULL || has_checksum[i];
            corrupt_out[i] = (uint8_t)(has && checksum[i] != c);
            if (corrupt_out[i] && first_corrupt[r] < 0) first_corrupt[r] = (int32_t)(i - req_off[r]);
        }
    }
}

/* ======================= leader lease (JC/core/NodeImpl.java) ============== */

static int32_t mask_to_ids(uint32_t mask, int32_t *ids);

int jo_check_dead_nodes(const int32_t *peers, int32_t n, const int64_t *ts, int32_t self,
                        int64_t now_ms, int64_t lease_timeout_ms, int64_t *lease_start,
                        uint32_t *dead_mask) {
    int alive = 0;
    int64_t start = INT64_MAX; /* long startLease = Long.MAX_VALUE */
    for (int32_t i = 0; i < n; ++i) {
        const int32_t p = peers[i];
        if (p == self) { /* peer.equals(this.serverId) */
            alive++;
            continue;
        }
        /* monotonicNowMs - lastRpcSendTimestamp, Java long (wrapping) arithmetic */
        const int64_t age = (int64_t)((uint64_t)now_ms - (uint64_t)ts[p]);
        if (age <= lease_timeout_ms) {
            alive++;
            if (start > ts[p]) start = ts[p];
            continue;
        }
        *dead_mask |= 1u << p;
    }
    if (alive >= n / 2 + 1) {
        *lease_start = start; /* updateLastLeaderTimestamp(startLease) */
        return 1;
    }
    return 0;
}

void jo_lease_check(uint32_t G, uint32_t P, const int64_t *ts, const uint64_t *conf,
                    const uint8_t *self_slot, int64_t now_ms, int64_t lease_timeout_ms,
                    uint8_t *ok, int64_t *lease_start, uint16_t *dead) {
    int64_t *t = (int64_t *)malloc(sizeof(int64_t) * (P ? P : 1));
    for (uint32_t g = 0; g < G; ++g) {
        for (uint32_t p = 0; p < P; ++p) t[p] = ts[(size_t)p * G + g];
        int32_t nids[16], oids[16];
        const int32_t nn = mask_to_ids((uint32_t)(conf[g] & 0xFFFF), nids);
        const int32_t no = mask_to_ids((uint32_t)((conf[g] >> 16) & 0xFFFF), oids);
        uint32_t dm = 0;
        uint8_t k = 0;
        if (jo_check_dead_nodes(nids, nn, t, self_slot[g], now_ms, lease_timeout_ms, &lease_start[g], &dm))
            k |= 1;
        if (no > 0) { /* if (!this.conf.getOldConf().isEmpty()) */
            if (jo_check_dead_nodes(oids, no, t, self_slot[g], now_ms, lease_timeout_ms, &lease_start[g], &dm))
                k |= 2;
        } else {
            k |= 2;
        }
        ok[g] = k;
        if (dead) dead[g] = (uint16_t)dm;
    }
    free(t);
}

/* ReadIndex, ReadOnlySafe (JC/core/NodeImpl.java:1343-1396): getQuorum (:1321-1327), then
 * ReadIndexHeartbeatResponseClosure (:1246-1291) run on each heartbeat response in arrival
 * order -- position 1..15 from order's nibble per slot, equal positions in slot order --
 * from the conf peers the leader sent a heartbeat to (every peer but itself). */
uint8_t jo_readindex_round(uint32_t mask, uint32_t P, uint32_t self, uint64_t order, uint32_t ok_mask) {
    int32_t ids[16];
    /* a conf naming a slot >= P: outside the batch contract (include/jrq.h), reported INVALID */
    if (P < 16 && (mask >> P) != 0) return 3;
    const int32_t n = mask_to_ids(mask, ids); /* conf.getConf().getPeers() */
    const int32_t quorum = n == 0 ? 0 : n / 2 + 1;
    if (quorum <= 1) return 1; /* "Only one peer, fast path": success */
    const int32_t failPeersThreshold = n % 2 == 0 ? (quorum - 1) : quorum;
    int32_t ackSuccess = 0, ackFailures = 0;
    for (uint32_t pos = 1; pos < 16; ++pos) {
        for (int32_t i = 0; i < n; ++i) {
            const uint32_t p = (uint32_t)ids[i];
            if (p == self || p >= P || ((order >> (4 * p)) & 0xF) != pos) continue;
            if ((ok_mask >> p) & 1u) ackSuccess++; else ackFailures++;
            if (ackSuccess + 1 >= quorum) return 1;             /* respond success */
            else if (ackFailures >= failPeersThreshold) return 2; /* respond !success */
        }
    }
    return 0; /* not decided yet */
}

void jo_readindex_quorum(uint32_t G, uint32_t P, const uint64_t *conf, const uint8_t *self_slot,
                         const uint64_t *order, const uint16_t *ok_mask, uint8_t *result) {
    for (uint32_t g = 0; g < G; ++g)
        result[g] = jo_readindex_round((uint32_t)(conf[g] & 0xFFFF), P, self_slot[g], order[g], ok_mask[g]);
}

/* ======================= Ballot (JC/entity/Ballot.java) ==================== */

static void list_init(jo_peer_list *l, const int32_t *ids, int32_t n) {
    l->n = 0;
    if (n > JO_MAX_CONF) {
        fprintf(stderr, "jraft_oracle: conf larger than JO_MAX_CONF\n");
        abort();
    }
    for (int32_t i = 0; i < n; ++i) {
        l->peer[i] = ids[i];
        l->found[i] = 0;
    }
    l->n = n > 0 ? n : 0;
}

/* Ballot.init (:63-85): peers from conf (learners never iterate, JC/conf/Configuration.java:184-186),
 * quorum = size/2+1; oldQuorum = 0 when oldConf == null, else oldSize/2+1. */
int jo_ballot_init(jo_ballot *b, const int32_t *conf, int32_t nconf, const int32_t *old, int32_t nold) {
    list_init(&b->peers, conf, nconf);
    list_init(&b->old_peers, old, 0);
    b->quorum = b->old_quorum = 0;
    b->quorum = b->peers.n / 2 + 1;
    if (nold < 0) return 1;
    list_init(&b->old_peers, old, nold);
    b->old_quorum = b->old_peers.n / 2 + 1;
    return 1;
}

/* Ballot.findPeer (:87-98): the hint slot if it holds the peer, else the first equal slot. */
static int find_peer(const jo_peer_list *l, int32_t peer, int32_t hint) {
    if (hint < 0 || hint >= l->n || l->peer[hint] != peer) {
        for (int32_t i = 0; i < l->n; ++i)
            if (l->peer[i] == peer) return i;
        return -1;
    }
    return hint;
}

/* Ballot.grant(peerId, hint) (:100-127). */
jo_pos_hint jo_ballot_grant_hint(jo_ballot *b, int32_t peer, jo_pos_hint hint) {
    int i = find_peer(&b->peers, peer, hint.pos0);
    if (i >= 0) {
        if (!b->peers.found[i]) {
            b->peers.found[i] = 1;
            b->quorum--;
        }
        hint.pos0 = i;
    } else {
        hint.pos0 = -1;
    }
    if (b->old_peers.n == 0) {
        hint.pos1 = -1;
        return hint;
    }
    i = find_peer(&b->old_peers, peer, hint.pos1);
    if (i >= 0) {
        if (!b->old_peers.found[i]) {
            b->old_peers.found[i] = 1;
            b->old_quorum--;
        }
        hint.pos1 = i;
    } else {
        hint.pos1 = -1;
    }
    return hint;
}

void jo_ballot_grant(jo_ballot *b, int32_t peer) {
    jo_pos_hint h = {-1, -1};
    (void)jo_ballot_grant_hint(b, peer, h);
}

int jo_ballot_is_granted(const jo_ballot *b) { return b->quorum <= 0 && b->old_quorum <= 0; }

/* ======================= BallotBox (JC/core/BallotBox.java) ================ */

struct jo_ballot_box {
    int64_t last_committed_index; /* :53 */
    int64_t pending_index;        /* :54 */
    /* pendingMetaQueue (:55): util.ArrayDeque is an ArrayList whose removeRange(0,k)
     * drops the head (JC/util/ArrayDeque.java:106-109); kept here as array + head. */
    jo_ballot *q;
    int64_t head, tail, cap;
    int64_t on_committed_calls, on_committed_last; /* the FSMCaller waiter */
    int64_t grants;                                /* Ballot.grant calls executed */
};

jo_ballot_box *jo_bb_new(void) {
    jo_ballot_box *bb = (jo_ballot_box *)calloc(1, sizeof *bb);
    return bb;
}

void jo_bb_free(jo_ballot_box *bb) {
    if (!bb) return;
    free(bb->q);
    free(bb);
}

int64_t jo_bb_last_committed_index(const jo_ballot_box *bb) { return bb->last_committed_index; }
int64_t jo_bb_pending_index(const jo_ballot_box *bb) { return bb->pending_index; }
int64_t jo_bb_queue_size(const jo_ballot_box *bb) { return bb->tail - bb->head; }
int64_t jo_bb_on_committed_calls(const jo_ballot_box *bb) { return bb->on_committed_calls; }
int64_t jo_bb_on_committed_last(const jo_ballot_box *bb) { return bb->on_committed_last; }

static void on_committed(jo_ballot_box *bb, int64_t idx) {
    bb->on_committed_calls++;
    bb->on_committed_last = idx;
}

/* BallotBox.commitAt (:96-139). */
int jo_bb_commit_at(jo_ballot_box *bb, int64_t first, int64_t last, int32_t peer) {
    int64_t last_committed = 0;
    if (bb->pending_index == 0) return JO_FALSE;
    if (last < bb->pending_index) return JO_TRUE;
    if (last >= bb->pending_index + (bb->tail - bb->head)) return JO_AIOOBE;
    int64_t start_at = first > bb->pending_index ? first : bb->pending_index;
    jo_pos_hint hint = {-1, -1};
    for (int64_t log_index = start_at; log_index <= last; ++log_index) {
        jo_ballot *bl = &bb->q[bb->head + (log_index - bb->pending_index)];
        hint = jo_ballot_grant_hint(bl, peer, hint);
        bb->grants++;
        if (jo_ballot_is_granted(bl)) last_committed = log_index;
    }
    if (last_committed == 0) return JO_TRUE;
    bb->head += (last_committed - bb->pending_index) + 1; /* removeRange(0, lc - pending + 1) */
    bb->pending_index = last_committed + 1;
    bb->last_committed_index = last_committed;
    on_committed(bb, last_committed); /* after unlock in the reference */
    return JO_TRUE;
}

/* BallotBox.clearPendingTasks (:147-156). */
void jo_bb_clear_pending_tasks(jo_ballot_box *bb) {
    bb->head = bb->tail = 0;
    bb->pending_index = 0;
}

/* BallotBox.resetPendingIndex (:167-186). */
int jo_bb_reset_pending_index(jo_ballot_box *bb, int64_t n) {
    if (!(bb->pending_index == 0 && bb->tail == bb->head)) return JO_FALSE;
    if (n <= bb->last_committed_index) return JO_FALSE;
    bb->pending_index = n;
    bb->head = bb->tail = 0;
    return JO_TRUE;
}

/* BallotBox.appendPendingTask (:197-215). */
int jo_bb_append_pending_task(jo_ballot_box *bb, const int32_t *conf, int32_t nconf,
                              const int32_t *old, int32_t nold) {
    jo_ballot bl;
    if (!jo_ballot_init(&bl, conf, nconf, old, nold)) return JO_FALSE;
    if (bb->pending_index <= 0) return JO_FALSE;
    if (bb->tail == bb->cap) {
        if (bb->head > 0) { /* compact, keeps queue order */
            memmove(bb->q, bb->q + bb->head, (size_t)(bb->tail - bb->head) * sizeof(jo_ballot));
            bb->tail -= bb->head;
            bb->head = 0;
        }
        if (bb->tail == bb->cap) {
            int64_t nc = bb->cap ? bb->cap * 2 : 64;
            jo_ballot *nq = (jo_ballot *)realloc(bb->q, (size_t)nc * sizeof(jo_ballot));
            if (!nq) abort();
            bb->q = nq;
            bb->cap = nc;
        }
    }
    bb->q[bb->tail++] = bl;
    return JO_TRUE;
}

/* BallotBox.setLastCommittedIndex (:223-248). */
int jo_bb_set_last_committed_index(jo_ballot_box *bb, int64_t idx) {
    if (bb->pending_index != 0 || bb->tail != bb->head) {
        if (!(idx < bb->pending_index)) return JO_IAE; /* Requires.requireTrue */
        return JO_FALSE;
    }
    if (idx < bb->last_committed_index) return JO_FALSE;
    if (idx > bb->last_committed_index) {
        bb->last_committed_index = idx;
        on_committed(bb, idx);
    }
    return JO_TRUE;
}

/* ======================= epoch replay ===================================== */

static int32_t mask_to_ids(uint32_t mask, int32_t *ids) {
    int32_t n = 0;
    for (int32_t s = 0; s < 16; ++s)
        if (mask & (1u << s)) ids[n++] = s;
    return n;
}

int64_t jo_quorum_epoch_replay(uint32_t G, uint32_t P, const int64_t *match, const int64_t *pending_index,
                               const int64_t *last_appended, const int64_t *last_committed,
                               const uint64_t *conf, const uint32_t *run_off, const int64_t *run_start,
                               const uint64_t *run_conf, int64_t chunk, int64_t *committed_out,
                               uint8_t *status_out) {
    int64_t grants = 0;
    if (chunk <= 0) chunk = 1;
    jo_ballot_box *bb = jo_bb_new();
    int64_t *next = (int64_t *)malloc(sizeof(int64_t) * (P ? P : 1));
    for (uint32_t g = 0; g < G; ++g) {
        /* fresh box seeded to the group's state: follower path sets lastCommitted,
         * then the leader's resetPendingIndex (NodeImpl.becomeLeader). */
        bb->head = bb->tail = 0;
        bb->pending_index = 0;
        bb->last_committed_index = 0;
        bb->on_committed_calls = 0;
        bb->grants = 0;
        const int64_t lc0 = last_committed[g], pi = pending_index[g], la = last_appended[g];
        uint8_t st = JO_ST_OK;
        jo_bb_set_last_committed_index(bb, lc0);
        if (pi == 0) {
            committed_out[g] = lc0;
            status_out[g] = JO_ST_NOT_LEADER;
            continue;
        }
        if (jo_bb_reset_pending_index(bb, pi) != JO_TRUE) {
            fprintf(stderr, "jraft_oracle: group %u violates pendingIndex > lastCommitted\n", g);
            abort();
        }
        /* appendPendingTask for each pending index with the conf of its run. */
        uint32_t r0 = run_off ? run_off[g] : 0, r1 = run_off ? run_off[g + 1] : 1;
        uint32_t r = r0;
        for (int64_t i = pi; i <= la; ++i) {
            uint64_t cw;
            if (run_off) {
                while (r + 1 < r1 && run_start[r + 1] <= i) ++r;
                cw = run_conf[r];
            } else {
                cw = conf[g];
            }
            int32_t nids[16], oids[16];
            int32_t nn = mask_to_ids((uint32_t)(cw & 0xFFFF), nids);
            int32_t no = ((cw >> 40) & 0xFF) ? mask_to_ids((uint32_t)((cw >> 16) & 0xFFFF), oids) : -1;
            if (nn == 0) st |= JO_ST_EMPTY_CONF;
            jo_bb_append_pending_task(bb, nids, nn, oids, no);
        }
        /* acks, Replicator-style: contiguous chunks, round-robin over peers. */
        for (uint32_t p = 0; p < P; ++p) next[p] = pi;
        for (uint32_t p = 0; p < P; ++p) {
            if (match[(size_t)p * G + g] > la) {
                int rc = jo_bb_commit_at(bb, pi, match[(size_t)p * G + g], (int32_t)p);
                if (rc == JO_AIOOBE) st |= JO_ST_OUT_OF_RANGE;
                next[p] = INT64_MAX; /* this peer's ack threw: no grants from it */
            }
        }
        for (;;) {
            int any = 0;
            for (uint32_t p = 0; p < P; ++p) {
                const int64_t m = match[(size_t)p * G + g];
                if (next[p] == INT64_MAX || next[p] > m) continue;
                int64_t last = next[p] + chunk - 1;
                if (last > m) last = m;
                jo_bb_commit_at(bb, next[p], last, (int32_t)p);
                next[p] = last + 1;
                any = 1;
            }
            if (!any) break;
        }
        committed_out[g] = bb->last_committed_index;
        status_out[g] = st;
        grants += bb->grants;
    }
    free(next);
    jo_bb_free(bb);
    return grants;
}


/* ---------------- commit fan-out (ClosureQueueImpl, FSMCallerImpl) -------- */

/* ClosureQueueImpl (JC/closure/ClosureQueueImpl.java:45-142) with closures as the log index
 * they were appended for (a LinkedList in the reference; a ring of ids here). */
typedef struct {
    int64_t first_index;
    int64_t *ids;
    int64_t head, size;
} jo_closure_queue;

/* popClosureUntil(endIndex, closures) (:113-142); returns the first index or endIndex+1 / -1,
 * and the number popped in *popped. */
static int64_t jo_cq_pop_until(jo_closure_queue *q, int64_t end_index, int64_t *popped) {
    *popped = 0;
    const int64_t queue_size = q->size;
    if (queue_size == 0 || end_index < q->first_index) return end_index + 1;
    if (end_index > q->first_index + queue_size - 1) return -1; /* LOG.error + return -1 */
    const int64_t out_first = q->first_index;
    for (int64_t i = out_first; i <= end_index; i++) { /* queue.pollFirst() per index */
        (void)q->ids[q->head];
        q->head++;
        q->size--;
        (*popped)++;
    }
    q->first_index = end_index + 1;
    return out_first;
}

int64_t jo_commit_fanout_replay(uint32_t G, const uint64_t *seq_off, const int64_t *seq,
                                int64_t *last_applied, int64_t *cq_first, int64_t *cq_size,
                                int64_t *first_closure, uint8_t *status) {
    int64_t total = 0;
    for (uint32_t g = 0; g < G; g++) {
        jo_closure_queue q;
        q.first_index = cq_first[g];
        q.head = 0;
        q.size = cq_size[g];
        q.ids = (int64_t *)malloc((size_t)(q.size > 0 ? q.size : 1) * sizeof(int64_t));
        for (int64_t i = 0; i < q.size; i++) q.ids[i] = q.first_index + i; /* appendPendingClosure */
        uint8_t st = seq_off[g] == seq_off[g + 1] ? JO_FAN_NONE : JO_FAN_SKIP;
        int64_t first = 0, first_pop = 0, last_c = 0;
        int have_first = 0;
        for (uint64_t k = seq_off[g]; k < seq_off[g + 1]; k++) {
            const int64_t c = seq[k]; /* FSMCallerImpl.doCommitted(c) */
            if (last_applied[g] >= c) continue; /* :466-470 */
            int64_t popped;
            const int64_t r = jo_cq_pop_until(&q, c, &popped);
            if (r < 0) { /* Requires.requireTrue(firstClosureIndex >= 0) throws (:480) */
                st = JO_FAN_INVALID;
                break;
            }
            total += popped;
            if (popped > 0 && !have_first) {
                first_pop = r;
                have_first = 1;
            }
            last_c = c;
            st = JO_FAN_APPLY;
            last_applied[g] = c; /* setLastApplied after the iterator ran to c */
        }
        if (st == JO_FAN_APPLY) first = have_first ? first_pop : last_c + 1;
        else if (st == JO_FAN_INVALID) first = -1;
        first_closure[g] = first;
        status[g] = st;
        cq_first[g] = q.first_index;
        cq_size[g] = q.size;
        free(q.ids);
    }
    return total;
}

/* ---------------- V2 log entry decode + verify (entity/codec/v2) ----------- */

/* CodedInputStream over one record body (protobuf-java 3.5.1, the reference's pinned version,
 * pom.xml:74; array-backed decoder semantics). */
typedef struct {
    const uint8_t *b;
    int64_t pos, limit;
    uint32_t last_tag;
    int err; /* InvalidProtocolBufferException raised */
} jo_cis;

static uint8_t jo_cis_byte(jo_cis *in) {
    if (in->pos >= in->limit) {
        in->err = 1; /* truncatedMessage */
        return 0;
    }
    return in->b[in->pos++];
}

/* readRawVarint32: 5 bytes of value; a 5th byte with its high bit set is followed by up to
 * 5 discarded bytes; more -> malformedVarint. */
static uint32_t jo_cis_varint32(jo_cis *in) {
    uint32_t r = 0;
    for (int i = 0; i < 5; i++) {
        const uint8_t x = jo_cis_byte(in);
        if (in->err) return 0;
        r |= (uint32_t)(x & 0x7F) << (7 * i);
        if (!(x & 0x80)) return r;
    }
    for (int i = 0; i < 5; i++) {
        const uint8_t x = jo_cis_byte(in);
        if (in->err) return 0;
        if (!(x & 0x80)) return r;
    }
    in->err = 1;
    return 0;
}

/* readRawVarint64: up to 10 bytes, bits past 64 dropped; an 11th byte -> malformedVarint. */
static uint64_t jo_cis_varint64(jo_cis *in) {
    uint64_t r = 0;
    for (int shift = 0; shift < 64; shift += 7) {
        const uint8_t x = jo_cis_byte(in);
        if (in->err) return 0;
        r |= (uint64_t)(x & 0x7F) << shift;
        if (!(x & 0x80)) return r;
    }
    in->err = 1;
    return 0;
}

/* readTag: 0 at the end of input; field number 0 -> invalidTag. */
static uint32_t jo_cis_tag(jo_cis *in) {
    if (in->pos >= in->limit) {
        in->last_tag = 0;
        return 0;
    }
    in->last_tag = jo_cis_varint32(in);
    if (!in->err && (in->last_tag >> 3) == 0) in->err = 1;
    return in->err ? 0 : in->last_tag;
}

/* length-delimited payload: returns its offset, *len its size */
static int64_t jo_cis_bytes(jo_cis *in, int64_t *len) {
    const int32_t size = (int32_t)jo_cis_varint32(in);
    if (in->err) return 0;
    if (size < 0 || size > in->limit - in->pos) { /* negativeSize / truncatedMessage */
        in->err = 1;
        return 0;
    }
    const int64_t at = in->pos;
    in->pos += size;
    *len = size;
    return at;
}

static int jo_cis_skip_field(jo_cis *in, uint32_t tag, int depth);

/* UnknownFieldSet.mergeFieldFrom for a START_GROUP: readGroup (recursion limit 100) until the
 * matching END_GROUP tag. */
static void jo_cis_skip_group(jo_cis *in, uint32_t field, int depth) {
    if (depth + 1 >= 100) { /* recursionLimitExceeded */
        in->err = 1;
        return;
    }
    for (;;) {
        const uint32_t t = jo_cis_tag(in);
        if (in->err) return;
        if (t == 0 || !jo_cis_skip_field(in, t, depth + 1)) break;
        if (in->err) return;
    }
    if (in->last_tag != ((field << 3) | 4)) in->err = 1; /* checkLastTagWas(END_GROUP) */
}

/* skipField/mergeFieldFrom: 0 = END_GROUP seen (stop), 1 = skipped */
static int jo_cis_skip_field(jo_cis *in, uint32_t tag, int depth) {
    int64_t len;
    switch (tag & 7) {
    case 0: (void)jo_cis_varint64(in); return 1;
    case 1: for (int i = 0; i < 8; i++) (void)jo_cis_byte(in); return 1;
    case 2: (void)jo_cis_bytes(in, &len); return 1;
    case 3: jo_cis_skip_group(in, tag >> 3, depth); return 1;
    case 4: return 0;
    case 5: for (int i = 0; i < 4; i++) (void)jo_cis_byte(in); return 1;
    default: in->err = 1; return 1; /* invalidWireType */
    }
}

static int jo_is_java_whitespace(uint8_t c) {
    return c == ' ' || (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x1F);
}

/* Integer.parseInt over latin-1 chars: optional sign, ASCII digits, int32 range. */
static int jo_parse_int(const uint8_t *s, int64_t n, int32_t *out) {
    int64_t i = 0, v = 0;
    int neg = 0;
    if (n == 0) return 0;
    if (s[0] == '-' || s[0] == '+') {
        neg = s[0] == '-';
        i = 1;
        if (n == 1) return 0;
    }
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return 0;
        v = v * 10 + (s[i] - '0');
        if (v > 2147483648LL) return 0;
    }
    if (neg) v = -v;
    if (v > 2147483647LL || v < -2147483648LL) return 0;
    *out = (int32_t)v;
    return 1;
}

/* JRaftUtils.getPeerId(AsciiStringUtil.unsafeDecode(bytes)).checksum()
 * (JC/JRaftUtils.java:113-122, JC/entity/PeerId.java:60-65,135-171): blank -> the empty
 * PeerId "0.0.0.0:0"; else StringUtils.split(s, ':') (empty tokens dropped), 2 or 3 tokens,
 * Integer.parseInt port [and idx]; toString = ip ":" port [":" idx if idx != 0].
 * *kind: 0 = the bytes are already the canonical toString, 1 = parsed but re-rendered
 * differently, 2 = IllegalArgumentException ("Invalid peer str"). */
uint64_t jo_v2_peer_checksum(const uint8_t *s, int64_t n, int *kind) {
    int blank = 1;
    for (int64_t i = 0; i < n; i++)
        if (!jo_is_java_whitespace(s[i])) blank = 0;
    char buf[1024];
    int len;
    if (blank) {
        len = snprintf(buf, sizeof buf, "0.0.0.0:0");
    } else {
        int64_t tb[4], te[4];
        int nt = 0;
        for (int64_t i = 0; i < n;) {
            while (i < n && s[i] == ':') i++;
            if (i >= n) break;
            const int64_t b = i;
            while (i < n && s[i] != ':') i++;
            if (nt < 4) {
                tb[nt] = b;
                te[nt] = i;
            }
            nt++;
        }
        int32_t port = 0, idx = 0;
        if ((nt != 2 && nt != 3) || !jo_parse_int(s + tb[1], te[1] - tb[1], &port) ||
            (nt == 3 && !jo_parse_int(s + tb[2], te[2] - tb[2], &idx))) {
            *kind = 2;
            return 0;
        }
        const int64_t iplen = te[0] - tb[0];
        if (iplen > 900) {
            *kind = 2;
            return 0;
        }
        memcpy(buf, s + tb[0], (size_t)iplen);
        len = (int)iplen;
        len += idx != 0 ? snprintf(buf + len, sizeof buf - (size_t)len, ":%d:%d", port, idx)
                        : snprintf(buf + len, sizeof buf - (size_t)len, ":%d", port);
    }
    *kind = (len == n && memcmp(buf, s, (size_t)n) == 0) ? 0 : 1;
    return jo_crc64((const uint8_t *)buf, (size_t)len);
}

void jo_v2_decode_batch(const uint8_t *rec, const uint64_t *off, uint32_t n, uint8_t *status,
                        uint8_t *type, int64_t *index, int64_t *term, uint64_t *stored,
                        uint8_t *has_checksum, uint64_t *data_off, uint64_t *data_len,
                        uint32_t *peer_counts, uint64_t *computed, uint8_t *corrupt) {
    static const uint8_t MAGIC0 = 0xBB, MAGIC1 = 0xD2, VERSION = 1; /* LogEntryV2CodecFactory.java:52-57 */
    const int HEADER = 6;
    for (uint32_t r = 0; r < n; r++) {
        const uint8_t *bs = rec + off[r];
        const int64_t L = (int64_t)(off[r + 1] - off[r]);
        uint8_t st = JO_V2_OK;
        int64_t idx = 0, tm = 0, doff = (int64_t)off[r], dlen = 0;
        uint64_t ck = 0, pxor = 0;
        int have_type = 0, have_term = 0, have_index = 0, have_data = 0, have_ck = 0, worst = 0;
        int32_t etype = 0;
        uint32_t counts = 0;
        /* AutoDetectDecoder.decode (JC/entity/codec/AutoDetectDecoder.java:41-52) */
        if (L < 1) st = JO_V2_NULL;
        else if (bs[0] != MAGIC0) st = JO_V2_V1;
        /* V2Decoder.decode (JC/entity/codec/v2/V2Decoder.java:46-63) */
        else if (L < HEADER || bs[1] != MAGIC1 || bs[2] != VERSION) st = JO_V2_NULL;
        else {
            jo_cis in = {bs, HEADER, L, 0, 0};
            for (;;) { /* PBLogEntry parsing constructor (generated, log.proto:10-20) */
                const uint32_t tag = jo_cis_tag(&in);
                if (in.err || tag == 0) break;
                int64_t at, len;
                switch (tag) {
                case 8: { /* type: readEnum, unknown numbers go to the unknown fields */
                    const int32_t v = (int32_t)jo_cis_varint32(&in);
                    if (!in.err && v >= 0 && v <= 3) {
                        etype = v;
                        have_type = 1;
                    }
                    break;
                }
                case 16: tm = (int64_t)jo_cis_varint64(&in); have_term = 1; break;
                case 24: idx = (int64_t)jo_cis_varint64(&in); have_index = 1; break;
                case 34: case 42: case 66: case 74: { /* peers, old_peers, learners, old_learners */
                    at = jo_cis_bytes(&in, &len);
                    if (in.err) break;
                    int kind;
                    pxor ^= jo_v2_peer_checksum(bs + at, len, &kind);
                    if (kind > worst) worst = kind;
                    const int list = tag == 34 ? 0 : tag == 42 ? 1 : tag == 66 ? 2 : 3;
                    if (((counts >> (8 * list)) & 0xFF) != 0xFF) counts += 1u << (8 * list);
                    break;
                }
                case 50: /* data: the last occurrence wins */
                    at = jo_cis_bytes(&in, &len);
                    if (!in.err) {
                        doff = (int64_t)off[r] + at;
                        dlen = len;
                        have_data = 1;
                    }
                    break;
                case 56: ck = jo_cis_varint64(&in); have_ck = 1; break;
                default:
                    if (!jo_cis_skip_field(&in, tag, 0)) goto end_group; /* END_GROUP stops */
                }
                if (in.err) break;
            }
            if (0) {
            end_group:
                in.err = 1; /* checkLastTagWas(0) fails after a top-level END_GROUP */
            }
            /* required type/term/index/data (isInitialized) */
            if (in.err || !have_type || !have_term || !have_index || !have_data) st = JO_V2_NULL;
            else if (worst == 2) st = JO_V2_PEER_THROWS;
            else if (worst == 1) st = JO_V2_PEER_NONCANON;
        }
        const int ok = st == JO_V2_OK || st == JO_V2_PEER_NONCANON;
        if (!ok) {
            etype = 0;
            idx = tm = 0;
            ck = 0;
            have_ck = 0;
            doff = (int64_t)off[r];
            dlen = 0;
            counts = 0;
        }
        /* LogEntry.checksum / isCorrupted (JC/entity/LogEntry.java:88-108,156-158) */
        const uint64_t c = ok ? jo_logentry_checksum(etype, idx, tm, pxor, rec + doff, (size_t)dlen) : 0;
        status[r] = st;
        type[r] = (uint8_t)etype;
        index[r] = idx;
        term[r] = tm;
        stored[r] = ck;
        has_checksum[r] = (uint8_t)have_ck;
        data_off[r] = (uint64_t)doff;
        data_len[r] = (uint64_t)dlen;
        if (peer_counts) peer_counts[r] = counts;
        computed[r] = c;
        corrupt[r] = (uint8_t)(ok && have_ck && ck != c);
    }
}
