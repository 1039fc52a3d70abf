/*
 * jrq_jni_core.c -- see jrq_jni_core.h.  Each function: check the Java ints, cast the Java longs
 * to the exact pointer types of one include/jrq.h entry point, call it.  Nothing else: no state,
 * no allocation, no second code path.
 */
#include "jrq_jni_core.h"

#include <stddef.h>

#include "jrq.h"

/* a Java long holding an address -> typed pointer */
#define A(T, a) ((T)(intptr_t)(a))
/* a Java int count -> uint32_t, refusing negatives (Java has no unsigned int) */
#define N(x)                                                                                   \
    do {                                                                                       \
        if ((x) < 0) return JRQ_E_INVALID;                                                     \
    } while (0)

jrq_addr jrq_jni_create(int32_t device, int32_t max_groups, int32_t max_peers, jrq_addr err_out) {
    int err = 0;
    jrq_engine *e = NULL;
    if (max_groups < 0 || max_peers <= 0 || max_peers > JRQ_MAX_PEERS) {
        err = JRQ_E_INVALID;
    } else {
        e = jrq_create(device, (uint32_t)max_groups, (uint8_t)max_peers, &err);
    }
    if (err_out) *A(int32_t *, err_out) = (int32_t)err;
    return (jrq_addr)(intptr_t)e;
}

void jrq_jni_destroy(jrq_addr eng) { jrq_destroy(A(jrq_engine *, eng)); }

int32_t jrq_jni_abi_version(void) { return jrq_abi_version(); }

const char *jrq_jni_build_id(void) { return jrq_build_id(); }

const char *jrq_jni_last_error(jrq_addr eng) { return jrq_last_error(A(const jrq_engine *, eng)); }

int32_t jrq_jni_synchronize(jrq_addr eng) { return jrq_synchronize(A(jrq_engine *, eng)); }

int32_t jrq_jni_host_register(jrq_addr ptr, int64_t bytes) {
    if (bytes < 0) return JRQ_E_INVALID;
    return jrq_host_register(A(void *, ptr), (size_t)bytes);
}

int32_t jrq_jni_host_unregister(jrq_addr ptr) { return jrq_host_unregister(A(void *, ptr)); }

int64_t jrq_jni_host_registered_bytes(jrq_addr ptr) {
    size_t bytes = 0;
    int rc = jrq_host_registered_bytes(A(const void *, ptr), &bytes);
    return rc < 0 ? (int64_t)rc : (int64_t)bytes;
}

jrq_addr jrq_jni_host_alloc(int64_t bytes) {
    void *p = NULL;
    if (bytes <= 0 || jrq_host_alloc((size_t)bytes, &p) != JRQ_OK) return 0;
    return (jrq_addr)(intptr_t)p;
}

int32_t jrq_jni_host_free(jrq_addr ptr) { return jrq_host_free(A(void *, ptr)); }

int32_t jrq_jni_quorum_epoch(jrq_addr eng, jrq_addr match, jrq_addr pending_index,
                             jrq_addr last_appended, jrq_addr last_committed, jrq_addr conf,
                             jrq_addr run_off, jrq_addr run_start, jrq_addr run_conf,
                             int32_t num_peers, int32_t num_runs, int32_t G,
                             jrq_addr committed_out, jrq_addr status_out) {
    jrq_group_batch b;
    N(num_peers);
    N(num_runs);
    N(G);
    b.match = A(const int64_t *, match);
    b.pending_index = A(const int64_t *, pending_index);
    b.last_appended = A(const int64_t *, last_appended);
    b.last_committed = A(const int64_t *, last_committed);
    b.conf = A(const uint64_t *, conf);
    b.run_off = A(const uint32_t *, run_off);
    b.run_start = A(const int64_t *, run_start);
    b.run_conf = A(const uint64_t *, run_conf);
    b.num_peers = (uint32_t)num_peers;
    b.num_runs = (uint32_t)num_runs;
    b.match_ld = (uint64_t)G; /* one direct buffer of P rows of G longs */
    return jrq_quorum_epoch(A(jrq_engine *, eng), &b, A(int64_t *, committed_out),
                            A(uint8_t *, status_out), (uint32_t)G);
}

int32_t jrq_jni_quorum_epoch_tiles(jrq_addr eng, jrq_addr tiles, int32_t num_peers,
                                   jrq_addr run_off, jrq_addr run_start, jrq_addr run_conf,
                                   int32_t G, jrq_addr committed_out, jrq_addr status_out) {
    jrq_group_tiles t;
    N(num_peers);
    N(G);
    t.tiles = A(const int64_t *, tiles);
    t.num_peers = (uint32_t)num_peers;
    t.run_off = A(const uint32_t *, run_off);
    t.run_start = A(const int64_t *, run_start);
    t.run_conf = A(const uint64_t *, run_conf);
    return jrq_quorum_epoch_tiles(A(jrq_engine *, eng), &t, A(int64_t *, committed_out),
                                  A(uint8_t *, status_out), (uint32_t)G);
}

jrq_addr jrq_jni_table_create(jrq_addr eng, int32_t G, int32_t num_peers, jrq_addr err_out) {
    int err = 0;
    jrq_table *t = NULL;
    if (G < 0 || num_peers < 0) {
        err = JRQ_E_INVALID;
    } else {
        t = jrq_table_create(A(jrq_engine *, eng), (uint32_t)G, (uint32_t)num_peers, &err);
    }
    if (err_out) *A(int32_t *, err_out) = (int32_t)err;
    return (jrq_addr)(intptr_t)t;
}

void jrq_jni_table_destroy(jrq_addr table) { jrq_table_destroy(A(jrq_table *, table)); }

int32_t jrq_jni_table_update(jrq_addr table, jrq_addr states, int32_t n_states, jrq_addr recs,
                             int32_t n_recs) {
    N(n_states);
    N(n_recs);
    return jrq_table_update(A(jrq_table *, table), A(const jrq_group_state *, states),
                            (uint32_t)n_states, A(const uint64_t *, recs), (uint32_t)n_recs);
}

int32_t jrq_jni_table_update_gather(jrq_addr table, int32_t parts, jrq_addr states,
                                    jrq_addr n_states, jrq_addr recs, jrq_addr n_recs) {
    enum { MAX_PARTS = 64 };
    const jrq_group_state *sp[MAX_PARTS];
    const uint64_t *rp[MAX_PARTS];
    uint32_t ns[MAX_PARTS], nr[MAX_PARTS];
    const jrq_addr *sa = A(const jrq_addr *, states), *ra = A(const jrq_addr *, recs);
    const int32_t *nsa = A(const int32_t *, n_states), *nra = A(const int32_t *, n_recs);
    int32_t i;
    if (parts < 0 || parts > MAX_PARTS || (parts > 0 && (!sa || !ra || !nsa || !nra)))
        return JRQ_E_INVALID;
    for (i = 0; i < parts; ++i) {
        N(nsa[i]);
        N(nra[i]);
        sp[i] = A(const jrq_group_state *, sa[i]);
        rp[i] = A(const uint64_t *, ra[i]);
        ns[i] = (uint32_t)nsa[i];
        nr[i] = (uint32_t)nra[i];
    }
    return jrq_table_update_gather(A(jrq_table *, table), (uint32_t)parts, sp, ns, rp, nr);
}

int32_t jrq_jni_table_stage_reserve(jrq_addr table, int32_t max_states, int32_t max_recs) {
    N(max_states);
    N(max_recs);
    return jrq_table_stage_reserve(A(jrq_table *, table), (uint32_t)max_states,
                                   (uint32_t)max_recs);
}

int32_t jrq_jni_table_stage(jrq_addr table, jrq_addr states, int32_t n_states, jrq_addr recs,
                            int32_t n_recs) {
    N(n_states);
    N(n_recs);
    return jrq_table_stage(A(jrq_table *, table), A(const jrq_group_state *, states),
                           (uint32_t)n_states, A(const uint64_t *, recs), (uint32_t)n_recs);
}

int32_t jrq_jni_table_stage_apply(jrq_addr table) {
    return jrq_table_stage_apply(A(jrq_table *, table));
}

int32_t jrq_jni_table_stage_reserve_acks(jrq_addr table, int32_t max_acks, int32_t max_segments) {
    N(max_acks);
    N(max_segments);
    return jrq_table_stage_reserve_acks(A(jrq_table *, table), (uint32_t)max_acks,
                                        (uint32_t)max_segments);
}

int32_t jrq_jni_table_stage_acks(jrq_addr table, int64_t stamp, jrq_addr acks, int32_t n) {
    N(n);
    if (stamp < 0) return JRQ_E_INVALID;
    return jrq_table_stage_acks(A(jrq_table *, table), (uint64_t)stamp, A(const uint64_t *, acks),
                                (uint32_t)n);
}

int32_t jrq_jni_table_ack_region(jrq_addr table, int64_t capacity, jrq_addr region_out) {
    uint64_t *r = NULL;
    int rc;
    if (capacity <= 0 || !region_out) return JRQ_E_INVALID;
    rc = jrq_table_ack_region(A(jrq_table *, table), (uint64_t)capacity, &r);
    if (rc == JRQ_OK) *A(jrq_addr *, region_out) = (jrq_addr)(intptr_t)r;
    return rc;
}

int32_t jrq_jni_table_ack_region_free(jrq_addr table, jrq_addr region) {
    return jrq_table_ack_region_free(A(jrq_table *, table), A(uint64_t *, region));
}

int32_t jrq_jni_table_ack_push(jrq_addr table, jrq_addr region_dst, jrq_addr host_src, int32_t from,
                               int32_t n) {
    N(from);
    N(n);
    if (!region_dst || !host_src) return JRQ_E_INVALID;
    return jrq_table_ack_push(A(jrq_table *, table), A(uint64_t *, region_dst) + from,
                              A(const uint64_t *, host_src) + from, (uint32_t)n);
}

int32_t jrq_jni_table_epoch(jrq_addr table, jrq_addr changed, jrq_addr status_out) {
    uint32_t n = 0;
    int rc = jrq_table_epoch(A(jrq_table *, table), A(uint64_t *, changed), &n,
                             A(uint8_t *, status_out));
    if (rc != JRQ_OK) return rc;
    return n > (uint32_t)INT32_MAX ? JRQ_E_INVALID : (int32_t)n;
}

int32_t jrq_jni_table_read(jrq_addr table, jrq_addr pending_index, jrq_addr last_appended,
                           jrq_addr last_committed, jrq_addr match) {
    return jrq_table_read(A(jrq_table *, table), A(int64_t *, pending_index),
                          A(int64_t *, last_appended), A(int64_t *, last_committed),
                          A(int64_t *, match));
}

int32_t jrq_jni_table_check(jrq_addr table) { return jrq_table_check(A(jrq_table *, table)); }

int32_t jrq_jni_table_fsm_update(jrq_addr table, jrq_addr groups, jrq_addr last_applied,
                                 jrq_addr cq_first, jrq_addr cq_size, int32_t n) {
    N(n);
    return jrq_table_fsm_update(A(jrq_table *, table), A(const uint32_t *, groups),
                                A(const int64_t *, last_applied), A(const int64_t *, cq_first),
                                A(const int64_t *, cq_size), (uint32_t)n);
}

int32_t jrq_jni_table_fsm_read(jrq_addr table, jrq_addr last_applied, jrq_addr cq_first,
                               jrq_addr cq_size) {
    return jrq_table_fsm_read(A(jrq_table *, table), A(int64_t *, last_applied),
                              A(int64_t *, cq_first), A(int64_t *, cq_size));
}

int32_t jrq_jni_table_epoch_fanout(jrq_addr table, jrq_addr changed, jrq_addr fan_first,
                                   jrq_addr fan_status) {
    uint32_t n = 0;
    int rc = jrq_table_epoch_fanout(A(jrq_table *, table), A(uint64_t *, changed), &n,
                                    A(int64_t *, fan_first), A(uint8_t *, fan_status));
    if (rc != JRQ_OK) return rc;
    return (int32_t)n;
}

/* jrq_addr words are handles; on an LP64 host they are pointer-sized, checked below */
typedef char jrq_jni_addr_is_a_pointer[sizeof(jrq_addr) == sizeof(void *) ? 1 : -1];

int32_t jrq_jni_rccl_init_all(jrq_addr engines, int32_t n) {
    if (n <= 0 || !engines) return JRQ_E_INVALID;
    return jrq_rccl_init_all(A(jrq_engine *const *, engines), n);
}

jrq_addr jrq_jni_snapshot_create(jrq_addr tables, int32_t n, jrq_addr err_out) {
    int err = 0;
    jrq_snapshot *s = NULL;
    if (n <= 0 || !tables) {
        err = JRQ_E_INVALID;
    } else {
        s = jrq_snapshot_create(A(jrq_table *const *, tables), n, &err);
    }
    if (err_out) *A(int32_t *, err_out) = (int32_t)err;
    return (jrq_addr)(intptr_t)s;
}

void jrq_jni_snapshot_destroy(jrq_addr snap) { jrq_snapshot_destroy(A(jrq_snapshot *, snap)); }

int32_t jrq_jni_snapshot_publish(jrq_addr snap) {
    return jrq_snapshot_publish(A(jrq_snapshot *, snap));
}

int32_t jrq_jni_snapshot_read(jrq_addr snap, int32_t i, jrq_addr host_out) {
    N(i);
    return jrq_snapshot_read(A(jrq_snapshot *, snap), i, A(int64_t *, host_out));
}

int32_t jrq_jni_snapshot_via(jrq_addr snap) {
    return jrq_snapshot_via(A(const jrq_snapshot *, snap));
}

int32_t jrq_jni_crc64_batch(jrq_addr eng, jrq_addr payload, jrq_addr offsets, int32_t n,
                            jrq_addr crc_out) {
    N(n);
    return jrq_crc64_batch(A(jrq_engine *, eng), A(const uint8_t *, payload),
                           A(const uint64_t *, offsets), (uint32_t)n, A(uint64_t *, crc_out));
}

int32_t jrq_jni_crc64_stream_update(jrq_addr eng, jrq_addr state, jrq_addr payload,
                                    jrq_addr offsets, int32_t streams) {
    N(streams);
    return jrq_crc64_stream_update(A(jrq_engine *, eng), A(uint64_t *, state),
                                   A(const uint8_t *, payload), A(const uint64_t *, offsets),
                                   (uint32_t)streams);
}

int32_t jrq_jni_logentry_checksum_batch(jrq_addr eng, jrq_addr type, jrq_addr index,
                                        jrq_addr term, jrq_addr peer_xor, jrq_addr payload,
                                        jrq_addr offsets, int32_t n, jrq_addr out,
                                        jrq_addr expected, jrq_addr has, jrq_addr corrupt_out) {
    N(n);
    return jrq_logentry_checksum_batch(
        A(jrq_engine *, eng), A(const uint8_t *, type), A(const int64_t *, index),
        A(const int64_t *, term), A(const uint64_t *, peer_xor), A(const uint8_t *, payload),
        A(const uint64_t *, offsets), (uint32_t)n, A(uint64_t *, out),
        A(const uint64_t *, expected), A(const uint8_t *, has), A(uint8_t *, corrupt_out));
}

int32_t jrq_jni_append_entries_verify(jrq_addr eng, int32_t R, jrq_addr req_off,
                                      jrq_addr prev_log_index, int32_t n, jrq_addr term,
                                      jrq_addr type, jrq_addr data_len, jrq_addr peer_xor,
                                      jrq_addr checksum, jrq_addr has_checksum, jrq_addr data,
                                      jrq_addr checksum_out, jrq_addr corrupt_out,
                                      jrq_addr first_corrupt_out) {
    N(R);
    N(n);
    return jrq_append_entries_verify(
        A(jrq_engine *, eng), (uint32_t)R, A(const uint32_t *, req_off),
        A(const int64_t *, prev_log_index), (uint32_t)n, A(const int64_t *, term),
        A(const uint8_t *, type), A(const int64_t *, data_len), A(const uint64_t *, peer_xor),
        A(const uint64_t *, checksum), A(const uint8_t *, has_checksum), A(const uint8_t *, data),
        A(uint64_t *, checksum_out), A(uint8_t *, corrupt_out), A(int32_t *, first_corrupt_out));
}

int32_t jrq_jni_lease_check(jrq_addr eng, jrq_addr last_rpc_ts, int64_t ld, int32_t num_peers,
                            jrq_addr conf, jrq_addr self_slot, int32_t G, int64_t now_ms,
                            int64_t lease_timeout_ms, jrq_addr ok_out, jrq_addr lease_start_inout,
                            jrq_addr dead_out) {
    N(num_peers);
    N(G);
    if (ld < 0) return JRQ_E_INVALID;
    return jrq_lease_check(A(jrq_engine *, eng), A(const int64_t *, last_rpc_ts), (uint64_t)ld,
                           (uint32_t)num_peers, A(const uint64_t *, conf),
                           A(const uint8_t *, self_slot), (uint32_t)G, now_ms, lease_timeout_ms,
                           A(uint8_t *, ok_out), A(int64_t *, lease_start_inout),
                           A(uint16_t *, dead_out));
}

int32_t jrq_jni_readindex_quorum(jrq_addr eng, jrq_addr conf, jrq_addr self_slot, jrq_addr order,
                                 jrq_addr ok_mask, int32_t num_peers, int32_t G,
                                 jrq_addr result_out) {
    N(num_peers);
    N(G);
    return jrq_readindex_quorum(A(jrq_engine *, eng), A(const uint64_t *, conf),
                                A(const uint8_t *, self_slot), A(const uint64_t *, order),
                                A(const uint16_t *, ok_mask), (uint32_t)num_peers, (uint32_t)G,
                                A(uint8_t *, result_out));
}

int32_t jrq_jni_leader_tick(jrq_addr eng, jrq_addr last_rpc_ts, int64_t ld, int32_t num_peers,
                            jrq_addr conf, jrq_addr self_slot, int32_t G, int64_t now_ms,
                            int64_t lease_timeout_ms, jrq_addr ok_out, jrq_addr lease_start_inout,
                            jrq_addr dead_out, jrq_addr order, jrq_addr ok_mask,
                            jrq_addr ri_result_out) {
    N(num_peers);
    N(G);
    if (ld < 0) return JRQ_E_INVALID;
    return jrq_leader_tick(A(jrq_engine *, eng), A(const int64_t *, last_rpc_ts), (uint64_t)ld,
                           (uint32_t)num_peers, A(const uint64_t *, conf),
                           A(const uint8_t *, self_slot), (uint32_t)G, now_ms, lease_timeout_ms,
                           A(uint8_t *, ok_out), A(int64_t *, lease_start_inout),
                           A(uint16_t *, dead_out), A(const uint64_t *, order),
                           A(const uint16_t *, ok_mask), A(uint8_t *, ri_result_out));
}

int32_t jrq_jni_commit_fanout(jrq_addr eng, int32_t G, jrq_addr prev_committed,
                              jrq_addr committed, jrq_addr last_applied, jrq_addr cq_first,
                              jrq_addr cq_size, jrq_addr first_closure_out, jrq_addr status_out,
                              jrq_addr listed_bitmap_out, jrq_addr num_listed_out) {
    N(G);
    return jrq_commit_fanout(A(jrq_engine *, eng), (uint32_t)G, A(const int64_t *, prev_committed),
                             A(const int64_t *, committed), A(const int64_t *, last_applied),
                             A(int64_t *, cq_first), A(int64_t *, cq_size),
                             A(int64_t *, first_closure_out), A(uint8_t *, status_out),
                             A(uint64_t *, listed_bitmap_out), A(uint32_t *, num_listed_out));
}

int32_t jrq_jni_v2_decode_verify(jrq_addr eng, jrq_addr records, jrq_addr offsets, int32_t n,
                                 jrq_addr status_out, jrq_addr type_out, jrq_addr index_out,
                                 jrq_addr term_out, jrq_addr stored_checksum_out,
                                 jrq_addr has_checksum_out, jrq_addr data_off_out,
                                 jrq_addr data_len_out, jrq_addr peer_counts_out,
                                 jrq_addr checksum_out, jrq_addr corrupt_out) {
    N(n);
    return jrq_v2_decode_verify(
        A(jrq_engine *, eng), A(const uint8_t *, records), A(const uint64_t *, offsets),
        (uint32_t)n, A(uint8_t *, status_out), A(uint8_t *, type_out), A(int64_t *, index_out),
        A(int64_t *, term_out), A(uint64_t *, stored_checksum_out),
        A(uint8_t *, has_checksum_out), A(uint64_t *, data_off_out), A(uint64_t *, data_len_out),
        A(uint32_t *, peer_counts_out), A(uint64_t *, checksum_out), A(uint8_t *, corrupt_out));
}
