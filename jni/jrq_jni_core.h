/*
 * jrq_jni_core.h -- the plain-C core of the JNI binding (jrq_jni.c) over include/jrq.h.
 *
 * Every JNIEXPORT in jrq_jni.c resolves its DirectByteBuffers to raw addresses
 * (GetDirectBufferAddress) and calls exactly one function below; every function below casts
 * those addresses to the parameter types of exactly one include/jrq.h entry point and calls it.
 * The split keeps all type knowledge of the ABI in this C file, which the CPU test suite
 * compiles with -Wall -Wextra -Werror against include/jrq.h (tests/test_jni.py), and which a GPU
 * test calls through ctypes: a header change that breaks the glue fails the build, not a JVM.
 *
 * Conventions (the Java side's view):
 *   - jrq_addr is a Java long: an engine / table handle, or the address of a direct buffer
 *     (0 = null buffer, which libjrq treats as the reference's null where the header allows
 *     it and rejects with JRQ_E_INVALID elsewhere);
 *   - counts are Java ints (jint) and are checked to be >= 0 before they become uint32_t;
 *   - returns are those of libjrq: 0 or a negative jrq_error, except where noted.
 * Reference interfaces each call replaces: INTEGRATION.md §1 (file:line per entry point).
 */
#ifndef JRQ_JNI_CORE_H
#define JRQ_JNI_CORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int64_t jrq_addr;

/* engine (NodeImpl.java:829-836 `new BallotBox()`; CrcUtil.java:28 ThreadLocal CRC64) */
jrq_addr jrq_jni_create(int32_t device, int32_t max_groups, int32_t max_peers, jrq_addr err_out);
void jrq_jni_destroy(jrq_addr eng);
int32_t jrq_jni_abi_version(void);
const char *jrq_jni_build_id(void);
const char *jrq_jni_last_error(jrq_addr eng);
int32_t jrq_jni_synchronize(jrq_addr eng);

/* DirectByteBuffer pinning (jrq_host_register / jrq_host_alloc) */
int32_t jrq_jni_host_register(jrq_addr ptr, int64_t bytes);
int32_t jrq_jni_host_unregister(jrq_addr ptr);
int64_t jrq_jni_host_registered_bytes(jrq_addr ptr);   /* bytes, or a negative jrq_error */
jrq_addr jrq_jni_host_alloc(int64_t bytes);             /* 0 on failure */
int32_t jrq_jni_host_free(jrq_addr ptr);

/* stateless quorum epoch (BallotBox.java:96-139 for G groups) */
int32_t jrq_jni_quorum_epoch(jrq_addr eng, jrq_addr match, jrq_addr pending_index,
                             jrq_addr last_appended, jrq_addr last_committed, jrq_addr conf,
                             jrq_addr run_off, jrq_addr run_start, jrq_addr run_conf,
                             int32_t num_peers, int32_t num_runs, int32_t G,
                             jrq_addr committed_out, jrq_addr status_out);
int32_t jrq_jni_quorum_epoch_tiles(jrq_addr eng, jrq_addr tiles, int32_t num_peers,
                                   jrq_addr run_off, jrq_addr run_start, jrq_addr run_conf,
                                   int32_t G, jrq_addr committed_out, jrq_addr status_out);

/* resident group table (GpuGroupBatch) */
jrq_addr jrq_jni_table_create(jrq_addr eng, int32_t G, int32_t num_peers, jrq_addr err_out);
void jrq_jni_table_destroy(jrq_addr table);
int32_t jrq_jni_table_update(jrq_addr table, jrq_addr states, int32_t n_states, jrq_addr recs,
                             int32_t n_recs);
/* states / recs: addresses of `parts` jrq_addr words (one buffer address per part);
 * n_states / n_recs: addresses of `parts` int32 counts */
int32_t jrq_jni_table_update_gather(jrq_addr table, int32_t parts, jrq_addr states,
                                    jrq_addr n_states, jrq_addr recs, jrq_addr n_recs);
int32_t jrq_jni_table_stage_reserve(jrq_addr table, int32_t max_states, int32_t max_recs);
int32_t jrq_jni_table_stage(jrq_addr table, jrq_addr states, int32_t n_states, jrq_addr recs,
                            int32_t n_recs);
int32_t jrq_jni_table_stage_apply(jrq_addr table);
int32_t jrq_jni_table_stage_reserve_acks(jrq_addr table, int32_t max_acks, int32_t max_segments);
int32_t jrq_jni_table_stage_acks(jrq_addr table, int64_t stamp, jrq_addr acks, int32_t n);
/* records streamed while they are written: region_out is the address of
 * one jrq_addr word receiving the region's device address; ack_push may be called from any
 * thread (host_src: a page-locked direct buffer's address) */
int32_t jrq_jni_table_ack_region(jrq_addr table, int64_t capacity, jrq_addr region_out);
int32_t jrq_jni_table_ack_region_free(jrq_addr table, jrq_addr region);
/* records [from, from + n) of the buffer at host_src to the same positions of the region */
int32_t jrq_jni_table_ack_push(jrq_addr table, jrq_addr region_dst, jrq_addr host_src, int32_t from,
                               int32_t n);
/* returns the number of changed groups written to `changed` (>= 0), or a jrq_error */
int32_t jrq_jni_table_epoch(jrq_addr table, jrq_addr changed, jrq_addr status_out);
int32_t jrq_jni_table_read(jrq_addr table, jrq_addr pending_index, jrq_addr last_appended,
                           jrq_addr last_committed, jrq_addr match);
int32_t jrq_jni_table_check(jrq_addr table);
/* FSMCaller state and the fused fan-out epoch (FSMCallerImpl.java:462-482,
 * ClosureQueueImpl.java:113-142) */
int32_t jrq_jni_table_fsm_update(jrq_addr table, jrq_addr groups, jrq_addr last_applied,
                                 jrq_addr cq_first, jrq_addr cq_size, int32_t n);
int32_t jrq_jni_table_fsm_read(jrq_addr table, jrq_addr last_applied, jrq_addr cq_first,
                               jrq_addr cq_size);
/* returns the number of changed groups (>= 0), or a jrq_error */
int32_t jrq_jni_table_epoch_fanout(jrq_addr table, jrq_addr changed, jrq_addr fan_first,
                                   jrq_addr fan_status);

/* one JVM, N engines (ShardedGroupBatch): `engines` / `tables` is the
 * address of n jrq_addr words */
int32_t jrq_jni_rccl_init_all(jrq_addr engines, int32_t n);
jrq_addr jrq_jni_snapshot_create(jrq_addr tables, int32_t n, jrq_addr err_out);
void jrq_jni_snapshot_destroy(jrq_addr snap);
int32_t jrq_jni_snapshot_publish(jrq_addr snap);
int32_t jrq_jni_snapshot_read(jrq_addr snap, int32_t i, jrq_addr host_out);
int32_t jrq_jni_snapshot_via(jrq_addr snap);

/* checksums (CrcUtil.java:36-80, CRC64.java:100-126, LogEntry.java:88-108,156-158) */
int32_t jrq_jni_crc64_batch(jrq_addr eng, jrq_addr payload, jrq_addr offsets, int32_t n,
                            jrq_addr crc_out);
int32_t jrq_jni_crc64_stream_update(jrq_addr eng, jrq_addr state, jrq_addr payload,
                                    jrq_addr offsets, int32_t streams);
int32_t jrq_jni_logentry_checksum_batch(jrq_addr eng, jrq_addr type, jrq_addr index,
                                        jrq_addr term, jrq_addr peer_xor, jrq_addr payload,
                                        jrq_addr offsets, int32_t n, jrq_addr out,
                                        jrq_addr expected, jrq_addr has, jrq_addr corrupt_out);

/* §8f callers */
int32_t jrq_jni_append_entries_verify(jrq_addr eng, int32_t R, jrq_addr req_off,
                                      jrq_addr prev_log_index, int32_t n, jrq_addr term,
                                      jrq_addr type, jrq_addr data_len, jrq_addr peer_xor,
                                      jrq_addr checksum, jrq_addr has_checksum, jrq_addr data,
                                      jrq_addr checksum_out, jrq_addr corrupt_out,
                                      jrq_addr first_corrupt_out);
int32_t jrq_jni_lease_check(jrq_addr eng, jrq_addr last_rpc_ts, int64_t ld, int32_t num_peers,
                            jrq_addr conf, jrq_addr self_slot, int32_t G, int64_t now_ms,
                            int64_t lease_timeout_ms, jrq_addr ok_out, jrq_addr lease_start_inout,
                            jrq_addr dead_out);
int32_t jrq_jni_readindex_quorum(jrq_addr eng, jrq_addr conf, jrq_addr self_slot, jrq_addr order,
                                 jrq_addr ok_mask, int32_t num_peers, int32_t G,
                                 jrq_addr result_out);
int32_t jrq_jni_leader_tick(jrq_addr eng, jrq_addr last_rpc_ts, int64_t ld, int32_t num_peers,
                            jrq_addr conf, jrq_addr self_slot, int32_t G, int64_t now_ms,
                            int64_t lease_timeout_ms, jrq_addr ok_out, jrq_addr lease_start_inout,
                            jrq_addr dead_out, jrq_addr order, jrq_addr ok_mask,
                            jrq_addr ri_result_out);
int32_t jrq_jni_commit_fanout(jrq_addr eng, int32_t G, jrq_addr prev_committed,
                              jrq_addr committed, jrq_addr last_applied, jrq_addr cq_first,
                              jrq_addr cq_size, jrq_addr first_closure_out, jrq_addr status_out,
                              jrq_addr listed_bitmap_out, jrq_addr num_listed_out);
int32_t jrq_jni_v2_decode_verify(jrq_addr eng, jrq_addr records, jrq_addr offsets, int32_t n,
                                 jrq_addr status_out, jrq_addr type_out, jrq_addr index_out,
                                 jrq_addr term_out, jrq_addr stored_checksum_out,
                                 jrq_addr has_checksum_out, jrq_addr data_off_out,
                                 jrq_addr data_len_out, jrq_addr peer_counts_out,
                                 jrq_addr checksum_out, jrq_addr corrupt_out);

#ifdef __cplusplus
}
#endif
#endif /* JRQ_JNI_CORE_H */
