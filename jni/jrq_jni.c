/*
 * jrq_jni.c -- JNI glue of com.alipay.sofa.jraft.core.JrqNative (JDK 8) over libjrq.so.
 *
 * Every native method resolves its java.nio direct buffers to addresses and calls one function
 * of the plain-C core (jrq_jni_core.c), which owns every cast to include/jrq.h's types.  A buffer
 * that is null, or not direct, becomes address 0: libjrq treats it as the reference's null where
 * the header allows one and refuses the call with JRQ_E_INVALID elsewhere.  No exception is
 * thrown from here; the Java shim maps negative returns to exceptions.
 *
 * Built only where a JDK exists (jni/Makefile: `make jni` with JAVA_HOME set).  Without one the
 * CPU suite type-checks this file against jni/typecheck/jni.h (tests/test_jni.py).
 *
 * The Java side:
 *   package com.alipay.sofa.jraft.core;
 *   final class JrqNative {
 *       static { System.loadLibrary("jrq_jni"); }
 *       static native long create(int device, int maxGroups, int maxPeers, ByteBuffer err);
 *       static native int quorumEpochTiles(long eng, ByteBuffer tiles, int numPeers, ...);
 *       ... one method per function below, same argument order ...
 *   }
 */
#include <jni.h>
#include <stddef.h>

#include "jrq_jni_core.h"

#define ADDR(b) ((b) ? (jrq_addr)(intptr_t)(*env)->GetDirectBufferAddress(env, (b)) : 0)
#define FN(name) JNICALL Java_com_alipay_sofa_jraft_core_JrqNative_##name
#define ENG(h) ((jrq_addr)(h))

JNIEXPORT jlong FN(create)(JNIEnv *env, jclass cls, jint device, jint maxGroups, jint maxPeers,
                           jobject errOut) {
    (void)cls;
    return (jlong)jrq_jni_create(device, maxGroups, maxPeers, ADDR(errOut));
}

JNIEXPORT void FN(destroy)(JNIEnv *env, jclass cls, jlong eng) {
    (void)env;
    (void)cls;
    jrq_jni_destroy(ENG(eng));
}

JNIEXPORT jint FN(abiVersion)(JNIEnv *env, jclass cls) {
    (void)env;
    (void)cls;
    return jrq_jni_abi_version();
}

JNIEXPORT jstring FN(buildId)(JNIEnv *env, jclass cls) {
    (void)cls;
    return (*env)->NewStringUTF(env, jrq_jni_build_id());
}

JNIEXPORT jstring FN(lastError)(JNIEnv *env, jclass cls, jlong eng) {
    const char *t = jrq_jni_last_error(ENG(eng));
    (void)cls;
    return (*env)->NewStringUTF(env, t ? t : "");
}

JNIEXPORT jint FN(synchronize)(JNIEnv *env, jclass cls, jlong eng) {
    (void)env;
    (void)cls;
    return jrq_jni_synchronize(ENG(eng));
}

/* DirectByteBuffer pinning: the whole buffer (capacity), registered once; the Cleaner must
 * call hostUnregister before the memory is freed (jrq.h). */
JNIEXPORT jint FN(hostRegister)(JNIEnv *env, jclass cls, jobject buf) {
    (void)cls;
    return jrq_jni_host_register(ADDR(buf), buf ? (int64_t)(*env)->GetDirectBufferCapacity(env, buf) : 0);
}

JNIEXPORT jint FN(hostUnregister)(JNIEnv *env, jclass cls, jobject buf) {
    (void)cls;
    return jrq_jni_host_unregister(ADDR(buf));
}

JNIEXPORT jlong FN(hostRegisteredBytes)(JNIEnv *env, jclass cls, jobject buf) {
    (void)cls;
    return (jlong)jrq_jni_host_registered_bytes(ADDR(buf));
}

/* driver-owned page-locked memory wrapped as a direct buffer (null on failure); release it with
 * hostFree after the last call that used it */
JNIEXPORT jobject FN(hostAlloc)(JNIEnv *env, jclass cls, jlong bytes) {
    jrq_addr p = jrq_jni_host_alloc((int64_t)bytes);
    (void)cls;
    return p ? (*env)->NewDirectByteBuffer(env, (void *)(intptr_t)p, bytes) : NULL;
}

JNIEXPORT jint FN(hostFree)(JNIEnv *env, jclass cls, jobject buf) {
    (void)cls;
    return jrq_jni_host_free(ADDR(buf));
}

JNIEXPORT jint FN(quorumEpoch)(JNIEnv *env, jclass cls, jlong eng, jobject match, jobject pending,
                               jobject lastApp, jobject lastCommitted, jobject conf,
                               jobject runOff, jobject runStart, jobject runConf, jint numPeers,
                               jint numRuns, jint G, jobject committedOut, jobject statusOut) {
    (void)cls;
    return jrq_jni_quorum_epoch(ENG(eng), ADDR(match), ADDR(pending), ADDR(lastApp),
                                ADDR(lastCommitted), ADDR(conf), ADDR(runOff), ADDR(runStart),
                                ADDR(runConf), numPeers, numRuns, G, ADDR(committedOut),
                                ADDR(statusOut));
}

/* the stateless JNI contract: one direct buffer of 256-group tiles */
JNIEXPORT jint FN(quorumEpochTiles)(JNIEnv *env, jclass cls, jlong eng, jobject tiles,
                                    jint numPeers, jobject runOff, jobject runStart,
                                    jobject runConf, jint G, jobject committedOut,
                                    jobject statusOut) {
    (void)cls;
    return jrq_jni_quorum_epoch_tiles(ENG(eng), ADDR(tiles), numPeers, ADDR(runOff),
                                      ADDR(runStart), ADDR(runConf), G, ADDR(committedOut),
                                      ADDR(statusOut));
}

JNIEXPORT jlong FN(tableCreate)(JNIEnv *env, jclass cls, jlong eng, jint G, jint numPeers,
                                jobject errOut) {
    (void)cls;
    return (jlong)jrq_jni_table_create(ENG(eng), G, numPeers, ADDR(errOut));
}

JNIEXPORT void FN(tableDestroy)(JNIEnv *env, jclass cls, jlong table) {
    (void)env;
    (void)cls;
    jrq_jni_table_destroy(ENG(table));
}

JNIEXPORT jint FN(tableUpdate)(JNIEnv *env, jclass cls, jlong table, jobject states, jint nStates,
                               jobject recs, jint nRecs) {
    (void)cls;
    return jrq_jni_table_update(ENG(table), ADDR(states), nStates, ADDR(recs), nRecs);
}

/* one (states, recs) buffer pair per pack thread.  Each GetObjectArrayElement makes a local
 * reference; JNI guarantees only 16 per native frame, so each is deleted as soon as its
 * address is read (the markdown glue kept up to 32 alive). */
JNIEXPORT jint FN(tableUpdateGather)(JNIEnv *env, jclass cls, jlong table, jint parts,
                                     jobjectArray states, jintArray nStates, jobjectArray recs,
                                     jintArray nRecs) {
    enum { MAX_PARTS = 64 };
    jrq_addr sa[MAX_PARTS], ra[MAX_PARTS];
    jint ns[MAX_PARTS], nr[MAX_PARTS];
    jint i;
    (void)cls;
    if (parts < 0 || parts > MAX_PARTS || !states || !recs || !nStates || !nRecs) return -1;
    if ((*env)->GetArrayLength(env, states) < parts || (*env)->GetArrayLength(env, recs) < parts ||
        (*env)->GetArrayLength(env, nStates) < parts || (*env)->GetArrayLength(env, nRecs) < parts)
        return -1; /* JRQ_E_INVALID */
    for (i = 0; i < parts; ++i) {
        jobject s = (*env)->GetObjectArrayElement(env, states, i);
        jobject r = (*env)->GetObjectArrayElement(env, recs, i);
        sa[i] = ADDR(s);
        ra[i] = ADDR(r);
        if (s) (*env)->DeleteLocalRef(env, s);
        if (r) (*env)->DeleteLocalRef(env, r);
    }
    (*env)->GetIntArrayRegion(env, nStates, 0, parts, ns);
    (*env)->GetIntArrayRegion(env, nRecs, 0, parts, nr);
    return jrq_jni_table_update_gather(ENG(table), parts, (jrq_addr)(intptr_t)sa,
                                       (jrq_addr)(intptr_t)ns, (jrq_addr)(intptr_t)ra,
                                       (jrq_addr)(intptr_t)nr);
}

JNIEXPORT jint FN(tableStageReserve)(JNIEnv *env, jclass cls, jlong table, jint maxStates,
                                     jint maxRecs) {
    (void)env;
    (void)cls;
    return jrq_jni_table_stage_reserve(ENG(table), maxStates, maxRecs);
}

JNIEXPORT jint FN(tableStage)(JNIEnv *env, jclass cls, jlong table, jobject states, jint nStates,
                              jobject recs, jint nRecs) {
    (void)cls;
    return jrq_jni_table_stage(ENG(table), ADDR(states), nStates, ADDR(recs), nRecs);
}

JNIEXPORT jint FN(tableStageApply)(JNIEnv *env, jclass cls, jlong table) {
    (void)env;
    (void)cls;
    return jrq_jni_table_stage_apply(ENG(table));
}

/* order-free ack records (JRQ_ACK) recorded by the Java BallotBox at call time, one segment per
 * reset stamp: what GpuGroupBatch.flush ships without a pack pass */
JNIEXPORT jint FN(tableStageReserveAcks)(JNIEnv *env, jclass cls, jlong table, jint maxAcks,
                                         jint maxSegments) {
    (void)env;
    (void)cls;
    return jrq_jni_table_stage_reserve_acks(ENG(table), maxAcks, maxSegments);
}

JNIEXPORT jint FN(tableStageAcks)(JNIEnv *env, jclass cls, jlong table, jlong stamp, jobject acks,
                                  jint n) {
    (void)cls;
    return jrq_jni_table_stage_acks(ENG(table), stamp, ADDR(acks), n);
}

/* regionOut: a direct buffer of one long receiving the region's device address */
JNIEXPORT jint FN(tableAckRegion)(JNIEnv *env, jclass cls, jlong table, jlong capacity,
                                  jobject regionOut) {
    (void)cls;
    return jrq_jni_table_ack_region(ENG(table), capacity, ADDR(regionOut));
}

JNIEXPORT jint FN(tableAckRegionFree)(JNIEnv *env, jclass cls, jlong table, jlong region) {
    (void)env;
    (void)cls;
    return jrq_jni_table_ack_region_free(ENG(table), ENG(region));
}

/* from any thread: the calling thread's page-locked record buffer, from element `from` */
JNIEXPORT jint FN(tableAckPush)(JNIEnv *env, jclass cls, jlong table, jlong regionDst, jobject records,
                                jint from, jint n) {
    (void)cls;
    return jrq_jni_table_ack_push(ENG(table), ENG(regionDst), ADDR(records), from, n);
}

/* returns the number of changed groups (>= 0) or a negative jrq_error */
JNIEXPORT jint FN(tableEpoch)(JNIEnv *env, jclass cls, jlong table, jobject changed,
                              jobject statusOut) {
    (void)cls;
    return jrq_jni_table_epoch(ENG(table), ADDR(changed), ADDR(statusOut));
}

JNIEXPORT jint FN(tableRead)(JNIEnv *env, jclass cls, jlong table, jobject pending,
                             jobject lastApp, jobject lastCommitted, jobject match) {
    (void)cls;
    return jrq_jni_table_read(ENG(table), ADDR(pending), ADDR(lastApp), ADDR(lastCommitted),
                              ADDR(match));
}

JNIEXPORT jint FN(tableCheck)(JNIEnv *env, jclass cls, jlong table) {
    (void)env;
    (void)cls;
    return jrq_jni_table_check(ENG(table));
}

/* engines / tables: a direct buffer of n longs (native handles) */
JNIEXPORT jint FN(rcclInitAll)(JNIEnv *env, jclass cls, jobject engines, jint n) {
    (void)cls;
    return jrq_jni_rccl_init_all(ADDR(engines), n);
}

JNIEXPORT jlong FN(snapshotCreate)(JNIEnv *env, jclass cls, jobject tables, jint n,
                                   jobject errOut) {
    (void)cls;
    return (jlong)jrq_jni_snapshot_create(ADDR(tables), n, ADDR(errOut));
}

JNIEXPORT void FN(snapshotDestroy)(JNIEnv *env, jclass cls, jlong snap) {
    (void)env;
    (void)cls;
    jrq_jni_snapshot_destroy(ENG(snap));
}

JNIEXPORT jint FN(snapshotPublish)(JNIEnv *env, jclass cls, jlong snap) {
    (void)env;
    (void)cls;
    return jrq_jni_snapshot_publish(ENG(snap));
}

JNIEXPORT jint FN(snapshotRead)(JNIEnv *env, jclass cls, jlong snap, jint i, jobject out) {
    (void)cls;
    return jrq_jni_snapshot_read(ENG(snap), i, ADDR(out));
}

JNIEXPORT jint FN(snapshotVia)(JNIEnv *env, jclass cls, jlong snap) {
    (void)env;
    (void)cls;
    return jrq_jni_snapshot_via(ENG(snap));
}

JNIEXPORT jint FN(tableFsmUpdate)(JNIEnv *env, jclass cls, jlong table, jobject groups,
                                  jobject lastApplied, jobject cqFirst, jobject cqSize, jint n) {
    (void)cls;
    return jrq_jni_table_fsm_update(ENG(table), ADDR(groups), ADDR(lastApplied), ADDR(cqFirst),
                                    ADDR(cqSize), n);
}

JNIEXPORT jint FN(tableFsmRead)(JNIEnv *env, jclass cls, jlong table, jobject lastApplied,
                                jobject cqFirst, jobject cqSize) {
    (void)cls;
    return jrq_jni_table_fsm_read(ENG(table), ADDR(lastApplied), ADDR(cqFirst), ADDR(cqSize));
}

/* returns the number of changed groups (>= 0) or a negative jrq_error */
JNIEXPORT jint FN(tableEpochFanout)(JNIEnv *env, jclass cls, jlong table, jobject changed,
                                    jobject fanFirst, jobject fanStatus) {
    (void)cls;
    return jrq_jni_table_epoch_fanout(ENG(table), ADDR(changed), ADDR(fanFirst), ADDR(fanStatus));
}

JNIEXPORT jint FN(crc64Batch)(JNIEnv *env, jclass cls, jlong eng, jobject payload,
                              jobject offsets, jint n, jobject out) {
    (void)cls;
    return jrq_jni_crc64_batch(ENG(eng), ADDR(payload), ADDR(offsets), n, ADDR(out));
}

JNIEXPORT jint FN(crc64StreamUpdate)(JNIEnv *env, jclass cls, jlong eng, jobject state,
                                     jobject payload, jobject offsets, jint streams) {
    (void)cls;
    return jrq_jni_crc64_stream_update(ENG(eng), ADDR(state), ADDR(payload), ADDR(offsets),
                                       streams);
}

JNIEXPORT jint FN(logEntryChecksumBatch)(JNIEnv *env, jclass cls, jlong eng, jobject type,
                                         jobject index, jobject term, jobject peerXor,
                                         jobject payload, jobject offsets, jint n, jobject out,
                                         jobject expected, jobject has, jobject corrupt) {
    (void)cls;
    return jrq_jni_logentry_checksum_batch(ENG(eng), ADDR(type), ADDR(index), ADDR(term),
                                           ADDR(peerXor), ADDR(payload), ADDR(offsets), n,
                                           ADDR(out), ADDR(expected), ADDR(has), ADDR(corrupt));
}

JNIEXPORT jint FN(appendEntriesVerify)(JNIEnv *env, jclass cls, jlong eng, jint R,
                                       jobject reqOff, jobject prevLogIndex, jint n, jobject term,
                                       jobject type, jobject dataLen, jobject peerXor,
                                       jobject checksum, jobject hasChecksum, jobject data,
                                       jobject checksumOut, jobject corruptOut,
                                       jobject firstCorruptOut) {
    (void)cls;
    return jrq_jni_append_entries_verify(ENG(eng), R, ADDR(reqOff), ADDR(prevLogIndex), n,
                                         ADDR(term), ADDR(type), ADDR(dataLen), ADDR(peerXor),
                                         ADDR(checksum), ADDR(hasChecksum), ADDR(data),
                                         ADDR(checksumOut), ADDR(corruptOut),
                                         ADDR(firstCorruptOut));
}

JNIEXPORT jint FN(leaseCheck)(JNIEnv *env, jclass cls, jlong eng, jobject lastRpcTs, jlong ld,
                              jint numPeers, jobject conf, jobject selfSlot, jint G, jlong nowMs,
                              jlong leaseTimeoutMs, jobject okOut, jobject leaseStart,
                              jobject deadOut) {
    (void)cls;
    return jrq_jni_lease_check(ENG(eng), ADDR(lastRpcTs), ld, numPeers, ADDR(conf),
                               ADDR(selfSlot), G, nowMs, leaseTimeoutMs, ADDR(okOut),
                               ADDR(leaseStart), ADDR(deadOut));
}

JNIEXPORT jint FN(readIndexQuorum)(JNIEnv *env, jclass cls, jlong eng, jobject conf,
                                   jobject selfSlot, jobject order, jobject okMask, jint numPeers,
                                   jint G, jobject result) {
    (void)cls;
    return jrq_jni_readindex_quorum(ENG(eng), ADDR(conf), ADDR(selfSlot), ADDR(order),
                                    ADDR(okMask), numPeers, G, ADDR(result));
}

/* the step-down timer of every leader group, with the ReadIndex responses since the last tick
 * (order / okMask / riResult null: the lease check alone) */
JNIEXPORT jint FN(leaderTick)(JNIEnv *env, jclass cls, jlong eng, jobject lastRpcTs, jlong ld,
                              jint numPeers, jobject conf, jobject selfSlot, jint G, jlong nowMs,
                              jlong leaseTimeoutMs, jobject okOut, jobject leaseStart,
                              jobject deadOut, jobject order, jobject okMask, jobject riResult) {
    (void)cls;
    return jrq_jni_leader_tick(ENG(eng), ADDR(lastRpcTs), ld, numPeers, ADDR(conf),
                               ADDR(selfSlot), G, nowMs, leaseTimeoutMs, ADDR(okOut),
                               ADDR(leaseStart), ADDR(deadOut), ADDR(order), ADDR(okMask),
                               ADDR(riResult));
}

JNIEXPORT jint FN(commitFanout)(JNIEnv *env, jclass cls, jlong eng, jint G,
                                jobject prevCommitted, jobject committed, jobject lastApplied,
                                jobject cqFirst, jobject cqSize, jobject firstClosureOut,
                                jobject statusOut, jobject listedBitmapOut,
                                jobject numListedOut) {
    (void)cls;
    return jrq_jni_commit_fanout(ENG(eng), G, ADDR(prevCommitted), ADDR(committed),
                                 ADDR(lastApplied), ADDR(cqFirst), ADDR(cqSize),
                                 ADDR(firstClosureOut), ADDR(statusOut), ADDR(listedBitmapOut),
                                 ADDR(numListedOut));
}

JNIEXPORT jint FN(v2DecodeVerify)(JNIEnv *env, jclass cls, jlong eng, jobject records,
                                  jobject offsets, jint n, jobject status, jobject type,
                                  jobject index, jobject term, jobject stored,
                                  jobject hasChecksum, jobject dataOff, jobject dataLen,
                                  jobject peerCounts, jobject checksum, jobject corrupt) {
    (void)cls;
    return jrq_jni_v2_decode_verify(ENG(eng), ADDR(records), ADDR(offsets), n, ADDR(status),
                                    ADDR(type), ADDR(index), ADDR(term), ADDR(stored),
                                    ADDR(hasChecksum), ADDR(dataOff), ADDR(dataLen),
                                    ADDR(peerCounts), ADDR(checksum), ADDR(corrupt));
}
