/*
 * jrq.h -- C ABI of libjrq.so, the MI355X-native batched quorum + CRC64 engine
 * that takes over SOFAJRaft's data-parallel hot path.
 *
 * The reference has no plug-in point for this path: BallotBox is
 * instantiated directly (NodeImpl.java:829-836) and CrcUtil is a static utility.
 * The drop-in surface is therefore the Java class API, and this header is what a
 * JDK 8 JNI shim behind those classes binds.  Every entry
 * point below names the reference interface it replaces.
 *   JC = jraft-core/src/main/java/com/alipay/sofa/jraft
 *
 * Conventions
 *   - extern "C", plain pointers and sizes, no C++ or torch types.
 *   - Return value: 0 = OK, negative = jrq_error.  Per-group outcomes go to
 *     status_out (jrq_group_status bit flags); no exceptions cross the ABI.  The
 *     Java shim re-throws ArrayIndexOutOfBoundsException / IllegalArgumentException
 *     itself (its synchronous checks), so the reference's error
 *     behaviour is preserved.
 *   - Ownership: the caller owns every buffer; the engine never frees them.
 *   - *_dev functions take DEVICE pointers and are asynchronous on the engine's
 *     stream (jrq_get_stream / jrq_set_stream); the other variants take HOST
 *     pointers, stage through device memory and return after synchronising.
 *   - Threading: one engine per host thread; calls on one handle are not
 *     re-entrant.  Different handles may run concurrently.
 */
#ifndef JRQ_H
#define JRQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JRQ_ABI_VERSION 3
#define JRQ_MAX_PEERS 16 /* peer slots per group (16-bit masks) */

typedef struct jrq_engine jrq_engine;

typedef enum {
    JRQ_OK = 0,
    JRQ_E_INVALID = -1,     /* bad argument (null pointer, size, peer count ...) */
    JRQ_E_NOMEM = -2,       /* device or host allocation failed */
    JRQ_E_HIP = -3,         /* a HIP runtime call failed (jrq_last_error for text) */
    JRQ_E_RCCL = -4,        /* an RCCL call failed */
    JRQ_E_NODEV = -5,       /* no usable gfx950 device */
    JRQ_E_STATE = -6        /* call not valid in the engine's state (e.g. no communicator) */
} jrq_error;

/* Per-group status flags (uint8 per group).  Mirrors the reference outcomes:
 *   NOT_LEADER   pendingIndex == 0: BallotBox.commitAt returns false (JC/core/BallotBox.java:101-103)
 *   OUT_OF_RANGE a peer's match exceeds lastAppended: that ack would throw
 *                ArrayIndexOutOfBoundsException (:107-109) and is ignored
 *   EMPTY_CONF   a pending run has an empty conf: its ballots can never be granted
 *                (Ballot.init with an empty Configuration, JC/entity/Ballot.java:63-85) */
typedef enum {
    JRQ_ST_OK = 0,
    JRQ_ST_NOT_LEADER = 1,
    JRQ_ST_OUT_OF_RANGE = 2,
    JRQ_ST_EMPTY_CONF = 4
} jrq_group_status;

/* Packed per-run configuration word (uint64):
 *   bits  0-15  new-conf peer mask over the group's peer slots   (Ballot.peers)
 *   bits 16-31  old-conf peer mask                               (Ballot.oldPeers)
 *   bits 32-39  new quorum  = |conf|/2+1                          (Ballot.quorum)
 *   bits 40-47  old quorum  = |oldConf|/2+1, or 0 if oldConf==null (Ballot.oldQuorum)
 * Learners are never in a mask (Configuration.iterator yields peers only,
 * JC/conf/Configuration.java:184-186).  Explicit quorums keep Ballot.init's
 * size-based arithmetic (JC/entity/Ballot.java:77-83) for any conf list. */
#define JRQ_CONF(newMask, oldMask, newQ, oldQ)                                                 \
    ((uint64_t)(uint16_t)(newMask) | ((uint64_t)(uint16_t)(oldMask) << 16) |                    \
     ((uint64_t)(uint8_t)(newQ) << 32) | ((uint64_t)(uint8_t)(oldQ) << 40))
/* Flag bit of conf[g] (bits 48-62 are reserved, 0): group g's pending window holds more than
 * one conf run (a conf change inside it: NodeImpl.unsafeApplyConfiguration, JC/core/
 * NodeImpl.java:2065-2086, then (conf, oldConf) per entry, :1195-1196).  Only flagged groups
 * walk a run table; every other group is decided from its conf word alone, on the fast path. */
#define JRQ_CONF_RUNS (1ull << 63)

/* One epoch of a group batch, structure-of-arrays (all arrays length G unless noted).
 * Replaces the per-call state of JC/core/BallotBox.java:50-55 for G groups at once:
 *   match[p*match_ld + g]  highest log index peer slot p has acknowledged for group g
 *                          (the `last` of its BallotBox.commitAt(first,last,peer) calls;
 *                          Replicator acks are contiguous from pendingIndex, Replicator.java:
 *                          1387-1392,1401, so one index per peer is the whole ack set)
 *   pending_index[g]       BallotBox.pendingIndex (0 = not leader)
 *   last_appended[g]       pendingIndex + pendingMetaQueue.size() - 1
 *   last_committed[g]      BallotBox.lastCommittedIndex before the epoch
 *   conf[g]                packed conf of every pending entry, or JRQ_CONF_RUNS: the group's
 *                          entries follow its runs in the run table
 *   run_off[G+1]           optional CSR of conf runs (joint consensus, conf changes):
 *                          runs of group g are [run_off[g], run_off[g+1]); run r covers log
 *                          indices [run_start[r], run_start[r+1]) (the group's last run ends at
 *                          last_appended; the first run's start is treated as <= pendingIndex);
 *                          run_conf[r] is its packed conf.  *_dev: consulted only for groups
 *                          whose conf[g] carries JRQ_CONF_RUNS.  Host variant: the engine
 *                          derives the flags itself (a group with exactly one run is decided
 *                          from that run's conf; conf may then be NULL).
 */
typedef struct {
    const int64_t *match;
    const int64_t *pending_index;
    const int64_t *last_appended;
    const int64_t *last_committed;
    const uint64_t *conf;
    const uint32_t *run_off;   /* nullable */
    const int64_t *run_start;  /* [num_runs], nullable iff run_off is */
    const uint64_t *run_conf;  /* [num_runs], nullable iff run_off is */
    uint32_t num_peers;        /* P, 1..JRQ_MAX_PEERS */
    uint32_t num_runs;         /* R (host variant: bytes to stage) */
    uint64_t match_ld;         /* row stride of match in elements, >= G */
} jrq_group_batch;

/* ---------------------------------------------------------------- engine -- */

/* Create an engine on HIP device `device` sized for up to max_groups groups per
 * epoch and max_peers peer slots (host-variant staging; device variants take any G).
 * Replaces: `new BallotBox()` per group (JC/core/NodeImpl.java:829-836) and the
 * ThreadLocal CRC64 of CrcUtil (JC/util/CrcUtil.java:28). */
jrq_engine *jrq_create(int device, uint32_t max_groups, uint8_t max_peers, int *err);
/* Replaces BallotBox.shutdown (JC/core/BallotBox.java:250-253) for the whole batch. */
void jrq_destroy(jrq_engine *e);

int jrq_abi_version(void);
/* Content hash of the kernel sources this library was compiled from (16 hex digits: SHA-256 of
 * the files in csrc/, sofa-jraft_amd/jraft_amd/_srcsha.py), so a host can tell which sources made the binary
 * it loaded.  No reference counterpart. */
const char *jrq_build_id(void);
/* Text of the last error on this engine (or of jrq_create's last failure when e==NULL). */
const char *jrq_last_error(const jrq_engine *e);
/* hipStream_t the engine launches on (as void*); jrq_set_stream adopts an external
 * stream (not owned).  NULL restores the engine's own stream. */
void *jrq_get_stream(jrq_engine *e);
int jrq_set_stream(jrq_engine *e, void *hip_stream);
int jrq_synchronize(jrq_engine *e);
/* Page-lock a host buffer (e.g. a DirectByteBuffer's address) for fast staging.  Host
 * variants (the functions without _dev) DMA registered memory straight to and from the device;
 * other caller memory, inputs and outputs alike, goes through the engine's two pinned 8 MiB
 * bounce chunks (a CPU copy overlapped with the other chunk's DMA): libjrq never hands pageable
 * memory to a HIP copy.
 * The driver pins whole pages, so registrations are tracked by page: a range sharing a page
 * with a live jrq_host_register / jrq_host_alloc range is refused with JRQ_E_STATE and nothing
 * is pinned (its uploads still work, through the bounce chunks).  Page-aligned buffers of
 * whole pages never collide (ByteBuffer.allocateDirect memory need not be: a JNI host that
 * pins many small buffers should carve them from one aligned slab). */
int jrq_host_register(void *ptr, size_t bytes);
/* Call only after the last call that used the buffer has returned, and before the memory is
 * freed: a registration left over freed pages is a stale device mapping of that address.
 * ptr must be the start of a live jrq_host_register range (else JRQ_E_INVALID); on JRQ_E_HIP
 * the range stays registered and known, and the caller must not free the memory. */
int jrq_host_unregister(void *ptr);
/* Leak check: the bytes of the live range starting at ptr (returns 1, or 0 if none), or with
 * ptr == NULL the bytes of every live range (returns their count).  No reference counterpart. */
int jrq_host_registered_bytes(const void *ptr, size_t *bytes);
/* Page-locked host memory owned by the HIP driver (hipHostMalloc): staging for a host that has
 * no buffer of its own to register (the C++ mirror's pack buffers).  The pages never return to
 * the process heap while the device may map them.  *out = NULL on failure. */
int jrq_host_alloc(size_t bytes, void **out);
int jrq_host_free(void *ptr);

/* Test and A/B hooks: per-engine overrides of kernel and staging choices.  A host never needs
 * them, and the library reads nothing from the environment (a JVM that loads libjrq gets the
 * defaults).  No reference counterpart. */
typedef enum {
    JRQ_DBG_CRC_SEG_BYTES = 1,   /* fixed segment size of the CRC segment walk, 0 = automatic */
    JRQ_DBG_CRC_REGS = 2,        /* boundary path: -1 per call site (default), 0 global, 1 registers */
    JRQ_DBG_CRC_PRIO = 3,        /* progress-stepped wave priority steps, 0..3 (default 1) */
    JRQ_DBG_CRC_SEG_MAP = 4,     /* 1 contiguous chunks per workgroup (default), 0 interleaved */
    JRQ_DBG_UPLOAD_PAGEABLE = 5  /* 1: host variants hand unregistered caller memory to HIP's
                                    pageable copies (uploads and result downloads) instead of the
                                    pinned bounce chunks */
} jrq_debug_option;
int jrq_debug_set(jrq_engine *e, int option, int64_t value);

/* ---------------------------------------------------------------- quorum -- */

/* One quorum epoch for G groups: committed_out[g] = the lastCommittedIndex that
 * BallotBox.commitAt (JC/core/BallotBox.java:96-139, Ballot.grant/isGranted
 * JC/entity/Ballot.java:100-140) reaches after all of group g's acks of the epoch,
 * in any order; status_out[g] = jrq_group_status flags.  committed_out may alias
 * in->last_committed.  pendingIndex after the epoch is committed_out[g]+1 when it
 * advanced (BallotBox.java:130-132). */
int jrq_quorum_epoch_dev(jrq_engine *e, const jrq_group_batch *in_dev, int64_t *committed_out_dev,
                         uint8_t *status_out_dev, uint32_t G);
int jrq_quorum_epoch(jrq_engine *e, const jrq_group_batch *in_host, int64_t *committed_out,
                     uint8_t *status_out, uint32_t G);

/* The same epoch with the per-group inputs in tiles of 256 groups (the resident table's tiling
 * with int64 match words): tile i holds match[0..num_peers-1], pending_index, last_appended,
 * last_committed, conf of groups [256 i, 256 i + 256), each field as 256 consecutive int64
 * words, so a tile is 256 (num_peers + 4) words and the tiles sit back to back from `tiles`
 * (G rounded up to whole tiles).  A wave then reads one contiguous block instead of num_peers
 * + 4 rows.  The conf runs and the outputs are as jrq_quorum_epoch_dev's.
 * tiles and committed_out 16-B aligned, status_out 2-B aligned, G >= 2 (JRQ_E_INVALID
 * otherwise). */
typedef struct {
    const int64_t *tiles;
    uint32_t num_peers;
    const uint32_t *run_off;    /* nullable: no group flagged JRQ_CONF_RUNS */
    const int64_t *run_start;
    const uint64_t *run_conf;
} jrq_group_tiles;
int jrq_quorum_epoch_tiles_dev(jrq_engine *e, const jrq_group_tiles *in_dev, int64_t *committed_out_dev,
                               uint8_t *status_out_dev, uint32_t G);
/* Host variant (the JNI binding's stateless contract, INTEGRATION.md §2.5: one direct buffer
 * of tiles per batch): the tiles and the run table are host memory, uploaded in one copy each;
 * G >= 2.  Groups with several runs must carry JRQ_CONF_RUNS in their tile's conf word. */
int jrq_quorum_epoch_tiles(jrq_engine *e, const jrq_group_tiles *in_host, int64_t *committed_out,
                           uint8_t *status_out, uint32_t G);

/* K successive epochs of the same G groups in one launch (the launch-bound small-G case,
 * e.g. C2's 10k groups; SURVEY.md §7 hard part 4).  Epoch k reads
 *   match + k*match_epoch_ld   (rows of in->match_ld, as jrq_quorum_epoch)
 *   last_appended + k*la_epoch_ld
 * and the group state carried from epoch k-1 exactly as BallotBox carries it: a commit sets
 * lastCommittedIndex and pendingIndex = lastCommittedIndex + 1 (JC/core/BallotBox.java:
 * 131-134); pendingIndex 0 (not leader) stays 0.  in->pending_index / last_committed / conf
 * are the state before epoch 0; the conf runs (JRQ_CONF_RUNS groups, as for
 * jrq_quorum_epoch_dev) hold for all K epochs, entries appended in later epochs extending a
 * group's last run.
 * Out: committed_out[k*G + g], status_out[k*G + g] after each epoch. */
int jrq_quorum_epochs_dev(jrq_engine *e, const jrq_group_batch *in_dev, uint32_t K,
                          uint64_t match_epoch_ld, uint64_t la_epoch_ld,
                          int64_t *committed_out_dev, uint8_t *status_out_dev, uint32_t G);

/* K epochs as jrq_quorum_epochs_dev, every epoch's inputs in the tile layout of
 * jrq_quorum_epoch_tiles_dev: epoch k's tiles start epoch_ld int64 words after epoch 0's
 * (epoch_ld even, >= the tiles' extent 256 (num_peers + 4) ceil(G / 256)); epoch k's match and
 * last_appended words come from its own tiles, pending_index / last_committed / conf (the state
 * before epoch 0) from epoch 0's.  Out as jrq_quorum_epochs_dev: committed_out[k*G + g],
 * status_out[k*G + g].  tiles and committed_out 16-B aligned, status_out 2-B aligned, G >= 2,
 * G even when K > 1 (JRQ_E_INVALID otherwise). */
int jrq_quorum_epochs_tiles_dev(jrq_engine *e, const jrq_group_tiles *in_dev, uint32_t K,
                                uint64_t epoch_ld, int64_t *committed_out_dev,
                                uint8_t *status_out_dev, uint32_t G);

/* -------------------------------------------------- resident group table -- */

/* The drop-in path for a long-running multi-Raft host: the BallotBox state of G groups lives
 * on the device (HBM), the host ships only what changed since the previous epoch, and an epoch
 * returns only the groups whose lastCommittedIndex advanced.  Per group it holds exactly what
 * BallotBox holds (JC/core/BallotBox.java:50-55): pendingIndex, lastCommittedIndex, the
 * pending queue as lastAppended plus its conf runs (one Ballot.init(conf, oldConf) per run
 * instead of per entry, :197-215), and, per peer slot, the highest index the peer has
 * acknowledged through commitAt (Replicator acks are contiguous, Replicator.java:1387-1401).
 *
 * Device layout: tiles of 256 groups (jrq_table_view) holding match[P] as u32 words relative to
 * the group's match base (below), pending_index, last_appended, last_committed, conf (run 0 +
 * JRQ_CONF_RUNS) as int64 words, and JRQ_TABLE_MAX_RUNS - 1 inline extra runs (run_start,
 * run_conf) in rows read only by flagged groups.  After its first commit a group's
 * pending_index word holds JRQ_PI_FOLLOWS_LC (pendingIndex = lastCommittedIndex + 1,
 * BallotBox.java:131-132), so a commit writes one word of state.
 * Match base: pendingIndex - 1 rounded down to a multiple of 2^JRQ_TABLE_MATCH_PAGE (0 when not
 * the leader); a slot's word is its match minus the base, 0 for a match below the base (it
 * grants no pending entry either way).  Headers with a negative pendingIndex, one >= 2^62, a
 * lastAppended below pendingIndex - 1, or a pending queue longer than 2^31 - 1 entries (a Java
 * ArrayList's bound) are refused as invalid, as are lastAppended records with v > 2^31 - 1.  A
 * header without JRQ_STATE_RESET_MATCH that lowers the match base (never one the BallotBox API
 * produces: resetPendingIndex resets the matches) keeps words at 0 at 0: no grant is invented. */
#define JRQ_TABLE_MATCH_PAGE 30
#define JRQ_TABLE_MAX_RUNS 4            /* conf runs per pending window (NodeImpl has <= 2) */
#define JRQ_TABLE_MAX_GROUPS (1u << 27) /* groups per table (27-bit group ids in records) */
#define JRQ_PI_FOLLOWS_LC INT64_MIN
#define JRQ_TABLE_SLICE 128             /* groups per slice of an epoch's changed list (_dev) */

typedef struct jrq_table jrq_table;

/* Full header of one group: what resetPendingIndex (:167-186), clearPendingTasks (:147-156),
 * setLastCommittedIndex (:223-248) and a conf-changing appendPendingTask (:197-215) leave
 * behind.  Runs: run 0 covers [pendingIndex, run_start[1]), run r covers [run_start[r],
 * run_start[r+1]) and the last run ends at last_appended; num_runs 0 = nothing pending. */
typedef struct {
    uint32_t group;
    uint16_t num_runs;       /* 0..JRQ_TABLE_MAX_RUNS */
    uint16_t flags;          /* JRQ_STATE_RESET_MATCH: every slot's match = pendingIndex - 1 */
    int64_t pending_index;   /* 0 = not the leader; JRQ_PI_FOLLOWS_LC = last_committed + 1 */
    int64_t last_appended;   /* pendingIndex + pendingMetaQueue.size() - 1 */
    int64_t last_committed;
    uint64_t run_conf[JRQ_TABLE_MAX_RUNS];  /* JRQ_CONF words */
    int64_t run_start[JRQ_TABLE_MAX_RUNS];  /* run_start[0] is ignored (<= pendingIndex) */
} jrq_group_state;           /* 96 bytes */
#define JRQ_STATE_RESET_MATCH 1u  /* (JRQ_STATE_STAMP: see the order-free ack records below) */

/* 8-byte update record: bits 0-4 field, bits 5-31 group, bits 32-63 v, a value relative to
 * the group's pendingIndex pi (after this call's group states are applied):
 *   field 0..15  match of peer slot `field` = pi - 1 + v: the `last` of the peer's latest
 *                BallotBox.commitAt(first, last, peer) (v = 0: no pending entry acked)
 *   field 16     last_appended = pi - 1 + v: v = pendingMetaQueue.size() after
 *                appendPendingTask calls that kept the conf (BallotBox.java:197-215)
 * v fits 32 bits because the pending queue is a Java ArrayList (int size).  At most one
 * record per (group, field) per call. */
#define JRQ_REC_LAST_APPENDED 16u
#define JRQ_REC(group, field, v)                                                               \
    (((uint64_t)(uint32_t)(v) << 32) | ((uint64_t)(uint32_t)(group) << 5) | (uint64_t)(field))

/* A table of G groups x num_peers slots on the engine's device, every group initially not
 * the leader (pendingIndex 0, nothing pending).  Destroy before the engine. */
jrq_table *jrq_table_create(jrq_engine *e, uint32_t G, uint32_t num_peers, int *err);
void jrq_table_destroy(jrq_table *t);

/* Apply n_states group headers, then n_recs update records, on the engine's stream.  Host
 * variant: states / recs are host memory (ideally jrq_host_register'ed, e.g. DirectByteBuffers)
 * copied with one H2D transfer each; they must stay unchanged until the next jrq_table_epoch
 * or jrq_synchronize returns.  Invalid headers / records (group >= G, num_runs or field out of
 * range) are skipped on the device and counted: jrq_table_check reports them. */
int jrq_table_update(jrq_table *t, const jrq_group_state *states, uint32_t n_states,
                     const uint64_t *recs, uint32_t n_recs);
int jrq_table_update_dev(jrq_table *t, const jrq_group_state *states_dev, uint32_t n_states,
                         const uint64_t *recs_dev, uint32_t n_recs);
/* Host variant gathering `parts` pieces (e.g. one per packing thread, each its own registered
 * buffer): the same as one jrq_table_update with every part's headers back to back, then every
 * part's records back to back.  A group's header and its records must sit in the same part
 * (records are relative to the pendingIndex its header sets). */
int jrq_table_update_gather(jrq_table *t, uint32_t parts, const jrq_group_state *const *states,
                            const uint32_t *n_states, const uint64_t *const *recs,
                            const uint32_t *n_recs);

/* Streamed form of jrq_table_update_gather, for a host that packs its updates in parts on
 * several threads and wants each part's DMA to overlap the packing of the next:
 * jrq_table_stage_reserve sizes the device staging for up to max_states headers and max_recs
 * records (it may synchronise, and drops parts staged but never applied), each jrq_table_stage queues
 * the H2D copy of one part behind the previous ones (an asynchronous DMA when the memory is
 * page-locked: jrq_host_alloc / jrq_host_register; the memory must stay unchanged until the
 * next jrq_table_epoch or jrq_synchronize returns), and jrq_table_stage_apply applies every
 * staged header, then every staged record, as jrq_table_update_gather does with its parts. */
int jrq_table_stage_reserve(jrq_table *t, uint32_t max_states, uint32_t max_recs);
int jrq_table_stage(jrq_table *t, const jrq_group_state *states, uint32_t n_states,
                    const uint64_t *recs, uint32_t n_recs);
int jrq_table_stage_apply(jrq_table *t);

/* Order-free ack records (r06): what BallotBox.commitAt (the `last` of an ack) and
 * appendPendingTask (the new lastAppended) record at call time, shipped as they were written --
 * no pack pass over the groups' state at flush time (BallotBox.java:96-139, 197-215).
 *   JRQ_ACK(group, field, index): bits 0-4 field (0..15 a peer slot, JRQ_REC_LAST_APPENDED),
 *   bits 5-31 group, bits 32-63 the low 32 bits of the absolute log index.
 * jrq_table_stage_apply applies them after the staged headers and JRQ_REC records, in any order
 * (an order-free max): the device reconstructs the absolute index as the one within 2^31 of the
 * group's pendingIndex - 1 (an ack lies in [pendingIndex - 1, pendingIndex + 2^31 - 1): the
 * window of an ArrayList-bounded queue) and raises the slot's match, or lastAppended, to it.
 * Records of a group that is not the leader (pendingIndex 0) are ignored.
 * Stamps: records are staged in segments, each with a stamp S (a host-wide counter of resets,
 * read when the segment was started).  A header with JRQ_STATE_STAMP sets the group's reset
 * stamp R (from its run_start[0], which a header otherwise ignores); a record of that group
 * from a segment with S < R is dropped -- it was recorded before the reset that header ships
 * (an ack of an ended leadership, clearPendingTasks :147-156, or of a slot's previous peer).
 * jrq_table_stage_reserve_acks sizes the staging for max_acks records in max_segments segments
 * (it may synchronise, and drops acks staged but never applied); jrq_table_stage_acks queues
 * one segment's H2D copy (asynchronous from page-locked memory, which must then stay unchanged
 * until the next jrq_table_epoch or jrq_synchronize returns).  Invalid records (group >= G, a
 * field past the slots, a lastAppended window >= 2^31 - 1) are skipped and counted
 * (jrq_table_check). */
#define JRQ_ACK(group, field, index)                                                           \
    (((uint64_t)(uint32_t)(int64_t)(index) << 32) | ((uint64_t)(uint32_t)(group) << 5) |       \
     (uint64_t)(field))
#define JRQ_STATE_STAMP 2u
int jrq_table_stage_reserve_acks(jrq_table *t, uint32_t max_acks, uint32_t max_segments);
int jrq_table_stage_acks(jrq_table *t, uint64_t stamp, const uint64_t *acks, uint32_t n);
/* Records streamed to the device while they are written (r06): a caller keeps device regions of
 * the table (jrq_table_ack_region: `capacity` records, freed with the table or by
 * jrq_table_ack_region_free, which synchronises), queues copies of page-locked records into them
 * as they fill (jrq_table_ack_push: from any thread, concurrently with the table's other calls --
 * it only queues an H2D copy on the engine's stream and reports failure by code alone; pageable
 * memory is refused with JRQ_E_INVALID), and at the flush registers each segment where it lies
 * (jrq_table_stage_acks_dev: `n` records at a device address, after jrq_table_stage_reserve_acks,
 * whose max_acks then counts only the records copied by jrq_table_stage_acks).  The copies queued
 * before jrq_table_stage_apply are on the stream ahead of the apply. */
int jrq_table_ack_region(jrq_table *t, uint64_t capacity, uint64_t **region_out);
int jrq_table_ack_region_free(jrq_table *t, uint64_t *region);
int jrq_table_ack_push(jrq_table *t, uint64_t *region_dst, const uint64_t *host_src, uint32_t n);
int jrq_table_stage_acks_dev(jrq_table *t, uint64_t stamp, const uint64_t *acks_dev, uint32_t n);

/* One quorum epoch over every group of the table, state updated in place as BallotBox.commitAt
 * leaves it (BallotBox.java:96-139; commit -> lastCommittedIndex, pendingIndex = commit + 1).
 * Each group whose lastCommittedIndex advanced is listed once, as the word
 * (uint64)(commit - pi + 1) << 32 | group (pi = its pendingIndex before the epoch), in no
 * particular order; status_out[g] (nullable) = jrq_group_status.
 * Host variant: changed_out[0 .. *n_changed) (capacity G); synchronises and copies back only
 * the listed entries.
 * _dev: the list comes in jrq_table_slices(t) fixed slices, one per JRQ_TABLE_SLICE groups
 * (no reservation, no atomics: each slice is written by the one wave that decides its groups),
 * slice s at changed_out_dev + 128 s (capacity JRQ_TABLE_SLICE * jrq_table_slices(t) words):
 * words 0-1 a 128-bit map (bit i: group 128 s + i advanced), then from byte 16 the listed
 * groups' (commit - pi + 1) as uint32, in group order; n_changed_dev[s] = the map's popcount. */
int jrq_table_epoch_dev(jrq_table *t, uint64_t *changed_out_dev, uint32_t *n_changed_dev,
                        uint8_t *status_out_dev);
int jrq_table_epoch(jrq_table *t, uint64_t *changed_out, uint32_t *n_changed,
                    uint8_t *status_out);
uint32_t jrq_table_slices(const jrq_table *t);  /* ceil(G / JRQ_TABLE_SLICE) */

/* Copy the table's state to host arrays (each nullable): pendingIndex resolved (never
 * JRQ_PI_FOLLOWS_LC), last_appended, last_committed [G], match [num_peers][G]. */
int jrq_table_read(jrq_table *t, int64_t *pending_index, int64_t *last_appended,
                   int64_t *last_committed, int64_t *match);

/* JRQ_E_INVALID if headers or records were skipped as invalid since the last check (the
 * count is then reset); synchronises. */
int jrq_table_check(jrq_table *t);

/* Copy the whole state of src into dst (same G and num_peers), on dst's engine stream: a
 * device-side snapshot / restore of the group table. */
int jrq_table_copy(jrq_table *dst, const jrq_table *src);

/* Device views of the table.  The per-group fields live in tiles of tile_groups (256) groups:
 * element g of an int64 field is field[(g / tile_groups) * tile_stride + g % tile_groups] (each
 * tile holds every field of its groups in one contiguous block: an epoch wave reads one block).
 * The u32 match words of tile i start at match + 2 i tile_stride, slot p's 256 words at
 * + 256 p, group k of the tile at position k; match = match base + word
 * (JRQ_TABLE_MATCH_PAGE). */
typedef struct {
    uint32_t *match;         /* u32 words of tile 0 */
    int64_t *pending_index;  /* JRQ_PI_FOLLOWS_LC after a commit */
    int64_t *last_appended;
    int64_t *last_committed;
    uint64_t *conf;
    uint64_t ld;             /* row stride of the table's cold (per-run) fields */
    uint32_t G, num_peers;
    uint32_t tile_groups;    /* 256 (2 JRQ_TABLE_SLICE) */
    uint64_t tile_stride;    /* int64 words from a tile to the next: 128 num_peers + 1024 */
} jrq_table_view;
int jrq_table_view_get(jrq_table *t, jrq_table_view *view_out);

/* --------------------------------------------------------------- checksum -- */

/* crc_out[i] = CrcUtil.crc64(payload[offsets[i] .. offsets[i+1]))
 * (JC/util/CrcUtil.java:36-80 -> CRC64.update JC/util/CRC64.java:100-110):
 * CRC-64/ECMA-182, MSB first, init 0, xorout 0.  offsets has N+1 monotone entries
 * (byte positions into payload; offsets[0] need not be 0).  Zero-length ranges give 0. */
int jrq_crc64_batch_dev(jrq_engine *e, const uint8_t *payload_dev, const uint64_t *offsets_dev,
                        uint32_t N, uint64_t *crc_out_dev);
int jrq_crc64_batch(jrq_engine *e, const uint8_t *payload, const uint64_t *offsets, uint32_t N,
                    uint64_t *crc_out);
/* Fixed-size entries: N entries of entry_bytes each, back to back from payload_dev (no offsets
 * array).  The batch jrq_crc64_batch_dev would see with offsets[i] = i * entry_bytes -- same
 * results.  Entries that split into k = 1, 2, 4 .. 64 pieces of whole 256-B multiples, one
 * piece per lane of the engine's grid, on a 16-B aligned payload, run the one-launch
 * fixed-size kernel (crc64.hip crc64_fixed_kernel); anything else goes through the offsets
 * path.  The host variants route batches of equal entries there by themselves. */
int jrq_crc64_fixed_dev(jrq_engine *e, const uint8_t *payload_dev, uint64_t entry_bytes, uint32_t N,
                        uint64_t *crc_out_dev);

/* Streaming CRC64 as a java.util.zip.Checksum (JC/util/CRC64.java:26,106-126), batched over S
 * independent streams: the RheaKV snapshot archive checksum, fed by CheckedOutputStream /
 * CheckedInputStream around ZipUtil.compress / decompress
 * (RK/storage/AbstractKVStoreSnapshotFile.java:121-123,139-143; RK/util/ZipUtil.java:45-94).
 * For each s: state[s] = the CRC64 register after CRC64.update(chunk_s) where
 * chunk_s = payload[offsets[s] .. offsets[s+1]) and the register held state[s] before, i.e.
 *   state[s] = state[s] * x^(8 |chunk_s|) ^ crc64(chunk_s)   (mod the ECMA-182 poly).
 * getValue() = state[s]; reset() = set it to 0 (host-side, no call).  Successive calls on
 * the same state array continue the streams, so an archive can be fed in pieces of any size.
 * The _dev variant keeps state on the device (in/out); the host variant copies it both ways. */
int jrq_crc64_stream_update_dev(jrq_engine *e, uint64_t *state_dev, const uint8_t *payload_dev,
                                const uint64_t *offsets_dev, uint32_t S);
int jrq_crc64_stream_update(jrq_engine *e, uint64_t *state, const uint8_t *payload,
                            const uint64_t *offsets, uint32_t S);

/* out[i] = LogEntry.checksum() of entry i (JC/entity/LogEntry.java:88-108):
 *   (uint64)type[i] ^ LogId(index[i],term[i]).checksum() ^ peer_xor[i] ^ crc64(data_i)
 * with LogId.checksum = crc64(BE64(index) || BE64(term)) (JC/entity/LogId.java:45-50) and
 * peer_xor[i] = XOR of PeerId.checksum() over peers/oldPeers/learners/oldLearners
 * (precomputed per conf on the host; NULL = 0 for data entries, NodeImpl.java:1201-1203).
 * Verify mode (expected != NULL): corrupt_out[i] = LogEntry.isCorrupted()
 * = has[i] && expected[i] != out[i] (:156-158); has == NULL means every entry has one. */
int jrq_logentry_checksum_batch_dev(jrq_engine *e, const uint8_t *type_dev, const int64_t *index_dev,
                                    const int64_t *term_dev, const uint64_t *peer_xor_dev,
                                    const uint8_t *payload_dev, const uint64_t *offsets_dev,
                                    uint32_t N, uint64_t *out_dev, const uint64_t *expected_dev,
                                    const uint8_t *has_dev, uint8_t *corrupt_out_dev);
int jrq_logentry_checksum_batch(jrq_engine *e, const uint8_t *type, const int64_t *index,
                                const int64_t *term, const uint64_t *peer_xor,
                                const uint8_t *payload, const uint64_t *offsets, uint32_t N,
                                uint64_t *out, const uint64_t *expected, const uint8_t *has,
                                uint8_t *corrupt_out);
/* Fixed-size entries (see jrq_crc64_fixed_dev): entry i = payload_dev[i*entry_bytes, +entry_bytes). */
int jrq_logentry_checksum_fixed_dev(jrq_engine *e, const uint8_t *type_dev, const int64_t *index_dev,
                                    const int64_t *term_dev, const uint64_t *peer_xor_dev,
                                    const uint8_t *payload_dev, uint64_t entry_bytes, uint32_t N,
                                    uint64_t *out_dev, const uint64_t *expected_dev,
                                    const uint8_t *has_dev, uint8_t *corrupt_out_dev);

/* ------------------------------------------- follower verify on receive -- */

/* Batched follower-side verify of R AppendEntries requests holding N EntryMetas in total
 * (NodeImpl.handleAppendEntriesRequest, JC/core/NodeImpl.java:1766-1792; logEntryFromMeta
 * :1809-1823; wire format raft.proto EntryMeta / rpc.proto AppendEntriesRequest):
 *   req_off[R+1]      entries of request r are [req_off[r], req_off[r+1])
 *   prev_log_index[R] entry i of request r has index prev_log_index[r] + 1 + (i - req_off[r])
 *   term/type/data_len/checksum/has_checksum[N]   the EntryMeta fields (has_checksum nullable:
 *                     every entry carries one); peer_xor[N] nullable (XOR of the entry's
 *                     PeerId checksums, as for jrq_logentry_checksum_batch)
 *   data              every request's consumed data bytes, back to back in request order;
 *                     an ENTRY_TYPE_UNKNOWN (0) entry consumes no bytes and is never corrupt
 * Out: checksum_out[N] = LogEntry.checksum() of each entry as received, corrupt_out[N] =
 * isCorrupted(), first_corrupt_out[R] = position in its request of the first corrupt
 * entry (the one the reference rejects with EINVAL, :1777-1789), or -1. */
int jrq_append_entries_verify_dev(jrq_engine *e, uint32_t R, const uint32_t *req_off_dev,
                                  const int64_t *prev_log_index_dev, uint32_t N,
                                  const int64_t *term_dev, const uint8_t *type_dev,
                                  const int64_t *data_len_dev, const uint64_t *peer_xor_dev,
                                  const uint64_t *checksum_dev, const uint8_t *has_checksum_dev,
                                  const uint8_t *data_dev, uint64_t *checksum_out_dev,
                                  uint8_t *corrupt_out_dev, int32_t *first_corrupt_out_dev);
int jrq_append_entries_verify(jrq_engine *e, uint32_t R, const uint32_t *req_off,
                              const int64_t *prev_log_index, uint32_t N, const int64_t *term,
                              const uint8_t *type, const int64_t *data_len,
                              const uint64_t *peer_xor, const uint64_t *checksum,
                              const uint8_t *has_checksum, const uint8_t *data,
                              uint64_t *checksum_out, uint8_t *corrupt_out,
                              int32_t *first_corrupt_out);

/* ------------------------------------------------- leader lease / alive quorum -- */

/* The q-of-n primitive on timestamps for G leader groups:
 * NodeImpl.handleStepDownTimeout (JC/core/NodeImpl.java:2003-2016) -> checkDeadNodes0
 * (:1970-2000) for the conf and, when not empty, the old conf.  Per group g:
 *   last_rpc_ts[p*ld + g]  ReplicatorGroup.getLastRpcSendTimestamp of peer slot p
 *   conf[g]                packed conf word (masks + quorums, JRQ_CONF)
 *   self_slot[g]           the leader's own slot (always alive)
 * A member is alive if now_ms - ts <= lease_timeout_ms.  ok_out[g] bit0 = the conf has an
 * alive quorum, bit1 = the old conf has one (or there is none); lease_start_inout[g] is
 * lastLeaderTimestamp, moved to the oldest alive timestamp by every passing check;
 * dead_out[g] (nullable) = slots found dead.  A group with ok_out != 3 steps down
 * (ERAFTTIMEDOUT "Majority of the group dies"). */
int jrq_lease_check_dev(jrq_engine *e, const int64_t *last_rpc_ts_dev, uint64_t ld,
                        uint32_t num_peers, const uint64_t *conf_dev, const uint8_t *self_slot_dev,
                        uint32_t G, int64_t now_ms, int64_t lease_timeout_ms, uint8_t *ok_out_dev,
                        int64_t *lease_start_inout_dev, uint16_t *dead_out_dev);
int jrq_lease_check(jrq_engine *e, const int64_t *last_rpc_ts, uint64_t ld, uint32_t num_peers,
                    const uint64_t *conf, const uint8_t *self_slot, uint32_t G, int64_t now_ms,
                    int64_t lease_timeout_ms, uint8_t *ok_out, int64_t *lease_start_inout,
                    uint16_t *dead_out);

/* ------------------------------------------------ ReadIndex heartbeat quorum -- */

/* The ReadOnlySafe round of NodeImpl.readLeader (JC/core/NodeImpl.java:1343-1396) for G leader
 * groups, one heartbeat round per group (ReadOnlyServiceImpl batches a group's reads into one
 * ReadIndexRequest), decided as ReadIndexHeartbeatResponseClosure.run does (:1246-1291).
 * Per group g:
 *   conf[g]       packed conf word (JRQ_CONF): its new-conf mask is the peer list (getQuorum,
 *                 :1321-1327: quorum = peers.size()/2 + 1; <= 1 answers at once)
 *   self_slot[g]  the leader's own slot (no heartbeat to it)
 *   order[g]      4 bits per peer slot: the arrival position (1..15) of that slot's heartbeat
 *                 response so far, 0 = none yet (equal positions: lower slot first)
 *   ok_mask[g]    bit p = slot p's response was OK with success = true (else a failure)
 * result_out[g] = JRQ_READINDEX_SUCCESS once ackSuccess + 1 >= quorum, JRQ_READINDEX_FAILURE
 * once ackFailures >= failPeersThreshold (quorum - 1 for an even peer count, quorum for an
 * odd one), whichever the arrival order reached first, else JRQ_READINDEX_PENDING;
 * JRQ_READINDEX_INVALID when conf[g] names a slot >= num_peers (no response can come from it:
 * the input is outside the contract, and the group would otherwise stay pending).  Stateless:
 * call again with the round's later responses added; a verdict never changes.  The host keeps
 * readLeader's other checks (the term of lastCommittedIndex, the requester in the conf, the
 * lease-based option). */
#define JRQ_READINDEX_PENDING 0
#define JRQ_READINDEX_SUCCESS 1
#define JRQ_READINDEX_FAILURE 2
#define JRQ_READINDEX_INVALID 3
int jrq_readindex_quorum_dev(jrq_engine *e, const uint64_t *conf_dev, const uint8_t *self_slot_dev,
                             const uint64_t *order_dev, const uint16_t *ok_mask_dev,
                             uint32_t num_peers, uint32_t G, uint8_t *result_out_dev);
int jrq_readindex_quorum(jrq_engine *e, const uint64_t *conf, const uint8_t *self_slot,
                         const uint64_t *order, const uint16_t *ok_mask, uint32_t num_peers,
                         uint32_t G, uint8_t *result_out);

/* ---------------------------------------------------------------- leader tick -- */

/* The leader's periodic pass over G leader groups in one launch: jrq_lease_check_dev's lease
 * check (NodeImpl.handleStepDownTimeout -> checkDeadNodes, JC/core/NodeImpl.java:1970-2016)
 * and jrq_readindex_quorum_dev's ReadIndex round (:1246-1396) of the same groups, which read
 * the same conf word and self slot once.  The arguments and outputs are those two calls';
 * order / ok_mask / ri_result_out may all be NULL (the lease check alone).  A JNI host calls it
 * from the step-down timer (handleStepDownTimeout runs every electionTimeout / 2) with the
 * heartbeat responses collected since the last tick.  No single reference counterpart: it
 * batches two per-node timer / callback paths into one device pass. */
int jrq_leader_tick_dev(jrq_engine *e, const int64_t *last_rpc_ts_dev, uint64_t ld,
                        uint32_t num_peers, const uint64_t *conf_dev, const uint8_t *self_slot_dev,
                        uint32_t G, int64_t now_ms, int64_t lease_timeout_ms, uint8_t *ok_out_dev,
                        int64_t *lease_start_inout_dev, uint16_t *dead_out_dev,
                        const uint64_t *order_dev, const uint16_t *ok_mask_dev,
                        uint8_t *ri_result_out_dev);
int jrq_leader_tick(jrq_engine *e, const int64_t *last_rpc_ts, uint64_t ld, uint32_t num_peers,
                    const uint64_t *conf, const uint8_t *self_slot, uint32_t G, int64_t now_ms,
                    int64_t lease_timeout_ms, uint8_t *ok_out, int64_t *lease_start_inout,
                    uint16_t *dead_out, const uint64_t *order, const uint16_t *ok_mask,
                    uint8_t *ri_result_out);

/* ------------------------------------------------------- commit fan-out -- */

/* What each group's FSMCaller does with the epoch's commit, for G groups:
 * BallotBox.commitAt -> onCommitted(committed) (JC/core/BallotBox.java:131-137) ->
 * FSMCallerImpl.doCommitted (JC/core/FSMCallerImpl.java:462-482) ->
 * ClosureQueueImpl.popClosureUntil (JC/closure/ClosureQueueImpl.java:113-142).
 *   prev_committed[g]  lastCommittedIndex before the epoch (the quorum epoch's input)
 *   committed[g]       after the epoch (the quorum epoch's output)
 *   last_applied[g]    FSMCaller lastAppliedIndex
 *   cq_first/cq_size   the group's ClosureQueue (firstIndex, number of queued closures),
 *                      updated in place by the pop
 * Out: status_out[g] (jrq_fanout_status); first_closure_out[g] = popClosureUntil's return
 * for APPLY (the log index of the first popped closure, or committed+1 when none is popped),
 * -1 for INVALID, 0 otherwise; listed_bitmap_out[ceil(G/64)]: bit (g & 63) of word g >> 6 is
 * set for the APPLY and INVALID groups -- those whose state machine must apply
 * (last_applied, committed] (or fail with "Invalid firstClosureIndex") -- and
 * *num_listed_out counts them. */
typedef enum {
    JRQ_FAN_NONE = 0,    /* commit did not move: no onCommitted */
    JRQ_FAN_APPLY = 1,   /* doCommitted pops closures (maybe none) and applies entries */
    JRQ_FAN_SKIP = 2,    /* lastAppliedIndex >= committed: doCommitted returns at once */
    JRQ_FAN_INVALID = 3  /* committed beyond the closure queue: popClosureUntil returns -1 */
} jrq_fanout_status;

int jrq_commit_fanout_dev(jrq_engine *e, uint32_t G, const int64_t *prev_committed_dev,
                          const int64_t *committed_dev, const int64_t *last_applied_dev,
                          int64_t *cq_first_inout_dev, int64_t *cq_size_inout_dev,
                          int64_t *first_closure_out_dev, uint8_t *status_out_dev,
                          uint64_t *listed_bitmap_out_dev, uint32_t *num_listed_out_dev);
int jrq_commit_fanout(jrq_engine *e, uint32_t G, const int64_t *prev_committed,
                      const int64_t *committed, const int64_t *last_applied,
                      int64_t *cq_first_inout, int64_t *cq_size_inout,
                      int64_t *first_closure_out, uint8_t *status_out,
                      uint64_t *listed_bitmap_out, uint32_t *num_listed_out);

/* ----------------------------------------- V2 decode + verify on read -- */

/* Batched read-side decode of N stored V2 log entries and their checksum verify
 * (SURVEY §8f #4): AutoDetectDecoder.decode (JC/entity/codec/AutoDetectDecoder.java:41-52)
 * -> V2Decoder.decode (JC/entity/codec/v2/V2Decoder.java:46-110; PBLogEntry, log.proto:10-20,
 * protobuf 3.5.1) -> LogEntry.isCorrupted (JC/entity/LogEntry.java:88-108,156-158), as
 * LogManagerImpl checks every entry it reads (JC/core/LogManagerImpl.java:733-745).
 *   records[offsets[r] .. offsets[r+1])  the stored bytes of entry r (any base/alignment;
 *   a 128-B aligned base lets a batch of equal data lengths take the one-pass fixed-size path) 
 * Out per record: status_out (jrq_v2_status); for JRQ_V2_OK: type (EntryType number), index,
 * term, stored checksum + has_checksum, data_off (absolute into `records`) / data_len of the
 * data field, peer_counts (nullable: peers | old_peers<<8 | learners<<16 | old_learners<<24,
 * each saturating at 255), checksum_out = LogEntry.checksum() of the decoded entry and
 * corrupt_out = isCorrupted().  Other statuses zero those fields (data_off = offsets[r]). */
typedef enum {
    JRQ_V2_OK = 0,
    JRQ_V2_NULL = 1,  /* the reference decoder returns null (empty record, short header, bad
                         magic/version, InvalidProtocolBufferException, missing required field) */
    JRQ_V2_V1 = 2,    /* first byte is not the V2 magic: AutoDetectDecoder routes it to V1Decoder */
    JRQ_V2_HOST = 3   /* decode on the host with the reference decoder: a peer string that is not
                         PeerId.toString() of itself (re-rendered or rejected by getPeerId), or
                         unknown-field groups nested deeper than 2 */
} jrq_v2_status;

int jrq_v2_decode_verify_dev(jrq_engine *e, const uint8_t *records_dev, const uint64_t *offsets_dev,
                             uint32_t N, uint8_t *status_out_dev, uint8_t *type_out_dev,
                             int64_t *index_out_dev, int64_t *term_out_dev,
                             uint64_t *stored_checksum_out_dev, uint8_t *has_checksum_out_dev,
                             uint64_t *data_off_out_dev, uint64_t *data_len_out_dev,
                             uint32_t *peer_counts_out_dev, uint64_t *checksum_out_dev,
                             uint8_t *corrupt_out_dev);
int jrq_v2_decode_verify(jrq_engine *e, const uint8_t *records, const uint64_t *offsets, uint32_t N,
                         uint8_t *status_out, uint8_t *type_out, int64_t *index_out,
                         int64_t *term_out, uint64_t *stored_checksum_out,
                         uint8_t *has_checksum_out, uint64_t *data_off_out,
                         uint64_t *data_len_out, uint32_t *peer_counts_out,
                         uint64_t *checksum_out, uint8_t *corrupt_out);

/* --------------------------------------------------- node-wide publication -- */

/* Multi-GPU (one process per GPU): groups are sharded by contiguous groupId blocks.
 * jrq_publish_committed_dev all-gathers each rank's int64 committed[count_per_rank]
 * into global_dev[nranks*count_per_rank] over RCCL/xGMI, the node-wide snapshot read
 * by getLastCommittedIndex consumers (JC/core/BallotBox.java:67-79, Replicator.java:1433).
 * The unique id is 128 opaque bytes produced on rank 0 and shared out of band. */
int jrq_rccl_get_unique_id(uint8_t id_out[128]);
int jrq_rccl_init(jrq_engine *e, int nranks, int rank, const uint8_t id[128]);
/* Ranks of the engine's communicator as RCCL itself counts them (ncclCommCount); 0 before
 * jrq_rccl_init, negative on error. */
int jrq_rccl_nranks(jrq_engine *e);
int jrq_publish_committed_dev(jrq_engine *e, const int64_t *local_dev, int64_t *global_dev,
                              uint64_t count_per_rank);

/* Single-process form (r06): one host process -- a JVM holding every region of its node, as
 * RheaKV's StoreEngine does (RK/StoreEngine.java:93) -- drives n engines, one per GPU, each with
 * a resident table over a contiguous block of the node's groups (jraft::ShardedGroupBatch).
 * jrq_rccl_init_all creates one communicator per engine in one call (ncclCommInitAll over the
 * engines' devices, rank i = engines[i]); JRQ_E_RCCL if RCCL refuses (e.g. two engines on one
 * device), and the engines then have none. */
int jrq_rccl_init_all(jrq_engine *const *engines, int n);
/* The node-wide snapshot of n engines' committed[count_per_engine] arrays: global_dev[i] (on
 * engine i's device, n * count_per_engine words) receives every local_dev[j] at j *
 * count_per_engine.  One grouped RCCL all-gather when every engine has a communicator from
 * jrq_rccl_init_all; else device-to-device copies (hipMemcpyPeerAsync, each destination stream
 * waiting for the source engine's stream, and each source stream then waiting for the copies
 * that read its buffer, so a later write of local_dev[j] on engine j's stream follows them).
 * Asynchronous on each engine's stream. */
int jrq_publish_committed_all_dev(jrq_engine *const *engines, int n, const int64_t *const *local_dev,
                                  int64_t *const *global_dev, uint64_t count_per_engine);
/* FSMCaller state beside the table (r06): per group lastAppliedIndex (FSMCallerImpl, JC/core/
 * FSMCallerImpl.java:462-470) and its ClosureQueue's (firstIndex, size) (JC/closure/
 * ClosureQueueImpl.java:83-142), all 0 at creation.  jrq_table_fsm_update sets n groups' values
 * (each group at most once per call; a group >= G is skipped and counted, jrq_table_check);
 * jrq_table_fsm_read returns every group's (G words each, nullable outputs).
 * jrq_table_epoch_fanout[_dev] is jrq_table_epoch with jrq_commit_fanout fused in: for every
 * group whose commit moved, FSMCallerImpl.doCommitted's gate and popClosureUntil on its new
 * lastCommittedIndex (jrq_commit_fanout's closed form), the queue updated in place.  Host
 * variant: changed_out as jrq_table_epoch's; fan_first_out[i] / fan_status_out[i] for list
 * entry i (popClosureUntil's result -- the first popped closure's index, committed + 1 when none
 * pops, -1 for INVALID -- and the jrq_fanout_status; NONE is never listed).  Device variant:
 * slices as jrq_table_epoch_dev; fan_first_out[s * JRQ_TABLE_SLICE + r] / fan_status_out[...]
 * for the slice's r-th committing group (r < n_changed_out[s]), jrq_table_slices(t) slices each. */
int jrq_table_fsm_update(jrq_table *t, const uint32_t *groups, const int64_t *last_applied,
                         const int64_t *cq_first, const int64_t *cq_size, uint32_t n);
int jrq_table_fsm_update_dev(jrq_table *t, const uint32_t *groups_dev, const int64_t *last_applied_dev,
                             const int64_t *cq_first_dev, const int64_t *cq_size_dev, uint32_t n);
int jrq_table_fsm_read(jrq_table *t, int64_t *last_applied, int64_t *cq_first, int64_t *cq_size);
int jrq_table_epoch_fanout(jrq_table *t, uint64_t *changed_out, uint32_t *n_changed,
                           int64_t *fan_first_out, uint8_t *fan_status_out);
int jrq_table_epoch_fanout_dev(jrq_table *t, uint64_t *slices_out, uint32_t *n_changed_out,
                               int64_t *fan_first_out, uint8_t *fan_status_out);

/* lastCommittedIndex of every group of the table, contiguous: out_dev[g] for g < G (the tiled
 * lc row de-tiled on the device), asynchronous on the engine's stream -- the local part of a
 * snapshot. */
int jrq_table_committed_dev(jrq_table *t, int64_t *out_dev);

/* A node-wide snapshot object for a single-process host: n tables (one per engine, in group
 * order: table i holds groups [i k, i k + G_i), k = the first table's G; every table but the last
 * has exactly k groups) and, per engine, device buffers of k local and n k gathered words
 * (rank-major, the last block padded with -1).  jrq_snapshot_publish de-tiles every table's
 * committed[] (jrq_table_committed_dev) and gathers them (jrq_publish_committed_all_dev) on the
 * engines' streams; jrq_snapshot_read synchronises engine i and copies its gathered snapshot to
 * host_out[0 .. sum G_i), unpadded (what getLastCommittedIndex readers on any GPU see,
 * BallotBox.java:67-79).  jrq_snapshot_via: 1 = RCCL (jrq_rccl_init_all succeeded), 0 = copies. */
typedef struct jrq_snapshot jrq_snapshot;
jrq_snapshot *jrq_snapshot_create(jrq_table *const *tables, int n, int *err);
void jrq_snapshot_destroy(jrq_snapshot *s);
int jrq_snapshot_publish(jrq_snapshot *s);
int jrq_snapshot_read(jrq_snapshot *s, int i, int64_t *host_out);
int jrq_snapshot_via(const jrq_snapshot *s);

#ifdef __cplusplus
}
#endif
#endif /* JRQ_H */
