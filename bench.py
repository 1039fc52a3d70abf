#!/usr/bin/env python3
"""bench.py -- quorum commit decisions/s (+ LogEntry CRC64 GB/s) on 1..8 MI355X.

Driver contract: `python bench.py --gpus N --steps K --warmup W`; N>1 is launched by
torch.distributed.run (one rank per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from env).
Rank 0 prints ONE JSON line.

Headline (`value`): quorum commit decisions/s, whole job.  Workload per GPU = 1M Raft
groups x 5 peers with joint-consensus masks (BASELINE config C3 at N=1; at N>1 config
C4: 8M groups sharded by contiguous groupId blocks, 1M per GPU, weak scaling).  One
step = one quorum epoch kernel over the GPU's groups; at N>1 the step also publishes
the node-wide committed-index snapshot with an RCCL all-gather over xGMI every
--publish-every steps (jraft_amd.dist.ShardedEpochs: the loop the gloo tests run).
Inputs are device-resident; the step cycles through several distinct epochs (> the
256 MiB Infinity Cache) so every launch reads its inputs from HBM.

Other legs in the same run (--legs selects; the PMC passes run one leg each so every kernel
name carries one workload): C2 (configs[1]) one epoch and 64 epochs per launch, C5 as
BASELINE states it (CRC64 verify + commit), C1 on the GPU, the SURVEY §8f legs, HIP-event
kernel times -> `roofline`, and the oracle (Java-faithful C restatement) timed on this
host -> `cpu_baseline` (per config, 1 / 16 / all threads).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
QUORUM_EPOCH_BUFFERS = 6
LEGS = ("quorum", "table", "drive", "C2", "C2L", "C3K", "C5", "C1", "ae", "v2", "snapshot", "pinned",
        "lease", "readindex", "tick", "fanout", "peak", "cpu")


def quorum_bytes_per_group(P: int) -> int:
    """Bytes one group decision moves in this layout: reads match 8P,
    pendingIndex 8, lastAppended 8, lastCommitted 8, conf 8; writes committed 8, status 1.
    SURVEY §8(d) prices it at 8P + 38 (2+2 B masks + 1 B flags); the 8-B conf word (masks +
    explicit quorums + the JRQ_CONF_RUNS flag) is 3 B more: +3.7 % at P = 5."""
    return 8 * P + 41


def crc_bytes(n_entries: int, payload_bytes: int, verify: bool = True, offsets: bool = True) -> int:
    # payload + offsets (N+1)*8 (not for fixed-size entries) + per entry type 1, index 8, term 8,
    # out 8 (+ expected 8, corrupt 1)
    b = payload_bytes + (8 * (n_entries + 1) if offsets else 0) + n_entries * (1 + 8 + 8 + 8)
    if verify:
        b += n_entries * (8 + 1)
    return b


def to_dev(arr, dev):
    """A device copy of numpy `arr`, staged through page-locked host memory: the bench hands no
    pageable memory to a HIP copy.  HIP locks the pages of a large pageable copy itself and may
    keep them locked after the copy; an array freed afterwards and a later allocation at the
    same address then meet a lock over pages that no longer exist -- rounds 4 and 5 each saw one
    run end in "illegal memory access" at a result copy of the lease leg, after the C5 / C1 legs'
    GiB-sized pageable transfers (profiles/faults/)."""
    import torch
    if arr is None:
        return None
    a = arr.view(np.int64) if arr.dtype == np.uint64 else arr
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(dev)


def host_np(t):
    """numpy copy of device tensor `t` through page-locked host memory (see to_dev)."""
    import torch
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h.numpy()


# ------------------------------------------------------------------ PMC citations --

def csrc_sha() -> str:
    """Content hash of the kernel sources: a committed PMC summary is cited only when it was
    collected from these exact kernels (tools/summarize_profiles.py writes the same hash), and
    the library must carry the same hash as its jrq_build_id() (main() checks)."""
    from jraft_amd._srcsha import src_sha
    return src_sha()


def pmc_traffic(leg: str, *kernels: str):
    """HBM bytes per launch of the timed op (summed over `kernels`, name substrings), from the
    committed PMC summary of this leg's own pass (profiles/*_pmc.json, "legs" section, written
    by tools/summarize_profiles.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
    of `bench.py --legs <leg>`), only if it was collected from the current kernel sources."""
    sha = csrc_sha()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("csrc_sha") != sha:
            continue
        ks = d.get("legs", {}).get(leg, {})
        total = 0.0
        for kern in kernels:
            hit = [v["hbm_bytes_per_launch"] for name, v in ks.items() if kern in name]
            if not hit:
                break
            total += hit[0]
        else:
            return {"traffic": total, "traffic_source": os.path.relpath(f, ROOT) +
                    f" [legs.{leg}] ({d.get('correction', '2*FETCH_SIZE+WRITE_SIZE')})"}
    return {"traffic": None, "traffic_source": None}


def roofline(alg_bytes: float, ms: float, **extra) -> dict:
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS, "bytes_per_launch": alg_bytes, "kernel_ms": ms,
            **extra}


# ------------------------------------------------------------------ timing --

# Untimed warm-up: besides the --warmup calls, each timed series first runs its own work for
# at least this much GPU time.  A GPU coming out of idle (every leg starts after seconds of
# host-side input generation) runs its first few ms of streaming kernels up to 15 % slower
# (C5 verify: 0.255 ms/launch over 20 launches after 3 warm-up calls, 0.222 ms in steady
# state, same box, tools/ab_inproc.py); the timed region should see the steady state.
WARM_MS = 200.0


def warm_until(fn, stream, sync, warm_ms=None, calls=None):
    """Call fn(i) back to back until `warm_ms` of its GPU time has run (at most 4096 calls) --
    or exactly `calls` times: a function holding a collective must make the same number of
    calls on every rank."""
    import torch
    if calls is not None:
        for i in range(calls):
            fn(i)
        sync()
        return calls
    warm_ms = WARM_MS if warm_ms is None else warm_ms
    done, n, batch = 0.0, 0, 4
    while done < warm_ms and n < 4096:
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for j in range(batch):
            fn(n + j)
        z.record(stream)
        sync()
        done += a.elapsed_time(z)
        n += batch
        batch = min(batch * 2, 256)
    return n


_MARK = {}
# the leg each timed series belongs to, in mark order (the full result's `timed_series_legs`:
# tools/leg_traces.py pairs them with the start marks of a trace of the same run)
_SERIES = []
_LEG = [None]


def mark(stream, end=False):
    """A one-element kernel on `stream` right outside a timed series' event pair -- a
    bitwise-not before it, a negation after it (ops the legs use nowhere else): in a rocprofv3
    kernel trace the launches between the two are exactly one timed series (tools/leg_traces.py
    reads them that way).  Costs nothing inside the pair."""
    import torch
    t = _MARK.get(stream.device)
    if t is None:
        t = _MARK[stream.device] = torch.zeros(1, dtype=torch.int32, device=stream.device)
    with torch.cuda.stream(stream):
        if end:
            t.neg_()
        else:
            _SERIES.append(_LEG[0])
            t.bitwise_not_()


def timed_launches(fn, steps, warmup, stream, sync, warm_calls=None):
    """`warmup` untimed calls plus WARM_MS of untimed calls (warm_until), then `steps` calls
    back to back between ONE pair of HIP events on `stream` (the engine's stream): the
    per-launch time is that span / steps.  This is the only timing method used for `roofline`
    (rocprofv3's per-kernel averages in profiles/ agree with it; per-launch event pairs stretch
    a ~17 us kernel by 2-3 us)."""
    import torch
    for i in range(warmup):
        fn(i)
    sync()
    warm_until(fn, stream, sync, calls=warm_calls)
    b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    mark(stream)
    t0 = time.perf_counter()
    b0.record(stream)
    for i in range(steps):
        fn(i)
    b1.record(stream)
    mark(stream, end=True)
    sync()
    wall = time.perf_counter() - t0
    return b0.elapsed_time(b1) / steps, wall


# ------------------------------------------------------------------ CPU side --

def cpu_info() -> dict:
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "cgroup_cpu_quota": quota}


def thread_counts(info: dict) -> list[int]:
    """1 thread, the box's per-GPU CPU share (16), and every CPU this process may run on
    (capped by a cgroup quota when one is set)."""
    full = info["affinity_cpus"] or 1
    if info["cgroup_cpu_quota"]:
        full = max(1, min(full, int(info["cgroup_cpu_quota"])))
    return sorted({1, min(16, full), full})


def _threaded(fn, items, threads, budget_s):
    """Run fn(item) over `items` round-robin on `threads` threads until budget_s has passed
    (ctypes releases the GIL inside the oracle's C calls, so the threads run in parallel).
    Returns (calls completed, wall seconds, sum of fn results)."""
    import threading
    lock = threading.Lock()
    state = {"next": 0, "done": 0, "acc": 0}
    t0 = time.perf_counter()

    def worker():
        while time.perf_counter() - t0 < budget_s:
            with lock:
                i = state["next"]
                state["next"] += 1
            r = fn(items[i % len(items)])
            with lock:
                state["done"] += 1
                state["acc"] += r
    ts = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return state["done"], time.perf_counter() - t0, state["acc"]


def _per_threads(fn, items, unit_per_call, counts, budget_s):
    out = {}
    for n in counts:
        calls, wall, acc = _threaded(fn, items, n, budget_s)
        out[str(n)] = {"value": calls * unit_per_call / wall, "calls": calls, "seconds": wall,
                       "grants": acc or None}
    return out


def cpu_quorum_baseline(cfg, info, budget_s):
    """Oracle (Java-faithful BallotBox replay, oracle/jraft_oracle.c) on groups of `cfg`
    (C3 / C2), over disjoint group chunks per thread -- one BallotBox per group, as in the
    reference: groups never share a lock -- plus the optimised-CPU line (oracle/cpu_fast.c)."""
    import jraft_oracle as O
    from jraft_amd import workloads as W
    counts = thread_counts(info)
    chunk_groups = 256
    chunks = [W.quorum_batch(cfg, groups=chunk_groups, group_offset=k * chunk_groups)
              for k in range(2 * max(counts))]

    def replay(b):
        return O.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                     b["last_committed"], b["conf"], chunk=1024)[2]
    faithful = _per_threads(replay, chunks, chunk_groups, counts, budget_s)
    fast_groups = 1 << 16
    fchunks = [W.quorum_batch(cfg, groups=fast_groups, group_offset=k * fast_groups)
               for k in range(min(16, max(counts)))]

    def fast(b):
        O.fast_quorum_epoch(b["match"], b["pending_index"], b["last_appended"],
                            b["last_committed"], b["conf"])
        return 0
    opt = _per_threads(fast, fchunks, fast_groups, counts, 1.0)
    best = str(max(counts))
    return {"value": faithful[best]["value"], "unit": "decisions/s", "cores": max(counts),
            "kind": "port", "per_threads": faithful,
            "optimised": {"per_threads": {k: v["value"] for k, v in opt.items()},
                          "how": "closed-form q-th largest per conf mask per group "
                                 "(oracle/cpu_fast.c, same results as the BallotBox replay)"},
            "sample": f"{cfg} groups (1k pending each) replayed through the Java-faithful "
                      f"BallotBox restatement in chunks of {chunk_groups} groups, "
                      f"{budget_s:.0f} s per thread count"}


def cpu_crc_baseline(info, budget_s):
    """Byte-at-a-time LogEntry.checksum restatement over C5 entries (16 KiB)."""
    import jraft_oracle as O
    from jraft_amd import workloads as W
    counts = thread_counts(info)
    n = 256  # 4 MiB of C5 entries per call
    batches = [W.entry_batch(n, 16 << 10, seed=5 + k) for k in range(min(16, max(counts)))]
    gb = n * (16 << 10) / 1e9

    def run(b):
        O.logentry_checksum_batch(b["etype"], b["index"], b["term"], None, b["payload"],
                                  b["offsets"])
        return 0
    faithful = _per_threads(run, batches, gb, counts, budget_s)

    def fast(b):
        O.fast_crc64_batch(b["payload"], b["offsets"])
        return 0
    fast(batches[0])  # builds the slice tables before the threads start
    opt = _per_threads(fast, batches, gb, counts, 1.0)
    best = str(max(counts))
    return {"value": faithful[best]["value"], "unit": "GB/s", "cores": max(counts),
            "kind": "port", "per_threads": faithful,
            "optimised": {"per_threads": {k: v["value"] for k, v in opt.items()},
                          "how": "slice-by-8 CRC64 (oracle/cpu_fast.c) over the same payloads"},
            "sample": f"C5 LogEntries x 16 KiB through the byte-at-a-time CRC64.update "
                      f"restatement, 4 MiB per call, {budget_s:.0f} s per thread count"}


def cpu_c1_baseline(info):
    """C1 exactly as configs[0] states it, on the host: 1M appended 256-B DATA LogEntries
    checksummed byte-at-a-time (LogManagerImpl.appendEntries stamps each on one thread,
    LogManagerImpl.java:313-318) plus the group's BallotBox.commitAt replay over its 1M pending
    ballots, acks in 1024-entry chunks from 3 peers (one BallotBox = one lock: single thread).
    The checksum leg is also timed split across threads (not what the reference does)."""
    import jraft_oracle as O
    from jraft_amd import workloads as W
    c1 = W.CONFIGS["C1"]
    n = c1["pending"]
    e1 = W.entry_batch(n, c1["entry_bytes"], seed=W.SEED_BASE ^ 1)
    q1 = W.quorum_batch("C1")
    t0 = time.perf_counter()
    O.logentry_checksum_batch(e1["etype"], e1["index"], e1["term"], None, e1["payload"],
                              e1["offsets"])
    t_crc = time.perf_counter() - t0
    t0 = time.perf_counter()
    _, _, grants = O.quorum_epoch_replay(q1["match"], q1["pending_index"], q1["last_appended"],
                                         q1["last_committed"], q1["conf"], chunk=1024)
    t_commit = time.perf_counter() - t0
    counts = thread_counts(info)
    split = {}
    for T in counts:
        if T == 1:
            continue
        step = -(-n // T)
        parts = [(i, min(n, i + step)) for i in range(0, n, step)]

        def part(p):
            a, b = p
            O.logentry_checksum_batch(e1["etype"][a:b], e1["index"][a:b], e1["term"][a:b], None,
                                      e1["payload"], e1["offsets"][a:b + 1])
            return 0
        import threading
        t0 = time.perf_counter()
        ths = [threading.Thread(target=part, args=(p,)) for p in parts]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        wall = time.perf_counter() - t0
        split[str(T)] = {"entries_per_s": n / (wall + t_commit), "checksum_s": wall}
    return {"value": n / (t_crc + t_commit), "unit": "entries/s (checksum + commit)", "cores": 1,
            "kind": "port", "checksum_s": t_crc, "commit_s": t_commit, "grants": grants,
            "checksum_GBps": n * c1["entry_bytes"] / t_crc / 1e9,
            "checksum_split_threads": split,
            "sample": "the whole C1 step: 1M x 256 B byte-at-a-time LogEntry.checksum + one "
                      "BallotBox replay of 1M pending entries (Java-faithful C restatement)"}


# ------------------------------------------------------------------ legs --

class Ctx:
    def __init__(self, eng, stream, dev, world, rank, args):
        self.eng, self.stream, self.dev = eng, stream, dev
        self.world, self.rank, self.args = world, rank, args
        self.oracle_checks = rank == 0 and not args.no_cpu
        # the process group's backend: "nccl" (RCCL, the driver's scaling runs) or "gloo"
        # (tests/test_gpu_bench_ranks.py: several ranks on one GPU, which RCCL refuses);
        # gloo reduces host tensors
        self.backend = getattr(args, "dist_backend", "nccl")

    def coll_device(self):
        """Where this process group's small collectives (max over ranks, gathers) run."""
        import torch
        return self.dev if self.backend == "nccl" else torch.device("cpu")

    def sync(self):
        import torch
        torch.cuda.synchronize(self.dev)

    def gather(self, x: float) -> list:
        """x from every rank, in rank order (a one-float all-reduce per call)."""
        if self.world == 1:
            return [x]
        import torch
        import torch.distributed as dist
        t = torch.zeros(self.world, dtype=torch.float64, device=self.coll_device())
        t[self.rank] = x
        dist.all_reduce(t)
        return [float(v) for v in (host_np(t) if t.is_cuda else t.numpy())]

    def timed(self, fn, steps=None, warmup=None, warm_calls=None):
        a = self.args
        return timed_launches(fn, a.steps if steps is None else steps,
                              a.warmup if warmup is None else warmup, self.stream, self.sync,
                              warm_calls)


def leg_quorum(ctx, args, barrier, max_over_ranks):
    """The headline: C3 (N=1) / C4 (N>1) epochs through dist.ShardedEpochs."""
    import torch

    from jraft_amd import Engine
    from jraft_amd import dist as D
    from jraft_amd import workloads as W
    eng, dev, world, rank = ctx.eng, ctx.dev, ctx.world, ctx.rank
    G = args.groups_per_gpu
    cfg = "C3" if world == 1 else "C4"
    P = W.CONFIGS[cfg]["peers"]
    Gtot = G * world
    epochs, tiled = [], []
    for e in range(QUORUM_EPOCH_BUFFERS):
        b = W.quorum_batch(cfg, groups=G, group_offset=rank * G,
                           seed=(W.SEED_BASE ^ int(cfg[1])) + 7919 * e)
        epochs.append({k: to_dev(v, dev) for k, v in b.items()})
        # the same epoch in the resident table's tile layout (jrq_quorum_epoch_tiles_dev)
        tiled.append(to_dev(W.to_tiles(b["match"], b["pending_index"], b["last_appended"],
                                       b["last_committed"], b["conf"]), dev))
    k = D.per_rank(Gtot, world)
    local = torch.empty(k, dtype=torch.int64, device=dev)
    status = torch.empty(G, dtype=torch.uint8, device=dev)
    # one GPU: the local committed[] already is the node-wide snapshot (nothing to gather)
    snapshot = torch.empty(k * world, dtype=torch.int64, device=dev) if world > 1 else local
    def rccl_init():
        uid = [Engine.rccl_unique_id() if rank == 0 else None]
        import torch.distributed as dist
        dist.broadcast_object_list(uid, src=0)
        if os.environ.get("JRAFT_AMD_INJECT_RCCL_FAIL"):  # tests of the fallback
            raise RuntimeError("injected jrq_rccl_init failure (JRAFT_AMD_INJECT_RCCL_FAIL)")
        eng.rccl_init(world, rank, uid[0])
        return eng.rccl_nranks()

    def pg_publish(send, recv):
        import torch.distributed as dist
        if ctx.backend == "nccl":  # device tensors through the process group (RCCL via torch)
            dist.all_gather_into_tensor(recv, send)
            return
        ctx.sync()
        h = torch.empty(send.numel() * world, dtype=send.dtype)
        dist.all_gather_into_tensor(h, torch.from_numpy(host_np(send)))
        recv.copy_(to_dev(h.numpy(), recv.device))

    def agree(ok):
        import torch.distributed as dist
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=ctx.coll_device())
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    publish_fn, pub_info = D.choose_publish(world, ctx.backend, rccl_init, eng.publish_committed_dev,
                                            pg_publish, agree)

    # one prepared launch per epoch buffer (arguments resolved once, as a C / JNI host keeps
    # its jrq_group_batch): the step loop then costs the GPU epoch, not Python marshalling
    # The headline launches the epoch on tiled inputs (each wave reads one contiguous block:
    # DESIGN.md §4.1); the same epochs from rows (jrq_quorum_epoch_dev) are timed beside it.
    rows = [eng.quorum_epoch_launcher(t["match"], t["pending_index"], t["last_appended"],
                                      t["last_committed"], t["conf"], local, status)
            for t in epochs]
    launchers = [eng.quorum_epoch_tiles_launcher(tt, P, G, local, status) for tt in tiled]

    def epoch_fn(i, out):
        if out is local:
            launchers[i % QUORUM_EPOCH_BUFFERS]()
            return
        t = epochs[i % QUORUM_EPOCH_BUFFERS]
        eng.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                             t["last_committed"], t["conf"], out, status)

    def allgather(send, recv):
        if publish_fn is not None:
            publish_fn(send, recv)
    se = D.ShardedEpochs(Gtot, world, rank, epoch_fn, allgather, local, snapshot,
                         publish_every=args.publish_every)
    # kernel only (HIP events on the engine's stream)
    rows_ms, _ = ctx.timed(lambda i: rows[i % QUORUM_EPOCH_BUFFERS]())
    rows_ms = max_over_ranks(rows_ms)
    k_ms, _ = ctx.timed(lambda i: epoch_fn(i, local))
    pub_ms = None
    k_ms_max = max_over_ranks(k_ms)
    # the same number of warm-up steps on every rank (they hold the all-gather)
    warm_steps = int(min(4096, max(1, WARM_MS / max(k_ms_max, 1e-3))))
    if world > 1:
        pub_ms, _ = ctx.timed(lambda i: se.publish(), warm_calls=64)
    # the contract's timed region: K steps between barrier + sync on both sides (after the
    # --warmup steps and WARM_MS of untimed steps)
    for _ in range(args.warmup):
        se.step()
    ctx.sync()
    warm_until(lambda i: se.step(), ctx.stream, ctx.sync, calls=warm_steps)
    barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        se.step()
    ctx.sync()
    barrier()
    ctx.sync()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    value = Gtot * args.steps / elapsed
    ok = None
    if ctx.oracle_checks:  # 4096 groups of the last epoch against the oracle replay
        import jraft_oracle as O
        i = (se.steps - 1) % QUORUM_EPOCH_BUFFERS
        b = W.quorum_batch(cfg, groups=G, group_offset=rank * G,
                           seed=(W.SEED_BASE ^ int(cfg[1])) + 7919 * i)
        idx = np.random.default_rng(7).choice(G, 4096, replace=False)
        ce, _, _ = O.quorum_epoch_replay(b["match"][:, idx], b["pending_index"][idx],
                                         b["last_appended"][idx], b["last_committed"][idx],
                                         b["conf"][idx], chunk=1024)
        ok = bool(np.array_equal(host_np(local)[idx], ce))
    bpg = quorum_bytes_per_group(P)
    rl = roofline(bpg * G, k_ms, kernel="quorum_epoch_pair_kernel<5, false, true>", bytes_per_group=bpg,
                  survey_bytes_per_group=8 * P + 38,
                  frac_survey_bytes=(8 * P + 38) * G / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                  timing="one HIP event pair around --steps back-to-back launches / steps",
                  inputs="tiles (jrq_quorum_epoch_tiles_dev)",
                  **pmc_traffic("quorum", "quorum_epoch_pair_kernel<5, false, true>"))
    rl_rows = roofline(bpg * G, rows_ms, kernel="quorum_epoch_pair_kernel<5, false, false>",
                       inputs="rows (jrq_quorum_epoch_dev)",
                       **pmc_traffic("quorum", "quorum_epoch_pair_kernel<5, false, false>"))
    return {
        "value": value, "elapsed": elapsed, "cfg": cfg, "G": G, "P": P, "roofline": rl,
        "multi_gpu": {**pub_info,
                      "publish_every": args.publish_every,
                      "kernel_only_ms": k_ms_max, "publish_ms": pub_ms,
                      "kernel_plus_publish_ms": elapsed * 1e3 / args.steps,
                      "kernel_only_decisions_per_s": Gtot / (k_ms_max * 1e-3),
                      "snapshot_bytes": 8 * k * world},
        "bit_exact_vs_oracle_4096_groups": ok,
        "rows_entry_point": rl_rows,
    }


def table_load(table, s):
    """Load epoch 0 of a host_series batch into a Table the way a host does: one header per
    group (resetPendingIndex + its conf runs), then one 8-B record per peer slot (its acks)."""
    from jraft_amd import Table, _lib
    G = len(s["pending_index"])
    pi = s["pending_index"]
    st = Table.states(G)
    joint = s["switch_at"] != 0
    st["group"] = np.arange(G)
    st["num_runs"] = np.where(joint, 2, 1)
    st["flags"] = _lib.STATE_RESET_MATCH
    # pendingIndex = lastCommitted + 1 (every C3 group): the table's steady-state encoding
    st["pending_index"] = np.where(pi == s["last_committed"] + 1, _lib.PI_FOLLOWS_LC, pi)
    st["last_appended"] = s["last_appended"][0]
    st["last_committed"] = s["last_committed"]
    st["run_conf"][:, 0] = s["conf_a"]
    st["run_conf"][:, 1] = np.where(joint, s["conf_b"], 0)
    st["run_start"][:, 1] = s["switch_at"]
    m = s["match"][0]
    gs = np.arange(G)
    recs = np.concatenate([_lib.rec(gs, p, np.maximum(m[p] - (pi - 1), 0)) for p in range(m.shape[0])])
    table.update(st, recs)  # on the engine stream, before any later epoch
    return st, recs


def leg_table_fanout(ctx, series, pristine, work, lists, series_ms, G, NB, t_ms, alg):
    """The commit fan-out fused into the table epoch (jrq_table_epoch_fanout_dev: FSMCallerImpl
    .doCommitted / ClosureQueueImpl.popClosureUntil of every committing group, FSMCallerImpl.java:
    462-482, ClosureQueueImpl.java:113-142) against the same epoch followed by the separate
    fan-out over dense arrays (jrq_table_committed_dev + jrq_commit_fanout_dev), same timing.
    Each group's FSMCaller is caught up (lastAppliedIndex = lastCommittedIndex) with one closure
    per pending entry (NodeImpl.executeApplyingTasks appends one per task), so every committing
    group pops."""
    import torch

    from jraft_amd import decode_changed
    eng, dev = ctx.eng, ctx.dev
    fsm = []
    for i, t in enumerate(pristine):
        s = series[i]
        lc0 = s["last_committed"].astype(np.int64)
        la0 = s["last_appended"][0].astype(np.int64)
        fsm.append((lc0.copy(), lc0 + 1, np.maximum(la0 - lc0, 0)))
        t.fsm_update(np.arange(G, dtype=np.uint32), *fsm[-1])
    fans = [w.fan_buffers(dev) for w in work]

    def fused(i):
        work[i].epoch_fanout_dev(*lists[i], *fans[i])
    _LEG[0] = "table_fanout"  # (its own label in the trace's timed series)
    f_ms = series_ms(pristine, fused)
    fw = [work[i].gather_dev_list(*lists[i]) for i in range(NB)]
    fn = [host_np(lists[i][1]) for i in range(NB)]
    ff = [host_np(fans[i][0]) for i in range(NB)]
    fs = [host_np(fans[i][1]) for i in range(NB)]
    fq = [work[i].fsm_read() for i in range(NB)]
    prev = [to_dev(series[i]["last_committed"].astype(np.int64), dev) for i in range(NB)]
    appl = [to_dev(fsm[i][0], dev) for i in range(NB)]
    cq0 = [(to_dev(fsm[i][1], dev), to_dev(fsm[i][2], dev)) for i in range(NB)]
    cq = [(torch.empty_like(a), torch.empty_like(b)) for a, b in cq0]
    com = [torch.empty(G, dtype=torch.int64, device=dev) for _ in range(NB)]
    ufc = [torch.empty(G, dtype=torch.int64, device=dev) for _ in range(NB)]
    ust = [torch.empty(G, dtype=torch.uint8, device=dev) for _ in range(NB)]
    ubm = torch.empty((G + 63) // 64, dtype=torch.int64, device=dev)
    unum = torch.zeros(1, dtype=torch.int32, device=dev)

    def restore():
        for (a, b), (a0, b0) in zip(cq, cq0):
            a.copy_(a0)
            b.copy_(b0)

    def unfused(i):
        work[i].epoch_dev(*lists[i])
        work[i].committed_dev(com[i])
        eng.commit_fanout_dev(prev[i], com[i], appl[i], cq[i][0], cq[i][1], ufc[i], ust[i], ubm, unum)
    u_ms = series_ms(pristine, unfused, restore)
    _LEG[0] = "table"
    ok = True
    for i in range(NB):  # fused == epoch + separate fan-out, every group of every table
        g, _ = decode_changed(fw[i])
        ffl = np.concatenate([ff[i][k * 128: k * 128 + fn[i][k]] for k in range(len(fn[i]))])
        fsl = np.concatenate([fs[i][k * 128: k * 128 + fn[i][k]] for k in range(len(fn[i]))])
        st_u, fc_u = host_np(ust[i]), host_np(ufc[i])
        ok = ok and bool(np.array_equal(fsl, st_u[g]) and np.array_equal(ffl, fc_u[g]))
        ok = ok and bool(np.count_nonzero(st_u) == len(g))
        ok = ok and bool(np.array_equal(fq[i][1], host_np(cq[i][0])) and np.array_equal(fq[i][2], host_np(cq[i][1])))
    n_changed = len(fw[-1])
    # the fused epoch reads the FSMCaller rows (24 B per group) and writes per committing group
    # its fan result (9 B) and the popped queue (16 B)
    falg = alg + G * 24 + n_changed * 25
    return {"kernel_ms": f_ms, "epoch_then_fanout_ms": u_ms, "epoch_alone_ms": t_ms,
            "fused_over_epoch_alone": f_ms / t_ms, "fused_over_unfused": f_ms / u_ms,
            "bit_exact_vs_epoch_then_fanout": ok,
            "roofline": roofline(falg, f_ms, kernel="table_epoch_kernel<5, true>",
                                 bytes_note="the epoch's bytes + 24 B of FSMCaller state read per "
                                            "group + 25 B per committing group (fan result, "
                                            "popped queue)",
                                 **pmc_traffic("table", "table_epoch_kernel<5, true>"))}


def leg_table(ctx, args, G, pair_ms):
    """The drop-in path's device cost: one epoch of the resident group table (csrc/table.hip)
    over C3 (1M groups x 5 peers, joint) with 1% of the groups holding a conf change inside
    their pending window, against the stateless pair kernel on the same inputs.  Timed as the
    headline is -- one HIP event pair around back-to-back launches -- over NB distinct tables,
    each restored from its pristine copy (jrq_table_copy) before the series and outside the
    event pair, so that every launch starts from a fresh table and commits as many groups as a
    first epoch does.  (Round 3 timed one launch per event pair after a copy: 2-3 us of
    per-launch overhead on a ~20 us kernel)"""
    import torch

    from jraft_amd import Table, decode_changed
    from jraft_amd import workloads as W
    eng, dev = ctx.eng, ctx.dev
    P = 5
    NB = 4  # distinct inputs per series (4 x ~190 MB of table state: > the 256 MiB Infinity Cache)
    pristine, series, plain = [], [], []
    for e in range(NB):
        s = W.host_series("C3", 1, groups=G, joint_frac=0.01, seed=(W.SEED_BASE ^ 3) + 7919 * e)
        t = Table(eng, G, P)
        table_load(t, s)
        pristine.append(t)
        series.append(s)
    for e in range(NB):  # the same shape with no conf change in any window (no flagged group)
        s0 = W.host_series("C3", 1, groups=G, joint_frac=0.0, seed=(W.SEED_BASE ^ 3) + 7919 * e)
        t = Table(eng, G, P)
        table_load(t, s0)
        plain.append(t)
    work = [Table(eng, G, P) for _ in range(NB)]
    ctx.sync()
    lists = [w.list_buffers(dev) for w in work]
    reps = max(3, args.steps // 4)

    def series_ms(src, launch, restore=None):
        """median over reps of (event pair around NB back-to-back launches) / NB"""
        for w, t in zip(work, src):
            w.copy_from(t)
        if restore:
            restore()
        def warm(i):  # untimed series, each from fresh tables too
            if i % NB == 0:
                for w, t in zip(work, src):
                    w.copy_from(t)
                if restore:
                    restore()
            launch(i % NB)
        warm_until(warm, ctx.stream, ctx.sync, warm_ms=WARM_MS / 4)
        out = []
        for _ in range(reps):
            for w, t in zip(work, src):
                w.copy_from(t)
            if restore:
                restore()
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            mark(ctx.stream)
            a.record(ctx.stream)
            for i in range(NB):
                launch(i)
            z.record(ctx.stream)
            mark(ctx.stream, end=True)
            ctx.sync()
            out.append(a.elapsed_time(z) / NB)
        return float(np.median(out))

    def table_epoch(i):
        work[i].epoch_dev(*lists[i])
    t_ms = series_ms(pristine, table_epoch)
    # the results of the last series (every table fresh): table i's list vs table i's inputs
    words = [work[i].gather_dev_list(*lists[i]) for i in range(NB)]
    n_changed = len(words[-1])
    t_plain_ms = series_ms(plain, table_epoch)
    # the stateless pair kernel on the same inputs (CSR run table, flagged groups), same timing
    dd = []
    for s in series:
        d = {k: to_dev(s[k] if k != "match" else s["match"][0], dev)
             for k in ("match", "pending_index", "last_committed", "conf", "run_off", "run_start",
                       "run_conf")}
        d["last_appended"] = to_dev(s["last_appended"][0], dev)
        d["conf_a"] = to_dev(s["conf_a"], dev)
        dd.append(d)
    pcs = [torch.empty(G, dtype=torch.int64, device=dev) for _ in range(NB)]
    pst = torch.empty(G, dtype=torch.uint8, device=dev)

    def pair(i):
        d = dd[i]
        eng.quorum_epoch_dev(d["match"], d["pending_index"], d["last_appended"],
                             d["last_committed"], d["conf"], pcs[i], pst, run_off=d["run_off"],
                             run_start=d["run_start"], run_conf=d["run_conf"])

    def pair_plain(i):  # the same groups without any conf change
        d = dd[i]
        eng.quorum_epoch_dev(d["match"], d["pending_index"], d["last_appended"],
                             d["last_committed"], d["conf_a"], pcs[i], pst)
    p_ms = series_ms(pristine, pair)  # (the table copies run too: the same cache state)
    pc_flagged = [host_np(x) for x in pcs]
    pp_ms = series_ms(pristine, pair_plain)
    ok = True
    for i in range(NB):  # table == stateless kernel, every group of every table
        s = series[i]
        g, delta = decode_changed(words[i])
        got = s["last_committed"].copy()
        got[g] = s["pending_index"][g] - 1 + delta
        ok = ok and bool(np.array_equal(got, pc_flagged[i]))
    if ctx.oracle_checks:  # and 512 groups (the joint ones first) against the oracle
        import jraft_oracle as O
        s = series[-1]
        g, delta = decode_changed(words[-1])
        got = s["last_committed"].copy()
        got[g] = s["pending_index"][g] - 1 + delta
        jg = np.nonzero(s["switch_at"])[0][:256]
        sub = np.unique(np.concatenate([jg, np.random.default_rng(5).choice(G, 256, replace=False)]))
        ro = s["run_off"]
        cnt = (ro[sub + 1] - ro[sub]).astype(np.uint32)
        idx = np.concatenate([np.arange(ro[x], ro[x + 1]) for x in sub])
        ce, _, _ = O.quorum_epoch_replay(s["match"][0][:, sub], s["pending_index"][sub],
                                         s["last_appended"][0][sub], s["last_committed"][sub],
                                         s["conf"][sub], np.concatenate([[0], np.cumsum(cnt)]),
                                         s["run_start"][idx], s["run_conf"][idx], chunk=1024)
        ok = ok and bool(np.array_equal(got[sub], ce))
    # per group: u32 match words 4P + pendingIndex, lastAppended, lastCommitted, conf 32 read;
    # per committing group lastCommitted 8 + list delta 4 written; per 128-group slice its
    # 16-B map and 4-B count (the flagged groups' run words, ~1 %, not counted)
    alg = G * (4 * P + 32) + n_changed * 12 + ((G + 127) // 128) * 20
    fan = leg_table_fanout(ctx, series, pristine, work, lists, series_ms, G, NB, t_ms, alg)
    for t in pristine + plain + work:
        t.close()
    return {"workload": f"C3 resident table: {G} groups x {P} peers, joint, 1% with a conf "
                        f"change in the pending window; one epoch, in place",
            "kernel_ms": t_ms, "changed_groups": n_changed,
            "kernel_ms_no_conf_change": t_plain_ms,
            "flagged_over_no_conf_change": t_ms / t_plain_ms,
            "stateless_pair_kernel_ms_same_inputs": p_ms,
            "stateless_pair_kernel_ms_no_conf_change": pp_ms,
            "table_over_pair": t_ms / p_ms,
            "no_conf_table_over_pair": t_plain_ms / pp_ms,
            "headline_pair_kernel_ms": pair_ms,
            "timing": f"median over {reps} series of (one HIP event pair around {NB} back-to-back "
                      f"launches on {NB} distinct fresh tables) / {NB}; the restores run before the "
                      f"pair; the pair kernel timed the same way on the same inputs",
            "bit_exact_vs_stateless_kernel_and_oracle": ok,
            "fused_fanout": fan,
            "roofline": roofline(alg, t_ms, kernel="table_epoch_kernel<5, false>",
                                 bytes_note="reads 4P+32 B per group (u32 match words), writes "
                                            "lastCommitted + list delta 12 B per committing group "
                                            "+ 20 B per 128-group slice",
                                 **pmc_traffic("table", "table_epoch_kernel<5, false>"))}


def leg_drive(ctx, args, G):
    """The drop-in path end to end from the host: C3 epochs replayed through the C++ host
    mirror's BallotBox API (appendPendingTask / commitAt) over the resident table, one
    GroupBatch::flush() per epoch (libjraft_drive.so): changed records from page-locked
    buffers -> H2D -> apply + epoch kernels -> D2H of the changed commits -> closures /
    onCommitted.  Reported per steady epoch (epochs 3..K-1: epoch 0 loads every group, epochs 1-2
    size the calling threads' record buffers and their device regions), with
    the epoch's API calls made by 1 and by 16 threads (contiguous group slices), and the
    end-to-end rate including those calls.  Then the ack -> onCommitted latency under the
    background flusher's policy, with 16 producer threads."""
    import torch

    from jraft_amd import drive
    from jraft_amd import workloads as W
    K = 10
    out = {}
    for active, threads, shards in ((1.0, 1, 1), (1.0, 16, 1), (0.1, 16, 1), (1.0, 16, 2)):
        s = W.host_series("C3", K, groups=G, joint_frac=0.01, active=active)
        committed, st = drive.drive_epochs(ctx.dev.index, s, threads=threads, shards=shards)
        ok = None
        if active == 1.0:  # every group against the stateless K-epoch kernel
            d = {k: to_dev(s[k], ctx.dev) for k in ("match", "last_appended", "pending_index",
                                                    "last_committed", "conf", "run_off",
                                                    "run_start", "run_conf")}
            c = torch.empty((K, G), dtype=torch.int64, device=ctx.dev)
            cs = torch.empty((K, G), dtype=torch.uint8, device=ctx.dev)
            ctx.eng.quorum_epochs_dev(d["match"], d["pending_index"], d["last_appended"],
                                      d["last_committed"], d["conf"], c, cs, run_off=d["run_off"],
                                      run_start=d["run_start"], run_conf=d["run_conf"])
            ctx.sync()
            ok = bool(np.array_equal(committed, host_np(c)))
            del d, c, cs
        sl = slice(3, K)
        f = float(np.mean(st["flush_ms"][sl]))
        api = float(np.mean(st["api_ms"][sl]))
        pcie = float(np.mean(st["h2d_bytes"][sl] + st["d2h_bytes"][sl]))
        key = f"active_{int(active * 100)}pct_{threads}_threads"
        out[key + (f"_{shards}_engines" if shards > 1 else "")] = {
            "api_threads": threads, "engines": shards,
            "flush_ms": f, "pack_ms": float(np.mean(st["pack_ms"][sl])),
            "device_ms": float(np.mean(st["device_ms"][sl])),
            "deliver_ms": float(np.mean(st["deliver_ms"][sl])),
            "deliver_apply_ms": float(np.mean(st["deliver_apply_ms"][sl])),
            "deliver_callbacks_ms": float(np.mean(st["deliver_callbacks_ms"][sl])),
            "api_ms_per_epoch": api,
            "api_calls_per_epoch": float(np.mean(st["api_calls"][sl])),
            "end_to_end_ms_per_epoch": api + f,
            "decisions_per_s_end_to_end": G / ((api + f) * 1e-3),
            "decisions_per_s_flush_only": G / (f * 1e-3),
            "api_share_of_end_to_end": api / (api + f),
            "records_per_epoch": float(np.mean(st["records"][sl])),
            "changed_per_epoch": float(np.mean(st["changed"][sl])),
            "pcie_bytes_per_epoch": pcie, "pcie_GBps": pcie / (f * 1e-3) / 1e9,
            "first_epoch_flush_ms": float(st["flush_ms"][0]),
            "sizing_epochs_flush_ms": [float(x) for x in st["flush_ms"][1:3]],
            "bit_exact_vs_stateless_kernel": ok}
    lats = {}
    # (1M groups at one entry per group per second -- 1M entries/s, 5M acks/s -- and at ten:
    # the producers then run at ~90 % duty and contend with the flush for every group's lines)
    for lg, prod, fl, delay, pace, secs in ((G, 8, 8, 1000, 1_000_000, 3.0), (G, 8, 8, 1000, 100_000, 2.0),
                                            (1 << 16, 4, 4, 500, 10_000, 2.0)):
        lat = drive.drive_latency(ctx.dev.index, lg, 5, prod, secs, delay, 1 << 16, flush_threads=fl,
                                  pass_us=pace)
        lat.update({"groups": lg, "producer_threads": prod, "flush_threads": fl,
                    "producer_pass_us": pace,
                    "policy": {"maxDelayUs": delay, "maxDirtyGroups": 1 << 16},
                    "commits_per_s": lat["commits"] / lat["seconds"],
                    "api_calls_per_s": (lat["entries"] + lat["acks"]) / lat["seconds"],
                    "flushes_per_s": lat["flushes"] / lat["seconds"]})
        lat["entries_per_s"] = lat["entries"] / lat["seconds"]
        lats[f"{lg}_groups_pass_{pace // 1000}ms"] = lat
    lats["how"] = ("producer threads loop over their slices of the groups -- one pass per "
                   "producer_pass_us (paced: acks arrive with the network; spinning producers also "
                   "hit the box's cgroup CPU quota, whose throttling then sets the latency) -- "
                   "appendPendingTask of one entry, then commitAt of it by each of the 5 peers; GroupBatch::"
                   "startFlusher flushes when the oldest unflushed change is maxDelayUs old or "
                   "65536 groups changed, packing and delivering on flush_threads threads (producers "
                   "+ flush threads = the 16-CPU share of the box); latency = onCommitted(c) time "
                   "- time of entry c's last ack")
    return {"workload": f"C3 through the C++ BallotBox host mirror: {G} groups x 5 peers, joint, "
                        f"1% with a conf change in the pending window, {K} epochs",
            "how": "flush = pack changed records + H2D (pinned) + apply + epoch kernels + D2H of "
                   "the changed commits + closures / onCommitted; api = the appendPendingTask / "
                   "commitAt calls of the epoch (made before the flush, from `api_threads` threads); "
                   "engines = 2: the groups in two contiguous blocks over two engines on this GPU "
                   "(ShardedGroupBatch), both shards' epochs concurrent, then the node-wide "
                   "committed snapshot published to both engines inside flush_ms (device copies: RCCL "
                   "needs one device per rank), then read back against every BallotBox",
            **out, "ack_to_onCommitted_latency": lats}


def leg_c2(ctx, args):
    """configs[1]: 10k groups x 3 peers x 1k pending -- one epoch per launch (launch-bound) and
    64 successive epochs per launch (jrq_quorum_epochs_dev, the scan kernel)."""
    import torch

    from jraft_amd import workloads as W
    eng, dev = ctx.eng, ctx.dev
    c2 = W.quorum_batch("C2")
    c2d = {k: to_dev(v, dev) for k, v in c2.items()}
    G2 = c2["pending_index"].shape[0]
    c2c = torch.empty(G2, dtype=torch.int64, device=dev)
    c2s = torch.empty(G2, dtype=torch.uint8, device=dev)

    # prepared launches (arguments resolved once, as a C / JNI host would): Python's per-call
    # marshalling (~10 us) otherwise outlasts these 6-9 us kernels in the timed loop
    c2_launch = eng.quorum_epoch_launcher(c2d["match"], c2d["pending_index"], c2d["last_appended"],
                                          c2d["last_committed"], c2d["conf"], c2c, c2s)

    def c2_step(i):
        c2_launch()
    one_ms, one_wall = ctx.timed(c2_step)
    # the product default for a batch this small (< ~50k groups): 256 epochs per launch, which
    # spreads the scan kernel's launch ramp and tail over 256 epochs; 64 epochs
    # per launch are the C2L leg
    KE = 256
    ser = W.quorum_epoch_series("C2", KE)
    ser_d = {k: to_dev(v, dev) for k, v in ser.items()}
    kc = torch.empty((KE, G2), dtype=torch.int64, device=dev)
    ks = torch.empty((KE, G2), dtype=torch.uint8, device=dev)

    c2k_launch = eng.quorum_epochs_launcher(ser_d["match"], ser_d["pending_index"],
                                            ser_d["last_appended"], ser_d["last_committed"],
                                            ser_d["conf"], kc, ks)

    def c2k_step(i):
        c2k_launch()
    k_ms, _ = ctx.timed(c2k_step)
    ok = None
    if ctx.oracle_checks:
        import jraft_oracle as O
    if ctx.oracle_checks:  # the oracle on 128 groups, all KE epochs, state carried
        sub = np.random.default_rng(2).choice(G2, 128, replace=False)
        pi = ser["pending_index"][sub].copy()
        lc = ser["last_committed"][sub].copy()
        got = host_np(kc)
        ok = True
        for k in range(KE):
            ce, _, _ = O.quorum_epoch_replay(ser["match"][k][:, sub], pi,
                                             ser["last_appended"][k][sub], lc,
                                             ser["conf"][sub], chunk=1024)
            pi = np.where((pi != 0) & (ce > lc), ce + 1, pi)
            lc = ce
            ok = ok and bool(np.array_equal(got[k, sub], ce))
    # per group-epoch: match 8P + lastAppended 8 read, committed 8 + status 1 written (41 B at
    # P = 3); pendingIndex / lastCommitted / conf once per group
    alg = G2 * KE * 41 + G2 * 24
    return {"workload": "C2: 10k groups x 3 peers x 1k pending (configs[1])",
            "decisions_per_s": G2 / (one_ms * 1e-3), "kernel_ms": one_ms,
            "entry_ballots_per_s": G2 * 1024 / (one_ms * 1e-3),
            "batched_epochs": {"epochs_per_launch": KE, "kernel_ms": k_ms,
                               "decisions_per_s": G2 * KE / (k_ms * 1e-3),
                               "roofline": roofline(alg, k_ms, kernel="quorum_epochs_kernel<3, 8, 16, 4>",
                                                    **pmc_traffic("C2", "quorum_epochs_kernel<3,")),
                               "bit_exact_vs_oracle_128_groups": ok}}


def leg_c2l(ctx, args):
    """configs[1] with 64 successive epochs per launch (jrq_quorum_epochs_dev), beside the C2
    leg's 256 (the product default): the scan kernel's ramp and tail over a quarter of the work.
    Its own leg, so its PMC pass (one leg per pass) attributes this launch shape's bytes to it
    alone."""
    import torch

    from jraft_amd import workloads as W
    eng, dev = ctx.eng, ctx.dev
    G2 = W.quorum_batch("C2")["pending_index"].shape[0]
    KL = 64
    serl = W.quorum_epoch_series("C2", KL)
    serl_d = {k: to_dev(v, dev) for k, v in serl.items()}
    klc = torch.empty((KL, G2), dtype=torch.int64, device=dev)
    kls = torch.empty((KL, G2), dtype=torch.uint8, device=dev)
    c2l_launch = eng.quorum_epochs_launcher(serl_d["match"], serl_d["pending_index"],
                                            serl_d["last_appended"], serl_d["last_committed"],
                                            serl_d["conf"], klc, kls)
    kl_ms, _ = ctx.timed(lambda i: c2l_launch())
    ok_l = None
    if ctx.oracle_checks:  # 64 groups, all KL epochs, state carried
        import jraft_oracle as O
        sub = np.random.default_rng(3).choice(G2, 64, replace=False)
        pi = serl["pending_index"][sub].copy()
        lc = serl["last_committed"][sub].copy()
        got = host_np(klc)
        ok_l = True
        for k in range(KL):
            ce, _, _ = O.quorum_epoch_replay(serl["match"][k][:, sub], pi,
                                             serl["last_appended"][k][sub], lc,
                                             serl["conf"][sub], chunk=1024)
            pi = np.where((pi != 0) & (ce > lc), ce + 1, pi)
            lc = ce
            ok_l = ok_l and bool(np.array_equal(got[k, sub], ce))
    alg_l = G2 * KL * 41 + G2 * 24
    del serl_d, klc, kls
    return {"epochs_per_launch": KL, "kernel_ms": kl_ms,
            "decisions_per_s": G2 * KL / (kl_ms * 1e-3),
            "roofline": roofline(alg_l, kl_ms, kernel="quorum_epochs_kernel<3, 4, 16, 4>",
                                 **pmc_traffic("C2L", "quorum_epochs_kernel<3,")),
            "bit_exact_vs_oracle_64_groups": ok_l}


def leg_c3k(ctx, args, G):
    """C3 through the K-epochs-per-launch kernel (jrq_quorum_epochs_dev): K successive epochs of
    the 1M groups x 5 peers, joint, state carried between them as BallotBox carries it, in one
    launch -- the headline epoch's launch ramp and tail spread over K epochs."""
    import torch

    from jraft_amd import workloads as W
    eng, dev = ctx.eng, ctx.dev
    K = 8
    ser = W.quorum_epoch_series("C3", K, groups=G)
    d = {k: to_dev(v, dev) for k, v in ser.items()}
    kc = torch.empty((K, G), dtype=torch.int64, device=dev)
    ks = torch.empty((K, G), dtype=torch.uint8, device=dev)
    launch = eng.quorum_epochs_launcher(d["match"], d["pending_index"], d["last_appended"],
                                        d["last_committed"], d["conf"], kc, ks)
    rows_ms, _ = ctx.timed(lambda i: launch())
    rows_c = host_np(kc)
    # the same K epochs with every epoch's inputs in the tile layout (jrq_quorum_epochs_tiles_dev,
    # the headline's layout): the leg's number; the rows entry point is timed beside it
    tiles = to_dev(np.stack([W.to_tiles(ser["match"][k], ser["pending_index"], ser["last_appended"][k],
                                        ser["last_committed"], ser["conf"]) for k in range(K)]), dev)
    tlaunch = eng.quorum_epochs_tiles_launcher(tiles, 5, G, kc, ks)
    ms, _ = ctx.timed(lambda i: tlaunch())
    same_as_rows = bool(np.array_equal(host_np(kc), rows_c))
    ok = None
    if ctx.oracle_checks:  # the oracle on 2048 groups, all K epochs, state carried
        import jraft_oracle as O
        sub = np.random.default_rng(4).choice(G, 2048, replace=False)
        pi = ser["pending_index"][sub].copy()
        lc = ser["last_committed"][sub].copy()
        got, gst = host_np(kc), host_np(ks)
        ok = True
        for k in range(K):
            ce, se, _ = O.quorum_epoch_replay(ser["match"][k][:, sub], pi,
                                              ser["last_appended"][k][sub], lc, ser["conf"][sub],
                                              chunk=1024)
            pi = np.where((pi != 0) & (ce > lc), ce + 1, pi)
            lc = ce
            ok = ok and bool(np.array_equal(got[k, sub], ce)) and bool(np.array_equal(gst[k, sub], se))
    P = 5
    # per group-epoch: match 8P + lastAppended 8 read, committed 8 + status 1 written; per
    # group pendingIndex / lastCommitted / conf once
    alg = G * K * (8 * P + 17) + G * 24
    del d, kc, ks, tiles
    return {"workload": f"C3: {G} groups x {P} peers, joint, {K} successive epochs per launch, "
                        "inputs in tiles (jrq_quorum_epochs_tiles_dev)",
            "epochs_per_launch": K, "kernel_ms": ms,
            "decisions_per_s": G * K / (ms * 1e-3),
            "roofline": roofline(alg, ms, kernel="quorum_epochs_pair_kernel<5, false, true>",
                                 bytes_note="8P+17 B per group-epoch + 24 B per group",
                                 **pmc_traffic("C3K", "quorum_epochs_pair_kernel<5, false, true>")),
            "rows_entry_point": {"kernel_ms": rows_ms, "frac": alg / (rows_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                                 "how": "jrq_quorum_epochs_dev (one array per field)",
                                 "bit_exact_vs_tiles": same_as_rows},
            "bit_exact_vs_oracle_2048_groups": ok}


def leg_pinned(ctx, args, c5state):
    """The host-pointer entry points from caller memory registered with jrq_host_register (a
    JNI host's pinned DirectByteBuffers): LogEntry checksum + verify of the C5
    batch (1 GiB) and the C1 batch (256 MB) with every input and output in registered memory,
    PCIe transfers included; beside them the same calls from unregistered memory (the engine's
    pinned bounce chunks).  The reference copies a direct buffer into a new byte[] before
    checksumming it (CrcUtil.java:65-80)."""
    from jraft_amd import _lib
    from jraft_amd import workloads as W
    eng = ctx.eng
    d, eb, expected, flip, out = c5state
    c1 = W.CONFIGS["C1"]
    e1 = W.entry_batch(c1["pending"], c1["entry_bytes"], seed=W.SEED_BASE ^ 1)
    res = {}
    regs_before = _lib.host_registrations()
    for name, e, exp in (("C5", eb, expected ^ flip.astype(np.uint64)), ("C1", e1, None)):
        n = len(e["offsets"]) - 1
        arrs = {"payload": e["payload"], "etype": e["etype"], "index": e["index"], "term": e["term"],
                "offsets": e["offsets"]}
        if exp is not None:
            arrs["expected"] = np.ascontiguousarray(exp)
        row = {}
        for pinned in (True, False):
            # registered: page-aligned copies that own their pages (a JNI host's DirectByteBuffers
            # carved from an aligned slab), kept alive until after their unregistration, which
            # must succeed (_lib.Registered raises otherwise).  Round 4 registered the arrays in
            # place -- small ones share heap pages with their neighbours -- ignored the
            # unregister codes and freed them; the next legs' copies faulted once.
            src = {k: _lib.page_aligned_copy(a) for k, a in arrs.items()} if pinned else arrs
            with _lib.Registered(src.values() if pinned else ()) as regs:
                def call():
                    return eng.logentry_checksum_batch(src["etype"], src["index"], src["term"],
                                                       None, src["payload"], src["offsets"],
                                                       expected=src.get("expected"))
                call()
                walls = []
                for _ in range(max(3, min(10, args.steps // 5))):
                    t0 = time.perf_counter()
                    r = call()
                    walls.append(time.perf_counter() - t0)
                wall = float(np.median(walls))
                n_regs = len(regs.live)
            del src
            got = r[0] if isinstance(r, tuple) else r
            ok = None
            if ctx.oracle_checks:
                if name == "C5":
                    ok = bool(np.array_equal(got, expected)) and bool(np.array_equal(r[1].astype(bool), flip))
                else:
                    import jraft_oracle as O
                    ok = bool(np.array_equal(got[:4096], O.logentry_checksum_batch(
                        e["etype"][:4096], e["index"][:4096], e["term"][:4096], None, e["payload"],
                        e["offsets"][:4097])))
            pay = int(e["offsets"][-1] - e["offsets"][0])
            h2d = pay + sum(a.nbytes for k, a in arrs.items() if k != "payload")
            row["registered" if pinned else "unregistered"] = {
                "ms_per_call": wall * 1e3, "GBps_payload_pcie_inclusive": pay / wall / 1e9,
                "h2d_bytes": h2d, "registered_arrays": n_regs, "bit_exact_vs_oracle": ok}
        res[name] = {"entries": n, "payload_bytes": int(e["offsets"][-1]), **row}
    regs_after = _lib.host_registrations()
    if regs_after != regs_before:
        raise RuntimeError(f"libjrq page-lock registry {regs_before} -> {regs_after} after the "
                           f"pinned leg: a registration outlived its leg")
    return {"how": "jrq_logentry_checksum_batch (host variant: H2D of every input, the fixed-size "
                   "kernel, D2H of the results, synchronised) timed by wall clock per call; "
                   "registered = every caller array copied to page-aligned memory and "
                   "jrq_host_register'ed first (DMA straight from it), unregistered = through the "
                   "engine's 8 MiB pinned bounce chunks",
            "registry_after": {"ranges": regs_after[0], "bytes": regs_after[1]},
            **res}


def leg_c5(ctx, args, barrier, max_over_ranks, time_it=True):
    """C5 as BASELINE states it: 64k regions x 3 replicas, one 16 KiB DATA entry per region:
    one step = LogEntry CRC64 verify of the 64k entries (1/1024 corrupted) + the commit epoch
    of the 64k groups.  Also reports the verify alone (the `crc64` metric)."""
    import torch

    from jraft_amd import workloads as W
    eng, dev, rank, world = ctx.eng, ctx.dev, ctx.rank, ctx.world
    c5 = W.CONFIGS["C5"]
    n = c5["groups"]
    eb = W.entry_batch(n, c5["entry_bytes"], seed=W.SEED_BASE ^ 5 ^ rank)
    qb = W.quorum_batch("C5", group_offset=rank * n)
    expected = None
    # every rank checks its own shard (rank r's regions r*64k .. (r+1)*64k-1 carry their own
    # payload seed): the oracle's byte-at-a-time pass over 1 GiB takes ~2 s per rank
    checks = not args.no_cpu
    if checks:
        import jraft_oracle as O
        expected = O.logentry_checksum_batch(eb["etype"], eb["index"], eb["term"], None,
                                             eb["payload"], eb["offsets"])
    if expected is None:
        expected = np.zeros(n, np.uint64)
    flip = np.zeros(n, bool)
    flip[::1024] = True  # 1/1024 entries corrupted
    d = {k: to_dev(v, dev) for k, v in eb.items() if isinstance(v, np.ndarray)}
    q = {k: to_dev(v, dev) for k, v in qb.items()}
    d_exp = to_dev(expected ^ flip.astype(np.uint64), dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    corrupt = torch.empty(n, dtype=torch.uint8, device=dev)
    qc = torch.empty(n, dtype=torch.int64, device=dev)
    qs = torch.empty(n, dtype=torch.uint8, device=dev)

    def verify(i):  # 16 KiB entries back to back: the fixed-size entry point (no offsets array)
        eng.logentry_checksum_fixed_dev(d["etype"], d["index"], d["term"], None, d["payload"],
                                        c5["entry_bytes"], out, expected=d_exp, corrupt=corrupt)

    def verify_offsets(i):  # the same batch through the general offsets entry point
        eng.logentry_checksum_batch_dev(d["etype"], d["index"], d["term"], None, d["payload"],
                                        d["offsets"], out, expected=d_exp, corrupt=corrupt)

    def commit(i):
        eng.quorum_epoch_dev(q["match"], q["pending_index"], q["last_appended"],
                             q["last_committed"], q["conf"], qc, qs)

    def step(i):
        verify(i)
        commit(i)
    if not time_it:  # setup for the legs that reuse the C5 entries (one verify for `out`)
        verify(0)
        ctx.sync()
        return None, None, (d, eb, expected, flip, out)
    steps = max(10, args.steps)
    vo_ms, _ = ctx.timed(verify_offsets, steps, 2)
    ok_off = None
    if checks:
        ok_off = bool(np.array_equal(host_np(out).view(np.uint64), expected)) and \
            bool(np.array_equal(host_np(corrupt).astype(bool), flip))
    v_ms, _ = ctx.timed(verify, steps, 2)
    c_ms, _ = ctx.timed(commit, steps, 2)
    s_ms, _ = ctx.timed(step, steps, 2)
    barrier()
    v_max, s_max = max_over_ranks(v_ms), max_over_ranks(s_ms)
    pay = n * c5["entry_bytes"]
    ok = step_ok = None
    if checks:
        ok = bool(np.array_equal(host_np(out).view(np.uint64), expected)) and \
            bool(np.array_equal(host_np(corrupt).astype(bool), flip))
        ce, se, _ = O.quorum_epoch_replay(qb["match"], qb["pending_index"], qb["last_appended"],
                                          qb["last_committed"], qb["conf"], chunk=1024)
        step_ok = ok and bool(np.array_equal(host_np(qc), ce)) and \
            bool(np.array_equal(host_np(qs), se))
    alg_v = crc_bytes(n, pay, verify=True, offsets=False)
    alg_c = quorum_bytes_per_group(3) * n
    per_rank_ms = ctx.gather(v_ms)
    per_rank_ok = ctx.gather(-1.0 if ok is None else float(ok))
    crc = {"metric": "LogEntry CRC64 verify GB/s",
           "value": pay * world / (v_max * 1e-3) / 1e9, "unit": "GB/s (payload)",
           "per_rank_GBps": [pay / (m * 1e-3) / 1e9 for m in per_rank_ms],
           "per_rank_bit_exact": [None if x < 0 else bool(x) for x in per_rank_ok],
           "timing": "max over ranks of each rank's per-launch time (one event pair around "
                     "the launches on its own stream)",
           "workload": "C5: 64k x 16 KiB DATA LogEntries per GPU, checksum + isCorrupted verify "
                       "(jrq_logentry_checksum_fixed_dev: 2 lanes per entry)",
           "ms_per_launch": v_ms, "bit_exact_vs_oracle": ok,
           "offsets_path": {"ms_per_launch": vo_ms, "bit_exact_vs_oracle": ok_off,
                            "GBps_payload": pay / (vo_ms * 1e-3) / 1e9,
                            "how": "jrq_logentry_checksum_batch_dev (segment walk + finish kernel)"},
           "roofline": roofline(alg_v, v_ms, kernel="crc64_fixed_kernel<true, false, 512>",
                                **pmc_traffic("C5", "crc64_fixed_kernel<true, false, 512>"))}
    per_rank_step_ok = ctx.gather(-1.0 if step_ok is None else float(step_ok))
    c5_step = {"workload": f"C5 as BASELINE states it: 64k regions x 3 replicas x 16 KiB entries "
                           f"per GPU ({n * world} regions over {world} GPU(s), region shards by "
                           f"regionId); one step = CRC64 verify of the GPU's entries + commit of "
                           f"its groups",
               "per_rank_bit_exact": [None if x < 0 else bool(x) for x in per_rank_step_ok],
               "ms_per_step": s_ms, "verify_ms": v_ms, "commit_ms": c_ms,
               "regions_per_s": n * world / (s_max * 1e-3),
               "GBps_payload": pay * world / (s_max * 1e-3) / 1e9,
               "bit_exact_vs_oracle": step_ok,
               "roofline": roofline(alg_v + alg_c, s_ms,
                                    bytes_note="verify (payload + 34 B/entry) + commit 65 B/group")}
    return crc, c5_step, (d, eb, expected, flip, out)


def leg_ae(ctx, args, c5state):
    import torch
    from jraft_amd import workloads as W
    eng, dev = ctx.eng, ctx.dev
    d, eb, expected, flip, out = c5state
    c5 = W.CONFIGS["C5"]
    n = c5["groups"]
    R = n // 1024
    req_off = torch.arange(0, n + 1, 1024, dtype=torch.int32, device=dev)
    prev = torch.arange(0, n, 1024, dtype=torch.int64, device=dev)  # index = 1..n
    dlen = torch.full((n,), c5["entry_bytes"], dtype=torch.int64, device=dev)
    d_exp = to_dev(expected ^ flip.astype(np.uint64), dev)
    ae_out = torch.empty(n, dtype=torch.int64, device=dev)
    ae_cor = torch.empty(n, dtype=torch.uint8, device=dev)
    ae_first = torch.empty(R, dtype=torch.int32, device=dev)

    def ae_step(i):
        eng.append_entries_verify_dev(req_off, prev, d["term"], d["etype"], dlen, d_exp,
                                      d["payload"], ae_out, ae_cor, ae_first)
    ms, _ = ctx.timed(ae_step, max(10, args.steps), 2)
    ok = None
    if ctx.oracle_checks:
        ok = bool(np.array_equal(host_np(ae_out).view(np.uint64), expected)) and \
            bool((host_np(ae_first) == 0).all())  # entry 0 of each request is flipped
    pay = n * c5["entry_bytes"]
    # payload + per entry term 8, type 1, data_len 8, stored checksum 8, checksum out 8, corrupt
    # 1 + per request req_off 4, prevLogIndex 8, first corrupt 4 (scratch offsets / indices not
    # counted)
    alg = pay + 34 * n + 16 * R + 4
    return {"workload": f"{R} AppendEntries requests x 1024 EntryMeta x 16 KiB (C5 payload)",
            "GBps_payload": pay / (ms * 1e-3) / 1e9, "ms_per_batch": ms,
            "bit_exact_vs_oracle": ok,
            "roofline": roofline(alg, ms, kernel="AppendEntries verify (scan + segment-walk CRC "
                                                 "+ finish + first-corrupt)",
                                 **pmc_traffic("ae", "ae_block_sums", "ae_scan_sums", "ae_meta",
                                               "crc64_rounds_kernel<512u, false>",
                                               "crc64_finish_kernel<true>", "ae_first_corrupt"))}


def leg_v2(ctx, args, c5state):
    import torch

    from jraft_amd import Engine
    from jraft_amd import workloads as W
    eng, dev = ctx.eng, ctx.dev
    d, eb, expected, flip, out = c5state
    n = len(eb["offsets"]) - 1
    ck = expected ^ flip.astype(np.uint64)
    rec_np, lens = W.v2_records(eb["etype"], eb["index"], eb["term"], eb["payload"],
                                eb["offsets"], ck)
    d_rec = to_dev(rec_np, dev)
    d_roff = to_dev(lens, dev)
    v2_out = {k: torch.empty(n, dtype={np.uint8: torch.uint8, np.uint32: torch.int32}.get(t, torch.int64),
                             device=dev) for k, t in Engine.V2_FIELDS}

    def v2_step(i):
        eng.v2_decode_verify_dev(d_rec, d_roff, v2_out)
    ms, _ = ctx.timed(v2_step, max(10, args.steps), 2)
    cor = host_np(v2_out["corrupt"]).astype(bool)
    ok = None  # the stored checksums are the oracle's: nothing to compare without it
    if ctx.oracle_checks:
        ok = bool((host_np(v2_out["status"]) == 0).all()) and bool(np.array_equal(cor, flip))
        ok = ok and bool(np.array_equal(host_np(v2_out["computed"]).view(np.uint64), expected))
    sample_ok = None
    if ctx.oracle_checks:  # the oracle decoder on the first 512 records
        import jraft_oracle as O
        m = 512
        so = O.v2_decode_batch(rec_np[:int(lens[m])], lens[:m + 1])
        sample_ok = bool(np.array_equal(so["computed"], host_np(v2_out["computed"])[:m].view(np.uint64)))
    tot = int(lens[-1])
    alg = tot + 8 * (n + 1) + 56 * n
    return {"workload": f"{n} stored V2 records (C5 entries, 16 KiB data + header + checksum "
                        f"field), decode + isCorrupted",
            "GBps_records": tot / (ms * 1e-3) / 1e9, "ms_per_batch": ms,
            "bit_exact_vs_oracle": ok, "oracle_decoder_sample_ok": sample_ok,
            "roofline": roofline(alg, ms, kernel="v2_parse + crc64_fixed_kernel<true, true, 512> (+ the "
                                                 "segment walk's two launches, which return at once)",
                                 **pmc_traffic("v2", "v2_parse", "crc64_fixed_kernel<true, true, 512>",
                                               "crc64_rounds_kernel<768u, true>", "v2_finish"))}


def leg_snapshot(ctx, args, c5state):
    """RheaKV snapshot archive CRC64 (java.util.zip.Checksum, AbstractKVStoreSnapshotFile.java:
    121,139): (a) one archive = the whole C5 payload as a single stream chunk; (b) every
    region's 16 KiB chunk folded into its own register."""
    import torch
    eng, dev = ctx.eng, ctx.dev
    d, eb, expected, flip, out = c5state
    n = len(eb["offsets"]) - 1
    pay_u8 = d["payload"]
    tot_b = int(pay_u8.numel())
    one_off = torch.tensor([0, tot_b], dtype=torch.int64, device=dev)
    reg1 = torch.zeros(1, dtype=torch.int64, device=dev)
    regS = torch.zeros(n, dtype=torch.int64, device=dev)
    s1_ms, _ = ctx.timed(lambda i: eng.crc64_stream_update_dev(reg1, pay_u8, one_off),
                         max(10, args.steps), 2)
    sS_ms, _ = ctx.timed(lambda i: eng.crc64_stream_update_dev(regS, pay_u8, d["offsets"]),
                         max(10, args.steps), 2)
    ok = None
    if ctx.oracle_checks:
        # chained pieces == one chunk (the combine law), and the oracle on a 16 MiB prefix
        import jraft_oracle as O
        reg1.zero_()
        eng.crc64_stream_update_dev(reg1, pay_u8, one_off)
        whole = int(host_np(reg1).view(np.uint64)[0])
        reg1.zero_()
        for a in range(0, tot_b, 64 << 20):
            eng.crc64_stream_update_dev(
                reg1, pay_u8, torch.tensor([a, min(tot_b, a + (64 << 20))], dtype=torch.int64,
                                           device=dev))
        chained = int(host_np(reg1).view(np.uint64)[0])
        pre = 16 << 20
        reg1.zero_()
        eng.crc64_stream_update_dev(reg1, pay_u8, torch.tensor([0, pre], dtype=torch.int64, device=dev))
        got_pre = int(host_np(reg1).view(np.uint64)[0])
        ok = whole == chained and got_pre == O.crc64(eb["payload"][:pre].tobytes())
    return {"workload": f"C5 payload ({tot_b >> 20} MiB) as (a) one snapshot archive stream, "
                        f"(b) {n} region streams x 16 KiB chunks (CRC64.update on resident registers)",
            "archive_GBps": tot_b / (s1_ms * 1e-3) / 1e9, "archive_ms": s1_ms,
            "regions_GBps": tot_b / (sS_ms * 1e-3) / 1e9, "regions_ms": sS_ms,
            "bit_exact_vs_oracle": ok,
            "roofline": roofline(tot_b + 24, s1_ms, kernel="archive leg (one 1 GiB chunk)",
                                 **pmc_traffic("snapshot", "crc64_rounds_kernel<512u, false>",
                                               "crc64_finish_kernel<false>"))}


def leg_c1(ctx, args):
    """C1 (configs[0], the reference's CPU case) on the GPU: 1 group x 3 peers, 1M appended
    256-B DATA entries -- one step = LogEntry.checksum of every entry (stamped on append,
    LogManagerImpl.java:313-318) + the group's commit over its 1M pending ballots."""
    import torch

    from jraft_amd import workloads as W
    eng, dev = ctx.eng, ctx.dev
    c1 = W.CONFIGS["C1"]
    n1 = c1["pending"]
    e1 = W.entry_batch(n1, c1["entry_bytes"], seed=W.SEED_BASE ^ 1)
    d1 = {k: to_dev(v, dev) for k, v in e1.items() if isinstance(v, np.ndarray)}
    out1 = torch.empty(n1, dtype=torch.int64, device=dev)
    q1 = W.quorum_batch("C1")
    q1d = {k: to_dev(v, dev) for k, v in q1.items()}
    c1c = torch.empty(1, dtype=torch.int64, device=dev)
    c1s = torch.empty(1, dtype=torch.uint8, device=dev)

    def crc(i):  # 256-B entries back to back: the fixed-size entry point (no offsets array)
        eng.logentry_checksum_fixed_dev(d1["etype"], d1["index"], d1["term"], None,
                                        d1["payload"], c1["entry_bytes"], out1)

    def step(i):
        crc(i)
        eng.quorum_epoch_dev(q1d["match"], q1d["pending_index"], q1d["last_appended"],
                             q1d["last_committed"], q1d["conf"], c1c, c1s)

    def crc_offsets(i):  # the same entries through the general offsets entry point
        eng.logentry_checksum_batch_dev(d1["etype"], d1["index"], d1["term"], None,
                                        d1["payload"], d1["offsets"], out1)
    off_ms, _ = ctx.timed(crc_offsets, max(10, args.steps), 2)
    ok_off = None
    exp1 = None
    if ctx.oracle_checks:
        import jraft_oracle as O
        exp1 = O.logentry_checksum_batch(e1["etype"], e1["index"], e1["term"], None,
                                         e1["payload"], e1["offsets"])
        ok_off = bool(np.array_equal(host_np(out1).view(np.uint64), exp1))
    crc_ms, _ = ctx.timed(crc, max(10, args.steps), 2)
    ms, _ = ctx.timed(step, max(10, args.steps), 2)
    ok = None
    if ctx.oracle_checks:
        ce, se, _ = O.quorum_epoch_replay(q1["match"], q1["pending_index"], q1["last_appended"],
                                          q1["last_committed"], q1["conf"], chunk=1024)
        ok = bool(np.array_equal(host_np(out1).view(np.uint64), exp1)) and \
            bool(np.array_equal(host_np(c1c), ce))
    alg = crc_bytes(n1, n1 * c1["entry_bytes"], verify=False, offsets=False)
    return {"workload": "C1: 1 group x 3 peers, 1M appended 256-B LogEntries: checksum + commitAt",
            "ms_per_step": ms, "entries_per_s": n1 / (ms * 1e-3),
            "GBps_payload": n1 * c1["entry_bytes"] / (ms * 1e-3) / 1e9,
            "bit_exact_vs_oracle": ok,
            "offsets_path": {"ms_per_launch": off_ms, "bit_exact_vs_oracle": ok_off,
                             "how": "jrq_logentry_checksum_batch_dev (segment walk + finish kernel)",
                             "frac": crc_bytes(n1, n1 * c1["entry_bytes"], verify=False) /
                             (off_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS},
            "roofline": roofline(alg, crc_ms, kernel="crc64_fixed_kernel<true, false, 1024> (1M x 256 B LogEntries, "
                                                    "jrq_logentry_checksum_fixed_dev)",
                                 **pmc_traffic("C1", "crc64_fixed_kernel<true, false, 1024>"))}


def leg_lease(ctx, args, quorum_conf_dev, G, P):
    import torch
    eng, dev, rank = ctx.eng, ctx.dev, ctx.rank
    rng = np.random.default_rng(rank)
    now_ms, lease_to = 1 << 40, 900
    # rotating timestamp buffers: no launch re-reads the previous launch's inputs from MALL / L2
    ts_bufs = [to_dev((now_ms - rng.integers(0, 2 * lease_to, (P, G))).astype(np.int64), dev)
               for _ in range(QUORUM_EPOCH_BUFFERS)]
    self_slot = torch.zeros(G, dtype=torch.uint8, device=dev)
    lead = torch.zeros(G, dtype=torch.int64, device=dev)
    lok = torch.empty(G, dtype=torch.uint8, device=dev)
    ldead = torch.empty(G, dtype=torch.int16, device=dev)

    # prepared launches (arguments resolved once, as a JNI host keeps its buffers): a Python
    # call per launch costs about as much as the 13-us kernel and would starve the GPU
    launchers = [eng.leader_tick_launcher(ts, quorum_conf_dev, self_slot, now_ms, lease_to, lok,
                                          lead, ldead, None, None, None) for ts in ts_bufs]

    def step(i):
        launchers[i % QUORUM_EPOCH_BUFFERS]()
    ms, _ = ctx.timed(step)
    ok = None
    if ctx.oracle_checks:  # one launch on buffer 0 from fresh lease starts, every group
        import jraft_oracle as O
        lead.zero_()
        step(0)
        ctx.sync()
        eok, elead, edead = O.lease_check(host_np(ts_bufs[0]), host_np(quorum_conf_dev).view(np.uint64),
                                          np.zeros(G, np.uint8), now_ms, lease_to, np.zeros(G, np.int64))
        ok = bool(np.array_equal(host_np(lok), eok)) and \
            bool(np.array_equal(host_np(lead), elead)) and \
            bool(np.array_equal(host_np(ldead).view(np.uint16), edead))
    lb = (8 * P + 28) * G
    return {"workload": f"{G} leader groups x {P} peers (conf + old conf), checkDeadNodes0",
            "decisions_per_s": G / (ms * 1e-3), "kernel_ms": ms, "bit_exact_vs_oracle": ok,
            "roofline": roofline(lb, ms, kernel=f"leader_tick_pair_kernel<{P}, false>",
                                 **pmc_traffic("lease", f"leader_tick_pair_kernel<{P}, false>"))}


def leg_readindex(ctx, args, quorum_conf_dev, quorum_conf, G, P):
    """The ReadIndex heartbeat quorum (NodeImpl.java:1246-1396) over G leader
    groups, one heartbeat round each: conf C3's, the leader in slot 0, a random subset of the
    four followers answered in a random order, 55 % of the answers successful."""
    import torch
    eng, dev, rank = ctx.eng, ctx.dev, ctx.rank
    rng = np.random.default_rng(rank ^ 0x4EAD)
    self_np = np.zeros(G, np.uint8)
    bufs = []
    for _ in range(QUORUM_EPOCH_BUFFERS):  # rotating inputs, as the other legs
        pos = np.argsort(rng.random((G, P - 1)), axis=1).astype(np.uint64) + np.uint64(1)
        pos[rng.random((G, P - 1)) < 0.3] = 0  # not answered yet
        order = (pos << (4 * np.arange(1, P, dtype=np.uint64))).sum(axis=1).astype(np.uint64)
        okm = ((rng.random((G, P - 1)) < 0.55) << np.arange(1, P)).sum(axis=1).astype(np.uint16)
        bufs.append((order, okm, to_dev(order, dev), to_dev(okm.view(np.int16), dev)))
    self_slot = to_dev(self_np, dev)
    res = torch.empty(G, dtype=torch.uint8, device=dev)

    launchers = [eng.readindex_launcher(quorum_conf_dev, self_slot, b[2], b[3], P, res) for b in bufs]

    def step(i):
        launchers[i % QUORUM_EPOCH_BUFFERS]()
    ms, _ = ctx.timed(step)
    ok = None
    counts = None
    if ctx.oracle_checks:
        import jraft_oracle as O
        step(0)
        ctx.sync()
        exp = O.readindex_quorum(quorum_conf, self_np, bufs[0][0], bufs[0][1], P)
        got = host_np(res)
        ok = bool(np.array_equal(got, exp))
        counts = {k: int((exp == v).sum()) for k, v in (("pending", 0), ("success", 1), ("failure", 2))}
    rb = 20 * G  # conf 8 + order 8 + ok mask 2 + self slot 1 read, verdict 1 written
    return {"workload": f"{G} leader groups x {P} peers, one ReadIndex heartbeat round each",
            "rounds_per_s": G / (ms * 1e-3), "kernel_ms": ms, "bit_exact_vs_oracle": ok,
            "verdicts": counts,
            "roofline": roofline(rb, ms, **pmc_traffic("readindex", f"readindex_quorum_kernel<{P}, true>"))}


def leg_tick(ctx, args, quorum_conf_dev, quorum_conf, G, P):
    """The leader tick (jrq_leader_tick_dev): the lease check and the ReadIndex round of the
    same G leader groups in one launch (the lease leg's timestamps and the ReadIndex leg's
    responses, generated the same way), checked against both oracles on every group."""
    import torch
    eng, dev, rank = ctx.eng, ctx.dev, ctx.rank
    rng = np.random.default_rng(rank ^ 0x71C4)
    now_ms, lease_to = 1 << 40, 900
    self_np = np.zeros(G, np.uint8)
    bufs = []
    for _ in range(QUORUM_EPOCH_BUFFERS):  # rotating inputs: no launch re-reads the last one's
        ts = (now_ms - rng.integers(0, 2 * lease_to, (P, G))).astype(np.int64)
        pos = np.argsort(rng.random((G, P - 1)), axis=1).astype(np.uint64) + np.uint64(1)
        pos[rng.random((G, P - 1)) < 0.3] = 0
        order = (pos << (4 * np.arange(1, P, dtype=np.uint64))).sum(axis=1).astype(np.uint64)
        okm = ((rng.random((G, P - 1)) < 0.55) << np.arange(1, P)).sum(axis=1).astype(np.uint16)
        bufs.append({"ts": ts, "order": order, "okm": okm, "d_ts": to_dev(ts, dev),
                     "d_order": to_dev(order, dev), "d_okm": to_dev(okm.view(np.int16), dev)})
    self_slot = to_dev(self_np, dev)
    lead = torch.zeros(G, dtype=torch.int64, device=dev)
    lok = torch.empty(G, dtype=torch.uint8, device=dev)
    ldead = torch.empty(G, dtype=torch.int16, device=dev)
    ri = torch.empty(G, dtype=torch.uint8, device=dev)
    launchers = [eng.leader_tick_launcher(b["d_ts"], quorum_conf_dev, self_slot, now_ms, lease_to,
                                          lok, lead, ldead, b["d_order"], b["d_okm"], ri)
                 for b in bufs]
    ms, _ = ctx.timed(lambda i: launchers[i % QUORUM_EPOCH_BUFFERS]())
    ok = None
    if ctx.oracle_checks:  # one launch on buffer 0 from fresh lease starts, every group
        import jraft_oracle as O
        lead.zero_()
        launchers[0]()
        ctx.sync()
        b = bufs[0]
        eok, elead, edead = O.lease_check(b["ts"], quorum_conf, self_np, now_ms, lease_to,
                                          np.zeros(G, np.int64))
        eri = O.readindex_quorum(quorum_conf, self_np, b["order"], b["okm"], P)
        ok = bool(np.array_equal(host_np(lok), eok)) and \
            bool(np.array_equal(host_np(lead), elead)) and \
            bool(np.array_equal(host_np(ldead).view(np.uint16), edead)) and \
            bool(np.array_equal(host_np(ri), eri))
    # per group: timestamps 8P + conf 8 + self 1 + lease start 8 read, 8 written + ok 1 + dead 2
    # (the lease check, 8P + 28) + order 8 + ok mask 2 read, verdict 1 written (ReadIndex, 11)
    tb = (8 * P + 39) * G
    return {"workload": f"{G} leader groups x {P} peers: lease check + one ReadIndex heartbeat "
                        f"round each, one launch (jrq_leader_tick_dev)",
            "groups_per_s": G / (ms * 1e-3), "kernel_ms": ms, "bit_exact_vs_oracle": ok,
            "roofline": roofline(tb, ms, kernel=f"leader_tick_pair_kernel<{P}, true>",
                                 bytes_note="8P+39 B per group",
                                 **pmc_traffic("tick", f"leader_tick_pair_kernel<{P}, true>"))}


def leg_fanout(ctx, args, G):
    """commit fan-out (FSMCaller.doCommitted / ClosureQueue.popClosureUntil) of C3 epochs: each
    epoch's committed[] feeds the fan-out of its groups; every launch starts from fresh closure
    queues (restored outside the timed event pair)."""
    import torch

    from jraft_amd import workloads as W
    eng, dev = ctx.eng, ctx.dev
    fan_sets = []
    status = torch.empty(G, dtype=torch.uint8, device=dev)
    for e in range(QUORUM_EPOCH_BUFFERS):
        b = W.quorum_batch("C3", groups=G, seed=(W.SEED_BASE ^ 3) + 7919 * e)
        t = {k: to_dev(v, dev) for k, v in b.items()}
        c = torch.empty(G, dtype=torch.int64, device=dev)
        eng.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                             t["last_committed"], t["conf"], c, status)
        cq_size0 = t["last_appended"] - t["pending_index"] + 1
        # lastApplied: its own array (FSMCaller's), equal to lastCommitted before the epoch
        fan_sets.append({"prev": t["last_committed"], "c": c, "la": t["last_committed"].clone(),
                         "cf0": t["pending_index"], "cs0": cq_size0,
                         "cf": torch.empty_like(c), "cs": torch.empty_like(c)})
    fan_fc = torch.empty(G, dtype=torch.int64, device=dev)
    fan_st = torch.empty(G, dtype=torch.uint8, device=dev)
    fan_list = torch.empty((G + 63) // 64, dtype=torch.int64, device=dev)
    fan_num = torch.zeros(1, dtype=torch.int32, device=dev)

    def restore():
        for f in fan_sets:
            f["cf"].copy_(f["cf0"])
            f["cs"].copy_(f["cs0"])

    def launch(f):
        eng.commit_fanout_dev(f["prev"], f["c"], f["la"], f["cf"], f["cs"], fan_fc, fan_st,
                              fan_list, fan_num)
    restore()
    launch(fan_sets[0])
    ctx.sync()
    n_listed = int(fan_num.item())
    n_pop = int((fan_sets[0]["cf"] != fan_sets[0]["cf0"]).sum().item())
    fan_ms = []
    warm = max(1, args.warmup) + 50  # (~WARM_MS of work, as warm_until gives the other legs)
    for rep in range(warm + max(1, args.steps // 4)):
        restore()
        ctx.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        mark(ctx.stream)
        e0.record(ctx.stream)
        for f in fan_sets:
            launch(f)
        e1.record(ctx.stream)
        mark(ctx.stream, end=True)
        ctx.sync()
        if rep >= warm:
            fan_ms.append(e0.elapsed_time(e1) / len(fan_sets))
    ms = float(np.mean(fan_ms))
    ok = None
    if ctx.oracle_checks:  # set 0 from fresh queues, every group, call-by-call replay
        import jraft_oracle as O
        restore()
        launch(fan_sets[0])
        ctx.sync()
        f = fan_sets[0]
        prev_c, c = host_np(f["prev"]), host_np(f["c"])
        adv = c > prev_c
        seq_off = np.zeros(G + 1, np.uint64)
        seq_off[1:] = np.cumsum(adv)
        est, efc, _, ecf, ecs, _ = O.commit_fanout_replay(seq_off, c[adv], host_np(f["la"]),
                                                          host_np(f["cf0"]), host_np(f["cs0"]))
        ok = bool(np.array_equal(host_np(fan_st), est)) and \
            bool(np.array_equal(host_np(fan_fc), efc)) and \
            bool(np.array_equal(host_np(f["cf"]), ecf)) and bool(np.array_equal(host_np(f["cs"]), ecs))
    # reads prev/committed/lastApplied/cqFirst/cqSize 40 B, writes firstClosure 8 + status 1
    # + the listed bitmap 1/8; + 16 B queue write-back per popping group
    fb = 49 * G + G // 8 + 16 * n_pop
    return {"workload": f"{G} groups (C3 epoch output) -> doCommitted/popClosureUntil, "
                        f"{n_listed} listed, {n_pop} popping",
            "groups_per_s": G / (ms * 1e-3), "ms_per_launch": ms, "bit_exact_vs_oracle": ok,
            "roofline": roofline(fb, ms, kernel="fanout_pair", **pmc_traffic("fanout", "fanout_pair"))}


def leg_peak(ctx):
    """device-to-device copy of 2 GiB and a 2-read/1-write xor stream: the "peak_measured" of
    SURVEY.md §8d (frac stays against the 8 TB/s spec)."""
    import torch
    src = torch.empty(1 << 31, dtype=torch.uint8, device=ctx.dev)
    dst = torch.empty_like(src)
    cp_ms, _ = ctx.timed(lambda i: dst.copy_(src), 5, 2)
    words = src.view(torch.int64)
    h = words.numel() // 2
    rd_ms, _ = ctx.timed(lambda i: torch.bitwise_xor(words[:h], words[h:],
                                                     out=dst.view(torch.int64)[:h]), 5, 2)
    acc = torch.empty((), dtype=torch.int64, device=ctx.dev)
    sm_ms, _ = ctx.timed(lambda i: torch.sum(words, dim=0, out=acc), 5, 2)
    return {"copy_GBps": 2 * src.numel() / (cp_ms * 1e-3) / 1e9,
            "xor_GBps": 1.5 * src.numel() / (rd_ms * 1e-3) / 1e9,
            "read_GBps": src.numel() / (sm_ms * 1e-3) / 1e9,
            "how": "torch kernels on 2 GiB: D2D copy (read + write bytes), a 2-input xor into "
                   "half-size output (2 reads + 1 write) and a read-only int64 sum / time; "
                   "torch's generic kernels, so lower bounds on the ceiling -- this run's own "
                   "streaming kernels (the headline, the C5 verify) may exceed them"}


# ------------------------------------------------------------------ the printed line --

# The driver parses the one stdout line from a bounded tail of the run's output (round 3's
# 20.8 KB line was not parsed; round 2's 13.2 KB one was).  The printed line keeps the contract
# keys plus one small summary per leg; everything else goes to the detail file it names.
LINE_BUDGET = 6000
DETAIL_FILE = "bench_detail.json"


def _r(x, nd=4):
    """Round a float to `nd` significant digits (None passes through)."""
    if x is None or isinstance(x, bool) or not isinstance(x, (int, float)):
        return x
    if x == 0 or isinstance(x, int):
        return x
    return float(f"{x:.{nd}g}")


def _roof_summary(rl: dict | None) -> dict | None:
    """The contract's roofline object (+ kernel name, per-launch ms and bytes)."""
    if not rl:
        return None
    out = {k: _r(rl.get(k)) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic")}
    out["kernel"] = rl.get("kernel")
    out["kernel_ms"] = _r(rl.get("kernel_ms"), 5)
    out["bytes_per_launch"] = rl.get("bytes_per_launch")
    if rl.get("traffic") and rl.get("bytes_per_launch"):
        out["traffic_ratio"] = _r(rl["traffic"] / rl["bytes_per_launch"], 3)
    if rl.get("frac_survey_bytes") is not None:
        out["frac_survey_bytes"] = _r(rl["frac_survey_bytes"])
    pm = rl.get("peak_measured")
    if pm:
        out["peak_measured"] = {k: _r(v) for k, v in pm.items() if k != "how"}
    return out


def _cpu_summary(cb: dict | None) -> dict | None:
    if not cb:
        return None
    out = {k: _r(cb.get(k)) for k in ("value", "unit", "cores", "kind")}
    pt = cb.get("per_threads") or {}
    out["per_threads"] = {k: _r(v["value"] if isinstance(v, dict) else v, 3) for k, v in pt.items()}
    opt = (cb.get("optimised") or {}).get("per_threads")
    if opt:
        out["optimised_per_threads"] = {k: _r(v, 3) for k, v in opt.items()}
    out["sample"] = cb.get("sample")
    host = cb.get("host")
    if host:
        out["host"] = f"{host.get('model')}, cgroup quota {host.get('cgroup_cpu_quota')} CPUs"
    return out


def _bit_exact(d: dict):
    """The leg's oracle verdict: every `bit_exact*` / `*_ok` flag it carries AND-ed (None when the
    oracle did not run)."""
    flags = [v for k, v in d.items() if (k.startswith("bit_exact") or k.endswith("_ok"))
             and isinstance(v, bool)]
    return all(flags) if flags else None


def _leg_summary(d: dict, ms_key: str) -> dict:
    rl = d.get("roofline") or {}
    s = {"ms": _r(d.get(ms_key, rl.get("kernel_ms")), 5), "frac": _r(rl.get("frac"), 3)}
    if rl.get("traffic") and rl.get("bytes_per_launch"):
        s["traffic_ratio"] = _r(rl["traffic"] / rl["bytes_per_launch"], 3)
    s["bit_exact"] = _bit_exact(d)
    return s


def compact_line(full: dict, detail_path: str | None = DETAIL_FILE) -> dict:
    """The printed line: the contract keys, the headline's roofline / cpu_baseline / multi_gpu,
    the second BASELINE metric (`crc64`) and one {ms, frac, traffic_ratio, bit_exact} per leg.
    `full` is the whole result (written to `detail_path`)."""
    keys = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config")
    line = {k: _r(full.get(k), 6) if k in ("value", "ms_per_step") else full.get(k) for k in keys}
    line["warm_ms"] = full.get("warm_ms")
    line["csrc_sha"] = full.get("csrc_sha")
    line["lib_sha"] = full.get("lib_sha")  # jrq_build_id() of the library that ran
    line["roofline"] = _roof_summary(full.get("roofline"))
    line["cpu_baseline"] = _cpu_summary(full.get("cpu_baseline"))
    mg = full.get("multi_gpu")
    if mg:
        line["multi_gpu"] = {k: _r(v) for k, v in mg.items()}
    if "bit_exact_vs_oracle_4096_groups" in full:
        line["bit_exact_vs_oracle_4096_groups"] = full["bit_exact_vs_oracle_4096_groups"]
    crc = full.get("crc64")
    if crc:
        c = {k: _r(crc.get(k)) for k in ("metric", "value", "unit")}
        c["ms_per_launch"] = _r(crc.get("ms_per_launch"), 5)
        c["frac"] = _r((crc.get("roofline") or {}).get("frac"), 3)
        c["bit_exact"] = _bit_exact(crc)
        if crc.get("per_rank_GBps"):
            c["per_rank_GBps"] = [_r(v) for v in crc["per_rank_GBps"]]
            c["per_rank_bit_exact"] = crc.get("per_rank_bit_exact")
        cb = crc.get("cpu_baseline")
        if cb:
            c["cpu_baseline"] = {k: _r(cb.get(k)) for k in ("value", "unit", "cores", "kind")}
        line["crc64"] = c
    legs = {}
    if full.get("roofline"):
        legs["quorum_C3"] = {"ms": _r(full["roofline"].get("kernel_ms"), 5),
                             "frac": _r(full["roofline"].get("frac"), 3),
                             "traffic_ratio": (_roof_summary(full["roofline"]) or {}).get("traffic_ratio"),
                             "bit_exact": full.get("bit_exact_vs_oracle_4096_groups")}
    qr = full.get("quorum_rows")
    if qr:  # the same epochs from rows (jrq_quorum_epoch_dev)
        legs["quorum_C3_rows"] = {"ms": _r(qr.get("kernel_ms"), 5), "frac": _r(qr.get("frac"), 3),
                                  "traffic_ratio": (_roof_summary(qr) or {}).get("traffic_ratio")}
    t = full.get("resident_table")
    if t:
        legs["table"] = _leg_summary(t, "kernel_ms")
        legs["table"]["over_no_conf"] = _r(t.get("flagged_over_no_conf_change"), 3)
        legs["table"]["over_pair"] = _r(t.get("table_over_pair"), 3)
        legs["table"]["no_conf_over_pair"] = _r(t.get("no_conf_table_over_pair"), 3)
        legs["table"]["no_conf_ms"] = _r(t.get("kernel_ms_no_conf_change"), 5)
        fz = t.get("fused_fanout")
        if fz:  # the epoch with the commit fan-out fused in, and the two-launch path it replaces
            legs["table_fanout"] = {"ms": _r(fz.get("kernel_ms"), 5),
                                    "frac": _r(fz["roofline"].get("frac"), 3),
                                    "epoch_then_fanout_ms": _r(fz.get("epoch_then_fanout_ms"), 5),
                                    "bit_exact": fz.get("bit_exact_vs_epoch_then_fanout")}
    c2 = full.get("C2") or {}
    if "kernel_ms" in c2:
        legs["C2_one_epoch"] = {"ms": _r(c2["kernel_ms"], 5), "bit_exact": None}
    if c2.get("batched_epochs"):
        legs["C2_epochs"] = _leg_summary(c2["batched_epochs"], "kernel_ms")
        legs["C2_epochs"]["epochs"] = c2["batched_epochs"].get("epochs_per_launch")
    if c2.get("batched_epochs_64"):
        legs["C2_epochs_64"] = _leg_summary(c2["batched_epochs_64"], "kernel_ms")
    if full.get("C3_k_epochs"):
        legs["C3_k_epochs"] = _leg_summary(full["C3_k_epochs"], "kernel_ms")
    if crc:
        legs["C5_verify"] = _leg_summary(crc, "ms_per_launch")
        if crc.get("offsets_path"):
            legs["C5_verify_offsets"] = {"ms": _r(crc["offsets_path"].get("ms_per_launch"), 5),
                                         "bit_exact": crc["offsets_path"].get("bit_exact_vs_oracle")}
    if full.get("C5"):
        legs["C5_step"] = _leg_summary(full["C5"], "ms_per_step")
    if full.get("C1"):
        legs["C1"] = _leg_summary(full["C1"], "ms_per_step")
        legs["C1"]["crc_ms"] = _r((full["C1"].get("roofline") or {}).get("kernel_ms"), 5)
    for name, d in (full.get("next_rows") or {}).items():
        ms_key = next((k for k in ("ms_per_batch", "archive_ms", "ms_per_launch", "kernel_ms") if k in d),
                      None)
        legs[name] = _leg_summary(d, ms_key)
    drv = full.get("end_to_end_host_mirror")
    if drv:
        for k, v in drv.items():
            if k.startswith("active_") and isinstance(v, dict):
                legs["drive_" + k] = {"ms": _r(v.get("end_to_end_ms_per_epoch"), 4),
                                      "flush_ms": _r(v.get("flush_ms"), 4),
                                      "decisions_per_s": _r(v.get("decisions_per_s_end_to_end"), 3),
                                      "bit_exact": v.get("bit_exact_vs_stateless_kernel")}
    pin = full.get("pinned_host_payload")
    if pin:
        for k in ("C5", "C1"):
            if k in pin:
                legs["pinned_" + k] = {
                    "GBps_pcie": _r(pin[k]["registered"]["GBps_payload_pcie_inclusive"], 3),
                    "bit_exact": pin[k]["registered"].get("bit_exact_vs_oracle")}
    line["legs"] = legs
    line["detail"] = detail_path
    return line


def emit_line(full: dict, path: str) -> str:
    """Write the whole result to the detail file `path` and return the compact line (checked
    against the budget: the per-leg summary is dropped first, never the contract keys)."""
    try:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as fh:
            json.dump(full, fh, indent=1)
    except OSError as e:  # a read-only tree: the line still prints
        print(f"warning: cannot write {path}: {e}", file=sys.stderr)
    line = compact_line(full, os.path.relpath(path, ROOT))
    s = json.dumps(line, separators=(",", ":"))
    if len(s) > LINE_BUDGET:
        line.pop("legs", None)
        s = json.dumps(line, separators=(",", ":"))
    return s


# ------------------------------------------------------------------ main --

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--groups-per-gpu", type=int, default=1 << 20)
    ap.add_argument("--publish-every", type=int, default=1,
                    help="N>1: all-gather the committed snapshot every K epochs")
    ap.add_argument("--cpu-budget", type=float, default=4.0,
                    help="seconds per CPU baseline leg and thread count")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--detail", default=os.path.join(ROOT, DETAIL_FILE),
                    help="file for the full per-leg result (the printed line is the summary)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 process group: nccl (RCCL, one GPU per rank) or gloo (tests: "
                         "several ranks on one GPU, the snapshot all-gathered through host copies)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on cuda:0 (tests of the N>1 orchestration on a 1-GPU box)")
    ap.add_argument("--legs", default="all",
                    help=f"comma list of {','.join(LEGS)} (the headline quorum leg always runs "
                         "unless the list omits it; PMC passes run one leg each)")
    args = ap.parse_args()
    legs = set(LEGS) if args.legs == "all" else set(args.legs.split(","))
    unknown = legs - set(LEGS)
    if unknown:
        ap.error(f"unknown legs {sorted(unknown)}")

    import torch
    import torch.distributed as dist

    from jraft_amd import Engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.legs == "all":
        # the scaling runs measure both BASELINE metrics: the headline (C4 sharded over the
        # ranks) and C5 (64k regions per GPU: CRC64 verify + commit); the other legs are
        # single-GPU measurements of one rank's work and would only lengthen every N > 1 run
        legs = {"quorum", "C5"}
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if args.one_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 and args.dist_backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    elif world > 1:
        dist.init_process_group("gloo")

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    eng = Engine(local)
    from jraft_amd import _lib
    lib_sha = _lib.check_build_id()  # raises unless libjrq.so was built from these csrc/
    # a dedicated (non-default) stream: the kernels and the HIP events bracketing them
    # must be on the same stream (the default stream's handle is 0 = "engine's own")
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng.use_stream(stream.cuda_stream)
    assert eng.stream() == stream.cuda_stream != 0
    ctx = Ctx(eng, stream, dev, world, rank, args)

    line = {"metric": "quorum commit decisions/sec", "value": None, "unit": "decisions/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "warm_ms": WARM_MS, "ms_per_step": None,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (seeded splitmix64, SURVEY.md §8d)", "legs": sorted(legs),
            "csrc_sha": csrc_sha(), "lib_sha": lib_sha}
    G = args.groups_per_gpu
    from jraft_amd import workloads as W
    if "quorum" in legs:
        _LEG[0] = "quorum"
        q = leg_quorum(ctx, args, barrier, max_over_ranks)
        line.update({
            "value": q["value"], "ms_per_step": q["elapsed"] * 1e3 / args.steps,
            "config": {
                "workload": ("C3: 1M Raft groups x 5 peers, joint consensus (old 3 + new 5), "
                             "1k pending/group" if world == 1 else
                             f"C4: {G * world} Raft groups x 5 peers sharded by groupId, "
                             f"{G} per GPU, + RCCL all-gather of committed[] every "
                             f"{args.publish_every} epoch(s)"),
                "groups_per_gpu": G, "peers": q["P"], "epoch_buffers": QUORUM_EPOCH_BUFFERS,
                "parallelism": f"groupId shards x{world}"},
            "roofline": q["roofline"], "multi_gpu": q["multi_gpu"],
            "quorum_rows": q["rows_entry_point"],
            "bit_exact_vs_oracle_4096_groups": q["bit_exact_vs_oracle_4096_groups"]})
    if "table" in legs:
        pair_ms = line.get("roofline", {}).get("kernel_ms")
        _LEG[0] = "table"
        line["resident_table"] = leg_table(ctx, args, G, pair_ms)
    if "drive" in legs:
        _LEG[0] = "drive"
        line["end_to_end_host_mirror"] = leg_drive(ctx, args, G)
    if "C2" in legs:
        _LEG[0] = "C2"
        line["C2"] = leg_c2(ctx, args)
    if "C2L" in legs:
        _LEG[0] = "C2L"
        line.setdefault("C2", {})["batched_epochs_64"] = leg_c2l(ctx, args)
    if "C3K" in legs:
        _LEG[0] = "C3K"
        line["C3_k_epochs"] = leg_c3k(ctx, args, G)
    extras = {}
    c5state = None
    if legs & {"C5", "ae", "v2", "snapshot", "pinned"}:
        _LEG[0] = "C5"
        crc, c5_step, c5state = leg_c5(ctx, args, barrier, max_over_ranks,
                                       time_it="C5" in legs)
        if "C5" in legs:
            line["crc64"] = crc
            line["C5"] = c5_step
    if "ae" in legs:
        _LEG[0] = "ae"
        extras["append_entries_verify"] = leg_ae(ctx, args, c5state)
    if "v2" in legs:
        _LEG[0] = "v2"
        extras["v2_decode_verify"] = leg_v2(ctx, args, c5state)
    if "snapshot" in legs:
        _LEG[0] = "snapshot"
        extras["snapshot_stream_crc64"] = leg_snapshot(ctx, args, c5state)
    if "pinned" in legs:
        _LEG[0] = "pinned"
        line["pinned_host_payload"] = leg_pinned(ctx, args, c5state)
    c5state = None
    if "C1" in legs:
        _LEG[0] = "C1"
        line["C1"] = leg_c1(ctx, args)
    c3conf = W.quorum_batch("C3", groups=G)["conf"] if legs & {"lease", "readindex", "tick"} else None
    if "lease" in legs:
        _LEG[0] = "lease"
        extras["lease_check"] = leg_lease(ctx, args, to_dev(c3conf, dev), G, 5)
    if "readindex" in legs:
        _LEG[0] = "readindex"
        extras["readindex_quorum"] = leg_readindex(ctx, args, to_dev(c3conf, dev), c3conf, G, 5)
    if "tick" in legs:
        _LEG[0] = "tick"
        extras["leader_tick"] = leg_tick(ctx, args, to_dev(c3conf, dev), c3conf, G, 5)
    if "fanout" in legs:
        _LEG[0] = "fanout"
        extras["commit_fanout"] = leg_fanout(ctx, args, G)
    if extras:
        line["next_rows"] = extras
    if "peak" in legs and "roofline" in line:
        _LEG[0] = "peak"
        line["roofline"]["peak_measured"] = leg_peak(ctx)
        # the best rate any kernel of this run reached on its algorithmic bytes
        def rates(o):
            if isinstance(o, dict):
                if o.get("unit") == "GB/s" and isinstance(o.get("achieved"), float):
                    yield o["achieved"]
                for v in o.values():
                    yield from rates(v)
        line["roofline"]["peak_measured"]["best_kernel_GBps_this_run"] = max(rates(line), default=None)

    if "cpu" in legs and rank == 0 and world == 1 and not args.no_cpu:
        info = cpu_info()
        line["cpu_baseline"] = cpu_quorum_baseline("C3", info, args.cpu_budget)
        line["cpu_baseline"]["host"] = info
        cpu = {"host": info, "C2": cpu_quorum_baseline("C2", info, args.cpu_budget),
               "C1": cpu_c1_baseline(info), "C5_crc": cpu_crc_baseline(info, args.cpu_budget)}
        line["cpu_baselines"] = cpu
        if "crc64" in line:
            line["crc64"]["cpu_baseline"] = cpu["C5_crc"]
    line["timed_series_legs"] = list(_SERIES)
    if rank == 0:
        s = emit_line(line, os.path.abspath(args.detail))
        sys.stderr.flush()
        print(s, flush=True)
    eng.use_stream(None)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
