#!/usr/bin/env python3
"""bench.py -- quorum commit decisions/s (+ LogEntry CRC64 GB/s) on 1..8 MI355X.

Driver contract: `python bench.py --gpus N --steps K --warmup W`; N>1 is launched by
torch.distributed.run (one rank per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from env).
Rank 0 prints ONE JSON line.

Headline (`value`): quorum commit decisions/s, whole job.  Workload per GPU = 1M Raft
groups x 5 peers with joint-consensus masks (BASELINE config C3 at N=1; at N>1 config
C4: 8M groups sharded by contiguous groupId blocks, 1M per GPU, weak scaling).  One
step = one quorum epoch kernel over the GPU's groups; at N>1 the step also publishes
the node-wide committed-index snapshot with an RCCL all-gather over xGMI.  Inputs are
device-resident; the step cycles through several distinct epochs (> the 256 MiB
Infinity Cache) so every launch reads its inputs from HBM.

Also measured in the same run (extra fields): LogEntry CRC64 verify GB/s on C5
(64k x 16 KiB entries per GPU), the C2 config (10k groups x 3 peers), HIP-event
kernel times -> `roofline`, and the oracle (Java-faithful C restatement) timed on
this host -> `cpu_baseline`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
QUORUM_EPOCH_BUFFERS = 6


def quorum_bytes_per_group(P: int) -> int:
    # reads: match 8P, pendingIndex 8, lastAppended 8, lastCommitted 8, conf 8;
    # writes: committed 8, status 1  
    return 8 * P + 41


def crc_bytes(n_entries: int, payload_bytes: int, verify: bool = True) -> int:
    # payload + offsets (N+1)*8 + per entry type 1, index 8, term 8, out 8 (+ expected 8, corrupt 1)
    b = payload_bytes + 8 * (n_entries + 1) + n_entries * (1 + 8 + 8 + 8)
    if verify:
        b += n_entries * (8 + 1)
    return b


def to_dev(arr, dev):
    import torch
    if arr is None:
        return None
    a = arr.view(np.int64) if arr.dtype == np.uint64 else arr
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def pmc_traffic(*kernels: str):
    """HBM bytes per launch of the timed op, summed over `kernels` (name substrings), from
    the newest committed PMC summary holding all of them (profiles/<tag>_pmc.json, written
    by tools/summarize_profiles.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
    passes of this bench); None if absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    for f in reversed(files):
        try:
            with open(f) as fh:
                ks = json.load(fh).get("kernels", {})
        except (OSError, ValueError):
            continue
        total = 0.0
        for kern in kernels:
            hit = [d["hbm_bytes_per_launch_corrected"] for name, d in ks.items()
                   if kern in name and "hbm_bytes_per_launch_corrected" in d]
            if not hit:
                break
            total += hit[0]
        else:
            return {"bytes": total,
                    "source": os.path.relpath(f, ROOT) + " (2*FETCH_SIZE+WRITE_SIZE, KiB->B)"}
    return None


def traffic_fields(*kernels: str) -> dict:
    t = pmc_traffic(*kernels)
    return {"traffic": t["bytes"] if t else None, "traffic_source": t["source"] if t else None}


def timed_launches(fn, steps, warmup, stream, sync):
    """warmup untimed, then `steps` launches each bracketed by HIP events on `stream`.

    Returns (wall_s, per-launch event ms, batched ms): the batched figure is one event pair
    around all `steps` launches, back to back, divided by `steps` -- the per-launch event
    packets themselves stretch a ~20 us kernel by 2-3 us (rocprofv3 kernel durations in
    profiles/ agree with the batched figure)."""
    import torch
    for _ in range(warmup):
        fn()
    sync()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        evs[i][0].record(stream)
        fn(i)
        evs[i][1].record(stream)
    sync()
    wall = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in evs]
    b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b0.record(stream)
    for i in range(steps):
        fn(i)
    b1.record(stream)
    sync()
    batched_ms = b0.elapsed_time(b1) / steps
    return wall, kern_ms, batched_ms


CPU_THREADS = 16  # the GPU box's CPU share per GPU (os.cpu_count() there shows the whole host)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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


def cpu_quorum_baseline(budget_s: float, threads: int = CPU_THREADS):
    """Oracle (Java-faithful BallotBox replay, oracle/jraft_oracle.c) on C3 groups: 1 thread,
    then `threads` threads over disjoint group chunks (one BallotBox per group, as in the
    reference: groups never share a lock)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import jraft_oracle as O
    from jraft_amd import workloads as W
    chunk_groups = 256
    chunks = [W.quorum_batch("C3", groups=chunk_groups, group_offset=k * chunk_groups)
              for k in range(2 * threads)]

    def replay(b):
        return O.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                     b["last_committed"], b["conf"], chunk=1024)[2]
    n1, t1, g1 = _threaded(replay, chunks, 1, budget_s / 2)
    nt, tt, gt = _threaded(replay, chunks, threads, budget_s / 2)
    # optimised CPU line: closed-form epoch per group (oracle/cpu_fast.c),
    # over full 64k-group C3 chunks
    fast_groups = 1 << 16
    fchunks = [W.quorum_batch("C3", groups=fast_groups, group_offset=k * fast_groups)
               for k in range(threads)]

    def fast(b):
        O.fast_quorum_epoch(b["match"], b["pending_index"], b["last_appended"],
                            b["last_committed"], b["conf"])
        return 0
    fn1, ft1, _ = _threaded(fast, fchunks, 1, 1.0)
    fnt, ftt, _ = _threaded(fast, fchunks, threads, 1.0)
    optimised = dict(value=fnt * fast_groups / ftt, single_thread=fn1 * fast_groups / ft1,
                     cores=threads, how="closed-form q-th largest per conf mask per group "
                     "(oracle/cpu_fast.c, same results as the BallotBox replay), C3 groups")
    return dict(value=nt * chunk_groups / tt, unit="decisions/s", cores=threads, kind="port",
                optimised=optimised,
                single_thread=n1 * chunk_groups / t1, cpu=cpu_model(),
                sample=f"C3 groups (1k pending, 5 peers, joint) replayed through the Java-faithful "
                       f"BallotBox restatement: {nt * chunk_groups} groups / {gt} Ballot.grant "
                       f"calls in {tt:.1f} s on {threads} threads; {n1 * chunk_groups} groups in "
                       f"{t1:.1f} s on 1 thread")


def cpu_crc_baseline(budget_s: float, threads: int = CPU_THREADS):
    """Byte-at-a-time CRC64.update restatement over C5 entries: 1 thread, then `threads`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import jraft_oracle as O
    from jraft_amd import workloads as W
    n = 256  # 4 MiB of C5 entries per call
    batches = [W.entry_batch(n, 16 << 10, seed=5 + k) for k in range(threads)]

    def run(b):
        O.logentry_checksum_batch(b["etype"], b["index"], b["term"], None, b["payload"],
                                  b["offsets"])
        return 0
    n1, t1, _ = _threaded(run, batches, 1, budget_s / 2)
    nt, tt, _ = _threaded(run, batches, threads, budget_s / 2)
    gb1, gbt = n1 * n * (16 << 10) / 1e9, nt * n * (16 << 10) / 1e9

    def fast(b):  # optimised CPU line: slice-by-8 CRC64 of the same payloads
        O.fast_crc64_batch(b["payload"], b["offsets"])
        return 0
    fast(batches[0])  # builds the slice tables before the threads start
    fn1, ft1, _ = _threaded(fast, batches, 1, 1.0)
    fnt, ftt, _ = _threaded(fast, batches, threads, 1.0)
    optimised = dict(value=fnt * n * (16 << 10) / 1e9 / ftt,
                     single_thread=fn1 * n * (16 << 10) / 1e9 / ft1, cores=threads,
                     how="slice-by-8 CRC64 (oracle/cpu_fast.c) over the same C5 payloads")
    return dict(value=gbt / tt, unit="GB/s", cores=threads, kind="port", optimised=optimised,
                single_thread=gb1 / t1, cpu=cpu_model(),
                sample=f"C5 LogEntries x 16 KiB through the byte-at-a-time CRC64.update "
                       f"restatement: {gbt:.2f} GB in {tt:.1f} s on {threads} threads; "
                       f"{gb1:.2f} GB in {t1:.1f} s on 1 thread")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--groups-per-gpu", type=int, default=1 << 20)
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds per CPU baseline leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-crc", action="store_true")
    ap.add_argument("--headline-only", action="store_true",
                    help="quorum + C2 + C5 CRC only (the PMC passes use it: per-kernel counters "
                         "are averaged over every dispatch of a kernel name)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from jraft_amd import Engine
    from jraft_amd import workloads as W

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    eng = Engine(local)
    # a dedicated (non-default) stream: the kernels and the HIP events bracketing them
    # must be on the same stream (the default stream's handle is 0 = "engine's own")
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng.use_stream(stream.cuda_stream)
    assert eng.stream() == stream.cuda_stream != 0

    def sync():
        torch.cuda.synchronize(dev)

    # ------------------------------------------------ quorum (headline) -----
    G = args.groups_per_gpu
    cfg = "C3" if world == 1 else "C4"
    P = W.CONFIGS[cfg]["peers"]
    epochs = []
    for e in range(QUORUM_EPOCH_BUFFERS):
        b = W.quorum_batch(cfg, groups=G, group_offset=rank * G,
                           seed=(W.SEED_BASE ^ int(cfg[1])) + 7919 * e)
        epochs.append({k: to_dev(v, dev) for k, v in b.items()})
    committed = torch.empty(G, dtype=torch.int64, device=dev)
    status = torch.empty(G, dtype=torch.uint8, device=dev)
    snapshot = torch.empty(G * world, dtype=torch.int64, device=dev) if world > 1 else None
    if world > 1:
        uid = [Engine.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.rccl_init(world, rank, uid[0])

    state = {"i": 0}

    def quorum_step(i=None):
        t = epochs[state["i"] % QUORUM_EPOCH_BUFFERS]
        state["i"] += 1
        eng.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                             t["last_committed"], t["conf"], committed, status)

    def full_step(i=None):
        quorum_step(i)
        if world > 1:
            eng.publish_committed_dev(committed, snapshot)

    # kernel-only timing (HIP events around each launch)
    _, kern_ms, q_batched_ms = timed_launches(quorum_step, args.steps, args.warmup, stream, sync)
    # the contract's timed region: K steps between barrier+sync on both sides
    for _ in range(args.warmup):
        full_step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        full_step()
    sync()
    barrier()
    sync()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    decisions = G * world * args.steps
    value = decisions / elapsed
    # the tighter of the two HIP-event methods (timed_launches); both agree with rocprofv3
    k_avg_ms = min(q_batched_ms, float(np.mean(kern_ms)))
    q_bytes = quorum_bytes_per_group(P) * G
    achieved = q_bytes / (k_avg_ms * 1e-3) / 1e9

    # ------------------------------------------------ C2 (configs[1]) -------
    c2 = W.quorum_batch("C2")
    c2d = {k: to_dev(v, dev) for k, v in c2.items()}
    G2 = c2["pending_index"].shape[0]
    c2c = torch.empty(G2, dtype=torch.int64, device=dev)
    c2s = torch.empty(G2, dtype=torch.uint8, device=dev)

    def c2_step(i=None):
        eng.quorum_epoch_dev(c2d["match"], c2d["pending_index"], c2d["last_appended"],
                             c2d["last_committed"], c2d["conf"], c2c, c2s)

    c2_wall, c2_ms, c2_b = timed_launches(c2_step, args.steps, args.warmup, stream, sync)
    c2_batched_ms = min(c2_b, float(np.mean(c2_ms)))
    # C2 is launch-bound one epoch at a time: K successive epochs per launch, the group state
    # carried between them on the GPU (jrq_quorum_epochs_dev)
    KE = 64
    ser = W.quorum_epoch_series("C2", KE)
    ser_d = {k: to_dev(v, dev) for k, v in ser.items()}
    kc = torch.empty((KE, G2), dtype=torch.int64, device=dev)
    ks = torch.empty((KE, G2), dtype=torch.uint8, device=dev)

    def c2k_step(i=None):
        eng.quorum_epochs_dev(ser_d["match"], ser_d["pending_index"], ser_d["last_appended"],
                              ser_d["last_committed"], ser_d["conf"], kc, ks)

    _, c2k_ms, c2k_b = timed_launches(c2k_step, args.steps, args.warmup, stream, sync)
    c2k_avg = min(c2k_b, float(np.mean(c2k_ms)))
    c2k_ok = None
    if rank == 0 and not args.no_cpu:  # oracle on the first 64 groups, all KE epochs
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import jraft_oracle as O
        sub = 64
        pi = ser["pending_index"][:sub].copy()
        lc = ser["last_committed"][:sub].copy()
        got = kc.cpu().numpy()
        c2k_ok = True
        for k in range(KE):
            ce, _, _ = O.quorum_epoch_replay(ser["match"][k][:, :sub], pi,
                                             ser["last_appended"][k][:sub], lc,
                                             ser["conf"][:sub], chunk=1024)
            pi = np.where((pi != 0) & (ce > lc), ce + 1, pi)
            lc = ce
            c2k_ok = c2k_ok and bool(np.array_equal(got[k, :sub], ce))

    # end to end from host buffers (the JNI/DirectByteBuffer path): H2D of the epoch's SoA,
    # the kernel, D2H of committed/status -- PCIe-inclusive, never the headline value
    hb = W.quorum_batch(cfg, groups=G, group_offset=rank * G)
    eng.quorum_epoch(hb["match"], hb["pending_index"], hb["last_appended"],
                     hb["last_committed"], hb["conf"])
    t0 = time.perf_counter()
    e2e_reps = 5
    for _ in range(e2e_reps):
        eng.quorum_epoch(hb["match"], hb["pending_index"], hb["last_appended"],
                         hb["last_committed"], hb["conf"])
    e2e_s = (time.perf_counter() - t0) / e2e_reps
    e2e = {"decisions_per_s": G / e2e_s, "ms_per_epoch": e2e_s * 1e3,
           "note": "jrq_quorum_epoch host variant (pageable numpy buffers): H2D + kernel + D2H"}
    del hb

    # ------------------------------------------------ CRC64 (C5) ------------
    crc = None
    if not args.no_crc:
        c5 = W.CONFIGS["C5"]
        n = c5["groups"]
        eb = W.entry_batch(n, c5["entry_bytes"], seed=W.SEED_BASE ^ 5 ^ rank)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        expected = None
        if rank == 0 and not args.no_cpu:
            import jraft_oracle as O
            expected = O.logentry_checksum_batch(eb["etype"], eb["index"], eb["term"], None,
                                                 eb["payload"], eb["offsets"])
        if expected is None:
            expected = np.zeros(n, np.uint64)
        flip = np.zeros(n, bool)
        flip[::1024] = True  # 1/1024 entries corrupted
        expected_c = expected ^ flip.astype(np.uint64)
        d = {k: to_dev(v, dev) for k, v in eb.items() if isinstance(v, np.ndarray)}
        d_exp = to_dev(expected_c, dev)
        out = torch.empty(n, dtype=torch.int64, device=dev)
        corrupt = torch.empty(n, dtype=torch.uint8, device=dev)

        def crc_step(i=None):
            eng.logentry_checksum_batch_dev(d["etype"], d["index"], d["term"], None, d["payload"],
                                            d["offsets"], out, expected=d_exp, corrupt=corrupt)

        _, crc_ms, crc_batched = timed_launches(crc_step, max(10, args.steps), 2, stream, sync)
        barrier()
        crc_avg = min(crc_batched, float(np.mean(crc_ms)))
        crc_ms_max = max_over_ranks(crc_avg)
        pay = n * c5["entry_bytes"]
        ok = None
        if rank == 0 and not args.no_cpu:
            got = out.cpu().numpy().view(np.uint64)
            ok = bool(np.array_equal(got, expected)) and \
                bool(np.array_equal(corrupt.cpu().numpy().astype(bool), flip))
        alg = crc_bytes(n, pay, verify=True)
        crc = {
            "metric": "LogEntry CRC64 verify GB/s",
            "value": pay * world / (crc_ms_max * 1e-3) / 1e9, "unit": "GB/s (payload)",
            "workload": "C5: 64k x 16 KiB DATA LogEntries per GPU, checksum + isCorrupted verify",
            "ms_per_launch": crc_avg,
            "bit_exact_vs_oracle": ok,
            "roofline": {"bound": "hbm", "achieved": alg / (crc_avg * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": alg / (crc_avg * 1e-3) / 1e9 / HBM_PEAK_GBPS, "traffic": None},
        }

    # ------------------------------------------------ §8f legs ---------------
    extras = {}
    if not args.no_crc and not args.headline_only:
        # follower verify on receive: the C5 payload as 64 AppendEntries of 1024 entries
        R = n // 1024
        req_off = torch.arange(0, n + 1, 1024, dtype=torch.int32, device=dev)
        prev = torch.arange(0, n, 1024, dtype=torch.int64, device=dev)  # index = 1..n
        dlen = torch.full((n,), c5["entry_bytes"], dtype=torch.int64, device=dev)
        ae_out = torch.empty(n, dtype=torch.int64, device=dev)
        ae_cor = torch.empty(n, dtype=torch.uint8, device=dev)
        ae_first = torch.empty(R, dtype=torch.int32, device=dev)

        def ae_step(i=None):
            eng.append_entries_verify_dev(req_off, prev, d["term"], d["etype"], dlen, d_exp,
                                          d["payload"], ae_out, ae_cor, ae_first)

        _, ae_ms, ae_b = timed_launches(ae_step, max(10, args.steps), 2, stream, sync)
        ae_avg = min(ae_b, float(np.mean(ae_ms)))
        ae_ok = None
        if rank == 0 and not args.no_cpu:
            ae_ok = bool(np.array_equal(ae_out.cpu().numpy().view(np.uint64), expected)) and \
                bool((ae_first.cpu().numpy() == 0).all())  # entry 0 of each request is flipped
        extras["append_entries_verify"] = {
            "workload": f"{R} AppendEntries requests x 1024 EntryMeta x 16 KiB (C5 payload)",
            "GBps_payload": pay / (ae_avg * 1e-3) / 1e9, "ms_per_batch": ae_avg,
            "bit_exact_vs_oracle": ae_ok}
    if not args.no_crc and not args.headline_only:
        # read path: the C5 entries as stored V2 records (header + PBLogEntry with the
        # checksum field, 1/1024 corrupted), decoded and verified in one batch
        ck = out.cpu().numpy().view(np.uint64) ^ flip.astype(np.uint64)
        rec_np, lens = W.v2_records(eb["etype"], eb["index"], eb["term"], eb["payload"],
                                    eb["offsets"], ck)
        d_rec = torch.from_numpy(rec_np).to(dev)
        d_roff = to_dev(lens, dev)
        v2_out = {k: torch.empty(n, dtype={np.uint8: torch.uint8, np.uint32: torch.int32}.get(t, torch.int64),
                                 device=dev) for k, t in Engine.V2_FIELDS}

        def v2_step(i=None):
            eng.v2_decode_verify_dev(d_rec, d_roff, v2_out)

        _, v2_ms, v2_b = timed_launches(v2_step, max(10, args.steps), 2, stream, sync)
        v2_avg = min(v2_b, float(np.mean(v2_ms)))
        cor = v2_out["corrupt"].cpu().numpy().astype(bool)
        v2_ok = bool((v2_out["status"].cpu().numpy() == 0).all()) and \
            bool(np.array_equal(cor, flip)) and \
            bool(np.array_equal(v2_out["computed"].cpu().numpy().view(np.uint64),
                                out.cpu().numpy().view(np.uint64)))
        sample_ok = None
        if rank == 0 and not args.no_cpu:  # the oracle decoder on the first 512 records
            import jraft_oracle as O
            m = 512
            so = O.v2_decode_batch(rec_np[:int(lens[m])], lens[:m + 1])
            sample_ok = bool(np.array_equal(so["computed"], v2_out["computed"].cpu().numpy()[:m].view(np.uint64)))
        tot = int(lens[-1])
        v2_alg = tot + 8 * (n + 1) + 56 * n
        extras["v2_decode_verify"] = {
            "workload": f"{n} stored V2 records (C5 entries, 16 KiB data + header + checksum "
                        f"field), decode + isCorrupted",
            "GBps_records": tot / (v2_avg * 1e-3) / 1e9, "ms_per_batch": v2_avg,
            "consistent_with_logentry_kernel": v2_ok, "oracle_sample_ok": sample_ok,
            "roofline": {"bound": "hbm", "achieved": v2_alg / (v2_avg * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": v2_alg / (v2_avg * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                         **traffic_fields("v2_parse", "crc64_rounds_kernel<true",
                                          "crc64_finish_kernel<false", "v2_finish")}}
        del d_rec, v2_out

    if not args.no_crc and not args.headline_only:
        # RheaKV snapshot archive CRC64 (java.util.zip.Checksum, AbstractKVStoreSnapshotFile
        # .java:121,139): (a) one archive = the whole C5 payload as a single stream chunk;
        # (b) every region's archive chunk of 16 KiB folded into its own register (S = n).
        pay_u8 = d["payload"]
        tot_b = int(pay_u8.numel())
        one_off = torch.tensor([0, tot_b], dtype=torch.int64, device=dev)
        reg1 = torch.zeros(1, dtype=torch.int64, device=dev)
        regS = torch.zeros(n, dtype=torch.int64, device=dev)

        def snap1_step(i=None):
            eng.crc64_stream_update_dev(reg1, pay_u8, one_off)

        def snapS_step(i=None):
            eng.crc64_stream_update_dev(regS, pay_u8, d["offsets"])

        _, s1_ms, s1_b = timed_launches(snap1_step, max(10, args.steps), 2, stream, sync)
        _, sS_ms, sS_b = timed_launches(snapS_step, max(10, args.steps), 2, stream, sync)
        s1_avg = min(s1_b, float(np.mean(s1_ms)))
        sS_avg = min(sS_b, float(np.mean(sS_ms)))
        snap_ok = None
        if rank == 0 and not args.no_cpu:
            # chained pieces == one chunk (the combine law), and the oracle on a 16 MiB prefix
            import jraft_oracle as O
            reg1.zero_()
            snap1_step()
            whole = int(reg1.cpu().numpy().view(np.uint64)[0])
            reg1.zero_()
            for a in range(0, tot_b, 64 << 20):
                eng.crc64_stream_update_dev(
                    reg1, pay_u8, torch.tensor([a, min(tot_b, a + (64 << 20))], dtype=torch.int64,
                                               device=dev))
            chained = int(reg1.cpu().numpy().view(np.uint64)[0])
            pre = 16 << 20
            reg1.zero_()
            eng.crc64_stream_update_dev(reg1, pay_u8,
                                        torch.tensor([0, pre], dtype=torch.int64, device=dev))
            got_pre = int(reg1.cpu().numpy().view(np.uint64)[0])
            exp_pre = O.crc64(eb["payload"][:pre].tobytes())
            snap_ok = whole == chained and got_pre == exp_pre
        alg1 = tot_b + 16 + 8
        algS = tot_b + 8 * (n + 1) + 16 * n
        extras["snapshot_stream_crc64"] = {
            "workload": f"C5 payload ({tot_b >> 20} MiB) as (a) one snapshot archive stream, "
                        f"(b) {n} region streams x 16 KiB chunks (CRC64.update on resident registers)",
            "archive_GBps": tot_b / (s1_avg * 1e-3) / 1e9, "archive_ms": s1_avg,
            "regions_GBps": tot_b / (sS_avg * 1e-3) / 1e9, "regions_ms": sS_avg,
            "bit_exact_vs_oracle": snap_ok,
            "roofline": {"bound": "hbm", "achieved": alg1 / (s1_avg * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": alg1 / (s1_avg * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                         "kernel": "archive leg (one 1 GiB chunk)", "traffic": None}}
        del regS

    if not args.no_crc and not args.headline_only:
        # C1 (configs[0], the reference's CPU case) on the GPU: 1 group x 3 peers, 1M appended
        # 256-B DATA entries -- one step = LogEntry.checksum of every entry (stamped on append,
        # LogManagerImpl.java:313-318) + the group's commit over its 1M pending ballots
        c1 = W.CONFIGS["C1"]
        n1 = c1["pending"]
        e1 = W.entry_batch(n1, c1["entry_bytes"], seed=W.SEED_BASE ^ 1)
        d1 = {k: to_dev(v, dev) for k, v in e1.items() if isinstance(v, np.ndarray)}
        out1 = torch.empty(n1, dtype=torch.int64, device=dev)
        q1 = W.quorum_batch("C1")
        q1d = {k: to_dev(v, dev) for k, v in q1.items()}
        c1c = torch.empty(1, dtype=torch.int64, device=dev)
        c1s = torch.empty(1, dtype=torch.uint8, device=dev)

        def c1_step(i=None):
            eng.logentry_checksum_batch_dev(d1["etype"], d1["index"], d1["term"], None,
                                            d1["payload"], d1["offsets"], out1)
            eng.quorum_epoch_dev(q1d["match"], q1d["pending_index"], q1d["last_appended"],
                                 q1d["last_committed"], q1d["conf"], c1c, c1s)

        _, c1_ms, c1_b = timed_launches(c1_step, max(10, args.steps), 2, stream, sync)
        c1_avg = min(c1_b, float(np.mean(c1_ms)))
        c1_ok = None
        if rank == 0 and not args.no_cpu:
            import jraft_oracle as O
            exp1 = O.logentry_checksum_batch(e1["etype"], e1["index"], e1["term"], None,
                                             e1["payload"], e1["offsets"])
            ce, se, _ = O.quorum_epoch_replay(q1["match"], q1["pending_index"],
                                              q1["last_appended"], q1["last_committed"],
                                              q1["conf"], chunk=1024)
            c1_ok = bool(np.array_equal(out1.cpu().numpy().view(np.uint64), exp1)) and \
                bool(np.array_equal(c1c.cpu().numpy(), ce))
        extras["C1"] = {
            "workload": "C1: 1 group x 3 peers, 1M appended 256-B LogEntries: checksum + commitAt",
            "ms_per_step": c1_avg, "entries_per_s": n1 / (c1_avg * 1e-3),
            "GBps_payload": n1 * c1["entry_bytes"] / (c1_avg * 1e-3) / 1e9,
            "bit_exact_vs_oracle": c1_ok}
        del d1, out1

    if not args.headline_only:
        # leader lease / alive quorum on C3-shaped groups
        rng = np.random.default_rng(rank)
        now_ms, lease_to = 1 << 40, 900
        # rotating timestamp buffers, as for the epochs: no launch re-reads the previous
        # launch's inputs out of the MALL / L2
        ts_bufs = [to_dev((now_ms - rng.integers(0, 2 * lease_to, (P, G))).astype(np.int64), dev)
                   for _ in range(QUORUM_EPOCH_BUFFERS)]
        self_slot = torch.zeros(G, dtype=torch.uint8, device=dev)
        lead = torch.zeros(G, dtype=torch.int64, device=dev)
        lok = torch.empty(G, dtype=torch.uint8, device=dev)
        ldead = torch.empty(G, dtype=torch.int16, device=dev)
        lconf = epochs[0]["conf"]

        lstate = {"i": 0}

        def lease_step(i=None):
            ts = ts_bufs[lstate["i"] % QUORUM_EPOCH_BUFFERS]
            lstate["i"] += 1
            eng.lease_check_dev(ts, lconf, self_slot, now_ms, lease_to, lok, lead, ldead)

        _, lease_ms, lease_b = timed_launches(lease_step, args.steps, args.warmup, stream, sync)
        lease_avg = min(lease_b, float(np.mean(lease_ms)))
        lb = (8 * P + 28) * G
        extras["lease_check"] = {
            "workload": f"{G} leader groups x {P} peers (conf + old conf), checkDeadNodes0",
            "decisions_per_s": G / (lease_avg * 1e-3), "kernel_ms": lease_avg,
            "roofline": {"bound": "hbm", "achieved": lb / (lease_avg * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": lb / (lease_avg * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                         **traffic_fields("lease_check_kernel<5")}}

        # commit fan-out (FSMCaller.doCommitted / ClosureQueue.popClosureUntil) of the C3 epochs:
        # each epoch's committed[] feeds the fan-out of its groups; every launch starts from
        # fresh closure queues (restored outside the timed event pair)
        fan_sets = []
        for t in epochs:
            c = torch.empty(G, dtype=torch.int64, device=dev)
            eng.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                                 t["last_committed"], t["conf"], c, status)
            cq_size0 = t["last_appended"] - t["pending_index"] + 1
            fan_sets.append({"prev": t["last_committed"], "c": c, "la": t["last_committed"],
                             "cf0": t["pending_index"], "cs0": cq_size0,
                             "cf": torch.empty_like(c), "cs": torch.empty_like(c)})
        fan_fc = torch.empty(G, dtype=torch.int64, device=dev)
        fan_st = torch.empty(G, dtype=torch.uint8, device=dev)
        fan_list = torch.empty((G + 63) // 64, dtype=torch.int64, device=dev)
        fan_num = torch.zeros(1, dtype=torch.int32, device=dev)

        def fan_restore():
            for f in fan_sets:
                f["cf"].copy_(f["cf0"])
                f["cs"].copy_(f["cs0"])

        def fan_launch(f):
            eng.commit_fanout_dev(f["prev"], f["c"], f["la"], f["cf"], f["cs"], fan_fc, fan_st,
                                  fan_list, fan_num)

        fan_restore()
        fan_launch(fan_sets[0])
        sync()
        n_listed = int(fan_num.item())
        n_pop = int((fan_sets[0]["cf"] != fan_sets[0]["cf0"]).sum().item())
        fan_ms = []
        for rep in range(max(1, args.warmup) + max(1, args.steps // 4)):
            fan_restore()
            sync()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for f in fan_sets:
                fan_launch(f)
            e1.record(stream)
            sync()
            if rep >= max(1, args.warmup):
                fan_ms.append(e0.elapsed_time(e1) / len(fan_sets))
        fan_avg = float(np.mean(fan_ms))
        # reads prev/committed/lastApplied/cqFirst/cqSize 40 B, writes firstClosure 8 + status 1
        # + the listed bitmap 1/8; + 16 B queue write-back per popping group
        fb = 49 * G + G // 8 + 16 * n_pop
        extras["commit_fanout"] = {
            "workload": f"{G} groups (C3 epoch output) -> doCommitted/popClosureUntil, "
                        f"{n_listed} listed, {n_pop} popping",
            "groups_per_s": G / (fan_avg * 1e-3), "ms_per_launch": fan_avg,
            "roofline": {"bound": "hbm", "achieved": fb / (fan_avg * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": fb / (fan_avg * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                         **traffic_fields("fanout_eval")}}

    # ------------------------------------------------ measured HBM ceiling --
    # device-to-device copy of 2 GiB (torch's copy kernel): read + write bytes / time, the
    # "peak_measured" of SURVEY.md §8d (frac stays against the 8 TB/s spec)
    src = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    _, _, cp_ms = timed_launches(lambda i=None: dst.copy_(src), 5, 2, stream, sync)
    words = src.view(torch.int64)
    _, _, rd_ms = timed_launches(lambda i=None: torch.bitwise_xor(words[: words.numel() // 2],
                                                                  words[words.numel() // 2:],
                                                                  out=dst.view(torch.int64)[: words.numel() // 2]),
                                 5, 2, stream, sync)
    peak_meas = {"copy_GBps": 2 * src.numel() / (cp_ms * 1e-3) / 1e9,
                 "xor_GBps": 1.5 * src.numel() / (rd_ms * 1e-3) / 1e9,
                 "how": "torch kernels on 2 GiB: D2D copy (read + write bytes) and a 2-input "
                        "xor into half-size output (2 reads + 1 write) / time"}
    del src, dst, words

    # ------------------------------------------------ CPU baselines ---------
    cpu_q = cpu_c = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu_q = cpu_quorum_baseline(args.cpu_budget)
        if not args.no_crc:
            cpu_c = cpu_crc_baseline(args.cpu_budget)
        if crc is not None and cpu_c is not None:
            crc["cpu_baseline"] = cpu_c

    if rank == 0:
        line = {
            "metric": "quorum commit decisions/sec",
            "value": value,
            "unit": "decisions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded splitmix64, SURVEY.md §8d)",
            "config": {
                "workload": ("C3: 1M Raft groups x 5 peers, joint consensus (old 3 + new 5), "
                             "1k pending/group" if world == 1 else
                             f"C4: {G * world} Raft groups x 5 peers sharded by groupId, "
                             f"{G} per GPU, + RCCL all-gather of committed[]"),
                "groups_per_gpu": G, "peers": P, "epoch_buffers": QUORUM_EPOCH_BUFFERS,
                "parallelism": f"groupId shards x{world}",
            },
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                         "kernel": "quorum_epoch_pair_kernel<5, ...>", "kernel_ms": k_avg_ms,
                         "kernel_ms_per_launch_events": float(np.mean(kern_ms)),
                         "bytes_per_launch": q_bytes, "peak_measured": peak_meas},
            "cpu_baseline": cpu_q,
            "crc64": crc,
            "C2": {"workload": "C2: 10k groups x 3 peers x 1k pending (configs[1])",
                   "decisions_per_s": G2 * args.steps / c2_wall,
                   "entry_ballots_per_s": G2 * 1024 * args.steps / c2_wall,
                   "kernel_ms": c2_batched_ms,
                   "batched_epochs": {
                       "epochs_per_launch": KE, "kernel_ms": c2k_avg,
                       "decisions_per_s": G2 * KE / (c2k_avg * 1e-3),
                       # per group-epoch: match 8P + lastAppended 8 read, committed 8 + status 1
                       # written (41 B at P = 3); pendingIndex/lastCommitted/conf once per group
                       "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBPS,
                                    "achieved": (G2 * KE * 41 + G2 * 24) / (c2k_avg * 1e-3) / 1e9},
                       "bit_exact_vs_oracle_64_groups": c2k_ok}},
            "next_rows": extras,
            "end_to_end_host_buffers": e2e,
        }
        tr = pmc_traffic("quorum_epoch_pair_kernel<5")
        if tr is not None:
            line["roofline"]["traffic"] = tr["bytes"]
            line["roofline"]["traffic_source"] = tr["source"]
        if crc is not None:
            tr = pmc_traffic("crc64_rounds_kernel<false", "crc64_finish_kernel<true")
            if tr is not None:
                crc["roofline"]["traffic"] = tr["bytes"]
                crc["roofline"]["traffic_source"] = tr["source"]
        print(json.dumps(line))
    eng.use_stream(None)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
