"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference (Java) holds no numeric known-answer vectors for this path
 and cannot run here (no JDK).  The fixtures are therefore
produced by the oracle's restatement, which is itself pinned by:
  * the CRC-64/ECMA-182 catalogue check value crc64("123456789") = 0x6C40DF5F0B497347
    (cited at jraft-core/.../util/CRC64.java:36-39),
  * crc64_table_pin.json: all 256 entries equal the literal table at CRC64.java:41-92
    (oracle/pin_table.py parses the Java file as text),
  * the reference's own test inputs (LogEntryTest, LogIdTest, PeerIdTest, BallotTest,
    BallotBoxTest) re-evaluated here.
Run: python tests/golden/gen_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import jraft_oracle as O  # noqa: E402


def hx(v):
    return f"0x{v:016X}"


def crc_vectors():
    rng = random.Random(0xC4C64)
    items = [b"", b"1", b"123456789", b"hello world", b"hello", b"hEllo",
             b"\x00" * 16, b"\xff" * 33, b"localhost:8081", b"192.168.1.1:8081:1"]
    for n in [2, 3, 7, 8, 9, 15, 16, 17, 31, 63, 64, 65, 127, 255, 256, 257, 1023, 1024, 4099]:
        items.append(bytes(rng.getrandbits(8) for _ in range(n)))
    payload = b"".join(items)
    offs = [0]
    for it in items:
        offs.append(offs[-1] + len(it))
    return {
        "note": "crc64 = CrcUtil.crc64(payload[offsets[i]:offsets[i+1]]) (oracle restatement)",
        "payload_hex": payload.hex(),
        "offsets": offs,
        "crc64": [hx(O.crc64(it)) for it in items],
    }


def entity_vectors():
    px = O.peerid_checksum("localhost", 99, 1) ^ O.peerid_checksum("localhost", 100, 2)
    return {
        "note": "inputs of the reference's own tests, values from the oracle restatement",
        "crc64_check_123456789": hx(O.crc64(b"123456789")),
        "logid": [  # LogIdTest.java:42-50 uses LogId(1,2)
            {"index": 1, "term": 2, "checksum": hx(O.logid_checksum(1, 2))},
            {"index": 100, "term": 3, "checksum": hx(O.logid_checksum(100, 3))},
            {"index": -1, "term": (1 << 63) - 1, "checksum": hx(O.logid_checksum(-1, (1 << 63) - 1))},
        ],
        "peerid": [  # PeerIdTest.java:72-78
            {"ip": "192.168.1.1", "port": 8081, "idx": 1,
             "checksum": hx(O.peerid_checksum("192.168.1.1", 8081, 1))},
            {"ip": "localhost", "port": 8081, "idx": 0,
             "checksum": hx(O.peerid_checksum("localhost", 8081, 0))},
        ],
        "logentry": [  # LogEntryTest.testChecksum (LogEntryTest.java:95-125)
            {"type": 1, "index": 100, "term": 3, "peer_xor": hx(px), "data": "hello",
             "checksum": hx(O.logentry_checksum(1, 100, 3, px, b"hello"))},
            {"type": 1, "index": 1, "term": 3, "peer_xor": hx(px), "data": "hello",
             "checksum": hx(O.logentry_checksum(1, 1, 3, px, b"hello"))},
            {"type": 1, "index": 100, "term": 3, "peer_xor": hx(px), "data": "hEllo",
             "checksum": hx(O.logentry_checksum(1, 100, 3, px, b"hEllo"))},
            {"type": 2, "index": 7, "term": 1, "peer_xor": hx(0), "data": "",
             "checksum": hx(O.logentry_checksum(2, 7, 1, 0, b""))},
        ],
    }


def ballot_box_traces():
    """Event traces through the oracle BallotBox: every call with its result and the
    state after it.  Peers are small ids (0 = localhost:8081, 1 = :8082, 2 = :8083, 3 = :8084)."""
    traces = []

    def run(name, calls):
        bb = O.BallotBox()
        steps = []
        for c in calls:
            op = c[0]
            try:
                if op == "reset":
                    r = bb.reset_pending_index(c[1])
                elif op == "append":
                    r = bb.append_pending_task(c[1], c[2])
                elif op == "commit":
                    r = bb.commit_at(c[1], c[2], c[3])
                elif op == "setlc":
                    r = bb.set_last_committed_index(c[1])
                elif op == "clear":
                    bb.clear_pending_tasks()
                    r = None
                res = r
            except IndexError:
                res = "AIOOBE"
            except ValueError:
                res = "IAE"
            steps.append({"call": list(c), "result": res,
                          "last_committed": bb.last_committed_index,
                          "pending_index": bb.pending_index, "queue_size": bb.queue_size,
                          "on_committed_calls": bb.on_committed_calls})
        traces.append({"name": name, "steps": steps})

    # BallotBoxTest.testCommitAt (BallotBoxTest.java:109-137)
    run("testCommitAt", [("commit", 1, 3, 0), ("reset", 1), ("append", [0, 1, 2], [0]),
                         ("commit", 1, 3, 0), ("commit", 1, 1, 0), ("commit", 1, 1, 1)])
    # BallotBoxTest.testAppendPendingTask / testClearPendingTasks / testResetPendingIndex
    run("testAppendPendingTask", [("append", [0, 1, 2], [0]), ("reset", 1), ("append", [0, 1, 2], [0]),
                                  ("clear",)])
    run("testSetLastCommittedIndexHasPending", [("reset", 1), ("setlc", 1)])
    run("testSetLastCommittedIndexLessThan", [("setlc", -1)])
    run("testSetLastCommittedIndex", [("setlc", 1)])
    # even-size removal: 4 -> 3 peers, later entry commits first (BallotBox.java:124-129)
    run("evenSizeRemoval", [("reset", 10)] + [("append", [0, 1, 2, 3], None)] * 3 +
        [("append", [0, 1, 2], None)] * 3 +
        [("commit", 10, 15, 0), ("commit", 10, 15, 1), ("commit", 10, 11, 2)])
    # unknown peer never counts (BallotTest.testGrant)
    run("unknownPeer", [("reset", 1), ("append", [0, 1, 2], None), ("commit", 1, 1, 0),
                        ("commit", 1, 1, 3), ("commit", 1, 1, 1)])
    # randomised contiguous ack interleavings with a joint-consensus stretch
    rng = random.Random(7)
    for t in range(6):
        calls = [("reset", 1)]
        for i in range(40):
            if 10 <= i < 20:
                calls.append(("append", [0, 1, 2, 3, 4], [0, 1, 2]))
            else:
                calls.append(("append", [0, 1, 2] if i < 10 else [0, 1, 2, 3, 4], None))
        nxt = [1, 1, 1, 1, 1]
        for _ in range(60):
            p = rng.randrange(5)
            k = rng.randint(1, 6)
            last = min(40, nxt[p] + k - 1)
            if nxt[p] <= 40:
                calls.append(("commit", nxt[p], last, p))
                nxt[p] = last + 1
        calls.append(("commit", 1, 41, 0))  # past the queue: AIOOBE
        run(f"random{t}", calls)
    return traces


def main():
    out = {
        "crc64_vectors.json": crc_vectors(),
        "entity_vectors.json": entity_vectors(),
        "ballot_box_traces.json": {"traces": ballot_box_traces()},
    }
    for name, obj in out.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1)
        print("wrote", name)


if __name__ == "__main__":
    main()
