"""Pin the oracle's CRC64 table against the reference's literal table.

Reads jraft-core/.../util/CRC64.java AS TEXT (study only; nothing is executed or
copied), parses the 256 long literals of CRC_TABLE (CRC64.java:41-92) and checks
them entry-for-entry against the table the oracle generates from the polynomial.
Writes tests/golden/crc64_table_pin.json: the SHA-256 of the table as 256
little-endian uint64 plus a few spot entries, so that later runs (and the GPU box,
where /root/reference does not exist) can re-check without the reference.

Run here (the container that has /root/reference):  python oracle/pin_table.py
"""
import hashlib
import json
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import jraft_oracle as O  # noqa: E402

REF = "/root/reference/jraft-core/src/main/java/com/alipay/sofa/jraft/util/CRC64.java"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden",
                   "crc64_table_pin.json")


def parse_reference_table(path):
    text = open(path, encoding="utf-8").read()
    body = text[text.index("CRC_TABLE"):]
    body = body[body.index("{") + 1: body.index("}")]
    vals = [int(h, 16) for h in re.findall(r"0x([0-9A-Fa-f]{16})L", body)]
    if len(vals) != 256:
        raise SystemExit(f"parsed {len(vals)} entries, expected 256")
    return vals


def main():
    ref = parse_reference_table(REF)
    gen = [int(x) for x in O.table()]
    py = O.py_table()
    bad = [i for i in range(256) if not (ref[i] == gen[i] == py[i])]
    if bad:
        raise SystemExit(f"table mismatch at entries {bad[:8]}")
    digest = hashlib.sha256(np.array(gen, dtype="<u8").tobytes()).hexdigest()
    pin = {
        "source": "jraft-core/src/main/java/com/alipay/sofa/jraft/util/CRC64.java:41-92 (parsed as text)",
        "entries_checked": 256,
        "sha256_le_u64": digest,
        "spot": {str(i): f"0x{gen[i]:016X}" for i in (1, 2, 127, 128, 255)},
    }
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(pin, f, indent=1)
    print("pinned", digest)


if __name__ == "__main__":
    main()
