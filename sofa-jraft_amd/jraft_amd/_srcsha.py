"""Content hash of libjrq's kernel sources (sofa-jraft_amd/csrc/*).

One definition, used three ways: the Makefile compiles it into libjrq.so (`jrq_build_id()`),
`__graft_entry__.build()` rebuilds when the library's id differs from the tree's, and bench.py /
smoke() refuse a library whose id is not the hash of the sources beside it (the binary that ran
is the one these sources make).  Committed PMC summaries carry the same hash (`csrc_sha`).

    python3 _srcsha.py <csrc dir>   prints the hash
"""
import glob
import hashlib
import os
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


def src_sha(csrc: str = CSRC) -> str:
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(csrc, "*"))):
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def lib_build_id(lib_path: str):
    """The id compiled into a libjrq.so file, read from its bytes (no loading, no GPU), or
    None when the file has none."""
    try:
        with open(lib_path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    tag = b"JRQ_BUILD_ID="
    i = data.find(tag)
    if i < 0:
        return None
    return data[i + len(tag): i + len(tag) + 16].decode("ascii", "replace")


if __name__ == "__main__":
    print(src_sha(sys.argv[1] if len(sys.argv) > 1 else CSRC))
