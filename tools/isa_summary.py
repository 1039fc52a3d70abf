#!/usr/bin/env python3
"""Summarise a hipcc --save-temps gfx950 .s file: per kernel, resource usage and the basic
blocks that carry the hot work (LDS table reads, buffer loads, DPP moves), with their
s_waitcnt vmcnt values -- enough to spot spills, waterfall loops and drained prefetches.

usage: isa_summary.py FILE.s [KERNEL_REGEX]
"""
import collections
import re
import sys


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r".")
    src = open(path).read().split("\n")
    funcs, cur = {}, None
    for ln in src:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            cur = m.group(1) if pat.search(m.group(1)) else None
            if cur:
                funcs[cur] = []
            continue
        if cur:
            funcs[cur].append(ln)
        if ln.startswith(".Lfunc_end"):
            cur = None
    meta = "\n".join(src)
    for f, lines in funcs.items():
        res = {}
        for key in ("vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
            m = re.search(r"\.name:\s+" + re.escape(f) + r"\n(?:.*\n){0,40}?\s+\." + key + r":\s+(\d+)", meta)
            res[key] = int(m.group(1)) if m else None
        print(f, res)
        blocks, b = [], None
        for ln in lines:
            m = re.match(r"^(\.LBB\w+):", ln)
            if m:
                b = [m.group(1), []]
                blocks.append(b)
                continue
            s = ln.strip()
            if b and s and not s.startswith(";") and not s.startswith("."):
                b[1].append(s)
        for name, ins in blocks:
            c = collections.Counter(i.split()[0] for i in ins)
            dpp = sum(1 for i in ins if "quad_perm" in i)
            ds = sum(v for k, v in c.items() if k.startswith("ds_read"))
            bl = sum(v for k, v in c.items() if k.startswith("buffer_load") or k.startswith("global_load"))
            sc = sum(v for k, v in c.items() if k.startswith("scratch_"))
            if ds >= 32 or dpp or sc or c["buffer_load_dwordx4"]:
                waits = [i.split()[1] for i in ins if i.startswith("s_waitcnt") and "vmcnt" in i]
                valu = sum(v for k, v in c.items() if k.startswith("v_"))
                print(f"   {name:12s} n={len(ins):4d} ds={ds:3d} valu={valu:4d} loads={bl:2d} dpp={dpp:3d} "
                      f"scratch={sc:2d} vmcnt={waits[:10]}")


if __name__ == "__main__":
    main()
