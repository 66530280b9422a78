#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc --save-temps .s file.

    python tools/asm_blocks.py FILE.s KERNEL_SUBSTRING [--min N]

Blocks are split at .LBB labels and '; %bb.N' markers; back-edges (branches to an earlier block)
are flagged so loop bodies stand out. Counts: MFMA, v_readlane / v_writelane (SGPR spills), s_nop,
LDS reads / writes, buffer loads / stores, barriers, waitcnts.
"""
import re
import sys
from collections import Counter


def main():
    path, key = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 0
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(key) + r"\S*:", l))
    end = start + 1
    while end < len(lines) and not lines[end].startswith(".Lfunc_end"):
        end += 1
    blocks, cur = [], ["entry", Counter(), []]
    for raw in lines[start + 1:end]:
        l = raw.strip()
        if not l:
            continue
        m = re.match(r"^(\.LBB\d+_\d+):", l) or re.match(r"^; (%bb\.\d+):", l)
        if m:
            blocks.append(cur)
            cur = [m.group(1), Counter(), []]
            continue
        if l.startswith((";", ".")):
            continue
        op = l.split()[0]
        cur[1][op] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            cur[2].append(l.split()[1])
    blocks.append(cur)
    idx = {b[0]: i for i, b in enumerate(blocks)}
    tot = Counter()
    for i, (name, c, br) in enumerate(blocks):
        tot.update(c)
        n = sum(c.values())
        if n < mn:
            continue
        mf = sum(v for k, v in c.items() if k.startswith("v_mfma"))
        back = [t for t in br if t in idx and idx[t] <= i]
        print(f"{name:14s} n={n:5d} mfma={mf:4d} rl={c['v_readlane_b32']:4d} wl={c['v_writelane_b32']:4d} "
              f"nop={c['s_nop']:3d} dsr={sum(v for k, v in c.items() if k.startswith('ds_read')):4d} "
              f"dsw={sum(v for k, v in c.items() if k.startswith('ds_write')):3d} "
              f"ld={sum(v for k, v in c.items() if k.startswith('buffer_load') or k.startswith('global_load')):3d} "
              f"st={sum(v for k, v in c.items() if k.startswith('buffer_store') or k.startswith('global_store')):3d} "
              f"bar={c['s_barrier']} wait={c['s_waitcnt']:3d}" + (f"  <- back to {','.join(back)}" if back else ""))
    mf = sum(v for k, v in tot.items() if k.startswith("v_mfma"))
    print(f"TOTAL n={sum(tot.values())} mfma={mf} readlane={tot['v_readlane_b32']} writelane={tot['v_writelane_b32']}")


if __name__ == "__main__":
    main()
