#!/usr/bin/env python3
"""Check a gfx950 assembly file for vector-memory ops scheduled between the LDS-DMA pieces of one
stage (``buffer_load ... lds`` runs): kernels whose counted ``vmcnt`` waits assume a stage's DMA
pieces, box / operand loads and stores issue in program order break when the scheduler interleaves
them (a wait that leaves "the load" outstanding then leaves a DMA piece in flight).

    hipcc --offload-arch=gfx950 -O3 -c csrc/X.hip --save-temps
    python tools/dma_order.py X-hip-amdgcn-amd-amdhsa-gfx950.s [kernel-substring]
"""
import re
import subprocess
import sys


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    src = open(path).read().split("\n")
    starts = [(i, l.split(":")[0]) for i, l in enumerate(src) if re.match(r"^_Z\S*:", l)]
    n_bad = 0
    for i, name in starts:
        end = next(j for j in range(i, len(src)) if src[j].startswith(".Lfunc_end"))
        seq = []
        for l in src[i:end]:
            l = l.strip()
            if re.match(r"buffer_load_dword\S* .* lds", l) or re.match(r"global_load_lds", l):
                seq.append("D")
            elif re.match(r"(buffer|global)_(load|store)", l):
                seq.append("M")
        s = "".join(seq)
        if "D" not in s:
            continue
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        if pat and pat not in dem:
            continue
        inter = len(re.findall(r"D+M+D", s))
        if inter:
            n_bad += 1
            print(f"{inter:4d} interleavings  {dem[:110]}")
    print(f"{n_bad} kernel(s) with vector-memory ops between LDS-DMA pieces")


if __name__ == "__main__":
    main()
