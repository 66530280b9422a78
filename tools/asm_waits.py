"""List the compiler's full vector-memory drains (``s_waitcnt vmcnt(0)``) per kernel of a gfx950
assembly file, with the instruction each one guards.

Why: LLVM puts a vmcnt(0) in front of every LDS store it can see after an LDS-DMA
(``buffer_load ... lds``) when it cannot prove the two disjoint -- with one dynamic LDS buffer it
never can -- so a compiled ``*(uint4*)(lds + ...) = v`` inside a DMA-pipelined loop drains every
stage in flight. The box conv kernels lost a DMA latency per channel block and two per tile that
way (conv_box.hip, bx_ds_write128). This lists where such drains sit, so a kernel's pipelined
loops can be checked to contain none.

    hipcc --offload-arch=gfx950 -O3 -c csrc/X.hip --save-temps
    python tools/asm_waits.py X-hip-amdgcn-amd-amdhsa-gfx950.s [kernel-substring]
"""
import re
import subprocess
import sys


def kernels(path):
    name, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
        elif name:
            if line.startswith(".Lfunc_end"):
                yield name, body
                name, body = None, []
            else:
                body.append(line.rstrip("\n"))


def demangle(n):
    try:
        return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, body in kernels(path):
        dn = demangle(name)
        if sub not in dn:
            continue
        insts = [(i, l.strip()) for i, l in enumerate(body) if l.startswith("\t") and not l.strip().startswith(";")]
        hits = []
        for k, (i, ins) in enumerate(insts):
            if not re.match(r"s_waitcnt\s+vmcnt\(0\)", ins):
                continue
            nxt = next((x for _, x in insts[k + 1:k + 12] if re.match(r"(ds_|buffer_|global_|v_mfma|s_barrier)", x)),
                       "")
            hits.append((i, ins, nxt))
        lds_dma = sum(1 for _, x in insts if re.search(r"\blds$", x))
        print(f"{dn[:110]}\n  {len(insts)} insts, {lds_dma} LDS-DMA, {len(hits)} vmcnt(0)")
        for i, ins, nxt in hits:
            print(f"    line {i:6d}: {ins:36s} -> {nxt}")


if __name__ == "__main__":
    main()
