#!/usr/bin/env python3
"""Static check of the LDS-DMA conv kernels (csrc/ym_conv_dma.hip) in the gfx950 assembly.

The K loop waits with a counted `s_waitcnt vmcnt(NL)` that assumes every stage issues exactly NL = SUB·(BM + BN)/(32·KG)
`buffer_load_dwordx4 … lds` wave-instructions (NSTAGE-1 prologue stages + 1 in the loop body = NSTAGE·NL per kernel;
NSTAGE and SUB are the kernel's last two template arguments).  If the
compiler ever duplicates a DMA into divergent branches, the count is off and the wait no longer covers the stage —
silently wrong results on the GPU.  This check compiles the file for gfx950 (device only, -S) and counts.

    python tools/check_dma_asm.py [path/to/ym_conv_dma.hip]   → exit 1 on a mismatch
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "yolo-infer_amd", "csrc", "ym_conv_dma.hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def kernel_dma_counts(asm: str):
    out = []
    labels = list(re.finditer(r"^(_ZN12_GLOBAL__N_18conv_dma\w+):", asm, re.M))
    for i, m in enumerate(labels):
        end = labels[i + 1].start() if i + 1 < len(labels) else len(asm)
        body = asm[m.end():end].split(".Lfunc_end")[0]
        bm, bn, kind, split, kg, nstage, sub = map(
            int, re.search(r"Li(\d+)ELi(\d+)ELi(\d)ELi(\d)ELi(\d)ELi(\d)ELi(\d)E", m.group(1)).groups())
        nl = sub * (bm // 8 + bn // 8) // (4 * kg)  # DMA instructions per wave per stage
        n = len(re.findall(r"buffer_load_dwordx4 .*\blds\b", body))
        out.append((m.group(1), bm, bn, kind, split, n, nstage * nl))  # (NSTAGE-1) prologue + 1 loop stage
    return out


def main(src=SRC):
    with tempfile.TemporaryDirectory() as d:
        s = os.path.join(d, "dma.s")
        subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", src, "-o", s],
                       check=True)
        rows = kernel_dma_counts(open(s).read())
    bad = [r for r in rows if r[5] != r[6]]
    for r in rows:
        print(f"{r[0][25:70]:45s} dma={r[5]:3d} expected={r[6]:3d} {'OK' if r[5] == r[6] else 'MISMATCH'}")
    print(f"{len(rows)} kernels, {len(bad)} mismatches")
    return 1 if bad or not rows else 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
