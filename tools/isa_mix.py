#!/usr/bin/env python3
"""Static VALU mix of the aligner's hot loops, priced with the issue costs
measured on gfx950 by tools/valu_rate.hip (profiles/r02/valu_rate_v9.txt).

Compiles csrc/kernels/dovetail_lane.hip to gfx950 assembly (same flags as the
Makefile), takes for each packed kernel the basic block with the most VALU
instructions (the unrolled unmasked row loop, where nearly all cells run) and
writes, per kernel: VALU count, cheap-issue count (~2.5 cycles per wave per
SIMD), full-cost count (~4.4) and the mix's average cost per VALU instruction.
bench.py multiplies the kernels' measured SQ_INSTS_VALU by that average for the
aligner's issue-bound time (roofline_align).

usage: python3 tools/isa_mix.py OUT.json
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "sequence-aligner_amd", "csrc", "kernels", "dovetail_lane.hip")
# measured at 16 waves per SIMD (valu_rate_v9.txt), cycles per wave-instruction per SIMD
CHEAP = ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_bitop3_b32",
         "v_lshrrev_b32", "v_ashrrev_i32", "v_max_u16", "v_add_u16", "v_sub_u16", "v_mov_b32")
COST_CHEAP, COST_FULL = 2.55, 4.35
# (phase 1 runs as dovetail_p1x2_seg_kernel since round 5: the same row loop as dovetail_p1x2_kernel)
KERNELS = {"dovetail_p1x2": "_ZN2sa24dovetail_p1x2_seg_kernel", "dovetail_p2tbx2": "_ZN2sa22dovetail_p2tbx2_kernel"}


def main(out):
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "dl.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-I" + os.path.join(ROOT, "sequence-aligner_amd", "csrc"), "--cuda-device-only", "-S",
                        SRC, "-o", asm], check=True, stderr=subprocess.DEVNULL)
        text = open(asm).read()
    res = {"source": "tools/isa_mix.py", "cost_cheap": COST_CHEAP, "cost_full": COST_FULL,
           "probe": "profiles/r02/valu_rate_v9.txt"}
    for name, sym in KERNELS.items():
        start = text.index("\n" + sym)
        end = text.index(".Lfunc_end", start)
        body = text[start:end].split("\n")
        labels = [i for i, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)]
        best = None
        for a, b in zip(labels, labels[1:] + [len(body)]):
            ins = [l.strip().split()[0] for l in body[a + 1:b]
                   if l.strip() and not l.strip().startswith((".", ";", "//"))]
            valu = [i for i in ins if i.startswith("v_")]
            if best is None or len(valu) > best[0]:
                best = (len(valu), valu, collections.Counter(ins))
        n, valu, hist = best
        cheap = sum(1 for i in valu if i.startswith(CHEAP))
        cyc = cheap * COST_CHEAP + (n - cheap) * COST_FULL
        res[name] = {"loop_valu": n, "cheap": cheap, "full": n - cheap, "s_nop": hist.get("s_nop", 0),
                     "avg_cycles_per_valu": round(cyc / n, 3),
                     "top": hist.most_common(12)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: (v if not isinstance(v, dict) else {kk: vv for kk, vv in v.items() if kk != "top"})
                      for k, v in res.items()}))


if __name__ == "__main__":
    main(sys.argv[1])
