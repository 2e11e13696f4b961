"""Kernel resource table (VGPRs, spills, occupancy, LDS) of one HIP source for
gfx950, from the compiler's -Rpass-analysis=kernel-resource-usage remarks:
    python tools/kres.py csrc/kernels/partition.hip [-DX=1 ...]   (run in sequence-aligner_amd/)"""
import re
import subprocess
import sys

src, extra = sys.argv[1], sys.argv[2:]
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-c", src,
                    "-o", "/tmp/kres.o", "--offload-device-only", "-Rpass-analysis=kernel-resource-usage"] + extra,
                   capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark: +(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for c in rows:
    print("%-70.70s vgpr %4s agpr %3s sspill %4s vspill %4s scratch %4s occ %2s lds %6s" % (
        c["name"].replace("sa::", ""), c.get("VGPRs"), c.get("AGPRs"), c.get("SGPRs Spill"), c.get("VGPRs Spill"),
        c.get("ScratchSize [bytes/lane]"), c.get("Occupancy [waves/SIMD]"), c.get("LDS Size [bytes/block]")))
