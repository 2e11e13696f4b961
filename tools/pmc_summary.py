"""Average rocprofv3 --pmc counters per kernel over the passes tools/prof/profile.sh
wrote (gpurun_out/pmc_*/pmc_counter_collection.csv) -> one CSV (stdout or path).
clk_GHz = GRBM_GUI_ACTIVE / 8 XCDs / the dispatch's duration, averaged per kernel
(the effective clock, MI355X_MICROARCH.md "DVFS give-back"; reads high below ~0.3 ms)."""
import collections
import csv
import glob
import os
import sys

COLS = ["FETCH_SIZE", "WRITE_SIZE", "SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES",
        "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_LDS",
        "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]


def main(root, out):
    agg = collections.OrderedDict()
    for path in sorted(glob.glob(os.path.join(root, "pmc_*", "pmc_counter_collection.csv"))):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Kernel_Name"].startswith("__amd"):
                    continue
                d = agg.setdefault(r["Kernel_Name"], collections.defaultdict(list))
                d[r["Counter_Name"]].append(float(r["Counter_Value"]))
                if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                    dur = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                    if dur > 0:
                        d["clk_GHz"].append(float(r["Counter_Value"]) / 8.0 / dur)
    w = csv.writer(out)
    w.writerow(["kernel", "dispatches"] + [c + "_avg" for c in COLS] + ["clk_GHz"])
    for k, d in agg.items():
        n = max(len(v) for v in d.values())
        clk = round(sum(d["clk_GHz"]) / len(d["clk_GHz"]), 3) if d.get("clk_GHz") else ""
        w.writerow([k, n] + [round(sum(d[c]) / len(d[c]), 1) if d.get(c) else "" for c in COLS] + [clk])


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            main(root, f)
    else:
        main(root, sys.stdout)
