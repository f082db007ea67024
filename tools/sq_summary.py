"""Median per-dispatch SQ counters of one kernel from a tools/pmc_sq.sh run.

    python tools/sq_summary.py <tag> <kernel-substring> [trajectories-per-launch] [out.json]
Prints JSON: counters, per-wave instruction counts and derived ratios
(VALU lane utilisation = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)),
and the EXECUTED FP64 work per trajectory: (2 FMA + MUL + ADD + TRANS) wave
instructions x 64 lanes x the lane utilisation / trajectories.  bench.py
reads that figure from the committed profiles/r03_sq_*.json to state real
pipe use beside the dense-equivalent roofline.  With out.json the summary is
also written there.
"""
import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, kernel = sys.argv[1:3]
    units = float(sys.argv[3]) if len(sys.argv) > 3 else None
    base = os.path.join(REPO, "gpurun_out", f"sq_{tag}")
    vals = {}
    for p in ("p1", "p2"):
        path = os.path.join(base, p, "run_counter_collection.csv")
        per = {}
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel not in row["Kernel_Name"]:
                    continue
                per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
                per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for k, d in per.items():
            vals[k] = statistics.median(d.values())
    out = {"counters": vals}
    w = vals.get("SQ_WAVES")
    if w:
        out["per_wave"] = {k: v / w for k, v in vals.items() if k.startswith("SQ_INSTS")}
    if units:
        out["per_trajectory"] = {k: v / units for k, v in vals.items() if k.startswith("SQ_INSTS")}
    if vals.get("SQ_ACTIVE_INST_VALU"):
        out["valu_lane_utilisation"] = vals["SQ_THREAD_CYCLES_VALU"] / (
            64.0 * vals["SQ_ACTIVE_INST_VALU"])
    f64 = sum(vals.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                          "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64"))
    if vals.get("SQ_INSTS_VALU"):
        out["f64_share_of_valu"] = f64 / vals["SQ_INSTS_VALU"]
    if units and vals.get("SQ_ACTIVE_INST_VALU"):
        flop_instr = (2.0 * vals.get("SQ_INSTS_VALU_FMA_F64", 0.0) +
                      vals.get("SQ_INSTS_VALU_MUL_F64", 0.0) +
                      vals.get("SQ_INSTS_VALU_ADD_F64", 0.0) +
                      vals.get("SQ_INSTS_VALU_TRANS_F64", 0.0))
        out["executed_f64_flop_per_trajectory"] = (
            flop_instr * 64.0 * out["valu_lane_utilisation"] / units)
    out["kernel"] = kernel
    out["trajectories_per_launch"] = units
    # the kernel's average duration in the same build's kernel-trace pass:
    # bench.py uses the entry only for a run within 15 % of it
    stats = os.path.join(base, "trace", "run_kernel_stats.csv")
    try:
        with open(stats) as f:
            rows = [r for r in csv.DictReader(f) if kernel in r["Name"]]
        if rows:
            out["avg_ns"] = float(rows[0]["AverageNs"])
    except (OSError, KeyError, ValueError):
        pass
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
