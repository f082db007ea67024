"""Summarise a tools/profile.sh run into profiles/.

python tools/pmc_summary.py <tag> <config_key> <kernel-substring>

Writes profiles/<ROUND>_<tag>_kernel_stats.csv (rocprofv3 --stats), and merges
{"<config_key>:<kernel>": {config, kernel, avg_ns, fetch_kb, write_kb,
bytes_per_launch}} into profiles/pmc_traffic.json (bench.py reads the entry
of its own workload, batch, segments and kernel, and only if its avg_ns is
within 15 % of the run's kernel time).  HBM bytes per launch follow
MI355X_MICROARCH.md's HBM section: FETCH_SIZE and WRITE_SIZE (KB) from
separate --pmc passes, FETCH_SIZE doubled on gfx950.
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(path, kernel, name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
    return statistics.median(vals), len(vals)


def main():
    tag, config_key, kernel = sys.argv[1:4]
    rnd = os.environ.get("ROUND", "r01")
    src = os.path.join(REPO, "gpurun_out", f"prof_{tag}")
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{rnd}_{tag}_kernel_stats.csv"))
    avg_ns = None
    with open(stats) as f:
        for row in csv.DictReader(f):
            if kernel in row["Name"]:
                avg_ns = float(row["AverageNs"])
    fetch, nf = counter(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), kernel,
                        "FETCH_SIZE")
    write, nw = counter(os.path.join(src, "pmc_write", "run_counter_collection.csv"), kernel,
                        "WRITE_SIZE")
    entry = dict(config=config_key, kernel=kernel, avg_ns=avg_ns, fetch_kb_raw=fetch,
                 write_kb=write, dispatches=[nf, nw],
                 bytes_per_launch=(2.0 * fetch + write) * 1024.0,
                 note="FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KB->B")
    path = os.path.join(prof, "pmc_traffic.json")
    data = {}
    if os.path.exists(path):
        with open(path) as f:
            data = json.load(f)
    data[f"{config_key}:{kernel}"] = entry
    with open(path, "w") as f:
        json.dump(data, f, indent=1)
    print(json.dumps(entry))


if __name__ == "__main__":
    main()
