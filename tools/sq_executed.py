"""Collects executed FP64 FLOP per trajectory from tools/sq_summary.py
outputs into profiles/sq_executed.json (read by bench.py's roofline):

    python tools/sq_executed.py <bench config key> <summary json> [...]

key = "<workload>:B<batch>:S<segments>[:soft]:<device kernel>", e.g.
linear:B1024:S10:linear_wave_kernel (bench.py device_kernel()).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    path = os.path.join(REPO, "profiles", "sq_executed.json")
    try:
        with open(path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        data = {}
    args = sys.argv[1:]
    for key, src in zip(args[::2], args[1::2]):
        with open(src) as f:
            summ = json.load(f)
        data[key] = {"executed_f64_flop_per_trajectory": summ["executed_f64_flop_per_trajectory"],
                     "valu_lane_utilisation": summ.get("valu_lane_utilisation"),
                     "avg_ns": summ.get("avg_ns"),
                     "source": os.path.relpath(src, REPO)}
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
