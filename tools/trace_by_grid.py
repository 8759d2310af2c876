"""Per-kernel, per-grid-size dispatch statistics from a rocprofv3 --kernel-trace CSV: the bench runs
the step kernel at 2^20 (the headline leg) and at 2^22 (size_2p22) in one process, so --stats'
single average for `step_kernel<1, false>` mixes both sizes. Usage:

    python tools/trace_by_grid.py gpurun_out/r04m/prof/r04m_kernel_trace.csv [--out file.json]
"""
import argparse
import csv
import json
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    a = ap.parse_args()
    durs = defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
        durs[(name, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    for (name, grid), d in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        if sum(d) < 1000:  # under 1 ms in total
            continue
        out.append({"kernel": name, "grid_threads": grid, "calls": len(d), "avg_us": statistics.mean(d),
                    "median_us": statistics.median(d), "min_us": min(d), "max_us": max(d)})
    for o in out:
        print(f"{o['kernel']:48s} grid {o['grid_threads']:>9d} calls {o['calls']:5d} avg {o['avg_us']:9.1f} us "
              f"median {o['median_us']:9.1f}")
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
