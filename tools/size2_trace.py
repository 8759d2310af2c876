"""Per-dispatch view of the 2^22 step-kernel launches in a rocprofv3 --kernel-trace CSV of bench.py:
for each launch its duration and the gap since the previous dispatch on the queue, so a slow
window can be told apart as one long dispatch (memory), long gaps (host / queue) or uniformly
slower dispatches (clock / placement). Usage: python tools/size2_trace.py kernel_trace.csv [envs]"""

import csv
import json
import sys


def main(path, envs=1 << 22):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out, prev_end = [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "step_kernel" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == envs:
            out.append({"dur_us": (e - s) / 1e3, "gap_us": None if prev_end is None else (s - prev_end) / 1e3,
                        "name": r["Kernel_Name"][:40]})
        prev_end = e
    durs = [o["dur_us"] for o in out]
    print(json.dumps({"launches": len(out), "first_60": out[:60],
                      "mean_dur_us_windows_of_20": [round(sum(durs[i:i + 20]) / len(durs[i:i + 20]), 1)
                                                    for i in range(0, len(durs), 20)]}, indent=0))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 22)
