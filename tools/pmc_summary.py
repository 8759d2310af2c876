"""Per-launch memory-side bytes from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, separate runs).

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR --envs 1048576 4194304 8388608 [--out profiles/pmc_traffic.json]

Dispatch order inside each env count is reset x reps, observe x reps, step x reps (tools/profile_pmc.py),
so rows are grouped by kernel name and then split evenly over the env counts.
Bytes follow MI355X_MICROARCH.md's HBM/rocprofv3 rule for gfx950: FETCH_SIZE reports half the
bytes of a wide streaming read, so it is doubled; WRITE_SIZE is taken as it reads. Both count
L2 -> fabric traffic, so Infinity Cache (MALL) hits are counted too: the 2^22-env rows (past
the 256 MiB cache) are the DRAM-side figure. The reset kernel (writes exactly 50 B/env) and the
observe kernel (reads exactly 32 B/env) are profiled beside the step kernel as a check of the
rule on this build; their ratios are reported, not applied.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d, counter):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)  # kernel -> [(dispatch, value)]
    for p in paths:
        for r in csv.DictReader(open(p)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            key = "reset" if "reset_kernel" in name else "observe" if "observe_kernel" in name else \
                "step" if "step_kernel" in name else "rollout" if "rollout_kernel" in name else None
            if key:
                per[key].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return {k: [v for _, v in sorted(vals)] for k, vals in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--envs", type=int, nargs="+", required=True)
    ap.add_argument("--out")
    a = ap.parse_args()
    f = load(a.fetch_dir, "FETCH_SIZE")
    w = load(a.write_dir, "WRITE_SIZE")
    res = {}
    for i, n in enumerate(a.envs):
        def mean(tab, k):
            v = tab[k]
            per = len(v) // len(a.envs)
            chunk = v[i * per:(i + 1) * per]
            return 1024.0 * sum(chunk) / len(chunk)  # counters are in KiB
        chk_w = mean(w, "reset") / (50.0 * n)       # ~1.0 expected (narrow 2-byte tf stores included)
        chk_r = 2.0 * mean(f, "observe") / (32.0 * n)  # ~1.0 expected
        sf, sw = mean(f, "step"), mean(w, "step")
        total = 2.0 * sf + sw
        res[n] = {"envs": n, "fetch_raw_bytes": sf, "write_raw_bytes": sw,
                  "fetch_bytes": 2.0 * sf, "write_bytes": sw,
                  "hbm_bytes_per_launch": total,
                  "algorithmic_bytes_per_launch": 152.0 * n,
                  "ratio_to_algorithmic": total / (152.0 * n),
                  "check_observe_read_ratio": chk_r, "check_reset_write_ratio": chk_w,
                  "rule": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md, gfx950)"}
        if "rollout" in f and "rollout" in w:  # T = 16: 52 B per env-step + 100 B of state per env
            rf, rw = mean(f, "rollout"), mean(w, "rollout")
            alg = (52.0 * 16 + 100.0) * n
            res[n]["rollout"] = {"fetch_bytes": 2.0 * rf, "write_bytes": rw, "hbm_bytes_per_launch": 2.0 * rf + rw,
                                 "algorithmic_bytes_per_launch": alg, "ratio_to_algorithmic": (2.0 * rf + rw) / alg,
                                 "note": "the algorithmic bytes leave out the statistics records (32 B read per "
                                         "env per launch, the finishing envs' 64 B written back)"}
    print(json.dumps(res, indent=1))
    if a.out:
        first = res[a.envs[0]]
        json.dump(dict(first, by_envs=res, source="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                       "tools/profile_pmc.py + tools/pmc_summary.py"), open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
