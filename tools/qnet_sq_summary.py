"""SQ counters of the config-5 kernel from the four PMC passes of tools/pmc_qnet.sh.

    python tools/qnet_sq_summary.py gpurun_out/pmcq [--out profiles/r01/qnet_sq_s3/summary.json]

Per launch = mean over the qnet_rollout*_kernel dispatches of tools/profile_qnet.py (2^20 envs,
16 steps each); per wave-step = per launch / (2^20 / 64 x 16) 64-env tile-steps.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ENVS, STEPS = 1 << 20, 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    for p in glob.glob(os.path.join(a.pmc_dir, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if "qnet_rollout" not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]][(p, r["Dispatch_Id"])] += float(r["Counter_Value"])
    per = {c: sum(d.values()) / len(d) for c, d in vals.items()}
    tiles = ENVS / 64 * STEPS
    out = {"kernel": "qnet_rollout_ws_kernel<0>, 2^20 envs, 16 steps per launch, steady state",
           "per_launch": per,
           "per_wave_step": {"valu_insts_incl_mfma": per["SQ_INSTS_VALU"] / tiles,
                             "mfma_insts": per["SQ_INSTS_MFMA"] / tiles,
                             "lds_insts": per["SQ_INSTS_LDS"] / tiles,
                             "salu_insts": per["SQ_INSTS_SALU"] / tiles},
           "wave_time_split": {"wait_any(s_waitcnt)": per["SQ_WAIT_ANY"] / per["SQ_WAVE_CYCLES"],
                               "wait_inst_any(issue stall)": per["SQ_WAIT_INST_ANY"] / per["SQ_WAVE_CYCLES"],
                               "active_inst_any": per["SQ_ACTIVE_INST_ANY"] / per["SQ_WAVE_CYCLES"]}}
    print(json.dumps(out, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
