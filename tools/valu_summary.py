"""Per-kernel compute-side summary of the tools/pmc_valu.sh passes.

    python tools/valu_summary.py gpurun_out/pmcv [--out profiles/valu_busy.json]

For each kernel of tools/profile_valu.py (8 dispatches each, 2^20 envs): VALUBusy / SALUBusy
(rocprofv3's derived metrics: issue cycles of the four SIMDs of every CU over the kernel's
GPU time), and per 64 env-steps (one wave-step) the VALU / SALU / LDS instruction counts and
the fp64 share -- the VALU-issue roofline the kernel is judged against.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ENVS = 1 << 20
STEPS = {"step_kernel": 1, "rollout_kernel": 16, "qnet_rollout": 16, "hdqn_rollout": 16}


def kernel_key(name):
    """qnet_rollout / hdqn_rollout for the opponent-mode-0 instances (the names earlier rounds
    used), qnet_rollout<2> etc. for the others; step_kernel / rollout_kernel."""
    import re

    for k in ("hdqn_rollout", "qnet_rollout", "step_kernel", "rollout_kernel"):  # most specific first
        if k in name:
            m = re.search(k + r"\w*<(\d)", name)
            if k in ("hdqn_rollout", "qnet_rollout") and m and m.group(1) != "0":
                return f"{k}<{m.group(1)}>"
            return k
    return None


def base_key(k):
    return k.split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
    for p in glob.glob(os.path.join(a.pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(p)):
            k = kernel_key(r["Kernel_Name"])
            if k:
                per[(k, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, c, _), v in per.items():
            vals[k][c].append(v)
    out = {}
    for k, cs in vals.items():
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        wave_steps = ENVS / 64 * STEPS[base_key(k)]
        row = {"per_dispatch": mean, "env_steps_per_dispatch": ENVS * STEPS[base_key(k)]}
        for c in ("VALUBusy", "SALUBusy"):
            if c in mean:
                row[c] = mean[c]
        per_ws = {c[9:].lower(): mean[c] / wave_steps for c in mean if c.startswith("SQ_INSTS_")}
        row["insts_per_64_env_steps"] = per_ws
        f64 = sum(per_ws.get(c, 0.0) for c in ("valu_fma_f64", "valu_mul_f64", "valu_add_f64", "valu_trans_f64"))
        if "valu" in per_ws:
            row["fp64_share_of_valu"] = f64 / per_ws["valu"]
        if "MfmaUtil" in mean:
            # rocprofv3's derived MfmaUtil: MFMA-pipe busy cycles summed over the SIMDs over
            # (GPU-active cycles x SIMD count), in percent
            row["mfma_busy_frac"] = mean["MfmaUtil"] / 100.0
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in mean:
            row["mfma_bf16_flops_per_env_step"] = mean["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / (wave_steps * 64)
        if "SQ_LDS_BANK_CONFLICT" in mean and "SQ_LDS_IDX_ACTIVE" in mean and mean["SQ_LDS_IDX_ACTIVE"]:
            row["lds_bank_conflict_frac"] = mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_LDS_IDX_ACTIVE"]
        if "SQ_WAVE_CYCLES" in mean:
            row["wave_time_split"] = {"wait_any": mean.get("SQ_WAIT_ANY", 0) / mean["SQ_WAVE_CYCLES"],
                                      "wait_inst_any": mean.get("SQ_WAIT_INST_ANY", 0) / mean["SQ_WAVE_CYCLES"],
                                      "active_inst_any": mean.get("SQ_ACTIVE_INST_ANY", 0) / mean["SQ_WAVE_CYCLES"]}
        out[k] = row
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
