"""HBM traffic of the replay store (mg_replay_store) from rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o pmc -- python tools/profile_pmc_replay.py run OUT
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o pmc -- python tools/profile_pmc_replay.py run OUT
    python tools/profile_pmc_replay.py summary OUT [--out profiles/...json]

`run` builds the bench's replay workload (bench.py replay_leg: a 16-step config-5 rollout of 2^20
envs with the shipped l1 checkpoint, appended to a 2^24-row ring) and stores it `--reps` times
after two untimed stores; before that it launches mg_reset and mg_observe `--reps` times each as
the calibration of the counter rule (50 B/env written, 32 B/env read). It writes the store's
algorithmic bytes (bench.replay_algorithmic_bytes) to OUT/replay_workload.json. `summary` applies
MI355X_MICROARCH.md's gfx950 rule (2 x FETCH_SIZE + WRITE_SIZE) per launch of each kernel.
"""
import argparse
import csv
import ctypes
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

KEYS = (("reset_kernel", "reset"), ("observe_kernel", "observe"), ("replay_scan_kernel", "scan"),
        ("replay_group_scan_kernel", "group_scan"), ("replay_write_kernel", "write"))


def run(out, n, T, reps):
    import numpy as np
    import torch

    import bench
    from merging_gym import MergeVecEnv, ReplayRing, _native
    from merging_gym.policy import QNet

    env = MergeVecEnv(n, device="cuda:0", autoreset=True, final_observation=True, episode_stats=True)
    for k in range(30):
        env.step_random(1, step_idx=k)
    for _ in range(reps):
        _native.check(_native.lib.mg_reset(ctypes.byref(env.params), ctypes.byref(env._state), None,
                                           None, n, env._stream()), "mg_reset")
    obs_only = _native.Outputs(env._out.obs, None, None, None, None, None, None, None)
    for _ in range(reps):
        _native.check(_native.lib.mg_observe(ctypes.byref(env.params), ctypes.byref(env._state),
                                             ctypes.byref(obs_only), n, env._stream()), "mg_observe")
    f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    qnet = QNet.from_state_dict({k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l1/")}, device=env.device)
    obs0 = env.observe().clone()
    traj = env.rollout_qnet(T, qnet, 1234, first_step=30_000_000)
    ring = ReplayRing(1 << 24, device=env.device)
    for _ in range(2):
        ring.store_rollout(obs0, traj)
    torch.cuda.synchronize()
    c0 = ring.memory_counter
    for _ in range(reps):
        ring.store_rollout(obs0, traj)
    torch.cuda.synchronize()
    kept = (ring.memory_counter - c0) / reps
    done = int(traj["done"].sum().item())
    alg = bench.replay_algorithmic_bytes(n, T, kept, done, ring.capacity)
    os.makedirs(out, exist_ok=True)
    json.dump({"envs": n, "T": T, "reps": reps, "kept_per_store": kept, "done_rows": done,
               "algorithmic_bytes_per_store": alg}, open(os.path.join(out, "replay_workload.json"), "w"))
    print(f"replay workload: {n} envs x {T} steps, kept {kept:.0f}, algorithmic {alg / 1e9:.3f} GB", flush=True)


def load(d, counter):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if r.get("Counter_Name") != counter:
                continue
            for sub, key in KEYS:
                if sub in r["Kernel_Name"] and not (key == "scan" and "group_scan" in r["Kernel_Name"]):
                    per[key].append((int(r["Dispatch_Id"]), 1024.0 * float(r["Counter_Value"])))  # KiB
    return {k: [v for _, v in sorted(vals)] for k, vals in per.items()}


def summary(out, dest):
    wl = json.load(open(os.path.join(out, "replay_workload.json")))
    n, reps = wl["envs"], wl["reps"]
    f, w = load(os.path.join(out, "fetch"), "FETCH_SIZE"), load(os.path.join(out, "write"), "WRITE_SIZE")

    def last(tab, k):  # the timed stores are the last `reps` launches of each kernel
        v = tab.get(k, [])[-reps:]
        return sum(v) / len(v) if v else 0.0

    kern = {k: {"fetch_bytes": 2.0 * last(f, k), "write_bytes": last(w, k),
                "hbm_bytes": 2.0 * last(f, k) + last(w, k)} for _, k in KEYS}
    store = sum(kern[k]["hbm_bytes"] for k in ("scan", "group_scan", "write"))
    res = {"workload": wl, "per_launch": kern,
           "store_hbm_bytes": store, "store_algorithmic_bytes": wl["algorithmic_bytes_per_store"],
           "ratio_to_algorithmic": store / wl["algorithmic_bytes_per_store"],
           "check_reset_write_ratio": kern["reset"]["write_bytes"] / (50.0 * n),
           "check_observe_read_ratio": kern["observe"]["fetch_bytes"] / (32.0 * n),
           "rule": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md, gfx950); counters count L2 -> fabric, "
                   "so Infinity Cache hits are included",
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, tools/profile_pmc_replay.py"}
    print(json.dumps(res, indent=1))
    if dest:
        json.dump(res, open(dest, "w"), indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("run", "summary"))
    ap.add_argument("out")
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dest")
    a = ap.parse_args()
    run(a.out, a.envs, a.T, a.reps) if a.mode == "run" else summary(a.out, a.dest)
