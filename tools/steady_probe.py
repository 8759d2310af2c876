"""What finishing envs cost the one-step kernel past the Infinity Cache.

    python tools/steady_probe.py [--envs 4194304] [--steps 100]

At `--envs` (default 2^22), per variant: burn in 320 steps (fused rollouts), 5 warm steps,
then `--steps` mg_step_random launches timed with HIP events on the launch stream. Variants:
final observations on/off x episode statistics on/off, and "fresh" (no burn-in: nothing
finishes yet). Run it once per library build (MERGING_HIP_LIB picks the build).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=1 << 22)
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--tag", default=os.path.basename(os.environ.get("MERGING_HIP_LIB", "default")))
a = ap.parse_args()

import torch  # noqa: E402

import bench  # noqa: E402
from merging_gym import MergeVecEnv  # noqa: E402

res = {"tag": a.tag, "envs": a.envs}
for name, fo, st, burn in (("full", True, True, 320), ("no_final_obs", False, True, 320),
                           ("no_stats", True, False, 320), ("neither", False, False, 320),
                           ("fresh", True, True, 0), ("full_again", True, True, 320)):
    env = MergeVecEnv(a.envs, device="cuda:0", final_observation=fo, episode_stats=st)
    k = bench.burn_in(env, burn, 1234, 0)
    for _ in range(5):
        env.step_random(1234, step_idx=k)
        k += 1
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for j in range(a.steps):
        env.step_random(1234, step_idx=k + j)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.steps
    res[name] = {"us": round(us, 2), "frac": round(152 * a.envs / (us * 1e-6) / 8e12, 4)}
    del env
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
