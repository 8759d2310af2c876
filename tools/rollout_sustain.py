"""Per-launch time of 120 back-to-back fused rollouts (mg_rollout_random, 2^20 envs, T = 16),
from dispatch-recorded events: does the kernel slow down under sustained load?

    python tools/rollout_sustain.py [--lib merging-gym_amd/merging_gym/libmerging_hip.so]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import ab_kernels as ab  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=os.path.join(ROOT, "merging-gym_amd", "merging_gym", "libmerging_hip.so"))
ap.add_argument("--launches", type=int, default=120)
ap.add_argument("--qnet", action="store_true")
ap.add_argument("--vecenv", action="store_true", help="drive MergeVecEnv like bench.py's rollout leg")
a = ap.parse_args()
b = ab.Bed(ab.bind(a.lib), 1 << 20, 16)
if a.vecenv:
    from merging_gym import MergeVecEnv, _native
    env = MergeVecEnv(1 << 20, device="cuda:0", autoreset=True, final_observation=True, episode_stats=True)
    for k in range(1000):
        env.step_random(1234, opponent_random=True, step_idx=k)

    def vec_rollout(evp, k=[10_000_000]):
        _native.lib.mg_time_next_launch(*evp)
        env.rollout_random(16, 1234, first_step=k[0], final_observation=False, won_mask=False)
        k[0] += 16
else:
    for _ in range(1000):
        b.step()
if a.qnet:
    import numpy as np
    f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    b.pack_net({k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l1/")})
ev = ab.Events(a.launches)
torch.cuda.synchronize()
for j in range(a.launches):
    if a.vecenv:
        vec_rollout(ev.ev[j])
    elif a.qnet:
        b.qrollout(0, ev.ev[j])
    else:
        b.rollout(ev.ev[j])
torch.cuda.synchronize()
us = [1e3 * ev.ms(j) / 16 for j in range(a.launches)]
for j in range(0, a.launches, 10):
    print(f"launches {j:3d}-{j + 9:3d}: " + " ".join(f"{u:6.2f}" for u in us[j:j + 10]), flush=True)
