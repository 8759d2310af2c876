"""Does a sustained matrix-core load slow the HBM-bound step kernel that follows it?

    python tools/throttle_probe.py [--load other|self|hdqn|none] [--seconds 1.5]

Times 20-launch windows of the step kernel at 2^22 envs (steady state) before the load, then
runs the chosen Q-net rollout leg for the given time, then times windows again every ~50 ms for
two seconds: a per-window µs/launch timeline (HIP events on the launch stream).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--load", default="other")
ap.add_argument("--seconds", type=float, default=1.5)
ap.add_argument("--envs", type=int, default=1 << 22)
a = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from merging_gym import MergeVecEnv  # noqa: E402
from merging_gym.policy import QNet  # noqa: E402

big = MergeVecEnv(a.envs, device="cuda:0")
k = bench.burn_in(big, 1024, 3, 0)
for _ in range(20):
    big.step_random(3, step_idx=k)
    k += 1


def window():
    global k
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        big.step_random(3, step_idx=k)
        k += 1
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 20 * 1e3


before = [round(window(), 1) for _ in range(5)]
env = MergeVecEnv(1 << 20, device="cuda:0", final_observation=False)
f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
net = lambda key: QNet.from_state_dict({kk.split("/", 1)[1]: f[kk] for kk in f.files if kk.startswith(key + "/")},  # noqa: E731
                                       device="cuda:0")
q1, q3 = net("l1"), net("l3")
kk = 5_000_000
t0 = time.perf_counter()
launches = 0
while a.load != "none" and time.perf_counter() - t0 < a.seconds:
    opp = {"other": q3, "self": "self", "none": "none"}.get(a.load, "self")
    env.rollout_qnet(16, q1, 1, opponent=opp, first_step=kk, final_observation=False, won_mask=False)
    kk += 16
    launches += 1
    if launches % 8 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
t_end = time.perf_counter()
after = []
while time.perf_counter() - t_end < 2.0:
    after.append((round((time.perf_counter() - t_end) * 1e3), round(window(), 1)))
    time.sleep(0.03)
print(json.dumps({"load": a.load, "load_launches": launches, "envs": a.envs, "before_us": before, "after_ms_us": after}))
