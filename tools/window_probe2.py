"""Host timeline of bench.py's driver-style timed window (K = 20 step launches), per launch.

    python tools/window_probe2.py [--spin 0|1] [--reps 6]

Mirrors bench.py's step leg (burn-in, 48 burn-in launches, 5 warm-up launches, statistics
cleared, synchronize) and then, per repetition, records perf_counter after every host launch,
after the closing event record and after the synchronize, with HIP events around the launches.
Prints per repetition: wall per launch, event time per launch, the host time of launch 0, the
mean host time of launches 1..K-1 and the tail (event record + synchronize).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--spin", type=int, default=1)
ap.add_argument("--reps", type=int, default=6)
ap.add_argument("--K", type=int, default=20)
a = ap.parse_args()
if a.spin:
    print("spin rc", ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)

import torch  # noqa: E402

import bench  # noqa: E402
from merging_gym import MergeVecEnv  # noqa: E402

torch.cuda.set_device(0)
env = MergeVecEnv(1 << 20, device="cuda:0", autoreset=True, final_observation=True, episode_stats=True)
k = bench.burn_in(env, 1024, 1234, 0)
step = lambda j: env.step_random(1234, opponent_random=True, step_idx=j)  # noqa: E731
for _ in range(48 + 5):
    step(k)
    k += 1
out = []
for rep in range(a.reps):
    env.clear_statistics()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    t0 = time.perf_counter()
    e0.record()
    for j in range(a.K):
        step(k + j)
        ts.append(time.perf_counter())
    e1.record()
    t_rec = time.perf_counter()
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    k += a.K
    ev = e0.elapsed_time(e1) * 1e3
    host = [(ts[0] - t0) * 1e6] + [(ts[i] - ts[i - 1]) * 1e6 for i in range(1, a.K)]
    out.append({"wall_us_per_launch": round((t_end - t0) * 1e6 / a.K, 2), "event_us_per_launch": round(ev / a.K, 2),
                "host_us_launch0": round(host[0], 1), "host_us_mean_rest": round(sum(host[1:]) / (a.K - 1), 2),
                "host_us_max_rest": round(max(host[1:]), 1), "tail_us": round((t_end - ts[-1]) * 1e6, 1),
                "enqueue_done_us": round((ts[-1] - t0) * 1e6, 1)})
    print(json.dumps(out[-1]), flush=True)
print(json.dumps({"spin": a.spin, "K": a.K, "reps": out}), flush=True)
