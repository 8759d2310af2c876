"""Where the fixed cost of a short timed window goes (bench.py's driver run is K = 20 launches).

    python tools/window_probe.py [--spin 0|1] [--envs N]

Same env, burn-in and step as bench.py. Reports, per variant, the host wall time of the
window (barrier-free: synchronize, perf_counter, launches, synchronize, perf_counter) and the
HIP-event time on the launch stream, per launch:
  empty      : the two event records + synchronize around nothing (the window's floor)
  graph20    : K = 20 launches replayed from a HIP graph (first replay of that graph)
  graph20_2  : the same graph replayed again (graph already launched once)
  direct20   : K = 20 host launches
  graph1000  : K = 1000 from a graph
--spin 1 sets hipDeviceScheduleSpin before the HIP context exists (synchronize spins instead
of yielding).
"""
import argparse
import ctypes
import json
import re
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--spin", type=int, default=0)
ap.add_argument("--envs", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()

if a.spin:
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))
    print("hipSetDeviceFlags(spin) ->", rc, flush=True)

import torch  # noqa: E402

import bench  # noqa: E402
from merging_gym import MergeVecEnv  # noqa: E402

torch.cuda.set_device(0)
env = MergeVecEnv(a.envs, device="cuda:0", autoreset=True, final_observation=True, episode_stats=True)
k = bench.burn_in(env, 320, 1234, 0)
step = lambda j: env.step_random(1234, opponent_random=True, step_idx=j)  # noqa: E731
for _ in range(5):
    step(k)
    k += 1
torch.cuda.synchronize()


def window(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return wall * 1e6, e0.elapsed_time(e1) * 1e3


res = {"spin": a.spin, "envs": a.envs}
rows = {n: [] for n in ("empty", "graph20", "graph20_2", "graph20up", "direct20", "direct20clr", "graph1000")}
hip = ctypes.CDLL("libamdhip64.so")


def upload(g):
    """hipGraphUpload of the instantiated graph on the current stream, then synchronize."""
    ex = ctypes.c_void_p(g.raw_cuda_graph_exec())
    rc = hip.hipGraphUpload(ex, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return rc
for rep in range(a.reps):
    rows["empty"].append(window(lambda: None))
    g = bench.capture_steps(step, k, 20, torch)
    k += 20
    torch.cuda.synchronize()
    rows["graph20"].append(window(g.replay))
    rows["graph20_2"].append(window(g.replay))
    del g
    g = bench.capture_steps(step, k, 20, torch)
    k += 20
    res["upload_rc"] = upload(g)
    rows["graph20up"].append(window(g.replay))
    del g

    def direct():
        global k
        for j in range(20):
            step(k + j)
    rows["direct20"].append(window(direct))
    k += 20
    g = bench.capture_steps(step, k + 5000, 20, torch)  # bench.py's sequence: capture, clear, sync
    env.clear_statistics()
    torch.cuda.synchronize()
    rows["direct20clr"].append(window(direct))
    k += 20
    del g
    g = bench.capture_steps(step, k, 1000, torch)
    k += 1000
    torch.cuda.synchronize()
    rows["graph1000"].append(window(g.replay))
    del g
for n, v in rows.items():
    K = 1 if n == "empty" else int(re.search(r"\d+", n).group())
    res[n] = {"wall_us_per_launch": [round(w / K, 3) for w, _ in v],
              "event_us_per_launch": [round(e / K, 3) for _, e in v],
              "wall_over_event": [round(w / e, 4) if e else None for w, e in v]}
print(json.dumps(res), flush=True)
