"""Does the relative placement of the SoA arrays matter at large batches? mg_step_random at n envs
with the state / output arrays as separate torch allocations vs carved from one buffer with a
per-array stagger (bytes added between consecutive arrays).

    python tools/stagger_probe.py --envs 8388608 --stagger 0 4160 65600
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from merging_gym import _native as nat  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=1 << 23)
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--stagger", type=int, nargs="+", default=[-1, 0, 4160, 65600])
ap.add_argument("--stats", action="store_true", help="episode statistics on (as bench.py)")
ap.add_argument("--warm", type=int, default=30, help="untimed steps first (1000: steady state, episodes ending)")
ap.add_argument("--no-autoreset", action="store_true")
a = ap.parse_args()
n = a.envs
# (name, bytes per env, dtype)
ARR = [("p1", 8, torch.float64), ("v1", 8, torch.float64), ("p2", 8, torch.float64), ("v2", 8, torch.float64),
       ("ret1", 8, torch.float64), ("ret2", 8, torch.float64), ("tf", 2, torch.int16), ("obs", 40, torch.float32),
       ("rew", 8, torch.float32), ("done", 1, torch.uint8), ("coll", 1, torch.uint8), ("a1", 1, torch.int8),
       ("a2", 1, torch.int8), ("fobs", 40, torch.float32)]


def arrays(stagger):
    if stagger < 0:  # separate allocations (what MergeVecEnv does)
        return {k: torch.empty(n * b // torch.tensor([], dtype=dt).element_size(), dtype=dt, device="cuda")
                for k, b, dt in ARR}, None
    total = sum(n * b + stagger + 256 for _, b, _ in ARR)
    flat = torch.empty(total, dtype=torch.uint8, device="cuda")
    out, off = {}, 0
    for k, b, dt in ARR:
        nbytes = n * b
        out[k] = flat[off:off + nbytes].view(dt)
        off += nbytes + stagger
        off = (off + 255) // 256 * 256
    return out, flat


def run(stagger):
    t, keep = arrays(stagger)
    p = nat.default_params()
    p.angle0 = float(np.arctan2(1000, 30000))
    ptr = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    st = nat.State(*(ptr(t[k]) for k in ("p1", "v1", "p2", "v2", "ret1", "ret2", "tf")))
    out = nat.Outputs(ptr(t["obs"]), ptr(t["rew"]), ptr(t["done"]), ptr(t["coll"]), None, ptr(t["fobs"]), None,
                      None, None)
    if a.stats:
        keep_stats = torch.zeros((n, 4), dtype=torch.float64, device="cuda")  # mg_episode_stats [n]
        stats = nat.Stats(ptr(keep_stats))
    else:
        stats = nat.Stats()
    s = torch.cuda.current_stream().cuda_stream
    assert nat.lib.mg_reset(ctypes.byref(p), ctypes.byref(st), None, None, n, s) == 0

    def step(k):
        rc = nat.lib.mg_step_random(ctypes.byref(p), ctypes.byref(st), ptr(t["a1"]), ptr(t["a2"]), ctypes.byref(out),
                                    ctypes.byref(stats), n, 0, 5, k, 1, 0 if a.no_autoreset else nat.AUTORESET, s)
        assert rc == 0

    for k in range(a.warm):
        step(k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for k in range(a.steps):
        step(a.warm + k)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.steps * 1e3
    starts = [t[k].data_ptr() for k, _, _ in ARR[:7]]
    print(f"envs {n} warm {a.warm} stats {int(a.stats)} stagger {stagger:6d}: {us:8.2f} us/step  {152 * n / us / 1e6:5.2f} TB/s  "
          f"state array starts mod 2 MiB: {[hex(x % (1 << 21)) for x in starts]}", flush=True)
    del t, keep


for sg in a.stagger:
    run(sg)
