"""Drop-in single env (config 1): per-step latency with device copies vs zero-copy pinned host
memory, and that both give identical outputs.   python tools/dropin_ab.py   (on an MI355X)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "merging-gym_amd"))

import numpy as np  # noqa: E402

from merging_gym.envs.merging_env import MergeEnv  # noqa: E402
rng = np.random.default_rng(0)
acts = rng.integers(0, 5, (3000, 2)).tolist()
res = {}
for zc in (False, True, False, True):
    env = MergeEnv(zero_copy=zc)
    env.reset()
    outs = []
    t0 = time.perf_counter()
    for a1, a2 in acts:
        o, r, d, info = env.step(a1, a2)
        outs.append((tuple(o), tuple(r), d))
        if d:
            env.reset()
    dt = time.perf_counter() - t0
    res.setdefault(zc, []).append(dt / len(acts) * 1e6)
    res[("o", zc)] = outs
print({k: v for k, v in res.items() if not isinstance(k, tuple)})
print("identical outputs:", res[("o", False)] == res[("o", True)])
