"""Segment times of the h-DQN Q-net waves' phase (tools/clk_variant.py hnow builds): medians over
blocks 0..63, waves 0-3 and the middle phases of 16-step launches at 2^20 envs, in s_memtime cycles,
between consecutive marks 0 (phase start) 2 8 3 9 6 12 7 13 1 (closing barrier).

    python tools/clk_segments.py tools/variants/lib_clk_hnow.so
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from merging_gym import MergeVecEnv, _native  # noqa: E402
from merging_gym.policy import NUM_GOALS, QNet  # noqa: E402

NAMES = {(0, 2): "meta inputs", (2, 8): "meta forward", (8, 3): "goal logic", (3, 9): "opponent meta pass",
         (9, 6): "goal outputs", (6, 12): "lower forward", (12, 7): "lower scatter + opp inputs",
         (7, 13): "opponent lower forward", (13, 1): "to the barrier"}
ORDER = [0, 2, 8, 3, 9, 6, 12, 7, 13, 1]
lib = _native._load(sys.argv[1])
_native.lib = lib
lib.mg_debug_clocks.argtypes = [ctypes.c_void_p]
env = MergeVecEnv(1 << 20, device="cuda", final_observation=False)
k = 1_000_000
for _ in range(100):
    env.rollout_random(16, 7, first_step=k)
    k += 16
rng = np.random.default_rng(0)


def net(i, o):
    sd = {}
    for name, (r, c) in zip(("fc1", "fc2", "out"), [(200, i), (100, 200), (o, 100)]):
        sd[f"{name}.weight"] = rng.uniform(-c ** -0.5, c ** -0.5, (r, c)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-c ** -0.5, c ** -0.5, r).astype(np.float32)
    return QNet.from_state_dict(sd, device="cuda")


meta, lower, mop, lop = net(10, NUM_GOALS), net(11, 5), net(10, NUM_GOALS), net(11, 5)
for leg, opp in (("L0", "none"), ("self", "self"), ("other", (mop, lop))):
    env.hdqn_goal_op = None
    for _ in range(4):
        env.rollout_hdqn(16, meta, lower, 11, opponent=opp, first_step=k, final_observation=False)
        k += 16
    torch.cuda.synchronize()
    buf = np.zeros(64 * 8 * 64 * 16, np.uint32)
    assert lib.mg_debug_clocks(buf.ctypes.data) == 0
    c = buf.reshape(64, 8, 64, 16).astype(np.int64)[:, :4, 6:30, :]  # blocks, Q waves, middle phases
    marks = [m for m in ORDER if (c[..., m] > 0).mean() > 0.5]
    out = []
    for a, b in zip(marks, marks[1:]):
        d = (c[..., b] - c[..., a]).ravel()
        d = d[(d >= 0) & (d < 1e6)]
        out.append(f"{NAMES.get((a, b), f'{a}->{b}')} {np.median(d):.0f}")
    tot = np.median((c[..., 1] - c[..., 0]).ravel())
    print(f"{leg:6s} Q work {tot:.0f}: " + "; ".join(out), flush=True)
