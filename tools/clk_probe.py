"""Phase clocks of the h-DQN kernel (tools/clk_variant.py builds): per phase, the working time of the
Q-net waves (0-3) and of the env waves (4-7) from the phase start to their closing barrier, and the
phase length, averaged over blocks 0..63 and the middle phases of a 16-step launch at 2^20 envs.

    python tools/clk_probe.py tools/variants/lib_clk_*.so
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

libs = {os.path.basename(p): _native._load(p) for p in sys.argv[1:]}
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


for name, lib in libs.items():
    _native.lib = lib
    meta, lower, mop, lop = net(10, NUM_GOALS), net(11, 5), net(10, NUM_GOALS), net(11, 5)
    lib.mg_debug_clocks.argtypes = [ctypes.c_void_p]
    for leg, opp in (("L0", "none"), ("self", "self"), ("other", (mop, lop))):
        env.hdqn_goal_op = None
        for _ in range(4):
            env.rollout_hdqn(16, meta, lower, 11, opponent=opp, first_step=k, final_observation=False)
            k += 16
        torch.cuda.synchronize()
        buf = np.zeros(64 * 8 * 64 * 16, np.uint32)
        assert lib.mg_debug_clocks(buf.ctypes.data) == 0
        c = buf.reshape(64, 8, 64, 16).astype(np.int64)
        ph = range(6, 30)
        q_work = np.mean([(c[:, w, p, 1] - c[:, w, p, 0]) for w in range(4) for p in ph])
        e_work = np.mean([(c[:, w, p, 1] - c[:, w, p, 0]) for w in range(4, 8) for p in ph])
        length = np.mean([(c[:, 0, p + 1, 0] - c[:, 0, p, 0]) for p in ph])
        qmax = np.mean([np.max(c[:, 0:4, p, 1] - c[:, 0:4, p, 0], axis=1) for p in ph])
        print(f"{name:20s} {leg:5s}  phase {length:8.0f}  Q work {q_work:8.0f} (max of 4 {qmax:8.0f})  env work {e_work:8.0f}"
              "  (s_memtime cycles)", flush=True)
        # the passes' marks (tools/clk_variant.py): forward s of the phase from mark 2 + s to 8 + s
        marks = []
        for s_ in range(6):
            d = [(c[:, w, p, 8 + s_] - c[:, w, p, 2 + s_]) for w in range(4) for p in ph]
            d = np.concatenate(d)
            ok = (d > 0) & (d < 1e6) & (c[:, 0, 0, 2 + s_].max() > 0)
            if ok.mean() > 0.5:
                marks.append(f"fwd{s_} {np.median(d[ok]):6.0f} ({100 * ok.mean():.0f}%)")
        if marks:
            print("    " + "  ".join(marks), flush=True)
        buf[:] = 0
        lib.mg_debug_clocks  # noqa: B018
