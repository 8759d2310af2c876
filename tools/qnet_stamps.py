"""Phase clocks of the config-5 kernel (diagnostic build with -DMG_QNET_STAMPS=1).

    MERGING_HIP_LIB=tools/variants/lib_stamps.so python tools/qnet_stamps.py [--opp none|self]

2^20 envs burned in, then 8 ego-only (or self-play) 16-step rollouts; prints, per role, the mean
shader-clock cycles per wave per phase spent working and waiting at the phase barrier, and the
in-kernel clock (s_memtime / s_memrealtime at 100 MHz).
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--opp", default="none")
ap.add_argument("--launches", type=int, default=8)
a = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from merging_gym import MergeVecEnv, _native  # noqa: E402
from merging_gym.policy import QNet  # noqa: E402

env = MergeVecEnv(1 << 20, device="cuda:0", final_observation=False)
bench.burn_in(env, 1024, 7, 0)
f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
qnet = QNet.from_state_dict({k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l1/")}, device="cuda:0")
out = (ctypes.c_ulonglong * 8)()
for j in range(4):
    env.rollout_qnet(16, qnet, 7, opponent=a.opp, first_step=5000 + 16 * j, final_observation=False, won_mask=False)
torch.cuda.synchronize()
_native.lib.mg_debug_qstamps(out)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for j in range(a.launches):
    env.rollout_qnet(16, qnet, 7, opponent=a.opp, first_step=6000 + 16 * j, final_observation=False, won_mask=False)
e1.record()
torch.cuda.synchronize()
assert _native.lib.mg_debug_qstamps(out) == 0
v = list(out)
wave_phases = v[4] / 4.0  # Q-net waves counted: 4 per block, so / 4 = block-phases; both roles have 4 waves
res = {"opp": a.opp, "us_per_step": e0.elapsed_time(e1) * 1e3 / (16 * a.launches),
       "q_work_cyc_per_phase": v[0] / v[4], "q_wait_cyc_per_phase": v[1] / v[4],
       "env_work_cyc_per_phase": v[2] / v[4], "env_wait_cyc_per_phase": v[3] / v[4],
       "clock_ghz": v[5] / v[6] * 0.1 if v[6] else None, "raw": v}
print(json.dumps(res), flush=True)
