"""Workload for rocprofv3 --pmc comparisons of library variants on the policy kernels: 2^20 envs,
then 6 launches (T = 16) each of the config-5 rollout with the self-play opponent and the h-DQN
rollout with the self-play opponent. The library is MERGING_HIP_LIB (default: the in-tree one).

    MERGING_HIP_LIB=tools/variants/lib_x.so rocprofv3 --pmc ... -- python tools/profile_policy.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from merging_gym import MergeVecEnv  # noqa: E402
from merging_gym.policy import NUM_GOALS, QNet  # noqa: E402

env = MergeVecEnv(1 << 20, device="cuda:0", final_observation=False)
k = bench.burn_in(env, 512, 7, 0)
f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
qnet = QNet.from_state_dict({kk.split("/", 1)[1]: f[kk] for kk in f.files if kk.startswith("l1/")}, device="cuda:0")
for j in range(6):
    env.rollout_qnet(16, qnet, 7, opponent="self", first_step=k, final_observation=False, won_mask=False)
    k += 16
rng = np.random.default_rng(0)


def net(i, o):
    sd = {}
    for name, (a, b) in zip(("fc1", "fc2", "out"), [(200, i), (100, 200), (o, 100)]):
        sd[f"{name}.weight"] = rng.uniform(-b ** -0.5, b ** -0.5, (a, b)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-b ** -0.5, b ** -0.5, a).astype(np.float32)
    return QNet.from_state_dict(sd, device="cuda:0")


meta, lower = net(10, NUM_GOALS), net(11, 5)
for j in range(6):
    env.rollout_hdqn(16, meta, lower, 7, opponent="self", first_step=k, final_observation=False)
    k += 16
import torch  # noqa: E402

torch.cuda.synchronize()
print("ok")
