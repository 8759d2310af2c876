"""Workload for rocprofv3 --pmc passes on the compute side of the kernels (tools/pmc_valu.sh):
2^20 envs in steady state, then 8 launches each of mg_step_random, the fused random rollout
(T = 16), the config-5 Q-net rollout (ego, T = 16) and the h-DQN rollout (T = 16).
tools/valu_summary.py turns the counters into per-kernel VALU busy fractions and instruction
mixes per env-step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from merging_gym import MergeVecEnv  # noqa: E402
from merging_gym.policy import QNet  # noqa: E402

env = MergeVecEnv(1 << 20, device="cuda:0", final_observation=False)
k = bench.burn_in(env, 1024, 7, 0)
for j in range(8):
    env.step_random(7, step_idx=k)
    k += 1
for j in range(8):
    env.rollout_random(16, 7, first_step=k, final_observation=False, won_mask=False)
    k += 16
f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
qnet = QNet.from_state_dict({kk.split("/", 1)[1]: f[kk] for kk in f.files if kk.startswith("l1/")}, device="cuda:0")
for j in range(8):
    env.rollout_qnet(16, qnet, 7, first_step=k, final_observation=False, won_mask=False)
    k += 16
rng = np.random.default_rng(0)


def signed(i, o):
    """bench.py's h-DQN nets: torch.nn.Linear's signed default initialisation (hdqn.py:41-47's
    uniform(0, 1) weights pick one action for > 90 % of inputs, tests/test_hdqn_test_nets.py)"""
    sd = {}
    for name, (a, b) in zip(("fc1", "fc2", "out"), [(200, i), (100, 200), (o, 100)]):
        sd[f"{name}.weight"] = rng.uniform(-b ** -0.5, b ** -0.5, (a, b)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-b ** -0.5, b ** -0.5, a).astype(np.float32)
    return QNet.from_state_dict(sd, device="cuda:0")


meta, lower = signed(10, 3), signed(11, 5)
for j in range(8):
    env.rollout_hdqn(16, meta, lower, 7, first_step=k, final_observation=False)
    k += 16
# round 3: the other opponents of both fused policies (8 launches each): config 5 with the same net
# on the swapped observation and with another checkpoint (l3); h-DQN self-play and another
# checkpoint's nets
if os.environ.get("MG_PROFILE_ALL_OPPONENTS", "1") != "0":
    qnet3 = QNet.from_state_dict({kk.split("/", 1)[1]: f[kk] for kk in f.files if kk.startswith("l3/")}, device="cuda:0")
    for opp in ("self", qnet3):
        for j in range(8):
            env.rollout_qnet(16, qnet, 7, opponent=opp, first_step=k, final_observation=False, won_mask=False)
            k += 16

    for opp in ("self", (signed(10, 3), signed(11, 5))):
        env.hdqn_goal_op = None
        for j in range(8):
            env.rollout_hdqn(16, meta, lower, 7, opponent=opp, first_step=k, final_observation=False)
            k += 16
torch.cuda.synchronize()
print("ok")
