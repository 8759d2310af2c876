"""Workload for PMC passes on the fused Q-net rollout (rocprofv3 --pmc ...): 2^20 envs in
steady state (1200 random steps), then a few 16-step ego-only Q-net rollouts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from merging_gym import MergeVecEnv  # noqa: E402
from merging_gym.policy import QNet  # noqa: E402

env = MergeVecEnv(1 << 20, device="cuda:0", final_observation=False)
for k in range(1200):
    env.step_random(7, step_idx=k)
f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
qnet = QNet.from_state_dict({k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l1/")}, device="cuda:0")
for j in range(int(os.environ.get("QNET_LAUNCHES", "4"))):
    env.rollout_qnet(16, qnet, 7, opponent=os.environ.get("QNET_OPP", "none"), first_step=5000 + 16 * j,
                     final_observation=False, won_mask=False)
torch.cuda.synchronize()
print("ok")
