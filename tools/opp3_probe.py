"""Diagnostic of mg_rollout_hdqn opponent mode 3 (hdqn.py:265-268): the opponent's step-0 greedy
actions against QNet.forward of its lower net on [goal_op] + swapped state, for the ego's own
nets, byte-identical copies of them in other buffers, and different nets."""
import sys

import numpy as np
import torch

sys.path.insert(0, "merging-gym_amd")
from merging_gym import MergeVecEnv  # noqa: E402
from merging_gym.policy import NUM_GOALS, QNet  # noqa: E402


def _net(rng, in_dim, out_dim):  # as tests/test_gpu_hdqn.py (hdqn.py:41-47's initialisation)
    sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), [(200, in_dim), (100, 200), (out_dim, 100)]):
        sd[f"{name}.weight"] = rng.uniform(0, 1, (o, i)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    return sd

dev, n, seed = "cuda:0", 1000, 6
rng = np.random.default_rng(5)
msd, lsd = _net(rng, 10, NUM_GOALS), _net(rng, 11, 5)
meta, lower = QNet.from_state_dict(msd, device=dev), QNet.from_state_dict(lsd, device=dev)
osd_m, osd_l = _net(rng, 10, NUM_GOALS), _net(rng, 11, 5)
cases = {"own": (meta, lower), "copy": (QNet.from_state_dict(msd, device=dev), QNet.from_state_dict(lsd, device=dev)),
         "other": (QNet.from_state_dict(osd_m, device=dev), QNet.from_state_dict(osd_l, device=dev)),
         "other_lower_only": (meta, QNet.from_state_dict(osd_l, device=dev)),
         "other_meta_only": (QNet.from_state_dict(osd_m, device=dev), lower)}
for name, (om, ol) in cases.items():
    env = MergeVecEnv(n, device=dev, final_observation=True)
    for k in range(190):
        env.step_random(seed, opponent_random=False, step_idx=k)
    obs = env.observe().clone()
    tr = env.rollout_hdqn(4, meta, lower, seed, opponent=(om, ol), first_step=190)
    gop = tr["goal_op"][0]
    sw = torch.cat([obs[:, 5:], obs[:, :5]], dim=1)
    q = ol.forward(torch.cat([gop[:, None], sw], dim=1))
    qm = om.forward(sw)
    a2 = tr["a2"][0].to(torch.int64)
    print(f"{name:>16}: a2 == argmax {float((a2 == q.argmax(1)).float().mean()):.3f}  goal_op == meta argmax "
          f"{float((gop.to(torch.int64) == qm.argmax(1)).float().mean()):.3f}  a2 hist {torch.bincount(a2, minlength=5).tolist()}"
          f"  q row0 {q[0].tolist()}", flush=True)
