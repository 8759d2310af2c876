"""Inputs and mg_qnet_forward outputs of the shipped checkpoints (l1, l3, both views) and of seeded
signed h-DQN nets, saved for the offline summation-order study (oracle.qnet_reference_blocked)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "merging-gym_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import merge_oracle as mo  # noqa: E402
from merging_gym.policy import QNet  # noqa: E402

co = mo.COracle(mo.build_c_oracle())
f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
envs = co.new_envs(8192)
co.reset(envs)
rng = np.random.default_rng(3)
obs = []
for k in range(240):
    o, *_ = co.step(envs, rng.integers(0, 5, 8192).astype(np.int8), rng.integers(0, 5, 8192).astype(np.int8), autoreset=True)
    if k % 30 == 0:
        obs.append(o.astype(np.float32))
obs = np.concatenate(obs)
out = {"obs": obs}
for key in ("l1", "l3"):
    sd = {n.split("/", 1)[1]: f[n] for n in f.files if n.startswith(key + "/")}
    qn = QNet.from_state_dict(sd, device="cuda:0")
    for swap in (0, 1):
        out[f"{key}_swap{swap}"] = qn.forward(torch.from_numpy(obs).cuda(), swap_halves=bool(swap)).cpu().numpy()
rng = np.random.default_rng(0)
for name, (i, o) in (("meta", (10, 3)), ("lower", (11, 5))):
    sd = {}
    for nm, (a, b) in zip(("fc1", "fc2", "out"), [(200, i), (100, 200), (o, 100)]):
        sd[f"{nm}.weight"] = rng.uniform(-b ** -0.5, b ** -0.5, (a, b)).astype(np.float32)
        sd[f"{nm}.bias"] = rng.uniform(-b ** -0.5, b ** -0.5, a).astype(np.float32)
    x = obs if i == 10 else np.concatenate([rng.integers(0, 3, (len(obs), 1)).astype(np.float32), obs], 1)
    out[f"{name}_x"] = x
    out[f"{name}_q"] = QNet.from_state_dict(sd, device="cuda:0").forward(torch.from_numpy(x).cuda()).cpu().numpy()
    for k, v in sd.items():
        out[f"{name}/{k}"] = v
np.savez_compressed(sys.argv[1], **out)
print("saved", sys.argv[1])
