"""Which fp32 summation the matrix cores perform: the Q-net forwards against bf16 emulations
(oracle.merge_oracle): qnet_reference (bf16 operands, one fp32 matmul: another order) and
qnet_reference_blocked (each MFMA adds the exact sum of its K products with one rounding; K blocks
of 32 for the 16x16x32 forward, 16 for the 32x32x16 one). Prints the share of bit-equal Q-values.

    python tools/mfma_order_probe.py     (GPU)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "merging-gym_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import merge_oracle as mo  # noqa: E402
from merging_gym import MergeVecEnv  # noqa: E402
from merging_gym.policy import QNet  # noqa: E402

co = mo.COracle(mo.build_c_oracle())
f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
nets = {k: {n.split("/", 1)[1]: f[n] for n in f.files if n.startswith(k + "/")} for k in ("l1", "l3")}
envs = co.new_envs(8192)
co.reset(envs)
rng = np.random.default_rng(3)
obs = []
for k in range(240):
    o, *_ = co.step(envs, rng.integers(0, 5, 8192).astype(np.int8), rng.integers(0, 5, 8192).astype(np.int8), autoreset=True)
    if k % 30 == 0:
        obs.append(o.astype(np.float32))
obs = np.concatenate(obs)
for key in ("l1", "l3"):
    for swap in (False, True):
        q = QNet.from_state_dict(nets[key], device="cuda:0").forward(torch.from_numpy(obs).cuda(), swap_halves=swap).cpu().numpy()
        line = f"mg_qnet_forward {key} swap={swap}:"
        for name, ref in (("fp32 matmul", mo.qnet_reference(nets[key], obs, swap=swap)),
                          ("blocked 32", mo.qnet_reference_blocked(nets[key], obs, swap=swap, block=32)),
                          ("blocked 16", mo.qnet_reference_blocked(nets[key], obs, swap=swap, block=16))):
            line += f"  {name} {np.mean(q == ref):.6f} equal (max |d| {np.abs(q - ref).max():.3g})"
        print(line, flush=True)
# the 32x32 forward (config 5 without a net opponent): through q_eval of single-episode envs
n, T, seed = 8192, 40, 5
for opponent in ("none", "self"):
    env = MergeVecEnv(n, device="cuda:0")
    for k in range(200):
        env.step_random(seed + 1, step_idx=k)
    env.clear_statistics()
    qnet = QNet.from_state_dict(nets["l1"], device="cuda:0")
    obs_in = env.observe().cpu().numpy().copy()
    traj = env.rollout_qnet(T, qnet, seed, opponent=opponent, first_step=777)
    a1 = traj["a1"].cpu().numpy()
    done = traj["done"].cpu().numpy()
    o = traj["obs"].cpu().numpy()
    sums = {b: np.zeros(n) for b in (16, 32)}
    for t in range(T):
        for b in (16, 32):
            q = mo.qnet_reference_blocked(nets["l1"], obs_in, block=b)
            sums[b] += np.where(done[t], q[np.arange(n), a1[t].astype(np.int64)], 0.0)
        obs_in = o[t]
    dev = env.q_eval.cpu().numpy()
    logged = done.any(0)
    print(f"config-5 q_eval ({opponent}, {int(logged.sum())} envs with an episode end):" +
          "".join(f"  blocked {b} {np.mean(dev[logged] == sums[b][logged]):.6f} equal" for b in (16, 32)), flush=True)
