"""Does where a MergeVecEnv's arena lands change the step kernel's speed?

    python tools/alloc_probe.py

Times the step kernel at 2^22 envs (20-launch windows, steady state) for an env allocated
(a) first in the process, (b) after allocating and freeing gigabytes of other tensors the way
bench.py's legs do (trajectories of 2^20 x 16 steps, a 2^24 x 24 goal ring), without and with
torch.cuda.empty_cache(). Prints each case's µs per launch and the arena's address / alignment.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from merging_gym import MergeVecEnv  # noqa: E402


def measure(tag):
    env = MergeVecEnv(1 << 22, device="cuda:0")
    k = bench.burn_in(env, 1024, 3, 0)
    for _ in range(20):
        env.step_random(3, step_idx=k)
        k += 1
    res = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            env.step_random(3, step_idx=k)
            k += 1
        e1.record()
        torch.cuda.synchronize()
        res.append(round(e0.elapsed_time(e1) / 20 * 1e3, 1))
    addr = env._arena.data_ptr()
    out = {"case": tag, "us_per_launch": res, "arena_addr_hex": hex(addr), "arena_2MiB_aligned": addr % (2 << 20) == 0,
           "arena_bytes": env._arena.numel()}
    print(json.dumps(out), flush=True)
    del env
    return out


def churn(keep):
    """bench.py-like traffic: 2^20-env trajectory buffers (some kept alive) and a 1.6 GB ring."""
    n, T = 1 << 20, 16
    for _ in range(3):
        keep.append(torch.empty((T, n, 10), device="cuda:0"))
        keep.append(torch.empty((T, n, 4), dtype=torch.uint8, device="cuda:0"))
        tmp = torch.empty((1 << 24, 24), device="cuda:0")
        tmp.fill_(1.0)
        del tmp
        keep.append(torch.empty((T, n, 2), device="cuda:0"))


def qnet_load(opponent_key):
    """bench.py's Q-net legs on a 2^20-env batch: 50 launches of rollout_qnet."""
    import numpy as np

    from merging_gym.policy import QNet

    f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    net = lambda key: QNet.from_state_dict({kk.split("/", 1)[1]: f[kk] for kk in f.files  # noqa: E731
                                            if kk.startswith(key + "/")}, device="cuda:0")
    env = MergeVecEnv(1 << 20, device="cuda:0", final_observation=False)
    q1 = net("l1")
    opp = net("l3") if opponent_key == "other" else opponent_key
    for j in range(50):
        env.rollout_qnet(16, q1, 1, opponent=opp, first_step=1000 + 16 * j, final_observation=False, won_mask=False)
    torch.cuda.synchronize()
    return env


mode = sys.argv[1] if len(sys.argv) > 1 else "churn"
results = [measure("first allocation")]
if mode == "churn":
    keep = []
    churn(keep)
    results.append(measure("after churn, no empty_cache"))
    torch.cuda.empty_cache()
    results.append(measure("after churn + empty_cache"))
    churn(keep)
    torch.cuda.empty_cache()
    results.append(measure("after 2x churn + empty_cache"))
else:  # after the Q-net leg with opponent `mode` (none / self / other), its env kept alive
    keep = qnet_load(mode)
    results.append(measure(f"after rollout_qnet opponent={mode}"))
    results.append(measure(f"again after rollout_qnet opponent={mode}"))
print(json.dumps({"results": results}))
