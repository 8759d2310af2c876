"""Which of bench.py's legs slows a 2^22-env batch allocated BEFORE it?

    python tools/cliff_probe.py > gpurun_out/cliff_probe.json

r03c (profiles/r03/): the 2^22 leg run after every other leg measures 0.107 ms per launch when its
env is allocated after the legs, 0.280 ms when it was allocated before them. This allocates the
bench's 2^20 env and the 2^22 env, times the 2^22 step kernel (3 windows of 20 launches, steady
state), then runs bench.py's legs one at a time with default arguments and times the 2^22 env
again after each; last, a 2^22 env allocated at that point. One JSON line per measurement.
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

sys.argv = [sys.argv[0]] + sys.argv[1:]
args = bench.parse()
K = {"k": 0}


def measure(env, tag, extra=None):
    res = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            env.step_random(args.seed, step_idx=K["k"])
            K["k"] += 1
        e1.record()
        torch.cuda.synchronize()
        res.append(round(e0.elapsed_time(e1) / 20 * 1e3, 1))
    out = {"case": tag, "us_per_launch": res, "arena_addr_hex": hex(env._arena.data_ptr()),
           "reserved_GiB": round(torch.cuda.memory_reserved() / 2**30, 2),
           "allocated_GiB": round(torch.cuda.memory_allocated() / 2**30, 2)}
    if extra:
        out.update(extra)
    print(json.dumps(out), flush=True)
    return out


def main():
    torch.cuda.set_device(0)
    E = args.envs
    env = MergeVecEnv(E, device="cuda:0", autoreset=True, final_observation=True, episode_stats=True)
    k0 = bench.burn_in(env, args.burn_in, args.seed, 0)
    for k in range(k0, k0 + 200):
        env.step_random(args.seed, opponent_random=True, step_idx=k)
    env2 = bench.size2_env(args, torch)
    K["k"] = bench.burn_in(env2, args.burn_in, args.seed, 0)
    for _ in range(200):
        env2.step_random(args.seed, step_idx=K["k"])
        K["k"] += 1
    measure(env2, "allocated first")
    legs = [("rollout", lambda: bench.rollout_leg(env, args, 1, None, torch)),
            ("replay", lambda: bench.replay_leg(env, args, torch)),
            ("qnet none", lambda: bench.qnet_leg(env, args, 1, None, torch, "none")),
            ("qnet self", lambda: bench.qnet_leg(env, args, 1, None, torch, "self")),
            ("qnet other", lambda: bench.qnet_leg(env, args, 1, None, torch, "other")),
            ("hdqn", lambda: bench.hdqn_leg(env, args, 1, None, torch))]
    for name, leg in legs:
        leg()
        torch.cuda.synchronize()
        measure(env2, f"after {name}")
    torch.cuda.empty_cache()
    measure(env2, "after empty_cache")
    env3 = bench.size2_env(args, torch)
    K["k"] = bench.burn_in(env3, args.burn_in, args.seed, 0)
    for _ in range(200):
        env3.step_random(args.seed, step_idx=K["k"])
        K["k"] += 1
    measure(env3, "allocated last")
    measure(env2, "first env again")


if __name__ == "__main__":
    main()
