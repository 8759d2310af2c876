"""Is the 2^22-env step kernel's speed a property of where its arena lands?

    python tools/placement_probe.py [count] > gpurun_out/placement_probe.json

Allocates `count` (default 8) bench-shaped 2^22-env batches one after another, all kept alive,
burns each in, then times the step kernel on each (3 windows of 20 launches, twice round the
list). A slow batch on both rounds, beside fast ones, points at placement; all slow or all
fast at the process's state. One JSON line per batch and round.
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


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.cuda.set_device(0)
    envs, ks = [], []
    for _ in range(count):
        env = MergeVecEnv(1 << 22, device="cuda:0", autoreset=True, final_observation=True, episode_stats=True)
        k = bench.burn_in(env, 1024, 1234, 0)
        for _ in range(100):
            env.step_random(1234, step_idx=k)
            k += 1
        envs.append(env)
        ks.append(k)
    torch.cuda.synchronize()
    for rnd in range(2):
        for i, env in enumerate(envs):
            res = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(20):
                    env.step_random(1234, step_idx=ks[i])
                    ks[i] += 1
                e1.record()
                torch.cuda.synchronize()
                res.append(round(e0.elapsed_time(e1) / 20 * 1e3, 1))
            a = env._arena.data_ptr()
            print(json.dumps({"round": rnd, "batch": i, "us_per_launch": res, "arena_addr_hex": hex(a),
                              "arena_mod_2MiB": a % (2 << 20), "stats_addr_hex": hex(env._ep_stats.data_ptr())}),
                  flush=True)


if __name__ == "__main__":
    main()
