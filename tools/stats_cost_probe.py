"""What do the in-kernel episode statistics cost the step kernel? (round 3: 64-byte record)

    python tools/stats_cost_probe.py [envs]

Two bench-shaped batches, one with episode_stats=True and one without, burned in to the steady
state, then timed in interleaved 100-launch windows (HIP events on the launch stream), 6 rounds.
Prints µs per launch per window and the medians.
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from merging_gym import MergeVecEnv  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    envs = {}
    ks = {}
    for tag, st in (("stats", True), ("nostats", False)):
        env = MergeVecEnv(n, device="cuda:0", autoreset=True, final_observation=True, episode_stats=st)
        k = bench.burn_in(env, 0, 1234, 0)
        for _ in range(1072):
            env.step_random(1234, opponent_random=True, step_idx=k)
            k += 1
        envs[tag], ks[tag] = env, k
    res = {t: [] for t in envs}
    for rnd in range(6):
        for tag, env in envs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(100):
                env.step_random(1234, opponent_random=True, step_idx=ks[tag])
                ks[tag] += 1
            e1.record()
            torch.cuda.synchronize()
            res[tag].append(round(e0.elapsed_time(e1) / 100 * 1e3, 2))
    out = {"envs": n, "us_per_launch": res, "median": {t: statistics.median(v) for t, v in res.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
