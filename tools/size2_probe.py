"""Why the first timed window of bench.py's 2^22 leg runs slow.

The rocprofv3 kernel trace of the r04a bench (profiles/r04/size2_trace_r04a.json) shows no gap
between the 2^22 step dispatches and no single long dispatch: per-launch durations rise and fall
smoothly over ~40 launches (101 -> 119 -> 103 us around the rehearsal / first window), as they do
in humps all through the burn-in. Hypothesis: the per-launch cost follows the number of envs that
finish in it (a finishing env's 64-byte statistics read-modify-write and 40-byte final observation
miss to DRAM past the Infinity Cache), and the finishing rate still oscillates because every env
started its first episode at the same step. This probe times each launch from its dispatch packet
(mg_time_next_launch) beside its finish count, after bench.py's burn-in ("plain") and after a
burn-in whose first 256 launches reset one 256th of the envs each ("staggered": uniform episode
phases). Usage: python tools/size2_probe.py [envs] > out.json"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))


def run(mode, E, torch, launches=240):
    from merging_gym import MergeVecEnv
    from merging_gym.profiling import KernelTimer

    env = MergeVecEnv(E, device="cuda:0", autoreset=True, final_observation=True, episode_stats=True)
    seed, k = 1, 0
    if mode == "staggered":  # env i restarts at launch i % 256: first-episode phases spread over 256 steps
        phase = torch.arange(E, device="cuda:0") % 256
        for j in range(256):
            env.step_random(seed, step_idx=k)
            env.reset(phase == j)
            k += 1
    for _ in range(1072):  # bench.py's burn-in for this leg: 1,072 single launches (--burn-in 0)
        env.step_random(seed, step_idx=k)
        k += 1
    timer = KernelTimer(launches)
    done = torch.zeros(launches, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    for j in range(launches):
        timer.arm(j)
        env.step_random(seed, step_idx=k)
        done[j] = env.done.sum()
        k += 1
    torch.cuda.synchronize()
    dur = [round(d * 1e3, 1) for d in timer.durations_ms()]
    timer.close()
    fin = done.cpu().tolist()
    import numpy as np

    corr = float(np.corrcoef(dur, fin)[0, 1])
    fit = np.polyfit(fin, dur, 1)
    return {"mode": mode, "envs": E, "dispatch_us": dur, "finished": fin,
            "windows_of_20_us": [round(float(np.mean(dur[i:i + 20])), 1) for i in range(0, launches, 20)],
            "corr_duration_finished": corr, "us_per_1000_finishes": float(fit[0]) * 1e3,
            "us_at_zero_finishes": float(fit[1])}


def main():
    import torch

    E = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
    out = [run(m, E, torch) for m in ("plain", "staggered")]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
