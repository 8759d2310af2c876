"""What disturbs the 2^22 step launches after the burn-in (round 4): the
bench's clear_statistics() (three strided torch fills over the 268 MB of records, or the one
full-record pass that replaced them) or an idle gap (synchronize). After bench.py's staggered burn-in this probe times every launch from its dispatch
packet (mg_time_next_launch) in segments of 200 launches, each preceded by: nothing, a statistics
clear of either kind, or a synchronize plus 0.5 ms of host sleep. Usage: python tools/size2_probe2.py > out.json"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))


def main():
    import numpy as np
    import torch
    from merging_gym import MergeVecEnv
    from merging_gym.profiling import KernelTimer

    E = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
    env = MergeVecEnv(E, device="cuda:0", autoreset=True, final_observation=True, episode_stats=True)
    seed, k = 1, 0
    phase = torch.arange(E, device="cuda:0") % 256
    for j in range(256):
        env.step_random(seed, step_idx=k)
        env.reset(phase == j)
        k += 1
    for _ in range(1072):
        env.step_random(seed, step_idx=k)
        k += 1
    n = 200
    out = []
    for before in ("none", "clear_strided", "clear", "gap", "none", "clear_strided", "clear"):
        if before == "clear_strided":  # round 4's first clear_statistics: three fills of partial lines
            env.returns.zero_()
            env.counts.zero_()
            env.q_eval.zero_()
        if before == "clear":  # clear_statistics now: one pass over whole records
            env.clear_statistics()
        if "gap" in before:
            torch.cuda.synchronize()
            time.sleep(0.5e-3)
        timer = KernelTimer(n)
        for j in range(n):
            timer.arm(j)
            env.step_random(seed, step_idx=k)
            k += 1
        torch.cuda.synchronize()
        dur = timer.durations_ms()
        timer.close()
        us = [d * 1e3 for d in dur]
        out.append({"before": before, "first10_us": [round(x, 1) for x in us[:10]],
                    "windows_of_20_us": [round(float(np.mean(us[i:i + 20])), 1) for i in range(0, n, 20)]})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
