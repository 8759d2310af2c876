"""The driver's 20-launch window (bench.py --steps 20 --warmup 5) on the wall clock: how much of
the ~4 % between wall time and kernel time is host work between the first synchronize and the
first dispatch (round 4). Per window, after the bench's burn-in: (A) as bench.py: synchronize,
t0, event record, 20 launches, event record, synchronize; (B) the events carried by the first
and last dispatch packets themselves (mg_time_next_launch): no separate event packet ahead of the
first launch. Prints per-mode medians over interleaved windows: wall us, event / dispatch-span us.
Usage: python tools/window_probe3.py [windows]"""

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from merging_gym import MergeVecEnv, _native
    from merging_gym.profiling import KernelTimer

    nwin = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    K = 20
    env = MergeVecEnv(1 << 20, device="cuda:0", autoreset=True, final_observation=True, episode_stats=True)
    k = bench.stagger(env, 256, 1, 0, torch)
    for _ in range(1072):
        env.step_random(1, opponent_random=True, step_idx=k)
        k += 1
    step = lambda k: env.step_random(1, opponent_random=True, step_idx=k)  # noqa: E731
    res = {"A": [], "B": []}
    timer = KernelTimer(1)
    (ea, eb) = timer.events[0]
    import gc
    gc.disable()
    for w in range(nwin):
        for mode in (("A", "B") if w % 2 == 0 else ("B", "A")):
            torch.cuda.synchronize()
            if mode == "A":
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record()
                for j in range(K):
                    step(k + j)
                e1.record()
                torch.cuda.synchronize()
                wall = time.perf_counter() - t0
                span = e0.elapsed_time(e1)
            else:
                t0 = time.perf_counter()
                _native.lib.mg_time_next_launch(ea, None)
                step(k)
                for j in range(1, K - 1):
                    step(k + j)
                _native.lib.mg_time_next_launch(None, eb)
                step(k + K - 1)
                torch.cuda.synchronize()
                wall = time.perf_counter() - t0
                span = timer.durations_ms(1)[0]
            k += K
            res[mode].append((wall * 1e6, span * 1e3))
    gc.enable()
    out = {m: {"wall_us_median": statistics.median(x[0] for x in v), "span_us_median": statistics.median(x[1] for x in v),
               "wall_over_span": statistics.median(x[0] / x[1] for x in v)} for m, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
