"""Workload for rocprofv3 PMC passes (run under `rocprofv3 --pmc ... -- python tools/profile_pmc.py`).

Per env count it launches, in order: `reps` x reset_kernel (writes 50 B/env: 6 f64 + 1 u16 --
the write calibration), `reps` x observe_kernel (reads 32 B/env of f64 -- the read
calibration), `reps` x step_kernel<philox> (the bench kernel), `reps` x rollout_kernel (T = 16,
the bench's rollout leg). tools/pmc_summary.py turns the counter CSVs into per-launch bytes.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, nargs="+", default=[1 << 20, 1 << 22, 1 << 23])
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()

import torch  # noqa: E402

from merging_gym import MergeVecEnv, _native  # noqa: E402

for n in args.envs:
    env = MergeVecEnv(n, device="cuda:0")
    for k in range(30):  # reach steady state (mixed episode phases)
        env.step_random(1, step_idx=k)
    torch.cuda.synchronize()
    for _ in range(args.reps):
        _native.check(_native.lib.mg_reset(ctypes.byref(env.params), ctypes.byref(env._state), None,
                                           None, n, env._stream()), "mg_reset")
    obs_only = _native.Outputs(env._out.obs, None, None, None, None, None, None, None)
    for _ in range(args.reps):
        _native.check(_native.lib.mg_observe(ctypes.byref(env.params), ctypes.byref(env._state),
                                             ctypes.byref(obs_only), n, env._stream()), "mg_observe")
    for k in range(30):
        env.step_random(1, step_idx=k)
    for k in range(args.reps):
        env.step_random(2, step_idx=k)
    for k in range(args.reps):  # the random rollout, T = 16 (its trajectory buffers allocated once)
        env.rollout_random(16, 2, first_step=1000 + 16 * k, final_observation=False, won_mask=False)
    torch.cuda.synchronize()
    print(f"envs={n} done", flush=True)
    del env
    torch.cuda.empty_cache()
