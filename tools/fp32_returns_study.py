"""Would fp32 returns meet the north_star bar?

The step kernel keeps r1_accumulate / r2_accumulate (merging_env.py:191-192) as fp64, 16 of its
152 bytes per env-step (SURVEY.md 8(d) counts 136 with fp32 returns). This runs the NumPy
restatement (oracle/merge_numpy.py, the reference's fp64 step) over many episodes -- random play,
slow-ego play, and constant-brake episodes that run to the 2,501-step timeout -- and accumulates
each env's rewards three ways beside the fp64 sum the reference keeps:
  fp32       ret = fl32(ret + fl32(r))               (4 B per return)
  kahan32    fp32 sum + fp32 compensation            (8 B per return: no saving over fp64)
  fp32+f64ep fp32 running sum, the episode's total re-added in fp64 at its end -- not
             computable: the fp64 terms are gone by then, so this is the fp32 column
At each episode end it compares with the fp64 sum: relative error, and failures of the
north_star bar (rtol 1e-5; also numpy's allclose rtol 1e-5 / atol 1e-5), and whether the
statistics record (a sum of per-episode returns) could stay bit-exact (it cannot with any fp32 form).

    python tools/fp32_returns_study.py [--envs 65536 --steps 3000] > profiles/r03/fp32_returns.json
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import merge_numpy as mn  # noqa: E402


def run(n, steps, policy, seed):
    rng = np.random.default_rng(seed)
    nb = mn.NumpyMergeBatch(n)
    r64 = np.zeros((n, 2))
    r32 = np.zeros((n, 2), np.float32)
    k32 = np.zeros((n, 2), np.float32)  # Kahan sum
    c32 = np.zeros((n, 2), np.float32)  # Kahan compensation
    rel, rel_k, lens, fails, fails_ac, exact = [], [], [], 0, 0, 0
    for k in range(steps):
        if policy == "random":
            a1, a2 = rng.integers(0, 5, n), rng.integers(0, 5, n)
        elif policy == "slow":
            a1, a2 = rng.choice(5, n, p=[0.6, 0.1, 0.1, 0.1, 0.1]), rng.integers(-1, 5, n)
        else:  # brake: ego action 0, opponent L0 -- every episode runs to the 2,501-step timeout
            a1, a2 = np.zeros(n, np.int64), np.full(n, -1)
        steps_before = nb.steps.copy()
        _, rew, done, _ = nb.step(a1, a2)
        r64 += rew
        r32 = (r32 + rew.astype(np.float32)).astype(np.float32)
        y = (rew.astype(np.float32) - c32).astype(np.float32)
        t = (k32 + y).astype(np.float32)
        c32 = ((t - k32).astype(np.float32) - y).astype(np.float32)
        k32 = t
        if done.any():
            d = done
            ref = r64[d]
            e = np.abs(r32[d].astype(np.float64) - ref) / np.maximum(np.abs(ref), 1e-300)
            ek = np.abs(k32[d].astype(np.float64) - ref) / np.maximum(np.abs(ref), 1e-300)
            rel.append(e.max(axis=1))
            rel_k.append(ek.max(axis=1))
            lens.append(steps_before[d] + 1)
            fails += int((e > 1e-5).any(axis=1).sum())
            fails_ac += int((~np.isclose(r32[d].astype(np.float64), ref, rtol=1e-5, atol=1e-5)).any(axis=1).sum())
            exact += int((r32[d].astype(np.float64) == ref).all(axis=1).sum())
            r64[d] = 0.0
            r32[d] = 0.0
            k32[d] = 0.0
            c32[d] = 0.0
    rel = np.concatenate(rel) if rel else np.zeros(0)
    rel_k = np.concatenate(rel_k) if rel_k else np.zeros(0)
    lens = np.concatenate(lens) if lens else np.zeros(0, np.int64)
    long = lens >= 2000
    return {"policy": policy, "envs": n, "steps": steps, "episodes": int(len(rel)),
            "mean_length": float(lens.mean()) if len(lens) else None, "episodes_ge_2000_steps": int(long.sum()),
            "fp32_rel_err_max": float(rel.max()) if len(rel) else None,
            "fp32_rel_err_p99": float(np.quantile(rel, 0.99)) if len(rel) else None,
            "fp32_rel_err_max_long": float(rel[long].max()) if long.any() else None,
            "fp32_fail_rtol_1e-5": fails, "fp32_fail_allclose_1e-5": fails_ac,
            "fp32_bit_exact_episodes": exact,
            "kahan32_rel_err_max": float(rel_k.max()) if len(rel_k) else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=3000)
    args = ap.parse_args()
    out = {"study": "fp32 vs fp64 r_accumulate over whole episodes (oracle/merge_numpy.py step)",
           "bar": "north_star: float state / reward within 1e-5 (fp32)",
           "runs": [run(args.envs, args.steps, p, s) for p, s in (("random", 1), ("slow", 2), ("brake", 3))]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
