"""CPU baselines of the bench workload (BASELINE.md "CPU baseline plan"), timed on the host cores.

TEST INFRASTRUCTURE / BASELINE ONLY: bench.py runs this file as a child process (it never
touches the GPU) on rank 0 at N = 1 and reports what it prints next to the GPU line. Three
restatements of the reference step (merging_env.py:138-195), each on a bounded sample:

  c_oracle       oracle/merge_oracle.c (OpenMP, the QP solved from scratch per car-step), one
                 thread per core the process may run on (os.sched_getaffinity), Philox actions
                 for both players, autoreset -- the GPU line's workload on 16,384 envs;
  numpy          oracle/merge_numpy.py at 2^20 envs (the GPU batch): one process on one core,
                 then one process per core, each owning a contiguous shard of the 2^20 envs;
  scalar         the list-API restatement oracle.PyMergeEnv (one env, Python floats, the QP
                 solved per car-step), one process per core, >= 20,000 steps each, random
                 actions, reset on done (config 1's loop).

The process-per-core legs use min(affinity, cgroup CPU quota) processes: more processes than
the quota grants only time-share the same cores. Both counts are printed.

    python oracle/cpu_baselines.py [--seconds 6] [--envs 1048576] [--legs c_oracle,numpy,scalar]
"""

from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def cgroup_cpu_quota():
    """CPUs the cgroup grants (cpu.max quota / period, cgroup v2; cfs files, v1), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return None if q <= 0 else max(1, q // p)
    except (OSError, ValueError):
        return None


def host_cores():
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    return {"affinity": aff, "cgroup_quota": quota, "procs": min(aff, quota) if quota else aff}


def c_oracle(seconds: float, threads: int):
    import numpy as np

    import merge_oracle

    co = merge_oracle.COracle(merge_oracle.build_c_oracle())
    co.set_threads(threads)
    n = 16384
    envs = co.new_envs(n)
    co.reset(envs)
    ret_sum, counts = np.zeros((n, 3)), np.zeros((n, 6), np.uint32)
    done_steps, chunk, k = 0, 25, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        done_steps += co.rollout_random(envs, chunk, 1234, k, True, stats=(ret_sum, counts))
        k += chunk
    dt = time.perf_counter() - t0
    return {"value": done_steps / dt, "unit": "env-steps/s", "threads": threads,
            "sample": f"{n} envs x {k} autoreset steps, {dt:.1f} s"}


def _numpy_shard(args):
    n, offset, seconds, min_steps = args
    import merge_numpy as mn

    b = mn.NumpyMergeBatch(n, env_offset=offset)
    b.rollout_random(1, 1234, 0)  # first touch of every array
    k, t0 = 1, time.perf_counter()
    while k - 1 < min_steps or time.perf_counter() - t0 < seconds:
        b.rollout_random(1, 1234, k)
        k += 1
    return n * (k - 1), time.perf_counter() - t0


def numpy_leg(envs: int, procs: int, seconds: float):
    t1 = _numpy_shard((envs, 0, seconds, 2))
    out = {"one_core": {"value": t1[0] / t1[1], "unit": "env-steps/s", "procs": 1,
                        "sample": f"{envs} envs x {t1[0] // envs} steps, {t1[1]:.1f} s"}}
    if procs > 1:
        base, extra = divmod(envs, procs)
        shards, off = [], 0
        for r in range(procs):
            c = base + (1 if r < extra else 0)
            shards.append((c, off, seconds, 2))
            off += c
        with mp.get_context("fork").Pool(procs) as pool:
            res = pool.map(_numpy_shard, shards)
        steps = sum(r[0] for r in res)
        wall = max(r[1] for r in res)
        out["all_cores"] = {"value": steps / wall, "unit": "env-steps/s", "procs": procs,
                            "sample": f"{envs} envs in {procs} shards, {steps // envs} steps each "
                                      f"on average, {wall:.1f} s"}
    return out


def _scalar_proc(args):
    steps, seed = args
    import numpy as np

    import merge_oracle

    rng = np.random.default_rng(seed)
    acts = rng.integers(0, 5, (steps, 2)).tolist()
    env = merge_oracle.PyMergeEnv()
    env.reset()
    t0 = time.perf_counter()
    for a1, a2 in acts:
        if env.step(a1, a2)[2]:
            env.reset()
    return steps, time.perf_counter() - t0


def scalar_leg(procs: int, steps: int = 20000):
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_scalar_proc, [(steps, 100 + r) for r in range(procs)])
    total = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": total / wall, "unit": "env-steps/s", "procs": procs,
            "per_proc": steps / (sum(r[1] for r in res) / procs),
            "sample": f"{procs} processes x {steps} list-API steps (random actions, reset on done), "
                      f"{wall:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0, help="per leg")
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--legs", default="c_oracle,numpy,scalar")
    a = ap.parse_args()
    for v in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ.pop(v, None) if v == "OMP_NUM_THREADS" else os.environ.setdefault(v, "1")
    cores = host_cores()
    out = {"cores": cores}
    legs = a.legs.split(",")
    if "c_oracle" in legs:
        out["c_oracle"] = c_oracle(a.seconds, cores["affinity"])
    if "numpy" in legs:
        out["numpy"] = numpy_leg(a.envs, cores["procs"], a.seconds / 2)
    if "scalar" in legs:
        out["scalar"] = scalar_leg(cores["procs"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
