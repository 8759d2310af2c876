"""In-process A/B of libmerging_hip.so variants on the fused h-DQN acting loop (mg_rollout_hdqn,
scripts/hdqn.py:280-323) and the config-5 Q-net rollout (mg_rollout_qnet), through the package's own
API: every variant library is bound like the in-tree one (_native._load) and swapped in as
_native.lib between timed windows, so the env batch, the nets (packed once: the variants share the
ABI and the packed layout) and the stream are the same for all of them.

    python tools/ab_hdqn.py tools/variants/lib_*.so [--envs N] [--rounds R] [--launches L]

Prints the median kernel time per 16-step launch (HIP events on the launch stream) per variant and
opponent: h-DQN L0, self-play, another checkpoint's nets (read from L2).
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from merging_gym import MergeVecEnv, _native  # noqa: E402
from merging_gym.policy import NUM_GOALS, QNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--T", type=int, default=16)
    a = ap.parse_args()
    libs = {os.path.basename(p): _native._load(p) for p in a.libs}
    rng = None

    def net(i, o):  # bench.py's hdqn_leg nets: torch.nn.Linear's signed default initialisation
        nonlocal rng
        sd = {}
        for name, (r, c) in zip(("fc1", "fc2", "out"), [(200, i), (100, 200), (o, 100)]):
            sd[f"{name}.weight"] = rng.uniform(-c ** -0.5, c ** -0.5, (r, c)).astype(np.float32)
            sd[f"{name}.bias"] = rng.uniform(-c ** -0.5, c ** -0.5, r).astype(np.float32)
        return QNet.from_state_dict(sd, device="cuda")

    # every variant packs its own copies of the same nets (the packed layout may differ between them)
    nets = {}
    for name, lib in libs.items():
        _native.lib = lib
        rng = np.random.default_rng(0)
        meta, lower, meta_op, lower_op = net(10, NUM_GOALS), net(11, 5), net(10, NUM_GOALS), net(11, 5)
        nets[name] = (meta, lower, {"hdqn_L0": "none", "hdqn_self": "self", "hdqn_other": (meta_op, lower_op)})
    legs = ("hdqn_L0", "hdqn_self", "hdqn_other")
    env = MergeVecEnv(a.envs, device="cuda", final_observation=False)
    k = 1_000_000
    for _ in range(200):
        env.rollout_random(a.T, 7, first_step=k)
        k += a.T
    res = {name: {leg: [] for leg in legs} for name in libs}
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.launches)]
    for r in range(a.rounds + 1):  # round 0 warms every variant up and is not kept
        for name in (list(libs) if r % 2 == 0 else list(reversed(libs))):
            _native.lib = libs[name]
            meta, lower, opps = nets[name]
            for leg in legs:
                for j in range(a.launches):
                    ev[j][0].record()
                    env.rollout_hdqn(a.T, meta, lower, 11, opponent=opps[leg], first_step=k, final_observation=False)
                    ev[j][1].record()
                    k += a.T
                torch.cuda.synchronize()
                if r:
                    res[name][leg] += [e0.elapsed_time(e1) for e0, e1 in ev]
    for name, d in res.items():
        print(f"{name:22s} " + "   ".join(f"{leg} {statistics.median(v):6.3f} ms" for leg, v in d.items()), flush=True)


if __name__ == "__main__":
    main()
