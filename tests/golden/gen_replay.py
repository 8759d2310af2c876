"""Golden vectors for the replay memory, from the reference's own DQN.store_transition.

Test infrastructure only: run here, in the build container, never on the GPU box. Imports
scripts/main.py from /root/reference (read-only) with the same stand-ins as gen_golden.py,
builds its DQN() (main.py:80-95: memory = np.zeros((MEMORY_CAPACITY, NUM_STATES*2+2)),
MEMORY_CAPACITY = 2000 at :17) and drives it with main.py's collection loop (:189-220): the
reference env steps, and `if env.winner is not 1: dqn.store_transition(state, action, reward,
next_state)` (:209-211). learn() is not called (it would only read the memory). Actions come
from a seeded numpy generator instead of choose_action, so the run is reproducible.

Committed: the action sequences, per-step done/stored flags, the final memory [2000, 22]
(fp64, as the reference holds it) and memory_counter. Only data is written.

Usage:  python tests/golden/gen_replay.py   (writes tests/golden/replay_golden.npz)
"""

from __future__ import annotations

import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "replay_golden.npz")


def run(main_mod, env, steps, opp_random, seed):
    rng = np.random.default_rng(seed)
    dqn = main_mod.DQN()
    a1s = rng.integers(0, 5, steps).astype(np.int8)
    a2s = rng.integers(0, 5, steps).astype(np.int8) if opp_random else np.full(steps, -1, np.int8)
    done_f = np.zeros(steps, np.bool_)
    stored = np.zeros(steps, np.bool_)
    with contextlib.redirect_stdout(io.StringIO()):
        state = env.reset()
        for k in range(steps):
            a2 = None if a2s[k] < 0 else int(a2s[k])
            next_state, rewards, done, info = env.step(int(a1s[k]), a2)
            reward, _ = rewards
            if env.winner is not 1:  # noqa: F632 -- main.py:209 verbatim semantics
                dqn.store_transition(state, int(a1s[k]), reward, next_state)
                stored[k] = True
            done_f[k] = bool(done)
            state = next_state
            if done:
                state = env.reset()
    return {"a1": a1s, "a2": a2s, "done": done_f, "stored": stored,
            "memory": np.asarray(dqn.memory, np.float64), "counter": np.int64(dqn.memory_counter),
            "capacity": np.int64(dqn.memory.shape[0])}


def main():
    sys.path.insert(0, HERE)
    from gen_golden import load_reference_env

    env = load_reference_env()  # puts the stand-ins and /root/reference/scripts on sys.path
    with contextlib.redirect_stdout(io.StringIO()):
        import main as main_mod  # scripts/main.py (module-level gym.make uses the stand-in gym)
    out = {}
    for tag, opp, seed in (("L0", False, 7), ("RR", True, 8)):
        res = run(main_mod, env, 3200, opp, seed)
        out.update({f"{tag}_{k}": v for k, v in res.items()})
        print(tag, "stored", int(res["stored"].sum()), "of", len(res["stored"]),
              "episodes", int(res["done"].sum()), "counter", int(res["counter"]))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
