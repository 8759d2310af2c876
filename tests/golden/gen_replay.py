"""Golden vectors for the replay memory, from the reference's own DQN.store_transition.

Test infrastructure only: run here, in the build container, never on the GPU box. Imports
scripts/main.py from /root/reference (read-only) with the same stand-ins as gen_golden.py,
builds its DQN() (main.py:80-95: memory = np.zeros((MEMORY_CAPACITY, NUM_STATES*2+2)),
MEMORY_CAPACITY = 2000 at :17) and drives it with main.py's collection loop (:189-220): the
reference env steps, and `if env.winner is not 1: dqn.store_transition(state, action, reward,
next_state)` (:209-211). learn() is not called (it would only read the memory). Actions come
from a seeded numpy generator instead of choose_action, so the run is reproducible.

Committed: the action sequences, per-step done/stored flags, the final memory [2000, 22]
(fp64, as the reference holds it) and memory_counter. Only data is written. The same for
scripts/hdqn.py's lower-level memory (tags HL0 / HRR, run_hdqn): goal-augmented rows [2000, 24]
plus the per-step goals and intrinsic rewards that fed them.

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


def run_hdqn(hdqn_mod, env, steps, opp_random, seed):
    """hdqn.py's lower-level memory: its own HDQN() (:142-184, memory = np.zeros((2000, (NUM_STATES
    + 1) * 2 + 2)), MEMORY_CAPACITY = 2000 at :21) driven by main()'s inner loop (:280-323):
    goal_state = [goal] + state (:291), env.step, goal = upper.choose_goal(next_state) (:303),
    next_goal_state (:304), intrinsic reward 1.0 if goal == goal_status(state) (:314, the
    reference's own goal_status), lower.store_transition (:316), state = next_state (:320), and a
    fresh goal at :283 after the :322 break or an episode end. Goals and actions come from a
    seeded numpy generator instead of the meta-controller / choose_action. Goal_DQN's own memory
    rides along: extrinsic_reward += reward each step (:286, :313) and, after each :322 break or
    episode end, upper.store_transition(state, goal, extrinsic_reward, next_state) (:325, with
    state = next_state already and goal the :303 choice) into its (200, 22) memory (:75)."""
    import torch

    rng = np.random.default_rng(seed)
    lower = hdqn_mod.HDQN()
    upper = hdqn_mod.Goal_DQN()
    extrinsic = 0
    a1s = rng.integers(0, 5, steps).astype(np.int8)
    a2s = rng.integers(0, 5, steps).astype(np.int8) if opp_random else np.full(steps, -1, np.int8)
    goal_s = np.zeros(steps, np.float32)
    goal_s2 = np.zeros(steps, np.float32)
    intrinsic = np.zeros(steps, np.float32)
    done_f = np.zeros(steps, np.bool_)
    with contextlib.redirect_stdout(io.StringIO()):
        state = env.reset()
        goal = int(rng.integers(0, 3))  # :283 upper.choose_goal(state)
        for k in range(steps):
            goal_state = torch.unsqueeze(torch.FloatTensor([goal] + state), dim=0)  # :291
            a2 = None if a2s[k] < 0 else int(a2s[k])
            next_state, rewards, done, info = env.step(int(a1s[k]), a2)
            extrinsic += rewards[0]  # :311-313
            new_goal = int(rng.integers(0, 3))  # :303 upper.choose_goal(next_state)
            next_goal_state = torch.unsqueeze(torch.FloatTensor([new_goal] + next_state), dim=0)  # :304
            r_int = 1.0 if new_goal == hdqn_mod.goal_status(state) else 0.0  # :314
            lower.store_transition(goal_state, int(a1s[k]), r_int, next_goal_state)  # :316
            goal_s[k], goal_s2[k], intrinsic[k], done_f[k] = goal, new_goal, r_int, bool(done)
            state = next_state  # :320
            goal = new_goal
            if done or goal == hdqn_mod.goal_status(state):  # :322 break -> :325, then :286
                upper.store_transition(state, goal, extrinsic, next_state)
                extrinsic = 0
            if done:  # episode over: reset, then :283 picks a goal
                state = env.reset()
                goal = int(rng.integers(0, 3))
            elif goal == hdqn_mod.goal_status(state):  # :322 break, then :283 picks a fresh goal
                goal = int(rng.integers(0, 3))
    return {"a1": a1s, "a2": a2s, "done": done_f, "goal": goal_s, "next_goal": goal_s2,
            "intrinsic": intrinsic, "memory": np.asarray(lower.memory, np.float64),
            "counter": np.int64(lower.memory_counter), "capacity": np.int64(lower.memory.shape[0]),
            "meta_memory": np.asarray(upper.memory, np.float64), "meta_counter": np.int64(upper.memory_counter),
            "meta_capacity": np.int64(upper.memory.shape[0])}


def main():
    sys.path.insert(0, HERE)
    from gen_golden import load_reference_env

    env = load_reference_env()  # puts the stand-ins and /root/reference/scripts on sys.path
    with contextlib.redirect_stdout(io.StringIO()):
        import main as main_mod  # scripts/main.py (module-level gym.make uses the stand-in gym)
        import hdqn as hdqn_mod  # scripts/hdqn.py (main() runs only under __main__)
    out = {}
    for tag, opp, seed in (("L0", False, 7), ("RR", True, 8)):
        res = run(main_mod, env, 3200, opp, seed)
        out.update({f"{tag}_{k}": v for k, v in res.items()})
        print(tag, "stored", int(res["stored"].sum()), "of", len(res["stored"]),
              "episodes", int(res["done"].sum()), "counter", int(res["counter"]))
    for tag, opp, seed in (("HL0", False, 9), ("HRR", True, 10)):
        res = run_hdqn(hdqn_mod, env, 3200, opp, seed)
        out.update({f"{tag}_{k}": v for k, v in res.items()})
        print(tag, "episodes", int(res["done"].sum()), "counter", int(res["counter"]),
              "intrinsic", float(res["intrinsic"].mean()))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
