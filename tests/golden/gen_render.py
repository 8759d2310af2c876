"""Golden UI call logs: the reference MergeEnv's own pygame UI, recorded.

Test infrastructure only: run here, in the build container, never on the GPU box. The
reference MergeEnv is imported as in gen_golden.py, except that pygame is the recording
stand-in under tests/stubs/pygame. A scripted human-experiment session (human_player.py:91-198:
intro, per episode prepare / render every step / a "Finished" render / feedback, then
finish) runs against it with seeded random actions. For every UI call the file holds the
arguments, the env attributes the call reads (state1, state2, r1_accumulate, r2_accumulate,
with their Python types) and the pygame calls it made; the resets and steps between them
are listed in order too, so the session can be replayed. The committed JSON is that data.

Usage:  python tests/golden/gen_render.py   (writes tests/golden/render_golden.json)
"""

from __future__ import annotations

import contextlib
import io
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
STUBS = os.path.join(os.path.dirname(HERE), "stubs")
OUT = os.path.join(HERE, "render_golden.json")
REFERENCE = "/root/reference"


def _plain(v):
    """JSON value keeping the reference's int / float distinction."""
    if isinstance(v, (bool, np.bool_)):
        return bool(v)
    if isinstance(v, (int, np.integer)):
        return int(v)
    return float(v)


def env_view(env):
    return {"state1": {k: _plain(v) for k, v in env.state1.items()},
            "state2": {k: _plain(v) for k, v in env.state2.items()},
            "r1_accumulate": _plain(env.r1_accumulate), "r2_accumulate": _plain(env.r2_accumulate)}


def load_reference_env_recording():
    if not os.path.isdir(REFERENCE):
        raise SystemExit(f"{REFERENCE} not found: golden vectors are generated only in the build container")
    sys.path.insert(0, HERE)
    from gen_golden import _write_shims

    shim_dir = tempfile.mkdtemp(prefix="mg_shims_")
    _write_shims(shim_dir)
    shutil.rmtree(os.path.join(shim_dir, "pygame"))  # the recording stand-in replaces it
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    # the shims first (gym etc.; their pygame is removed), so pygame resolves to the recording stub
    sys.path[:0] = [shim_dir, STUBS, os.path.join(REFERENCE, "scripts"), REFERENCE]
    import pygame  # the recording stand-in

    assert os.path.dirname(pygame.__file__) == os.path.join(STUBS, "pygame"), pygame.__file__
    pygame.clear()
    with contextlib.redirect_stdout(io.StringIO()):
        import gym
        import merging_gym  # noqa: F401  (the reference package)

        env = gym.make("merging_env-v0").unwrapped
    init_log = [list(e) for e in pygame.LOG]
    return env, pygame, init_log


def main():
    env, pygame, init_log = load_reference_env_recording()
    calls = []

    def ui(name, wait_seed=None, **kw):
        view = env_view(env)
        pygame.LOG.clear()
        if wait_seed is not None:
            np.random.seed(wait_seed)  # prepare() draws its wait from the global numpy RNG
        with contextlib.redirect_stdout(io.StringIO()):
            getattr(env, name)(**kw)
        calls.append({"call": name, "kwargs": kw, "wait_seed": wait_seed, "env": view,
                      "log": [list(e) for e in pygame.LOG]})

    rng = np.random.default_rng(7)
    tags = [None, "3", "2", "1", "Finished", "Win!", "Lose!"]
    ui("intro", player=1)
    ui("intro", player=2)
    sum_r1 = sum_r2 = 0
    for ep, opp in enumerate(("int", "none", "int")):
        player = 1 + (ep % 2)
        with contextlib.redirect_stdout(io.StringIO()):
            env.reset()
        calls.append({"call": "reset"})
        ui("prepare", wait_seed=100 + ep, player=player)
        ui("render", player=player)  # straight after reset: int positions, zero accumulators
        done, k = False, 0
        while not done and k < 400:
            a1 = int(rng.integers(0, 5))
            a2 = int(rng.integers(0, 5)) if opp == "int" else None
            with contextlib.redirect_stdout(io.StringIO()):
                _, _, done, _ = env.step(a1, a2)
            calls.append({"call": "step", "kwargs": {"action1": a1, "action2": a2}})
            k += 1
            if k % 9 == 1 or done:
                goal = [None, 0, 1, 2][int(rng.integers(0, 4))]
                goal_op = [None, 0, 1, 2][int(rng.integers(0, 4))]
                ui("render", goal=goal, goal_op=goal_op, player=player,
                   sum_r1=float(sum_r1), sum_r2=float(sum_r2),
                   tag_left=tags[int(rng.integers(0, len(tags)))],
                   tag_right=tags[int(rng.integers(0, len(tags)))],
                   last_r1=0.5, last_r2=-0.25)
        sum_r1 += env.r1_accumulate
        sum_r2 += env.r2_accumulate
        ui("render", player=player, sum_r1=sum_r1, sum_r2=sum_r2, tag_left="Finished", tag_right="Finished")
        ui("feedback", player=player)
    ui("finish", sum_r1=sum_r1, sum_r2=sum_r2, player=1)
    ui("finish", sum_r1=-3.14159, sum_r2=12, player=2)
    ui("plot", player=3)  # neither branch: only the display update

    with open(OUT, "w") as f:
        json.dump({"init": init_log, "calls": calls}, f, separators=(",", ":"))
    print(OUT, len(calls), "calls", os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
