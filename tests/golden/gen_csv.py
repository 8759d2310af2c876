"""Golden CSV trajectory logs, written by the reference's own env with human_player.py's loop.

Test infrastructure only: run here, in the build container, never on the GPU box. The
reference MergeEnv is imported with gen_golden.py's stand-ins; each episode is stepped and
logged exactly as scripts/human_player.py:108-111, :178-181 does it (header row, then
`if env.winner is not 1: writer.writerow(state + [action, action_op] + rewards)`), with
seeded random actions in place of the keyboard and the opponent model. The committed
files are that writer's output (data); the actions are stored beside them.

Usage:  python tests/golden/gen_csv.py   (writes tests/golden/csv/*)
"""

from __future__ import annotations

import contextlib
import csv
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "csv")

HEADER = None  # taken from the reference run below (human_player.py:110)


def main():
    sys.path.insert(0, HERE)
    from gen_golden import load_reference_env

    env = load_reference_env()
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(99)
    actions = {}
    # (episode, opponent): the human player's opponent is always a model (an int action);
    # the last episode has the None (L0) opponent that other callers use
    for i, opp in enumerate(("int", "int", "int", "none")):
        a1 = rng.integers(0, 5, 3000)
        a2 = rng.integers(0, 5, 3000)
        filename = os.path.join(OUT, f"episode{i}")
        with contextlib.redirect_stdout(io.StringIO()):
            state = env.reset()
        done = False
        k = 0
        with open(filename, "w") as f:
            writer = csv.writer(f)
            writer.writerow(["x2 - x1", "y2 - y1", "self.state2['vel'] - self.state1['vel']",
                             "END_POINT - self.state1['pos']", "self.state1['vel']", "x1 - x2", "y1 - y2",
                             "self.state1['vel'] - self.state2['vel']", "END_POINT - self.state2['pos']",
                             "self.state2['vel']", "action1", "action2", "reward1", "reward2"])
            while not done:
                action = int(a1[k])
                action_op = int(a2[k]) if opp == "int" else None
                with contextlib.redirect_stdout(io.StringIO()):
                    next_state, rewards, done, info = env.step(action, action_op)
                if env.winner is not 1:  # noqa: F632 -- human_player.py:180 verbatim semantics
                    writer.writerow(state + [action, action_op] + rewards)
                state = next_state
                k += 1
        actions[f"ep{i}_a1"] = a1[:k].astype(np.int8)
        actions[f"ep{i}_a2"] = (a2[:k] if opp == "int" else np.full(k, -1)).astype(np.int8)
        print(filename, k, "steps", os.path.getsize(filename), "bytes")
    np.savez_compressed(os.path.join(OUT, "actions.npz"), **actions)


if __name__ == "__main__":
    main()
