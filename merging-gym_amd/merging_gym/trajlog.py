"""Trajectory CSV logs in the format of the reference's human experiments.

scripts/human_player.py:108-111 opens one CSV per episode, writes the header row below, and
for every step appends `state + [action, action_op] + rewards` unless the ego has already
won (`if env.winner is not 1`, :180-181); scripts/data/data_analysis.ipynb reads the files
back with `float(row[k])` per column.

* EpisodeCSVWriter -- that writer for the single-env drop-in loop. Fed with MergeEnv's list
  values (the reference's Python ints and floats), the file is byte-identical to the
  reference's (tests/golden/csv, written by the reference env itself).
* TrajectoryCSVLogger -- the same format streamed from batched device trajectories
  (MergeVecEnv.rollout_random / rollout_qnet dicts) for a chosen set of envs: one file per
  (env, episode), rows filtered by the trajectory's won bits, episodes cut at done and
  continued across successive rollouts. Values are the kernels' fp32 outputs written in
  their shortest round-trip form, so float(text) is the fp32 rounding of the reference's
  value; an L0 (None) opponent action is an empty field, as csv writes None.
"""

from __future__ import annotations

import csv
import os

import numpy as np

HEADER = ["x2 - x1", "y2 - y1", "self.state2['vel'] - self.state1['vel']",
          "END_POINT - self.state1['pos']", "self.state1['vel']", "x1 - x2", "y1 - y2",
          "self.state1['vel'] - self.state2['vel']", "END_POINT - self.state2['pos']",
          "self.state2['vel']", "action1", "action2", "reward1", "reward2"]  # human_player.py:110


class EpisodeCSVWriter:
    """One episode's log (human_player.py:108-111, :180-181)."""

    def __init__(self, path: str):
        self._f = open(path, "w")
        self._w = csv.writer(self._f)
        self._w.writerow(HEADER)
        self.rows = 0

    def record(self, state, action, action_op, rewards, winner) -> bool:
        """Log the step taken from `state` unless the ego has won (winner after the step)."""
        if winner == 1:
            return False
        self._w.writerow(list(state) + [action, action_op] + list(rewards))
        self.rows += 1
        return True

    def close(self):
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _fmt32(x) -> str:
    return repr(float(x)) if np.isnan(x) else np.format_float_positional(np.float32(x), unique=True, trim="0")


class TrajectoryCSVLogger:
    """Per-episode CSV files for envs `env_ids` of a MergeVecEnv, from its trajectories.

        log = TrajectoryCSVLogger([0, 17, 4095], "log/run1", tag="Formal_L1")
        obs0 = env.observe().clone()
        traj = env.rollout_qnet(16, qnet, seed)
        log.log(obs0, traj)              # call again with the next rollout; episodes continue
        log.close()

    File name: f"env{i} episode{k} {tag}" (human_player.py:107: "episode" + str(i) + " " + load_path).
    Only the selected envs' rows are copied to the host.
    """

    def __init__(self, env_ids, out_dir: str, tag: str = ""):
        self.env_ids = [int(i) for i in env_ids]
        self.out_dir = out_dir
        self.tag = tag
        os.makedirs(out_dir, exist_ok=True)
        self._open = {}     # env -> (file, writer)
        self._episode = {i: 0 for i in self.env_ids}
        self.paths = []

    def _writer(self, i):
        if i not in self._open:
            name = f"env{i} episode{self._episode[i]}" + (f" {self.tag}" if self.tag else "")
            path = os.path.join(self.out_dir, name)
            f = open(path, "w", newline="")
            w = csv.writer(f)
            w.writerow(HEADER)
            self._open[i] = (f, w)
            self.paths.append(path)
        return self._open[i][1]

    def log(self, obs_first, traj):
        import torch

        if traj.get("won_mask") is None:
            raise ValueError("the rollout has no won_mask (human_player.py:180's filter needs it): "
                             "roll out with won_mask=True")

        ids = torch.as_tensor(self.env_ids, dtype=torch.long, device=traj["obs"].device)
        sel = lambda t: t.index_select(1, ids).cpu().numpy()  # noqa: E731  [T, k, ...]
        obs = sel(traj["obs"])
        a1, a2 = sel(traj["a1"]), sel(traj["a2"])
        rew = sel(traj["rew"])
        done = sel(traj["done"]).astype(bool)
        words = traj["won_mask"].cpu().numpy().view(np.uint64)
        first = obs_first.index_select(0, ids).cpu().numpy()
        T = obs.shape[0]
        for j, i in enumerate(self.env_ids):
            state = first[j]
            for t in range(T):
                w = self._writer(i)
                won = (int(words[t, i >> 6]) >> (i & 63)) & 1
                if not won:
                    w.writerow([_fmt32(v) for v in state] + [int(a1[t, j]), "" if a2[t, j] < 0 else int(a2[t, j])]
                               + [_fmt32(rew[t, j, 0]), _fmt32(rew[t, j, 1])])
                if done[t, j]:
                    f, _ = self._open.pop(i)
                    f.close()
                    self._episode[i] += 1
                state = obs[t, j]  # autoreset: the next episode starts from the reset observation

    def close(self):
        for f, _ in self._open.values():
            f.close()
        self._open.clear()
