"""The drop-in and device sides of the CSV trajectory logs (scripts/human_player.py:108-111, :180-181).

* The drop-in MergeEnv, logged with EpisodeCSVWriter in human_player.py's loop, reproduces
  the reference env's own files (tests/golden/csv): same rows, same int-typed field text,
  floats within 1e-9 (test_trajlog.assert_csv_equivalent).
* TrajectoryCSVLogger over batched rollouts: one file per (env, episode) with episodes cut at
  done and continued across rollouts, rows dropped exactly where the won bit is set, and every
  field parsing (as data_analysis.ipynb's read_csv does, float(row[k])) to the trajectory's
  fp32 value exactly.
"""

import csv
import os

import numpy as np
import pytest

from test_trajlog import CSV_DIR, assert_csv_equivalent

BACKENDS = ["host", pytest.param("gpu", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("ep", [0, 1, 2, 3])
def test_dropin_episode_csv_matches_reference(tmp_path, ep, backend):
    import merging_gym
    from merging_gym.trajlog import EpisodeCSVWriter

    acts = np.load(os.path.join(CSV_DIR, "actions.npz"))
    a1, a2 = acts[f"ep{ep}_a1"], acts[f"ep{ep}_a2"]
    env = merging_gym.make("merging_env-v0", backend=backend)
    state = env.reset()
    path = tmp_path / f"episode{ep}"
    with EpisodeCSVWriter(str(path)) as w:
        for k in range(len(a1)):
            action, action_op = int(a1[k]), (None if a2[k] < 0 else int(a2[k]))
            next_state, rewards, done, info = env.step(action, action_op)
            w.record(state, action, action_op, rewards, env.winner)
            state = next_state
        assert done
    assert_csv_equivalent(path.read_bytes(), open(os.path.join(CSV_DIR, f"episode{ep}"), "rb").read())


def _read_rows(path):
    with open(path, newline="") as f:
        rows = list(csv.reader(f))
    assert rows[0][0] == "x2 - x1" and len(rows[0]) == 14
    return rows[1:]


@pytest.mark.gpu
@pytest.mark.parametrize("opp", [True, False])
def test_trajectory_logger_segments_filters_and_round_trips(tmp_path, opp):
    from merging_gym import MergeVecEnv
    from merging_gym.trajlog import TrajectoryCSVLogger

    n, T, seed = 300, 100, 3
    ids = [0, 7, 64, 299]
    env = MergeVecEnv(n, device="cuda:0")
    log = TrajectoryCSVLogger(ids, str(tmp_path), tag="Formal_L1")
    expect = {i: [[]] for i in ids}  # env -> episodes -> rows (fp32 values)
    obs0 = env.observe().clone()
    for r in range(4):  # 400 steps: every env finishes at least one episode
        traj = env.rollout_random(T, seed, opponent_random=opp, first_step=r * T)
        h = {k: v.cpu().numpy() for k, v in traj.items() if v is not None}
        won = ((h["won_mask"].view(np.uint64)[:, :, None] >> np.arange(64, dtype=np.uint64)) & 1)
        won = won.reshape(T, -1)[:, :n].astype(bool)
        prev = obs0.cpu().numpy()
        for t in range(T):
            for i in ids:
                if not won[t, i]:
                    expect[i][-1].append(np.concatenate([prev[i], [h["a1"][t, i], h["a2"][t, i]], h["rew"][t, i]]))
                if h["done"][t, i]:
                    expect[i].append([])
            prev = h["obs"][t]
        log.log(obs0, traj)
        obs0 = traj["obs"][-1].clone()
    log.close()
    for i in ids:
        episodes = list(expect[i])
        if not episodes[-1] and len(episodes) > 1:  # finished on the very last step: no file yet
            n_files = sum(os.path.basename(p).startswith(f"env{i} ") for p in log.paths)
            if n_files == len(episodes) - 1:
                episodes = episodes[:-1]
        files = sorted((p for p in log.paths if os.path.basename(p).startswith(f"env{i} ")),
                       key=lambda p: int(os.path.basename(p).split()[1][7:]))
        assert len(files) == len(episodes) and len(files) >= 2, (i, len(files))
        for path, rows_exp in zip(files, episodes):
            assert path.endswith(" Formal_L1")
            rows = _read_rows(path)
            assert len(rows) == len(rows_exp), (path, len(rows), len(rows_exp))
            for got, ex in zip(rows, rows_exp):
                vals = [float(x) for x in got[:10]] + [float(got[12]), float(got[13])]
                exp_vals = list(ex[:10]) + list(ex[12:14])
                assert np.array_equal(np.float32(vals), np.float32(exp_vals)), (path, got)
                assert int(got[10]) == int(ex[10])
                assert got[11] == ("" if ex[11] < 0 else str(int(ex[11])))
