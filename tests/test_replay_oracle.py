"""The replay-memory oracle (oracle/merge_oracle.py replay_store) against the reference's own
DQN.store_transition run (tests/golden/replay_golden.npz, made by gen_replay.py from
scripts/main.py:115-119 under the :209 filter), and against a literal per-transition loop."""

import os

import numpy as np
import pytest

import merge_oracle as mo
from conftest import ROOT

REPLAY = os.path.join(ROOT, "tests", "golden", "replay_golden.npz")


@pytest.fixture(scope="module")
def replay_golden():
    return np.load(REPLAY)


def _oracle_episode_run(coracle, a1, a2):
    """Single env, T steps, autoreset: the [T, 1, ...] arrays a batched store consumes."""
    T = len(a1)
    envs = coracle.new_envs(1)
    obs0 = coracle.reset(envs).astype(np.float32)
    obs = np.empty((T, 1, 10), np.float32)
    fobs = np.full((T, 1, 10), np.nan, np.float32)
    rew = np.empty((T, 1, 2), np.float32)
    done = np.empty((T, 1), np.uint8)
    won = np.empty((T, 1), bool)
    for t in range(T):
        o, r, d, _, fo, w, err = mo.step_with_won(coracle, envs, a1[t:t + 1], None if a2[t] < 0 else a2[t:t + 1])
        assert err == 0
        obs[t], rew[t], done[t], won[t], fobs[t] = o, r, d, w, fo
    return obs0, obs, fobs, rew, done, won


@pytest.mark.parametrize("tag", ["L0", "RR"])
def test_oracle_store_reproduces_reference_memory(coracle, replay_golden, tag):
    g = {k.split("_", 1)[1]: replay_golden[k] for k in replay_golden.files if k.startswith(tag + "_")}
    cap = int(g["capacity"])
    obs0, obs, fobs, rew, done, won = _oracle_episode_run(coracle, g["a1"], g["a2"])
    np.testing.assert_array_equal(done[:, 0].astype(bool), g["done"])
    np.testing.assert_array_equal(~won[:, 0], g["stored"])  # main.py:209
    mem = np.zeros((cap, 22), np.float32)
    counter = mo.replay_store(mem, 0, obs0, obs, g["a1"][:, None], rew, done, fobs, won)
    assert counter == int(g["counter"]) > cap  # the ring wrapped
    ref = g["memory"].astype(np.float32)  # learn() reads it through torch.FloatTensor
    np.testing.assert_array_equal(mem, ref)


@pytest.mark.parametrize("tag", ["HL0", "HRR"])
def test_oracle_goal_store_reproduces_hdqn_memory(coracle, replay_golden, tag):
    """hdqn.py's lower-level memory (HDQN.store_transition :180-184 on goal states [goal] + state,
    intrinsic reward :314, every transition stored :316): the reference's own run, recorded by
    gen_replay.run_hdqn, equals the oracle's goal rows bit for bit (the reference's rows are
    torch.FloatTensor values, i.e. fp32)."""
    g = {k[len(tag) + 1:]: replay_golden[k] for k in replay_golden.files if k.startswith(tag + "_")}
    cap = int(g["capacity"])
    obs0, obs, fobs, rew, done, won = _oracle_episode_run(coracle, g["a1"], g["a2"])
    np.testing.assert_array_equal(done[:, 0].astype(bool), g["done"])
    mem = np.zeros((cap, 24), np.float32)
    counter = mo.replay_store(mem, 0, obs0, obs, g["a1"][:, None], rew, done, fobs, won, skip_ego_won=False,
                              goal=g["goal"][:, None], next_goal=g["next_goal"][:, None],
                              reward=g["intrinsic"][:, None])
    assert counter == int(g["counter"]) == len(g["a1"]) > cap  # every step stored, the ring wrapped
    np.testing.assert_array_equal(mem, g["memory"].astype(np.float32))


def _literal_loop(cap, obs0, obs, a1, rew, done, fobs, won, skip):
    """main.py:115-119 line by line, envs stepped in index order at each step."""
    memory = np.zeros((cap, 22), np.float64)
    counter = 0
    T, n = a1.shape
    for t in range(T):
        for i in range(n):
            if skip and won[t, i]:
                continue
            state = obs0[i] if t == 0 else obs[t - 1, i]
            nxt = fobs[t, i] if done[t, i] else obs[t, i]
            transition = np.hstack((state, [a1[t, i], rew[t, i, 0]], nxt))
            memory[counter % cap, :] = transition
            counter += 1
    return memory.astype(np.float32), counter


@pytest.mark.parametrize("cap,T,n,skip", [(7, 5, 13, True), (1000, 3, 50, True), (64, 4, 16, False),
                                          (1, 2, 3, True), (150, 2, 75, True)])
def test_vectorised_store_equals_literal_loop(cap, T, n, skip):
    rng = np.random.default_rng(cap * 1000 + T * 10 + n)
    obs0 = rng.standard_normal((n, 10)).astype(np.float32)
    obs = rng.standard_normal((T, n, 10)).astype(np.float32)
    fobs = rng.standard_normal((T, n, 10)).astype(np.float32)
    a1 = rng.integers(0, 5, (T, n)).astype(np.int8)
    rew = rng.standard_normal((T, n, 2)).astype(np.float32)
    done = rng.random((T, n)) < 0.2
    won = rng.random((T, n)) < 0.3
    ref, c_ref = _literal_loop(cap, obs0, obs, a1, rew, done, fobs, won, skip)
    mem = np.zeros((cap, 22), np.float32)
    c = mo.replay_store(mem, 0, obs0, obs, a1, rew, done, fobs, won, skip_ego_won=skip)
    assert c == c_ref
    np.testing.assert_array_equal(mem, ref)


def test_sample_index_range_and_uniformity(coracle):
    idx = mo.replay_sample_index(coracle, 2000, 5000, seed=3, draw=11, batch=200000)
    assert idx.min() >= 0 and idx.max() < 2000
    counts = np.bincount(idx, minlength=2000)
    assert abs(counts.mean() - 100) < 1e-9 and counts.std() < 15  # Poisson(100): std 10
    small = mo.replay_sample_index(coracle, 2000, 37, seed=3, draw=11, batch=4096, filled_only=True)
    assert small.max() < 37
    empty = mo.replay_sample_index(coracle, 2000, 0, seed=3, draw=11, batch=64, filled_only=True)
    assert (empty == 0).all()


@pytest.mark.parametrize("tag", ["HL0", "HRR"])
def test_goal_status_matches_reference_intrinsic_rewards(coracle, replay_golden, tag):
    """policy.goal_status (hdqn.py:223-237) on the oracle's observations reproduces every intrinsic
    reward of the reference run (1.0 iff next_goal == goal_status(state), hdqn.py:314), scalar and
    batched."""
    import torch

    from merging_gym.policy import goal_status

    g = {k[len(tag) + 1:]: replay_golden[k] for k in replay_golden.files if k.startswith(tag + "_")}
    obs0, obs, *_ = _oracle_episode_run(coracle, g["a1"], g["a2"])
    prev = np.concatenate([obs0[None], obs[:-1]], axis=0)[:, 0]  # the state before each step
    batch = goal_status(torch.from_numpy(prev)).numpy()
    scalar = np.array([goal_status([float(x) for x in row]) for row in prev])
    np.testing.assert_array_equal(batch, scalar)
    np.testing.assert_array_equal((g["next_goal"] == batch).astype(np.float32), g["intrinsic"])


def meta_rows_inputs(rew1, done, next_goal, status_next):
    """Goal_DQN's memory inputs of one env's run (hdqn.py:286, :311-313, :322, :325): the
    no-break mask (a step that did not end the inner loop stores nothing) and the extrinsic
    reward summed in fp64 since the inner loop began, as stored at a break."""
    brk = np.asarray(done, bool) | (np.asarray(next_goal) == np.asarray(status_next))
    ext = np.zeros(len(brk))
    acc = 0.0
    for k in range(len(brk)):
        acc += float(rew1[k])
        ext[k] = acc
        if brk[k]:
            acc = 0.0
    return ~brk, ext


@pytest.mark.parametrize("tag", ["HL0", "HRR"])
def test_oracle_meta_store_reproduces_goal_dqn_memory(coracle, replay_golden, tag):
    """Goal_DQN's memory (Goal_DQN.store_transition :97-101 at :325 after each inner-loop break or
    episode end; rows [state, goal, extrinsic_reward, next_state] with state = next_state and the
    :303 goal): the reference's own run (gen_replay.run_hdqn) equals the oracle's meta rows fed by
    the oracle's own steps (fp64 rewards summed as the reference sums them) bit for bit."""
    g = {k[len(tag) + 1:]: replay_golden[k] for k in replay_golden.files if k.startswith(tag + "_")}
    T = len(g["a1"])
    envs = coracle.new_envs(1)
    obs0 = coracle.reset(envs).astype(np.float32)
    obs = np.empty((T, 1, 10), np.float32)
    fobs = np.full((T, 1, 10), np.nan, np.float32)
    rew = np.empty((T, 1, 2), np.float32)
    done = np.empty((T, 1), bool)
    rew1 = np.empty(T)
    nxt64 = np.empty((T, 10))
    for t in range(T):
        o, r, d, _, _, fo, err = coracle.step(envs, g["a1"][t:t + 1], None if g["a2"][t] < 0 else g["a2"][t:t + 1],
                                              autoreset=True, final_obs=True)
        assert err == 0
        obs[t], rew[t], done[t] = o.astype(np.float32), r.astype(np.float32), bool(d[0])
        fobs[t] = fo.astype(np.float32)
        rew1[t] = r[0, 0]
        nxt64[t] = fo[0] if d[0] else o[0]
    np.testing.assert_array_equal(done[:, 0], g["done"])
    status = np.where(nxt64[:, 0] < -0.5 * nxt64[:, 9], 0, np.where(nxt64[:, 0] < 0.5 * nxt64[:, 9], 1, 2))
    nobrk, ext = meta_rows_inputs(rew1, done[:, 0], g["next_goal"], status)
    cap = int(g["meta_capacity"])
    mem = np.zeros((cap, 22), np.float32)
    counter = mo.replay_store(mem, 0, obs0, obs, g["a1"][:, None], rew, done, fobs, nobrk[:, None],
                              reward=ext[:, None], meta_goal=g["next_goal"][:, None])
    assert counter == int(g["meta_counter"]) > cap  # the ring wrapped
    np.testing.assert_array_equal(mem, g["meta_memory"].astype(np.float32))
