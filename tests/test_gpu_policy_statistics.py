"""The fused policy kernels' episode statistics over many launches (round 4: they record finished
episodes with no-return atomics and keep main.py's pending value in a register, loaded only for the
envs whose ego arrived first in an earlier launch). 14 launches of 16 steps over envs started at
staggered phases: every episode's sums and counts, and the pending value of the episodes in
progress, must equal the C oracle stepping the same actions -- bit for bit, including the
episodes whose ego-first arrival and end fall in different launches.

Reference: scripts/main.py:189-228 and scripts/hdqn.py:276-346 (what the records hold)."""

import os

import numpy as np
import pytest

import merge_oracle as mo
from conftest import ROOT

pytestmark = pytest.mark.gpu


def _checkpoint(key):
    f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    return {name.split("/", 1)[1]: f[name] for name in f.files if name.startswith(key + "/")}


def _signed(rng, in_dim, out_dim):
    sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), [(200, in_dim), (100, 200), (out_dim, 100)]):
        sd[f"{name}.weight"] = rng.uniform(-i ** -0.5, i ** -0.5, (o, i)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    return sd


def _staggered_env(n, seed):
    import torch

    from merging_gym import MergeVecEnv

    env = MergeVecEnv(n, device="cuda:0")
    phase = torch.arange(n, device="cuda:0") % 97
    for k in range(97):  # first episodes at 97 different phases
        env.step_random(seed, step_idx=k)
        env.reset(phase == k)
    for k in range(97, 300):
        env.step_random(seed, step_idx=k)
    return env


def _replay_and_compare(coracle, env, launch, launches, T):
    envs = mo.oracle_envs_from(coracle, env)
    stats = (env.returns.cpu().numpy().copy(), env.counts.cpu().numpy().astype(np.uint32).copy())
    pend_seen = 0
    for _ in range(launches):
        winner_before = env.winner.cpu().numpy().copy()
        episodes_before = env.counts[:, 0].cpu().numpy().copy()
        traj = launch()
        a1, a2 = traj["a1"].cpu().numpy(), traj["a2"].cpu().numpy()
        for t in range(T):
            *_, err = coracle.step(envs, a1[t], a2[t], autoreset=True, stats=stats)
            assert err == 0
        # episodes that ended in this launch after an ego-first arrival in an earlier one: their
        # main.py term is the pending value the launch loaded (pend_load)
        pend_seen += int(((winner_before == 1) & (env.counts[:, 0].cpu().numpy() > episodes_before)).sum())
    np.testing.assert_array_equal(env.p1.cpu().numpy(), envs["pos1"])
    np.testing.assert_array_equal(env.counts.cpu().numpy().astype(np.uint32), stats[1])
    np.testing.assert_array_equal(env.returns.cpu().numpy(), stats[0])
    w1 = envs["winner"] == 1
    np.testing.assert_array_equal(env._ep_stats[:, 3].cpu().numpy()[w1], envs["ep_reward_main"][w1])
    assert int(stats[1][:, 0].sum()) > env.num_envs
    return pend_seen, int(w1.sum()), bool((stats[0][:, 2] != stats[0][:, 0]).any())


@pytest.mark.parametrize("opponent", ["none", "other"])
def test_qnet_statistics_over_many_launches(coracle, opponent):
    from merging_gym.policy import QNet

    n, T, launches, seed = 3001, 16, 14, 31
    env = _staggered_env(n, seed)
    qnet = QNet.from_state_dict(_checkpoint("l1"), device="cuda:0")
    opp = QNet.from_state_dict(_checkpoint("l3"), device="cuda:0") if opponent == "other" else opponent
    k = [1000]

    def launch():
        tr = env.rollout_qnet(T, qnet, seed, opponent=opp, first_step=k[0], final_observation=False)
        k[0] += T
        return tr

    pend_seen, pending_now, filtered = _replay_and_compare(coracle, env, launch, launches, T)
    print(f"[policy statistics] config 5 ({opponent}): {pend_seen} episodes ended after an ego-first arrival "
          f"in an earlier launch; {pending_now} pending at the end")
    if opponent == "none":  # against main.py's L0 opponent the ego often arrives first and waits
        assert pend_seen > 0 and pending_now > 0 and filtered


@pytest.mark.parametrize("opponent", ["none", "self"])
def test_hdqn_statistics_over_many_launches(coracle, opponent):
    from merging_gym.policy import NUM_GOALS, QNet

    n, T, launches, seed = 2049, 16, 14, 37
    env = _staggered_env(n, seed)
    rng = np.random.default_rng(5)
    meta = QNet.from_state_dict(_signed(rng, 10, NUM_GOALS), device="cuda:0")
    lower = QNet.from_state_dict(_signed(rng, 11, 5), device="cuda:0")
    k = [2000]

    def launch():
        tr = env.rollout_hdqn(T, meta, lower, seed, opponent=opponent, first_step=k[0], final_observation=False)
        k[0] += T
        return tr

    pend_seen, pending_now, filtered = _replay_and_compare(coracle, env, launch, launches, T)
    print(f"[policy statistics] h-DQN ({opponent}): {pend_seen} episodes ended after an ego-first arrival "
          f"in an earlier launch; {pending_now} pending at the end")
    assert pend_seen > 0 and filtered
