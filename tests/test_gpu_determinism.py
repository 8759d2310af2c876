"""Run-to-run determinism of the fused policy kernels (round 5). Their Q-net and env waves hand
work to each other inside a phase through LDS flags: config 5's ego waves wait for the opponent
waves to have read the may-finish rows before overwriting them with Q-values (qrows_read), env waves
run the Q-net waves' list tails once those waves publish their lists (qtail), and the h-DQN opponent
meta-net pass is compacted within each wave. A missing or misplaced wait shows up as a result that
depends on the waves' timing. Two runs from the same state must agree bit for bit -- trajectories,
env state and the 64-byte episode records (q_eval included) -- over many launches at a size that
fills the chip, with the clocks staggered so episode ends (and may-finish items) come every step.

Reference: scripts/main.py:99-112, :221 (config 5) and scripts/hdqn.py:280-330 (h-DQN)."""

import os

import numpy as np
import pytest

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


def _env(n, seed):
    import torch

    from merging_gym import MergeVecEnv

    env = MergeVecEnv(n, device="cuda:0")
    phase = torch.arange(n, device="cuda:0") % 251
    for k in range(251):  # episodes at 251 different phases: ends at every step
        env.step_random(seed, step_idx=k)
        env.reset(phase == k)
    return env


def _snapshot(env, trajs):
    out = {k: v.clone() for k, v in env.state_dict().items() if hasattr(v, "clone")}
    for t, tr in enumerate(trajs):
        for k, v in tr.items():
            if v is not None and hasattr(v, "clone"):
                out[f"traj{t}/{k}"] = v.clone()
    return out


def _assert_same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        x, y = a[k].cpu().numpy(), b[k].cpu().numpy()
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), k


@pytest.mark.parametrize("opponent", ["self", "other"])
def test_rollout_qnet_runs_are_bit_identical(opponent):
    from merging_gym.policy import QNet

    n, T, launches, seed = 1 << 18, 16, 12, 23
    qnet = QNet.from_state_dict(_checkpoint("l1"), device="cuda:0")
    opp = QNet.from_state_dict(_checkpoint("l3"), device="cuda:0") if opponent == "other" else "self"
    env = _env(n, seed)
    start = env.state_dict()
    runs = []
    for _ in range(2):
        env.load_state_dict(start)
        trajs = [env.rollout_qnet(T, qnet, seed, opponent=opp, first_step=1000 + T * k) for k in range(launches)]
        runs.append(_snapshot(env, trajs[-1:]))  # (the buffers are reused: the last launch)
        ends = int(env.counts[:, 0].sum().item())
    assert ends > n  # episodes ended (q_eval logged) throughout
    _assert_same(*runs)


@pytest.mark.parametrize("opponent", ["self", "other"])
def test_rollout_hdqn_runs_are_bit_identical(opponent):
    from merging_gym.policy import NUM_GOALS, QNet

    rng = np.random.default_rng(5)
    n, T, launches, seed = 1 << 17, 16, 8, 29
    meta = QNet.from_state_dict(_signed(rng, 10, NUM_GOALS), device="cuda:0")
    lower = QNet.from_state_dict(_signed(rng, 11, 5), device="cuda:0")
    opp = ((QNet.from_state_dict(_signed(rng, 10, NUM_GOALS), device="cuda:0"),
            QNet.from_state_dict(_signed(rng, 11, 5), device="cuda:0")) if opponent == "other" else "self")
    env = _env(n, seed)
    start = env.state_dict()
    runs = []
    for _ in range(2):
        env.load_state_dict(start)  # taken before any h-DQN launch: no goals, no extrinsic sums yet
        assert env.hdqn_goal is None and env.hdqn_goal_op is None and env.hdqn_ext is None
        trajs = [env.rollout_hdqn(T, meta, lower, seed, opponent=opp, first_step=1000 + T * k) for k in range(launches)]
        runs.append(_snapshot(env, trajs[-1:]))
    _assert_same(*runs)
