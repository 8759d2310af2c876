"""reset() and rollout_hdqn's per-env loop state (scripts/hdqn.py:277-286): hdqn.py starts every
episode with env.reset(), a fresh upper.choose_goal(state) (and upper_op's) and
extrinsic_reward = 0. So after MergeVecEnv.reset() the next rollout_hdqn launch must act exactly
as a fresh batch does -- no goal carried over, no running extrinsic sum -- and a masked reset
must clear only the masked envs. hdqn.py resets at every episode end, so an env without autoreset
is refused (the kernel's terminal-observation path assumes the reset)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


def _net_signed(rng, in_dim, out_dim):
    sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), [(200, in_dim), (100, 200), (out_dim, 100)]):
        sd[f"{name}.weight"] = rng.uniform(-i ** -0.5, i ** -0.5, (o, i)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    return sd


@pytest.fixture(scope="module")
def nets(torch):
    from merging_gym.policy import QNet

    rng = np.random.default_rng(123)
    return (QNet.from_state_dict(_net_signed(rng, 10, 3), device="cuda:0"),
            QNet.from_state_dict(_net_signed(rng, 11, 5), device="cuda:0"))


def test_rollout_hdqn_needs_autoreset(torch, nets):
    from merging_gym import MergeVecEnv

    env = MergeVecEnv(64, device="cuda:0", autoreset=False)
    with pytest.raises(ValueError):
        env.rollout_hdqn(4, nets[0], nets[1], seed=1)


@pytest.mark.parametrize("opponent", ["none", "self"])
def test_reset_between_launches_acts_as_a_fresh_batch(torch, nets, opponent):
    from merging_gym import MergeVecEnv

    meta, lower = nets
    n, T = 1000, 24
    a = MergeVecEnv(n, device="cuda:0")
    a.rollout_hdqn(T, meta, lower, seed=9, opponent=opponent, first_step=0, goal_memory=True)
    torch.cuda.synchronize()
    assert (a.hdqn_goal >= 0).all() and a.hdqn_ext.abs().sum() > 0  # the first launch left loop state
    a.reset()
    assert (a.hdqn_goal == -1).all() and (a.hdqn_ext == 0).all()
    if opponent == "self":
        assert (a.hdqn_goal_op == -1).all()
    ta = a.rollout_hdqn(T, meta, lower, seed=9, opponent=opponent, first_step=500, goal_memory=True)
    b = MergeVecEnv(n, device="cuda:0")
    tb = b.rollout_hdqn(T, meta, lower, seed=9, opponent=opponent, first_step=500, goal_memory=True)
    torch.cuda.synchronize()
    assert set(ta) == set(tb)
    for k in ta:
        if ta[k] is None or tb[k] is None:  # outputs not requested
            assert ta[k] is None and tb[k] is None, k
            continue
        assert torch.equal(ta[k], tb[k]) or (ta[k].is_floating_point() and torch.allclose(
            ta[k], tb[k], rtol=0, atol=0, equal_nan=True)), k
    for name in ("p1", "v1", "p2", "v2", "ret1", "ret2", "tf", "hdqn_goal", "hdqn_ext"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


def test_masked_reset_clears_only_the_masked_envs(torch, nets):
    from merging_gym import MergeVecEnv

    meta, lower = nets
    n = 640
    env = MergeVecEnv(n, device="cuda:0")
    env.rollout_hdqn(20, meta, lower, seed=4, opponent="self", first_step=0, goal_memory=True)
    torch.cuda.synchronize()
    goal, goal_op, ext = env.hdqn_goal.clone(), env.hdqn_goal_op.clone(), env.hdqn_ext.clone()
    p1 = env.p1.clone()
    mask = np.zeros(n, bool)
    mask[::3] = True
    env.reset(mask)
    torch.cuda.synchronize()
    m = torch.as_tensor(mask, device="cuda:0")
    assert (env.hdqn_goal[m] == -1).all() and (env.hdqn_goal_op[m] == -1).all() and (env.hdqn_ext[m] == 0).all()
    assert torch.equal(env.hdqn_goal[~m], goal[~m]) and torch.equal(env.hdqn_goal_op[~m], goal_op[~m])
    assert torch.equal(env.hdqn_ext[~m], ext[~m])
    assert (env.p1[m] == 50.0).all() and torch.equal(env.p1[~m], p1[~m])
