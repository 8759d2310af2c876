"""gym 0.20's VectorEnv protocol (merging_gym/envs/gym_vector.py) over MergeVecEnv.

CPU: the adapter's protocol logic (step_async / step_wait, numpy outputs in the space's dtype,
per-env infos with "terminal_observation" where an env finished, the action layouts) over a stand-in
env with MergeVecEnv's interface whose step is the C oracle. GPU: the adapter over a real
MergeVecEnv equals the device-tensor API on the same actions."""
import numpy as np
import pytest

import merge_oracle
from merging_gym import spaces
from merging_gym.envs.gym_vector import GymVectorEnv


class OracleVecEnv:
    """MergeVecEnv's interface (reset / step returning CPU tensors, batched info dict) stepped by the
    C oracle with autoreset and final observations."""

    def __init__(self, n):
        import torch

        self.torch, self.num_envs, self.device, self.autoreset = torch, n, torch.device("cpu"), True
        self.co = merge_oracle.COracle(merge_oracle.build_c_oracle())
        self.envs = self.co.new_envs(n)
        self.single_observation_space = spaces.observation_space()
        self.single_action_space = spaces.action_space()
        self.observation_space = spaces.batched_observation_space(n)
        self.action_space = spaces.batched_action_space(n)
        self.closed = False

    def reset(self):
        return self.torch.from_numpy(self.co.reset(self.envs).astype(np.float32))

    def step(self, a1, a2=None):
        obs, rew, done, coll, _, fobs, err = self.co.step(self.envs, a1, a2, autoreset=True, final_obs=True)
        assert err == 0
        t = self.torch
        info = {"collision": t.from_numpy(coll.astype(bool)), "terminal_observation": t.from_numpy(fobs.astype(np.float32))}
        return t.from_numpy(obs.astype(np.float32)), t.from_numpy(rew.astype(np.float32)), t.from_numpy(done.astype(bool)), info

    def close(self):
        self.closed = True


def test_gym020_protocol_over_the_oracle(coracle):
    n, steps = 512, 400
    venv = GymVectorEnv(OracleVecEnv(n))
    ref = coracle.new_envs(n)
    obs = venv.reset()
    assert obs.dtype == np.float16 and obs.shape == (n, 10)  # the space's dtype, as gym 0.20's create_empty_array
    np.testing.assert_array_equal(obs, coracle.reset(ref).astype(np.float32).astype(np.float16))
    rng = np.random.default_rng(3)
    finished = 0
    for k in range(steps):
        a1 = rng.integers(0, 5, n).astype(np.int8)
        a2 = rng.integers(-1, 5, n).astype(np.int8)
        acts = (a1, a2) if k % 3 == 0 else (np.stack([a1, a2], 1) if k % 3 == 1 else a1)
        if k % 3 == 2:
            a2 = None
        venv.step_async(acts)
        obs, rew, dones, infos = venv.step_wait()
        o, r, d, c, _, f, err = coracle.step(ref, a1, a2, autoreset=True, final_obs=True)
        assert isinstance(infos, tuple) and len(infos) == n
        assert obs.dtype == np.float16 and rew.dtype == np.float64 and dones.dtype == bool
        np.testing.assert_array_equal(obs, o.astype(np.float32).astype(np.float16))
        np.testing.assert_array_equal(rew, r.astype(np.float32).astype(np.float64))
        np.testing.assert_array_equal(dones, d.astype(bool))
        for i in range(n):
            assert infos[i]["collision"] == bool(c[i])
            assert ("terminal_observation" in infos[i]) == bool(d[i])
            if d[i]:
                np.testing.assert_array_equal(infos[i]["terminal_observation"], f[i].astype(np.float32).astype(np.float16))
        finished += int(d.sum())
    assert finished > 500
    assert venv.seed(1) == [None] * n and len(venv) == n
    with pytest.raises(ValueError):
        venv.step(np.zeros((n, 3), np.int8))
    with pytest.raises(RuntimeError):
        venv.step_wait()
    venv.close()
    assert venv.env.closed


@pytest.mark.gpu
def test_gym020_protocol_equals_the_device_api():
    import torch

    from merging_gym import MergeVecEnv

    n = 4096
    fast = MergeVecEnv(n, device="cuda:0")
    venv = MergeVecEnv(n, device="cuda:0").gym_vector(obs_dtype=np.float32)
    assert np.array_equal(venv.reset(), fast.reset().cpu().numpy())
    rng = np.random.default_rng(4)
    ends = 0
    for _ in range(300):
        a = rng.integers(0, 5, (n, 2)).astype(np.int8)
        obs, rew, dones, infos = venv.step(a)
        o, r, d, info = fast.step(torch.from_numpy(a[:, 0]), torch.from_numpy(a[:, 1]))
        assert np.array_equal(obs, o.cpu().numpy()) and np.array_equal(rew, r.cpu().numpy().astype(np.float64))
        assert np.array_equal(dones, d.cpu().numpy())
        term = info["terminal_observation"].cpu().numpy()
        for i in np.flatnonzero(dones):
            assert np.array_equal(infos[i]["terminal_observation"], term[i])
        ends += int(dones.sum())
    assert ends > 100


def test_pair_split_and_ego_reward_only():
    """A 2-tuple is read as (a1, a2) only when each part is a whole batch (a2 may be None); with two
    envs a tuple of two scalars is the two envs' ego actions. ego_reward_only returns rewards [n] (the
    ego's), the vector stock gym 0.20 wrappers expect."""
    env = OracleVecEnv(2)
    v = GymVectorEnv(env)
    v.reset()
    a1, a2 = v._split((np.array([1, 2]), np.array([3, 4])))
    assert a1.tolist() == [1, 2] and a2.tolist() == [3, 4]
    a1, a2 = v._split((np.array([1, 2]), None))
    assert a1.tolist() == [1, 2] and a2 is None
    a1, a2 = v._split((3, 4))  # two envs' ego actions, not a pair
    assert np.asarray(a1).tolist() == [3, 4] and a2 is None
    _, rew, _, _ = v.step(np.array([1, 2]))
    assert rew.shape == (2, 2) and rew.dtype == np.float64
    ve = GymVectorEnv(OracleVecEnv(2), ego_reward_only=True)
    ve.reset()
    _, rew1, _, _ = ve.step(np.array([1, 2]))
    assert rew1.shape == (2,) and np.array_equal(rew1, rew[:, 0])
