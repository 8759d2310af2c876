"""Host-side surface that needs no GPU: registration ids, spaces, and loud failure without a GPU."""

import numpy as np
import pytest

import merging_gym
from merging_gym import spaces


def test_env_ids_match_reference():
    # merging_gym/__init__.py:3-11 of the reference, plus the alias used by BASELINE config 1
    assert merging_gym.ENV_IDS["merging_env-v0"] == "merging_gym.envs:MergeEnv"
    assert merging_gym.ENV_IDS["merging_env_extend-v0"] == "merging_gym.envs:MergeEnvExtend"
    assert merging_gym.ENV_IDS["merging-v0"] == "merging_gym.envs:MergeEnv"
    with pytest.raises(KeyError):
        merging_gym.make("CartPole-v0")


def test_spaces_match_golden(golden):
    obs = spaces.observation_space()
    np.testing.assert_array_equal(obs.low.astype(np.float64), golden["obs_low"])
    np.testing.assert_array_equal(obs.high.astype(np.float64), golden["obs_high"])
    assert str(obs.dtype) == str(golden["obs_dtype"])
    assert obs.shape == (10,)
    act = spaces.action_space()
    assert act.n == int(golden["n_actions"]) == 5
    assert isinstance(act.sample(), int)  # scripts test isinstance(sample(), int), hdqn.py:33
    assert act.contains(4) and not act.contains(5)


def test_constants_module(golden):
    from merging_gym.envs import merging_env as me

    assert (me.RFirst, me.RSecond, me.RCollision, me.vel_penalty) == tuple(golden["show_reward"])
    assert (me.START_POINT, me.END_POINT, me.VEHICLE_W, me.VEHICLE_H) == (50, 950, 4, 8)


def test_no_cpu_fallback():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        merging_gym.MergeVecEnv(8)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        merging_gym.make("merging_env-v0")


def test_extend_env_is_the_print_stub(capsys):
    e = merging_gym.make("merging_env_extend-v0")
    e.reset()
    e.step()
    assert "MergeEnvExtend" in capsys.readouterr().out
