"""Observation / action spaces of merging_env-v0 (merging_gym/envs/merging_env.py:75-78, :101-102).

When gym is importable its own spaces are used, so `isinstance(env.action_space,
gym.spaces.Discrete)` holds for drop-in callers. This image has no gym, so a minimal
stand-in with the attributes the reference's callers read (`.n`, `.shape`, `.sample()`,
`.low`, `.high`, `.dtype`, `.contains`) is used instead.
"""

from __future__ import annotations

import numpy as np

H, W = 1000, 300
OBS_LOW = np.array([-H, -W, -100, 0, 0, -H, -W, -100, 0, 0])
OBS_HIGH = np.array([H, W, 100, H, 100, H, W, 100, H, 100])

try:  # pragma: no cover - gym is not installed in this image
    from gym import spaces as _gym_spaces
except Exception:  # noqa: BLE001
    _gym_spaces = None


class Box:
    def __init__(self, low, high, dtype=np.float32, shape=None):
        self.dtype = np.dtype(dtype)
        self.low = np.asarray(low, dtype=self.dtype)
        self.high = np.asarray(high, dtype=self.dtype)
        self.shape = self.low.shape if shape is None else tuple(shape)
        self._rng = np.random.default_rng()

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class Discrete:
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)
        self._rng = np.random.default_rng()

    def sample(self):
        return int(self._rng.integers(self.n))

    def contains(self, x):
        try:
            v = int(x)
        except (TypeError, ValueError):
            return False
        return v == x and 0 <= v < self.n

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def __repr__(self):
        return f"Discrete({self.n})"


def observation_space():
    """Box(10,) declared float16 like the reference (the values themselves are fp64)."""
    if _gym_spaces is not None:  # pragma: no cover
        return _gym_spaces.Box(low=OBS_LOW, high=OBS_HIGH, dtype=np.float16)
    return Box(OBS_LOW, OBS_HIGH, dtype=np.float16)


def action_space(n=5):
    if _gym_spaces is not None:  # pragma: no cover
        return _gym_spaces.Discrete(n)
    return Discrete(n)


class MultiDiscrete:
    """gym.spaces.MultiDiscrete stand-in: one Discrete(n) per entry of nvec."""

    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
        self.dtype = np.dtype(np.int64)
        self._rng = np.random.default_rng()

    def sample(self):
        return self._rng.integers(0, self.nvec).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and np.issubdtype(x.dtype, np.integer) and bool(
            np.all((x >= 0) & (x < self.nvec)))

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def __repr__(self):
        return f"MultiDiscrete({self.nvec.tolist() if self.nvec.size <= 8 else self.shape})"


def batched_action_space(num_envs, n=5):
    """gym 0.20's batch_space(Discrete(n), num_envs): MultiDiscrete([n] * num_envs), one ego
    action per env (the opponent's actions are step()'s second argument)."""
    if _gym_spaces is not None:  # pragma: no cover
        return _gym_spaces.MultiDiscrete(np.full(num_envs, n))
    return MultiDiscrete(np.full(num_envs, n))


def batched_observation_space(num_envs):
    low = np.tile(OBS_LOW, (num_envs, 1))
    high = np.tile(OBS_HIGH, (num_envs, 1))
    if _gym_spaces is not None:  # pragma: no cover
        return _gym_spaces.Box(low=low, high=high, dtype=np.float32)
    return Box(low, high, dtype=np.float32)
