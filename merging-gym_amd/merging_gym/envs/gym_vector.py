"""gym 0.20's VectorEnv protocol over MergeVecEnv (the version the reference pins, requirements.txt:2).

MergeVecEnv's own API is the fast path: device tensors in and out, ONE dict of batched infos. A
caller written against gym 0.20's vector envs (gym/vector/vector_env.py: reset_async / reset_wait,
step_async / step_wait, numpy outputs, a tuple of N per-env info dicts with the last observation of
a finished env under infos[i]["terminal_observation"], autoreset as SyncVectorEnv does) gets that
protocol here, at the cost of one device-to-host copy per step:

    venv = MergeVecEnv(n, device="cuda:0").gym_vector()
    obs = venv.reset()                           # [n, 10] numpy, the space's dtype (float16)
    obs, rew, dones, infos = venv.step(actions)  # rew [n, 2] float64 (both players, the
                                                 # reference's step(a1, a2) returns [r1, r2])

Rewards are the kernel's fp32 [r1, r2] widened to float64: the reference's Python floats are fp64,
so they agree to fp32 rounding (the path's stated tolerance), not beyond. Stock gym 0.20 wrappers
expect a reward vector [n]: `gym_vector(ego_reward_only=True)` returns the ego's reward only.

Observations take the observation space's dtype: gym 0.20's vector envs build their output
arrays from the single space (create_empty_array), and the reference's space is float16
(merging_env.py:75-78). actions: [n] ego actions (the opponent then None, merging_env.py:152),
[n, 2] (ego, opponent; -1 = None), or a pair (a1, a2) of [n] arrays.
"""

from __future__ import annotations

import numpy as np


class GymVectorEnv:
    """gym 0.20 VectorEnv protocol (duck-typed: gym is not a dependency) over a MergeVecEnv."""

    def __init__(self, env, obs_dtype=None, ego_reward_only=False):
        self.env = env
        self.ego_reward_only = ego_reward_only
        self.num_envs = env.num_envs
        self.single_observation_space = env.single_observation_space
        self.single_action_space = env.single_action_space
        self.observation_space = env.observation_space
        self.action_space = env.action_space
        self.obs_dtype = np.dtype(obs_dtype if obs_dtype is not None else self.single_observation_space.dtype)
        self._actions = None
        self.closed = False

    # ---------------------------------------------------------------- gym 0.20 vector API
    def reset_async(self):
        pass

    def reset_wait(self, **kwargs):
        return self._host_obs(self.env.reset())

    def reset(self):
        self.reset_async()
        return self.reset_wait()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self, **kwargs):
        if self._actions is None:
            raise RuntimeError("step_wait() without step_async()")
        actions, self._actions = self._actions, None
        a1, a2 = self._split(actions)
        obs, rew, done, info = self.env.step(a1, a2)
        dones = done.cpu().numpy().astype(bool)
        coll = info["collision"].cpu().numpy().astype(bool)
        infos = [{"collision": bool(c)} for c in coll]
        if dones.any() and self.env.autoreset:
            term = info.get("terminal_observation")
            if term is None:
                raise RuntimeError("gym 0.20's terminal_observation needs MergeVecEnv(final_observation=True)")
            idx = np.flatnonzero(dones)
            rows = term[self._torch_index(idx)].cpu().numpy().astype(self.obs_dtype)
            for k, i in enumerate(idx):
                infos[i]["terminal_observation"] = rows[k]
        r = rew.cpu().numpy().astype(np.float64)
        return self._host_obs(obs), (r[:, 0].copy() if self.ego_reward_only else r), dones, tuple(infos)

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def seed(self, seeds=None):
        """The reference's reset is deterministic and its env has no seeding API."""
        return [None] * self.num_envs

    def close(self, **kwargs):
        if not self.closed:
            self.env.close()
            self.closed = True

    def __len__(self):
        return self.num_envs

    def __repr__(self):
        return f"GymVectorEnv({self.num_envs} envs on {getattr(self.env, 'device', '?')})"

    # ---------------------------------------------------------------- helpers
    def _host_obs(self, obs):
        return obs.cpu().numpy().astype(self.obs_dtype)

    def _torch_index(self, idx):
        import torch

        return torch.as_tensor(idx, device=getattr(self.env, "device", "cpu"))

    def _split(self, actions):
        # a pair (a1, a2) only when each part is a whole batch of actions (a2 may be None): with
        # num_envs == 2 a tuple of two scalars is the two envs' ego actions, not a pair
        if isinstance(actions, tuple) and len(actions) == 2 and all(
                x is None or np.shape(x.cpu() if hasattr(x, "cpu") else x) == (self.num_envs,) for x in actions) \
                and actions[0] is not None:
            return actions
        a = np.asarray(actions.cpu() if hasattr(actions, "cpu") else actions)
        if a.ndim == 2 and a.shape == (self.num_envs, 2):
            return a[:, 0].copy(), a[:, 1].copy()
        if a.shape == (self.num_envs,):
            return a, None
        raise ValueError(f"actions must be [{self.num_envs}], [{self.num_envs}, 2] or a pair of [{self.num_envs}]")
