"""ReplayRing: the DQN replay memory kept on the GPU.

Device twin of the reference's memory (scripts/main.py:91-92 `np.zeros((MEMORY_CAPACITY,
NUM_STATES * 2 + 2))`, :115-119 store_transition, :129-135 the minibatch draw in learn(); the
same structure in scripts/hdqn.py:157-158, :180-184, :194-199). Rows are
[s(10), a, r, s'(10)] fp32 -- the reference keeps fp64 rows and reads them back through
torch.FloatTensor, so the values learn() sees are the same. `ReplayRing(cap, goal=True)` holds
hdqn.py's lower-level rows [goal, s(10), a, r, next_goal, s'(10)] (goal_state = [goal] + state,
:291 and :304; intrinsic reward :314): store() then takes the per-transition goals and the
reward column.

Transitions go in straight from a MergeVecEnv's trajectory buffers (one batched store per
rollout, three kernel launches from libmerging_hip.so) instead of one store_transition call
per env step; the order is (step, env), i.e. what stepping env 0..N-1 and storing each in
turn would give. The ring position lives on the device; reading `memory_counter`
synchronises.

    ring = ReplayRing(capacity=2000, device="cuda:0")
    obs0 = env.observe().clone()
    traj = env.rollout_qnet(16, qnet, seed)
    ring.store_rollout(obs0, traj)                       # main.py:209 filter by default
    s, a, r, s2 = ring.sample(128, seed=1, draw=step)    # main.py:130-135
"""

from __future__ import annotations

import ctypes

from . import _native

_OBS_DIM = 10
ROW = 2 * _OBS_DIM + 2        # main.py:91: NUM_STATES * 2 + 2
ROW_GOAL = 2 * _OBS_DIM + 4   # hdqn.py:158: (NUM_STATES + 1) * 2 + 2


class ReplayRing:
    def __init__(self, capacity: int = 2000, device=None, goal: bool = False):
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("ReplayRing needs a ROCm GPU; there is no CPU fallback")
        if capacity < 1:
            raise ValueError("capacity must be >= 1")
        self._torch = torch
        self.capacity = int(capacity)
        self.goal = bool(goal)
        self.row = ROW_GOAL if self.goal else ROW
        self._s0 = 1 if self.goal else 0  # column of s[0]
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.memory = torch.zeros((self.capacity, self.row), dtype=torch.float32, device=self.device)
        self._counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._scratch = torch.empty(0, dtype=torch.int64, device=self.device)
        self._sample_bufs = {}

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        return self._torch.cuda.current_stream(self.device).cuda_stream

    def _scratch_for(self, n, T):
        need = int(_native.lib.mg_replay_scratch_bytes(n, T))
        if self._scratch.numel() * 8 < need:
            self._scratch = self._torch.empty((need + 7) // 8, dtype=self._torch.int64, device=self.device)
        return self._scratch

    def _f32(self, t, shape):
        torch = self._torch
        t = torch.as_tensor(t, device=self.device)
        if t.dtype != torch.float32 or not t.is_contiguous():
            t = t.to(torch.float32).contiguous()
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"expected shape {tuple(shape)}, got {tuple(t.shape)}")
        return t

    # ------------------------------------------------------------------ stores
    @property
    def memory_counter(self) -> int:
        """Transitions stored so far (main.py:119). Synchronises the stream."""
        return int(self._counter.item())

    def store(self, obs_first, obs, a1, rew, done=None, final_obs=None, won_mask=None,
              skip_ego_won: bool = True, goal=None, next_goal=None, reward=None, flags=None, meta_goal=None):
        """Append T steps of N envs ([T, N, ...] tensors; obs_first [N, 10] = observation
        before step 0). skip_ego_won drops the transitions whose won bit is set (main.py:209;
        hdqn.py:316 stores all: pass False). A goal ring needs goal / next_goal [T, N] (the goal
        columns of s and s'); reward [T, N] replaces the ego's env reward rew[..., 0] as the r
        column (hdqn.py:314's intrinsic reward). flags: a rollout's interleaved [T, N, 4] buffer
        (a1, a2, done, collision), read in place of a1 / done. Stream-ordered; nothing is
        synchronised. meta_goal [T, N]: Goal_DQN's memory instead (hdqn.py:97-101 at :325, a plain
        22-float ring): rows [s', meta_goal, reward, s'] for the steps whose won_mask bit is clear,
        the mask then being the rollout's no_break and reward its ext_reward (store_meta)."""
        torch = self._torch
        if self.goal != (goal is not None) or (goal is None) != (next_goal is None):
            raise ValueError("a goal ring takes goal and next_goal; a plain ring takes neither")
        if meta_goal is not None:
            if self.goal or reward is None or won_mask is None:
                raise ValueError("Goal_DQN rows need a plain ring, reward (ext_reward) and won_mask (no_break)")
            skip_ego_won = True
        a1 = torch.as_tensor(a1, device=self.device)
        if a1.dim() == 1:  # one step
            goal = None if goal is None else torch.as_tensor(goal, device=self.device)[None]
            next_goal = None if next_goal is None else torch.as_tensor(next_goal, device=self.device)[None]
            reward = None if reward is None else torch.as_tensor(reward, device=self.device)[None]
            meta_goal = None if meta_goal is None else torch.as_tensor(meta_goal, device=self.device)[None]
            a1 = a1[None]
            obs = torch.as_tensor(obs, device=self.device)[None]
            rew = torch.as_tensor(rew, device=self.device)[None]
            done = None if done is None else torch.as_tensor(done, device=self.device)[None]
            final_obs = None if final_obs is None else torch.as_tensor(final_obs, device=self.device)[None]
            won_mask = None if won_mask is None else torch.as_tensor(won_mask, device=self.device)[None]
            flags = None if flags is None else torch.as_tensor(flags, device=self.device)[None]
        T, n = a1.shape
        if flags is not None:
            flags = torch.as_tensor(flags, device=self.device)
            if flags.dtype != torch.uint8 or tuple(flags.shape) != (T, n, 4) or not flags.is_contiguous():
                raise ValueError(f"flags must be a contiguous [{T}, {n}, 4] uint8 tensor")
            a1, done = None, None  # read from flags
        elif a1.dtype != torch.int8:
            a1 = a1.to(torch.int8)
        if a1 is not None:
            a1 = a1.contiguous()
        obs_first = self._f32(obs_first, (n, _OBS_DIM))
        obs = self._f32(obs, (T, n, _OBS_DIM))
        rew = self._f32(rew, (T, n, 2))
        if final_obs is not None:
            final_obs = self._f32(final_obs, (T, n, _OBS_DIM))
        if goal is not None:
            goal, next_goal = self._f32(goal, (T, n)), self._f32(next_goal, (T, n))
        if reward is not None:
            reward = self._f32(reward, (T, n))
        if meta_goal is not None:
            meta_goal = self._f32(meta_goal, (T, n))
        if done is not None:
            done = torch.as_tensor(done, device=self.device)
            if done.dtype == torch.bool:
                done = done.view(torch.uint8)
            done = done.to(torch.uint8).contiguous()
            if tuple(done.shape) != (T, n):
                raise ValueError(f"done must have shape {(T, n)}")
        if skip_ego_won and won_mask is not None:
            won_mask = torch.as_tensor(won_mask, device=self.device).to(torch.int64).contiguous()
            if tuple(won_mask.shape) != (T, (n + 63) // 64):
                raise ValueError(f"won_mask must have shape {(T, (n + 63) // 64)}")
        elif skip_ego_won:
            raise ValueError("skip_ego_won needs the won_mask of the step(s) (main.py:209): roll out "
                             "with won_mask=True / MergeVecEnv(won_mask=True), or pass skip_ego_won=False")
        ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        tr = _native.Transitions(ptr(obs_first), ptr(obs), ptr(final_obs), ptr(a1), ptr(rew),
                                 ptr(done), ptr(won_mask) if skip_ego_won else None, ptr(goal),
                                 ptr(next_goal), ptr(reward), ptr(flags), ptr(meta_goal))
        scratch = self._scratch_for(n, T)
        rc = _native.lib.mg_replay_store(
            self.memory.data_ptr(), self._counter.data_ptr(), self.capacity, self.row, ctypes.byref(tr), n,
            T, 1 if skip_ego_won else 0, scratch.data_ptr(), scratch.numel() * 8, self._stream())
        _native.check(rc, "mg_replay_store")
        self._keepalive = (obs_first, obs, a1, rew, done, final_obs, won_mask, goal, next_goal, reward, flags,
                           meta_goal)

    def store_rollout(self, obs_first, traj, skip_ego_won: bool = True, goal=None, next_goal=None,
                      reward=None):
        """Append a MergeVecEnv rollout (the dict rollout_random / rollout_qnet return). With
        autoreset the obs row of a finished env is already the reset observation, so the
        terminal one must come from final_observation (roll out with final_observation=True)."""
        if traj.get("final_observation") is None:
            raise ValueError("the rollout has no final_observation: episode ends would store the "
                             "reset observation as next_state; roll out with final_observation=True")
        self.store(obs_first, traj["obs"], traj["a1"], traj["rew"], traj["done"],
                   traj["final_observation"], traj.get("won_mask"), skip_ego_won, goal, next_goal, reward,
                   traj.get("flags"))

    def store_meta(self, traj):
        """Append Goal_DQN's rows of an h-DQN rollout (MergeVecEnv.rollout_hdqn(...,
        goal_memory=True)): upper.store_transition(state, goal, extrinsic_reward, next_state) at
        every inner-loop break or episode end (hdqn.py:325; state is already next_state and goal
        the :303 choice), in (t, i) order, into a plain ring (GOAL_MEMORY_CAPACITY = 200, :22,
        :75)."""
        if traj.get("final_observation") is None or traj.get("no_break") is None:
            raise ValueError("roll out with final_observation=True and goal_memory=True")
        self.store(traj["obs"][0], traj["obs"], traj["a1"], traj["rew"], traj["done"], traj["final_observation"],
                   traj["no_break"], True, None, None, traj["ext_reward"], traj.get("flags"),
                   meta_goal=traj["next_goal"])

    def store_transition(self, state, action, reward, next_state):
        """The reference's single-transition call (main.py:115-119; hdqn.py:180-184 for a goal
        ring, where state / next_state are the 11-value goal states [goal] + state), through the
        same kernels."""
        torch = self._torch
        if self.goal:
            gs, gs2 = [float(x) for x in state], [float(x) for x in next_state]
            s = torch.as_tensor([gs[1:]], dtype=torch.float32)
            s2 = torch.as_tensor([[gs2[1:]]], dtype=torch.float32)
            a = torch.as_tensor([[int(action)]], dtype=torch.int8)
            r = torch.as_tensor([[[float(reward), 0.0]]], dtype=torch.float32)
            g = torch.as_tensor([[gs[0]]], dtype=torch.float32)
            g2 = torch.as_tensor([[gs2[0]]], dtype=torch.float32)
            self.store(s.to(self.device), s2.to(self.device), a.to(self.device), r.to(self.device),
                       skip_ego_won=False, goal=g.to(self.device), next_goal=g2.to(self.device))
            return
        s = torch.as_tensor([list(map(float, state))], dtype=torch.float32)
        s2 = torch.as_tensor([[list(map(float, next_state))]], dtype=torch.float32)
        a = torch.as_tensor([[int(action)]], dtype=torch.int8)
        r = torch.as_tensor([[[float(reward), 0.0]]], dtype=torch.float32)
        self.store(s.to(self.device), s2.to(self.device), a.to(self.device), r.to(self.device),
                   skip_ego_won=False)

    # ------------------------------------------------------------------ checkpoint / resume
    def state_dict(self):
        """memory (copy) and memory_counter -- what DQN's memory and counter hold."""
        return {"memory": self.memory.clone(), "counter": self._counter.clone(), "goal": self.goal}

    def load_state_dict(self, sd):
        mem = self._torch.as_tensor(sd["memory"])
        if tuple(mem.shape) != tuple(self.memory.shape) or bool(sd.get("goal", False)) != self.goal:
            raise ValueError(f"expected a {tuple(self.memory.shape)} ring (goal={self.goal})")
        self.memory.copy_(mem)
        self._counter.copy_(self._torch.as_tensor(sd["counter"]))

    # ------------------------------------------------------------------ sampling
    def sample_rows(self, batch_size: int = 128, seed: int = 0, draw: int = 0,
                    filled_only: bool = False, return_index: bool = False):
        """[B, 22] (goal ring: [B, 24]) rows at Philox-drawn slots: np.random.choice(MEMORY_CAPACITY, BATCH_SIZE)
        (main.py:130-131); filled_only draws from the stored rows only. The returned tensor is
        reused by the next call with the same batch size."""
        torch = self._torch
        B = int(batch_size)
        buf = self._sample_bufs.get(B)
        if buf is None:
            buf = (torch.empty((B, self.row), dtype=torch.float32, device=self.device),
                   torch.empty(B, dtype=torch.int64, device=self.device))
            self._sample_bufs[B] = buf
        rows, idx = buf
        rc = _native.lib.mg_replay_sample(
            self.memory.data_ptr(), self._counter.data_ptr(), self.capacity, self.row, seed & 0xFFFFFFFFFFFFFFFF,
            draw & 0xFFFFFFFFFFFFFFFF, 1 if filled_only else 0, rows.data_ptr(), idx.data_ptr(), B,
            self._stream())
        _native.check(rc, "mg_replay_sample")
        return (rows, idx) if return_index else rows

    def sample(self, batch_size: int = 128, seed: int = 0, draw: int = 0, filled_only: bool = False):
        """(batch_state [B,10] f32, batch_action [B,1] int64, batch_reward [B,1] f32,
        batch_next_state [B,10] f32) -- the slices of main.py:131-135; for a goal ring the
        states are the 11-value goal states, as hdqn.py:196-199 slices them."""
        rows = self.sample_rows(batch_size, seed, draw, filled_only)
        k = _OBS_DIM + self._s0  # state width
        return (rows[:, :k], rows[:, k:k + 1].to(self._torch.int64), rows[:, k + 1:k + 2], rows[:, -k:])
