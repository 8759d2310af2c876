"""MergeVecEnv: N merging envs stepped together by one HIP kernel on an MI355X.

Batched form of MergeEnv (merging_gym/envs/merging_env.py:72-399 in the reference). State
lives on the GPU as a struct of arrays (fp64 positions / speeds / returns + one packed
uint32 of step count, winner and done); a step is one launch of `mg_step` (or
`mg_step_random`, actions drawn on the device) from libmerging_hip.so. Nothing is computed
on the host and there is no CPU fallback.

API (after gym 0.20's VectorEnv, with two players like the reference's step(a1, a2=None)):

    env = MergeVecEnv(num_envs, device="cuda:0")
    obs = env.reset()                                # [N,10] float32 tensor
    obs, rew, done, info = env.step(a1, a2=None)     # rew [N,2] f32, done [N] bool
    info["collision"]                                # [N] bool
    info["final_observation"]                        # [N,10] f32, valid where done (autoreset)

Outputs are views of buffers the env owns and overwrites on the next call (clone them to
keep them). With autoreset (the default) an env that finishes is reset inside the same
kernel: `obs` holds its reset observation and `info["final_observation"]` the terminal one.

Deviation from gym 0.20 (the version the reference pins, requirements.txt:2): its vector envs
return `infos` as N per-env dicts with the last observation of a finished env in
`infos[i]["terminal_observation"]`. This env returns ONE dict of batched device tensors (the layout
of later gym versions' batched infos), so no host loop over N envs runs per step; the terminal
observations are also under `info["terminal_observation"]` (the same [N,10] tensor). Observations,
rewards and dones are device tensors, and `step` takes both players' action arrays.
`gym_vector()` gives the gym 0.20 protocol itself (step_async / step_wait, numpy outputs, per-env
infos; envs/gym_vector.py) for callers written against it.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from .. import spaces

_OBS_DIM = 10
# The streamed per-env arrays (state + one step's outputs) are carved from one allocation, each
# array starting this many bytes (plus 256-byte alignment) after the previous one ends. As
# separate allocations they all start on 2 MiB boundaries, so element i of every array shares its
# low address bits; staggered, the step measured 2-3 % faster at 2^20 and 2^23 envs
# (tools/stagger_probe.py). MG_ARENA_STAGGER=-1 restores separate allocations (A/B).
_ARENA_STAGGER = int(os.environ.get("MG_ARENA_STAGGER", "4160"))
# One interleaved [N, 4] uint8 record (a1, a2, done, collision) per step instead of four byte
# arrays (mg_outputs.flags). MG_STEP_FLAGS=0 restores the four arrays (A/B, and the tests run both).
_STEP_FLAGS = os.environ.get("MG_STEP_FLAGS", "1") != "0"
# mg_rollout_random's limit per launch (16-bit per-launch episode counts in registers)
_MAX_ROLLOUT_STEPS = 65535


class MergeVecEnv:
    metadata = {"render.modes": []}

    def __init__(self, num_envs: int, device=None, autoreset: bool = True, env_offset: int = 0,
                 final_observation: bool = True, episode_stats: bool = True,
                 done_mask: bool = False, won_mask: bool = False, strict_actions: bool = False):
        """strict_actions: step() raises KeyError for an action outside action_dict the way the
        reference's step does (merging_env.py:101, :134-136), at the cost of one stream
        synchronisation per step; by default the kernel only flags it on the device and
        check_actions() raises later (the stream stays asynchronous)."""
        import torch

        from .. import _native

        if not torch.cuda.is_available():
            raise RuntimeError("MergeVecEnv needs a ROCm GPU (torch.cuda.is_available() is False); "
                               "there is no CPU fallback")
        if num_envs < 1:
            raise ValueError("num_envs must be >= 1")
        self._torch = torch
        self._nat = _native
        self.num_envs = int(num_envs)
        self.device = torch.device(device if device is not None else "cuda", )
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.autoreset = bool(autoreset)
        self.env_offset = int(env_offset)
        self.params = _native.default_params()
        self.params.angle0 = float(np.arctan2(1000, 30000))  # merging_env.py:49

        n, dev = self.num_envs, self.device
        f64, f32 = torch.float64, torch.float32
        specs = [("p1", (n,), f64), ("v1", (n,), f64), ("p2", (n,), f64), ("v2", (n,), f64),
                 ("ret1", (n,), f64), ("ret2", (n,), f64),
                 ("tf", (n,), torch.int16),  # uint16 bits, see MG_TF_*
                 ("obs", (n, _OBS_DIM), f32), ("rew", (n, 2), f32)]
        if _STEP_FLAGS:
            # a1, a2, done, collision interleaved per env (mg_outputs.flags): one 32-bit store per
            # env-step instead of four byte streams; the four are strided views of self.flags.
            # step()'s host actions are staged in separate contiguous buffers.
            specs += [("flags", (n, 4), torch.uint8), ("_a1_in", (n,), torch.int8), ("_a2_in", (n,), torch.int8)]
        else:
            specs += [("done", (n,), torch.uint8), ("coll", (n,), torch.uint8), ("a1_buf", (n,), torch.int8),
                      ("a2_buf", (n,), torch.int8)]
        if final_observation:
            specs.append(("final_obs", (n, _OBS_DIM), f32))
        self._arena = self._carve(specs, dev)
        if _STEP_FLAGS:
            self.a1_buf, self.a2_buf = self.flags[:, 0].view(torch.int8), self.flags[:, 1].view(torch.int8)
            self.done, self.coll = self.flags[:, 2], self.flags[:, 3]
            self.flags.zero_()
        else:
            self.flags = None
            self._a1_in, self._a2_in = self.a1_buf, self.a2_buf
        self.done.zero_()
        self.coll.zero_()
        if final_observation:
            self.final_obs.fill_(float("nan"))
        else:
            self.final_obs = None
        self.done_mask = (torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
                          if done_mask else None)
        # bit i = env i's winner == 1 after the step, before autoreset (main.py:209's store filter)
        self.won_mask = (torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
                         if won_mask else None)
        self.error = torch.zeros(1, dtype=torch.int32, device=dev)
        self.strict_actions = bool(strict_actions)
        # one 64-byte mg_episode_stats record per env (include/merging_hip.h), seen through strided
        # views: returns [N,3] f64 = sums of r1_accumulate, r2_accumulate (hdqn.py's ep_reward) and
        # main.py's winner-filtered ep_reward; ret_sum = returns[:, :2], ret_main = returns[:, 2];
        # counts [N,6] i32 = episodes, collisions, ego-first arrivals, steps, main.py:225 wins,
        # hdqn.py:342 wins
        self._ep_stats = torch.zeros((n, 8), dtype=torch.float64, device=dev) if episode_stats else None
        self._keep_pending = None  # clear_statistics' record mask
        self.returns = self._ep_stats[:, :3] if episode_stats else None
        self.ret_sum = self._ep_stats[:, :2] if episode_stats else None
        self.ret_main = self._ep_stats[:, 2] if episode_stats else None
        self.counts = self._ep_stats[:, 4:].view(torch.int32)[:, :6] if episode_stats else None
        # [N] f64: sum of each completed episode's logged Q value (q_eval_value, main.py:221 /
        # hdqn.py:330), kept by the fused policy rollouts (rollout_qnet, rollout_hdqn)
        self.q_eval = self._ep_stats[:, 7] if episode_stats else None

        ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        self._state = _native.State(*(ptr(t) for t in (self.p1, self.v1, self.p2, self.v2,
                                                        self.ret1, self.ret2, self.tf)))
        packed = self.flags is not None
        self._out = _native.Outputs(ptr(self.obs), ptr(self.rew), None if packed else ptr(self.done),
                                    None if packed else ptr(self.coll), ptr(self.done_mask),
                                    ptr(self.final_obs), None, ptr(self.error), ptr(self.won_mask),
                                    ptr(self.flags))
        self._stats = _native.Stats(ptr(self._ep_stats))
        self._flags = _native.AUTORESET if self.autoreset else 0
        self._step_idx = 0
        # pre-bound call arguments: a step costs one ctypes call and no allocations
        self._p_ref, self._s_ref = ctypes.byref(self.params), ctypes.byref(self._state)
        self._o_ref, self._st_ref = ctypes.byref(self._out), ctypes.byref(self._stats)
        # mg_step_random's a1_out / a2_out: NULL when the actions land in self.flags
        self._a1_ptr, self._a2_ptr = (None, None) if packed else (self.a1_buf.data_ptr(), self.a2_buf.data_ptr())
        self._raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        info = {"collision": self.coll.view(torch.bool)}
        if self.final_obs is not None and self.autoreset:
            info["final_observation"] = self.final_obs
            info["terminal_observation"] = self.final_obs  # gym 0.20's key (batched here, see above)
        self._result = (self.obs, self.rew, self.done.view(torch.bool), info)

        self.single_observation_space = spaces.observation_space()
        self.single_action_space = spaces.action_space()
        self.observation_space = spaces.batched_observation_space(n)
        self.action_space = spaces.batched_action_space(n)
        self.reset()

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        """Raw handle of torch's current stream on this device (honours `torch.cuda.stream(...)`)."""
        if self._raw_stream is not None:
            return self._raw_stream(self.device.index)
        return self._torch.cuda.current_stream(self.device).cuda_stream

    def _actions(self, a, buf, allow_none: bool):
        torch = self._torch
        if a is None:
            if not allow_none:
                raise KeyError(None)
            return None
        if isinstance(a, torch.Tensor):
            t = a
        else:
            t = torch.as_tensor(np.asarray(a))
        if t.shape != (self.num_envs,):
            raise ValueError(f"actions must have shape ({self.num_envs},), got {tuple(t.shape)}")
        if t.dtype == torch.int8 and t.device == self.device and t.is_contiguous():
            return t
        if t.is_floating_point() or t.dtype == torch.bool:
            t = t.to(torch.int64)
        # values outside int8 must stay invalid, not wrap into {0..4}
        t = t.to(self.device, non_blocking=True)
        if t.dtype != torch.int8:
            t = torch.where((t >= -1) & (t < 5), t, torch.full_like(t, self._nat.ACTION_INVALID))
        buf.copy_(t)
        return buf

    def _outputs(self):
        return self._result

    # ------------------------------------------------------------------ gym API
    def _carve(self, specs, dev):
        """Set self.<name> to a contiguous tensor of each (name, shape, dtype), staggered in one
        allocation (see _ARENA_STAGGER). Returns the backing buffer."""
        torch = self._torch
        if _ARENA_STAGGER < 0:
            for name, shape, dt in specs:
                setattr(self, name, torch.empty(shape, dtype=dt, device=dev))
            return None
        sizes = [int(np.prod(shape)) * torch.empty((), dtype=dt).element_size() for _, shape, dt in specs]
        offs, off = [], 0
        for nb in sizes:
            offs.append(off)
            off = (off + nb + _ARENA_STAGGER + 255) // 256 * 256
        arena = torch.empty(off, dtype=torch.uint8, device=dev)
        for (name, shape, dt), o, nb in zip(specs, offs, sizes):
            setattr(self, name, arena[o:o + nb].view(dt).view(shape))
        return arena

    def reset(self, mask=None):
        """Reset all envs (mask None) or those where mask is true; returns obs [N,10] f32.
        merging_env.py:208-230. rollout_hdqn's per-env loop state restarts with the episode, as
        hdqn.py's outer loop does after env.reset() (:277-286): no goal yet (the next launch's
        meta-net chooses one on the reset state) and a zero extrinsic-reward sum."""
        m = None
        mt = None
        if mask is not None:
            mt = self._torch.as_tensor(mask, device=self.device).to(self._torch.uint8).contiguous()
            self._mask_keepalive = mt
            m = ctypes.c_void_p(mt.data_ptr())
        for name, fresh in (("hdqn_goal", -1), ("hdqn_goal_op", -1), ("hdqn_ext", 0)):
            t = getattr(self, name, None)
            if t is not None:
                if mt is None:
                    t.fill_(fresh)
                else:
                    t.masked_fill_(mt.bool(), fresh)
        out = self._nat.Outputs(self._out.obs)
        self._nat.check(self._nat.lib.mg_reset(ctypes.byref(self.params), ctypes.byref(self._state),
                                               m, ctypes.byref(out), self.num_envs,
                                               ctypes.c_void_p(self._stream())),
                        "mg_reset")
        if mask is None:
            self.done.zero_()
            self.coll.zero_()
        return self.obs

    def step(self, actions1, actions2=None):
        """One step of every env: merging_env.py:138-195 batched. actions2=None is the
        reference's L0 opponent (constant speed); per-env -1 also means None."""
        a1 = self._actions(actions1, self._a1_in, allow_none=False)
        a2 = self._actions(actions2, self._a2_in, allow_none=True)
        rc = self._nat.lib.mg_step(
            self._p_ref, self._s_ref, a1.data_ptr(), None if a2 is None else a2.data_ptr(),
            self._o_ref, self._st_ref, self.num_envs, self._flags, self._stream())
        self._nat.check(rc, "mg_step")
        if self.strict_actions:
            self.check_actions()
        return self._outputs()

    def step_random(self, seed: int, opponent_random: bool = True, step_idx=None,
                    record_actions: bool = True):
        """One step with actions drawn on the GPU (word (step div 2) mod 4 of Philox4x32-10 keyed by
        seed, counter = (global env index, step index div 8), two draws per word; mg_step_random,
        include/merging_hip.h). The actions used land in
        self.a1_buf / a2_buf (always, when they are views of self.flags)."""
        k = self._step_idx if step_idx is None else int(step_idx)
        rc = self._nat.lib.mg_step_random(
            self._p_ref, self._s_ref, self._a1_ptr if record_actions else None,
            self._a2_ptr if record_actions else None, self._o_ref, self._st_ref, self.num_envs,
            self.env_offset, seed & 0xFFFFFFFFFFFFFFFF, k & 0xFFFFFFFFFFFFFFFF,
            1 if opponent_random else 0, self._flags, self._stream())
        self._nat.check(rc, "mg_step_random")
        self._step_idx = k + 1
        return self._outputs()

    def rollout_random(self, num_steps: int, seed: int, opponent_random: bool = True,
                       first_step=None, final_observation: bool = True, won_mask: bool = True):
        """`num_steps` steps with device-drawn actions in ONE kernel launch (the env stays in
        registers; its state is read and written once). Bit-identical to `num_steps` calls of
        step_random(seed, step_idx=first_step + t). Returns a dict of [T, N, ...] tensors:
        obs, rew, done (bool), collision (bool), a1, a2, final_observation (rows where done)
        and won_mask ([T, ceil(N/64)] int64, bit i of step t = env i's winner == 1 after that
        step -- ReplayRing.store_rollout's filter; None with won_mask=False, which saves a
        ballot and a store per wave-step). a1, a2, done and collision are strided views of one
        [T, N, 4] uint8 buffer, returned as "flags" (one 32-bit store per env-step in the
        kernel). The buffers are reused by the next rollout with the same T and output choices.
        A launch keeps each env's episode counts in 16-bit registers, so mg_rollout_random takes at
        most 65,535 steps: longer rollouts run as consecutive launches into slices of the same
        buffers, bit-identical to one launch (the step index keys the draws)."""
        nat = self._nat
        T, n = int(num_steps), self.num_envs
        k0 = self._step_idx if first_step is None else int(first_step)
        buf = self._traj(T, final_observation, won_mask)
        for t0 in range(0, max(T, 1), _MAX_ROLLOUT_STEPS):
            tc = min(_MAX_ROLLOUT_STEPS, T - t0)
            traj = buf["_traj"] if t0 == 0 else self._traj_slice(buf, t0)
            rc = nat.lib.mg_rollout_random(
                self._p_ref, self._s_ref, ctypes.byref(traj), self._st_ref, n, self.env_offset,
                seed & 0xFFFFFFFFFFFFFFFF, (k0 + t0) & 0xFFFFFFFFFFFFFFFF, tc, 1 if opponent_random else 0,
                self._flags, self._stream())
            nat.check(rc, "mg_rollout_random")
        self._step_idx = k0 + T
        return buf["_result"]

    def _traj_slice(self, buf, t0):
        """mg_traj of the trajectory buffers from step t0 on (a chunk of a long rollout)."""
        n = self.num_envs
        ptr = lambda t, row: None if t is None else t.data_ptr() + t0 * row  # noqa: E731
        return self._nat.Traj(ptr(buf["obs"], n * _OBS_DIM * 4), ptr(buf["rew"], n * 8), None, None, None, None,
                              ptr(buf["final_observation"], n * _OBS_DIM * 4), ptr(buf["won_mask"], (n + 63) // 64 * 8),
                              ptr(buf["flags"], n * 4))

    def _traj(self, T, final_observation, won_mask=True):
        """[T, N, ...] trajectory buffers, reused while T and the output choices stay the same."""
        torch, nat, n = self._torch, self._nat, self.num_envs
        buf = getattr(self, "_traj_bufs", None)
        if (buf is None or buf["T"] != T or (buf["final_observation"] is None) == final_observation
                or (buf["won_mask"] is None) == won_mask):
            dev = self.device
            # a1, a2, done, collision interleaved per env-step (mg_traj.flags): one 32-bit store
            # per env-step instead of four byte stores; the four outputs are strided views
            flags = torch.empty((T, n, 4), dtype=torch.uint8, device=dev)
            buf = {"T": T,
                   "obs": torch.empty((T, n, _OBS_DIM), dtype=torch.float32, device=dev),
                   "rew": torch.empty((T, n, 2), dtype=torch.float32, device=dev),
                   "flags": flags,
                   "final_observation": (torch.full((T, n, _OBS_DIM), float("nan"), dtype=torch.float32,
                                                    device=dev) if final_observation else None),
                   "won_mask": (torch.zeros((T, (n + 63) // 64), dtype=torch.int64, device=dev)
                                if won_mask else None)}
            ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
            buf["_traj"] = nat.Traj(ptr(buf["obs"]), ptr(buf["rew"]), None, None, None, None,
                                    ptr(buf["final_observation"]), ptr(buf["won_mask"]), ptr(flags))
            buf["_result"] = {"obs": buf["obs"], "rew": buf["rew"], "done": flags[..., 2].view(torch.bool),
                              "collision": flags[..., 3].view(torch.bool), "a1": flags[..., 0].view(torch.int8),
                              "a2": flags[..., 1].view(torch.int8), "final_observation": buf["final_observation"],
                              "won_mask": buf["won_mask"], "flags": flags}
            self._traj_bufs = buf
        return buf

    def rollout_qnet(self, num_steps: int, qnet, seed: int, opponent: str = "none",
                     episilo: float = 0.7, opp_episilo: float = 0.7, first_step=None,
                     final_observation: bool = True, won_mask: bool = True):
        """`num_steps` steps with the reference's epsilon-greedy DQN policy (main.py:99-112)
        computed on the device (bf16 MFMA) and fused with the env step, one launch.
        opponent: "none" (L0), "uniform", "self" (the same net on the swapped observation,
        main.py:199, Strategy_OP "selfplay"), or another QNet with the same out_dim (main.py's
        default Strategy_OP "L1", :161-168: a separately trained DQN acting epsilon-greedily on
        the swapped observation). Returns the same [T, N, ...] dict as rollout_random."""
        from ..policy import greedy_threshold

        torch, nat = self._torch, self._nat
        T, n = int(num_steps), self.num_envs
        opp_net = None
        if isinstance(opponent, str):
            mode = {"none": 0, "uniform": 1, "self": 2}[opponent]
        else:  # a QNet: the opponent's own DQN
            mode, opp_net = 3, opponent
            if opp_net.in_dim != _OBS_DIM or opp_net.out_dim != qnet.out_dim:
                raise ValueError("the opponent's net needs in_dim 10 and the ego net's out_dim")
        if qnet.in_dim != _OBS_DIM:
            raise ValueError("the fused rollout feeds the 10-value observation: the net needs in_dim 10")
        k0 = self._step_idx if first_step is None else int(first_step)
        buf = self._traj(T, final_observation, won_mask)
        rc = nat.lib.mg_rollout_qnet(
            self._p_ref, self._s_ref, ctypes.byref(buf["_traj"]), self._st_ref, n, self.env_offset,
            seed & 0xFFFFFFFFFFFFFFFF, k0 & 0xFFFFFFFFFFFFFFFF, T, qnet.packed.data_ptr(), qnet.out_dim,
            greedy_threshold(episilo), mode, greedy_threshold(opp_episilo),
            None if opp_net is None else opp_net.packed.data_ptr(), self._flags, self._stream())
        nat.check(rc, "mg_rollout_qnet")
        self._step_idx = k0 + T
        return buf["_result"]

    def rollout_hdqn(self, num_steps: int, meta, lower, seed: int, opponent="none",
                     episilo: float = 0.7, first_step=None, final_observation: bool = True,
                     won_mask: bool = False, ring=None, goal_memory: bool = False):
        """`num_steps` steps of hdqn.py's inner loop (scripts/hdqn.py:280-323) in one launch:
        Goal_DQN's meta-net (`meta`, a QNet 10 -> num_goals) picks each env's sub-goal on every
        next state, the lower-level Net (`lower`, a QNet 11 -> 5) acts epsilon-greedily on the
        goal state [goal] + state, goal_status gives the intrinsic reward, and a fresh goal is
        chosen once a goal is reached or an episode ends. opponent: "none" (L0, hdqn.py's default
        Strategy_OP), "uniform", or "self" (Strategy_OP "selfplay", :262-264: the same two nets
        choose the opponent's goal on the swapped state at every outer-loop iteration, :285, and
        its action on [goal_op] + swapped state, :299-300), or a (meta_op, lower_op) pair of
        QNets from another h-DQN checkpoint (any other Strategy_OP, :265-268: Goal_DQN and HDQN
        loaded from load_path_op, acting the same way). Each env's current goal persists across
        launches in `self.hdqn_goal` ([N] int8, -1 = none yet), the opponent's in
        `self.hdqn_goal_op`. Returns rollout_random's [T, N, ...] dict plus "goal",
        "next_goal" and "reward" ([T, N] fp32: the goal columns and the intrinsic reward of
        HDQN.store_transition's rows, :316 -- ReplayRing(goal=True).store_rollout takes them as
        they are), and with an h-DQN opponent "goal_op" ([T, N] fp32, the opponent's goal of each
        step). ring: a ReplayRing(goal=True) the same launch appends every
        transition to (hdqn.py:316 stores them all, so the kernel needs no scan): the rows
        store_rollout(obs0, traj, skip_ego_won=False, goal=..., next_goal=..., reward=...) would
        write, without re-reading the trajectory. goal_memory: also return "ext_reward" ([T, N]
        fp32, the extrinsic reward summed since each env's inner loop began, :286, :311-313) and
        "no_break" ([T, ceil(N/64)] int64 bits: the step did not end the inner loop, :322), from
        which ReplayRing.store_meta appends Goal_DQN's rows (:325); the running sums persist in
        `self.hdqn_ext` ([N] f64, checkpointed)."""
        from ..policy import greedy_threshold

        torch, nat = self._torch, self._nat
        T, n = int(num_steps), self.num_envs
        opp_meta = opp_lower = None
        if isinstance(opponent, (tuple, list)):
            opp_meta, opp_lower = opponent
            if (opp_meta.in_dim != _OBS_DIM or opp_meta.out_dim != meta.out_dim or opp_lower.in_dim != _OBS_DIM + 1
                    or opp_lower.out_dim != nat.NUM_ACTIONS):
                raise ValueError("the opponent's nets must be shaped like meta and lower (10 -> goals, 11 -> 5)")
            mode = 3
        else:
            mode = {"none": 0, "uniform": 1, "self": 2}[opponent]
        if ring is not None and (not ring.goal or ring.device != self.device):
            raise ValueError("the fused store needs a goal ring (ReplayRing(goal=True)) on this env's device")
        if meta.in_dim != _OBS_DIM or lower.in_dim != _OBS_DIM + 1 or lower.out_dim != nat.NUM_ACTIONS:
            raise ValueError("need hdqn.py's nets: meta-net in_dim 10, lower-level Net in_dim 11 -> 5")
        k0 = self._step_idx if first_step is None else int(first_step)
        buf = self._traj(T, final_observation, won_mask)
        hb = getattr(self, "_hdqn_bufs", None)
        if hb is None or hb["goal"].shape[0] != T:
            hb = {k: torch.empty((T, n), dtype=torch.float32, device=self.device)
                  for k in ("goal", "next_goal", "reward", "goal_op", "ext_reward")}
            hb["no_break"] = torch.empty((T, (n + 63) // 64), dtype=torch.int64, device=self.device)
            hb["_h"] = nat.HdqnTraj(*(hb[k].data_ptr() for k in ("goal", "next_goal", "reward", "goal_op")))
            hb["_hm"] = nat.HdqnTraj(*(hb[k].data_ptr() for k in ("goal", "next_goal", "reward", "goal_op",
                                                                   "ext_reward", "no_break")))
            self._hdqn_bufs = hb
        if not self.autoreset:
            raise ValueError("rollout_hdqn runs hdqn.py's loop, which resets every finished episode: "
                             "it needs MergeVecEnv(autoreset=True)")
        if getattr(self, "hdqn_ext", None) is None:
            # the extrinsic-reward sums are kept from the first launch on, whether or not this
            # launch returns Goal_DQN's columns, so turning goal_memory on later is consistent
            self.hdqn_ext = torch.zeros(n, dtype=torch.float64, device=self.device)
        if getattr(self, "hdqn_goal", None) is None:
            self.hdqn_goal = torch.full((n,), -1, dtype=torch.int8, device=self.device)
        if mode >= 2 and getattr(self, "hdqn_goal_op", None) is None:
            self.hdqn_goal_op = torch.full((n,), -1, dtype=torch.int8, device=self.device)
        gop = getattr(self, "hdqn_goal_op", None)
        ext = self.hdqn_ext
        rc = nat.lib.mg_rollout_hdqn(
            self._p_ref, self._s_ref, ctypes.byref(buf["_traj"]), ctypes.byref(hb["_hm" if goal_memory else "_h"]),
            self._st_ref, self.hdqn_goal.data_ptr(), None if gop is None else gop.data_ptr(),
            None if ext is None else ext.data_ptr(), n, self.env_offset, seed & 0xFFFFFFFFFFFFFFFF, k0 & 0xFFFFFFFFFFFFFFFF,
            T, meta.packed.data_ptr(), meta.out_dim, lower.packed.data_ptr(), meta.reset_argmax(),
            greedy_threshold(episilo), mode, None if opp_meta is None else opp_meta.packed.data_ptr(),
            None if opp_lower is None else opp_lower.packed.data_ptr(), None if ring is None else ring.memory.data_ptr(),
            None if ring is None else ring._counter.data_ptr(), 0 if ring is None else ring.capacity,
            self._flags, self._stream())
        nat.check(rc, "mg_rollout_hdqn")
        self._step_idx = k0 + T
        out = dict(buf["_result"])
        out.update(goal=hb["goal"], next_goal=hb["next_goal"], reward=hb["reward"])
        if mode >= 2:
            out["goal_op"] = hb["goal_op"]
        if goal_memory:
            out.update(ext_reward=hb["ext_reward"], no_break=hb["no_break"])
        return out

    def gym_vector(self, obs_dtype=None, ego_reward_only=False):
        """gym 0.20's VectorEnv protocol over this env (envs/gym_vector.py): step_async / step_wait,
        numpy outputs and per-env infos with "terminal_observation" (ego_reward_only: rewards [n] of the
        ego, for stock wrappers). The device-tensor API above stays the fast path."""
        from .gym_vector import GymVectorEnv

        return GymVectorEnv(self, obs_dtype, ego_reward_only)

    def observe(self):
        """Observation of the current state without stepping (merging_env.py:118-132)."""
        out = self._nat.Outputs(self._out.obs, None, None, self._out.coll)
        out.flags = self._out.flags  # collision byte 3 of the interleaved record
        self._nat.check(self._nat.lib.mg_observe(ctypes.byref(self.params), ctypes.byref(self._state),
                                                 ctypes.byref(out), self.num_envs,
                                                 ctypes.c_void_p(self._stream())),
                        "mg_observe")
        return self.obs

    def check_actions(self):
        """Raise KeyError if any step since the last check saw an action outside the
        reference's action_dict (merging_env.py:101). Synchronises the stream."""
        err = int(self.error.item())
        if err:
            self.error.zero_()
            raise KeyError(f"invalid action in batch (a1: {bool(err & 1)}, a2: {bool(err & 2)})")

    # ------------------------------------------------------------------ state views
    @property
    def steps(self):
        return self.tf & self._nat.TF_STEPS_MASK

    @property
    def winner(self):
        return (self.tf & self._nat.TF_WINNER_MASK) >> self._nat.TF_WINNER_SHIFT

    def render_view(self, i: int, acc=(0.0, 0.0)):
        """Env i's state as envs/ui.py draws it (`MergeUI(...).render(env.render_view(i))`):
        positions, speeds and accumulated rewards of row i, read back from the device. The
        last step's accelerations are not kept on the device; `acc` stands in for
        state{1,2}['acc'], which only picks the cars' colour (merging_env.py:270-288). A row
        that has not stepped since its reset has the reference's reset types (int 50, int 0)."""
        i = int(i)
        if not 0 <= i < self.num_envs:
            raise IndexError(f"env {i} out of range [0, {self.num_envs})")
        torch = self._torch
        row = torch.stack([t[i] for t in (self.p1, self.v1, self.p2, self.v2, self.ret1, self.ret2)])
        p1, v1, p2, v2, r1, r2 = (float(x) for x in row.cpu())
        if int(self.tf[i].item()) & self._nat.TF_STEPS_MASK == 0 and (p1, p2, r1, r2) == (50.0, 50.0, 0.0, 0.0):
            p1 = p2 = 50
            r1 = r2 = 0
        return {"pos1": p1, "vel1": v1, "acc1": float(acc[0]), "pos2": p2, "vel2": v2,
                "acc2": float(acc[1]), "r1": r1, "r2": r2}

    def episode_statistics(self):
        """Completed-episode totals per env (views of the device records): "returns" [N,3] f64
        (sums of r1_accumulate = hdqn.py's ep_reward, r2_accumulate, main.py's winner-filtered
        ep_reward, scripts/main.py:209-211), "ret_sum" = returns[:, :2], "ret_main" =
        returns[:, 2], "counts" [N,6] i32 (episodes, collisions, ego-first arrivals, steps,
        main.py:225 wins, hdqn.py:342 wins), "q_eval" [N] f64 (the sum of the Q value logged per
        episode by the fused policy rollouts: main.py:221, hdqn.py:330)."""
        return {"returns": self.returns, "ret_sum": self.ret_sum, "ret_main": self.ret_main,
                "counts": self.counts, "q_eval": self.q_eval}

    def episode_summary(self):
        """This batch's completed episodes summarised as the scripts log them (distributed.summarize:
        rates, mean rewards, mean_q_eval), reduced on the device by mg_stats_reduce."""
        from ..distributed import summarize

        if self.returns is None:
            raise ValueError("built with episode_stats=False")
        return summarize(self.returns, self.counts)

    def clear_statistics(self):
        """Zero the sums and counts (each env's pending main.py value stays: it belongs to the
        episode in progress)."""
        if self.ret_sum is not None:
            # one pass over whole 64-byte records (an int64 multiply by 0 / 1 keeps ret1_pending's
            # bits): zeroing the strided fields instead (three fills of partial lines) slowed the
            # step launches that followed by up to 6 % until every env had finished an episode
            # (2^22 envs, tools/size2_probe2.py, DESIGN.md section 4 "The 2^22 first window")
            if self._keep_pending is None:
                self._keep_pending = self._torch.tensor([0, 0, 0, 1, 0, 0, 0, 0], dtype=self._torch.int64,
                                                        device=self._ep_stats.device)
            self._ep_stats.view(self._torch.int64).mul_(self._keep_pending)

    # ------------------------------------------------------------------ checkpoint / resume
    _STATE_KEYS = ("p1", "v1", "p2", "v2", "ret1", "ret2", "tf")

    def state_dict(self):
        """The batch's full state as tensors (copies, on this device) plus the step index that
        keys the Philox actions: `torch.save(env.state_dict(), path)` checkpoints a run, and
        `load_state_dict` resumes it bit for bit (the reference keeps no env checkpoint; its
        scripts save only the agents, main.py:244-245, hdqn.py:362-366)."""
        sd = {k: getattr(self, k).clone() for k in self._STATE_KEYS}
        sd["step_idx"] = self._step_idx
        sd["env_offset"] = self.env_offset
        if self.ret_sum is not None:
            sd["episode_stats"] = self._ep_stats.clone()  # the 64-byte records, pending value included
            sd["episode_stats_format"] = self._nat.EPISODE_STATS_FORMAT
        if getattr(self, "hdqn_goal", None) is not None:
            sd["hdqn_goal"] = self.hdqn_goal.clone()  # rollout_hdqn's current goals
        if getattr(self, "hdqn_goal_op", None) is not None:
            sd["hdqn_goal_op"] = self.hdqn_goal_op.clone()  # and the self-play opponent's
        if getattr(self, "hdqn_ext", None) is not None:
            sd["hdqn_ext"] = self.hdqn_ext.clone()  # extrinsic reward of the running inner loops
        return sd

    def load_state_dict(self, sd):
        for k in self._STATE_KEYS:
            src = self._torch.as_tensor(sd[k])
            dst = getattr(self, k)
            if tuple(src.shape) != tuple(dst.shape) or src.dtype != dst.dtype:
                raise ValueError(f"{k}: expected {tuple(dst.shape)} {dst.dtype}, got {tuple(src.shape)} {src.dtype}")
            dst.copy_(src)  # in place: the kernels hold these buffers' addresses
        if int(sd.get("env_offset", self.env_offset)) != self.env_offset:
            raise ValueError("the checkpoint is of another env shard (env_offset differs)")
        self._step_idx = int(sd["step_idx"])
        if self.ret_sum is not None:
            self._load_episode_stats(sd)
        # rollout_hdqn's carried state as it was when the checkpoint was taken: absent = none yet (the
        # next launch chooses every env's first goals), not whatever a later launch left here
        for name, dtype in (("hdqn_goal", self._torch.int8), ("hdqn_goal_op", self._torch.int8),
                            ("hdqn_ext", self._torch.float64)):
            setattr(self, name, self._torch.as_tensor(sd[name]).to(self.device, dtype).clone() if name in sd else None)

    def _load_episode_stats(self, sd):
        """The 64-byte records of a checkpoint. ABI <= 16 checkpoints kept 'ret_sum' / 'counts'
        arrays: main.py's filtered return and both scripts' win counts are not in them, so they are
        refused rather than loaded half. ABI 17-19 records (format 1) lack q_eval: it loads as NaN
        (unknown), so a summary over them says so instead of reporting a diluted mean."""
        if "episode_stats" not in sd:
            if "ret_sum" in sd or "counts" in sd:
                raise ValueError("checkpoint holds the ABI <= 16 statistics ('ret_sum' / 'counts'); the 64-byte "
                                 "records (ABI 17+) add main.py's filtered ep_reward and both scripts' win counts, "
                                 "which cannot be recovered: rebuild the env or load with episode_stats=False")
            raise ValueError("checkpoint holds no episode statistics ('episode_stats'): build the env with "
                             "episode_stats=False to resume it")
        self._ep_stats.copy_(self._torch.as_tensor(sd["episode_stats"]))
        if int(sd.get("episode_stats_format", 1)) < 2:
            self.q_eval.fill_(float("nan"))

    def close(self):
        pass
