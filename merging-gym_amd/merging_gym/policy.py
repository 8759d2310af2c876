"""The reference's DQN policy on the device: Net (scripts/main.py:30-47, scripts/hdqn.py:38-55)
and epsilon-greedy choose_action (main.py:99-112), packed for the fused bf16 MFMA kernels.

    qnet = QNet.from_state_dict(torch.load(path, weights_only=True), device="cuda:0")
    q = qnet.forward(obs)                       # [N, out_dim] fp32 (bf16 operands, fp32 sums)
    traj = env.rollout_qnet(T, qnet, seed=0)    # policy + env step fused, T steps per launch
"""

from __future__ import annotations

import math

EPISILO = 0.7  # main.py:16, hdqn.py:20 -- greedy when np.random.randn() <= EPISILO
NUM_GOALS = 3  # hdqn.py:31


def goal_status(states):
    """hdqn.py:223-237: the sub-goal an observation is in -- 0 if dx1 < -0.5 v2, 1 if dx1 < 0.5 v2,
    else 2 (dx1 = obs[0], v2 = obs[9]). One observation (10 values) gives an int, as the reference;
    a [N, 10] tensor gives int64 [N] on its device.

    Pass fp64 observations for the reference's decisions: the reference compares the Python floats
    env.step returned, and the fused h-DQN kernel compares the fp64 x2 - x1 and v2 of its state
    (mg_goal_status). On MergeVecEnv's fp32 observations the rounding of dx1 to fp32 flips the status
    of states near the thresholds (a sixth of the boundary rows in
    tests/test_gpu_episode_stats.py::test_hdqn_intrinsic_reward_uses_fp64_goal_status), so the result
    can disagree with the kernel's intrinsic rewards there; use mg_goal_status on the env's fp64
    state (the mg_observe rec64 path) when it must agree."""
    try:
        import torch

        if isinstance(states, torch.Tensor) and states.dim() == 2:
            dx1, v2 = states[:, 0], states[:, 9]
            one, two = torch.ones_like(dx1, dtype=torch.int64), torch.full_like(dx1, 2, dtype=torch.int64)
            return torch.where(dx1 < -0.5 * v2, torch.zeros_like(one), torch.where(dx1 < 0.5 * v2, one, two))
    except ImportError:  # pragma: no cover - torch is part of the image
        pass
    dx1, v2 = states[0], states[9]
    if dx1 < -0.5 * v2:
        return 0
    elif dx1 < 0.5 * v2:
        return 1
    return 2


def greedy_threshold(episilo: float = EPISILO) -> int:
    """u32 threshold t with P(u < t) = P(randn <= episilo) = Phi(episilo)."""
    phi = 0.5 * (1.0 + math.erf(episilo / math.sqrt(2.0)))
    return min(1 << 32, max(0, int(round(phi * (1 << 32)))))


class QNet:
    """A Net(in, out) with hidden sizes 200 / 100, packed on the device (bf16 weights)."""

    def __init__(self, fc1_w, fc1_b, fc2_w, fc2_b, out_w, out_b, device=None):
        import torch

        from . import _native

        self._nat = _native
        dev = torch.device(device if device is not None else "cuda")
        ts = [torch.as_tensor(t, dtype=torch.float32).to(dev).contiguous()
              for t in (fc1_w, fc1_b, fc2_w, fc2_b, out_w, out_b)]
        self.in_dim, self.out_dim = int(ts[0].shape[1]), int(ts[4].shape[0])
        if tuple(ts[0].shape) != (200, self.in_dim) or tuple(ts[2].shape) != (100, 200) or \
                tuple(ts[4].shape) != (self.out_dim, 100):
            raise ValueError("expected the reference Net: fc1 [200,in], fc2 [100,200], out [out,100]")
        self.device = dev
        self.fp32 = ts  # kept for reference checks
        self.packed = torch.empty(_native.lib.mg_qnet_packed_bytes(), dtype=torch.uint8, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        _native.check(_native.lib.mg_qnet_pack(*(t.data_ptr() for t in ts), self.in_dim, self.out_dim,
                                               self.packed.data_ptr(), stream), "mg_qnet_pack")

    @property
    def fragments(self):
        """Deprecated alias of `packed` (ABI 18 kept a separate fragment-major copy here): since ABI 19
        the packed layout begins with the fragment-major 16x16 forward mg_rollout_hdqn reads an
        opponent from another checkpoint in, so the kernels take `packed` itself and no second copy
        can go stale when `packed` changes."""
        return self.packed

    def reset_argmax(self) -> int:
        """argmax of this net on the reset observation (merging_env.py:208-230), computed once on
        the device: the greedy goal Goal_DQN picks after every episode end (hdqn.py:278-283),
        which mg_rollout_hdqn takes as a constant."""
        if getattr(self, "_reset_argmax", None) is None:
            from .envs.vector_env import MergeVecEnv

            if self.in_dim != 10:
                raise ValueError("reset_argmax needs a net on the 10-value observation")
            one = MergeVecEnv(1, device=self.device, final_observation=False, episode_stats=False)
            self._reset_argmax = int(self.forward(one.reset())[0].argmax())
        return self._reset_argmax

    @classmethod
    def from_state_dict(cls, sd, device=None):
        return cls(sd["fc1.weight"], sd["fc1.bias"], sd["fc2.weight"], sd["fc2.bias"], sd["out.weight"],
                   sd["out.bias"], device=device)

    def forward(self, obs, swap_halves: bool = False):
        """Q-values [N, out_dim] of inputs [N, in_dim] (device tensor), computed by
        mg_qnet_forward: observations for main.py's Net (in_dim 10; swap_halves feeds the
        opponent's view, main.py:199), goal states [goal] + state for hdqn.py's lower-level Net
        (in_dim 11, :145, :291), or any other width up to 13 (e.g. Goal_DQN's meta-net, 10 -> 3); the three
        input slots past 13 carry the folded first-layer bias."""
        import torch

        obs = obs.to(self.device, torch.float32).contiguous()
        if obs.dim() != 2 or obs.shape[1] != self.in_dim:
            raise ValueError(f"expected inputs [N, {self.in_dim}], got {tuple(obs.shape)}")
        if swap_halves and self.in_dim != 10:
            raise ValueError("swap_halves is the opponent's view of a 10-value observation")
        q = torch.empty((obs.shape[0], 8), dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self._nat.check(self._nat.lib.mg_qnet_forward(self.packed.data_ptr(), obs.data_ptr(), self.in_dim,
                                                      1 if swap_halves else 0, q.data_ptr(),
                                                      obs.shape[0], stream), "mg_qnet_forward")
        return q[:, : self.out_dim]
