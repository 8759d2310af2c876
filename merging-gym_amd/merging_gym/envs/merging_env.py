"""MergeEnv: the drop-in single env behind gym id "merging_env-v0".

Same surface as the reference's MergeEnv (merging_gym/envs/merging_env.py:72-399):
`reset() -> list[10]`, `step(action1, action2=None) -> (list[10], [r1, r2], done,
{"collision": bool})`, the attributes its callers read (`winner`, `done`, `time_stamp`,
`state1`, `state2`, `r1_accumulate`, `r2_accumulate`, `action_dict`, `action_space`,
`observation_space`, `show_reward()`) and the reference's Python value types (an int 0
reward after the winner's arrival, int 900 gaps straight after reset, ...), so
scripts/hdqn.py, scripts/main.py and scripts/human_player.py's list arithmetic
(`state[5:] + state[:5]`, `[goal] + state`) keeps working.

The step is the library's own: by default (backend "host") the kernels' step functions compiled
for the CPU (mg_host_step), one ctypes call per step -- the reference's MergeEnv is a CPU object
(BASELINE config 1) and a kernel launch plus a stream sync per step costs four times a host step;
with backend "gpu" a batch of one env in the same step kernel as MergeVecEnv. Either writes a
packed fp64 record (mg_rec64) the list API is read from. The pygame UI methods (render / plot /
intro / prepare / feedback / finish) draw that state through envs/ui.py, importing pygame at the
first UI call.
"""

from __future__ import annotations

import ctypes
import struct

import numpy as np

from .. import spaces

# merging_env.py:22-46 (the constants callers may import from the module)
R = 30000
H, W = 1000, 300
WINDOW_H, WINDOW_W = 1000, 300
dT = 0.2
RFirst = 2.0
RSecond = 1.0
RCollision = -10
vel_penalty = 0.001
time_penalty = 0
START_POINT = 50
END_POINT = H - 50
VEHICLE_W, VEHICLE_H = 4, 8
prediction_t = 3.0
scale = 5.0

try:  # pragma: no cover - gym is not installed in this image
    import gym as _gym

    _EnvBase = _gym.Env
except Exception:  # noqa: BLE001
    class _EnvBase:  # minimal gym.Env stand-in: the attributes callers touch
        metadata = {"render.modes": []}

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass

        def seed(self, seed=None):
            return [seed]


class _HostStep:
    """The step on the host (mg_host_step / mg_host_reset / mg_host_observe): the kernels' own step
    functions compiled for the CPU, on a host-memory env. One ctypes call per step, no device."""

    def __init__(self, nat, params):
        c = ctypes
        self._nat, self.params = nat, params
        self._st = (c.c_double * 6)()              # p1 v1 p2 v2 ret1 ret2
        self._tf = (c.c_uint16 * 1)()
        self._a = (c.c_int8 * 2)()
        self._coll = (c.c_uint8 * 1)()
        self._err = (c.c_int32 * 1)()
        self.rec = nat.Rec64()
        base = c.addressof(self._st)
        self._state = nat.State(*(c.c_void_p(base + 8 * k) for k in range(6)), c.c_void_p(c.addressof(self._tf)))
        self._out = nat.Outputs(None, None, None, None, None, None, c.c_void_p(c.addressof(self.rec)),
                                c.c_void_p(c.addressof(self._err)))
        self._obs_out = nat.Outputs(None, None, None, c.c_void_p(c.addressof(self._coll)), None, None,
                                    c.c_void_p(c.addressof(self.rec)), None)
        P, S = c.byref(params), c.byref(self._state)
        a1 = c.c_void_p(c.addressof(self._a))
        a2 = c.c_void_p(c.addressof(self._a) + 1)
        self._stats = nat.Stats(None)
        self._step_args = (P, S, a1, a2, c.byref(self._out), c.byref(self._stats), 1, 0)
        self._reset_args = (P, S, None, c.byref(self._out), 1)
        self._obs_args = (P, S, c.byref(self._obs_out), 1)

    def push(self, vals, tf):
        self._st[:] = vals
        self._tf[0] = tf

    def reset(self):
        self._nat.check(self._nat.lib.mg_host_reset(*self._reset_args), "mg_host_reset")
        return self.rec

    def step(self, c1, c2):
        a = self._a
        a[0], a[1] = c1, c2
        rc = self._nat.lib.mg_host_step(*self._step_args)
        if rc:
            self._nat.check(rc, "mg_host_step")
        return self.rec

    def after_error(self):
        self._err[0] = 0
        return self._st[0], self._st[1], self._tf[0]

    def observe(self):
        self._nat.check(self._nat.lib.mg_host_observe(*self._obs_args), "mg_host_observe")
        return self.rec, bool(self._coll[0])


class _GpuStep:
    """The step on the GPU: a batch of one env in the step kernel (mg_step), its packed fp64 record
    copied back once per call. zero_copy: the kernel reads the two actions from, and writes its
    168-byte record to, pinned host memory (device-addressable on ROCm) -- one launch and one stream
    sync per step instead of two copies around the launch."""

    def __init__(self, nat, params, device, zero_copy):
        import torch

        self._torch, self._nat, self.params, self.device = torch, nat, params, device
        dev = device
        self._dstate = torch.zeros(7, dtype=torch.float64, device=dev)  # p1 v1 p2 v2 ret1 ret2 tf
        self._rec_dev = torch.zeros(nat.REC64_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        self._rec_host = torch.zeros(nat.REC64_DTYPE.itemsize, dtype=torch.uint8).pin_memory()
        self.rec = nat.Rec64.from_address(self._rec_host.data_ptr())
        self._a_dev = torch.zeros(2, dtype=torch.int8, device=dev)
        self._a_host = torch.zeros(2, dtype=torch.int8).pin_memory()
        self._coll_dev = torch.zeros(8, dtype=torch.uint8, device=dev)
        self._err = torch.zeros(1, dtype=torch.int32, device=dev)
        base = self._dstate.data_ptr()
        self._state = nat.State(*(ctypes.c_void_p(base + 8 * k) for k in range(7)))
        self._out = nat.Outputs(None, None, None, None, None, None, ctypes.c_void_p(self._rec_dev.data_ptr()),
                                ctypes.c_void_p(self._err.data_ptr()))
        self._stats = nat.Stats(None)
        self._a1 = ctypes.c_void_p(self._a_dev.data_ptr())
        self._a2 = ctypes.c_void_p(self._a_dev.data_ptr() + 1)
        self._zero_copy = bool(zero_copy)
        if self._zero_copy:
            self._a1 = ctypes.c_void_p(self._a_host.data_ptr())
            self._a2 = ctypes.c_void_p(self._a_host.data_ptr() + 1)
            self._out_zc = nat.Outputs(None, None, None, None, None, None,
                                       ctypes.c_void_p(self._rec_host.data_ptr()),
                                       ctypes.c_void_p(self._err.data_ptr()))

    def _stream(self):
        return self._torch.cuda.current_stream(self.device)

    def _fetch(self):
        self._rec_host.copy_(self._rec_dev, non_blocking=True)
        self._stream().synchronize()
        return self.rec

    def push(self, vals, tf):
        host = np.array(list(vals) + [0.0], dtype=np.float64)
        host[6:7].view(np.uint16)[0] = tf
        self._dstate.copy_(self._torch.from_numpy(host))

    def reset(self):
        nat = self._nat
        nat.check(nat.lib.mg_reset(ctypes.byref(self.params), ctypes.byref(self._state), None,
                                   ctypes.byref(self._out), 1, ctypes.c_void_p(self._stream().cuda_stream)),
                  "mg_reset")
        return self._fetch()

    def step(self, c1, c2):
        nat = self._nat
        stream = self._stream()
        if self._zero_copy:
            stream.synchronize()  # the previous launch has read the host action bytes
            a = self._a_host.numpy()
            a[0], a[1] = c1, c2
            out = self._out_zc
        else:
            self._a_host[0], self._a_host[1] = c1, c2
            self._a_dev.copy_(self._a_host, non_blocking=True)
            out = self._out
        nat.check(nat.lib.mg_step(ctypes.byref(self.params), ctypes.byref(self._state), self._a1, self._a2,
                                  ctypes.byref(out), ctypes.byref(self._stats), 1, 0,
                                  ctypes.c_void_p(stream.cuda_stream)), "mg_step")
        if c1 == nat.ACTION_INVALID or c2 == nat.ACTION_INVALID:
            return None
        if self._zero_copy:
            stream.synchronize()
            return self.rec
        return self._fetch()

    def after_error(self):
        self._err.zero_()
        st = self._dstate.cpu().numpy()
        return float(st[0]), float(st[1]), int(st[6:7].view(np.uint16)[0])

    def observe(self):
        nat = self._nat
        out = nat.Outputs(None, None, None, ctypes.c_void_p(self._coll_dev.data_ptr()), None, None,
                          self._out.rec64, None)
        nat.check(nat.lib.mg_observe(ctypes.byref(self.params), ctypes.byref(self._state), ctypes.byref(out), 1,
                                     ctypes.c_void_p(self._stream().cuda_stream)), "mg_observe")
        rec = self._fetch()
        return rec, bool(self._coll_dev[0].item())


class MergeEnv(_EnvBase):
    """The reference's single MergeEnv with its list API, stepped by the library's own step code.

    backend "host" (the default for this one env): mg_host_step, the kernels' step functions
    compiled for the CPU, one ctypes call per step and no device -- BASELINE config 1 is a CPU
    single env, and scripts/human_player.py's 20 Hz keyboard loop needs no GPU. Measured per step
    (bench.py `dropin_single_env`): the host path ~7 us, the GPU path ~28 us (a launch plus a stream
    synchronisation per step), the reference-style Python step ~11 us. backend "gpu" (or any
    `device` given): the same step as a batch of one env in the step kernel (mg_step). Both give the
    same doubles bit for bit wherever |theta| < 1/16, i.e. positions below about 2,875 m. A live
    episode does go further: a car that has arrived keeps driving (up to 8 m per step) while the other
    car runs the episode to the 2501-step timeout, to about 20 km. There sin / cos come from glibc on
    the host and from the device library on the GPU, and an observation may differ by an ulp
    between the two backends, and from the reference's numpy values (a known divergence; positions,
    speeds, rewards and flags stay equal; tests/test_host_step.py). Batches belong in MergeVecEnv,
    which is GPU-only.
    """

    def __init__(self, device=None, zero_copy: bool = True, backend: str | None = None):
        super().__init__()
        from .. import _native

        if backend is None:
            backend = "host" if device is None else "gpu"
        if backend not in ("host", "gpu"):
            raise ValueError(f"backend must be 'host' or 'gpu', not {backend!r}")
        self._nat = _native
        self.backend = backend

        self.observation_shape = (10)
        self.observation_space = spaces.observation_space()
        self.action_dict = {0: 0, 1: 10, 2: 20, 3: 30, 4: 40}
        self.action_space = spaces.action_space(len(self.action_dict.items()))
        self.action1 = 1
        self.action2 = 1

        self.params = _native.default_params()
        self.params.angle0 = float(np.arctan2(H, R))
        if backend == "host":
            self.device = None
            self._be = _HostStep(_native, self.params)
        else:
            import torch

            if not torch.cuda.is_available():
                raise RuntimeError("MergeEnv(backend='gpu') runs its step on a ROCm GPU "
                                   "(torch.cuda.is_available() is False); there is no CPU fallback "
                                   "for the GPU backend (backend='host' is the CPU single env)")
            self.device = torch.device(device if device is not None else "cuda")
            if self.device.index is None:
                self.device = torch.device("cuda", torch.cuda.current_device())
            self._be = _GpuStep(_native, self.params, self.device, zero_copy)

        self._time, self._steps, self._dirty = 0, 0, False
        self._ui = None
        self.reset()

    # ------------------------------------------------------------------ plumbing
    def _push(self):
        """Write the host-side attributes (after a caller assigned state1, winner, ...) to the
        env state, like assigning the reference's attributes between steps."""
        nat = self._nat
        tf = (self._steps & nat.TF_STEPS_MASK) | ((0 if self._winner is None else int(self._winner))
                                                  << nat.TF_WINNER_SHIFT)
        tf |= nat.TF_DONE if self._done else 0
        self._be.push((float(self._s1["pos"]), float(self._s1["vel"]), float(self._s2["pos"]),
                       float(self._s2["vel"]), float(self._r1acc), float(self._r2acc)), tf)
        self._dirty = False

    def _apply(self, rec):
        nat = self._nat
        v = _REC64.unpack_from(rec)  # one read of the whole mg_rec64 (ctypes field access costs ~4x)
        tf, st = v[20], v[21]
        w = (tf & nat.TF_WINNER_MASK) >> nat.TF_WINNER_SHIFT
        self._winner = None if w == 0 else w
        self._done = bool(tf & nat.TF_DONE)
        self._steps = tf & nat.TF_STEPS_MASK
        obs = list(v[:10])
        v1 = 0 if st & nat.ST_V1_INT else v[16]
        v2 = 0 if st & nat.ST_V2_INT else v[17]
        if st & nat.ST_V1_INT:
            obs[4] = 0
        if st & nat.ST_V2_INT:
            obs[9] = 0
        self._s1 = {"pos": v[14], "vel": v1, "acc": v[12]}
        self._s2 = {"pos": v[15], "vel": v2, "acc": 0 if self.action2 is None else v[13]}
        r1 = int(v[10]) if st & nat.ST_R1_INT else v[10]
        r2 = int(v[11]) if st & nat.ST_R2_INT else v[11]
        # r_accumulate summed in fp64 in the reference's order; an int history stays int
        self._r1acc = _keep_int(self._r1acc, r1, v[18])
        self._r2acc = _keep_int(self._r2acc, r2, v[19])
        return obs, [r1, r2], bool(st & nat.ST_DONE), {"collision": bool(st & nat.ST_COLLISION)}

    # ------------------------------------------------------------------ reference attributes
    def _attr(name):  # noqa: N805 - property factory
        def get(self):
            return getattr(self, name)

        def put(self, v):
            setattr(self, name, v)
            self._dirty = True

        return property(get, put)

    state1 = _attr("_s1")
    state2 = _attr("_s2")
    winner = _attr("_winner")
    done = _attr("_done")
    r1_accumulate = _attr("_r1acc")
    r2_accumulate = _attr("_r2acc")
    del _attr

    @property
    def time_stamp(self):
        return self._time

    @time_stamp.setter
    def time_stamp(self, t):
        # the device counts steps; the fp64 clock exceeds 500 exactly from step 2501
        self._time = t
        self._steps = int(round(float(t) / dT))
        self._dirty = True

    # ------------------------------------------------------------------ reference API
    def show_reward(self):
        return RFirst, RSecond, RCollision, vel_penalty

    def reset(self):
        """merging_env.py:208-230 (mg_host_reset, or mg_reset on the GPU)."""
        rec = self._be.reset()
        self._done, self._winner, self._time, self._steps = False, None, 0, 0
        self._s1 = {"pos": START_POINT, "vel": 20.0, "acc": 0.0}
        self._s2 = {"pos": START_POINT, "vel": 20.0, "acc": 0.0}
        self._r1acc = self._r2acc = 0
        self._dirty = False
        obs = rec.obs[:]
        obs[3], obs[8] = int(obs[3]), int(obs[8])  # END_POINT - START_POINT: ints, as the reference
        return obs

    def step(self, action1, action2=None):
        """merging_env.py:138-195 (mg_host_step, or mg_step on the GPU: one env)."""
        nat = self._nat
        if self._dirty:
            self._push()
        self.action1, self.action2 = action1, action2
        c1 = _ACTION_CODE.get(action1, nat.ACTION_INVALID)
        c2 = nat.ACTION_NONE if action2 is None else _ACTION_CODE.get(action2, nat.ACTION_INVALID)
        self._time += dT
        rec = self._be.step(c1, c2)
        if c1 == nat.ACTION_INVALID or c2 == nat.ACTION_INVALID:
            self._sync_after_error()
            raise KeyError(action1 if c1 == nat.ACTION_INVALID else action2)
        return self._apply(rec)

    def _sync_after_error(self):
        # the step advanced the clock (and the ego when only action2 was bad) as the
        # reference does before its KeyError; refresh the host mirror from the env state
        p1, v1, tf = self._be.after_error()
        self._done = bool(tf & self._nat.TF_DONE)
        self._steps = tf & self._nat.TF_STEPS_MASK
        self._s1 = dict(self._s1, pos=p1, vel=v1)

    def observe(self):
        """merging_env.py:118-132: observation of the current state (no state change)."""
        if self._dirty:
            self._push()
        return self._be.observe()[0].obs[:]

    def is_collided(self):
        """merging_env.py:198-206 (no state change)."""
        if self._dirty:
            self._push()
        return self._be.observe()[1]

    # ------------------------------------------------------------------ UI (pygame, lazy)
    @property
    def ui(self):
        """The pygame window (envs/ui.py MergeUI), created at the first UI call -- the
        reference opens it in __init__ (:83-108); here the step path never touches pygame."""
        if self._ui is None:
            from .ui import MergeUI

            self._ui = MergeUI()
        return self._ui

    @ui.setter
    def ui(self, value):
        self._ui = value

    def render_view(self):
        """The state render() draws: the host mirror of the device step record (or what a
        caller assigned to state1 / state2 / r*_accumulate since)."""
        return {"pos1": self._s1["pos"], "vel1": self._s1["vel"], "acc1": self._s1["acc"],
                "pos2": self._s2["pos"], "vel2": self._s2["vel"], "acc2": self._s2["acc"],
                "r1": self._r1acc, "r2": self._r2acc}

    def render(self, goal=None, goal_op=None, player=1, sum_r1=0, sum_r2=0, tag_left=None,
               tag_right=None, last_r1=0, last_r2=0):
        """merging_env.py:241-342 (sum_r* / last_r* are accepted and unused, as there)."""
        self.ui.render(self.render_view(), goal, goal_op, player, tag_left, tag_right)

    def plot(self, player=1):
        self.ui.plot(player)

    def intro(self, player=1):
        self.ui.intro(player)

    def prepare(self, player=1):
        self.ui.prepare(player)

    def feedback(self, player=1):
        self.ui.feedback(self._r1acc, self._r2acc, player)

    def finish(self, sum_r1, sum_r2, player=1):
        self.ui.finish(sum_r1, sum_r2, player)

    def close(self):
        pass  # the reference's close() is cv2.destroyAllWindows() (:398-399): no cv2 window here


_REC64 = struct.Struct("=20d2I")  # struct mg_rec64: obs[10] rew[2] acc[2] pos[2] vel[2] ret[2] tf status
_ACTION_CODE = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4}  # keys of action_dict (merging_env.py:101)


def _keep_int(prev, r, device_sum):
    if isinstance(prev, int) and isinstance(r, int):
        return prev + r
    return device_sum


class MergeEnvExtend(_EnvBase):
    """merging_env.py:404-410: the reference's print-only placeholder env."""

    def __init__(self):
        print("MergeEnvExtend Environment initialized")

    def step(self):
        print("MergeEnvExtend Step successful!")

    def reset(self):
        print("MergeEnvExtend Environment reset")
