"""CPU oracle for the MergingEnv step path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker or the timed CPU baseline. The product (merging_gym) never calls it:
its step runs in libmerging_hip.so and fails loudly without it.

Two restatements of the reference algorithm live here:

* ``PyMergeEnv`` -- a scalar, pure-Python env with the reference's list API and its exact
  Python value types (int 0 rewards, int 900 gaps after reset, ...). It follows
  merging_gym/envs/merging_env.py (reference @ /root/reference) function by function:
  lon2coord :48-58, observe :118-132, action_to_acc :134-136 -> scripts/helper.py:152-191,
  step :138-195, is_collided :198-206, reset :208-230, corners :232-239.
* ``COracle`` -- ctypes binding of oracle/merge_oracle.c (same algorithm in C, batched,
  OpenMP), for the GPU parity tests at 4,096+ envs and for the CPU baseline.

Parity pinning: both are checked against tests/golden/reference_golden.npz, produced by
running the reference's own MergeEnv (tests/golden/gen_golden.py). Three third-party
boundaries (quadprog's QP solve, pygame Rect/Vector2, shapely intersects) were not
installable here; the oracle restates them (KKT/Goldfarb-Idnani equality step, C (int)
truncation + fp64 corner arithmetic, closed-box overlap) and their parity is pinned only
through the reference's call sites ("Oracle").
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

# merging_env.py:22-46, :101 (values, not code)
R = 30000
H, W = 1000, 300
DT = 0.2
R_FIRST, R_SECOND, R_COLLISION = 2.0, 1.0, -10
VEL_PENALTY, TIME_PENALTY = 0.001, 0
START_POINT, END_POINT = 50, H - 50
VEHICLE_W, VEHICLE_H = 4, 8
PREDICTION_T = 3.0
ACTION_SPEED = {0: 0, 1: 10, 2: 20, 3: 30, 4: 40}


def arc_position(lon, ego: bool):
    """lon2coord (merging_env.py:48-58): longitudinal x and lateral y on the mirrored arcs."""
    theta = np.arctan2(H, R) - lon / R
    x = R * np.sin(theta)
    bulge = R - R * np.cos(theta)
    return x, (W / 2 + bulge) if ego else (W / 2 - bulge)


def first_accel(x0, v0, xt, vt, t):
    """mpc_1d(...).action() (helper.py:152-191) restated.

    The reference builds the 10-step double-integrator constraint A (2 x 10), keeps only its
    velocity row (:172-173, :182) and asks quadprog for min u'Pu with P = D'D + 0.01 I,
    D the first-difference operator, subject to A[1] u = vt - v0. Starting from the
    unconstrained minimiser u = 0, the Goldfarb-Idnani method adds the single equality in
    one step: z = P^-1 n, u = (b / n'z) z. That step is computed here with numpy.
    """
    steps = 10
    dt = t / steps
    a = np.array([[1.0, dt], [0.0, 1.0]])
    b = np.array([0.0, dt])
    A = np.zeros((2, steps))
    power = np.eye(2)
    for i in reversed(range(steps)):
        A[:, i] = power @ b
        power = a @ power
    rhs = vt - (power @ np.array([x0, v0]))[1]
    D = np.eye(steps - 1, steps) - np.eye(steps - 1, steps, k=1)
    P = D.T @ D + 0.01 * np.eye(steps)
    n = A[1]
    z = np.linalg.solve(P, n)
    u = (rhs / (n @ z)) * z
    return u[0]


def vehicle_box(lateral, longitudinal):
    """corners(agent, y=x, x=y, 0) (merging_env.py:232-239) as a closed box.

    pygame's Rect(center=(lateral, longitudinal)) truncates the float centre with a C (int)
    cast and subtracts w//2, h//2 (w=VEHICLE_W=4 lateral, h=VEHICLE_H=8 longitudinal; the
    surfaces are make_surface(ones([4, 8])), :97-98). Each Vector2 corner is
    (corner - pivot).rotate(0) * 1.0 + pivot in fp64.
    """
    left = int(lateral) - VEHICLE_W // 2
    top = int(longitudinal) - VEHICLE_H // 2
    xs = [(float(c) - lateral) + lateral for c in (left, left + VEHICLE_W)]
    ys = [(float(c) - longitudinal) + longitudinal for c in (top, top + VEHICLE_H)]
    return min(xs), max(xs), min(ys), max(ys)


def boxes_touch(b1, b2) -> bool:
    """shapely Polygon.intersects for two axis-aligned rectangles: closed overlap."""
    return b1[0] <= b2[1] and b2[0] <= b1[1] and b1[2] <= b2[3] and b2[2] <= b1[3]


class PyMergeEnv:
    """Scalar restatement of MergeEnv's step/reset path with the reference's list API."""

    def __init__(self):
        self.reset()

    def reset(self):
        # merging_env.py:208-230 (deterministic start; the random start is commented out)
        self.done = False
        self.winner = None
        self.time_stamp = 0
        self.state1 = {"pos": START_POINT, "vel": 20.0, "acc": 0.0}
        self.state2 = {"pos": START_POINT, "vel": 20.0, "acc": 0.0}
        self.r1_accumulate = 0
        self.r2_accumulate = 0
        return self.observe()

    def observe(self):
        x1, y1 = arc_position(self.state1["pos"], True)
        x2, y2 = arc_position(self.state2["pos"], False)
        s1, s2 = self.state1, self.state2
        return [x2 - x1, y2 - y1, s2["vel"] - s1["vel"], END_POINT - s1["pos"], s1["vel"],
                x1 - x2, y1 - y2, s1["vel"] - s2["vel"], END_POINT - s2["pos"], s2["vel"]]

    @staticmethod
    def _advance(car, action):
        vt = ACTION_SPEED[action]  # KeyError for an invalid action, as the reference
        car["acc"] = first_accel(car["pos"], car["vel"], car["pos"] + vt * PREDICTION_T, vt,
                                 PREDICTION_T)
        car["vel"] = max(0, car["vel"] + car["acc"] * DT)
        car["pos"] += car["vel"] * DT

    def collided(self):
        x1, y1 = arc_position(self.state1["pos"], True)
        x2, y2 = arc_position(self.state2["pos"], False)
        return boxes_touch(vehicle_box(y1, x1), vehicle_box(y2, x2))

    def step(self, action1, action2=None):
        # merging_env.py:138-195
        self.time_stamp += DT
        if self.time_stamp > 500:
            self.done = True
        info = {"collision": False}
        self._advance(self.state1, action1)
        if action2 is None:
            self.state2["acc"] = 0
            self.state2["vel"] = max(0, self.state2["vel"] + 0 * DT)
            self.state2["pos"] += self.state2["vel"] * DT
        else:
            self._advance(self.state2, action2)
        obs = self.observe()
        r1 = -TIME_PENALTY - VEL_PENALTY * np.abs(self.state1["vel"] - 20.0)
        r2 = -TIME_PENALTY - VEL_PENALTY * np.abs(self.state2["vel"] - 20.0)
        # arrival: ego strict, opponent non-strict; the first arrival wins
        if self.state1["pos"] > END_POINT:
            if self.winner is None:
                self.winner, r1 = 1, r1 + R_FIRST
            elif self.winner == 1:
                r1 = 0
            else:
                r1, self.done = r1 + R_SECOND, True
        if self.state2["pos"] >= END_POINT:
            if self.winner is None:
                self.winner, r2 = 2, r2 + R_FIRST
            elif self.winner == 2:
                r2 = 0
            else:
                r2, self.done = r2 + R_SECOND, True
        if self.collided():
            self.done = True
            r1 += R_COLLISION
            r2 += R_COLLISION
            info["collision"] = True
        # np.float64 -> float so the list holds plain Python numbers like the reference's
        r1 = r1 if isinstance(r1, int) else float(r1)
        r2 = r2 if isinstance(r2, int) else float(r2)
        self.r1_accumulate += r1
        self.r2_accumulate += r2
        return [_plain(v) for v in obs], [r1, r2], self.done, info


def _plain(v):
    return v if isinstance(v, int) else float(v)


# --------------------------------------------------------------------------- C oracle

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libmerge_oracle.so")


class OracleEnvC(ctypes.Structure):
    """struct oracle_env in merge_oracle.c (one env, the reference's state fields)."""

    _fields_ = [
        ("pos1", ctypes.c_double), ("vel1", ctypes.c_double), ("acc1", ctypes.c_double),
        ("pos2", ctypes.c_double), ("vel2", ctypes.c_double), ("acc2", ctypes.c_double),
        ("time_stamp", ctypes.c_double), ("r1_acc", ctypes.c_double), ("r2_acc", ctypes.c_double),
        ("winner", ctypes.c_int32), ("done", ctypes.c_int32),
        ("steps", ctypes.c_int32), ("pad_", ctypes.c_int32),
    ]


ENV_DTYPE = np.dtype([(n, np.float64) for n in (
    "pos1", "vel1", "acc1", "pos2", "vel2", "acc2", "time_stamp", "r1_acc", "r2_acc")]
    + [("winner", np.int32), ("done", np.int32), ("steps", np.int32), ("pad_", np.int32)])


def build_c_oracle(force: bool = False) -> str:
    """Compile oracle/merge_oracle.c with gcc (no contraction, no fast-math)."""
    if force or not os.path.exists(LIB_PATH) or (
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "merge_oracle.c"))):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return LIB_PATH


def _ptr(a, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype)) if a is not None else None


class COracle:
    """Batched C restatement. Arrays are numpy; envs is a structured array of ENV_DTYPE."""

    def __init__(self, path: str | None = None):
        path = path or LIB_PATH
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        lib = ctypes.CDLL(path)
        P = ctypes.POINTER
        lib.oracle_reset_batch.argtypes = [ctypes.c_void_p, ctypes.c_int64, P(ctypes.c_double)]
        lib.oracle_step_batch.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, P(ctypes.c_int8), P(ctypes.c_int8), ctypes.c_int32,
            P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_uint8), P(ctypes.c_uint8),
            P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_uint32), P(ctypes.c_uint32),
            ctypes.c_int32]
        lib.oracle_step_batch.restype = ctypes.c_int32
        lib.oracle_philox4x32_10.argtypes = [P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32)]
        lib.oracle_random_actions.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.c_int32, P(ctypes.c_int8),
                                              P(ctypes.c_int8)]
        lib.oracle_rollout_random.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
            ctypes.c_uint64, ctypes.c_int32, ctypes.c_int64, P(ctypes.c_double), P(ctypes.c_uint32)]
        lib.oracle_rollout_random.restype = ctypes.c_int64
        lib.oracle_philox_batch.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64,
                                            P(ctypes.c_uint32)]
        lib.oracle_mpc_first_accel.argtypes = [ctypes.c_double] * 5
        lib.oracle_mpc_first_accel.restype = ctypes.c_double
        lib.oracle_set_threads.argtypes = [ctypes.c_int32]
        lib.oracle_max_threads.restype = ctypes.c_int32
        self.lib = lib

    def set_threads(self, n: int) -> None:
        self.lib.oracle_set_threads(int(n))

    def max_threads(self) -> int:
        return int(self.lib.oracle_max_threads())

    @staticmethod
    def new_envs(n: int) -> np.ndarray:
        return np.zeros(n, dtype=ENV_DTYPE)

    def reset(self, envs: np.ndarray) -> np.ndarray:
        obs = np.empty((len(envs), 10), np.float64)
        self.lib.oracle_reset_batch(envs.ctypes.data, len(envs), _ptr(obs, ctypes.c_double))
        return obs

    def step(self, envs, a1, a2=None, autoreset=False, final_obs=False, stats=None):
        """One step of every env. Returns obs[n,10] f64, rew[n,2] f64, done[n] u8, coll[n] u8,
        status[n] u32 (MG_ST_* bits), and final_obs[n,10] (NaN rows for envs not finished)."""
        n = len(envs)
        a1 = np.ascontiguousarray(a1, np.int8)
        a2 = None if a2 is None else np.ascontiguousarray(a2, np.int8)
        obs = np.empty((n, 10), np.float64)
        rew = np.empty((n, 2), np.float64)
        done = np.empty(n, np.uint8)
        coll = np.empty(n, np.uint8)
        status = np.empty(n, np.uint32)
        fobs = np.full((n, 10), np.nan) if final_obs else None
        ret_sum, counts = (None, None) if stats is None else stats
        err = self.lib.oracle_step_batch(
            envs.ctypes.data, n, _ptr(a1, ctypes.c_int8), _ptr(a2, ctypes.c_int8),
            int(bool(autoreset)), _ptr(obs, ctypes.c_double), _ptr(rew, ctypes.c_double),
            _ptr(done, ctypes.c_uint8), _ptr(coll, ctypes.c_uint8), _ptr(fobs, ctypes.c_double),
            _ptr(ret_sum, ctypes.c_double), _ptr(counts, ctypes.c_uint32),
            _ptr(status, ctypes.c_uint32), 0)
        return obs, rew, done, coll, status, fobs, err

    def mpc_first_accel(self, x0, v0, xt, vt, t=3.0):
        """mpc_1d(x0, v0, xt, vt, t).action() with the QP solved in C (helper.py:152-191)."""
        return float(self.lib.oracle_mpc_first_accel(x0, v0, xt, vt, t))

    def philox(self, ctr, key):
        c = np.ascontiguousarray(ctr, np.uint32)
        k = np.ascontiguousarray(key, np.uint32)
        out = np.empty(4, np.uint32)
        self.lib.oracle_philox4x32_10(_ptr(c, ctypes.c_uint32), _ptr(k, ctypes.c_uint32),
                                      _ptr(out, ctypes.c_uint32))
        return out

    def philox_batch(self, n, env_offset, seed, step_idx):
        """[n, 4] uint32 Philox words for (env_offset + i, step_idx) under key seed."""
        out = np.empty((n, 4), np.uint32)
        self.lib.oracle_philox_batch(n, env_offset, seed, step_idx, _ptr(out, ctypes.c_uint32))
        return out

    def random_actions(self, n, env_offset, seed, step_idx, opponent_random):
        a1 = np.empty(n, np.int8)
        a2 = np.empty(n, np.int8)
        self.lib.oracle_random_actions(n, env_offset, seed, step_idx, int(opponent_random),
                                       _ptr(a1, ctypes.c_int8), _ptr(a2, ctypes.c_int8))
        return a1, a2

    def rollout_random(self, envs, steps, seed, first_step, opponent_random, env_offset=0,
                       stats=None):
        """`steps` autoreset steps with Philox actions (the bench workload). Returns the
        number of env-steps done."""
        ret_sum, counts = (None, None) if stats is None else stats
        return int(self.lib.oracle_rollout_random(
            envs.ctypes.data, len(envs), int(steps), int(seed), int(first_step),
            int(opponent_random), int(env_offset), _ptr(ret_sum, ctypes.c_double),
            _ptr(counts, ctypes.c_uint32)))


# --------------------------------------------------------------------------- DQN policy oracle

def qnet_reference(weights, obs, bf16: bool = True, swap: bool = False):
    """The reference Net (scripts/main.py:30-47) on CPU: fc1 -> ReLU -> fc2 -> ReLU -> out.

    bf16=True rounds the input, every weight and each hidden activation to bf16 (round to
    nearest even) and sums in fp32 -- what the MFMA kernel computes up to summation order.
    bf16=False is the reference's own fp32 forward. swap feeds state[5:] + state[:5]
    (main.py:199)."""
    import torch

    x = torch.as_tensor(np.asarray(obs, np.float32))
    if swap:
        x = torch.cat([x[:, 5:], x[:, :5]], dim=1)
    ws = [torch.as_tensor(np.asarray(weights[k], np.float32)) for k in
          ("fc1.weight", "fc2.weight", "out.weight")]
    bs = [torch.as_tensor(np.asarray(weights[k], np.float32)) for k in ("fc1.bias", "fc2.bias", "out.bias")]
    rnd = (lambda t: t.to(torch.bfloat16).to(torch.float32)) if bf16 else (lambda t: t)
    h = rnd(x)
    for i, (w, b) in enumerate(zip(ws, bs)):
        h = h @ rnd(w).T + b
        if i < 2:
            h = rnd(torch.relu(h))
    return h.numpy()


# --------------------------------------------------------------------------- replay memory oracle

def step_with_won(coracle, envs, a1, a2=None):
    """One autoreset step of the C oracle that also reports env.winner == 1 after the step,
    read before the reset (the kernels' won bit; main.py:209). Returns obs (reset observation
    where done), rew, done, coll, final_obs (NaN rows where not done), won, err."""
    obs, rew, done, coll, _, _, err = coracle.step(envs, a1, a2, autoreset=False)
    won = envs["winner"] == 1
    d = done.astype(bool)
    fobs = np.full_like(obs, np.nan)
    fobs[d] = obs[d]
    if d.any():
        sub = envs[d]
        obs[d] = coracle.reset(sub)
        envs[d] = sub
    return obs, rew, done, coll, fobs, won, err


def replay_store(memory, counter, obs_first, obs, a1, rew, done=None, final_obs=None, won=None,
                 skip_ego_won=True, goal=None, next_goal=None, reward=None, meta_goal=None):
    """DQN.store_transition (scripts/main.py:115-119) applied to T steps of n envs in (t, i)
    order -- the order of stepping envs 0..n-1 each step and storing in turn -- with main.py:209's
    `if env.winner is not 1` filter. Row = np.hstack((s, [a, r], s')) with s the observation
    before the step, r the ego's reward, s' the terminal observation where done. Rows are
    float32 (the reference's float64 memory is read back through torch.FloatTensor, main.py:131-135).
    Vectorised; only the newest len(memory) transitions are written, as sequential stores leave
    them. Returns the new memory_counter.

    goal / next_goal [T, n]: hdqn.py's lower-level rows (HDQN.store_transition :180-184 on
    goal_state = [goal] + state, :291 and :304): [goal, s, a, r, next_goal, s'], 24 floats.
    reward [T, n] replaces the ego's env reward as r (hdqn.py:314's intrinsic reward).

    meta_goal [T, n]: Goal_DQN's memory instead (Goal_DQN.store_transition, hdqn.py:97-101, called
    at :325 once the inner loop broke, with state = next_state after :320 and goal the :303
    choice): rows [s', meta_goal, reward, s'] (22 floats) for the transitions whose `won` bit is
    clear -- here the mask marks the steps that did NOT end an inner loop -- and reward the
    extrinsic reward summed since that loop began (:286, :313)."""
    a1 = np.asarray(a1)
    T, n = a1.shape
    cap = memory.shape[0]
    obs = np.asarray(obs, np.float32).reshape(T, n, -1)
    prev = np.concatenate([np.asarray(obs_first, np.float32)[None], obs[:-1]], axis=0)
    nxt = obs.copy()
    if done is not None and final_obs is not None:
        d = np.asarray(done, bool).reshape(T, n)
        nxt[d] = np.asarray(final_obs, np.float32).reshape(T, n, -1)[d]
    keep = np.ones((T, n), bool)
    if (skip_ego_won or meta_goal is not None) and won is not None:
        keep = ~np.asarray(won, bool).reshape(T, n)
    r = (np.asarray(rew, np.float32).reshape(T, n, 2)[..., :1] if reward is None
         else np.asarray(reward, np.float32).reshape(T, n, 1))
    a = a1[..., None].astype(np.float32)
    if meta_goal is not None:  # Goal_DQN rows: [s', goal, extrinsic reward, s'] (:325)
        cols = [nxt, np.asarray(meta_goal, np.float32).reshape(T, n, 1), r, nxt]
    elif goal is None:
        cols = [prev, a, r, nxt]
    else:  # hdqn.py:180-184 on goal_state = [goal] + state (:291, :304)
        g = np.asarray(goal, np.float32).reshape(T, n, 1)
        g2 = np.asarray(next_goal, np.float32).reshape(T, n, 1)
        cols = [g, prev, a, r, g2, nxt]
    rows = np.concatenate(cols, axis=2)[keep]
    k = len(rows)
    last = rows[max(0, k - cap):]
    slots = (counter + np.arange(max(0, k - cap), k)) % cap
    memory[slots] = last
    return counter + k


def replay_sample_index(coracle, capacity, counter, seed, draw, batch, filled_only=False):
    """Slots of mg_replay_sample: floor(u0 * M / 2^32), u = Philox4x32-10(key seed, counter
    (b, draw)); M = capacity (np.random.choice(MEMORY_CAPACITY, BATCH_SIZE), main.py:130) or
    min(counter, capacity) (>= 1) when filled_only."""
    m = capacity if not filled_only else max(1, min(counter, capacity))
    u = coracle.philox_batch(batch, 0, seed, draw)
    return ((u[:, 0].astype(np.uint64) * np.uint64(m)) >> np.uint64(32)).astype(np.int64)
