"""merge_numpy.py -- vectorised NumPy restatement of the reference MergeEnv step at batch scale.

TEST INFRASTRUCTURE / CPU BASELINE ONLY: used by tests/test_oracle_numpy.py (checked against
the C oracle) and by bench.py's CPU-baseline leg (BASELINE.md "CPU baseline plan", item 2: the
NumPy step at 2^20 envs on one core and on all cores). The product never imports it.

Every line follows the reference's own step (YikangZhang1641/merging-gym, the same lines the C
oracle cites), one numpy expression per scalar statement, over arrays of envs:
  time_stamp += 0.2; done if > 500          merging_env.py:141-143
  action_to_acc -> mpc_1d().action()         merging_env.py:134-136, scripts/helper.py:152-191
  v = max(0, v + acc dT); p += v dT          merging_env.py:149-154 (action2 None: acc 0, :152)
  observe / lon2coord                        merging_env.py:118-132, :48-58
  rewards, arrival / winner                  merging_env.py:158-181 (ego first, '>' vs '>=')
  is_collided / corners                      merging_env.py:183-187, :198-206, :232-239
  accumulate returns                         merging_env.py:191-192
  reset (gym.vector autoreset)               merging_env.py:208-230
mpc_1d's QP is factored once the way quadprog's qpgen2 does it (dpofa, dpori, z = J J'n, z'n),
as the C oracle does per call: its first control is then (b / z'n) * z[0] for every env,
b = vt - v0 (0 where |b| < qpgen2's vsmall) -- the per-env arithmetic of the solver's equality
step. Actions: Philox4x32-10 keyed by (global env, step), as the GPU workload draws them.
"""

from __future__ import annotations

import math

import numpy as np

R, H, W, DT = 30000.0, 1000.0, 300.0, 0.2
R_FIRST, R_SECOND, R_COLLISION = 2.0, 1.0, -10.0
VEL_PENALTY, TIME_PENALTY = 0.001, 0.0
START_POINT, END_POINT, PREDICTION_T = 50.0, 950.0, 3.0
VEHICLE_W, VEHICLE_H = 4, 8
ACTION_SPEED = np.array([0.0, 10.0, 20.0, 30.0, 40.0])
ANGLE0 = math.atan2(H, R)  # merging_env.py:49 (np.arctan2(H, R) gives the same double)


def qp_step_constants(t: float = PREDICTION_T):
    """(z'n, z[0], vsmall) of mpc_1d's QP (helper.py:152-191) as quadprog's qpgen2 computes them
    (merge_oracle.qpgen2_factor: dpofa, dpori, d = J'n, z = J d, z'n in the Fortran loop order)."""
    from merge_oracle import qpgen2_factor

    _, z, ztn, vsmall = qpgen2_factor(t)
    return ztn, z[0], vsmall


QP_NZ, QP_Z0, QP_VSMALL = qp_step_constants()

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)
_S32 = np.uint64(32)


def philox4x32_10(c0, c1, c2, c3, seed: int):
    """Philox4x32-10 (Salmon et al., SC'11) over uint64 arrays holding 32-bit words."""
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & 0xFFFFFFFF
            k1 = (k1 + _W1) & 0xFFFFFFFF
        p0 = _M0 * c0
        p1 = _M1 * c2
        c0, c1, c2, c3 = ((p1 >> _S32) ^ c1 ^ np.uint64(k0), p1 & _MASK,
                          (p0 >> _S32) ^ c3 ^ np.uint64(k1), p0 & _MASK)
    return c0, c1, c2, c3


def random_actions(gidx, seed: int, step: int, opponent_random: bool = True):
    """Word w = (step div 2) mod 4 of Philox(counter (gi, step div 8)) per global env index; a draw
    of m outcomes is floor(m w / 2^32), an odd step drawing from m w mod 2^32 instead. Both random:
    m = 25, x = draw, a1 = x // 5, a2 = x % 5; opponent None: m = 5, a1 = draw, a2 = -1 (the device
    stream, mg_step_random)."""
    g = gidx.astype(np.uint64)
    z = np.zeros_like(g)
    blk = step >> 3
    u = philox4x32_10(g & _MASK, g >> _S32, z + np.uint64(blk & 0xFFFFFFFF), z + np.uint64(blk >> 32), seed)
    m = np.uint64(25 if opponent_random else 5)
    w = u[(step >> 1) & 3]
    if step & 1:
        w = (w * m) & _MASK
    x = ((w * m) >> _S32).astype(np.int64)
    if opponent_random:
        return x // 5, x % 5
    return x, np.full(len(g), -1)


class NumpyMergeBatch:
    """n envs as arrays in the reference's own state layout (fp64 car states, float clock)."""

    def __init__(self, n: int, env_offset: int = 0):
        self.n = int(n)
        self.gidx = np.arange(env_offset, env_offset + self.n, dtype=np.int64)
        # per env: sums of r1_accumulate, r2_accumulate, main.py's ep_reward; episodes, collisions,
        # ego-first arrivals, steps, main.py:225 wins, hdqn.py:342 wins (merge_oracle.STATS_DOC)
        self.ret_sum = np.zeros((self.n, 3))
        self.counts = np.zeros((self.n, 6), np.int64)
        self.reset()

    def reset(self, mask=None):
        """merging_env.py:208-230 for every env (mask None) or those where mask holds."""
        if mask is None:
            mask = np.ones(self.n, bool)
            for name in ("p1", "v1", "p2", "v2", "time_stamp", "r1", "r2", "ep_main"):
                setattr(self, name, np.zeros(self.n))
            self.winner = np.zeros(self.n, np.int8)
            self.done = np.zeros(self.n, bool)
            self.steps = np.zeros(self.n, np.int64)
        self.p1[mask] = START_POINT
        self.p2[mask] = START_POINT
        self.v1[mask] = 20.0
        self.v2[mask] = 20.0
        for arr in (self.time_stamp, self.r1, self.r2, self.ep_main, self.steps):
            arr[mask] = 0
        self.winner[mask] = 0
        self.done[mask] = False

    @staticmethod
    def _lon2coord(lon, ego: bool):
        a = ANGLE0 - lon / R
        x = R * np.sin(a)
        bulge = R - R * np.cos(a)
        return x, (W / 2 + bulge) if ego else (W / 2 - bulge)

    @staticmethod
    def _box(lat, lon):
        """corners(agent, y=x, x=y, 0): pygame Rect truncation, fp64 (k - c) + c corners."""
        left = np.trunc(lat) - VEHICLE_W // 2
        top = np.trunc(lon) - VEHICLE_H // 2
        return ((left - lat) + lat, ((left + VEHICLE_W) - lat) + lat,
                (top - lon) + lon, ((top + VEHICLE_H) - lon) + lon)

    def step(self, a1, a2, autoreset: bool = True):
        """One step of every env with valid actions a1 in 0..4, a2 in 0..4 or -1 (None).
        Returns obs [n,10] f64, rew [n,2], done [n] bool, coll [n] bool (before autoreset)."""
        win_pre = (END_POINT - self.p2) > (END_POINT - self.p1)  # main.py:225 on the state acted on
        self.time_stamp += DT
        self.steps += 1
        self.done |= self.time_stamp > 500
        b1 = ACTION_SPEED[a1] - self.v1
        acc1 = np.where(np.abs(b1) < QP_VSMALL, -0.0, (b1 / QP_NZ) * QP_Z0)
        v = self.v1 + acc1 * DT
        self.v1 = np.where(v > 0, v, 0.0)
        self.p1 = self.p1 + self.v1 * DT
        b2 = ACTION_SPEED[np.maximum(a2, 0)] - self.v2
        acc2 = np.where(a2 < 0, 0.0, np.where(np.abs(b2) < QP_VSMALL, -0.0, (b2 / QP_NZ) * QP_Z0))
        v = self.v2 + acc2 * DT
        self.v2 = np.where(v > 0, v, 0.0)
        self.p2 = self.p2 + self.v2 * DT
        x1, y1 = self._lon2coord(self.p1, True)
        x2, y2 = self._lon2coord(self.p2, False)
        obs = np.stack([x2 - x1, y2 - y1, self.v2 - self.v1, END_POINT - self.p1, self.v1,
                        x1 - x2, y1 - y2, self.v1 - self.v2, END_POINT - self.p2, self.v2], axis=1)
        r1 = (0.0 - TIME_PENALTY) - VEL_PENALTY * np.abs(self.v1 - 20.0)
        r2 = (0.0 - TIME_PENALTY) - VEL_PENALTY * np.abs(self.v2 - 20.0)
        arr = self.p1 > END_POINT  # the ego first; it may set the winner the opponent then sees
        first, again, second = arr & (self.winner == 0), arr & (self.winner == 1), arr & (self.winner == 2)
        self.winner[first] = 1
        r1 = np.where(first, r1 + R_FIRST, np.where(again, 0.0, np.where(second, r1 + R_SECOND, r1)))
        self.done |= second
        arr = self.p2 >= END_POINT
        first, again, second = arr & (self.winner == 0), arr & (self.winner == 2), arr & (self.winner == 1)
        self.winner[first] = 2
        r2 = np.where(first, r2 + R_FIRST, np.where(again, 0.0, np.where(second, r2 + R_SECOND, r2)))
        self.done |= second
        b1, b2 = self._box(y1, x1), self._box(y2, x2)
        coll = (b1[0] <= b2[1]) & (b2[0] <= b1[1]) & (b1[2] <= b2[3]) & (b2[2] <= b1[3])
        self.done |= coll
        r1 = np.where(coll, r1 + R_COLLISION, r1)
        r2 = np.where(coll, r2 + R_COLLISION, r2)
        self.r1 += r1
        self.r2 += r2
        self.ep_main = np.where(self.winner != 1, self.ep_main + r1, self.ep_main)  # main.py:209-211
        done = self.done.copy()
        if autoreset and done.any():
            d = done
            self.ret_sum[d, 0] += self.r1[d]
            self.ret_sum[d, 1] += self.r2[d]
            self.ret_sum[d, 2] += self.ep_main[d]
            self.counts[d, 0] += 1
            self.counts[d, 1] += coll[d]
            self.counts[d, 2] += self.winner[d] == 1
            self.counts[d, 3] += self.steps[d]
            self.counts[d, 4] += win_pre[d]
            self.counts[d, 5] += ((END_POINT - self.p2) > (END_POINT - self.p1))[d]  # hdqn.py:342
            self.reset(d)
        return obs, np.stack([r1, r2], axis=1), done, coll

    def rollout_random(self, steps: int, seed: int, first_step: int, opponent_random: bool = True):
        """`steps` autoreset steps with Philox actions (the bench workload); returns env-steps."""
        for k in range(steps):
            a1, a2 = random_actions(self.gidx, seed, first_step + k, opponent_random)
            self.step(a1, a2)
        return self.n * steps
