"""may_finish_next (merging_hip.hip): the config-5 kernels evaluate the ego's Q-net for an env whose
next step may end its episode even when the ego explores, because main.py:221 logs
eval_net(state)[action] of every episode's last step. The predicate must therefore flag EVERY step
that ends an episode. This restates it in numpy (same fp32 inputs: the observation the kernel keeps
in its tile row) and drives the C oracle through random, L0 and constant-action play -- collisions,
both arrival orders, same-step ties and timeouts at step 2501 -- checking that no finishing step goes
unflagged and that few steps are flagged. The device function itself is checked through q_eval
parity on the GPU (tests/test_gpu_qnet.py: an unflagged finish with a random action would log a value
of the observation instead of a Q-value)."""

from __future__ import annotations

import numpy as np
import pytest

import merge_oracle

DT, TIMEOUT = 0.2, 2501  # mg_params dT, timeout_steps
SMIN, SMAX, G = -0.5, 40.5, (0.2 * 30.000000000000533 / 90.0000000000015) * 1.01  # FinishBound as launched


def finish_bound(veh_w=4, veh_h=8, R=30000.0, dT=0.2, speeds=(0, 10, 20, 30, 40), start_vel=20.0):
    """merging_hip.hip finish_bound's collision reach (lat, lon), restated."""
    dl = dT * (max(max(speeds), start_vel) + 0.5)
    lat = veh_w + 1.75
    for _ in range(4):
        sn = np.sqrt(2.0 * lat / R) + dl / R
        lat = veh_w + 1.0 + max(0.75, 2.0 * dl * sn + 0.25)
    return np.float32(lat), np.float32(veh_h + 1)


LAT, LON = finish_bound()


def test_finish_bound_defaults_and_scaling():
    """The default params keep round 5's proven 5.75 / 9 m; the reach grows with the boxes, with a
    tighter arc (the lateral drift per step) and with faster action speeds."""
    assert finish_bound() == (np.float32(5.75), np.float32(9.0))
    lat, lon = finish_bound(veh_w=14, veh_h=30)
    assert lat >= 15.75 and lon == 31.0
    lat_tight, _ = finish_bound(R=300.0)
    assert lat_tight > 5.75
    lat_fast, _ = finish_bound(R=3000.0, speeds=(0, 50, 100, 150, 200))
    assert lat_fast > lat_tight - 1.0 and lat_fast > 5.75


def may_finish(obs64, winner, steps):
    o = obs64.astype(np.float32)
    f = np.float32
    dt = f(DT)
    ego = o[:, 3] < dt * np.maximum(o[:, 4], f(SMAX)) + f(0.5)
    opp = o[:, 8] < dt * np.maximum(o[:, 9], f(SMAX)) + f(0.5)
    arrive = np.where(winner == 1, opp, np.where(winner == 2, ego, ego & opp))
    spread = np.maximum(f(SMAX), np.maximum(o[:, 4], o[:, 9])) - np.minimum(f(SMIN), np.minimum(o[:, 4], o[:, 9]))
    rel = dt * (np.abs(o[:, 2]) + f(G) * spread) + f(0.5)
    coll = (-o[:, 1] < LAT) & (np.abs(o[:, 0]) < LON + rel)
    return (steps + 1 >= TIMEOUT) | arrive | coll


@pytest.fixture(scope="module")
def co():
    return merge_oracle.COracle(merge_oracle.build_c_oracle())


def _run(co, a1_fn, a2_fn, n, steps, rng):
    envs = co.new_envs(n)
    obs = co.reset(envs)
    flagged = finishes = missed = 0
    for k in range(steps):
        flag = may_finish(obs, envs["winner"], envs["steps"])
        a1, a2 = a1_fn(k, rng), a2_fn(k, rng)
        obs, rew, done, coll, status, _, err = co.step(envs, a1, a2, autoreset=True)
        assert err == 0
        d = done.astype(bool)
        missed += int((d & ~flag).sum())
        finishes += int(d.sum())
        flagged += int(flag.sum())
    return finishes, missed, flagged / (n * steps)


def test_may_finish_covers_every_finish(co):
    rng = np.random.default_rng(5)
    n = 2048
    cases = {
        # uniform random both players (the bench / config-5 exploration regime)
        "uniform": (lambda k, r: r.integers(0, 5, n).astype(np.int8), lambda k, r: r.integers(0, 5, n).astype(np.int8)),
        # ego random, opponent None (L0)
        "l0": (lambda k, r: r.integers(0, 5, n).astype(np.int8), lambda k, r: None),
        # sticky policies: an action held for a random number of steps, so cars meet at every
        # speed difference and long episodes reach the timeout
        "sticky": (None, None),
    }
    held1 = rng.integers(0, 5, n).astype(np.int8)
    held2 = rng.integers(-1, 5, n).astype(np.int8)

    def sticky1(k, r):
        ch = r.random(n) < 0.02
        held1[ch] = r.integers(0, 5, int(ch.sum()))
        return held1.copy()

    def sticky2(k, r):
        ch = r.random(n) < 0.02
        held2[ch] = r.integers(-1, 5, int(ch.sum()))
        return held2.copy()

    cases["sticky"] = (sticky1, sticky2)
    total = 0
    for name, (f1, f2) in cases.items():
        fin, missed, frac = _run(co, f1, f2, n, 700 if name != "sticky" else 2700, rng)
        assert missed == 0, (name, missed, fin)
        assert fin > 1000, (name, fin)
        assert frac < 0.05, (name, frac)
        total += fin
        print(f"[may_finish] {name}: {fin} finishes, all flagged; {100 * frac:.2f} % of env-steps flagged")
    assert total > 10000


def test_may_finish_known_answer_episodes(co):
    # SURVEY.md 8(a) KATs A-G: constant actions, collisions, arrivals in both orders, timeouts
    kats = [(2, -1), (0, -1), (4, -1), (4, 0), (0, 4), (3, 3), (1, 1)]
    n = len(kats)
    a1 = np.array([a for a, _ in kats], np.int8)
    a2 = np.array([b for _, b in kats], np.int8)
    envs = co.new_envs(n)
    obs = co.reset(envs)
    ends = np.zeros(n, np.int64)
    for k in range(2600):
        flag = may_finish(obs, envs["winner"], envs["steps"])
        obs, _, done, _, _, _, err = co.step(envs, a1, a2, autoreset=True)
        d = done.astype(bool)
        assert not (d & ~flag).any(), (k, np.flatnonzero(d & ~flag))
        ends[(ends == 0) & d] = k + 1
    assert ends.tolist() == [151, 2501, 225, 2501, 2501, 106, 288]
