"""The host step (mg_host_step / mg_host_reset / mg_host_observe, ABI 20): the kernels' own step
functions compiled for the CPU, on host arrays -- the single env's default backend (BASELINE
config 1). CPU suite: batched host steps against the C oracle (state bit-exact, flags exact, fp32
outputs to the rounding bar), every optional output of mg_outputs. GPU suite: host and kernel give
the same bytes for the same inputs."""

import ctypes

import numpy as np
import pytest

import merge_oracle as mo

OBS_TOL = dict(rtol=1e-6, atol=1e-5)


class HostBatch:
    """n envs in host numpy arrays, laid out as the device SoA (include/merging_hip.h mg_state)."""

    def __init__(self, n):
        from merging_gym import _native

        self.nat, self.n = _native, n
        self.params = _native.default_params()
        self.s = {k: np.zeros(n) for k in ("p1", "v1", "p2", "v2", "ret1", "ret2")}
        self.tf = np.zeros(n, np.uint16)
        p = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
        self.state = _native.State(*(p(self.s[k]) for k in ("p1", "v1", "p2", "v2", "ret1", "ret2")), p(self.tf))
        self.obs = np.zeros((n, 10), np.float32)
        self.rew = np.zeros((n, 2), np.float32)
        self.flags = np.zeros((n, 4), np.uint8)
        self.fobs = np.full((n, 10), np.nan, np.float32)
        words = (n + 63) // 64
        self.done_mask = np.zeros(words, np.uint64)
        self.won_mask = np.zeros(words, np.uint64)
        self.err = np.zeros(1, np.int32)
        self.stats = np.zeros(n, _native.EPISODE_STATS_DTYPE)
        self.out = _native.Outputs(p(self.obs), p(self.rew), None, None, p(self.done_mask), p(self.fobs), None,
                                   p(self.err), p(self.won_mask), p(self.flags))
        self.st = _native.Stats(p(self.stats))

    def reset(self):
        rc = self.nat.lib.mg_host_reset(ctypes.byref(self.params), ctypes.byref(self.state), None,
                                        ctypes.byref(self.out), self.n)
        self.nat.check(rc, "mg_host_reset")

    def step(self, a1, a2=None, autoreset=True):
        a1 = np.ascontiguousarray(a1, np.int8)
        a2 = None if a2 is None else np.ascontiguousarray(a2, np.int8)
        self.fobs[:] = np.nan
        rc = self.nat.lib.mg_host_step(ctypes.byref(self.params), ctypes.byref(self.state),
                                       ctypes.c_void_p(a1.ctypes.data),
                                       None if a2 is None else ctypes.c_void_p(a2.ctypes.data),
                                       ctypes.byref(self.out), ctypes.byref(self.st), self.n,
                                       self.nat.AUTORESET if autoreset else 0)
        self.nat.check(rc, "mg_host_step")


def _bits(words, n):
    return np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)


@pytest.mark.parametrize("opponent", ["uniform", "none", "mixed"])
def test_host_batch_equals_oracle(coracle, opponent):
    """Config-2 shape on the host path: 2,048 envs x 400 steps with autoreset, statistics, final
    observations, the interleaved step record and both ballot masks, against the C oracle."""
    n, steps = 2048, 400
    rng = np.random.default_rng(21)
    hb = HostBatch(n)
    hb.reset()
    envs = coracle.new_envs(n)
    np.testing.assert_allclose(hb.obs, coracle.reset(envs).astype(np.float32), **OBS_TOL)
    ret_sum, counts = mo.new_stats(n)
    for k in range(steps):
        a1 = rng.integers(0, 5, n).astype(np.int8)
        a2 = {"uniform": lambda: rng.integers(0, 5, n).astype(np.int8), "none": lambda: None,
              "mixed": lambda: rng.integers(-1, 5, n).astype(np.int8)}[opponent]()
        hb.step(a1, a2)
        won = None
        # the won bit is winner == 1 after the step, before autoreset: replay with step_with_won
        # on a copy for it, then the stats-keeping step on the real oracle envs
        probe = envs.copy()
        _, _, _, _, _, won, _ = mo.step_with_won(coracle, probe, a1, a2)
        o_obs, o_rew, o_done, o_coll, _, o_fobs, err = coracle.step(envs, a1, a2, autoreset=True, final_obs=True,
                                                                     stats=(ret_sum, counts))
        assert err == 0 and hb.err[0] == 0
        np.testing.assert_array_equal(hb.flags[:, 0].view(np.int8), a1)
        np.testing.assert_array_equal(hb.flags[:, 1].view(np.int8), -1 if a2 is None else a2)
        np.testing.assert_array_equal(hb.flags[:, 2], o_done, err_msg=f"done @ {k}")
        np.testing.assert_array_equal(hb.flags[:, 3], o_coll, err_msg=f"coll @ {k}")
        np.testing.assert_array_equal(_bits(hb.done_mask, n), o_done.astype(bool))
        np.testing.assert_array_equal(_bits(hb.won_mask, n), won)
        np.testing.assert_allclose(hb.obs, o_obs.astype(np.float32), **OBS_TOL, err_msg=f"obs @ {k}")
        np.testing.assert_allclose(hb.rew, o_rew.astype(np.float32), **OBS_TOL, err_msg=f"rew @ {k}")
        d = o_done.astype(bool)
        np.testing.assert_allclose(hb.fobs[d], o_fobs[d].astype(np.float32), **OBS_TOL)
        assert np.isnan(hb.fobs[~d]).all()
    for name, key in (("p1", "pos1"), ("v1", "vel1"), ("p2", "pos2"), ("v2", "vel2"), ("ret1", "r1_acc"),
                      ("ret2", "r2_acc")):
        np.testing.assert_array_equal(hb.s[name], envs[key], err_msg=name)  # fp64 state bit-exact
    np.testing.assert_array_equal(hb.tf & 0x1FFF, envs["steps"])
    np.testing.assert_array_equal((hb.tf & 0x6000) >> 13, envs["winner"])
    np.testing.assert_array_equal(hb.stats["ret"], ret_sum[:, :2])
    np.testing.assert_array_equal(hb.stats["ret_main"], ret_sum[:, 2])
    np.testing.assert_array_equal(hb.stats["counts"], counts)
    assert counts[:, 0].sum() > 0 and counts[:, 1].sum() > 0


def test_host_invalid_actions_and_observe(coracle):
    """An action outside action_dict sets the error bits and advances the env exactly as far as the
    reference gets before its KeyError (the clock, plus the ego for a bad action2); mg_host_observe
    is observe() / is_collided() without a state change."""
    n = 256
    rng = np.random.default_rng(3)
    hb = HostBatch(n)
    hb.reset()
    envs = coracle.new_envs(n)
    coracle.reset(envs)
    for k in range(160):  # constant-speed pairs: many collide around step 151 (KAT A)
        a1 = rng.integers(0, 5, n).astype(np.int8)
        a1[: n // 2] = 2
        hb.step(a1, None, autoreset=False)
        coracle.step(envs, a1, None)
    bad = np.full(n, 3, np.int8)
    bad[::7] = 9
    a2 = np.full(n, 1, np.int8)
    a2[3::11] = 40
    hb.step(bad, a2, autoreset=False)
    _, _, _, _, _, _, err = coracle.step(envs, bad, a2)
    assert hb.err[0] == err == 3
    for name, key in (("p1", "pos1"), ("v1", "vel1"), ("p2", "pos2"), ("v2", "vel2"), ("ret1", "r1_acc")):
        np.testing.assert_array_equal(hb.s[name], envs[key], err_msg=name)
    np.testing.assert_array_equal(hb.tf & 0x1FFF, envs["steps"])
    # observe / is_collided, no state change
    before = {k: v.copy() for k, v in hb.s.items()}
    out = hb.nat.Outputs(ctypes.c_void_p(hb.obs.ctypes.data), None, None, None, None, None, None, None, None,
                         ctypes.c_void_p(hb.flags.ctypes.data))
    hb.nat.check(hb.nat.lib.mg_host_observe(ctypes.byref(hb.params), ctypes.byref(hb.state), ctypes.byref(out), n),
                 "mg_host_observe")
    np.testing.assert_allclose(hb.obs, coracle.observe(envs).astype(np.float32), **OBS_TOL)
    ref_coll = [mo.boxes_touch(*_boxes(p1, p2)) for p1, p2 in zip(envs["pos1"], envs["pos2"])]
    np.testing.assert_array_equal(hb.flags[:, 3].astype(bool), ref_coll)
    assert any(ref_coll)
    for k, v in before.items():
        np.testing.assert_array_equal(hb.s[k], v)


def _boxes(p1, p2):
    x1, y1 = mo.arc_position(p1, True)
    x2, y2 = mo.arc_position(p2, False)
    return mo.vehicle_box(y1, x1), mo.vehicle_box(y2, x2)


def test_host_entry_validation():
    from merging_gym import _native

    P = ctypes.byref(_native.default_params())
    rc = _native.lib.mg_host_step(P, ctypes.byref(_native.State()), None, None, ctypes.byref(_native.Outputs()),
                                  None, 4, 0)
    assert rc != 0 and b"NULL" in _native.lib.mg_last_error()
    assert _native.lib.mg_host_reset(None, None, None, None, 1) != 0
    fake = ctypes.c_void_p(1 << 20)  # never dereferenced: n == 0
    st = ctypes.byref(_native.State(*([fake] * 7)))
    assert _native.lib.mg_host_step(P, st, fake, None, ctypes.byref(_native.Outputs()), None, 0, 0) == 0
    assert _native.lib.mg_host_observe(P, st, ctypes.byref(_native.Outputs()), 0) == 0


@pytest.mark.gpu
def test_host_step_equals_kernel():
    """The same inputs through mg_host_step and mg_step give the same bytes: every fp64 state word,
    the fp32 observations / rewards, the step record, the masks, the final observations and the
    statistics records. States span live episodes, finished ones driving on past the end point
    (the merge zone included) and the timeout; actions include None and invalid ones."""
    import torch

    from merging_gym import _native

    n = 1 << 16
    rng = np.random.default_rng(9)
    hb = HostBatch(n)
    hb.s["p1"][:] = rng.uniform(40, 1100, n)
    hb.s["p2"][:] = np.where(rng.random(n) < 0.3, hb.s["p1"] + rng.uniform(-6, 6, n), rng.uniform(40, 1100, n))
    hb.s["v1"][:] = rng.uniform(0, 45, n)
    hb.s["v2"][:] = rng.uniform(0, 45, n)
    hb.s["ret1"][:] = rng.normal(0, 3, n)
    hb.s["ret2"][:] = rng.normal(0, 3, n)
    steps = rng.integers(0, 2600, n)
    winner = rng.integers(0, 3, n)
    hb.tf[:] = (steps | (winner << 13) | ((rng.random(n) < 0.1) << 15)).astype(np.uint16)
    hb.stats["ret"] = rng.normal(0, 5, (n, 2))
    hb.stats["ret1_pending"] = rng.normal(0, 5, n)
    a1 = rng.integers(0, 5, n).astype(np.int8)
    a2 = rng.integers(-1, 5, n).astype(np.int8)
    a1[::997] = 7
    a2[5::1009] = 12
    dev = {k: torch.from_numpy(v.copy()).cuda() for k, v in hb.s.items()}
    dtf = torch.from_numpy(hb.tf.view(np.int16).copy()).cuda()
    d = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    dstate = _native.State(*(d(dev[k]) for k in ("p1", "v1", "p2", "v2", "ret1", "ret2")), d(dtf))
    dobs = torch.zeros((n, 10), dtype=torch.float32, device="cuda")
    drew = torch.zeros((n, 2), dtype=torch.float32, device="cuda")
    dflags = torch.zeros((n, 4), dtype=torch.uint8, device="cuda")
    dfobs = torch.full((n, 10), float("nan"), device="cuda")
    words = (n + 63) // 64
    ddm = torch.zeros(words, dtype=torch.int64, device="cuda")
    dwm = torch.zeros(words, dtype=torch.int64, device="cuda")
    derr = torch.zeros(1, dtype=torch.int32, device="cuda")
    dstats = torch.from_numpy(hb.stats.view(np.uint8).reshape(n, 64).copy()).cuda()
    dout = _native.Outputs(d(dobs), d(drew), None, None, d(ddm), d(dfobs), None, d(derr), d(dwm), d(dflags))
    da1, da2 = torch.from_numpy(a1).cuda(), torch.from_numpy(a2).cuda()
    rc = _native.lib.mg_step(ctypes.byref(hb.params), ctypes.byref(dstate), d(da1), d(da2), ctypes.byref(dout),
                             ctypes.byref(_native.Stats(d(dstats))), n, _native.AUTORESET, None)
    _native.check(rc, "mg_step")
    torch.cuda.synchronize()
    hb.step(a1, a2)
    for k in hb.s:
        np.testing.assert_array_equal(dev[k].cpu().numpy().view(np.uint64), hb.s[k].view(np.uint64), err_msg=k)
    np.testing.assert_array_equal(dtf.cpu().numpy().view(np.uint16), hb.tf)
    np.testing.assert_array_equal(dobs.cpu().numpy().view(np.uint32), hb.obs.view(np.uint32))
    np.testing.assert_array_equal(dflags.cpu().numpy(), hb.flags)
    np.testing.assert_array_equal(ddm.cpu().numpy().view(np.uint64), hb.done_mask)
    np.testing.assert_array_equal(dwm.cpu().numpy().view(np.uint64), hb.won_mask)
    np.testing.assert_array_equal(dfobs.cpu().numpy(), hb.fobs)
    np.testing.assert_array_equal(dstats.cpu().numpy(), hb.stats.view(np.uint8).reshape(n, 64))
    np.testing.assert_array_equal(drew.cpu().numpy().view(np.uint32), hb.rew.view(np.uint32))
    assert derr.item() == hb.err[0] == 3
    assert hb.flags[:, 2].any() and hb.flags[:, 3].any() and np.isfinite(hb.fobs).any()


@pytest.mark.gpu
def test_host_step_equals_kernel_past_the_polynomial_range():
    """Far past the end point (|theta| >= 1/16: positions beyond ~2,875 m) sin / cos leave the shared
    polynomial: glibc on the host, the device library on the GPU. Live episodes reach this range (an
    arrived car keeps driving while the other runs the episode to the 2501-step timeout, to ~20 km),
    as do cars stepped on after a finished episode without autoreset. The state, rewards and flags stay bit-equal (they do
    not depend on sin / cos there: the cars are far apart), and the observations agree to 1 fp32 ulp
    (the doubles differ by at most an ulp before the fp32 rounding)."""
    import torch

    from merging_gym import _native

    n = 1 << 14
    rng = np.random.default_rng(10)
    hb = HostBatch(n)
    hb.s["p1"][:] = rng.uniform(2800, 20000, n)
    hb.s["p2"][:] = rng.uniform(-3000, 20000, n)
    hb.s["v1"][:] = rng.uniform(0, 45, n)
    hb.s["v2"][:] = rng.uniform(0, 45, n)
    hb.tf[:] = (rng.integers(0, 2600, n) | (rng.integers(0, 3, n) << 13)).astype(np.uint16)
    a1 = rng.integers(0, 5, n).astype(np.int8)
    a2 = rng.integers(-1, 5, n).astype(np.int8)
    dev = {k: torch.from_numpy(v.copy()).cuda() for k, v in hb.s.items()}
    dtf = torch.from_numpy(hb.tf.view(np.int16).copy()).cuda()
    d = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    dstate = _native.State(*(d(dev[k]) for k in ("p1", "v1", "p2", "v2", "ret1", "ret2")), d(dtf))
    dobs = torch.zeros((n, 10), dtype=torch.float32, device="cuda")
    drew = torch.zeros((n, 2), dtype=torch.float32, device="cuda")
    dflags = torch.zeros((n, 4), dtype=torch.uint8, device="cuda")
    dout = _native.Outputs(d(dobs), d(drew), None, None, None, None, None, None, None, d(dflags))
    da1, da2 = torch.from_numpy(a1).cuda(), torch.from_numpy(a2).cuda()
    rc = _native.lib.mg_step(ctypes.byref(hb.params), ctypes.byref(dstate), d(da1), d(da2), ctypes.byref(dout),
                             None, n, 0, None)
    _native.check(rc, "mg_step")
    torch.cuda.synchronize()
    hb.step(a1, a2, autoreset=False)
    for k in hb.s:
        np.testing.assert_array_equal(dev[k].cpu().numpy().view(np.uint64), hb.s[k].view(np.uint64), err_msg=k)
    np.testing.assert_array_equal(dtf.cpu().numpy().view(np.uint16), hb.tf)
    np.testing.assert_array_equal(dflags.cpu().numpy(), hb.flags)
    np.testing.assert_array_equal(drew.cpu().numpy().view(np.uint32), hb.rew.view(np.uint32))
    np.testing.assert_array_max_ulp(dobs.cpu().numpy(), hb.obs, maxulp=1)


def test_host_collision_test_over_the_whole_plane(coracle):
    """The step's collision test takes integer lateral edges where they equal the fp64 ones (y >= 8,
    merging_hip.hip vehicles_collide) and the fp64 form elsewhere. Pairs of cars placed over the
    whole reachable plane -- positions far past the end point, where the opponent's mirror arc
    crosses y = 8 and 0, and pairs packed within a few metres of each other around the merge point
    x = 0 -- collide exactly when the C oracle's fp64 boxes do (no autoreset, both cars held still)."""
    n = 1 << 16
    rng = np.random.default_rng(12)
    hb = HostBatch(n)
    base = rng.uniform(-3000, 9000, n)
    p1 = np.where(rng.random(n) < 0.5, base, rng.uniform(985, 1016, n))
    p2 = np.where(rng.random(n) < 0.7, p1 + rng.uniform(-10, 10, n), rng.uniform(-3000, 9000, n))
    for k, v in (("p1", p1), ("p2", p2)):
        hb.s[k][:] = v
    hb.s["v1"][:] = hb.s["v2"][:] = 0.0
    envs = coracle.new_envs(n)
    envs["pos1"], envs["pos2"] = p1, p2
    a1 = np.zeros(n, np.int8)  # target speed 0 from speed 0: the cars stay where they are
    hb.step(a1, None, autoreset=False)
    _, _, _, o_coll, _, _, err = coracle.step(envs, a1, None)
    assert err == 0
    np.testing.assert_array_equal(hb.flags[:, 3], o_coll)
    y2 = 150.0 - 30000.0 * (1 - np.cos(np.arctan2(1000, 30000) - p2 / 30000))
    # the fp64 branch runs (y2 < 8: the ego's arc stays at y >= 150, so those pairs never touch)
    assert o_coll.sum() > 1000 and (y2 < 8).sum() > 1000
