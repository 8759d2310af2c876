"""GPU parity: libmerging_hip.so (through the C-ABI, via MergeVecEnv / MergeEnv) vs the CPU oracle.

Bar (north_star): done / collision / winner flags bit-exact; fp32 outputs equal to the
oracle's fp64 values rounded to fp32 (rtol 1e-6, atol 1e-5 -- tighter than the 1e-5 fp32
bound); fp64 state (positions, speeds, returns) BIT-EXACT against the C oracle: the kernel's
mpc_1d step carries the QP solver's own rounding (u0 = (b / z'n) z0, mg_params.qp_*, computed
in quadprog's qpgen2 order), the same two operations the oracle's full qpgen2 solve ends in,
and every other state operation is the same IEEE fp64 operation in the same order. Against the
reference's own recorded traces (tests/golden, generated with a qpgen2-restating stand-in for
quadprog) the state is bit-exact too.
"""

import ctypes

import numpy as np
import pytest

import merge_oracle as mo

pytestmark = pytest.mark.gpu

OBS_TOL = dict(rtol=1e-6, atol=1e-5)
STATE_TOL = dict(rtol=0, atol=0)  # vs the reference's golden traces: bit-exact (qpgen2 stand-in)
ANGLE0 = float(np.arctan2(1000, 30000))


def merge_zone(p1, p2):
    """Envs with a car within 4 m of the merge point (|x| < 4, pos ~ 995.6..1003.6). There the
    corner edges ((k - c) + c, merging_env.py:235-238) round, so whether touching boxes
    intersect depends on the last ulp of the positions. Reachable only after an episode is
    over (while it runs one car is at pos <= 950, x >= 49.6). Used to report where the
    collision checks below exercise that case; no flag is excused there."""
    x1 = 30000 * np.sin(ANGLE0 - np.asarray(p1) / 30000)
    x2 = 30000 * np.sin(ANGLE0 - np.asarray(p2) / 30000)
    return (np.abs(x1) < 4) | (np.abs(x2) < 4)


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


def _check_state(env, envs):
    """fp64 state bit for bit equal to the C oracle's."""
    for name, key in (("p1", "pos1"), ("p2", "pos2"), ("v1", "vel1"), ("v2", "vel2"),
                      ("ret1", "r1_acc"), ("ret2", "r2_acc")):
        np.testing.assert_array_equal(getattr(env, name).cpu().numpy(), envs[key], err_msg=name)
    np.testing.assert_array_equal(env.winner.cpu().numpy(), envs["winner"])
    np.testing.assert_array_equal(env.steps.cpu().numpy(), envs["steps"])


def _check_step(out, ref, k):
    obs, rew, done, info = out
    o_obs, o_rew, o_done, o_coll, _, o_fobs, err = ref
    assert err == 0
    np.testing.assert_array_equal(done.cpu().numpy(), o_done.astype(bool), err_msg=f"done @ {k}")
    np.testing.assert_array_equal(info["collision"].cpu().numpy(), o_coll.astype(bool), err_msg=f"coll @ {k}")
    np.testing.assert_allclose(obs.cpu().numpy(), o_obs.astype(np.float32), **OBS_TOL, err_msg=f"obs @ {k}")
    np.testing.assert_allclose(rew.cpu().numpy(), o_rew.astype(np.float32), **OBS_TOL, err_msg=f"rew @ {k}")
    if o_fobs is not None and "final_observation" in info:
        assert info["terminal_observation"] is info["final_observation"]  # gym 0.20's key, batched
        d = o_done.astype(bool)
        np.testing.assert_allclose(info["final_observation"].cpu().numpy()[d], o_fobs[d].astype(np.float32),
                                   **OBS_TOL, err_msg=f"final_obs @ {k}")


@pytest.mark.parametrize("opponent", ["uniform", "none", "mixed"])
def test_config2_host_actions_autoreset(torch, coracle, opponent):
    """BASELINE config 2: 4,096 envs, 500 steps, host-drawn actions, gym.vector autoreset."""
    from merging_gym import MergeVecEnv

    n, steps = 4096, 500
    rng = np.random.default_rng(11)
    env = MergeVecEnv(n, device="cuda:0")
    envs = coracle.new_envs(n)
    o0 = coracle.reset(envs)
    np.testing.assert_allclose(env.obs.cpu().numpy(), o0.astype(np.float32), **OBS_TOL)
    ret_sum, counts = mo.new_stats(n)  # [n,3] returns, [n,6] counts (both scripts' statistics)
    for k in range(steps):
        a1 = rng.integers(0, 5, n).astype(np.int8)
        if opponent == "uniform":
            a2 = rng.integers(0, 5, n).astype(np.int8)
        elif opponent == "none":
            a2 = None
        else:
            a2 = rng.integers(-1, 5, n).astype(np.int8)
        out = env.step(torch.from_numpy(a1).cuda(), None if a2 is None else torch.from_numpy(a2).cuda())
        ref = coracle.step(envs, a1, a2, autoreset=True, final_obs=True, stats=(ret_sum, counts))
        _check_step(out, ref, k)
    _check_state(env, envs)
    st = env.episode_statistics()
    np.testing.assert_array_equal(st["counts"].cpu().numpy().astype(np.uint32), counts)
    np.testing.assert_array_equal(st["returns"].cpu().numpy(), ret_sum)
    assert counts[:, 0].sum() > 0 and counts[:, 1].sum() > 0  # episodes finished, some collided
    # main.py's filtered return differs from r1_accumulate on ego-first episodes; both win tests fire
    assert (ret_sum[:, 2] != ret_sum[:, 0]).any() and counts[:, 4].sum() > 0 and counts[:, 5].sum() > 0
    # size-independent invariant: every step is in a finished episode or the running one
    np.testing.assert_array_equal(counts[:, 3] + envs["steps"], steps)


def test_past_done_no_autoreset(torch, coracle):
    """Reference semantics without reset: cars keep driving past done, the 2501-step timeout
    fires, the winner keeps its flag. Every flag bit-exact and the state bit-exact, including
    the steps where a car crosses the ill-conditioned merge zone (counted, none excused)."""
    from merging_gym import MergeVecEnv

    n, steps = 1024, 2600
    rng = np.random.default_rng(5)
    env = MergeVecEnv(n, device="cuda:0", autoreset=False)
    envs = coracle.new_envs(n)
    coracle.reset(envs)
    zone_steps = 0
    for k in range(steps):
        a1 = rng.integers(0, 5, n).astype(np.int8)
        a2 = rng.integers(-1, 5, n).astype(np.int8)
        obs, rew, done, info = env.step(torch.from_numpy(a1).cuda(), torch.from_numpy(a2).cuda())
        o_obs, o_rew, o_done, o_coll, _, _, err = coracle.step(envs, a1, a2)
        zone_steps += int(merge_zone(envs["pos1"], envs["pos2"]).sum())
        c = info["collision"].cpu().numpy()
        bad = c != o_coll.astype(bool)
        assert not bad.any(), f"collision flag mismatch @ {k}: envs {np.nonzero(bad)[0][:8]}"
        np.testing.assert_array_equal(done.cpu().numpy(), o_done.astype(bool))
        np.testing.assert_allclose(obs.cpu().numpy(), o_obs.astype(np.float32), **OBS_TOL)
        np.testing.assert_allclose(rew.cpu().numpy(), o_rew.astype(np.float32), **OBS_TOL)
    assert zone_steps > 1000, zone_steps  # the merge zone was actually crossed, many times
    _check_state(env, envs)
    assert envs["done"].all()  # the timeout caught every env


def test_device_random_actions_match_philox(torch, coracle):
    """mg_step_random: the device Philox stream equals the oracle's, and the step matches."""
    from merging_gym import MergeVecEnv

    n, steps, seed = 3000, 300, 99
    env = MergeVecEnv(n, device="cuda:0")
    envs = coracle.new_envs(n)
    coracle.reset(envs)
    for k in range(steps):
        out = env.step_random(seed, opponent_random=(k % 3 != 0), step_idx=k)
        a1, a2 = coracle.random_actions(n, 0, seed, k, k % 3 != 0)
        np.testing.assert_array_equal(env.a1_buf.cpu().numpy(), a1)
        np.testing.assert_array_equal(env.a2_buf.cpu().numpy(), a2)
        ref = coracle.step(envs, a1, a2, autoreset=True, final_obs=True)
        _check_step(out, ref, k)
    _check_state(env, envs)


def test_interleaved_step_record_equals_byte_arrays(torch, monkeypatch):
    """mg_outputs.flags (a1, a2, done, collision as one u32 per env, MergeVecEnv's default) gives
    the same outputs and state as the four byte arrays, for device and host actions (None
    opponent included), autoreset, and observe()."""
    from merging_gym import MergeVecEnv
    from merging_gym.envs import vector_env

    n, seed = 3001, 17
    monkeypatch.setattr(vector_env, "_STEP_FLAGS", False)
    plain = MergeVecEnv(n, device="cuda:0", final_observation=True, won_mask=True)
    monkeypatch.setattr(vector_env, "_STEP_FLAGS", True)
    packed = MergeVecEnv(n, device="cuda:0", final_observation=True, won_mask=True)
    assert plain.flags is None and packed.flags is not None and packed.done.stride() == (4,)
    rng = np.random.default_rng(5)
    ndone = 0

    def same(a, b, k):
        for x, y in zip(a[:3], b[:3]):
            assert torch.equal(x.nan_to_num(7.0) if x.is_floating_point() else x,
                               y.nan_to_num(7.0) if y.is_floating_point() else y), k
        assert torch.equal(a[3]["collision"], b[3]["collision"]), k
        assert torch.equal(a[3]["final_observation"].nan_to_num(7.0), b[3]["final_observation"].nan_to_num(7.0)), k
        for name in ("p1", "v1", "p2", "v2", "ret1", "ret2", "tf", "won_mask"):
            assert torch.equal(getattr(plain, name), getattr(packed, name)), (name, k)

    for k in range(260):
        if k % 4 == 3:  # host actions; the L0 opponent (None) on odd rounds
            a1 = torch.from_numpy(rng.integers(0, 5, n).astype(np.int8)).cuda()
            a2 = None if k % 8 == 3 else torch.from_numpy(rng.integers(0, 5, n).astype(np.int8)).cuda()
            outs = plain.step(a1, a2), packed.step(a1, a2)
            assert torch.equal(packed.a1_buf, a1)
            assert torch.equal(packed.a2_buf, a2 if a2 is not None else torch.full_like(a1, -1))
        else:
            outs = (plain.step_random(seed, opponent_random=k % 2 == 0, step_idx=k),
                    packed.step_random(seed, opponent_random=k % 2 == 0, step_idx=k))
            assert torch.equal(plain.a1_buf, packed.a1_buf) and torch.equal(plain.a2_buf, packed.a2_buf), k
        same(*outs, k)
        ndone += int(packed.done.sum())
    assert ndone > 0
    plain.coll.fill_(9)
    packed.coll.fill_(9)
    assert torch.equal(plain.observe(), packed.observe())
    assert torch.equal(plain.coll, packed.coll) and int(packed.coll.max()) <= 1
    assert torch.equal(plain.done, packed.done)


def test_golden_one_step_rows(torch, golden):
    """The reference's own one-step outputs from 8,000 states near the boundaries."""
    from merging_gym import MergeVecEnv

    g = golden
    n = len(g["one_a1"])
    env = MergeVecEnv(n, device="cuda:0", autoreset=False)
    dev = env.device
    env.p1.copy_(torch.from_numpy(g["one_p"][:, 0]))
    env.p2.copy_(torch.from_numpy(g["one_p"][:, 1]))
    env.v1.copy_(torch.from_numpy(g["one_v"][:, 0]))
    env.v2.copy_(torch.from_numpy(g["one_v"][:, 1]))
    env.ret1.copy_(torch.from_numpy(g["one_racc"][:, 0]))
    env.ret2.copy_(torch.from_numpy(g["one_racc"][:, 1]))
    nat = env._nat
    tf = (np.minimum(g["one_k"].astype(np.int64), nat.TF_STEPS_MASK)
          | (g["one_winner"].astype(np.int64) << nat.TF_WINNER_SHIFT)
          | (g["one_done"].astype(np.int64) * nat.TF_DONE))
    env.tf.copy_(torch.from_numpy(tf.astype(np.uint16).view(np.int16)))
    obs, rew, done, info = env.step(torch.from_numpy(g["one_a1"]).to(dev), torch.from_numpy(g["one_a2"]).to(dev))
    coll = info["collision"].cpu().numpy()
    bad = coll != g["one_coll"]
    zone = merge_zone(g["one_pos"][:, 0], g["one_pos"][:, 1])
    print(f"golden one-step rows: {n}, in the merge zone: {int(zone.sum())}, collision flips: {int(bad.sum())}")
    assert bad.sum() == 0, np.nonzero(bad)
    np.testing.assert_array_equal(done.cpu().numpy(), g["one_done_out"])
    np.testing.assert_array_equal(env.winner.cpu().numpy(), g["one_winner_out"])
    np.testing.assert_allclose(obs.cpu().numpy(), g["one_obs"].astype(np.float32), **OBS_TOL)
    np.testing.assert_allclose(rew.cpu().numpy(), g["one_rew"].astype(np.float32), **OBS_TOL)
    np.testing.assert_allclose(env.p1.cpu().numpy(), g["one_pos"][:, 0], **STATE_TOL)
    np.testing.assert_allclose(env.p2.cpu().numpy(), g["one_pos"][:, 1], **STATE_TOL)
    np.testing.assert_allclose(env.ret1.cpu().numpy(), g["one_racc_out"][:, 0], **STATE_TOL)
    np.testing.assert_allclose(env.ret2.cpu().numpy(), g["one_racc_out"][:, 1], **STATE_TOL)


def test_sharding_matches_unsharded(torch):
    """Two shards with env_offset draw the same actions and reach the same state as one batch."""
    from merging_gym import MergeVecEnv

    n, steps, seed = 5000, 200, 3
    full = MergeVecEnv(n, device="cuda:0")
    a = MergeVecEnv(2048, device="cuda:0", env_offset=0)
    b = MergeVecEnv(n - 2048, device="cuda:0", env_offset=2048)
    for k in range(steps):
        full.step_random(seed, step_idx=k)
        a.step_random(seed, step_idx=k)
        b.step_random(seed, step_idx=k)
    for name in ("p1", "v1", "p2", "v2", "ret1", "ret2", "tf", "obs"):
        whole = getattr(full, name)
        parts = torch.cat([getattr(a, name), getattr(b, name)])
        assert torch.equal(whole, parts), name


def test_full_size_properties(torch, coracle):
    """Config 3 size (2^20 envs): invariants over the whole batch plus oracle spot checks of
    2,048 random envs (Philox is keyed by the global env index, so any env can be replayed)."""
    from merging_gym import MergeVecEnv

    n, steps, seed = 1 << 20, 300, 2024
    env = MergeVecEnv(n, device="cuda:0", done_mask=True)
    reset_row = env.obs[0].clone()
    for k in range(steps):
        obs, rew, done, info = env.step_random(seed, step_idx=k)
        if k % 40 == 39:
            d = done.cpu().numpy()
            # autoreset: finished envs show the reset observation
            assert torch.equal(obs[done], reset_row.expand(int(d.sum()), -1))
            # the ballot mask agrees with the done bytes
            words = env.done_mask.cpu().numpy().view(np.uint64)
            bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)
            np.testing.assert_array_equal(bits, d)
            assert not torch.isnan(obs).any()
    counts = env.counts.cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(counts[:, 3] + env.steps.cpu().numpy(), steps)
    assert counts[:, 0].sum() > 0
    idx = np.sort(np.random.default_rng(0).choice(n, 2048, replace=False))
    p1 = env.p1.cpu().numpy()[idx]
    r1 = env.ret1.cpu().numpy()[idx]
    c = counts[idx]
    for j, gi in enumerate(idx):
        e = coracle.new_envs(1)
        coracle.reset(e)
        rs, ct = mo.new_stats(1)
        coracle.rollout_random(e, steps, seed, 0, True, env_offset=int(gi), stats=(rs, ct))
        assert e["pos1"][0] == p1[j] and e["r1_acc"][0] == r1[j], gi
        np.testing.assert_array_equal(ct[0], c[j])


def test_invalid_actions_flag_error(torch):
    from merging_gym import MergeVecEnv

    env = MergeVecEnv(64, device="cuda:0", autoreset=False)
    a1 = torch.full((64,), 2, dtype=torch.int8, device="cuda:0")
    a1[5] = 9
    env.step(a1)
    with pytest.raises(KeyError):
        env.check_actions()
    assert int(env.steps[5]) == 1 and float(env.p1[5]) == 50.0  # clock advanced, car not
    env.step(torch.full((64,), 2, dtype=torch.int8, device="cuda:0"))
    env.check_actions()


def test_strict_actions_raise_at_step(torch):
    """strict_actions: step() itself raises KeyError like the reference's action_dict lookup
    (merging_env.py:101, :134-136); the flag is cleared, so the next valid step goes through."""
    from merging_gym import MergeVecEnv

    env = MergeVecEnv(64, device="cuda:0", autoreset=False, strict_actions=True)
    a1 = torch.full((64,), 2, dtype=torch.int8, device="cuda:0")
    a2 = a1.clone()
    a2[7] = 5
    with pytest.raises(KeyError):
        env.step(a1, a2)
    env.step(a1, None)
    assert int(env.steps[0]) == 2


def test_native_errors_are_raised(torch):
    from merging_gym import _native

    st = _native.State()
    out = _native.Outputs()
    rc = _native.lib.mg_step(ctypes.byref(_native.default_params()), ctypes.byref(st), None, None,
                             ctypes.byref(out), None, 16, 0, None)
    assert rc != 0 and b"NULL" in _native.lib.mg_last_error()


@pytest.mark.parametrize("n,T", [(4096, 37), (3001, 64), (1, 5)])
def test_rollout_equals_step_sequence(torch, n, T):
    """mg_rollout_random (env in registers for T steps) is bit-identical to T launches of
    mg_step_random, including autoreset, final observations and episode statistics."""
    from merging_gym import MergeVecEnv

    seed = 77
    a = MergeVecEnv(n, device="cuda:0")
    b = MergeVecEnv(n, device="cuda:0")
    for k in range(180):  # start mid-episode
        a.step_random(seed, step_idx=k)
        b.step_random(seed, step_idx=k)
    traj = {key: v.clone() if v is not None else None
            for key, v in b.rollout_random(T, seed, first_step=180).items()}
    for t in range(T):
        obs, rew, done, info = a.step_random(seed, step_idx=180 + t)
        assert torch.equal(traj["obs"][t], obs), t
        assert torch.equal(traj["rew"][t], rew), t
        assert torch.equal(traj["done"][t], done), t
        assert torch.equal(traj["collision"][t], info["collision"]), t
        assert torch.equal(traj["a1"][t], a.a1_buf) and torch.equal(traj["a2"][t], a.a2_buf), t
        assert torch.equal(traj["final_observation"][t][done], info["final_observation"][done]), t
    # the whole 64-byte statistics records, main.py's pending value included
    for name in ("p1", "v1", "p2", "v2", "ret1", "ret2", "tf", "returns", "counts", "_ep_stats"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert b._step_idx == 180 + T


def test_rollout_longer_than_one_launch_is_chunked_bit_exactly(torch):
    """rollout_random splits a rollout longer than mg_rollout_random's 65,535-step limit into
    consecutive launches that write slices of the same buffers (_traj_slice's row strides). T =
    65,535 + 37 steps of 96 envs against the same steps as one-step launches: the rows around the
    chunk boundary (obs, flags, final observations, won bits, rewards), the final state and the
    statistics records bit for bit."""
    from merging_gym import MergeVecEnv

    n, T, seed, k0 = 96, 65535 + 37, 91, 120
    a = MergeVecEnv(n, device="cuda:0", won_mask=True)
    b = MergeVecEnv(n, device="cuda:0")
    for k in range(k0):
        a.step_random(seed, step_idx=k)
        b.step_random(seed, step_idx=k)
    traj = b.rollout_random(T, seed, first_step=k0)
    torch.cuda.synchronize()
    check = set(range(65530, T)) | {0, 1}
    for t in range(T):
        obs, rew, done, info = a.step_random(seed, step_idx=k0 + t)
        if t in check:
            assert torch.equal(traj["obs"][t], obs), t
            assert torch.equal(traj["rew"][t], rew), t
            assert torch.equal(traj["done"][t], done) and torch.equal(traj["collision"][t], info["collision"]), t
            assert torch.equal(traj["a1"][t], a.a1_buf) and torch.equal(traj["a2"][t], a.a2_buf), t
            assert torch.equal(traj["final_observation"][t][done], info["final_observation"][done]), t
            assert torch.equal(traj["won_mask"][t], a.won_mask), t
    for name in ("p1", "v1", "p2", "v2", "ret1", "ret2", "tf", "returns", "counts", "_ep_stats"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert b._step_idx == k0 + T and int(b.counts[:, 0].sum()) > 20000  # ~300 episodes per env


def test_config4_size_and_64bit_env_index(torch, coracle):
    """Config 4's global batch (2^23 envs) stepped on one GPU: step-count bookkeeping over the
    whole batch and oracle replays at both ends of the index range; then a small shard whose
    global env indices exceed 2^32 (Philox counter high word) against the oracle."""
    from merging_gym import MergeVecEnv

    n, steps, seed = 1 << 23, 96, 4040
    env = MergeVecEnv(n, device="cuda:0", final_observation=False)
    for k in range(steps):
        env.step_random(seed, step_idx=k, record_actions=False)
    counts = env.counts.cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(counts[:, 3] + env.steps.cpu().numpy(), steps)
    idx = np.array([0, 1, 63, 64, 1 << 22, n - 65, n - 2, n - 1])
    p1, r2 = env.p1.cpu().numpy()[idx], env.ret2.cpu().numpy()[idx]
    del env
    for j, gi in enumerate(idx):
        e = coracle.new_envs(1)
        coracle.reset(e)
        coracle.rollout_random(e, steps, seed, 0, True, env_offset=int(gi))
        assert e["pos1"][0] == p1[j] and e["r2_acc"][0] == r2[j], gi

    off = (1 << 33) + 5
    small = MergeVecEnv(300, device="cuda:0", env_offset=off)
    for k in range(40):
        small.step_random(seed, step_idx=k)
    a1, a2 = coracle.random_actions(300, off, seed, 39, True)
    np.testing.assert_array_equal(small.a1_buf.cpu().numpy(), a1)
    np.testing.assert_array_equal(small.a2_buf.cpu().numpy(), a2)
    e = coracle.new_envs(300)
    coracle.reset(e)
    coracle.rollout_random(e, 40, seed, 0, True, env_offset=off)
    np.testing.assert_array_equal(small.p2.cpu().numpy(), e["pos2"])


def test_checkpoint_resume_is_bit_exact(torch):
    """MergeVecEnv.state_dict / load_state_dict (checkpoint / resume):
    saving mid-run, continuing, then restoring and replaying the same steps gives the same
    state, outputs and statistics bit for bit; a ReplayRing round-trips too."""
    import io

    from merging_gym import MergeVecEnv, ReplayRing

    env = MergeVecEnv(3001, device="cuda:0", won_mask=True)
    for k in range(150):
        env.step_random(11, step_idx=k)
    buf = io.BytesIO()
    torch.save(env.state_dict(), buf)
    outs = []
    for _ in range(120):
        obs, rew, done, info = env.step_random(11)
        outs.append((obs.clone(), rew.clone(), done.clone(), info["collision"].clone()))
    end = env.state_dict()
    traj_a = env.rollout_random(8, 3)
    traj_a = {k: v.clone() for k, v in traj_a.items() if v is not None}
    buf.seek(0)
    env2 = MergeVecEnv(3001, device="cuda:0", won_mask=True)
    env2.load_state_dict(torch.load(buf, weights_only=True))
    for j in range(120):
        obs, rew, done, info = env2.step_random(11)
        for a, b in zip(outs[j], (obs, rew, done, info["collision"])):
            assert torch.equal(a, b), j
    for k, v in env2.state_dict().items():
        assert (torch.equal(v, end[k]) if isinstance(v, torch.Tensor) else v == end[k]), k
    traj_b = env2.rollout_random(8, 3)
    for k, v in traj_a.items():  # final_observation holds NaN rows where no episode ended
        same = torch.allclose(v, traj_b[k], rtol=0, atol=0, equal_nan=True) if v.is_floating_point() \
            else torch.equal(v, traj_b[k])
        assert same, k
    ring = ReplayRing(64, device="cuda:0")
    ring.store_rollout(env.obs.clone(), traj_b)
    ring2 = ReplayRing(64, device="cuda:0")
    ring2.load_state_dict(ring.state_dict())
    assert torch.equal(ring2.memory, ring.memory) and ring2.memory_counter == ring.memory_counter
    with pytest.raises(ValueError):
        MergeVecEnv(3000, device="cuda:0").load_state_dict(end)
    # older checkpoints: ABI <= 16 arrays are refused (their main.py / win statistics are gone); ABI
    # 17-19 records load with q_eval unknown (NaN), not a silently diluted sum
    legacy = {k: v for k, v in end.items() if k not in ("episode_stats", "episode_stats_format")}
    legacy.update(ret_sum=torch.zeros((3001, 2), dtype=torch.float64), counts=torch.zeros((3001, 4), dtype=torch.int32))
    with pytest.raises(ValueError, match="ABI <= 16"):
        MergeVecEnv(3001, device="cuda:0").load_state_dict(legacy)
    fmt1 = {k: v for k, v in end.items() if k != "episode_stats_format"}
    env3 = MergeVecEnv(3001, device="cuda:0")
    env3.load_state_dict(fmt1)
    assert bool(torch.isnan(env3.q_eval).all()) and torch.equal(env3.returns, end["episode_stats"][:, :3])
