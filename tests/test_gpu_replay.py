"""GPU parity for the device replay memory (mg_replay_store / mg_replay_sample, ReplayRing):
the reference's DQN.store_transition (scripts/main.py:115-119) under main.py:209's
`if env.winner is not 1` filter, and learn()'s minibatch draw (:130-135).

Bar: the ring contents and memory_counter equal the oracle's (merge_oracle.replay_store, itself
pinned to the reference's own memory in test_replay_oracle.py) bit for bit on the same inputs;
the won bits the kernels emit equal the CPU oracle's winner == 1 after each step; sampled rows
are exactly memory[idx] with idx the oracle's Philox slots.
"""

import os

import numpy as np
import pytest

import merge_oracle as mo
from conftest import ROOT

pytestmark = pytest.mark.gpu

OBS_TOL = dict(rtol=1e-6, atol=1e-5)


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


def _unpack(mask, n):
    """[..., ceil(n/64)] int64 words -> [..., n] bool (bit j of word w = env 64w + j)."""
    m = np.ascontiguousarray(mask).view(np.uint64)
    bits = (m[..., :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)
    return bits.reshape(*m.shape[:-1], -1)[..., :n].astype(bool)


def test_reference_run_through_the_ring(torch):
    """The reference fixture's action sequence through MergeVecEnv(1) + one store per step:
    the GPU ring equals the reference's memory (fp32) and counter."""
    from merging_gym import MergeVecEnv, ReplayRing

    g = np.load(os.path.join(ROOT, "tests", "golden", "replay_golden.npz"))
    for tag in ("L0", "RR"):
        a1, a2 = g[f"{tag}_a1"], g[f"{tag}_a2"]
        env = MergeVecEnv(1, device="cuda:0", won_mask=True)
        ring = ReplayRing(int(g[f"{tag}_capacity"]), device="cuda:0")
        prev = env.reset().clone()
        a1_d = torch.from_numpy(a1.astype(np.int8)).cuda()
        a2_d = torch.from_numpy(a2.astype(np.int8)).cuda()
        for k in range(len(a1)):
            obs, rew, done, info = env.step(a1_d[k:k + 1], a2_d[k:k + 1])
            ring.store(prev, obs, a1_d[k:k + 1], rew, done, info["final_observation"], env.won_mask)
            prev = obs.clone()
        assert ring.memory_counter == int(g[f"{tag}_counter"])
        np.testing.assert_allclose(ring.memory.cpu().numpy(), g[f"{tag}_memory"].astype(np.float32),
                                   **OBS_TOL)


@pytest.mark.parametrize("n,T,cap,opp", [(4096, 24, 200_000, True), (1000, 16, 5_000, False),
                                         (577, 9, 7, True), (64, 3, 1, True)])
def test_rollout_store_matches_oracle(torch, coracle, n, T, cap, opp):
    """A rollout's won bits equal the oracle's; storing the trajectory gives the oracle's ring
    (no wrap, wrap within one store, capacity far below one store, capacity 1)."""
    from merging_gym import MergeVecEnv, ReplayRing

    seed = 23
    env = MergeVecEnv(n, device="cuda:0")
    # random play arrives near step 225 and an L0 opponent exactly there (ending every episode
    # the ego won first): start where some envs have won and some not yet
    k0 = 230 if opp else 205
    for k in range(k0):
        env.step_random(seed + 1, opponent_random=opp, step_idx=k)
    envs = coracle.new_envs(n)
    for name, src in (("pos1", env.p1), ("vel1", env.v1), ("pos2", env.p2), ("vel2", env.v2),
                      ("r1_acc", env.ret1), ("r2_acc", env.ret2)):
        envs[name] = src.cpu().numpy()
    envs["steps"] = env.steps.cpu().numpy()
    envs["winner"] = env.winner.cpu().numpy()
    envs["time_stamp"] = np.cumsum(np.full(2700, 0.2))[np.maximum(envs["steps"] - 1, 0)] * (envs["steps"] > 0)
    obs0 = env.observe().clone()
    traj = env.rollout_random(T, seed, opponent_random=opp, first_step=k0)
    a1, a2 = traj["a1"].cpu().numpy(), traj["a2"].cpu().numpy()
    won_gpu = _unpack(traj["won_mask"].cpu().numpy(), n)
    for t in range(T):
        _, _, _, _, _, won, err = mo.step_with_won(coracle, envs, a1[t], a2[t] if opp else None)
        assert err == 0
        np.testing.assert_array_equal(won_gpu[t], won, err_msg=str(t))
    if n >= 1000:
        assert won_gpu.any() and not won_gpu.all()

    ring = ReplayRing(cap, device="cuda:0")
    ring.store_rollout(obs0, traj)
    ring.store_rollout(traj["obs"][-1].clone(), traj)  # a second store continues the ring
    mem = np.zeros((cap, 22), np.float32)
    host = {k: (v.cpu().numpy() if v is not None else None) for k, v in traj.items()}
    c = mo.replay_store(mem, 0, obs0.cpu().numpy(), host["obs"], host["a1"], host["rew"], host["done"],
                        host["final_observation"], won_gpu)
    c = mo.replay_store(mem, c, host["obs"][-1], host["obs"], host["a1"], host["rew"], host["done"],
                        host["final_observation"], won_gpu)
    assert ring.memory_counter == c
    np.testing.assert_array_equal(ring.memory.cpu().numpy(), mem)


def test_store_without_filter_and_single_transition(torch):
    from merging_gym import ReplayRing

    ring = ReplayRing(5, device="cuda:0")
    rows = []
    for k in range(8):  # wraps: slots 0..4 then 0..2 again
        s = [float(k + j) for j in range(10)]
        s2 = [float(100 + k + j) for j in range(10)]
        ring.store_transition(s, k % 5, -0.5 * k, s2)
        rows.append(np.hstack((s, [k % 5, -0.5 * k], s2)))
    assert ring.memory_counter == 8
    exp = np.zeros((5, 22), np.float32)
    for k, r in enumerate(rows):
        exp[k % 5] = r
    np.testing.assert_array_equal(ring.memory.cpu().numpy(), exp)
    with pytest.raises(ValueError):
        ring.store(torch.zeros((2, 10), device="cuda:0"), torch.zeros((1, 2, 10), device="cuda:0"),
                   torch.zeros((1, 2), dtype=torch.int8, device="cuda:0"),
                   torch.zeros((1, 2, 2), device="cuda:0"))  # filter asked for, no won bits
    from merging_gym import MergeVecEnv

    env = MergeVecEnv(64, device="cuda:0")
    traj = env.rollout_random(4, 1, final_observation=False)
    with pytest.raises(ValueError):  # episode ends need the terminal observation
        ring.store_rollout(env.obs.clone(), traj)


def test_step_won_mask_matches_oracle(torch, coracle):
    from merging_gym import MergeVecEnv

    n, seed = 3001, 5
    env = MergeVecEnv(n, device="cuda:0", won_mask=True)
    envs = coracle.new_envs(n)
    coracle.reset(envs)
    seen = False
    for k in range(260):
        env.step_random(seed, step_idx=k)
        a1, a2 = env.a1_buf.cpu().numpy(), env.a2_buf.cpu().numpy()
        _, _, _, _, _, won, err = mo.step_with_won(coracle, envs, a1, a2)
        assert err == 0
        np.testing.assert_array_equal(_unpack(env.won_mask.cpu().numpy(), n), won, err_msg=str(k))
        seen |= bool(won.any())
    assert seen


@pytest.mark.parametrize("filled_only", [False, True])
def test_sample_rows_are_memory_at_oracle_slots(torch, coracle, filled_only):
    from merging_gym import ReplayRing

    cap = 2000
    ring = ReplayRing(cap, device="cuda:0")
    ring.memory.copy_(torch.arange(cap * 22, dtype=torch.float32, device="cuda:0").view(cap, 22))
    ring._counter.fill_(1234)
    rows, idx = ring.sample_rows(4096, seed=9, draw=77, filled_only=filled_only, return_index=True)
    exp_idx = mo.replay_sample_index(coracle, cap, 1234, 9, 77, 4096, filled_only)
    np.testing.assert_array_equal(idx.cpu().numpy(), exp_idx)
    np.testing.assert_array_equal(rows.cpu().numpy(), ring.memory.cpu().numpy()[exp_idx])
    s, a, r, s2 = ring.sample(128, seed=9, draw=77, filled_only=filled_only)
    assert s.shape == (128, 10) and a.shape == (128, 1) and a.dtype == torch.int64
    assert r.shape == (128, 1) and s2.shape == (128, 10)


def test_goal_ring_reference_run(torch):
    """hdqn.py's lower-level memory: the reference run's goals, intrinsic rewards and actions
    (tests/golden/replay_golden.npz, HL0 / HRR) through MergeVecEnv(1) + a goal ring, one store
    per step: the ring equals the reference's [2000, 24] memory and counter."""
    from merging_gym import MergeVecEnv, ReplayRing

    g = np.load(os.path.join(ROOT, "tests", "golden", "replay_golden.npz"))
    for tag in ("HL0", "HRR"):
        a1, a2 = g[f"{tag}_a1"], g[f"{tag}_a2"]
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        goal, goal2, r_int = dev(g[f"{tag}_goal"][:, None]), dev(g[f"{tag}_next_goal"][:, None]), \
            dev(g[f"{tag}_intrinsic"][:, None])
        env = MergeVecEnv(1, device="cuda:0")
        ring = ReplayRing(int(g[f"{tag}_capacity"]), device="cuda:0", goal=True)
        prev = env.reset().clone()
        a1_d, a2_d = dev(a1.astype(np.int8)), dev(a2.astype(np.int8))
        for k in range(len(a1)):
            obs, rew, done, info = env.step(a1_d[k:k + 1], a2_d[k:k + 1])
            ring.store(prev, obs, a1_d[k:k + 1], rew, done, info["final_observation"], skip_ego_won=False,
                       goal=goal[k], next_goal=goal2[k], reward=r_int[k])
            prev = obs.clone()
        assert ring.memory_counter == int(g[f"{tag}_counter"])
        np.testing.assert_allclose(ring.memory.cpu().numpy(), g[f"{tag}_memory"].astype(np.float32), **OBS_TOL)


@pytest.mark.parametrize("cap", [7, 20_000])
def test_goal_rows_match_oracle(torch, coracle, cap):
    """Goal rows [goal, s, a, r, next_goal, s'] (24 floats, hdqn.py:158) with a reward column
    override, over stores of several shapes: bit-exact with the oracle; sampled rows are the
    memory at the oracle's slots and slice into hdqn.py:196-199's 11-value goal states."""
    from merging_gym import ReplayRing

    rng = np.random.default_rng(cap)
    ring = ReplayRing(cap, device="cuda:0", goal=True)
    mem = np.zeros((cap, 24), np.float32)
    c = 0
    dev = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    for n, T in ((3000, 7), (5, 1), (257, 33)):
        obs0 = rng.standard_normal((n, 10)).astype(np.float32)
        obs = rng.standard_normal((T, n, 10)).astype(np.float32)
        fobs = rng.standard_normal((T, n, 10)).astype(np.float32)
        a1 = rng.integers(0, 5, (T, n)).astype(np.int8)
        rew = rng.standard_normal((T, n, 2)).astype(np.float32)
        done = (rng.random((T, n)) < 0.1).astype(np.uint8)
        goal = rng.integers(0, 3, (T, n)).astype(np.float32)
        goal2 = rng.integers(0, 3, (T, n)).astype(np.float32)
        r_int = (rng.random((T, n)) < 0.3).astype(np.float32)
        ring.store(dev(obs0), dev(obs), dev(a1), dev(rew), dev(done), dev(fobs), skip_ego_won=False,
                   goal=dev(goal), next_goal=dev(goal2), reward=dev(r_int))
        c = mo.replay_store(mem, c, obs0, obs, a1, rew, done, fobs, None, skip_ego_won=False, goal=goal,
                            next_goal=goal2, reward=r_int)
        assert ring.memory_counter == c, (n, T)
        np.testing.assert_array_equal(ring.memory.cpu().numpy(), mem, err_msg=str((n, T)))
    rows, idx = ring.sample_rows(512, seed=3, draw=5, return_index=True)
    exp_idx = mo.replay_sample_index(coracle, cap, c, 3, 5, 512)
    np.testing.assert_array_equal(idx.cpu().numpy(), exp_idx)
    np.testing.assert_array_equal(rows.cpu().numpy(), mem[exp_idx])
    s, a, r, s2 = ring.sample(128, seed=3, draw=6)
    assert s.shape == (128, 11) and a.shape == (128, 1) and r.shape == (128, 1) and s2.shape == (128, 11)
    with pytest.raises(ValueError):  # a goal ring needs the goal columns
        ring.store(dev(obs0), dev(obs), dev(a1), dev(rew), skip_ego_won=False)


def test_mixed_size_stores_share_scratch(torch):
    """Stores of different shapes through one ring (the scratch buffer is reused across
    sizes); random won words, including bits past n that must be ignored; random done rows
    taking s' from final_obs."""
    from merging_gym import ReplayRing

    rng = np.random.default_rng(42)
    cap = 20_000
    ring = ReplayRing(cap, device="cuda:0")
    mem = np.zeros((cap, 22), np.float32)
    c = 0
    for n, T in ((3000, 7), (5, 1), (700, 33), (1, 2), (3000, 7), (257, 64)):
        obs0 = rng.standard_normal((n, 10)).astype(np.float32)
        obs = rng.standard_normal((T, n, 10)).astype(np.float32)
        fobs = rng.standard_normal((T, n, 10)).astype(np.float32)
        a1 = rng.integers(0, 5, (T, n)).astype(np.int8)
        rew = rng.standard_normal((T, n, 2)).astype(np.float32)
        done = (rng.random((T, n)) < 0.1).astype(np.uint8)
        words = rng.integers(0, 2**63, (T, (n + 63) // 64), dtype=np.int64)
        words &= rng.integers(0, 2**63, words.shape, dtype=np.int64)  # ~25% of bits set
        dev = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
        ring.store(dev(obs0), dev(obs), dev(a1), dev(rew), dev(done), dev(fobs), dev(words))
        c = mo.replay_store(mem, c, obs0, obs, a1, rew, done, fobs, _unpack(words, n))
        assert ring.memory_counter == c, (n, T)
        np.testing.assert_array_equal(ring.memory.cpu().numpy(), mem, err_msg=str((n, T)))


def test_goal_dqn_ring_reference_run(torch):
    """Goal_DQN's memory (Goal_DQN.store_transition :97-101 at hdqn.py:325): the reference run's
    actions and goals (tests/golden/replay_golden.npz, HL0 / HRR, gen_replay.run_hdqn) through
    MergeVecEnv(1); at every inner-loop break or episode end the row [s', goal, extrinsic_reward,
    s'] (extrinsic reward summed in fp64 from the env's rewards since the loop began, :286,
    :311-313) goes through the device store's Goal_DQN mode. The ring equals the reference's
    [200, 22] memory and counter (obs to fp32 tolerance, the rest exact)."""
    from merging_gym import MergeVecEnv, ReplayRing

    g = np.load(os.path.join(ROOT, "tests", "golden", "replay_golden.npz"))
    for tag in ("HL0", "HRR"):
        a1, a2, goal2 = g[f"{tag}_a1"], g[f"{tag}_a2"], g[f"{tag}_next_goal"]
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        env = MergeVecEnv(1, device="cuda:0")
        ring = ReplayRing(int(g[f"{tag}_meta_capacity"]), device="cuda:0")
        prev = env.reset().clone()
        a1_d, a2_d = dev(a1.astype(np.int8)), dev(a2.astype(np.int8))
        acc = 0.0
        for k in range(len(a1)):
            obs, rew, done, info = env.step(a1_d[k:k + 1], a2_d[k:k + 1])
            acc += float(rew[0, 0])  # the fp32 reward the batched API returns, summed in fp64
            s2 = info["final_observation"] if bool(done[0]) else obs
            st = s2.cpu().numpy()[0].astype(np.float64)
            status = 0 if st[0] < -0.5 * st[9] else (1 if st[0] < 0.5 * st[9] else 2)
            brk = bool(done[0]) or int(goal2[k]) == status
            nb = torch.tensor([0 if brk else 1], dtype=torch.int64, device="cuda:0")  # one step's mask word
            ring.store(prev, obs, a1_d[k:k + 1], rew, done, info["final_observation"], nb, True, None, None,
                       torch.tensor([acc], dtype=torch.float32, device="cuda:0"),
                       meta_goal=torch.tensor([float(goal2[k])], device="cuda:0"))
            if brk:
                acc = 0.0
            prev = obs.clone()
        assert ring.memory_counter == int(g[f"{tag}_meta_counter"])
        np.testing.assert_allclose(ring.memory.cpu().numpy(), g[f"{tag}_meta_memory"].astype(np.float32), **OBS_TOL)


@pytest.mark.parametrize("cap", [7, 200])
def test_goal_dqn_rows_match_oracle(torch, cap):
    """Goal_DQN rows [s', meta_goal, r, s'] (22 floats) kept where the no-break bit is clear, over
    stores of several shapes on random inputs: bit-exact with the oracle's replay_store."""
    from merging_gym import ReplayRing

    rng = np.random.default_rng(cap + 1)
    ring = ReplayRing(cap, device="cuda:0")
    mem = np.zeros((cap, 22), np.float32)
    c = 0
    dev = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    for n, T in ((3000, 7), (5, 1), (257, 33)):
        obs0 = rng.standard_normal((n, 10)).astype(np.float32)
        obs = rng.standard_normal((T, n, 10)).astype(np.float32)
        fobs = rng.standard_normal((T, n, 10)).astype(np.float32)
        a1 = rng.integers(0, 5, (T, n)).astype(np.int8)
        rew = rng.standard_normal((T, n, 2)).astype(np.float32)
        done = (rng.random((T, n)) < 0.1).astype(np.uint8)
        goal2 = rng.integers(0, 3, (T, n)).astype(np.float32)
        ext = rng.standard_normal((T, n)).astype(np.float32)
        nobrk = rng.random((T, n)) < 0.8
        words = np.zeros((T, (n + 63) // 64), np.uint64)
        for t in range(T):
            bits = np.zeros(words.shape[1] * 64, np.uint8)
            bits[:n] = nobrk[t]
            words[t] = np.packbits(bits, bitorder="little").view(np.uint64)
        ring.store(dev(obs0), dev(obs), dev(a1), dev(rew), dev(done), dev(fobs), dev(words.view(np.int64)), True,
                   reward=dev(ext), meta_goal=dev(goal2))
        c = mo.replay_store(mem, c, obs0, obs, a1, rew, done, fobs, nobrk, reward=ext, meta_goal=goal2)
        assert ring.memory_counter == c, (n, T)
        np.testing.assert_array_equal(ring.memory.cpu().numpy(), mem, err_msg=str((n, T)))
