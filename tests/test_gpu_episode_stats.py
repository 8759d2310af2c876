"""The statistics the reference's training scripts log, computed on the device (SURVEY.md 8(f)
row 2), against the reference's own loops; and hdqn.py's goal_status on fp64 values.

* tests/golden/replay_golden.npz holds, per episode of four long trajectories of the reference
  env, what scripts/main.py:189-227 logs (ep_reward summed only after steps where `env.winner is
  not 1`, :209-211; a win when `state[8] > state[3]` on the observation the last step acted on,
  :218-225) and what scripts/hdqn.py:276-346 logs (ep_reward = every reward, :312; the same test
  on the terminal observation, :320, :342). MergeVecEnv replays the four action sequences as four
  envs of one batch through mg_step with autoreset; after every finished episode the env's
  64-byte record (include/merging_hip.h mg_episode_stats) must hold exactly that episode's
  values. The device keeps main.py's filtered sum as r1_accumulate before the ego-first step
  (winner stays 1 once set); the oracle and the golden loops filter step by step -- equal bit
  for bit, so the shortcut is the reference's sum.
* goal_status (hdqn.py:223-236): mg_goal_status -- the device function mg_rollout_hdqn evaluates --
  equals the reference's own goal_status on fp64 rows around its thresholds; and the fused h-DQN
  kernel's intrinsic reward follows the fp64 status on states built so that fp32 evaluation
  would disagree.
"""

import ctypes
import os

import numpy as np
import pytest

import merge_oracle as mo
from conftest import ROOT

pytestmark = pytest.mark.gpu

REPLAY = os.path.join(ROOT, "tests", "golden", "replay_golden.npz")
TAGS = ["SU0", "SUU", "SFU", "SSU"]


@pytest.fixture(scope="module")
def g():
    return np.load(REPLAY)


def _trace(g, tag):
    return {k[len(tag) + 1:]: g[k] for k in g.files if k.startswith(tag + "_")}


def test_device_statistics_equal_reference_loops(g):
    import torch

    from merging_gym import MergeVecEnv

    trs = [_trace(g, t) for t in TAGS]
    T = min(len(t["a1"]) for t in trs)
    n = len(trs)
    env = MergeVecEnv(n, device="cuda:0")
    a1 = torch.from_numpy(np.stack([t["a1"][:T] for t in trs], 1).astype(np.int8)).cuda()
    a2 = torch.from_numpy(np.stack([t["a2"][:T] for t in trs], 1).astype(np.int8)).cuda()  # -1 = None
    seen = [0] * n
    rec = env._ep_stats  # [n, 8] f64 view of the records
    for k in range(T):
        _, _, done, _ = env.step(a1[k], a2[k])
        d = done.cpu().numpy()
        if not d.any():
            continue
        r = env.returns.cpu().numpy()
        c = env.counts.cpu().numpy()
        for i in np.flatnonzero(d):
            e, t = seen[i], trs[i]
            assert r[i, 0] == t["hdqn_reward"][e] == t["r1_accumulate"][e], (TAGS[i], e)
            assert r[i, 1] == t["r2_accumulate"][e], (TAGS[i], e)
            assert r[i, 2] == t["main_reward"][e], (TAGS[i], e, r[i, 2], t["main_reward"][e])
            assert c[i].tolist() == [1, int(t["collision"][e]), int(t["winner"][e] == 1), int(t["length"][e]),
                                     int(t["main_win"][e]), int(t["hdqn_win"][e])], (TAGS[i], e, c[i])
            seen[i] += 1
        rec[torch.from_numpy(d).cuda(), :3] = 0.0  # sums; the pending value (column 3) is the next episode's
        rec[torch.from_numpy(d).cuda(), 4:] = 0.0  # counts
    assert sum(seen) > 100 and all(s >= 20 for s in seen), seen


def test_rollout_and_step_keep_the_same_records():
    """The T-step kernel (statistics held in registers, counts as 16-bit fields, the pending value
    carried across launches) leaves the records exactly as T one-step launches do, for several
    launch lengths over the same stream of episodes."""
    import torch

    from merging_gym import MergeVecEnv

    n, seed = 5000, 123
    a = MergeVecEnv(n, device="cuda:0")
    b = MergeVecEnv(n, device="cuda:0")
    k = 0
    for T in (1, 7, 64, 300, 16, 211):
        for t in range(T):
            a.step_random(seed, step_idx=k + t)
        b.rollout_random(T, seed, first_step=k)
        k += T
        assert torch.equal(a._ep_stats, b._ep_stats), T
    c = b.counts.to(torch.int64)
    assert int(c[:, 0].sum()) > 5000 and int(c[:, 4].sum()) > 0 and int(c[:, 5].sum()) > 0
    assert bool((b.ret_main != b.ret_sum[:, 0]).any())


def test_goal_status_device_rows(g):
    """mg_goal_status on the golden rows: the reference's goal_status, bit for bit."""
    import torch

    from merging_gym import _native

    dx1 = torch.from_numpy(g["GS_dx1"]).cuda()
    v2 = torch.from_numpy(g["GS_v2"]).cuda()
    out = torch.full(dx1.shape, -1, dtype=torch.int8, device="cuda:0")
    _native.check(_native.lib.mg_goal_status(dx1.data_ptr(), v2.data_ptr(), out.data_ptr(), dx1.numel(), None),
                  "mg_goal_status")
    np.testing.assert_array_equal(out.cpu().numpy(), g["GS_status"])


def _rec64_obs(env):
    """The kernel's own fp64 observation of every env (mg_observe into mg_rec64 records)."""
    import torch

    nat = env._nat
    buf = torch.empty((env.num_envs, nat.REC64_DTYPE.itemsize), dtype=torch.uint8, device=env.device)
    out = nat.Outputs()
    out.rec64 = ctypes.c_void_p(buf.data_ptr())
    nat.check(nat.lib.mg_observe(ctypes.byref(env.params), ctypes.byref(env._state), ctypes.byref(out),
                                 env.num_envs, None), "mg_observe")
    torch.cuda.synchronize()
    return buf.cpu().numpy().view(nat.REC64_DTYPE)["obs"].reshape(env.num_envs, 10)


def test_hdqn_intrinsic_reward_uses_fp64_goal_status():
    """States where goal_status differs between fp64 (the reference's Python floats) and fp32:
    dx1 = x2 - x1 of each env's positions (the kernel's own fp64 value), v2 = 2 |dx1| and its
    neighbouring doubles, so dx1 sits exactly on, or one ulp inside / outside, +-v2 / 2. One
    fused h-DQN step: its intrinsic reward (hdqn.py:314) must be 1 exactly where the goal chosen
    on the next state equals the fp64 status of the state acted on."""
    import torch

    from merging_gym import MergeVecEnv
    from merging_gym.policy import NUM_GOALS, QNet

    rng = np.random.default_rng(4)
    n = 3 * 2048
    env = MergeVecEnv(n, device="cuda:0")
    p1 = rng.uniform(300.0, 900.0, n // 3)
    p2 = p1 + rng.uniform(-25.0, 25.0, n // 3)
    for name, v in (("p1", np.repeat(p1, 3)), ("p2", np.repeat(p2, 3))):
        getattr(env, name).copy_(torch.from_numpy(v))
    o = _rec64_obs(env)
    dx1 = o[:, 0]
    base = 2.0 * np.abs(dx1)
    v2 = base.copy()
    v2[1::3] = np.nextafter(base[1::3], np.inf)
    v2[2::3] = np.nextafter(base[2::3], -np.inf)
    env.v2.copy_(torch.from_numpy(v2))
    status64 = mo.goal_status64(np.stack([dx1] + [np.zeros(n)] * 8 + [v2], 1))
    f32 = lambda x: x.astype(np.float32)  # noqa: E731
    status32 = np.where(f32(dx1) < np.float32(-0.5) * f32(v2), 0, np.where(f32(dx1) < np.float32(0.5) * f32(v2), 1, 2))
    assert (status64 != status32).sum() > n // 6  # the construction separates the two evaluations
    nets = np.random.default_rng(9)

    def net(i, out):
        sd = {}
        for name, (a, b) in zip(("fc1", "fc2", "out"), [(200, i), (100, 200), (out, 100)]):
            sd[f"{name}.weight"] = nets.uniform(-b ** -0.5, b ** -0.5, (a, b)).astype(np.float32)
            sd[f"{name}.bias"] = nets.uniform(-b ** -0.5, b ** -0.5, a).astype(np.float32)
        return QNet.from_state_dict(sd, device="cuda:0")

    tr = env.rollout_hdqn(1, net(10, NUM_GOALS), net(11, 5), seed=3, first_step=50)
    r_int = tr["reward"][0].cpu().numpy()
    g2 = tr["next_goal"][0].cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(r_int, (g2 == status64).astype(np.float32))
    # and some of those rewards are ones fp32 evaluation would have got wrong
    assert ((g2 == status64) != (g2 == status32)).sum() > 100


@pytest.mark.parametrize("n", [0, 1, 255, 1024, 1025, 70_001, (1 << 20) + 37])
def test_stats_reduce_fixed_order(n):
    """mg_stats_reduce (ABI 20) sums the 64-byte records in its documented fixed order: bit for bit
    the oracle's restatement (merge_oracle.stats_reduce_fixed) on records with mixed signs, widely
    spread magnitudes, -0.0 and non-trivial counts; partial_stats uses it for MergeVecEnv's record
    views, so summarize() of a batch is that order's result."""
    import torch

    from merging_gym.distributed import device_totals, partial_stats, summarize_partials

    rng = np.random.default_rng(n)
    rec = np.zeros((max(n, 1), 8))[:n]
    rec[:, :4] = rng.normal(0, 1, (n, 4)) * 10.0 ** rng.integers(-12, 6, (n, 4))
    rec[:, 7] = rng.normal(0, 1, n) * 10.0 ** rng.integers(-6, 4, n)  # q_eval
    if n:
        rec[:: 7, 0] = -0.0
        rec[:: 11, 2] = rng.uniform(-1e-300, 1e-300, rec[:: 11, 2].shape)
    cnt = rec[:, 4:].view(np.uint32)
    cnt[:, :6] = rng.integers(0, 1 << 31, (n, 6), dtype=np.uint32)
    dev = torch.from_numpy(rec.copy()).cuda()
    tot = device_totals(dev).cpu().numpy()
    sums, counts = mo.stats_reduce_fixed(rec)
    np.testing.assert_array_equal(tot[:4].view(np.float64).view(np.uint64),
                                  np.array(sums, np.float64).view(np.uint64))
    assert tot[4:].tolist() == counts
    if n:  # the MergeVecEnv views (returns [n,3], counts [n,6] i32) take the same path
        views = dev[:, :3], dev[:, 4:].view(torch.int32)[:, :6]
        assert torch.equal(partial_stats(*views).cpu(), torch.from_numpy(tot))
        s = summarize_partials(torch.from_numpy(tot))
        assert s["completed"] == counts[0] and s["mean_return_ego"] == sums[0] / counts[0]
        assert s["mean_q_eval"] == sums[3] / counts[0]


def test_stats_reduce_is_cheap_at_full_size():
    """At 2^20 envs the reduction reads 64 MB: it takes tens of microseconds once warm (the torch
    sum over strided record columns it replaces took 7.6 ms in the round-3 bench)."""
    import torch

    from merging_gym.distributed import device_totals

    rec = torch.zeros((1 << 20, 8), dtype=torch.float64, device="cuda")
    for _ in range(3):
        device_totals(rec)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        device_totals(rec)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"mg_stats_reduce at 2^20: {ms * 1e3:.1f} us per call")
    assert ms < 0.1


def test_clear_statistics_keeps_only_the_pending_value():
    """MergeVecEnv.clear_statistics (one int64 pass over whole records since round 4): every sum,
    count and q_eval becomes +0 and main.py's pending value (ret1_pending, the episode in progress)
    keeps its bits, so the episodes that finish after the clear are recorded as without it."""
    import torch

    from merging_gym import MergeVecEnv

    n = 4096
    env = MergeVecEnv(n, device="cuda:0")
    for k in range(400):
        env.step_random(5, step_idx=k)
    before = env._ep_stats.clone()
    assert int(env.counts[:, 0].sum()) > 0 and bool((before[:, 3] != 0).any())
    env.clear_statistics()
    after = env._ep_stats
    assert torch.equal(after[:, 3].view(torch.int64), before[:, 3].view(torch.int64))
    cols = [0, 1, 2, 4, 5, 6, 7]
    assert bool((after[:, cols].view(torch.int64) == 0).all())  # +0.0 and zero counts, bit for bit
    # the episodes after the clear: the same records as a twin batch cleared by field
    twin = MergeVecEnv(n, device="cuda:0")
    for k in range(400):
        twin.step_random(5, step_idx=k)
    twin.returns.zero_()
    twin.counts.zero_()
    twin.q_eval.zero_()
    for k in range(400, 700):
        env.step_random(5, step_idx=k)
        twin.step_random(5, step_idx=k)
    assert torch.equal(env._ep_stats.view(torch.int64), twin._ep_stats.view(torch.int64))
    assert int(env.counts[:, 0].sum()) > 0
