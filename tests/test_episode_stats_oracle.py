"""The statistics the reference's training scripts log per episode, pinned on the CPU oracles.

tests/golden/replay_golden.npz (gen_replay.py) holds them as the reference's own loops compute
them over the reference env: scripts/main.py:189-227 (ep_reward summed only after steps where
`env.winner is not 1`, :209-211; win = `state[8] > state[3]` on the observation the episode's last
step acted on, :218-225) and scripts/hdqn.py:276-346 (ep_reward = every step's reward, :312;
the same win test on the terminal observation, :320, :342). The C oracle (literal per-step
restatement) and the NumPy restatement must give every episode's values bit for bit; so must the
device kernels (tests/test_gpu_episode_stats.py).
"""

import os

import numpy as np
import pytest

import merge_numpy as mn
import merge_oracle as mo
from conftest import ROOT

REPLAY = os.path.join(ROOT, "tests", "golden", "replay_golden.npz")
STATS_TAGS = ["SU0", "SUU", "SFU", "SSU"]


@pytest.fixture(scope="module")
def g():
    return np.load(REPLAY)


def _trace(g, tag):
    return {k[len(tag) + 1:]: g[k] for k in g.files if k.startswith(tag + "_")}


def oracle_episodes(coracle, a1, a2):
    """Step one C-oracle env through the actions with autoreset; after every episode read and
    clear its statistics: per-episode (returns [3], counts [6]) rows (merge_oracle.STATS_DOC)."""
    envs = coracle.new_envs(1)
    coracle.reset(envs)
    ret, cnt = mo.new_stats(1)
    rows_r, rows_c = [], []
    for t in range(len(a1)):
        _, _, d, _, _, _, err = coracle.step(envs, a1[t:t + 1], None if a2[t] < 0 else a2[t:t + 1],
                                             autoreset=True, stats=(ret, cnt))
        assert err == 0
        if d[0]:
            rows_r.append(ret[0].copy())
            rows_c.append(cnt[0].copy())
            ret[:] = 0
            cnt[:] = 0
    return np.array(rows_r), np.array(rows_c)


@pytest.mark.parametrize("tag", STATS_TAGS)
def test_c_oracle_episode_statistics_equal_reference_loops(coracle, g, tag):
    tr = _trace(g, tag)
    r, c = oracle_episodes(coracle, tr["a1"], tr["a2"])
    assert len(r) == len(tr["length"]) > 20
    np.testing.assert_array_equal(r[:, 0], tr["hdqn_reward"])  # = r1_accumulate
    np.testing.assert_array_equal(r[:, 0], tr["r1_accumulate"])
    np.testing.assert_array_equal(r[:, 1], tr["r2_accumulate"])
    np.testing.assert_array_equal(r[:, 2], tr["main_reward"])
    np.testing.assert_array_equal(c[:, 0], 1)
    np.testing.assert_array_equal(c[:, 1].astype(bool), tr["collision"])
    np.testing.assert_array_equal(c[:, 2].astype(bool), tr["winner"] == 1)
    np.testing.assert_array_equal(c[:, 3], tr["length"])
    np.testing.assert_array_equal(c[:, 4].astype(bool), tr["main_win"])
    np.testing.assert_array_equal(c[:, 5].astype(bool), tr["hdqn_win"])


def test_golden_statistics_cover_the_cases(g):
    """The recorded trajectories exercise what makes the scripts' statistics differ from the
    plain ones: ego-first episodes (main.py's filter drops their tail), episodes whose two win
    tests disagree, and opponent-first / collision endings."""
    tr = {t: _trace(g, t) for t in STATS_TAGS}
    filt = sum(int((x["main_reward"] != x["hdqn_reward"]).sum()) for x in tr.values())
    ego_first = sum(int((x["winner"] == 1).sum()) for x in tr.values())
    differ = sum(int((x["main_win"] != x["hdqn_win"]).sum()) for x in tr.values())
    coll = sum(int(x["collision"].sum()) for x in tr.values())
    assert filt == ego_first > 50 and coll > 10 and differ >= 1, (filt, ego_first, coll, differ)
    # main.py's sum stops at the ego's first arrival: for an ego-first episode that ends without a
    # collision it omits the arrival bonus (RFirst = 2 less the speed penalty), so it is below the
    # full return by more than 1
    for x in tr.values():
        e = (x["winner"] == 1) & ~x["collision"]
        assert e.any() or not (x["winner"] == 1).any()
        assert (x["hdqn_reward"][e] - x["main_reward"][e] > 1.0).all()


@pytest.mark.parametrize("tag", ["L0", "RR"])
def test_main_loop_statistics(coracle, g, tag):
    """main.py's own loop (gen_replay.run: the DQN memory run) -- its reward_list and win test."""
    tr = _trace(g, tag)
    r, c = oracle_episodes(coracle, tr["a1"], tr["a2"])
    np.testing.assert_array_equal(r[:, 2], tr["ep_reward"])
    np.testing.assert_array_equal(c[:, 4].astype(bool), tr["ep_win"])


@pytest.mark.parametrize("tag", ["HL0", "HRR"])
def test_hdqn_loop_statistics(coracle, g, tag):
    """hdqn.py's own loop (gen_replay.run_hdqn) -- its reward_list and win test."""
    tr = _trace(g, tag)
    r, c = oracle_episodes(coracle, tr["a1"], tr["a2"])
    np.testing.assert_array_equal(r[:, 0], tr["ep_reward"])
    np.testing.assert_array_equal(c[:, 5].astype(bool), tr["ep_win"])


def test_numpy_restatement_episode_statistics(g):
    """The vectorised NumPy restatement, the four traces as four envs of one batch."""
    trs = [_trace(g, t) for t in STATS_TAGS]
    T = min(len(t["a1"]) for t in trs)
    nb = mn.NumpyMergeBatch(len(trs))
    a1 = np.stack([t["a1"][:T] for t in trs], 1).astype(np.int64)
    a2 = np.stack([t["a2"][:T] for t in trs], 1).astype(np.int64)
    seen = [0] * len(trs)
    for k in range(T):
        before_r, before_c = nb.ret_sum.copy(), nb.counts.copy()
        _, _, done, _ = nb.step(a1[k], a2[k])
        for i in np.flatnonzero(done):
            e, t = seen[i], trs[i]
            assert nb.ret_sum[i, 0] == before_r[i, 0] + t["hdqn_reward"][e]  # sums start at 0: exact per episode
            seen[i] += 1
            for col, key in ((4, "main_win"), (5, "hdqn_win")):
                assert nb.counts[i, col] - before_c[i, col] == int(t[key][e]), (i, e, key)
    for i, t in enumerate(trs):
        e = seen[i]
        np.testing.assert_array_equal(nb.counts[i, :4], [e, t["collision"][:e].sum(), (t["winner"][:e] == 1).sum(),
                                                         t["length"][:e].sum()])
        exp = 0.0
        for v in t["main_reward"][:e]:
            exp += v
        assert nb.ret_sum[i, 2] == exp


def test_goal_status_rows(g):
    """hdqn.py's goal_status (:223-236) itself, on fp64 values at and around its thresholds:
    merging_gym.policy.goal_status (the list form the drop-in callers use) agrees on every row;
    evaluating the same rows after rounding to fp32 would not (what ABI <= 16's kernel did)."""
    from merging_gym.policy import goal_status

    dx1, v2, st = g["GS_dx1"], g["GS_v2"], g["GS_status"]
    got = np.array([goal_status([d, 0, 0, 0, 0, 0, 0, 0, 0, v]) for d, v in zip(dx1, v2)])
    np.testing.assert_array_equal(got, st)
    f32 = np.where(dx1.astype(np.float32) < np.float32(-0.5) * v2.astype(np.float32), 0,
                   np.where(dx1.astype(np.float32) < np.float32(0.5) * v2.astype(np.float32), 1, 2))
    assert (f32 != st).sum() > 10  # the rows do separate fp64 from fp32 evaluation


def test_stats_reduce_restatement_order():
    """merge_oracle.stats_reduce_fixed (the checker of mg_stats_reduce) against a scalar loop written
    from the header's description (include/merging_hip.h mg_stats_reduce): thread-strided adds onto
    -0.0, then the halving fold, per block and over the block partials."""
    import numpy as np

    import merge_oracle as mo

    def fold(v):
        v = list(v)
        o = len(v) // 2
        while o:
            v = [v[t] + v[t + o] for t in range(o)]
            o //= 2
        return v[0]

    def scalar(col):
        n = len(col)
        parts = []
        for b in range((n + 1023) // 1024):
            th = []
            for t in range(256):
                a = -0.0
                for j in range(4):
                    i = b * 1024 + j * 256 + t
                    if i < n:
                        a = a + col[i]
                th.append(a)
            parts.append(fold(th))
        th = []
        for t in range(256):
            a = -0.0
            for k in range(t, len(parts), 256):
                a = a + parts[k]
            th.append(a)
        return fold(th)

    rng = np.random.default_rng(4)
    for n in (0, 5, 1024, 3000):
        rec = rng.normal(0, 1, (n, 8)) * 10.0 ** rng.integers(-9, 5, (n, 8))
        sums, _ = mo.stats_reduce_fixed(rec)
        for k, col in enumerate((0, 1, 2, 7)):
            ref = scalar(rec[:, col].tolist())
            assert np.float64(sums[k]).view(np.uint64) == np.float64(ref).view(np.uint64), (n, k)


def test_q_eval_golden_semantics():
    """The q_eval the scripts log (tests/golden/gen_replay.py ran the reference's own loops):
    main.py:221 evaluates eval_net on the state the episode's last step acted on, at that step's
    action; hdqn.py:330 evaluates meta_eval_net on the terminal state, at the goal chosen on it.
    Replaying the recorded actions through the oracle env finds exactly those states, and the
    oracle's fp32 Net (merge_oracle.qnet_reference) gives the logged values -- the quantities the
    config-5 and h-DQN kernels add to mg_episode_stats.q_eval (checked on the GPU against the
    bf16-emulated nets, tests/choice_check.check_q_eval)."""
    import os

    import numpy as np

    import merge_oracle as mo
    from conftest import ROOT

    g = np.load(os.path.join(ROOT, "tests", "golden", "replay_golden.npz"))
    ck = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    l1 = {k.split("/", 1)[1]: ck[k] for k in ck.files if k.startswith("l1/")}
    # main.py: the pre-terminal state and the last action
    env, k, pre, last = mo.PyMergeEnv(), 0, [], []
    for _ in range(len(g["QM_q_eval"])):
        state = env.reset()
        while True:
            a = int(g["QM_actions"][k])
            k += 1
            nxt, _, done, _ = env.step(a, None)
            if done:
                break
            state = nxt
        pre.append(state)
        last.append(a)
    assert k == len(g["QM_actions"])
    np.testing.assert_allclose(np.asarray(pre, float), g["QM_state"], rtol=0, atol=1e-9)
    np.testing.assert_array_equal(last, g["QM_action"])
    q = mo.qnet_reference(l1, g["QM_state"].astype(np.float32), bf16=False)
    np.testing.assert_allclose(q[np.arange(len(last)), g["QM_action"]], g["QM_q_eval"], rtol=1e-5, atol=1e-6)
    # hdqn.py: the terminal state and the goal chosen on it
    meta = {k[len("QH_net_"):]: g[k] for k in g.files if k.startswith("QH_net_")}
    env, k, term = mo.PyMergeEnv(), 0, []
    for _ in range(len(g["QH_q_eval"])):
        env.reset()
        done = False
        while not done:
            nxt, _, done, _ = env.step(int(g["QH_actions"][k]), None)
            k += 1
        term.append(nxt)
    assert k == len(g["QH_actions"])
    np.testing.assert_allclose(np.asarray(term, float), g["QH_state"], rtol=0, atol=1e-9)
    qh = mo.qnet_reference(meta, g["QH_state"].astype(np.float32), bf16=False)
    np.testing.assert_allclose(qh[np.arange(len(term)), g["QH_goal"]], g["QH_q_eval"], rtol=1e-5, atol=1e-6)
