"""hdqn.py's acting-and-storing inner loop (scripts/hdqn.py:280-323) batched on the device with
this package's pieces: Goal_DQN's meta-net picks goals (QNet, in 10 -> 3), the lower-level net
acts on goal states [goal] + state (QNet, in 11 -> 5), MergeVecEnv steps (L0 opponent),
goal_status gives the intrinsic reward, a goal ReplayRing stores HDQN.store_transition's rows.

Bar: every env transition equals the CPU oracle's given the loop's actions; the ring equals the
oracle's replay_store of the loop's own arrays bit for bit; the goal and action choices are the
argmax of the bf16-emulated nets wherever the loop was greedy (near-ties excused, as in
test_gpu_qnet.py). The nets are seeded draws with hdqn.py:41-47's initialisation (no h-DQN
checkpoint ships with the reference); exploration uses torch's device generator.
"""

import numpy as np
import pytest

import merge_oracle as mo
from choice_check import ChoiceCheck, check_q_eval, exact_q, order_matched_q

pytestmark = pytest.mark.gpu

OBS_TOL = dict(rtol=1e-6, atol=1e-5)


def _net(rng, in_dim, out_dim):
    sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), [(200, in_dim), (100, 200), (out_dim, 100)]):
        sd[f"{name}.weight"] = rng.uniform(0, 1, (o, i)).astype(np.float32)  # hdqn.py:41-47
        sd[f"{name}.bias"] = rng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    return sd


def _net_signed(rng, in_dim, out_dim):
    """torch.nn.Linear's default initialisation, U(-1/sqrt(in), 1/sqrt(in)) for weights and
    biases: signed weights, so the greedy choice varies from env to env and depends on every
    input feature (the seeded uniform(0, 1) nets of hdqn.py:41-47 pick nearly one action)."""
    sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), [(200, in_dim), (100, 200), (out_dim, 100)]):
        sd[f"{name}.weight"] = rng.uniform(-i ** -0.5, i ** -0.5, (o, i)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    return sd


def _selector_net(c=10.0):
    """A lower-level Net (11 -> 5) whose greedy choice reads one input: Q0 = relu(x[1]),
    Q1 = c, Q2..4 = 0, so argmax = 0 iff x[1] > c. x[1] is state[0] on the ego's goal state and
    state[5] on the opponent's swapped one (hdqn.py:291, :299) -- the feature a swap that drops
    an element would lose. (Seeded uniform nets, hdqn.py:41-47, pick nearly the same action for
    every env and would not notice.)"""
    sd = {"fc1.weight": np.zeros((200, 11), np.float32), "fc1.bias": np.zeros(200, np.float32),
          "fc2.weight": np.zeros((100, 200), np.float32), "fc2.bias": np.zeros(100, np.float32),
          "out.weight": np.zeros((5, 100), np.float32), "out.bias": np.zeros(5, np.float32)}
    sd["fc1.weight"][0, 1] = 1.0
    sd["fc2.weight"][0, 0] = 1.0
    sd["out.weight"][0, 0] = 1.0
    sd["out.bias"][1] = c
    return sd


# excused greedy choices (tests/choice_check.py), per kind of net (hdqn.py:41-47's uniform(0, 1)
# draws, signed draws, one-feature selector nets)
MAX_EXCUSED = {"uniform": 1e-4, "signed": 1e-4, "selector": 1e-4}  # round 3 measured 0 of > 10^6


def _kind(opponent):
    return "signed" if opponent.endswith("-signed") else ("selector" if opponent.endswith("-selector") else "uniform")


def test_batched_hdqn_inner_loop(coracle):
    import torch

    from merging_gym import MergeVecEnv, ReplayRing
    from merging_gym.policy import EPISILO, NUM_GOALS, QNet, goal_status

    n, T, cap, dev = 2048, 40, 50_000, "cuda:0"
    rng = np.random.default_rng(12)
    meta_sd, lower_sd = _net(rng, 10, NUM_GOALS), _net(rng, 11, 5)
    meta, lower = QNet.from_state_dict(meta_sd, device=dev), QNet.from_state_dict(lower_sd, device=dev)
    gen = torch.Generator(device=dev).manual_seed(3)
    p_greedy = 0.5 * (1.0 + float(torch.erf(torch.tensor(EPISILO / 2 ** 0.5))))  # P(randn <= EPISILO)

    def eps_greedy(q, k):  # choose_goal / choose_action (hdqn.py:82-95, :165-177)
        greedy = torch.rand(q.shape[0], generator=gen, device=dev) < p_greedy
        rand = torch.randint(0, k, (q.shape[0],), generator=gen, device=dev)
        return torch.where(greedy, q.argmax(1), rand), greedy

    env = MergeVecEnv(n, device=dev, final_observation=True)
    ring = ReplayRing(cap, device=dev, goal=True)
    for k in range(190):  # start mid-episode so that episodes end inside the loop
        env.step_random(5, opponent_random=False, step_idx=k)
    envs = coracle.new_envs(n)
    for name, src in (("pos1", env.p1), ("vel1", env.v1), ("pos2", env.p2), ("vel2", env.v2),
                      ("r1_acc", env.ret1), ("r2_acc", env.ret2)):
        envs[name] = src.cpu().numpy()
    envs["steps"] = env.steps.cpu().numpy()
    envs["winner"] = env.winner.cpu().numpy()
    envs["time_stamp"] = np.cumsum(np.full(2700, 0.2))[np.maximum(envs["steps"] - 1, 0)] * (envs["steps"] > 0)
    obs = env.observe().clone()
    goal, _ = eps_greedy(meta.forward(obs), NUM_GOALS)  # :283
    rec = {k: [] for k in ("obs0", "obs", "fobs", "a1", "rew", "done", "goal", "goal2", "r_int")}
    cc = ChoiceCheck("host h-DQN loop, lower net (uniform init)", max_frac=MAX_EXCUSED["uniform"])
    for t in range(T):
        x = torch.cat([goal[:, None].to(torch.float32), obs], dim=1)  # goal_state, :291
        q1 = lower.forward(x)
        a1, greedy1 = eps_greedy(q1, 5)  # :292
        q1_ref = mo.qnet_reference(lower_sd, x.cpu().numpy(), bf16=True)
        g1 = greedy1.cpu().numpy()
        got = a1.cpu().numpy()
        cc.check(got, np.where(g1, q1_ref.argmax(1), got), g1, q1_ref, f"step {t}",
                 q_exact=exact_q(lower_sd, x.cpu().numpy()))
        nobs, rew, done, info = env.step(a1.to(torch.int8), None)  # :302, L0 opponent
        s2 = torch.where(done[:, None], info["final_observation"], nobs)  # next_state before any reset
        q2 = meta.forward(s2)
        goal2, _ = eps_greedy(q2, NUM_GOALS)  # :303
        r_int = (goal2 == goal_status(obs)).to(torch.float32)  # :314
        ring.store(obs, nobs, a1.to(torch.int8), rew, done, info["final_observation"], skip_ego_won=False,
                   goal=goal.to(torch.float32), next_goal=goal2.to(torch.float32), reward=r_int)  # :316
        # the oracle steps the same actions
        o_obs, o_rew, o_done, o_coll, _, o_fobs, err = coracle.step(
            envs, a1.to(torch.int8).cpu().numpy(), None, autoreset=True, final_obs=True)
        assert err == 0
        np.testing.assert_array_equal(done.cpu().numpy(), o_done.astype(bool), err_msg=str(t))
        np.testing.assert_allclose(nobs.cpu().numpy(), o_obs.astype(np.float32), **OBS_TOL)
        np.testing.assert_allclose(rew.cpu().numpy(), o_rew.astype(np.float32), **OBS_TOL)
        for k, v in (("obs0", obs), ("obs", nobs), ("fobs", info["final_observation"]), ("a1", a1),
                     ("rew", rew), ("done", done), ("goal", goal), ("goal2", goal2), ("r_int", r_int)):
            rec[k].append(v.cpu().numpy().copy())
        # :320-322 and :283: the next goal, or a fresh choice after a goal was reached / an episode ended
        brk = done | (goal2 == goal_status(nobs))
        fresh, _ = eps_greedy(meta.forward(nobs), NUM_GOALS)
        goal = torch.where(brk, fresh, goal2)
        obs = nobs.clone()
    assert np.stack(rec["done"]).any() and np.stack(rec["r_int"]).any()
    cc.finish()
    mem = np.zeros((cap, 24), np.float32)
    c = 0
    for t in range(T):
        c = mo.replay_store(mem, c, rec["obs0"][t], rec["obs"][t][None], rec["a1"][t][None].astype(np.int8),
                            rec["rew"][t][None], rec["done"][t][None], rec["fobs"][t][None], None,
                            skip_ego_won=False, goal=rec["goal"][t][None], next_goal=rec["goal2"][t][None],
                            reward=rec["r_int"][t][None])
    assert ring.memory_counter == c == n * T
    np.testing.assert_array_equal(ring.memory.cpu().numpy(), mem)
    s, a, r, s2 = ring.sample(128, seed=1, draw=2)  # learn()'s slices, hdqn.py:196-199
    assert s.shape == (128, 11) and s2.shape == (128, 11) and a.shape == (128, 1) and r.shape == (128, 1)


_status = mo.goal_status64  # hdqn.py:223-237 on the oracle's fp64 observations (the kernel's ABI 17 form)


def _pick(u, k):  # floor(k u / 2^32)
    return ((u.astype(np.uint64) * np.uint64(k)) >> np.uint64(32)).astype(np.int64)


def _swap(o):
    """state[5:] + state[:5], the opponent's view (hdqn.py:285, :299)."""
    return np.concatenate([o[:, 5:], o[:, :5]], axis=1)


@pytest.mark.parametrize("n,opponent", [(2048, "none"), (1000, "none"), (2048, "self"), (1000, "self"),
                                        (2048, "other"), (1000, "other"), (1000, "self-selector"),
                                        (1000, "other-selector"), (1000, "self-signed"), (1000, "other-signed")])
def test_fused_hdqn_rollout(coracle, n, opponent):
    """mg_rollout_hdqn -- hdqn.py:280-323 in one launch -- against the loop restated on the CPU:
    every transition equals the C oracle's given the kernel's actions; every action, next goal and
    fresh goal is the epsilon-greedy choice its Philox draws make with the bf16-emulated nets'
    argmax (near-ties excused); the intrinsic reward is goal_status's; the goal ring the
    trajectory feeds equals the oracle's replay_store bit for bit. Starts mid-episode, so goals
    are reached and episodes end inside the launch; a second launch continues the goals.
    opponent "self" (Strategy_OP "selfplay", :262-264): the opponent's goal is the meta-net's
    epsilon-greedy choice on the swapped state at every outer-loop iteration (:285) and kept in
    between, its action the lower net's on [goal_op] + swapped state (:299-300). opponent
    "other" (any other Strategy_OP, :265-268): the same, with a second pair of nets standing in
    for the checkpoint load_path_op holds (the kernel reads them from global memory)."""
    import torch

    from merging_gym import MergeVecEnv, ReplayRing
    from merging_gym.policy import NUM_GOALS, QNet, greedy_threshold

    T, seed, dev = 24, 9, "cuda:0"
    rng = np.random.default_rng(21)
    mk = _net_signed if opponent.endswith("-signed") else _net
    meta_sd, lower_sd = mk(rng, 10, NUM_GOALS), mk(rng, 11, 5)
    if opponent == "self-selector":  # both players act through the one-feature net
        lower_sd = _selector_net()
    meta, lower = QNet.from_state_dict(meta_sd, device=dev), QNet.from_state_dict(lower_sd, device=dev)
    op_meta_sd, op_lower_sd = meta_sd, lower_sd  # self-play: upper_op = upper, lower_op = lower
    opp_arg = "self" if opponent.startswith("self") else opponent
    if opponent.startswith("other"):
        op_meta_sd = mk(rng, 10, NUM_GOALS)
        op_lower_sd = _selector_net() if opponent == "other-selector" else mk(rng, 11, 5)
        opp_arg = (QNet.from_state_dict(op_meta_sd, device=dev), QNet.from_state_dict(op_lower_sd, device=dev))
    thr = greedy_threshold()
    env = MergeVecEnv(n, device=dev, final_observation=True)
    k0 = 190
    for k in range(k0):
        env.step_random(5, opponent_random=False, step_idx=k)
    envs = mo.oracle_envs_from(coracle, env)
    stats = (env.returns.cpu().numpy().copy(), env.counts.cpu().numpy().astype(np.uint32))
    qe, qe_abs = env.q_eval.cpu().numpy().copy(), np.zeros(n)  # hdqn.py:330's q_eval per episode
    qe_pin = qe.copy()  # the same sums of the kernel-order Q-values (choice_check.order_matched_q)
    obs = env.observe().cpu().numpy().copy()
    obs64 = coracle.observe(envs)  # the fp64 state goal_status reads
    kind = _kind(opponent)
    cc_a = ChoiceCheck(f"fused h-DQN {opponent} n={n}: ego actions", max_frac=MAX_EXCUSED[kind])
    cc_g = ChoiceCheck(f"fused h-DQN {opponent} n={n}: goals", max_frac=MAX_EXCUSED["signed" if kind == "signed" else "uniform"])
    cc_o = ChoiceCheck(f"fused h-DQN {opponent} n={n}: opponent", max_frac=MAX_EXCUSED[kind])
    reset_goal = meta.reset_argmax()
    reset_obs = coracle.reset(coracle.new_envs(1)).astype(np.float32)
    q_reset = mo.qnet_reference(meta_sd, reset_obs, bf16=True)
    ChoiceCheck("reset goal").check([reset_goal], q_reset.argmax(1), [True], q_reset, q_exact=exact_q(meta_sd, reset_obs))
    fresh_off = -(1 << 63)  # counter (env ^ 2^63, step): the fresh-goal stream
    op_off = 1 << 62  # counter (env ^ 2^62, step): the self-play opponent's stream
    selfplay = opponent != "none"  # the opponent acts through h-DQN nets
    goal_prev = gop_prev = None
    rows = {k: [] for k in ("obs0", "obs", "fobs", "a1", "rew", "done", "goal", "goal2", "r_int")}
    ring = ReplayRing(4 * n * T, device=dev, goal=True)
    # the same rows appended by the launch itself (fused store); a capacity below one launch's
    # n T transitions so the ring wraps inside a launch (only the newest capacity rows land)
    cap_f = n * T // 3 + 7
    ring_f = ReplayRing(cap_f, device=dev, goal=True)
    # Goal_DQN's memory (hdqn.py:325) from the same launches: a 200-row plain ring (:22, :75)
    ring_m = ReplayRing(200, device=dev)
    mem_m = np.zeros((200, 22), np.float32)
    c_m = 0
    acc = np.zeros(n)  # extrinsic reward since each inner loop began (:286, :311-313), fp64
    for launch in range(2):
        obs_first = obs.copy()
        tr = env.rollout_hdqn(T, meta, lower, seed, opponent=opp_arg, first_step=k0, ring=ring_f, goal_memory=True)
        ring_m.store_meta(tr)
        ext_all = tr["ext_reward"].cpu().numpy().copy()
        nb_all = tr["no_break"].cpu().numpy().copy()
        g = {k: tr[k].cpu().numpy().copy() for k in ("goal", "next_goal", "reward") + (("goal_op",) if selfplay else ())}
        a1_all, done_all = tr["a1"].cpu().numpy().copy(), tr["done"].cpu().numpy().copy()
        a2_all = tr["a2"].cpu().numpy().copy()
        o_all, fo_all, rew_all = (tr[k].cpu().numpy().copy() for k in ("obs", "final_observation", "rew"))
        ring.store_rollout(torch.from_numpy(obs_first).to(dev), tr, skip_ego_won=False, goal=tr["goal"],
                           next_goal=tr["next_goal"], reward=tr["reward"])
        # the launch's first goals: carried over, or a fresh choice with step k0 - 1's draw
        fresh_words = lambda c: coracle.philox_batch(n, fresh_off, seed, c)  # noqa: E731
        if goal_prev is None:
            fx, fy, _ = mo.hdqn_fresh_draws(fresh_words, k0 - 1, opponent)
            qm = mo.qnet_reference(meta_sd, obs, bf16=True)
            exp = np.where(fx < thr, qm.argmax(1), _pick(fy, NUM_GOALS))
            cc_g.check(g["goal"][0], exp, fx < thr, qm, f"launch {launch} first goals", q_exact=exact_q(meta_sd, obs))
        else:
            assert (g["goal"][0] == goal_prev).all(), launch
        if selfplay:  # the opponent's first goal (:285): carried over, or fresh with step k0 - 1's draw
            if gop_prev is None:
                fc = coracle.philox_batch(n, op_off, seed, k0 - 1)
                qo = mo.qnet_reference(op_meta_sd, _swap(obs), bf16=True)
                gf0 = fc[:, 2] < thr
                cc_g.check(g["goal_op"][0], np.where(gf0, qo.argmax(1), _pick(fc[:, 3], NUM_GOALS)), gf0, qo,
                           f"launch {launch} opponent's first goals", q_exact=exact_q(op_meta_sd, _swap(obs)))
            else:
                assert (g["goal_op"][0] == gop_prev).all(), launch
        else:
            assert (a2_all == -1).all()
        for t in range(T):
            k = k0 + t
            ua = coracle.philox_batch(n, 0, seed, k)
            ubx, uby, _ = mo.hdqn_fresh_draws(fresh_words, k, opponent)
            goal_t = g["goal"][t].astype(np.int64)
            x = np.concatenate([goal_t[:, None].astype(np.float32), obs], axis=1)  # [goal] + state
            q1 = mo.qnet_reference(lower_sd, x, bf16=True)
            greedy = ua[:, 0] < thr
            exp_a = np.where(greedy, q1.argmax(1), _pick(ua[:, 1], 5))
            cc_a.check(a1_all[t], exp_a, greedy, q1, f"ego action, launch {launch} step {t}", q_exact=exact_q(lower_sd, x))
            a2 = None
            if selfplay:  # lower_op.choose_action([goal_op] + swapped state), :299-300
                uc = coracle.philox_batch(n, op_off, seed, k)
                xo = np.concatenate([g["goal_op"][t][:, None].astype(np.float32), _swap(obs)], axis=1)
                qa = mo.qnet_reference(op_lower_sd, xo, bf16=True)
                go = uc[:, 0] < thr
                exp_a2 = np.where(go, qa.argmax(1), _pick(uc[:, 1], 5))
                cc_o.check(a2_all[t], exp_a2, go, qa, f"opponent action, launch {launch} step {t}",
                           q_exact=exact_q(op_lower_sd, xo))
                a2 = a2_all[t].astype(np.int8)
            o_obs, o_rew, o_done, o_coll, _, o_fobs, err = coracle.step(envs, a1_all[t].astype(np.int8), a2,
                                                                        autoreset=True, final_obs=True, stats=stats)
            assert err == 0
            np.testing.assert_array_equal(done_all[t], o_done.astype(bool), err_msg=str(t))
            np.testing.assert_allclose(o_all[t], o_obs.astype(np.float32), **OBS_TOL)
            np.testing.assert_allclose(rew_all[t], o_rew.astype(np.float32), **OBS_TOL)
            d = done_all[t]
            np.testing.assert_allclose(fo_all[t][d], o_fobs[d].astype(np.float32), **OBS_TOL)
            s2 = np.where(d[:, None], fo_all[t], o_all[t])  # the next state, terminal where done
            s2_64 = np.where(d[:, None], o_fobs, o_obs)
            q2 = mo.qnet_reference(meta_sd, s2, bf16=True)
            gg = ua[:, 2] < thr
            exp_g2 = np.where(gg, q2.argmax(1), _pick(ua[:, 3], NUM_GOALS))
            g2 = g["next_goal"][t].astype(np.int64)
            q2x = exact_q(meta_sd, s2)
            cc_g.check(g2, exp_g2, gg, q2, f"next goal, launch {launch} step {t}", q_exact=q2x)
            # meta_eval_net(state)[goal] on the terminal state and the goal chosen on it (:330)
            qg = q2[np.arange(n), g2]
            qe += np.where(d, qg, 0.0)
            qe_abs += np.where(d, np.abs(q2).max(1), 0.0)
            if d.any():
                qe_pin += np.where(d, order_matched_q(meta, meta_sd, s2, "16x16")[np.arange(n), g2], 0.0)
            # :314 on the state acted on and :322 on the next state, in fp64 as the reference
            np.testing.assert_array_equal(g["reward"][t], (g2 == _status(obs64)).astype(np.float32))
            # the goal of the next step: kept, or fresh once reached / after an episode end
            brk = d | (g2 == _status(s2_64))
            # Goal_DQN's row inputs: extrinsic reward through step t, and the no-break bits
            acc += o_rew[:, 0]
            np.testing.assert_array_equal(ext_all[t], acc.astype(np.float32), err_msg=str((launch, t)))
            bits = np.unpackbits(nb_all[t].view(np.uint8), bitorder="little")[:n].astype(bool)
            np.testing.assert_array_equal(bits, ~brk, err_msg=str((launch, t)))
            c_m = mo.replay_store(mem_m, c_m, obs, o_all[t][None], a1_all[t][None].astype(np.int8),
                                  rew_all[t][None], d[None], fo_all[t][None], ~brk[None],
                                  reward=acc.astype(np.float32)[None], meta_goal=g["next_goal"][t][None])
            acc[brk] = 0.0
            gf = ubx < thr
            fresh = np.where(gf, np.where(d, reset_goal, q2.argmax(1)), _pick(uby, NUM_GOALS))
            exp_next = np.where(brk, fresh, g2)
            nxt = g["goal"][t + 1] if t + 1 < T else env.hdqn_goal.cpu().numpy().astype(np.int64)
            cc_g.check(nxt, exp_next, brk & gf & ~d, q2, f"fresh goal, launch {launch} step {t}", q_exact=q2x)
            if selfplay:  # the opponent's goal of the next step: fresh at a new outer iteration (:285)
                qo = mo.qnet_reference(op_meta_sd, _swap(o_all[t]), bf16=True)  # the state acted on next (reset obs after an end)
                go = uc[:, 2] < thr
                exp_op = np.where(brk, np.where(go, qo.argmax(1), _pick(uc[:, 3], NUM_GOALS)), g["goal_op"][t])
                nxo = g["goal_op"][t + 1] if t + 1 < T else env.hdqn_goal_op.cpu().numpy().astype(np.int64)
                cc_g.check(nxo, exp_op, brk & go, qo, f"opponent's fresh goal, launch {launch} step {t}",
                           q_exact=exact_q(op_meta_sd, _swap(o_all[t])))
            for key, v in (("obs0", obs), ("obs", o_all[t]), ("fobs", fo_all[t]), ("a1", a1_all[t]),
                           ("rew", rew_all[t]), ("done", d), ("goal", g["goal"][t]), ("goal2", g["next_goal"][t]),
                           ("r_int", g["reward"][t])):
                rows[key].append(v.copy())
            obs = o_all[t]
            obs64 = o_obs
        goal_prev = env.hdqn_goal.cpu().numpy().astype(np.int64)
        if selfplay:
            gop_prev = env.hdqn_goal_op.cpu().numpy().astype(np.int64)
            assert (np.stack(a2_all) >= 0).all() and (np.stack(a2_all) <= 4).all()
        k0 += T
    assert np.stack(rows["done"]).any() and (np.stack(rows["r_int"]) == 1).any()
    assert (np.stack(rows["goal"]) != np.stack(rows["goal2"])).any()
    mem = np.zeros((ring.capacity, 24), np.float32)
    c = 0
    for t in range(len(rows["obs"])):
        c = mo.replay_store(mem, c, rows["obs0"][t], rows["obs"][t][None], rows["a1"][t][None].astype(np.int8),
                            rows["rew"][t][None], rows["done"][t][None], rows["fobs"][t][None], None,
                            skip_ego_won=False, goal=rows["goal"][t][None], next_goal=rows["goal2"][t][None],
                            reward=rows["r_int"][t][None])
    assert ring.memory_counter == c == 2 * n * T
    np.testing.assert_array_equal(ring.memory.cpu().numpy(), mem)
    mem_f = np.zeros((cap_f, 24), np.float32)
    c = 0
    for t in range(len(rows["obs"])):
        c = mo.replay_store(mem_f, c, rows["obs0"][t], rows["obs"][t][None], rows["a1"][t][None].astype(np.int8),
                            rows["rew"][t][None], rows["done"][t][None], rows["fobs"][t][None], None,
                            skip_ego_won=False, goal=rows["goal"][t][None], next_goal=rows["goal2"][t][None],
                            reward=rows["r_int"][t][None])
    assert ring_f.memory_counter == c
    np.testing.assert_array_equal(ring_f.memory.cpu().numpy(), mem_f)
    assert ring_m.memory_counter == c_m > 200  # Goal_DQN's ring wrapped
    np.testing.assert_array_equal(ring_m.memory.cpu().numpy(), mem_m)
    np.testing.assert_array_equal(env.hdqn_ext.cpu().numpy(), acc)
    # the episode statistics the launch's finishing envs recorded (both scripts' logged values)
    np.testing.assert_array_equal(env.returns.cpu().numpy(), stats[0])
    np.testing.assert_array_equal(env.counts.cpu().numpy().astype(np.uint32), stats[1])
    check_q_eval(env.q_eval.cpu().numpy(), qe, qe_abs, f"fused h-DQN {opponent} n={n}", pinned=qe_pin, model=qe_pin)
    cc_a.finish()
    cc_g.finish()
    if selfplay:
        cc_o.finish()


def _philox_words(gidx, seed, step):
    """[len(gidx), 4] uint32 Philox words for arbitrary global env indices (NumPy restatement)."""
    import merge_numpy as mn

    g = np.asarray(gidx, dtype=np.uint64)
    z = np.zeros_like(g)
    m = np.uint64(0xFFFFFFFF)
    u = mn.philox4x32_10(g & m, g >> np.uint64(32), z + np.uint64(step & 0xFFFFFFFF), z + np.uint64(step >> 32), seed)
    return np.stack([w.astype(np.uint32) for w in u], axis=1)


@pytest.mark.parametrize("nets", ["uniform", "signed"])
def test_fused_hdqn_rollout_full_size(coracle, nets):
    """hdqn.py's acting loop at the BASELINE batch, 2^20 envs x 16 steps in one launch (the
    kernel's 512-env blocks and the [T, N] goal outputs at full size). Whole batch: actions and
    goals in range, intrinsic rewards 0/1, no NaN, the step bookkeeping. 2,048 sampled global env
    indices: every action, next goal and fresh goal is its draws' epsilon-greedy choice (bf16
    reference argmax, near-ties excused), every transition equals the C oracle's and the state
    ends bit for bit equal. Reference: scripts/hdqn.py:280-323."""
    import torch

    from merging_gym import MergeVecEnv
    from merging_gym.policy import NUM_GOALS, QNet, greedy_threshold

    n, T, seed, k0, burn, dev = 1 << 20, 16, 17, 900, 240, "cuda:0"
    rng = np.random.default_rng(5)
    mk = _net_signed if nets == "signed" else _net  # signed: choices that vary per env
    meta_sd, lower_sd = mk(rng, 10, NUM_GOALS), mk(rng, 11, 5)
    meta, lower = QNet.from_state_dict(meta_sd, device=dev), QNet.from_state_dict(lower_sd, device=dev)
    env = MergeVecEnv(n, device=dev)
    for k in range(burn):
        env.step_random(seed + 1, step_idx=k)
    idx_np = np.sort(np.random.default_rng(3).choice(n, 2048, replace=False))
    idx = torch.from_numpy(idx_np).to(dev)
    envs = mo.oracle_envs_from(coracle, env, idx)
    stats = (env.returns[idx].cpu().numpy().copy(), env.counts[idx].cpu().numpy().astype(np.uint32))
    qe, qe_abs = env.q_eval[idx].cpu().numpy().copy(), np.zeros(len(idx_np))
    qe_pin = qe.copy()
    obs = env.observe()[idx].cpu().numpy().copy()
    obs64 = coracle.observe(envs)
    reset_goal = meta.reset_argmax()
    cc_a = ChoiceCheck(f"full-size h-DQN ({nets}): ego actions", max_frac=MAX_EXCUSED[nets])
    cc_g = ChoiceCheck(f"full-size h-DQN ({nets}): goals", max_frac=MAX_EXCUSED[nets])

    tr = env.rollout_hdqn(T, meta, lower, seed, first_step=k0)
    assert int(tr["a1"].min()) >= 0 and int(tr["a1"].max()) <= 4 and bool((tr["a2"] == -1).all())
    for key in ("goal", "next_goal"):
        assert float(tr[key].min()) >= 0 and float(tr[key].max()) <= NUM_GOALS - 1
    assert set(torch.unique(tr["reward"]).tolist()) <= {0.0, 1.0}
    assert not bool(torch.isnan(tr["obs"]).any()) and not bool(torch.isnan(tr["rew"]).any())
    assert bool((env.counts[:, 3].to(torch.int64) + env.steps.to(torch.int64) == burn + T).all())
    assert int(tr["done"].sum()) > 1000
    sub = {k: tr[k][:, idx].cpu().numpy() for k in ("a1", "done", "obs", "rew", "final_observation", "goal",
                                                       "next_goal", "reward")}
    thr = greedy_threshold()
    fresh_words = lambda c: _philox_words(idx_np.astype(np.uint64) ^ np.uint64(1 << 63), seed, c)  # noqa: E731
    fx, fy, _ = mo.hdqn_fresh_draws(fresh_words, k0 - 1, "none")
    qm = mo.qnet_reference(meta_sd, obs, bf16=True)
    exp0 = np.where(fx < thr, qm.argmax(1), _pick(fy, NUM_GOALS))
    cc_g.check(sub["goal"][0], exp0, fx < thr, qm, "first goals", q_exact=exact_q(meta_sd, obs))
    for t in range(T):
        ua = _philox_words(idx_np, seed, k0 + t)
        ubx, uby, _ = mo.hdqn_fresh_draws(fresh_words, k0 + t, "none")
        goal_t = sub["goal"][t].astype(np.int64)
        x1 = np.concatenate([goal_t[:, None].astype(np.float32), obs], axis=1)
        q1 = mo.qnet_reference(lower_sd, x1, bf16=True)
        greedy = ua[:, 0] < thr
        exp_a = np.where(greedy, q1.argmax(1), _pick(ua[:, 1], 5))
        cc_a.check(sub["a1"][t], exp_a, greedy, q1, f"step {t}", q_exact=exact_q(lower_sd, x1))
        o_obs, o_rew, o_done, o_coll, _, o_fobs, err = coracle.step(envs, sub["a1"][t].astype(np.int8), None,
                                                                    autoreset=True, final_obs=True, stats=stats)
        assert err == 0
        d = o_done.astype(bool)
        np.testing.assert_array_equal(sub["done"][t], d, err_msg=str(t))
        np.testing.assert_allclose(sub["obs"][t], o_obs.astype(np.float32), **OBS_TOL)
        np.testing.assert_allclose(sub["rew"][t], o_rew.astype(np.float32), **OBS_TOL)
        np.testing.assert_allclose(sub["final_observation"][t][d], o_fobs[d].astype(np.float32), **OBS_TOL)
        s2 = np.where(d[:, None], sub["final_observation"][t], sub["obs"][t])
        s2_64 = np.where(d[:, None], o_fobs, o_obs)
        q2 = mo.qnet_reference(meta_sd, s2, bf16=True)
        gg = ua[:, 2] < thr
        g2 = sub["next_goal"][t].astype(np.int64)
        q2x = exact_q(meta_sd, s2)
        cc_g.check(g2, np.where(gg, q2.argmax(1), _pick(ua[:, 3], NUM_GOALS)), gg, q2, f"next goal, step {t}",
                   q_exact=q2x)
        qg = q2[np.arange(len(idx_np)), g2]  # hdqn.py:330
        qe += np.where(d, qg, 0.0)
        qe_abs += np.where(d, np.abs(q2).max(1), 0.0)
        if d.any():
            qe_pin += np.where(d, order_matched_q(meta, meta_sd, s2, "16x16")[np.arange(len(idx_np)), g2], 0.0)
        np.testing.assert_array_equal(sub["reward"][t], (g2 == _status(obs64)).astype(np.float32))
        brk = d | (g2 == _status(s2_64))
        gf = ubx < thr
        exp_next = np.where(brk, np.where(gf, np.where(d, reset_goal, q2.argmax(1)), _pick(uby, NUM_GOALS)), g2)
        nxt = sub["goal"][t + 1] if t + 1 < T else env.hdqn_goal[idx].cpu().numpy()
        cc_g.check(nxt, exp_next, brk & gf & ~d, q2, f"fresh goal, step {t}", q_exact=q2x)
        obs = sub["obs"][t]
        obs64 = o_obs
    for name, src in (("pos1", env.p1), ("vel1", env.v1), ("pos2", env.p2), ("vel2", env.v2),
                      ("r1_acc", env.ret1), ("r2_acc", env.ret2)):
        np.testing.assert_array_equal(src[idx].cpu().numpy(), envs[name], err_msg=name)
    np.testing.assert_array_equal(env.returns[idx].cpu().numpy(), stats[0])
    np.testing.assert_array_equal(env.counts[idx].cpu().numpy().astype(np.uint32), stats[1])
    check_q_eval(env.q_eval[idx].cpu().numpy(), qe, qe_abs, f"full-size h-DQN ({nets})", pinned=qe_pin,
                 model=qe_pin)
    # main.py's pending value where the ego has arrived first: what the next launch reads back
    # (the no-wait statistics load it only for those envs, pend_load)
    w1 = envs["winner"] == 1
    np.testing.assert_array_equal(env._ep_stats[idx][:, 3].cpu().numpy()[w1], envs["ep_reward_main"][w1])
    cc_a.finish()
    cc_g.finish()


@pytest.mark.parametrize("opponent", ["none", "self", "other"])
def test_hdqn_checkpoint_resume_is_bit_exact(opponent):
    """A checkpoint taken between two h-DQN launches (MergeVecEnv.state_dict: the batch state, the
    step index keying the draws, the ego's goals and the self-play opponent's goals) resumes the
    acting loop bit for bit: the next launch from the restored env equals the uninterrupted one
    in every output, goal and state array."""
    import io

    import torch

    from merging_gym import MergeVecEnv
    from merging_gym.policy import NUM_GOALS, QNet

    n, T, seed, dev = 1500, 12, 4, "cuda:0"
    rng = np.random.default_rng(8)
    meta = QNet.from_state_dict(_net(rng, 10, NUM_GOALS), device=dev)
    lower = QNet.from_state_dict(_net(rng, 11, 5), device=dev)
    if opponent == "other":  # another h-DQN checkpoint's nets (hdqn.py:265-268)
        opponent = (QNet.from_state_dict(_net(rng, 10, NUM_GOALS), device=dev),
                    QNet.from_state_dict(_net(rng, 11, 5), device=dev))
    env = MergeVecEnv(n, device=dev, final_observation=True)
    for k in range(180):
        env.step_random(seed, opponent_random=False, step_idx=k)
    env.rollout_hdqn(T, meta, lower, seed, opponent=opponent, first_step=180)
    buf = io.BytesIO()
    torch.save(env.state_dict(), buf)
    tr_a = {k: v.clone() for k, v in env.rollout_hdqn(T, meta, lower, seed, opponent=opponent).items()
            if v is not None}
    end = env.state_dict()
    buf.seek(0)
    env2 = MergeVecEnv(n, device=dev, final_observation=True)
    env2.load_state_dict(torch.load(buf, weights_only=True))
    tr_b = env2.rollout_hdqn(T, meta, lower, seed, opponent=opponent)
    assert set(tr_a) <= set(k for k, v in tr_b.items() if v is not None)
    done = tr_a["done"]
    assert bool(done.any())
    for k, v in tr_a.items():
        if k == "final_observation":  # written on the rows that ended only (the rest is scratch)
            v, w = v[done], tr_b[k][done]
        else:
            w = tr_b[k]
        same = torch.equal(v, w)
        assert same, k
    for k, v in env2.state_dict().items():
        assert (torch.equal(v, end[k]) if isinstance(v, torch.Tensor) else v == end[k]), k
    assert ("hdqn_goal_op" in end) == (opponent != "none")


def test_other_checkpoint_opponent_with_own_nets_equals_selfplay():
    """An opponent checkpoint holding the ego's own nets (hdqn.py:265-268 with load_path_op =
    load_path) is self-play (:262-264): opponent mode 3, which reads the opponent's nets from
    global memory, must give mode 2's outputs bit for bit."""
    import torch

    from merging_gym import MergeVecEnv
    from merging_gym.policy import NUM_GOALS, QNet

    n, T, seed, dev = 1000, 16, 6, "cuda:0"
    rng = np.random.default_rng(5)
    meta = QNet.from_state_dict(_net(rng, 10, NUM_GOALS), device=dev)
    lower = QNet.from_state_dict(_net(rng, 11, 5), device=dev)
    outs = []
    for opp in ("self", (meta, lower)):
        env = MergeVecEnv(n, device=dev, final_observation=True)
        for k in range(190):
            env.step_random(seed, opponent_random=False, step_idx=k)
        tr = env.rollout_hdqn(T, meta, lower, seed, opponent=opp, first_step=190)
        outs.append({k: v.clone() for k, v in tr.items() if v is not None and k != "final_observation"})
    a, b = outs
    assert set(a) == set(b)
    for k in a:
        same = torch.equal(a[k], b[k])
        if not same and k == "a2":
            raise AssertionError(f"a2: {int((a[k] != b[k]).sum())} differ; self {a[k][0, :12].tolist()}, "
                                 f"other {b[k][0, :12].tolist()}")
        assert same, k
