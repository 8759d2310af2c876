"""GPU parity for the fused DQN policy (BASELINE config 5): the reference's Net and
epsilon-greedy choose_action (scripts/main.py:30-47, :99-112) in bf16 on the matrix cores.

Bar: Q-values equal the bf16-emulated CPU forward (oracle.qnet_reference: bf16 operands,
fp32 sums) to summation-order rounding; greedy actions equal its argmax except at near-ties;
exploration draws and random actions bit-exact (Philox); every env transition equal to the
CPU oracle stepping with the kernel's actions. Weights: two of the reference's shipped
checkpoints (tests/golden/dqn_checkpoints.npz, from test_params/dqn/*/eval.pth).
"""

import os

import numpy as np
import pytest

import merge_oracle as mo
from choice_check import ChoiceCheck, check_q_eval, exact_q, order_matched_q
from conftest import ROOT

pytestmark = pytest.mark.gpu

OBS_TOL = dict(rtol=1e-6, atol=1e-5)


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


@pytest.fixture(scope="module")
def nets():
    f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    out = {}
    for key in ("l1", "l3"):
        out[key] = {name.split("/", 1)[1]: f[name] for name in f.files if name.startswith(key + "/")}
    return out


def _obs_samples(coracle, n=8192, steps=240, seed=3):
    envs = coracle.new_envs(n)
    coracle.reset(envs)
    rng = np.random.default_rng(seed)
    out = []
    for k in range(steps):
        o, *_ = coracle.step(envs, rng.integers(0, 5, n).astype(np.int8), rng.integers(0, 5, n).astype(np.int8),
                             autoreset=True)
        if k % 30 == 0:
            out.append(o.astype(np.float32))
    return np.concatenate(out)


# excused greedy choices (tests/choice_check.py): bounds per net
MAX_EXCUSED = {"l1": 1e-4, "l3": 1e-4}  # round 3 measured 0 excused of > 10^6 greedy choices


@pytest.mark.parametrize("key", ["l1", "l3"])
@pytest.mark.parametrize("swap", [False, True])
def test_qnet_forward_matches_bf16_reference(torch, coracle, nets, key, swap):
    from merging_gym.policy import QNet

    obs = _obs_samples(coracle)
    qnet = QNet.from_state_dict(nets[key], device="cuda:0")
    q = qnet.forward(torch.from_numpy(obs).cuda(), swap_halves=swap).cpu().numpy()
    q_bf = mo.qnet_reference(nets[key], obs, bf16=True, swap=swap)
    q_32 = mo.qnet_reference(nets[key], obs, bf16=False, swap=swap)
    scale = np.maximum(1.0, np.abs(q_bf).max(axis=1, keepdims=True))
    err = np.abs(q - q_bf) / scale
    assert np.median(err) < 1e-5 and err.max() < 1e-2, (np.median(err), err.max())
    cc = ChoiceCheck(f"forward {key} swap={swap}", max_frac=MAX_EXCUSED[key])
    cc.check(q.argmax(1), q_bf.argmax(1), np.ones(len(q), bool), q_bf)
    cc.finish()
    # bf16 vs the reference's fp32 Net: the kernel loses nothing beyond bf16 itself
    agree = (q.argmax(1) == q_32.argmax(1)).mean()
    agree_bf16 = (q_bf.argmax(1) == q_32.argmax(1)).mean()
    assert agree >= agree_bf16 - 1e-3, (agree, agree_bf16)
    if key == "l1":  # the checkpoint the bench and human_player.py:68 use
        assert agree >= 0.999, agree


@pytest.mark.parametrize("key", ["l1", "l3", "meta-signed", "lower-signed"])
@pytest.mark.parametrize("swap", [False, True])
def test_qnet_forward_matches_the_mfma_model(torch, coracle, nets, key, swap):
    """oracle.qnet_reference_mfma -- bf16 operands in the packed k order, each group of 8 products added
    by the matrix cores' measured rule (oracle/merge_oracle.c oracle_mfma_layer: truncation onto
    2^(nom - 24), a floor onto 2^(E - 31), round to nearest even) -- against mg_qnet_forward: EVERY
    Q-value bit for bit, for the shipped checkpoints (both views) and for seeded signed h-DQN nets
    (hdqn.py's meta-net 10 -> 3 and lower net 11 -> 5 with torch.nn.Linear's default init), where
    round 5's exact-sum model left 0.8-1.4 % of rows unexplained (profiles/r06/mfma_order.txt)."""
    from merging_gym.policy import QNet

    obs = _obs_samples(coracle, n=4096)
    if key in ("l1", "l3"):
        sd, x = nets[key], obs
    else:
        if swap:
            pytest.skip("the swapped view is the 10-input config-5 nets'")
        rng = np.random.default_rng(0 if key.startswith("meta") else 1)
        i, o = (10, 3) if key.startswith("meta") else (11, 5)
        sd = {}
        for name, (a, b) in zip(("fc1", "fc2", "out"), [(200, i), (100, 200), (o, 100)]):
            sd[f"{name}.weight"] = rng.uniform(-b ** -0.5, b ** -0.5, (a, b)).astype(np.float32)
            sd[f"{name}.bias"] = rng.uniform(-b ** -0.5, b ** -0.5, a).astype(np.float32)
        x = obs if i == 10 else np.concatenate([rng.integers(0, 3, (len(obs), 1)).astype(np.float32), obs], 1)
    q = QNet.from_state_dict(sd, device="cuda:0").forward(torch.from_numpy(x).cuda(), swap_halves=swap)
    ref = mo.qnet_reference_mfma(sd, x, swap=swap)
    same = q.cpu().numpy().view(np.uint32) == ref.view(np.uint32)
    assert same.all(), (key, swap, int((~same.all(1)).sum()), "rows differ")


@pytest.mark.parametrize("in_dim,out_dim", [(11, 5), (10, 3)])
def test_qnet_forward_hdqn_nets(torch, coracle, in_dim, out_dim):
    """hdqn.py's two nets: the lower-level Net(NUM_STATES + 1, NUM_ACTIONS) on goal states
    [goal] + state (:145, :291) and Goal_DQN's meta-net Net(NUM_STATES, NUM_GOALS) (:63), with
    hdqn.py:41-47's initialisation (every weight U(0, 1); torch's default bias init). No h-DQN
    checkpoint ships with the reference, so the weights are seeded draws."""
    from merging_gym.policy import QNet

    rng = np.random.default_rng(in_dim * 10 + out_dim)
    dims = [(200, in_dim), (100, 200), (out_dim, 100)]
    sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), dims):
        sd[f"{name}.weight"] = rng.uniform(0, 1, (o, i)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    obs = _obs_samples(coracle, n=2048, steps=120)
    x = obs if in_dim == 10 else np.concatenate(
        [rng.integers(0, 3, (len(obs), 1)).astype(np.float32), obs], axis=1)  # [goal] + state
    qnet = QNet.from_state_dict(sd, device="cuda:0")
    q = qnet.forward(torch.from_numpy(x).cuda()).cpu().numpy()
    assert q.shape == (len(x), out_dim)
    q_bf = mo.qnet_reference(sd, x, bf16=True)
    scale = np.maximum(1.0, np.abs(q_bf).max(axis=1, keepdims=True))
    err = np.abs(q - q_bf) / scale
    assert np.median(err) < 1e-5 and err.max() < 1e-2, (np.median(err), err.max())
    cc = ChoiceCheck(f"forward hdqn.py net {in_dim}->{out_dim}", max_frac=1e-4)
    cc.check(q.argmax(1), q_bf.argmax(1), np.ones(len(q), bool), q_bf)
    cc.finish()
    with pytest.raises(ValueError):  # the input width is the net's
        qnet.forward(torch.zeros((4, in_dim + 1), device="cuda:0"))


@pytest.mark.parametrize("opponent,n,sync", [("none", 4096, False), ("uniform", 4096, False), ("self", 4096, False),
                                             ("none", 1000, False), ("uniform", 1001, False), ("self", 577, False),
                                             ("other", 4096, False), ("other", 577, False), ("other", 4096, True),
                                             ("self", 4096, True)])
def test_rollout_qnet_policy_and_transitions(torch, coracle, nets, opponent, n, sync):
    """Every action is the epsilon-greedy choice (Philox draws exact, greedy = argmax of the
    bf16 reference except near-ties) and every transition equals the CPU oracle's. The odd
    sizes leave partial waves / a partial block and unaligned trajectory rows. "other" is
    main.py's default Strategy_OP "L1" (:161-168): the opponent is another shipped checkpoint
    (l3) acting on the swapped observation, the kernel instance with both nets in LDS.
    sync: every env's clock three steps short of the timeout, so that whole waves' items are
    may-finish ones at once -- the round-5 lists' extremes: an ego wave whose every item writes its
    Q-values into the tile rows, and opponent lists whose may-finish items reach the tail that the
    env waves run (they then publish the rows-read flag the ego waves wait for)."""
    from merging_gym import MergeVecEnv
    from merging_gym.policy import QNet, greedy_threshold

    T, seed, k0 = 24, 17, 500 + n % 2  # odd sizes start on an odd step (the second word pair of a call)
    qnet = QNet.from_state_dict(nets["l1"], device="cuda:0")
    env = MergeVecEnv(n, device="cuda:0")
    for k in range(200):  # mid-episode start: episodes end inside the window (autoreset, q_eval)
        env.step_random(seed + 1, step_idx=k)
    if sync:  # the clock's bits of the packed time / flags word (MG_TF_*)
        m = env._nat.TF_STEPS_MASK
        env.tf.copy_((env.tf & ~m) | 2498)
        assert bool((env.steps == 2498).all())
    envs = coracle.new_envs(n)
    for name, src in (("pos1", env.p1), ("vel1", env.v1), ("pos2", env.p2), ("vel2", env.v2),
                      ("r1_acc", env.ret1), ("r2_acc", env.ret2)):
        envs[name] = src.cpu().numpy()
    envs["steps"] = env.steps.cpu().numpy()
    envs["winner"] = env.winner.cpu().numpy()
    envs["time_stamp"] = np.cumsum(np.full(2700, 0.2))[np.maximum(envs["steps"] - 1, 0)] * (envs["steps"] > 0)
    obs_in = env.observe().cpu().numpy().copy()
    opp_key = "l3" if opponent == "other" else "l1"
    opp = QNet.from_state_dict(nets["l3"], device="cuda:0") if opponent == "other" else opponent
    qe = env.q_eval.cpu().numpy().copy()  # main.py:221's q_eval, per finished episode
    qe_abs = np.zeros(n)
    qe_pin = qe.copy()  # the same sums of the kernel-order Q-values (choice_check.order_matched_q)
    qe_model = qe.copy()  # ... and of the oracle's CPU model of that order
    form = "16x16" if opponent in ("self", "other") else "32x32"
    traj = env.rollout_qnet(T, qnet, seed, opponent=opp, first_step=k0)
    traj = {k: (v.cpu().numpy() if v is not None else None) for k, v in traj.items()}
    thr = greedy_threshold(0.7)
    cc1 = ChoiceCheck(f"rollout ego l1 ({opponent}, n={n})", max_frac=MAX_EXCUSED["l1"])
    cc2 = ChoiceCheck(f"rollout opponent {opp_key} ({opponent}, n={n})", max_frac=MAX_EXCUSED[opp_key])
    mode = "self" if opponent == "other" else opponent  # the draw layout of a net opponent
    for t in range(T):
        ex, rnd1, ex2, rnd2 = mo.qnet_policy_draws(lambda c: coracle.philox_batch(n, 0, seed, c), k0 + t, mode)
        q = mo.qnet_reference(nets["l1"], obs_in, bf16=True)
        greedy = ex < thr
        exp1 = np.where(greedy, q.argmax(1), rnd1)
        cc1.check(traj["a1"][t], exp1, greedy, q, f"step {t}", q_exact=exact_q(nets["l1"], obs_in, form=form))
        if opponent == "none":
            assert (traj["a2"][t] == -1).all()
        elif opponent == "uniform":
            assert (traj["a2"][t] == rnd2).all()
        else:
            q2 = mo.qnet_reference(nets[opp_key], obs_in, bf16=True, swap=True)
            g2 = ex2 < thr
            cc2.check(traj["a2"][t], np.where(g2, q2.argmax(1), rnd2), g2, q2, f"step {t}",
                      q_exact=exact_q(nets[opp_key], obs_in, swap=True))
        # the transition, with the actions the kernel took
        o_obs, o_rew, o_done, o_coll, _, o_fobs, err = coracle.step(
            envs, traj["a1"][t], traj["a2"][t], autoreset=True, final_obs=True)
        assert err == 0
        np.testing.assert_array_equal(traj["done"][t], o_done.astype(bool), err_msg=str(t))
        np.testing.assert_array_equal(traj["collision"][t], o_coll.astype(bool), err_msg=str(t))
        np.testing.assert_allclose(traj["obs"][t], o_obs.astype(np.float32), **OBS_TOL)
        np.testing.assert_allclose(traj["rew"][t], o_rew.astype(np.float32), **OBS_TOL)
        d = o_done.astype(bool)
        np.testing.assert_allclose(traj["final_observation"][t][d], o_fobs[d].astype(np.float32), **OBS_TOL)
        # eval_net(state)[action] on the input and action of an episode's last step (main.py:221)
        qa = q[np.arange(n), traj["a1"][t].astype(np.int64)]
        qe += np.where(d, qa, 0.0)
        qe_abs += np.where(d, np.abs(q).max(1), 0.0)
        if d.any():
            qp = order_matched_q(qnet, nets["l1"], obs_in, form)
            qe_pin += np.where(d, qp[np.arange(n), traj["a1"][t].astype(np.int64)], 0.0)
            qm = mo.qnet_reference_mfma(nets["l1"], obs_in, form=form).astype(np.float64)
            qe_model += np.where(d, qm[np.arange(n), traj["a1"][t].astype(np.int64)], 0.0)
        obs_in = traj["obs"][t]
    np.testing.assert_array_equal(env.p1.cpu().numpy(), envs["pos1"])
    np.testing.assert_array_equal(env.ret2.cpu().numpy(), envs["r2_acc"])
    check_q_eval(env.q_eval.cpu().numpy(), qe, qe_abs, f"rollout ego l1 ({opponent}, n={n})", pinned=qe_pin,
                 model=qe_model)
    assert env._step_idx == k0 + T
    cc1.finish()
    if opponent in ("self", "other"):
        cc2.finish()


@pytest.mark.parametrize("opponent", ["none", "self", "other"])
def test_rollout_qnet_invalid_greedy_actions(torch, coracle, nets, opponent):
    """A net with 8 outputs (out_dim <= 8 is allowed) picks actions 5-7, which the reference's
    action_dict rejects with a KeyError after the clock (and the ego, for a bad action2) has
    advanced. The fused kernel steps such an env exactly that far and emits zeros (obs, rewards,
    flags), like the oracle's error path; every transition is compared with the oracle stepping
    the kernel's actions, invalid ones included."""
    from merging_gym import MergeVecEnv
    from merging_gym.policy import QNet

    def widened(key):
        sd = dict(nets[key])
        w3, b3 = sd["out.weight"], sd["out.bias"]
        # output 5 = action 2's row with a slightly larger bias: it wins wherever action 2 would
        # (most greedy choices of this checkpoint); outputs 6-7 never win
        sd["out.weight"] = np.concatenate([w3, w3[[2, 0, 1]]])
        sd["out.bias"] = np.concatenate([b3, [b3[2] + 0.01, b3[0] - 100.0, b3[1] - 100.0]]).astype(np.float32)
        return QNet.from_state_dict(sd, device="cuda:0")

    qnet = widened("l1")
    assert qnet.out_dim == 8
    if opponent == "other":  # the net-split kernel (round 5) with the other checkpoint widened alike
        opponent = widened("l3")
    n, T, seed, k0 = 1000, 16, 23, 300
    env = MergeVecEnv(n, device="cuda:0")
    for k in range(40):
        env.step_random(seed + 1, step_idx=k)
    envs = coracle.new_envs(n)
    for name, src in (("pos1", env.p1), ("vel1", env.v1), ("pos2", env.p2), ("vel2", env.v2),
                      ("r1_acc", env.ret1), ("r2_acc", env.ret2)):
        envs[name] = src.cpu().numpy()
    envs["steps"] = env.steps.cpu().numpy()
    envs["winner"] = env.winner.cpu().numpy()
    envs["time_stamp"] = np.cumsum(np.full(2700, 0.2))[np.maximum(envs["steps"] - 1, 0)] * (envs["steps"] > 0)
    traj = env.rollout_qnet(T, qnet, seed, opponent=opponent, first_step=k0)
    traj = {k: (v.cpu().numpy() if v is not None else None) for k, v in traj.items()}
    assert (traj["a1"] >= 5).sum() > 100
    if opponent == "self":
        assert (traj["a2"] >= 5).sum() > 100
    for t in range(T):
        o_obs, o_rew, o_done, o_coll, _, o_fobs, err = coracle.step(
            envs, traj["a1"][t], traj["a2"][t], autoreset=True, final_obs=True)
        assert err != 0
        np.testing.assert_array_equal(traj["done"][t], o_done.astype(bool), err_msg=str(t))
        np.testing.assert_array_equal(traj["collision"][t], o_coll.astype(bool), err_msg=str(t))
        np.testing.assert_allclose(traj["obs"][t], o_obs.astype(np.float32), **OBS_TOL)
        np.testing.assert_allclose(traj["rew"][t], o_rew.astype(np.float32), **OBS_TOL)
        d = o_done.astype(bool)
        np.testing.assert_allclose(traj["final_observation"][t][d], o_fobs[d].astype(np.float32), **OBS_TOL)
    for name, src in (("pos1", env.p1), ("vel1", env.v1), ("pos2", env.p2), ("vel2", env.v2),
                      ("r1_acc", env.ret1), ("r2_acc", env.ret2)):
        np.testing.assert_array_equal(src.cpu().numpy(), envs[name], err_msg=name)
    np.testing.assert_array_equal(env.steps.cpu().numpy(), np.minimum(envs["steps"], 0x1FFF))
    np.testing.assert_array_equal(env.winner.cpu().numpy(), envs["winner"])


def test_greedy_threshold_is_phi_of_episilo():
    from merging_gym.policy import greedy_threshold

    assert greedy_threshold(0.7) == round(0.7580363477769270 * 2**32)
    assert greedy_threshold(50.0) == 2**32 and greedy_threshold(-50.0) == 0


@pytest.mark.parametrize("opponent", ["none", "self", "other"])
def test_rollout_qnet_full_size(torch, coracle, nets, opponent):
    """BASELINE config 5 at its own size: 2^20 envs x 16 steps in one launch (the kernel's
    1,024-env blocks, both pipelined groups and the [T, N, .] trajectory indexing at full size).
    Whole batch: actions in range, flags 0/1, no NaN, the step bookkeeping. 2,048 sampled global
    env indices: every action is the epsilon-greedy choice (Philox draws exact, greedy = argmax
    of the bf16 reference except near-ties) and every transition equals the C oracle's,
    state bit for bit. Reference: scripts/main.py:99-112 (choose_action), :189-220 (the loop)."""
    from merging_gym import MergeVecEnv
    from merging_gym.policy import QNet, greedy_threshold

    n, T, seed, k0, burn = 1 << 20, 16, 41, 900, 240
    qnet = QNet.from_state_dict(nets["l1"], device="cuda:0")
    env = MergeVecEnv(n, device="cuda:0")
    for k in range(burn):  # mid-episode start, some envs already finished once
        env.step_random(seed + 1, step_idx=k)
    idx_np = np.sort(np.random.default_rng(3).choice(n, 2048, replace=False))
    idx = torch.from_numpy(idx_np).cuda()
    envs = mo.oracle_envs_from(coracle, env, idx)  # main.py's running ep_reward from the device's pending value
    obs_in = env.observe()[idx].cpu().numpy().copy()
    ret_sum0, counts0 = env.returns[idx].cpu().numpy(), env.counts[idx].cpu().numpy().astype(np.uint32)
    qe, qe_abs = env.q_eval[idx].cpu().numpy().copy(), np.zeros(len(idx_np))
    qe_pin = qe.copy()
    form = "16x16" if opponent in ("self", "other") else "32x32"

    opp_key = "l3" if opponent == "other" else "l1"
    opp = QNet.from_state_dict(nets["l3"], device="cuda:0") if opponent == "other" else opponent
    traj = env.rollout_qnet(T, qnet, seed, opponent=opp, first_step=k0)
    # whole batch
    a1, a2 = traj["a1"], traj["a2"]
    assert int(a1.min()) >= 0 and int(a1.max()) <= 4
    if opponent == "none":
        assert bool((a2 == -1).all())
    else:
        assert int(a2.min()) >= 0 and int(a2.max()) <= 4
    assert int(traj["flags"][..., 2:].max()) <= 1
    assert not bool(torch.isnan(traj["obs"]).any()) and not bool(torch.isnan(traj["rew"]).any())
    counts = env.counts.to(torch.int64)
    assert bool((counts[:, 3] + env.steps.to(torch.int64) == burn + T).all())
    assert int(traj["done"].sum()) > 1000  # episodes ended inside the window (autoreset path ran)
    # sampled envs, step by step against the bf16 reference policy and the C oracle
    sub = {k: (v[:, idx].cpu().numpy() if v is not None and v.dim() >= 2 and v.shape[1] == n else None)
           for k, v in traj.items()}
    thr = greedy_threshold(0.7)
    stats = (ret_sum0.copy(), counts0.copy())
    cc1 = ChoiceCheck(f"full-size ego l1 ({opponent})", max_frac=MAX_EXCUSED["l1"])
    cc2 = ChoiceCheck(f"full-size opponent {opp_key} ({opponent})", max_frac=MAX_EXCUSED[opp_key])
    words = lambda c: np.stack([coracle.philox_batch(1, int(gi), seed, c)[0] for gi in idx_np])  # noqa: E731
    mode = "none" if opponent == "none" else "self"
    for t in range(T):
        ex, rnd1, ex2, rnd2 = mo.qnet_policy_draws(words, k0 + t, mode)
        q = mo.qnet_reference(nets["l1"], obs_in, bf16=True)
        greedy = ex < thr
        exp1 = np.where(greedy, q.argmax(1), rnd1)
        cc1.check(sub["a1"][t], exp1, greedy, q, f"step {t}", q_exact=exact_q(nets["l1"], obs_in, form=form))
        if opponent in ("self", "other"):
            q2 = mo.qnet_reference(nets[opp_key], obs_in, bf16=True, swap=True)
            g2 = ex2 < thr
            cc2.check(sub["a2"][t], np.where(g2, q2.argmax(1), rnd2), g2, q2, f"step {t}",
                      q_exact=exact_q(nets[opp_key], obs_in, swap=True))
        o_obs, o_rew, o_done, o_coll, _, o_fobs, err = coracle.step(
            envs, sub["a1"][t], sub["a2"][t], autoreset=True, final_obs=True, stats=stats)
        assert err == 0
        np.testing.assert_array_equal(sub["done"][t], o_done.astype(bool), err_msg=str(t))
        np.testing.assert_array_equal(sub["collision"][t], o_coll.astype(bool), err_msg=str(t))
        np.testing.assert_allclose(sub["obs"][t], o_obs.astype(np.float32), **OBS_TOL)
        np.testing.assert_allclose(sub["rew"][t], o_rew.astype(np.float32), **OBS_TOL)
        d = o_done.astype(bool)
        np.testing.assert_allclose(sub["final_observation"][t][d], o_fobs[d].astype(np.float32), **OBS_TOL)
        qa = q[np.arange(len(idx_np)), sub["a1"][t].astype(np.int64)]  # main.py:221
        qe += np.where(d, qa, 0.0)
        qe_abs += np.where(d, np.abs(q).max(1), 0.0)
        if d.any():
            qp = order_matched_q(qnet, nets["l1"], obs_in, form)
            qe_pin += np.where(d, qp[np.arange(len(idx_np)), sub["a1"][t].astype(np.int64)], 0.0)
        obs_in = sub["obs"][t]
    for name, src in (("pos1", env.p1), ("vel1", env.v1), ("pos2", env.p2), ("vel2", env.v2),
                      ("r1_acc", env.ret1), ("r2_acc", env.ret2)):
        np.testing.assert_array_equal(src[idx].cpu().numpy(), envs[name], err_msg=name)
    np.testing.assert_array_equal(env.counts[idx].cpu().numpy().astype(np.uint32), stats[1])
    np.testing.assert_array_equal(env.returns[idx].cpu().numpy(), stats[0])
    assert stats[1][:, 0].sum() > counts0[:, 0].sum()  # episodes ended in the window
    # main.py's pending value where the ego has arrived first: what the next launch reads back
    # (the no-wait statistics load it only for those envs, pend_load)
    w1 = envs["winner"] == 1
    np.testing.assert_array_equal(env._ep_stats[idx][:, 3].cpu().numpy()[w1], envs["ep_reward_main"][w1])
    check_q_eval(env.q_eval[idx].cpu().numpy(), qe, qe_abs, f"full-size ego l1 ({opponent})", pinned=qe_pin,
                 model=qe_pin)
    cc1.finish()
    if opponent in ("self", "other"):
        cc2.finish()


@pytest.mark.parametrize("opponent", ["none", "self"])
def test_q_eval_with_non_default_vehicle_boxes(torch, nets, opponent):
    """may_finish_next's collision reach comes from the params (finish_bound: veh_w + 1 and veh_h + 1
    plus the arc's lateral drift), not the default boxes' 5.75 / 9 m: with 14 x 30 m boxes the cars
    collide far earlier, and every episode's logged q_eval must still be eval_net(state)[action] of
    its last step (main.py:221) -- the oracle MFMA rule's Q row of the kernel's own input
    observation -- on explore steps too. (The env dynamics at these params have no oracle; the
    transitions are the kernel's.)"""
    from merging_gym import MergeVecEnv
    from merging_gym.policy import QNet

    n, T, seed = 4096, 48, 3
    env = MergeVecEnv(n, device="cuda:0")
    env.params.veh_w, env.params.veh_h = 14, 30
    for k in range(150):
        env.step_random(seed + 1, step_idx=k)
    env.clear_statistics()
    qnet = QNet.from_state_dict(nets["l1"], device="cuda:0")
    form = "16x16" if opponent == "self" else "32x32"
    obs_in = env.observe().cpu().numpy().copy()
    qe0 = env.q_eval.cpu().numpy().copy()
    traj = env.rollout_qnet(T, qnet, seed, opponent=opponent, first_step=500)
    a1, done, coll = (traj[k].cpu().numpy() for k in ("a1", "done", "collision"))
    obs = traj["obs"].cpu().numpy()
    exp = qe0.copy()
    for t in range(T):
        d = done[t]
        if d.any():
            q = mo.qnet_reference_mfma(nets["l1"], obs_in, form=form).astype(np.float64)
            exp += np.where(d, q[np.arange(n), a1[t].astype(np.int64)], 0.0)
        obs_in = obs[t]
    assert coll.sum() > 100 and done.sum() > 500, (int(coll.sum()), int(done.sum()))
    got = env.q_eval.cpu().numpy()
    bad = np.flatnonzero(got != exp)
    assert bad.size == 0, (bad.size, bad[:8].tolist(), got[bad[:4]].tolist(), exp[bad[:4]].tolist())
