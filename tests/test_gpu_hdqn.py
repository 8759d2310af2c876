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

pytestmark = pytest.mark.gpu

OBS_TOL = dict(rtol=1e-6, atol=1e-5)


def _net(rng, in_dim, out_dim):
    sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), [(200, in_dim), (100, 200), (out_dim, 100)]):
        sd[f"{name}.weight"] = rng.uniform(0, 1, (o, i)).astype(np.float32)  # hdqn.py:41-47
        sd[f"{name}.bias"] = rng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    return sd


def _near_tie(q, tol=1e-2):
    s = np.sort(q, axis=1)
    return (s[:, -1] - s[:, -2]) <= tol * np.maximum(1.0, np.abs(s[:, -1]))


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
    for t in range(T):
        x = torch.cat([goal[:, None].to(torch.float32), obs], dim=1)  # goal_state, :291
        q1 = lower.forward(x)
        a1, greedy1 = eps_greedy(q1, 5)  # :292
        q1_ref = mo.qnet_reference(lower_sd, x.cpu().numpy(), bf16=True)
        g1 = greedy1.cpu().numpy()
        ok = (a1.cpu().numpy() == q1_ref.argmax(1)) | ~g1 | _near_tie(q1_ref)
        assert ok.all(), t
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
