"""Golden vectors for the replay memory, from the reference's own DQN.store_transition.

Test infrastructure only: run here, in the build container, never on the GPU box. Imports
scripts/main.py from /root/reference (read-only) with the same stand-ins as gen_golden.py,
builds its DQN() (main.py:80-95: memory = np.zeros((MEMORY_CAPACITY, NUM_STATES*2+2)),
MEMORY_CAPACITY = 2000 at :17) and drives it with main.py's collection loop (:189-220): the
reference env steps, and `if env.winner is not 1: dqn.store_transition(state, action, reward,
next_state)` (:209-211). learn() is not called (it would only read the memory). Actions come
from a seeded numpy generator instead of choose_action, so the run is reproducible.

Committed: the action sequences, per-step done/stored flags, the final memory [2000, 22]
(fp64, as the reference holds it) and memory_counter. Only data is written. The same for
scripts/hdqn.py's lower-level memory (tags HL0 / HRR, run_hdqn): goal-augmented rows [2000, 24]
plus the per-step goals and intrinsic rewards that fed them. Both loops also record the
per-episode statistics their scripts log (ep_reward, the win test); run_stats (tags S*) records
main.py's and hdqn.py's statistics side by side over longer trajectories, and goal_status_rows
(tag GS) calls hdqn.py's goal_status on fp64 values around its thresholds.

Usage:  python tests/golden/gen_replay.py   (writes tests/golden/replay_golden.npz)
"""

from __future__ import annotations

import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "replay_golden.npz")


def run(main_mod, env, steps, opp_random, seed):
    rng = np.random.default_rng(seed)
    dqn = main_mod.DQN()
    a1s = rng.integers(0, 5, steps).astype(np.int8)
    a2s = rng.integers(0, 5, steps).astype(np.int8) if opp_random else np.full(steps, -1, np.int8)
    done_f = np.zeros(steps, np.bool_)
    stored = np.zeros(steps, np.bool_)
    reward_list, win_list = [], []  # main.py:222-227, one entry per episode
    with contextlib.redirect_stdout(io.StringIO()):
        state = env.reset()
        ep_reward = 0  # :191
        for k in range(steps):
            a2 = None if a2s[k] < 0 else int(a2s[k])
            next_state, rewards, done, info = env.step(int(a1s[k]), a2)
            reward, _ = rewards
            if env.winner is not 1:  # noqa: F632 -- main.py:209 verbatim semantics
                dqn.store_transition(state, int(a1s[k]), reward, next_state)
                stored[k] = True
                ep_reward += reward  # :211
            done_f[k] = bool(done)
            if done:  # :218-219 break before `state = next_state` (:220): state is the last step's input
                reward_list.append(float(ep_reward))
                win_list.append(bool(state[8] > state[3]))  # :225
                state = env.reset()
                ep_reward = 0
            else:
                state = next_state
    return {"a1": a1s, "a2": a2s, "done": done_f, "stored": stored,
            "memory": np.asarray(dqn.memory, np.float64), "counter": np.int64(dqn.memory_counter),
            "capacity": np.int64(dqn.memory.shape[0]),
            "ep_reward": np.asarray(reward_list, np.float64), "ep_win": np.asarray(win_list, np.bool_)}


def run_stats(env, steps, seed, p_ego, opp_random):
    """The per-episode statistics both training scripts log, from one trajectory of the reference
    env (seeded actions stand in for the agents): main.py:189-227 -- ep_reward sums the ego's
    reward only after steps where `env.winner is not 1` (:209-211), a win is `state[8] > state[3]`
    on the observation the final step acted on (:218-225); hdqn.py:276-346 -- ep_reward sums every
    step's reward (:311-312), a win is the same test on the terminal observation (state =
    next_state at :320 before the break, :342). Also the per-episode length, collision and winner."""
    rng = np.random.default_rng(seed)
    a1s = rng.choice(5, steps, p=p_ego).astype(np.int8)
    a2s = rng.integers(0, 5, steps).astype(np.int8) if opp_random else np.full(steps, -1, np.int8)
    cols = {k: [] for k in ("main_reward", "main_win", "hdqn_reward", "hdqn_win", "length", "collision", "winner",
                            "r1_accumulate", "r2_accumulate")}
    with contextlib.redirect_stdout(io.StringIO()):
        state = env.reset()
        ep_main = ep_h = 0
        length = 0
        for k in range(steps):
            a2 = None if a2s[k] < 0 else int(a2s[k])
            next_state, rewards, done, info = env.step(int(a1s[k]), a2)
            reward, _ = rewards
            length += 1
            if env.winner is not 1:  # noqa: F632 -- main.py:209
                ep_main += reward
            ep_h += reward  # hdqn.py:312
            if done:
                cols["main_reward"].append(float(ep_main))
                cols["main_win"].append(bool(state[8] > state[3]))          # main.py:225
                cols["hdqn_reward"].append(float(ep_h))
                cols["hdqn_win"].append(bool(next_state[8] > next_state[3]))  # hdqn.py:342
                cols["length"].append(length)
                cols["collision"].append(bool(info["collision"]))
                cols["winner"].append(0 if env.winner is None else int(env.winner))
                cols["r1_accumulate"].append(float(env.r1_accumulate))
                cols["r2_accumulate"].append(float(env.r2_accumulate))
                state = env.reset()
                ep_main = ep_h = 0
                length = 0
            else:
                state = next_state
    dt = {"main_win": np.bool_, "hdqn_win": np.bool_, "collision": np.bool_, "length": np.int32, "winner": np.int8}
    out = {k: np.asarray(v, dt.get(k, np.float64)) for k, v in cols.items()}
    out.update(a1=a1s, a2=a2s)
    return out


def goal_status_rows(hdqn_mod):
    """hdqn.py's own goal_status (:223-236) on observation lists whose dx1 = state[0] and
    v2 = state[9] sit on and around its thresholds in fp64: dx1 = +-0.5 v2 and one or two ulps
    either side, v2 = 0 with dx1 = +-0.0 and +-tiny, speeds whose halves fp32 would merge with
    dx1, and random values. Returns dx1, v2 (fp64) and the status."""
    rng = np.random.default_rng(77)
    dx, vv = [], []
    speeds = [0.0, 20.0, 10.000000001, 7.3, 33.33333333333333, 1e-300, 40.0]
    speeds += list(rng.uniform(0.0, 45.0, 12))
    for v2 in speeds:
        for c in (-0.5 * v2, 0.5 * v2):
            x = c
            for k in range(3):
                x = np.nextafter(x, -np.inf)
            for k in range(7):  # c - 3 ulp .. c + 3 ulp
                dx.append(float(x))
                vv.append(float(v2))
                x = np.nextafter(x, np.inf)
        for d in (0.0, -0.0, 5e-324, -5e-324, 1e-50, -1e-50, 1e-13, -1e-13):
            dx.append(d)
            vv.append(float(v2))
        # dx1 = v2 / 2 within fp32 rounding but not equal in fp64
        for rel in (1e-9, -1e-9, 3e-8, -3e-8):
            dx.append(float(0.5 * v2 * (1 + rel)))
            vv.append(float(v2))
            dx.append(float(-0.5 * v2 * (1 + rel)))
            vv.append(float(v2))
    dx += list(rng.uniform(-60, 60, 500))
    vv += list(rng.uniform(0, 45, 500))
    st = [hdqn_mod.goal_status([d, 0, 0, 0, 0, 0, 0, 0, 0, v]) for d, v in zip(dx, vv)]
    return {"dx1": np.asarray(dx, np.float64), "v2": np.asarray(vv, np.float64), "status": np.asarray(st, np.int8)}


def run_hdqn(hdqn_mod, env, steps, opp_random, seed):
    """hdqn.py's lower-level memory: its own HDQN() (:142-184, memory = np.zeros((2000, (NUM_STATES
    + 1) * 2 + 2)), MEMORY_CAPACITY = 2000 at :21) driven by main()'s inner loop (:280-323):
    goal_state = [goal] + state (:291), env.step, goal = upper.choose_goal(next_state) (:303),
    next_goal_state (:304), intrinsic reward 1.0 if goal == goal_status(state) (:314, the
    reference's own goal_status), lower.store_transition (:316), state = next_state (:320), and a
    fresh goal at :283 after the :322 break or an episode end. Goals and actions come from a
    seeded numpy generator instead of the meta-controller / choose_action. Goal_DQN's own memory
    rides along: extrinsic_reward += reward each step (:286, :313) and, after each :322 break or
    episode end, upper.store_transition(state, goal, extrinsic_reward, next_state) (:325, with
    state = next_state already and goal the :303 choice) into its (200, 22) memory (:75)."""
    import torch

    rng = np.random.default_rng(seed)
    lower = hdqn_mod.HDQN()
    upper = hdqn_mod.Goal_DQN()
    extrinsic = 0
    ep_reward, reward_list, win_list = 0, [], []  # hdqn.py:279, :312, :334-346
    a1s = rng.integers(0, 5, steps).astype(np.int8)
    a2s = rng.integers(0, 5, steps).astype(np.int8) if opp_random else np.full(steps, -1, np.int8)
    goal_s = np.zeros(steps, np.float32)
    goal_s2 = np.zeros(steps, np.float32)
    intrinsic = np.zeros(steps, np.float32)
    done_f = np.zeros(steps, np.bool_)
    with contextlib.redirect_stdout(io.StringIO()):
        state = env.reset()
        goal = int(rng.integers(0, 3))  # :283 upper.choose_goal(state)
        for k in range(steps):
            goal_state = torch.unsqueeze(torch.FloatTensor([goal] + state), dim=0)  # :291
            a2 = None if a2s[k] < 0 else int(a2s[k])
            next_state, rewards, done, info = env.step(int(a1s[k]), a2)
            extrinsic += rewards[0]  # :311-313
            ep_reward += rewards[0]  # :312
            new_goal = int(rng.integers(0, 3))  # :303 upper.choose_goal(next_state)
            next_goal_state = torch.unsqueeze(torch.FloatTensor([new_goal] + next_state), dim=0)  # :304
            r_int = 1.0 if new_goal == hdqn_mod.goal_status(state) else 0.0  # :314
            lower.store_transition(goal_state, int(a1s[k]), r_int, next_goal_state)  # :316
            goal_s[k], goal_s2[k], intrinsic[k], done_f[k] = goal, new_goal, r_int, bool(done)
            state = next_state  # :320
            goal = new_goal
            if done or goal == hdqn_mod.goal_status(state):  # :322 break -> :325, then :286
                upper.store_transition(state, goal, extrinsic, next_state)
                extrinsic = 0
            if done:  # episode over (state = next_state, the terminal observation): reset, then :283
                reward_list.append(float(ep_reward))
                win_list.append(bool(state[8] > state[3]))  # :342
                ep_reward = 0
                state = env.reset()
                goal = int(rng.integers(0, 3))
            elif goal == hdqn_mod.goal_status(state):  # :322 break, then :283 picks a fresh goal
                goal = int(rng.integers(0, 3))
    return {"a1": a1s, "a2": a2s, "done": done_f, "goal": goal_s, "next_goal": goal_s2,
            "intrinsic": intrinsic, "memory": np.asarray(lower.memory, np.float64),
            "counter": np.int64(lower.memory_counter), "capacity": np.int64(lower.memory.shape[0]),
            "meta_memory": np.asarray(upper.memory, np.float64), "meta_counter": np.int64(upper.memory_counter),
            "meta_capacity": np.int64(upper.memory.shape[0]),
            "ep_reward": np.asarray(reward_list, np.float64), "ep_win": np.asarray(win_list, np.bool_)}


def _load_net(net, sd):
    """The reference Net's parameters from a state dict of numpy arrays (weights-only data)."""
    import torch

    net.load_state_dict({k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in sd.items()})


def run_q_eval_main(main_mod, env, episodes, seed, weights):
    """main.py's q_eval log (:189-228) from its own DQN: dqn.choose_action(state) (:195, the seeded
    np.random drives its epsilon-greedy branch), env.step, the :218-220 break, then
    q_eval_value = dqn.eval_net.forward(torch.Tensor(state))[action] (:221; .cuda() dropped: no GPU
    here) on the state the last step acted on and its action. eval_net carries the shipped
    checkpoint the bench uses (tests/golden/dqn_checkpoints.npz, l1). Records per episode the
    logged value, that state and that action, and every action taken."""
    import torch

    np.random.seed(seed)
    dqn = main_mod.DQN()
    _load_net(dqn.eval_net, weights)
    q_list, s_list, a_list, acts = [], [], [], []
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(episodes):
            state = env.reset()
            while True:
                action = int(dqn.choose_action(state))
                acts.append(action)
                next_state, rewards, done, info = env.step(action, None)  # Strategy_OP "L0"
                if done:
                    break
                state = next_state
            q = dqn.eval_net.forward(torch.Tensor(state))[action]  # :221
            q_list.append(float(q))
            s_list.append(np.asarray(state, np.float64))
            a_list.append(action)
    return {"q_eval": np.asarray(q_list, np.float32), "state": np.stack(s_list), "action": np.asarray(a_list, np.int8),
            "actions": np.asarray(acts, np.int8)}


def run_q_eval_hdqn(hdqn_mod, env, episodes, seed, meta_sd):
    """hdqn.py's q_eval log (:276-333): the loop of main() with its own Goal_DQN choosing the goals
    (upper.choose_goal at :283 and :303, seeded np.random) and seeded actions standing in for the
    lower-level net, then q_eval_value = upper.meta_eval_net.forward(torch.Tensor(state))[goal] (:330)
    with state the terminal observation (state = next_state, :320) and goal the :303 choice on it.
    meta_sd: seeded Net(10, 3) weights (no h-DQN checkpoint ships with the reference)."""
    import torch

    np.random.seed(seed)
    rng = np.random.default_rng(seed)
    upper = hdqn_mod.Goal_DQN()
    _load_net(upper.meta_eval_net, meta_sd)
    q_list, s_list, g_list, acts = [], [], [], []
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(episodes):
            state = env.reset()
            done = False
            while not done:
                goal = upper.choose_goal(state)  # :283
                while not done:
                    acts.append(int(rng.integers(0, 5)))
                    next_state, rewards, done, info = env.step(acts[-1], None)
                    goal = upper.choose_goal(next_state)  # :303
                    state = next_state  # :320
                    if done or goal == hdqn_mod.goal_status(state):  # :322
                        break
            q = upper.meta_eval_net.forward(torch.Tensor(state))[goal]  # :330
            q_list.append(float(q))
            s_list.append(np.asarray(state, np.float64))
            g_list.append(int(goal))
    return {"q_eval": np.asarray(q_list, np.float32), "state": np.stack(s_list), "goal": np.asarray(g_list, np.int8),
            "actions": np.asarray(acts, np.int8)}


def main():
    sys.path.insert(0, HERE)
    from gen_golden import load_reference_env

    env = load_reference_env()  # puts the stand-ins and /root/reference/scripts on sys.path
    with contextlib.redirect_stdout(io.StringIO()):
        import main as main_mod  # scripts/main.py (module-level gym.make uses the stand-in gym)
        import hdqn as hdqn_mod  # scripts/hdqn.py (main() runs only under __main__)
    out = {}
    for tag, opp, seed in (("L0", False, 7), ("RR", True, 8)):
        res = run(main_mod, env, 3200, opp, seed)
        out.update({f"{tag}_{k}": v for k, v in res.items()})
        print(tag, "stored", int(res["stored"].sum()), "of", len(res["stored"]),
              "episodes", int(res["done"].sum()), "counter", int(res["counter"]))
    for tag, opp, seed in (("HL0", False, 9), ("HRR", True, 10)):
        res = run_hdqn(hdqn_mod, env, 3200, opp, seed)
        out.update({f"{tag}_{k}": v for k, v in res.items()})
        print(tag, "episodes", int(res["done"].sum()), "counter", int(res["counter"]),
              "intrinsic", float(res["intrinsic"].mean()))
    # the scripts' logged episode statistics on longer trajectories (several ego policies)
    for tag, steps, seed, p_ego, opp in (("SU0", 9000, 31, [0.2] * 5, False),
                                         ("SUU", 9000, 32, [0.2] * 5, True),
                                         ("SFU", 9000, 33, [0.05, 0.05, 0.1, 0.3, 0.5], True),
                                         ("SSU", 9000, 34, [0.4, 0.3, 0.1, 0.1, 0.1], True)):
        res = run_stats(env, steps, seed, p_ego, opp)
        out.update({f"{tag}_{k}": v for k, v in res.items()})
        print(tag, "episodes", len(res["length"]), "ego first", int((res["winner"] == 1).sum()),
              "main wins", int(res["main_win"].sum()), "hdqn wins", int(res["hdqn_win"].sum()),
              "filtered != total", int((res["main_reward"] != res["hdqn_reward"]).sum()))
    out.update({f"GS_{k}": v for k, v in goal_status_rows(hdqn_mod).items()})
    # q_eval as the scripts log it (main.py:221, hdqn.py:330), from the reference's own nets
    ck = np.load(os.path.join(HERE, "dqn_checkpoints.npz"))
    l1 = {k.split("/", 1)[1]: ck[k] for k in ck.files if k.startswith("l1/")}
    res = run_q_eval_main(main_mod, env, 40, 51, l1)
    out.update({f"QM_{k}": v for k, v in res.items()})
    print("QM episodes", len(res["q_eval"]), "mean q_eval", float(res["q_eval"].mean()))
    mrng = np.random.default_rng(52)
    meta_sd = {}
    for name, (o, i) in zip(("fc1", "fc2", "out"), [(200, 10), (100, 200), (3, 100)]):
        meta_sd[f"{name}.weight"] = mrng.uniform(-i ** -0.5, i ** -0.5, (o, i)).astype(np.float32)
        meta_sd[f"{name}.bias"] = mrng.uniform(-i ** -0.5, i ** -0.5, o).astype(np.float32)
    res = run_q_eval_hdqn(hdqn_mod, env, 40, 53, meta_sd)
    out.update({f"QH_{k}": v for k, v in res.items()})
    out.update({f"QH_net_{k}": v for k, v in meta_sd.items()})
    print("QH episodes", len(res["q_eval"]), "mean q_eval", float(res["q_eval"].mean()))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
