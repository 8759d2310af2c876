"""Pin the CPU oracle to the reference: golden vectors from the reference's own MergeEnv.

tests/golden/reference_golden.npz was written by tests/golden/gen_golden.py, which runs the
reference (merging_gym/envs/merging_env.py @ /root/reference) with stand-ins for its absent
third-party deps (the QP one restates quadprog's qpgen2 statement by statement, on the matrices
the reference builds). Bar: done / collision / winner / value types exact; the fp64 state
(positions, speeds, accelerations, returns) and the rewards BIT-EXACT; observations exact for
the Python oracle (numpy sin / cos, as the reference) and to 1e-9 for the C oracle (glibc's).
"""

import numpy as np
import pytest

import merge_oracle as mo

TRACES = [f"kat{k}" for k in "ABCDEFG"] + ["rndL0", "rndRR", "past"]
FTOL = 1e-9

T_R1_INT, T_R2_INT, T_OBS3_INT, T_OBS8_INT, T_OBS4_INT, T_OBS9_INT = 1, 2, 4, 8, 16, 32


def _types(obs, rew):
    t = 0
    for bit, v in ((T_R1_INT, rew[0]), (T_R2_INT, rew[1]), (T_OBS3_INT, obs[3]),
                   (T_OBS8_INT, obs[8]), (T_OBS4_INT, obs[4]), (T_OBS9_INT, obs[9])):
        t |= bit if isinstance(v, int) else 0
    return t


def _winner(w):
    return 0 if w is None else w


@pytest.mark.parametrize("trace", TRACES)
def test_python_oracle_replays_reference_trace(golden, trace):
    env = mo.PyMergeEnv()
    g = {k[len(trace) + 1:]: golden[k] for k in golden.files if k.startswith(trace + "_")}
    for k in range(len(g["a1"])):
        if g["reset"][k]:
            obs, rew, done, coll = env.reset(), [0.0, 0.0], False, False
        else:
            a2 = int(g["a2"][k])
            obs, rew, done, info = env.step(int(g["a1"][k]), None if a2 < 0 else a2)
            coll = info["collision"]
        assert bool(done) == bool(g["done"][k]), (trace, k)
        assert coll == bool(g["coll"][k]), (trace, k)
        assert _winner(env.winner) == g["winner"][k], (trace, k)
        assert _types(obs, rew) == g["types"][k], (trace, k)
        np.testing.assert_array_equal(np.asarray(obs, float), g["obs"][k], err_msg=str((trace, k)))
        np.testing.assert_array_equal(np.asarray(rew, float), g["rew"][k], err_msg=str((trace, k)))
        np.testing.assert_array_equal([env.state1["pos"], env.state2["pos"]], g["pos"][k])
        np.testing.assert_array_equal([env.state1["vel"], env.state2["vel"]], g["vel"][k])
        np.testing.assert_array_equal([env.state1["acc"], env.state2["acc"]], g["acc"][k])
        np.testing.assert_array_equal([env.r1_accumulate, env.r2_accumulate], g["racc"][k])
        assert env.time_stamp == g["time"][k]


def _replay_c(coracle, golden, trace):
    g = {k[len(trace) + 1:]: golden[k] for k in golden.files if k.startswith(trace + "_")}
    envs = coracle.new_envs(1)
    for k in range(len(g["a1"])):
        if g["reset"][k]:
            obs = coracle.reset(envs)[0]
            rew, done, coll = np.zeros(2), 0, 0
        else:
            o, r, d, c, st, _, err = coracle.step(envs, g["a1"][k:k + 1], g["a2"][k:k + 1])
            assert err == 0
            obs, rew, done, coll = o[0], r[0], d[0], c[0]
            # the status bits that mark Python ints (rewards 0 / -10, vel int 0)
            t = g["types"][k]
            assert bool(st[0] & 4) == bool(t & T_R1_INT)
            assert bool(st[0] & 8) == bool(t & T_R2_INT)
            assert bool(st[0] & 16) == bool(t & T_OBS4_INT)
            assert bool(st[0] & 32) == bool(t & T_OBS9_INT)
        e = envs[0]
        assert bool(done) == bool(g["done"][k]), (trace, k)
        assert bool(coll) == bool(g["coll"][k]), (trace, k)
        assert e["winner"] == g["winner"][k], (trace, k)
        np.testing.assert_allclose(obs, g["obs"][k], rtol=0, atol=FTOL)  # glibc vs numpy sin / cos
        np.testing.assert_array_equal(rew, g["rew"][k], err_msg=str((trace, k)))
        np.testing.assert_array_equal([e["pos1"], e["pos2"]], g["pos"][k], err_msg=str((trace, k)))
        np.testing.assert_array_equal([e["vel1"], e["vel2"]], g["vel"][k], err_msg=str((trace, k)))
        np.testing.assert_array_equal([e["acc1"], e["acc2"]], g["acc"][k], err_msg=str((trace, k)))
        np.testing.assert_array_equal([e["r1_acc"], e["r2_acc"]], g["racc"][k], err_msg=str((trace, k)))
        assert e["time_stamp"] == g["time"][k]


@pytest.mark.parametrize("trace", TRACES)
def test_c_oracle_replays_reference_trace(coracle, golden, trace):
    _replay_c(coracle, golden, trace)


def test_known_answers(golden):
    """SURVEY.md section 8(a) KAT table, independently of the trace arrays' shape."""
    exp = {  # done step, collision, final returns
        "A": (151, True, (-10.0, -10.0)),
        "B": (2501, False, (-49.74000000000229, 2.0)),
        "C": (225, False, (-0.12007105116872352, 1.0)),
        "D": (2501, False, (-0.12007105116872352, -49.74000000000229)),
        "E": (2501, False, (-49.74000000000229, -0.12007105116872352)),
        "F": (106, True, (-10.920093331094245, -10.920093331094245)),
        "G": (288, True, (-12.740000000328639, -12.740000000328639)),
    }
    acts = {"A": (2, None), "B": (0, None), "C": (4, None), "D": (4, 0), "E": (0, 4),
            "F": (3, 3), "G": (1, 1)}
    for name, (steps, collided, rets) in exp.items():
        env = mo.PyMergeEnv()
        a1, a2 = acts[name]
        for k in range(1, 3000):
            _, _, done, info = env.step(a1, a2)
            if done:
                break
        assert k == steps, name
        assert info["collision"] == collided, name
        np.testing.assert_allclose([env.r1_accumulate, env.r2_accumulate], rets, rtol=0, atol=1e-9)
        assert len(golden[f"kat{name}_done"]) == steps + 1


def test_one_step_rows(coracle, golden):
    """8,000 single steps from random states near the collision / arrival boundaries."""
    n = len(golden["one_a1"])
    ts = [0.0]
    for _ in range(2700):
        ts.append(ts[-1] + 0.2)
    envs = coracle.new_envs(n)
    p, v = golden["one_p"], golden["one_v"]
    envs["pos1"], envs["pos2"] = p[:, 0], p[:, 1]
    envs["vel1"], envs["vel2"] = v[:, 0], v[:, 1]
    envs["winner"] = golden["one_winner"]
    envs["done"] = golden["one_done"]
    envs["time_stamp"] = np.asarray(ts)[golden["one_k"]]
    envs["r1_acc"], envs["r2_acc"] = golden["one_racc"][:, 0], golden["one_racc"][:, 1]
    obs, rew, done, coll, st, _, err = coracle.step(envs, golden["one_a1"], golden["one_a2"])
    assert err == 0
    np.testing.assert_array_equal(done.astype(bool), golden["one_done_out"])
    np.testing.assert_array_equal(coll.astype(bool), golden["one_coll"])
    np.testing.assert_array_equal(envs["winner"], golden["one_winner_out"])
    np.testing.assert_allclose(obs, golden["one_obs"], rtol=0, atol=FTOL)
    np.testing.assert_array_equal(rew, golden["one_rew"])
    np.testing.assert_array_equal(np.stack([envs["pos1"], envs["pos2"]], 1), golden["one_pos"])
    np.testing.assert_array_equal(np.stack([envs["vel1"], envs["vel2"]], 1), golden["one_vel"])
    np.testing.assert_array_equal(np.stack([envs["r1_acc"], envs["r2_acc"]], 1), golden["one_racc_out"])
    assert np.array_equal(envs["time_stamp"], golden["one_time"])


def test_reset_obs_and_spaces(golden):
    env = mo.PyMergeEnv()
    obs = env.reset()
    np.testing.assert_array_equal(np.asarray(obs, float), golden["reset_obs"])
    assert _types(obs, [0.0, 0.0]) == golden["reset_types"]


def test_mpc_closed_form(coracle, golden):
    """mpc_1d's first acceleration (helper.py:152-191 run by the reference itself, solve_qp being
    the qpgen2 stand-in) equals the oracles' bit for bit, and (vt - v0) / t up to fp64 rounding
    (SURVEY 8(a) a2)."""
    acc = np.array([mo.first_accel(x0, v0, x0 + vt * 3.0, vt, 3.0)
                    for x0, v0, vt in zip(golden["mpc_x0"], golden["mpc_v0"], golden["mpc_vt"])])
    np.testing.assert_array_equal(acc, golden["mpc_acc"])
    acc_c = np.array([coracle.mpc_first_accel(x0, v0, x0 + vt * 3.0, vt, 3.0)
                      for x0, v0, vt in zip(golden["mpc_x0"], golden["mpc_v0"], golden["mpc_vt"])])
    np.testing.assert_array_equal(acc_c, golden["mpc_acc"])
    np.testing.assert_array_equal(np.signbit(acc), np.signbit(golden["mpc_acc"]))  # -0.0 where vt == v0
    np.testing.assert_allclose((golden["mpc_vt"] - golden["mpc_v0"]) / 3.0, golden["mpc_acc"],
                               rtol=0, atol=1e-12)
