"""The vectorised NumPy restatement (oracle/merge_numpy.py, bench.py's NumPy CPU baseline) equals
the C oracle: Philox actions bit-exact, fp64 state and statistics bit-exact, flags exact,
observations to the last few ulps (numpy's sin/cos vs libm's)."""

import numpy as np

import merge_numpy as mn


def test_qp_constants_match_the_library():
    from merging_gym import _native

    p = _native.default_params()
    assert (mn.QP_NZ, mn.QP_Z0) == (p.qp_nz, p.qp_z0)


def test_philox_matches_c_oracle(coracle):
    g = np.arange(5, 5 + 3000, dtype=np.int64) + (1 << 33)
    a1, a2 = mn.random_actions(g, 1234, 77, True)
    c1, c2 = coracle.random_actions(3000, int(g[0]), 1234, 77, True)
    np.testing.assert_array_equal(a1, c1)
    np.testing.assert_array_equal(a2, c2)


def test_numpy_batch_equals_c_oracle(coracle):
    n, steps, seed = 4096, 420, 9
    nb = mn.NumpyMergeBatch(n)
    envs = coracle.new_envs(n)
    coracle.reset(envs)
    ret_sum, counts = np.zeros((n, 3)), np.zeros((n, 6), np.uint32)
    for k in range(steps):
        a1, a2 = mn.random_actions(nb.gidx, seed, k, opponent_random=k % 3 != 0)
        obs, rew, done, coll = nb.step(a1, a2)
        o_obs, o_rew, o_done, o_coll, _, o_fobs, err = coracle.step(
            envs, a1.astype(np.int8), a2.astype(np.int8), autoreset=True, final_obs=True,
            stats=(ret_sum, counts))
        assert err == 0
        np.testing.assert_array_equal(done, o_done.astype(bool), err_msg=str(k))
        np.testing.assert_array_equal(coll, o_coll.astype(bool), err_msg=str(k))
        np.testing.assert_array_equal(rew, o_rew, err_msg=str(k))
        fo = np.where(done[:, None], o_fobs, o_obs)  # numpy returns the terminal observation
        np.testing.assert_allclose(obs, fo, rtol=1e-13, atol=1e-9)
    for a, b in (("p1", "pos1"), ("v1", "vel1"), ("p2", "pos2"), ("v2", "vel2"), ("r1", "r1_acc"),
                 ("r2", "r2_acc")):
        np.testing.assert_array_equal(getattr(nb, a), envs[b], err_msg=a)
    np.testing.assert_array_equal(nb.ret_sum, ret_sum)
    np.testing.assert_array_equal(nb.counts, counts.astype(np.int64))
    assert counts[:, 0].sum() > 1000
