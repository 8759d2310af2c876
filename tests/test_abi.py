"""The C-ABI library loads on a CPU-only host and exports every entry point include/*.h declares."""

import ctypes
import glob
import os
import re

from conftest import ROOT


def _declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        names |= set(re.findall(r"^\s*(?:int|void|size_t|const char\*)\s+(mg_\w+)\s*\(", text, re.M))
    return names


def test_header_declares_the_step_path():
    assert {"mg_step", "mg_step_random", "mg_reset", "mg_observe", "mg_abi_version",
            "mg_last_error", "mg_params_default", "mg_rollout_random", "mg_rollout_qnet",
            "mg_qnet_pack", "mg_qnet_forward", "mg_qnet_packed_bytes", "mg_replay_store",
            "mg_replay_sample", "mg_replay_scratch_bytes", "mg_goal_status", "mg_qnet_fragments",
            "mg_qnet_fragment_bytes", "mg_host_step", "mg_host_reset", "mg_host_observe", "mg_stats_reduce",
            "mg_stats_reduce_scratch_bytes", "mg_build_info"} <= _declared()


def test_library_exports_every_declared_symbol():
    from merging_gym import _native

    lib = ctypes.CDLL(_native.LIB_PATH)
    for name in sorted(_declared()):
        assert hasattr(lib, name), name
    assert _native.lib.mg_abi_version() == _native.ABI_VERSION


def test_struct_layouts_match_header():
    from merging_gym import _native

    # mg_params: 15 doubles + 5 doubles + 4 int32 + 5 doubles; mg_rec64: 20 doubles + 2 uint32
    assert ctypes.sizeof(_native.Params) == 20 * 8 + 16 + 40
    assert ctypes.sizeof(_native.State) == 7 * 8
    assert ctypes.sizeof(_native.Outputs) == 10 * 8
    assert ctypes.sizeof(_native.Traj) == 9 * 8
    assert ctypes.sizeof(_native.Transitions) == 12 * 8
    assert ctypes.sizeof(_native.Stats) == 8
    assert ctypes.sizeof(_native.HdqnTraj) == 6 * 8
    assert ctypes.sizeof(_native.Rec64) == 168
    assert _native.EPISODE_STATS_BYTES == 64  # mg_episode_stats: 4 f64 + 8 u32 (ABI 17)
    assert _native.EPISODE_STATS_DTYPE.fields["counts"][1] == 32
    assert _native.REC64_DTYPE.itemsize == 168


def test_default_params_are_the_reference_constants():
    """merging_env.py:22-46, :101 -- filled by the library itself (host code, no GPU)."""
    import numpy as np

    from merging_gym import _native

    p = _native.default_params()
    assert (p.R, p.H, p.W, p.dT) == (30000.0, 1000.0, 300.0, 0.2)
    assert (p.r_first, p.r_second, p.r_collision, p.vel_penalty, p.time_penalty) == (2.0, 1.0, -10.0, 0.001, 0.0)
    assert (p.start_point, p.end_point, p.start_vel, p.vel_ref, p.prediction_t) == (50.0, 950.0, 20.0, 20.0, 3.0)
    assert list(p.action_speed) == [0.0, 10.0, 20.0, 30.0, 40.0]
    assert (p.veh_w, p.veh_h, p.timeout_steps) == (4, 8, 2501)
    assert p.angle0 == float(np.arctan2(1000, 30000))
    assert p.inv_R == 1.0 / 30000.0
    # mpc_1d's equality step (helper.py:152-191) in quadprog's qpgen2 order: z'n and z[0] of
    # z = J J'n, J = R^-1 (dpofa, dpori), for t = 3; qpgen2's vsmall probe
    assert (p.qp_nz, p.qp_z0) == (90.0000000000015, 30.000000000000533)
    assert p.qp_inv_nz == 1.0 / p.qp_nz
    assert p.qp_vsmall == 1.4272476927059598e-15


def test_qp_step_constants_reproduce_the_oracle_qp(coracle, golden):
    """The kernel's u0 = (b / qp_nz) * qp_z0, b = vt - v0, or -0.0 where |b| < qp_vsmall
    (merging_hip.hip mpc_acc) is bit for bit -- sign of zero included -- the first control of the
    oracle's full qpgen2 solve (dpofa, dposl, dpori, the equality step), and of the Python
    restatement, on the golden mpc inputs and on every (action, speed) pair a step can meet,
    including speeds decayed below vsmall under action 0 and speeds equal to the target."""
    import math

    import numpy as np

    import merge_oracle as mo
    from merging_gym import _native

    p = _native.default_params()
    rng = np.random.default_rng(5)
    cases = list(zip(golden["mpc_x0"], golden["mpc_v0"], golden["mpc_vt"]))
    cases += [(float(x), float(v), 10.0 * a) for x, v, a in
              zip(rng.uniform(0, 1100, 4000), np.concatenate([rng.uniform(0, 45, 3000),
                                                              rng.uniform(0, 1e-3, 1000)]),
                  rng.integers(0, 5, 4000))]
    vs = p.qp_vsmall
    cases += [(50.0, v, 0.0) for v in (0.0, vs / 2, np.nextafter(vs, 0), vs, np.nextafter(vs, 1), 2 * vs, 1e-300)]
    cases += [(50.0, 10.0 * a, 10.0 * a) for a in range(5)]  # b = 0 exactly
    cases += [(50.0, np.nextafter(10.0 * a, 50), 10.0 * a) for a in range(5)]
    for x0, v0, vt in cases:
        ref = coracle.mpc_first_accel(float(x0), float(v0), 0.0, float(vt), 3.0)
        b = float(vt) - float(v0)
        kern = -0.0 if abs(b) < vs else (b / p.qp_nz) * p.qp_z0
        assert kern == ref and math.copysign(1, kern) == math.copysign(1, ref), (x0, v0, vt, kern, ref)
        py = mo.first_accel(float(x0), float(v0), 0.0, float(vt), 3.0)
        assert py == ref and math.copysign(1, py) == math.copysign(1, ref), (x0, v0, vt, py, ref)


def test_argument_errors_without_gpu():
    """Validation happens before any launch, so it is testable on a CPU-only host."""
    from merging_gym import _native

    rc = _native.lib.mg_step(ctypes.byref(_native.default_params()), ctypes.byref(_native.State()),
                             None, None, ctypes.byref(_native.Outputs()), None, 16, 0, None)
    assert rc != 0 and b"NULL" in _native.lib.mg_last_error()
    rc = _native.lib.mg_reset(None, None, None, None, 1, None)
    assert rc != 0
    # a packed net (ABI 19): the 16x16 forward's fragments (56 of 64 lanes x 16 bytes + 4 of 512 B),
    # then the 32x32 layout (W1 [204 x 24], W2 [104 x 232], W3 [9 x 136] bf16); the fragment copy
    # is the first part
    assert _native.lib.mg_qnet_fragment_bytes() == 56 * 1024 + 4 * 512
    assert _native.lib.mg_qnet_packed_bytes() == 56 * 1024 + 4 * 512 + 2 * (204 * 24 + 104 * 232 + 9 * 136)
    assert _native.lib.mg_qnet_fragments(None, None, None) != 0 and b"NULL" in _native.lib.mg_last_error()
    odd = ctypes.c_void_p((1 << 20) + 8)
    assert _native.lib.mg_qnet_fragments(odd, odd, None) != 0 and b"aligned" in _native.lib.mg_last_error()
    # replay: missing buffers, bad capacity and short scratch are refused before any launch
    tr = _native.Transitions()
    rc = _native.lib.mg_replay_store(None, None, 16, 22, ctypes.byref(tr), 4, 1, 0, None, 0, None)
    assert rc != 0 and b"NULL" in _native.lib.mg_last_error()
    fake = ctypes.c_void_p(1 << 20)  # never dereferenced: validation fails first
    rc = _native.lib.mg_replay_store(fake, fake, 0, 22, ctypes.byref(tr), 4, 1, 0, None, 0, None)
    assert rc != 0 and b"capacity" in _native.lib.mg_last_error()
    tr = _native.Transitions(fake, fake, None, fake, fake, None, None)
    rc = _native.lib.mg_replay_store(fake, fake, 16, 22, ctypes.byref(tr), 4, 1, 0, fake, 8, None)
    assert rc != 0 and b"scratch" in _native.lib.mg_last_error()
    rc = _native.lib.mg_replay_sample(fake, fake, 0, 22, 0, 0, 0, fake, None, 4, None)
    assert rc != 0 and b"capacity" in _native.lib.mg_last_error()
    # row width must match the goal columns (hdqn.py:158's 24-float rows need goal + next_goal)
    rc = _native.lib.mg_replay_store(fake, fake, 16, 24, ctypes.byref(tr), 4, 1, 0, fake, 1 << 20, None)
    assert rc != 0 and b"row_floats" in _native.lib.mg_last_error()
    trg = _native.Transitions(fake, fake, None, fake, fake, None, None, fake, None, None)
    rc = _native.lib.mg_replay_store(fake, fake, 16, 24, ctypes.byref(trg), 4, 1, 0, fake, 1 << 20, None)
    assert rc != 0 and b"row_floats" in _native.lib.mg_last_error()
    rc = _native.lib.mg_replay_sample(fake, fake, 16, 23, 0, 0, 0, fake, None, 4, None)
    assert rc != 0 and b"row_floats" in _native.lib.mg_last_error()
    # the interleaved step record: 4-byte aligned, and it replaces done / coll / a1_out / a2_out
    P, st = ctypes.byref(_native.default_params()), ctypes.byref(_native.State(*([fake] * 7)))
    bad = _native.Outputs(flags=ctypes.c_void_p((1 << 20) + 2))
    rc = _native.lib.mg_step_random(P, st, None, None, ctypes.byref(bad), None, 16, 0, 1, 0, 1, 0, None)
    assert rc != 0 and b"4-byte" in _native.lib.mg_last_error()
    both = _native.Outputs(done=fake, flags=fake)
    rc = _native.lib.mg_step(P, st, fake, None, ctypes.byref(both), None, 16, 0, None)
    assert rc != 0 and b"flags replaces" in _native.lib.mg_last_error()
    rc = _native.lib.mg_step_random(P, st, fake, None, ctypes.byref(_native.Outputs(flags=fake)), None, 16, 0, 1,
                                    0, 1, 0, None)
    assert rc != 0 and b"a1_out" in _native.lib.mg_last_error()
    # h-DQN acting loop: the self-play / other-checkpoint opponent needs its goal array (mode 3
    # also both of its nets, 16-byte aligned), the fused ring its counter and 16-byte alignment,
    # opponent modes beyond 3 are refused
    traj, ht = ctypes.byref(_native.Traj()), ctypes.byref(_native.HdqnTraj())

    def hdqn(goal_op, mode, ring=None, counter=None, cap=0, opp=(None, None)):
        return _native.lib.mg_rollout_hdqn(P, st, traj, ht, None, fake, goal_op, None, 16, 0, 1, 0, 4, fake, 3, fake,
                                          0, 1 << 31, mode, opp[0], opp[1], ring, counter, cap, 0, None)
    assert hdqn(None, 2) != 0 and b"goal_op" in _native.lib.mg_last_error()
    assert hdqn(None, 3, opp=(fake, fake)) != 0 and b"goal_op" in _native.lib.mg_last_error()
    assert hdqn(fake, 3) != 0 and b"opp_meta_net" in _native.lib.mg_last_error()
    assert hdqn(fake, 3, opp=(fake, ctypes.c_void_p((1 << 20) + 8))) != 0
    assert b"opp_meta_net" in _native.lib.mg_last_error()
    assert hdqn(fake, 4) != 0 and b"opponent_mode" in _native.lib.mg_last_error()
    assert hdqn(None, 0, ring=fake) != 0 and b"ring_counter" in _native.lib.mg_last_error()
    assert hdqn(None, 0, ring=ctypes.c_void_p((1 << 20) + 8), counter=fake, cap=16) != 0
    assert b"16-byte" in _native.lib.mg_last_error()
    # hdqn.py resets at every episode end: a launch without MG_AUTORESET is refused (ABI 17)
    assert hdqn(None, 0) != 0 and b"MG_AUTORESET" in _native.lib.mg_last_error()
    # mg_goal_status: NULL arrays refused; n == 0 is a no-op
    assert _native.lib.mg_goal_status(None, fake, fake, 4, None) != 0 and b"NULL" in _native.lib.mg_last_error()
    assert _native.lib.mg_goal_status(fake, fake, fake, 0, None) == 0
    # the rollout's register-held episode counts are 16-bit per launch: num_steps <= 65535
    rc = _native.lib.mg_rollout_random(P, st, traj, None, 16, 0, 1, 0, 65536, 1, 0, None)
    assert rc != 0 and b"65535" in _native.lib.mg_last_error()
    # Goal_DQN's outputs (ext_reward / no_break) need the running sums, ext_acc
    htm = _native.HdqnTraj(None, None, None, None, fake, None)
    rc = _native.lib.mg_rollout_hdqn(P, st, traj, ctypes.byref(htm), None, fake, None, None, 16, 0, 1, 0, 4, fake,
                                     3, fake, 0, 1 << 31, 0, None, None, None, None, 0, 0, None)
    assert rc != 0 and b"ext_acc" in _native.lib.mg_last_error()
    # Goal_DQN rows in the replay store need reward and the no-break mask
    trm = _native.Transitions(fake, fake, None, fake, fake, None, None, None, None, None, None, fake)
    rc = _native.lib.mg_replay_store(fake, fake, 16, 22, ctypes.byref(trm), 4, 1, 0, fake, 1 << 20, None)
    assert rc != 0 and b"meta_goal" in _native.lib.mg_last_error()
    # 65536 write blocks in 1024 scan groups: ticket (8) + bases u64 + offsets u32 + totals u32
    assert _native.lib.mg_replay_scratch_bytes(1 << 20, 16) == 8 + 1024 * 8 + 65536 * 4 + 1024 * 4
    assert _native.lib.mg_replay_scratch_bytes(0, 4) == 0
    # the statistics reduction (ABI 20): one 80-byte partial per 1,024 records; NULL / misaligned refused
    assert _native.lib.mg_stats_reduce_scratch_bytes(1 << 20) == 1024 * 80
    assert _native.lib.mg_stats_reduce_scratch_bytes(1025) == 2 * 80 and _native.lib.mg_stats_reduce_scratch_bytes(0) == 0
    assert _native.lib.mg_stats_reduce(fake, 4, None, fake, 1 << 20, None) != 0 and b"NULL" in _native.lib.mg_last_error()
    assert _native.lib.mg_stats_reduce(fake, 4, fake, fake, 8, None) != 0 and b"scratch" in _native.lib.mg_last_error()
    assert _native.lib.mg_stats_reduce(odd, 4, fake, fake, 1 << 20, None) != 0
    assert b"aligned" in _native.lib.mg_last_error()


def test_empty_batches_are_no_ops_without_gpu():
    """n == 0 (or num_steps == 0) returns success before any launch, for every entry point."""
    from merging_gym import _native

    lib, P = _native.lib, ctypes.byref(_native.default_params())
    fake = ctypes.c_void_p(1 << 20)  # never dereferenced
    st = _native.State(*([fake] * 7))
    out = ctypes.byref(_native.Outputs())
    traj = ctypes.byref(_native.Traj())
    assert lib.mg_step(P, ctypes.byref(st), fake, None, out, None, 0, 0, None) == 0
    assert lib.mg_step_random(P, ctypes.byref(st), None, None, out, None, 0, 0, 1, 0, 1, 0, None) == 0
    assert lib.mg_rollout_random(P, ctypes.byref(st), traj, None, 0, 0, 1, 0, 16, 1, 0, None) == 0
    assert lib.mg_rollout_random(P, ctypes.byref(st), traj, None, 64, 0, 1, 0, 0, 1, 0, None) == 0
    assert lib.mg_rollout_qnet(P, ctypes.byref(st), traj, None, 0, 0, 1, 0, 16, fake, 5, 0, 0, 0, None, 0,
                               None) == 0
    # main.py's Strategy_OP "L1" opponent (its own net): opp_net required and 16-byte aligned
    assert lib.mg_rollout_qnet(P, ctypes.byref(st), traj, None, 16, 0, 1, 0, 4, fake, 5, 0, 3, 0, None, 0,
                               None) != 0 and b"opp_net" in lib.mg_last_error()
    assert lib.mg_rollout_qnet(P, ctypes.byref(st), traj, None, 16, 0, 1, 0, 4, fake, 5, 0, 3, 0,
                               ctypes.c_void_p((1 << 20) + 8), 0, None) != 0
    assert lib.mg_rollout_qnet(P, ctypes.byref(st), traj, None, 16, 0, 1, 0, 4, fake, 5, 0, 4, 0, fake, 0,
                               None) != 0 and b"opponent_mode" in lib.mg_last_error()
    assert lib.mg_reset(P, ctypes.byref(st), None, out, 0, None) == 0
    assert lib.mg_observe(P, ctypes.byref(st), out, 0, None) == 0
    assert lib.mg_qnet_forward(fake, fake, 10, 0, fake, 0, None) == 0
    assert lib.mg_qnet_forward(fake, fake, 11, 1, fake, 4, None) != 0  # swap needs in_dim 10
    tr = _native.Transitions(fake, fake, None, fake, fake, None, None)
    assert lib.mg_replay_store(fake, fake, 16, 22, ctypes.byref(tr), 0, 4, 1, None, 0, None) == 0
    assert lib.mg_replay_sample(fake, fake, 16, 22, 0, 0, 0, fake, None, 0, None) == 0


def test_timeout_step_is_2501():
    """time_stamp += 0.2 in fp64 first exceeds 500 at step 2501 (merging_env.py:141-143)."""
    t, k = 0.0, 0
    while not t > 500:
        t += 0.2
        k += 1
    assert k == 2501


def test_build_flags_disable_contraction():
    from merging_gym import build

    assert "-ffp-contract=off" in build.HIPCC_FLAGS and "--offload-arch=gfx950" in build.HIPCC_FLAGS
    src = open(build.SRC).read()
    assert "#pragma clang fp contract(off)" in src
