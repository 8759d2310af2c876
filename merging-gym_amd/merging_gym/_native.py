"""ctypes binding of libmerging_hip.so (C-ABI declared in include/merging_hip.h).

The library is built in-tree by __graft_entry__.build() / `python -m merging_gym.build`
(hipcc --offload-arch=gfx950). There is no CPU fallback: if the library is missing or the
ABI version differs, importing this module raises, and every env constructor fails loudly.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libmerging_hip.so"
LIB_PATH = os.environ.get("MERGING_HIP_LIB", os.path.join(_HERE, LIB_NAME))
ABI_VERSION = 20

OBS_DIM = 10
NUM_ACTIONS = 5
ACTION_NONE = -1
ACTION_INVALID = 127  # host marker for a value the reference's action_dict would reject

TF_STEPS_MASK = 0x1FFF  # mg_state.tf is one uint16 per env
TF_WINNER_SHIFT = 13
TF_WINNER_MASK = 0x6000
TF_DONE = 0x8000

AUTORESET = 0x1

ST_DONE, ST_COLLISION, ST_R1_INT, ST_R2_INT, ST_V1_INT, ST_V2_INT = 1, 2, 4, 8, 16, 32

_c = ctypes
_P = ctypes.c_void_p


class Params(_c.Structure):
    _fields_ = [(n, _c.c_double) for n in (
        "R", "H", "W", "dT", "r_first", "r_second", "r_collision", "vel_penalty",
        "time_penalty", "start_point", "end_point", "start_vel", "vel_ref", "prediction_t",
        "angle0")] + [("action_speed", _c.c_double * NUM_ACTIONS), ("veh_w", _c.c_int32),
                      ("veh_h", _c.c_int32), ("timeout_steps", _c.c_int32), ("_pad", _c.c_int32),
                      ("inv_R", _c.c_double), ("qp_nz", _c.c_double), ("qp_z0", _c.c_double),
                      ("qp_inv_nz", _c.c_double), ("qp_vsmall", _c.c_double)]


class State(_c.Structure):
    _fields_ = [(n, _P) for n in ("p1", "v1", "p2", "v2", "ret1", "ret2", "tf")]


class Outputs(_c.Structure):
    _fields_ = [(n, _P) for n in ("obs", "rew", "done", "coll", "done_mask", "final_obs",
                                  "rec64", "error", "won_mask", "flags")]


class Traj(_c.Structure):
    _fields_ = [(n, _P) for n in ("obs", "rew", "done", "coll", "a1", "a2", "final_obs", "won_mask", "flags")]


class Transitions(_c.Structure):
    _fields_ = [(n, _P) for n in ("obs_first", "obs", "final_obs", "a1", "rew", "done", "won_mask", "goal",
                                  "next_goal", "reward", "flags", "meta_goal")]


class HdqnTraj(_c.Structure):
    _fields_ = [(n, _P) for n in ("goal", "next_goal", "reward", "goal_op", "ext_reward", "no_break")]


class Stats(_c.Structure):
    _fields_ = [("rec", _P)]  # mg_episode_stats [n] (64 bytes each, see EPISODE_STATS_DTYPE)


# numpy view of struct mg_episode_stats (ABI 20): the fp64 sums, main.py's pending r1_accumulate,
# the counts (episodes, collisions, ego_first, steps, win_main, win_hdqn), then the q_eval sum
# (reserved zero bytes in ABI 17-19)
EPISODE_STATS_DTYPE = np.dtype([("ret", np.float64, (2,)), ("ret_main", np.float64),
                                ("ret1_pending", np.float64), ("counts", np.uint32, (6,)),
                                ("q_eval", np.float64)])
EPISODE_STATS_FORMAT = 2  # state_dict tag: 1 = ABI 17-19 records (no q_eval), 2 = ABI 20
EPISODE_STATS_BYTES = 64
assert EPISODE_STATS_DTYPE.itemsize == EPISODE_STATS_BYTES


# numpy view of struct mg_rec64 (168 bytes)
REC64_DTYPE = np.dtype([("obs", np.float64, (OBS_DIM,)), ("rew", np.float64, (2,)),
                        ("acc", np.float64, (2,)), ("pos", np.float64, (2,)),
                        ("vel", np.float64, (2,)), ("ret", np.float64, (2,)),
                        ("tf", np.uint32), ("status", np.uint32)])
assert REC64_DTYPE.itemsize == 168


class Rec64(_c.Structure):
    """struct mg_rec64 as a ctypes structure: the single env reads its fields straight from the
    record's memory (host memory, or pinned memory the kernel wrote) without a numpy view."""
    _fields_ = [("obs", _c.c_double * OBS_DIM), ("rew", _c.c_double * 2), ("acc", _c.c_double * 2),
                ("pos", _c.c_double * 2), ("vel", _c.c_double * 2), ("ret", _c.c_double * 2),
                ("tf", _c.c_uint32), ("status", _c.c_uint32)]


assert _c.sizeof(Rec64) == REC64_DTYPE.itemsize


class NativeError(RuntimeError):
    pass


def _load(path=LIB_PATH):
    """Bind libmerging_hip.so (or, for tools/ab_*.py, a variant build of the same ABI at `path`)."""
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found. Build the HIP library first: "
            "python -c 'import __graft_entry__ as g; g.build()' (hipcc --offload-arch=gfx950)")
    import torch  # noqa: F401  -- load torch's libamdhip64 first so the library binds to it

    lib = _c.CDLL(path)
    lib.mg_abi_version.restype = _c.c_int
    lib.mg_last_error.restype = _c.c_char_p
    lib.mg_build_info.restype = _c.c_char_p
    lib.mg_params_default.argtypes = [_c.POINTER(Params)]
    lib.mg_params_default.restype = None
    PP, SP, OP, STP = (_c.POINTER(Params), _c.POINTER(State), _c.POINTER(Outputs),
                       _c.POINTER(Stats))
    lib.mg_step.argtypes = [PP, SP, _P, _P, OP, STP, _c.c_int64, _c.c_uint32, _P]
    lib.mg_step_random.argtypes = [PP, SP, _P, _P, OP, STP, _c.c_int64, _c.c_int64,
                                   _c.c_uint64, _c.c_uint64, _c.c_int32, _c.c_uint32, _P]
    lib.mg_reset.argtypes = [PP, SP, _P, OP, _c.c_int64, _P]
    lib.mg_observe.argtypes = [PP, SP, OP, _c.c_int64, _P]
    lib.mg_rollout_random.argtypes = [PP, SP, _c.POINTER(Traj), STP, _c.c_int64, _c.c_int64,
                                      _c.c_uint64, _c.c_uint64, _c.c_int32, _c.c_int32, _c.c_uint32, _P]
    lib.mg_qnet_packed_bytes.restype = _c.c_size_t
    lib.mg_qnet_fragment_bytes.restype = _c.c_size_t
    lib.mg_qnet_fragments.argtypes = [_P, _P, _P]
    lib.mg_qnet_pack.argtypes = [_P] * 6 + [_c.c_int32, _c.c_int32, _P, _P]
    lib.mg_qnet_forward.argtypes = [_P, _P, _c.c_int32, _c.c_int32, _P, _c.c_int64, _P]
    lib.mg_rollout_qnet.argtypes = [PP, SP, _c.POINTER(Traj), STP, _c.c_int64, _c.c_int64, _c.c_uint64,
                                    _c.c_uint64, _c.c_int32, _P, _c.c_int32, _c.c_uint64, _c.c_int32,
                                    _c.c_uint64, _P, _c.c_uint32, _P]
    lib.mg_rollout_hdqn.argtypes = [PP, SP, _c.POINTER(Traj), _c.POINTER(HdqnTraj), STP, _P, _P, _P, _c.c_int64,
                                    _c.c_int64, _c.c_uint64, _c.c_uint64, _c.c_int32, _P, _c.c_int32, _P,
                                    _c.c_int32, _c.c_uint64, _c.c_int32, _P, _P, _P, _P, _c.c_int64, _c.c_uint32,
                                    _P]
    # ABI 20: the same step / reset / observe on host memory (the CPU single env, BASELINE config 1)
    lib.mg_host_step.argtypes = [PP, SP, _P, _P, OP, STP, _c.c_int64, _c.c_uint32]
    lib.mg_host_reset.argtypes = [PP, SP, _P, OP, _c.c_int64]
    lib.mg_host_observe.argtypes = [PP, SP, OP, _c.c_int64]
    lib.mg_stats_reduce_scratch_bytes.argtypes = [_c.c_int64]
    lib.mg_stats_reduce_scratch_bytes.restype = _c.c_size_t
    lib.mg_stats_reduce.argtypes = [_P, _c.c_int64, _P, _P, _c.c_size_t, _P]
    lib.mg_time_next_launch.argtypes = [_P, _P]
    lib.mg_goal_status.argtypes = [_P, _P, _P, _c.c_int64, _P]
    lib.mg_replay_scratch_bytes.argtypes = [_c.c_int64, _c.c_int32]
    lib.mg_replay_scratch_bytes.restype = _c.c_size_t
    lib.mg_replay_store.argtypes = [_P, _P, _c.c_int64, _c.c_int32, _c.POINTER(Transitions), _c.c_int64,
                                    _c.c_int32, _c.c_int32, _P, _c.c_size_t, _P]
    lib.mg_replay_sample.argtypes = [_P, _P, _c.c_int64, _c.c_int32, _c.c_uint64, _c.c_uint64, _c.c_int32, _P,
                                     _P, _c.c_int64, _P]
    for f in (lib.mg_step, lib.mg_step_random, lib.mg_reset, lib.mg_observe, lib.mg_rollout_random,
              lib.mg_time_next_launch, lib.mg_qnet_pack, lib.mg_qnet_forward, lib.mg_rollout_qnet,
              lib.mg_rollout_hdqn, lib.mg_replay_store, lib.mg_replay_sample, lib.mg_goal_status,
              lib.mg_qnet_fragments, lib.mg_host_step, lib.mg_host_reset, lib.mg_host_observe, lib.mg_stats_reduce):
        f.restype = _c.c_int
    v = lib.mg_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"{path}: ABI version {v}, expected {ABI_VERSION} (stale build?)")
    return lib


def _checked_path() -> str:
    """The in-tree library, built from this tree's source (build.is_current: the sha256 it carries).
    A stale one is rebuilt where hipcc exists, else refused; MERGING_HIP_LIB (a variant build for
    tools/ab_*.py) is taken as given."""
    if "MERGING_HIP_LIB" in os.environ:
        return LIB_PATH
    from . import build

    if os.path.exists(build.SRC) and os.path.exists(LIB_PATH) and not build.is_current(LIB_PATH):
        try:
            build.hipcc()
        except FileNotFoundError:
            raise ImportError(f"{LIB_PATH} was built from another source (src {build.embedded_sha(LIB_PATH)}, "
                              f"tree {build.source_sha()}) and hipcc is not available to rebuild it")
        build.build()
    return LIB_PATH


lib = _load(_checked_path())


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib.mg_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed (hipError {rc}): {msg}")


def build_info() -> str:
    """Compiler / HIP version the loaded library was built with (mg_build_info)."""
    return lib.mg_build_info().decode()


def default_params() -> Params:
    p = Params()
    lib.mg_params_default(_c.byref(p))
    return p
