"""UI drawn from the env's step record: the golden human-experiment session (human_player.py's
loop) replayed on the drop-in MergeEnv (host and GPU step backends) and on a GPU MergeVecEnv row.

tests/golden/render_golden.json (gen_render.py) is the reference MergeEnv's own session:
resets, steps with recorded actions and UI calls with the pygame calls they made. Here the
same resets and steps run through the library's step (mg_host_step on the CPU, the HIP step
kernel on the GPU), and each UI call draws the state read back from it -- MergeEnv's step
record, and row 0 of an 8-env MergeVecEnv stepped with the same actions -- through the same
recording stand-in. Text and structure must be
identical; coordinates agree to 1e-9 relative (the device state equals the reference's
fp64 state up to the last-bit rounding of the QP stand-in the golden traces were recorded with).
"""

import json
import math

import numpy as np
import pytest

from test_ui import GOLDEN, call_ui, load_stub

BACKENDS = ["host", pytest.param("gpu", marks=pytest.mark.gpu)]


def same_log(ours, ref, rel=1e-9):
    """Structural equality with float tolerance (texts, colours, names exact)."""
    if isinstance(ref, list):
        return isinstance(ours, list) and len(ours) == len(ref) and all(same_log(a, b, rel) for a, b in zip(ours, ref))
    if isinstance(ref, float) and not isinstance(ref, bool):
        return isinstance(ours, (int, float)) and math.isclose(ours, ref, rel_tol=rel, abs_tol=1e-9)
    return ours == ref


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.mark.parametrize("backend", BACKENDS)
def test_merge_env_ui_session_matches_reference(golden, backend):
    from merging_gym.envs.merging_env import MergeEnv
    from merging_gym.envs.ui import MergeUI

    stub = load_stub()
    stub.clear()
    env = MergeEnv(backend=backend)
    env.ui = MergeUI(pygame=stub)
    assert json.loads(json.dumps(stub.LOG)) == golden["init"]
    renders = 0
    for c in golden["calls"]:
        if c["call"] == "reset":
            env.reset()
            continue
        if c["call"] == "step":
            env.step(c["kwargs"]["action1"], c["kwargs"]["action2"])
            continue
        # the attributes the call reads, with the reference's Python types
        for ours, ref in ((env.state1, c["env"]["state1"]), (env.state2, c["env"]["state2"])):
            for k in ("pos", "vel", "acc"):
                assert type(ours[k]) is type(ref[k]) and math.isclose(ours[k], ref[k], rel_tol=1e-12, abs_tol=1e-12)
        for ours, ref in ((env.r1_accumulate, c["env"]["r1_accumulate"]), (env.r2_accumulate, c["env"]["r2_accumulate"])):
            assert type(ours) is type(ref) and math.isclose(ours, ref, rel_tol=1e-12, abs_tol=1e-12)
        stub.LOG.clear()
        if c["wait_seed"] is not None:
            np.random.seed(c["wait_seed"])
        getattr(env, c["call"])(**c["kwargs"])
        log = json.loads(json.dumps(stub.LOG))
        assert same_log(log, c["log"]), (c["call"], c["kwargs"])
        renders += c["call"] == "render"
    assert renders > 40


@pytest.mark.gpu
def test_vector_env_row_renders_like_reference(golden):
    """render_view(i) of a MergeVecEnv row (autoreset off, every env given the session's
    actions) drawn by MergeUI equals the reference's render of the same state."""
    import torch

    from merging_gym import MergeVecEnv
    from merging_gym.envs.ui import MergeUI

    stub = load_stub()
    stub.clear()
    ui = MergeUI(pygame=stub)
    env = MergeVecEnv(8, device="cuda:0", autoreset=False)
    renders = 0
    for c in golden["calls"]:
        if c["call"] == "reset":
            env.reset()
            continue
        if c["call"] == "step":
            a2 = c["kwargs"]["action2"]
            env.step(torch.full((8,), c["kwargs"]["action1"], dtype=torch.int8, device="cuda:0"),
                     None if a2 is None else torch.full((8,), a2, dtype=torch.int8, device="cuda:0"))
            continue
        if c["call"] != "render":
            continue
        e = c["env"]
        view = env.render_view(5, acc=(e["state1"]["acc"], e["state2"]["acc"]))
        stub.LOG.clear()
        call_ui(ui, c, view)
        assert same_log(json.loads(json.dumps(stub.LOG)), c["log"]), c["kwargs"]
        renders += 1
    assert renders > 40
    with pytest.raises(IndexError):
        env.render_view(8)
