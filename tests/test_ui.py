"""UI parity on the CPU: envs/ui.py against the reference MergeEnv's own pygame calls.

tests/golden/render_golden.json holds a human-experiment session run by the reference
MergeEnv (merging_env.py:83-108 construction, :241-395 render / plot / intro / prepare /
feedback / finish) against the recording pygame stand-in in tests/stubs (written by
tests/golden/gen_render.py). Here MergeUI draws each call from the same env state through the
same stand-in, and the two call logs must be identical: every surface, blit position,
circle, polygon corner, colour, text string and wait.
"""

import importlib.util
import json
import os

import numpy as np
import pytest

from merging_gym.envs import ui as mui

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "render_golden.json")


def load_stub():
    """The recording pygame stand-in, under a private name (never shadows a real pygame)."""
    pkg = os.path.join(HERE, "stubs", "pygame")
    spec = importlib.util.spec_from_file_location("mg_pygame_stub", os.path.join(pkg, "__init__.py"),
                                                  submodule_search_locations=[pkg])
    mod = importlib.util.module_from_spec(spec)
    import sys

    sys.modules["mg_pygame_stub"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="module")
def stub():
    return load_stub()


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def view_of(env):
    s1, s2 = env["state1"], env["state2"]
    return {"pos1": s1["pos"], "vel1": s1["vel"], "acc1": s1["acc"], "pos2": s2["pos"],
            "vel2": s2["vel"], "acc2": s2["acc"], "r1": env["r1_accumulate"], "r2": env["r2_accumulate"]}


def call_ui(u, c, view):
    kw = dict(c["kwargs"])
    name = c["call"]
    if c["wait_seed"] is not None:
        np.random.seed(c["wait_seed"])
    if name == "render":
        u.render(view, kw.get("goal"), kw.get("goal_op"), kw.get("player", 1), kw.get("tag_left"),
                 kw.get("tag_right"))
    elif name == "feedback":
        u.feedback(view["r1"], view["r2"], kw.get("player", 1))
    elif name == "finish":
        u.finish(kw["sum_r1"], kw["sum_r2"], kw.get("player", 1))
    else:
        getattr(u, name)(**kw)


def normalised(log):
    return json.loads(json.dumps(log))


def test_construction_matches_reference(stub, golden):
    stub.clear()
    mui.MergeUI(pygame=stub)
    assert normalised(stub.LOG) == golden["init"]


def test_every_ui_call_matches_reference(stub, golden):
    stub.clear()
    u = mui.MergeUI(pygame=stub)
    n = 0
    kinds = set()
    for c in golden["calls"]:
        if c["call"] in ("reset", "step"):
            continue
        stub.LOG.clear()
        call_ui(u, c, view_of(c["env"]))
        assert normalised(stub.LOG) == c["log"], (n, c["call"], c["kwargs"])
        n += 1
        kinds.add(c["call"])
    assert kinds == {"intro", "prepare", "render", "feedback", "finish", "plot"}
    assert n > 60


def test_golden_covers_colours_tags_and_types(golden):
    """The session exercises every branch render() has: goal / acceleration colours, tags,
    int and float text values, both players."""
    colours, texts, players = set(), set(), set()
    for c in golden["calls"]:
        if c["call"] != "render":
            continue
        players.add(c["kwargs"].get("player", 1))
        for e in c["log"]:
            if e[0] == "polygon":
                colours.add(tuple(e[2]))
            if e[0] == "blit" and isinstance(e[2], list):
                texts.add(e[2][2])
    assert {(255, 0, 0), (0, 0, 255), (0, 0, 0), (120, 120, 120)} <= colours
    assert {"Rwd:0", "Spd: 20.0", "Finished"} <= texts
    assert players == {1, 2}


def test_text_rounding_follows_numpy_float64():
    """round(np.float64, 2) (the reference's values after a step) is not Python's round."""
    assert mui._r2(2.675) == "2.68" and round(2.675, 2) == 2.67
    assert mui._r2(0) == "0" and mui._r2(20.0) == "20.0" and mui._r2(-0.0006) == "-0.0"


def test_scene_geometry_is_pure_numpy():
    v = {"pos1": 50, "vel1": 20.0, "acc1": 0.0, "pos2": 50, "vel2": 20.0, "acc2": 0.0, "r1": 0, "r2": 0}
    prims = mui.scene(v)
    assert [p[0] for p in prims].count("circle") == 8
    assert [p[0] for p in prims].count("polygon") == 6
    # each panel's own car: the 4 x 8 box around (150, 600), scaled 5x about its centre
    own = [(140.0, 580.0), (160.0, 580.0), (160.0, 620.0), (140.0, 620.0)]
    right = [p for p in prims if p[0] == "polygon" and p[1] == "right"]
    left = [p for p in prims if p[0] == "polygon" and p[1] == "left"]
    assert right[1][3] == own and left[2][3] == own
    # level cars: the other car is drawn one lane-gap away, mirrored between the panels
    dx = right[2][3][0][0] - 140.0
    assert dx < 0 and left[1][3][0][0] - 140.0 == pytest.approx(-dx)


def test_ui_without_pygame_raises_importerror(monkeypatch):
    import builtins

    real = builtins.__import__

    def deny(name, *a, **k):
        if name == "pygame" or name.startswith("pygame."):
            raise ImportError("no pygame")
        return real(name, *a, **k)

    monkeypatch.setattr(builtins, "__import__", deny)
    with pytest.raises(ImportError, match="pygame"):
        mui.MergeUI()
