"""CSV trajectory logs (scripts/human_player.py:108-111, :180-181): the writer fed by the
Python oracle reproduces the reference env's own files (tests/golden/csv, made by gen_csv.py)
row for row -- the same header, the same rows kept, the same text for every int-typed field
(Python ints such as 900, actions, an empty field for None) and floats within 1e-9, the
golden-trace tolerance (the QP solve differs from the generator's stand-in by ~1e-14, which
moves last digits) -- and the fp32 formatting of the batched logger round-trips exactly."""

import os

import numpy as np
import pytest

import merge_oracle as mo
from conftest import ROOT

CSV_DIR = os.path.join(ROOT, "tests", "golden", "csv")


@pytest.mark.parametrize("ep", [0, 1, 2, 3])
def test_oracle_episode_csv_is_byte_identical(tmp_path, ep):
    from merging_gym.trajlog import EpisodeCSVWriter

    acts = np.load(os.path.join(CSV_DIR, "actions.npz"))
    a1, a2 = acts[f"ep{ep}_a1"], acts[f"ep{ep}_a2"]
    env = mo.PyMergeEnv()
    state = env.reset()
    path = tmp_path / f"episode{ep}"
    with EpisodeCSVWriter(str(path)) as w:
        for k in range(len(a1)):
            action, action_op = int(a1[k]), (None if a2[k] < 0 else int(a2[k]))
            next_state, rewards, done, info = env.step(action, action_op)
            w.record(state, action, action_op, rewards, env.winner)
            state = next_state
        assert done
    assert_csv_equivalent(path.read_bytes(), open(os.path.join(CSV_DIR, f"episode{ep}"), "rb").read())


def _is_int_text(t: str) -> bool:
    return t != "" and all(c in "-0123456789" for c in t)


def assert_csv_equivalent(got: bytes, ref: bytes, tol=1e-9):
    """Same line structure and terminators; int-typed fields identical text; floats within tol."""
    g, r = got.split(b"\r\n"), ref.split(b"\r\n")
    assert len(g) == len(r), (len(g), len(r))
    assert g[0] == r[0]  # header
    for k, (lg, lr) in enumerate(zip(g[1:], r[1:]), 1):
        fg, fr = lg.decode().split(","), lr.decode().split(",")
        assert len(fg) == len(fr), k
        for a, b in zip(fg, fr):
            if _is_int_text(b) or b == "":
                assert a == b, (k, a, b)
            else:
                assert not _is_int_text(a), (k, a, b)
                assert abs(float(a) - float(b)) <= tol * max(1.0, abs(float(b))), (k, a, b)


def test_fp32_fields_round_trip():
    from merging_gym.trajlog import _fmt32

    rng = np.random.default_rng(0)
    v = np.concatenate([rng.standard_normal(20000).astype(np.float32) * 10.0 ** rng.integers(-6, 4, 20000),
                        np.float32([0.0, -0.0, 900.0, 20.0, -10.0, 1e-8])]).astype(np.float32)
    for x in v:
        s = _fmt32(x)
        assert np.float32(float(s)) == x, (x, s)
    assert _fmt32(np.float32(900.0)) == "900.0" and _fmt32(np.float32(-0.5)) == "-0.5"
