"""bench.py's inputs from the committed profiles (CPU): the HBM traffic and VALU summaries it
attaches to the JSON line load, and a malformed or extra entry in them never breaks the line
(a string note in profiles/valu_busy.json once raised inside load_valu)."""

import importlib.util
import json
import os

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_profile_loaders_read_the_committed_files():
    b = _bench()
    step = b.load_pmc(1 << 20)
    roll = b.load_pmc(1 << 20, "rollout")
    assert step is not None and 0.99 < step / (152 * (1 << 20)) < 1.05
    assert roll is not None and 1.0 < roll / ((52 * 16 + 100) * (1 << 20)) < 1.2
    assert b.load_pmc(12345) is None
    valu = b.load_valu()
    for k in ("step_kernel", "rollout_kernel", "qnet_rollout", "hdqn_rollout"):
        assert k in valu and 0.0 < valu[k]["valu_busy_frac"] < 1.0, k
    assert all(isinstance(v, dict) for v in valu.values())


def test_loaders_skip_notes(tmp_path, monkeypatch):
    b = _bench()
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "valu_busy.json").write_text(json.dumps({"source": "a note", "cmp": {"x": 1},
                                                     "k": {"VALUBusy": 50.0, "insts_per_64_env_steps": {"valu": 9}}}))
    (prof / "pmc_traffic.json").write_text(json.dumps({"envs": 4, "hbm_bytes_per_launch": 7.0, "source": "s"}))
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    assert b.load_valu() == {"k": {"valu_busy_frac": 0.5, "valu_insts_per_lane_step": 9, "fp64_share_of_valu": None,
                                   "source": "profiles/valu_busy.json (rocprofv3 --pmc VALUBusy + SQ_INSTS_VALU*, 2^20 envs)"}}
    assert b.load_pmc(4) == 7.0 and b.load_pmc(4, "rollout") is None
