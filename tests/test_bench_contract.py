"""The committed bench lines keep the driver's JSON contract (CPU: reads the recorded files only).

bench.py itself needs a GPU. This test checks that the lines it printed on the MI355X, which are
kept under profiles/r04/, carry the keys the driver and the judge read. It also checks that
their derived figures agree with their own inputs, e.g. roofline.frac = achieved / peak and
value = envs / ms_per_step.
"""
import glob
import json
import math
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINES = sorted(glob.glob(os.path.join(ROOT, "profiles", "r04", "bench_default_r04*.json")) +
               glob.glob(os.path.join(ROOT, "profiles", "r04", "bench_k20_r04*.json")))

TOP = {"metric": str, "value": float, "unit": str, "n_gpus": int, "steps": int, "warmup": int,
       "ms_per_step": float, "higher_is_better": bool, "scaling": str, "dtype": str, "data": str,
       "config": dict, "roofline": dict}


def _load(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


@pytest.mark.skipif(not LINES, reason="no recorded bench lines")
@pytest.mark.parametrize("path", LINES, ids=[os.path.basename(p) for p in LINES])
def test_recorded_bench_line_keeps_the_contract(path):
    d = _load(path)
    for k, t in TOP.items():
        assert k in d, k
        assert isinstance(d[k], (int, float) if t is float else t), (k, type(d[k]))
    assert "vs_baseline" in d
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["n_gpus"] == 1
    assert "workload" in d["config"]
    # value is whole-job env-steps/s: the envs of every rank stepped once per ms_per_step
    envs = d["config"]["global_envs"]
    assert math.isclose(d["value"], envs / (d["ms_per_step"] * 1e-3), rel_tol=1e-6)
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert math.isclose(r["frac"], r["achieved"] / r["peak"], rel_tol=1e-9)
    # achieved = algorithmic bytes per launch / the kernel's mean launch time (HIP events)
    per_launch = r["bytes_per_env_step"] * d["config"]["envs_per_gpu"]
    assert math.isclose(r["achieved"], per_launch / (r["kernel_ms_mean_max_rank"] * 1e-3) / 1e9, rel_tol=1e-6)
    if r.get("traffic") is not None:  # PMC HBM bytes per launch: close to the algorithmic bytes
        assert 0.9 < r["traffic"] / per_launch < 1.2
    if "cpu_baseline" in d:  # the default run times the oracle on the host (rank 0, N = 1)
        c = d["cpu_baseline"]
        assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0 and c["sample"]


GRIDS = sorted(glob.glob(os.path.join(ROOT, "profiles", "r04", "kernel_stats_by_grid_r04*.json")))


@pytest.mark.skipif(not GRIDS, reason="no recorded rocprofv3 summaries")
@pytest.mark.parametrize("path", GRIDS, ids=[os.path.basename(p) for p in GRIDS])
def test_rocprof_step_kernel_average_agrees_with_the_bench_line(path):
    """The committed rocprofv3 summary of a pass and that pass's bench line time the same kernel:
    the step kernel's average at the 2^20 grid agrees with roofline.kernel_ms_mean within 5 %."""
    tag = os.path.basename(path)[len("kernel_stats_by_grid_"):-len(".json")]
    bench = os.path.join(ROOT, "profiles", "r04", f"bench_default_{tag}.json")
    if not os.path.exists(bench):
        pytest.skip(f"no bench line for {tag}")
    d = _load(bench)
    r = d["roofline"]
    with open(path) as f:
        rows = json.load(f)
    step = [x for x in rows if x["kernel"] == r["kernel"] and x["grid_threads"] == d["config"]["envs_per_gpu"]]
    assert step, (r["kernel"], [x["kernel"] for x in rows])
    assert abs(step[0]["avg_us"] / (r["kernel_ms_mean"] * 1e3) - 1) < 0.05
