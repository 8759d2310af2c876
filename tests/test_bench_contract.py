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
# round 5: the compact last line (bench.compact_line), incl. the multi-rank rehearsals
LINES5 = sorted(glob.glob(os.path.join(ROOT, "profiles", "r05", "bench_*.json")) +
                glob.glob(os.path.join(ROOT, "profiles", "r06", "bench_*.json")))

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


GRIDS = sorted(glob.glob(os.path.join(ROOT, "profiles", "r04", "kernel_stats_by_grid_r04*.json")) +
               glob.glob(os.path.join(ROOT, "profiles", "r05", "kernel_stats_by_grid_r05*.json")) +
               glob.glob(os.path.join(ROOT, "profiles", "r06", "kernel_stats_by_grid_r06*.json")))


@pytest.mark.skipif(not GRIDS, reason="no recorded rocprofv3 summaries")
@pytest.mark.parametrize("path", GRIDS, ids=[os.path.basename(p) for p in GRIDS])
def test_rocprof_step_kernel_average_agrees_with_the_bench_line(path):
    """The committed rocprofv3 summary of a pass and that pass's bench line time the same kernel:
    the step kernel's average at the 2^20 grid agrees with roofline.kernel_ms_mean within 5 %."""
    tag = os.path.basename(path)[len("kernel_stats_by_grid_"):-len(".json")]
    rnd = os.path.basename(os.path.dirname(path))
    # round 4: the default bench line of the same pass; rounds 5-6: the profiled run's own line
    bench = os.path.join(ROOT, "profiles", rnd, f"bench_default_{tag}.json" if rnd == "r04" else f"prof_bench_{tag}.json")
    if not os.path.exists(bench):
        pytest.skip(f"no bench line for {tag}")
    d = _load(bench)
    r = d["roofline"]
    with open(path) as f:
        rows = json.load(f)
    step = [x for x in rows if x["kernel"] == r["kernel"] and x["grid_threads"] == d["config"]["envs_per_gpu"]]
    assert step, (r["kernel"], [x["kernel"] for x in rows])
    assert abs(step[0]["avg_us"] / (r["kernel_ms_mean"] * 1e3) - 1) < 0.05


def check_line(d):
    """The round-5 contract of a bench line at any world size: the driver's keys, the rank count the
    process group reported, the roofline with its all-rank aggregate, and -- at every world size
    (north_star: the reference-style step on the box's host cores in the same run) -- the CPU
    baseline with its core count."""
    for k, t in TOP.items():
        assert k in d, k
        assert isinstance(d[k], (int, float) if t is float else t), (k, type(d[k]))
    n = d["n_gpus"]
    assert n >= 1 and d["dist"]["world_size"] == n, d.get("dist")
    if n > 1:
        assert d["dist"]["backend"] in ("nccl", "gloo"), d["dist"]
    r = d["roofline"]
    for k in ("achieved", "peak", "frac", "kernel_ms_mean_max_rank", "achieved_aggregate", "frac_aggregate"):
        assert isinstance(r.get(k), (int, float)), k
    per_launch = r["bytes_per_env_step"] * d["config"]["envs_per_gpu"]
    assert math.isclose(r["achieved_aggregate"], n * per_launch / (r["kernel_ms_mean_max_rank"] * 1e-3) / 1e9,
                        rel_tol=1e-6)
    assert math.isclose(d["value"], d["config"]["global_envs"] / (d["ms_per_step"] * 1e-3), rel_tol=1e-6)
    c = d.get("cpu_baseline")
    assert c is not None, "no cpu_baseline"
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0 and c["sample"]


def _synthetic(n, with_cpu=True):
    ms = 0.03
    line = {"metric": "m", "value": n * (1 << 20) / (ms * 1e-3), "unit": "env-steps/s", "n_gpus": n, "steps": 20,
            "warmup": 5, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic", "dist": {"backend": "nccl" if n > 1 else None, "world_size": n},
            "config": {"workload": "w", "envs_per_gpu": 1 << 20, "global_envs": n << 20},
            "roofline": {"bound": "hbm", "achieved": 6000.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.75,
                         "bytes_per_env_step": 152, "kernel_ms_mean": 0.026, "kernel_ms_mean_max_rank": 0.027}}
    r = line["roofline"]
    r["achieved_aggregate"] = n * 152 * (1 << 20) / (0.027e-3) / 1e9
    r["frac_aggregate"] = r["achieved_aggregate"] / (n * 8000.0)
    if with_cpu:
        line["cpu_baseline"] = {"value": 1.6e8, "unit": "env-steps/s", "cores": 16, "kind": "port", "sample": "s"}
    return line


def test_multi_rank_line_without_cpu_baseline_is_rejected():
    check_line(_synthetic(8))
    check_line(_synthetic(1))
    with pytest.raises(AssertionError, match="cpu_baseline"):
        check_line(_synthetic(8, with_cpu=False))
    bad = _synthetic(8)
    bad["dist"]["world_size"] = 1  # n_gpus must be the process group's rank count
    with pytest.raises(AssertionError):
        check_line(bad)
    bad = _synthetic(8)
    del bad["roofline"]["achieved_aggregate"]
    with pytest.raises(AssertionError):
        check_line(bad)


@pytest.mark.skipif(not LINES5, reason="no recorded round-5 bench lines")
@pytest.mark.parametrize("path", LINES5, ids=[os.path.basename(p) for p in LINES5])
def test_recorded_round5_line(path):
    with open(path) as f:
        text = f.read().strip().splitlines()[-1]
    assert len(text) < 6144, len(text)  # the driver keeps ~8 KB of the output's tail
    d = json.loads(text)
    check_line(d)
    if "gpus_requested" in d["dist"]:  # round 6 on: the line names the --gpus it answers
        check_requested(d, d["dist"]["gpus_requested"])
    if "legs" in d and d["n_gpus"] == 1:
        for leg in ("rollout", "replay", "qnet_none", "qnet_self", "qnet_other", "hdqn_L0", "hdqn_self", "hdqn_other"):
            assert leg in d["legs"], leg


def test_compact_line_of_a_full_record_is_small():
    """bench.compact_line keeps every leg's headline figures under 6 KB, from the largest recorded
    round-4 record (all legs, VALU blocks and episode details)."""
    import sys

    sys.path.insert(0, ROOT)
    import bench

    full = json.loads(open(os.path.join(ROOT, "profiles", "r04", "bench_default_r04af.json")).read().strip()
                      .splitlines()[-1])
    full.setdefault("dist", {"backend": None, "world_size": 1})
    for leg in full["qnet_policy"]:
        leg.setdefault("reference_forwards_per_env_step", None)
    h = full["hdqn_policy"]
    for key in ("selfplay", "other_checkpoint"):
        h[key].setdefault("frac_useful", h[key].get("frac_useful_lower_bound"))
    out = json.dumps(bench.compact_line(full))
    assert len(out) < 6144, len(out)
    d = json.loads(out)
    for leg in ("rollout", "replay", "qnet_none", "qnet_self", "qnet_other", "hdqn_L0", "hdqn_self", "hdqn_other",
                "size_2p22"):
        assert leg in d["legs"], leg
    assert d["roofline"]["frac"] == full["roofline"]["frac"] and d["cpu_baseline"]["cores"] == 16


def check_requested(d, requested):
    """A line answers the run that asked for it: n_gpus (and the process group's rank count) equal the
    --gpus the driver passed, so an 8-GPU request cannot come back as a 1-GPU line."""
    check_line(d)
    assert d["n_gpus"] == requested, (d["n_gpus"], requested)
    gr = d["dist"].get("gpus_requested")
    assert gr is None or gr == requested, gr
    cr = d["dist"].get("collective_ranks")
    assert cr is None or cr == requested, cr


def test_line_for_another_gpu_count_is_rejected():
    check_requested(_synthetic(8), 8)
    check_requested(_synthetic(1), 1)
    with pytest.raises(AssertionError):
        check_requested(_synthetic(1), 8)  # the round-5 failure: --gpus 8 measured one GPU
    bad = _synthetic(8)
    bad["dist"]["collective_ranks"] = 4
    with pytest.raises(AssertionError):
        check_requested(bad, 8)


# ---- the self-launch (bench.py --gpus N > 1 without torchrun) -------------------------------------------

def _bench():
    import sys

    sys.path.insert(0, ROOT)
    import bench

    return bench


class _Args:
    def __init__(self, gpus, backend="nccl"):
        self.gpus, self.dist_backend = gpus, backend


def test_rank_environments_for_two_gpus():
    bench = _bench()
    envs = bench.rank_envs(_Args(2), {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 2, 29511)
    assert len(envs) == 2
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "2", "2")
        assert (e["MASTER_ADDR"], e["MASTER_PORT"]) == ("127.0.0.1", "29511")
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e[bench.SELF_LAUNCH_ENV] == "1"


def test_too_few_gpus_is_an_error_under_rccl_only():
    bench = _bench()
    with pytest.raises(SystemExit, match="only 1 GPU"):
        bench.rank_envs(_Args(2), {}, 1, 1)
    with pytest.raises(SystemExit, match="no GPU"):
        bench.rank_envs(_Args(2, "gloo"), {}, 0, 1)
    assert len(bench.rank_envs(_Args(8, "gloo"), {}, 1, 1)) == 8  # the gloo rehearsal shares one GPU


_SPAWN_PROBE = r"""
import json, os, sys
sys.path.insert(0, {root!r})
sys.argv = ["bench.py", "--gpus", "2", "--steps", "3"]
os.environ.pop("WORLD_SIZE", None)
os.environ["MG_BENCH_DEVICE_COUNT"] = "2"
import bench
calls = []
class P:
    def __init__(self, cmd, env):
        calls.append((cmd, {{k: env[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}}))
    def poll(self):
        return 0
    def terminate(self):
        pass
try:
    orig = bench.self_launch
    bench.self_launch = lambda a, argv: orig(a, argv, popen=P)
    bench.main()
except SystemExit as e:
    rc = e.code
maps = open("/proc/self/maps").read()
print(json.dumps({{"rc": rc, "calls": calls, "torch": "torch" in sys.modules,
                   "hip_loaded": "amdhip64" in maps, "ctypes": "ctypes" in sys.modules}}))
"""


def test_gpus_two_spawns_two_ranks_before_anything_touches_hip():
    """main() with --gpus 2 and no WORLD_SIZE starts two children of the same command with the
    rank environment, and the parent has neither imported torch nor mapped libamdhip64 by then."""
    import subprocess
    import sys

    out = subprocess.run([sys.executable, "-c", _SPAWN_PROBE.format(root=ROOT)], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["rc"] == 0 and not d["torch"] and not d["hip_loaded"], d
    assert len(d["calls"]) == 2
    for r, (cmd, env) in enumerate(d["calls"]):
        assert cmd[-4:] == ["--gpus", "2", "--steps", "3"] and cmd[-5].endswith("bench.py")
        assert env == {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1"}


def test_gpus_two_with_one_visible_gpu_exits_nonzero():
    import subprocess
    import sys

    env = dict(os.environ, MG_BENCH_DEVICE_COUNT="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                         text=True, timeout=120, env=env)
    assert out.returncode != 0 and "only 1 GPU" in out.stderr, (out.returncode, out.stderr[-500:])
    assert not out.stdout.strip()  # no bench line at all


def test_self_launch_relays_the_first_failure_and_stops_the_other_ranks(tmp_path):
    """Real child processes (a stand-in rank script): rank 1 fails at once, rank 0 would run for a
    minute; the launcher stops rank 0 and exits with rank 1's status."""
    bench = _bench()
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "open(os.path.join(%r, 'r' + os.environ['RANK']), 'w').write(os.environ['WORLD_SIZE'] + ' ' "
                      "+ os.environ['MASTER_PORT'])\n"
                      "if os.environ['RANK'] == '1':\n    sys.exit(3)\n"
                      "time.sleep(60)\n" % str(tmp_path))
    os.environ[bench.DEVICE_COUNT_ENV] = "2"
    try:
        import time

        t0 = time.time()
        rc = bench.self_launch(_Args(2), ["--gpus", "2"], script=str(script))
        assert rc == 3 and time.time() - t0 < 30
    finally:
        del os.environ[bench.DEVICE_COUNT_ENV]
    w0, p0 = (tmp_path / "r0").read_text().split()
    w1, p1 = (tmp_path / "r1").read_text().split()
    assert w0 == w1 == "2" and p0 == p1


def test_self_launch_all_ranks_green(tmp_path):
    bench = _bench()
    script = tmp_path / "rank.py"
    script.write_text("import os\nassert os.environ['WORLD_SIZE'] == '3'\n")
    os.environ[bench.DEVICE_COUNT_ENV] = "3"
    try:
        assert bench.self_launch(_Args(3), [], script=str(script)) == 0
    finally:
        del os.environ[bench.DEVICE_COUNT_ENV]


class _FakeHip:
    """Stands in for libamdhip64 in sync_spin: records the calls, reports `count` devices."""

    def __init__(self, count):
        self.count, self.calls = count, []

    def hipGetDeviceCount(self, ref):
        ref._obj.value = self.count
        self.calls.append(("count",))
        return 0

    def hipSetDevice(self, d):
        self.calls.append(("set", d.value))
        return 0 if d.value < self.count else 101

    def hipSetDeviceFlags(self, f):
        self.calls.append(("flags", f.value))
        return 0


@pytest.mark.parametrize("local,count,expect", [
    (None, 8, [("flags", 1)]),                                   # one process: the default device
    (3, 8, [("count",), ("set", 3), ("flags", 1)]),              # rank 3 of 8: its own device
    (5, 1, [("count",), ("set", 0), ("flags", 1)]),              # gloo rehearsal on one GPU
])
def test_sync_spin_sets_the_flags_on_the_ranks_own_device(monkeypatch, local, count, expect):
    import ctypes

    bench = _bench()
    fake = _FakeHip(count)
    monkeypatch.setattr(ctypes, "CDLL", lambda name: fake)
    assert bench.sync_spin(local) == 0
    assert fake.calls == expect


def test_replay_traffic_record_is_consistent():
    """profiles/pmc_replay.json (tools/profile_pmc_replay.py, FETCH_SIZE / WRITE_SIZE passes): the
    store's bytes are the sum of its three kernels', the calibration kernels read back the bytes
    they move (the gfx950 counter rule holds on that build), the row writes are exactly 88 B per
    kept transition, and bench.py attaches the figure only to the same workload shape."""
    path = os.path.join(ROOT, "profiles", "pmc_replay.json")
    if not os.path.exists(path):
        pytest.skip("no replay PMC record")
    with open(path) as f:
        d = json.load(f)
    k = d["per_launch"]
    total = sum(k[x]["hbm_bytes"] for x in ("scan", "group_scan", "write"))
    assert math.isclose(d["store_hbm_bytes"], total, rel_tol=1e-9)
    assert math.isclose(d["ratio_to_algorithmic"], total / d["store_algorithmic_bytes"], rel_tol=1e-9)
    assert abs(d["check_reset_write_ratio"] - 1) < 0.02 and abs(d["check_observe_read_ratio"] - 1) < 0.02
    w = d["workload"]
    assert abs(k["write"]["write_bytes"] / (88.0 * w["kept_per_store"]) - 1) < 0.01
    bench = _bench()
    assert bench.load_pmc_replay(w["envs"], w["T"]) == d["store_hbm_bytes"]
    assert bench.load_pmc_replay(w["envs"] * 2, w["T"]) is None
