"""The sharded multi-process path on the GPU: two fresh processes,
launched with torch.distributed.run (gloo; both ranks on cuda:0 of the one-GPU test box), each
step a MergeVecEnv(env_offset=...) shard for 200 Philox steps and gather the statistics. The
result must equal one unsharded run of the whole batch: per-env statistics and positions bit
for bit (Philox is keyed by the global env index, envs never interact), the 80-byte-per-rank
summary to fp64 summation order. The reference has no parallelism (its envs are independent,
merging_env.py:138-195); this pins the build's own sharding."""

import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_shards_equal_unsharded_run(tmp_path):
    import torch

    from merging_gym import MergeVecEnv
    from merging_gym.distributed import summarize

    n, steps, seed = 6002, 200, 31
    out = str(tmp_path / "rank0.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_shard_worker.py"), str(n), str(steps), str(seed), out]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    run = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert run.returncode == 0, run.stderr[-3000:]
    got = torch.load(out, weights_only=True)
    assert got["world"] == 2

    full = MergeVecEnv(n, device="cuda:0")
    for k in range(steps // 2):
        full.step_random(seed, step_idx=k)
    k = steps // 2
    while k < steps:
        T = min(16, steps - k)
        full.rollout_random(T, seed, first_step=k)
        k += T
    assert torch.equal(got["counts"], full.counts.cpu())
    assert torch.equal(got["returns"], full.returns.cpu())
    assert torch.equal(got["p1"], full.p1.cpu())
    exp = summarize(full.returns, full.counts)
    assert exp["completed"] > 0 and got["summary"]["completed"] == exp["completed"]
    for key, v in exp.items():
        assert abs(got["summary"][key] - v) <= 1e-12 * max(1.0, abs(v)), key


def test_rccl_device_gather(tmp_path):
    """The RCCL branch of the statistics gather (distributed.all_gather_rows, backend "nccl"):
    all_gather_into_tensor of the 80-byte partial totals and of the per-env rows, on device
    tensors, in a one-rank RCCL group on the test box's one GPU (RCCL refuses two ranks on one
    device; the 8-GPU runs are the driver's). What comes back must equal what went in, bit for bit."""
    import torch

    out = str(tmp_path / "rccl.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_rccl_worker.py"), "4099", "160", "17", out]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    run = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert run.returncode == 0, run.stderr[-3000:]
    got = torch.load(out, weights_only=True)
    assert got["got_part"].shape == (1, 10) and torch.equal(got["got_part"][0], got["part"])
    assert torch.equal(got["got_rows"], got["rows"]) and got["rows"].shape == (4099, 6)
    assert int(got["part"][4]) > 0  # episodes completed inside the run (after the four f64 sums)
