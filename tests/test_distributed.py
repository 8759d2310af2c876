"""Multi-process path on CPU (gloo, world size 2): sharding and the episode-statistics gather."""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from merging_gym.distributed import gather_episode_stats, shard, summarize


def test_shard_covers_every_env_once():
    for n in (1, 7, 4096, 1 << 20, 8 * (1 << 20) + 3):
        for w in (1, 2, 3, 8):
            spans = [shard(n, w, r) for r in range(w)]
            assert spans[0][0] == 0
            for (o, c), (o2, _) in zip(spans, spans[1:]):
                assert o + c == o2
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _worker(rank, world, port, n_per_rank, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(rank)
    ret = torch.randn((n_per_rank, 3), generator=g, dtype=torch.float64)
    cnt = torch.randint(0, 100, (n_per_rank, 6), generator=g, dtype=torch.int32)
    all_ret, all_cnt = gather_episode_stats(ret, cnt)
    if rank == 0:
        torch.save({"ret": all_ret, "cnt": all_cnt}, out_path)
    dist.destroy_process_group()


def test_gather_episode_stats_gloo(tmp_path):
    world, n = 2, 1000
    out = str(tmp_path / "g.pt")
    port = 29500 + (os.getpid() % 1000)
    mp.start_processes(_worker, args=(world, port, n, out), nprocs=world, start_method="spawn")
    res = torch.load(out, weights_only=True)
    exp_ret, exp_cnt = [], []
    for r in range(world):
        g = torch.Generator().manual_seed(r)
        exp_ret.append(torch.randn((n, 3), generator=g, dtype=torch.float64))
        exp_cnt.append(torch.randint(0, 100, (n, 6), generator=g, dtype=torch.int32))
    assert torch.equal(res["ret"], torch.cat(exp_ret))  # bit-exact through the int64 packing
    assert torch.equal(res["cnt"], torch.cat(exp_cnt))
    s = summarize(res["ret"], res["cnt"])
    c = torch.cat(exp_cnt).to(torch.int64).sum(0)
    assert s["completed"] == int(c[0])
    assert s["win_rate_main"] == int(c[4]) / int(c[0]) and s["win_rate_hdqn"] == int(c[5]) / int(c[0])


def _summary_worker(rank, world, port, n_per_rank, out_path):
    from merging_gym.distributed import PARTIAL_BYTES, gather_episode_summary, partial_stats

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(10 + rank)
    ret = torch.randn((n_per_rank, 3), generator=g, dtype=torch.float64)
    cnt = torch.randint(0, 100, (n_per_rank, 6), generator=g, dtype=torch.int32)
    assert partial_stats(ret, cnt).numel() * 8 == PARTIAL_BYTES
    s = gather_episode_summary(ret, cnt)
    torch.save(s, out_path + f".{rank}")
    dist.destroy_process_group()


def test_gather_episode_summary_gloo(tmp_path):
    """The default collective: 80 bytes per rank, every rank gets the global summary, equal to
    summarizing the concatenated per-env statistics (counts exactly, returns to fp64 rounding)."""
    world, n = 2, 1500
    out = str(tmp_path / "s")
    port = 30500 + (os.getpid() % 1000)
    mp.start_processes(_summary_worker, args=(world, port, n, out), nprocs=world, start_method="spawn")
    got = [torch.load(out + f".{r}", weights_only=True) for r in range(world)]
    assert got[0] == got[1]
    rets, cnts = [], []
    for r in range(world):
        g = torch.Generator().manual_seed(10 + r)
        rets.append(torch.randn((n, 3), generator=g, dtype=torch.float64))
        cnts.append(torch.randint(0, 100, (n, 6), generator=g, dtype=torch.int32))
    exp = summarize(torch.cat(rets), torch.cat(cnts))
    for k, v in exp.items():
        if k == "completed":
            assert got[0][k] == v
        else:
            assert abs(got[0][k] - v) <= 1e-12 * max(1.0, abs(v)), k
