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
    ret = torch.randn((n_per_rank, 2), generator=g, dtype=torch.float64)
    cnt = torch.randint(0, 100, (n_per_rank, 4), generator=g, dtype=torch.int32)
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
        exp_ret.append(torch.randn((n, 2), generator=g, dtype=torch.float64))
        exp_cnt.append(torch.randint(0, 100, (n, 4), generator=g, dtype=torch.int32))
    assert torch.equal(res["ret"], torch.cat(exp_ret))  # bit-exact through the int64 packing
    assert torch.equal(res["cnt"], torch.cat(exp_cnt))
    s = summarize(res["ret"], res["cnt"])
    assert s["completed"] == int(torch.cat(exp_cnt)[:, 0].sum())
