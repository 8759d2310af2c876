"""Multi-GPU layout: one process per GPU, envs sharded in contiguous slices.

Envs never interact, so the step needs no exchange: rank r owns global envs
[offset, offset + count) and steps them alone (MergeVecEnv(env_offset=offset) keys its
Philox stream by the global index, so a sharded run draws exactly the unsharded actions).
The only collective is gathering completed-episode statistics after a rollout -- one
all-gather over RCCL (torch backend "nccl" on ROCm, xGMI between MI355X GPUs), or gloo
for CPU tensors in tests.
"""

from __future__ import annotations


def shard(global_envs: int, world: int, rank: int):
    """(offset, count) of rank's contiguous slice; the first `global_envs % world` ranks get one more."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(int(global_envs), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def pack_stats(ret_sum, counts):
    """[n,2] f64 returns + [n,4] i32 counts -> one [n,4] int64 tensor (bit-preserving)."""
    import torch

    return torch.cat([ret_sum.contiguous().view(torch.int64), counts.contiguous().view(torch.int64)], dim=1)


def unpack_stats(packed):
    import torch

    ret_sum = packed[:, :2].contiguous().view(torch.float64)
    counts = packed[:, 2:].contiguous().view(torch.int32)
    return ret_sum, counts


def gather_episode_stats(ret_sum, counts, group=None):
    """All-gather every rank's per-env statistics (equal shard sizes). Returns the global
    (ret_sum [N,2] f64, counts [N,4] i32) on every rank."""
    import torch
    import torch.distributed as dist

    packed = pack_stats(ret_sum, counts)
    world = dist.get_world_size(group)
    if world == 1:
        return unpack_stats(packed)
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * packed.shape[0], packed.shape[1]), dtype=packed.dtype,
                          device=packed.device)
        dist.all_gather_into_tensor(out, packed, group=group)
    else:  # gloo: list form, on host memory
        host = packed.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        out = torch.cat(parts).to(packed.device)
    return unpack_stats(out)


def summarize(ret_sum, counts):
    """Mean episode return / collision rate / ego-first rate / mean length (hdqn.py:330-346)."""
    import torch

    c = counts.to(torch.int64).sum(0).tolist()
    r = ret_sum.sum(0).tolist()
    ep = max(c[0], 1)
    return {"completed": c[0], "mean_return_ego": r[0] / ep, "mean_return_opp": r[1] / ep,
            "collision_rate": c[1] / ep, "ego_first_rate": c[2] / ep, "mean_length": c[3] / ep}
