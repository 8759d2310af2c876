"""Multi-GPU layout: one process per GPU, envs sharded in contiguous slices.

Envs never interact, so the step needs no exchange: rank r owns global envs
[offset, offset + count) and steps them alone (MergeVecEnv(env_offset=offset) keys its
Philox stream by the global index, so a sharded run draws exactly the unsharded actions).
The only collective is reducing completed-episode statistics after a rollout: by default
each rank contributes its shard's six totals (return sums of both players as f64 bits, and
episodes / collisions / ego-first arrivals / steps as int64 -- 48 bytes) to one all-gather
over RCCL (torch backend "nccl" on ROCm, xGMI between MI355X GPUs), and every rank reduces
the [world, 6] result in rank order (hdqn.py:330-346 and main.py:221-228 log exactly these
rates). `gather_episode_stats` gathers the per-env rows instead ([N/W, 4] int64 per rank),
for a caller that needs them. gloo carries the same calls on CPU tensors in tests.
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


PARTIAL_BYTES = 6 * 8  # one rank's contribution to gather_episode_summary


def partial_stats(ret_sum, counts):
    """This shard's totals as one [6] int64 tensor on the stats' device: return sums of ego and
    opponent (f64, bit-preserved), then episodes, collisions, ego-first arrivals, steps."""
    import torch

    r = ret_sum.sum(0).contiguous().view(torch.int64)
    c = counts.to(torch.int64).sum(0)
    return torch.cat([r, c])


def summarize_partials(parts):
    """[world, 6] partial totals (partial_stats rows) -> the summary dict, reduced in rank order."""
    import torch

    parts = parts.reshape(-1, 6).cpu()
    r = parts[:, :2].contiguous().view(torch.float64)
    c = parts[:, 2:].sum(0).tolist()
    r1 = r2 = 0.0
    for a, b in r.tolist():
        r1 += a
        r2 += b
    ep = max(c[0], 1)
    return {"completed": c[0], "mean_return_ego": r1 / ep, "mean_return_opp": r2 / ep,
            "collision_rate": c[1] / ep, "ego_first_rate": c[2] / ep, "mean_length": c[3] / ep}


def gather_episode_summary(ret_sum, counts, group=None):
    """All-gather every rank's 48-byte partial totals and reduce them: the global summary on
    every rank (the default collective of a sharded run)."""
    import torch
    import torch.distributed as dist

    part = partial_stats(ret_sum, counts)
    world = dist.get_world_size(group)
    if world == 1:
        return summarize_partials(part)
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world, 6), dtype=torch.int64, device=part.device)
        dist.all_gather_into_tensor(out, part, group=group)
    else:  # gloo: host tensors
        host = part.cpu()
        rows = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(rows, host, group=group)
        out = torch.stack(rows)
    return summarize_partials(out)


def summarize(ret_sum, counts):
    """Mean episode return / collision rate / ego-first rate / mean length (hdqn.py:330-346)
    of one process's per-env statistics."""
    return summarize_partials(partial_stats(ret_sum, counts))
