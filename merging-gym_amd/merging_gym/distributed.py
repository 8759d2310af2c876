"""Multi-GPU layout: one process per GPU, envs sharded in contiguous slices.

Envs never interact, so the step needs no exchange: rank r owns global envs
[offset, offset + count) and steps them alone (MergeVecEnv(env_offset=offset) keys its
Philox stream by the global index, so a sharded run draws exactly the unsharded actions).
The only collective is reducing completed-episode statistics after a rollout: by default
each rank contributes its shard's ten totals (four sums as f64 bits -- both players'
r_accumulate, main.py's winner-filtered ep_reward and the logged q_eval -- and episodes /
collisions / ego-first arrivals / steps / main.py wins / hdqn.py wins as int64: 80 bytes, summed on
the device by mg_stats_reduce in a fixed order) to one all-gather over RCCL (torch backend "nccl"
on ROCm, xGMI between MI355X GPUs), and every rank reduces the [world, 10] result in rank order
(the quantities hdqn.py:330-346 and main.py:221-228 log).
`gather_episode_stats` gathers the per-env rows instead ([N/W, 6] int64 per rank), for a caller
that needs them. gloo carries the same calls on CPU tensors in tests.
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


def pack_stats(returns, counts):
    """[n,R] f64 return sums + [n,C] i32 counts (C even) -> one [n, R + C/2] int64 tensor
    (bit-preserving)."""
    import torch

    return torch.cat([returns.contiguous().view(torch.int64), counts.contiguous().view(torch.int64)], dim=1)


def unpack_stats(packed, num_returns: int = 3):
    import torch

    returns = packed[:, :num_returns].contiguous().view(torch.float64)
    counts = packed[:, num_returns:].contiguous().view(torch.int32)
    return returns, counts


def gather_episode_stats(returns, counts, group=None):
    """All-gather every rank's per-env statistics (equal shard sizes). Returns the global
    (returns [N,R] f64, counts [N,C] i32) on every rank -- MergeVecEnv.returns / .counts."""
    import torch
    import torch.distributed as dist

    packed = pack_stats(returns, counts)
    if dist.get_world_size(group) == 1:
        return unpack_stats(packed, returns.shape[1])
    return unpack_stats(all_gather_rows(packed, group).to(packed.device), returns.shape[1])


def all_gather_rows(rows, group=None):
    """[k, w] int64 on every rank -> [world * k, w] in rank order: one all_gather_into_tensor of the
    device tensor over RCCL (backend "nccl"), or gloo's list form on host memory. Used at any
    world size (tests run it on a one-rank RCCL group: the device branch a sharded run takes)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * rows.shape[0], rows.shape[1]), dtype=rows.dtype, device=rows.device)
        dist.all_gather_into_tensor(out, rows.contiguous(), group=group)
        return out
    host = rows.cpu()
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host, group=group)
    return torch.cat(parts)


NUM_RETURNS, NUM_COUNTS = 3, 6
NUM_SUMS = NUM_RETURNS + 1  # the return sums and the q_eval sum (mg_stats_totals)
PARTIAL_BYTES = (NUM_SUMS + NUM_COUNTS) * 8  # one rank's contribution to gather_episode_summary: 80


def _records_of(returns, counts):
    """The [n, 8] f64 record tensor (mg_episode_stats, 64 B per env) that returns / counts are the
    MergeVecEnv views of, or None when they are separate tensors."""
    n = returns.shape[0]
    if (returns.dtype.itemsize != 8 or returns.stride() != (8, 1) or counts.stride() != (16, 1)
            or counts.data_ptr() != returns.data_ptr() + 32 or returns.storage_offset() % 8):
        return None
    base = returns.as_strided((n, 8), (8, 1))
    return base if base.untyped_storage().nbytes() >= (returns.storage_offset() + 8 * n) * 8 else None


# mg_stats_reduce's scratch (block partials) is allocated per call on the stream that runs the
# reduction: the caching allocator hands a freed block out again only in that stream's order, so
# reductions on two streams never share partials, and nothing is cached per stream (round 6: the
# per-(device, stream) dict of rounds 4-5 grew by one buffer for every new stream and could hand a
# recycled stream handle a buffer of a dead one).


def device_totals(records, events=None):
    """[n, 8] f64 device records (mg_episode_stats) -> their totals as one [10] int64 device tensor,
    summed by mg_stats_reduce in its fixed order (bit-reproducible; include/merging_hip.h). Two
    launches on the current stream, no synchronisation. events: a pair of timing events recorded
    right around the launches (the output and scratch are set up before the first)."""
    import ctypes

    import torch

    from . import _native

    n = records.shape[0]
    dev = records.device
    out = torch.empty(NUM_SUMS + NUM_COUNTS, dtype=torch.int64, device=dev)
    words = max(1, (_native.lib.mg_stats_reduce_scratch_bytes(n) + 7) // 8)
    stream = torch.cuda.current_stream(dev)
    with torch.cuda.stream(stream):
        scratch = torch.empty(words, dtype=torch.int64, device=dev)
    args = (ctypes.c_void_p(records.data_ptr()), n, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(scratch.data_ptr()),
            scratch.numel() * 8, ctypes.c_void_p(stream.cuda_stream))
    if events:
        events[0].record()
    rc = _native.lib.mg_stats_reduce(*args)
    if events:
        events[1].record()
    _native.check(rc, "mg_stats_reduce")
    return out


def partial_stats(returns, counts, q_eval=None, events=None):
    """This shard's totals as one [10] int64 tensor on the stats' device: the three return sums
    (r1_accumulate, r2_accumulate, main.py's filtered ep_reward; f64, bit-preserved), the q_eval sum
    (the record's own for MergeVecEnv's views; else the q_eval [n] tensor given, or 0), then
    episodes, collisions, ego-first arrivals, steps, main.py wins, hdqn.py wins. On the GPU, for
    MergeVecEnv's record views, one mg_stats_reduce (fixed summation order, ~64 B of reads per env);
    other tensors (gloo tests on CPU) are summed by torch. events: timing events for device_totals."""
    import torch

    if returns.shape[1] != NUM_RETURNS or counts.shape[1] != NUM_COUNTS:
        raise ValueError(f"need returns [n,{NUM_RETURNS}] and counts [n,{NUM_COUNTS}] (MergeVecEnv.returns / .counts)")
    if returns.is_cuda:
        rec = _records_of(returns, counts)
        if rec is not None:
            return device_totals(rec, events)
    rec = _records_of(returns, counts)
    if q_eval is None and rec is not None:
        q_eval = rec[:, 7]
    timed = events and returns.is_cuda
    if timed:
        events[0].record()
    r = returns.sum(0)
    q = q_eval.sum().reshape(1).to(r) if q_eval is not None else torch.zeros(1, dtype=r.dtype, device=r.device)
    c = counts.to(torch.int64).sum(0)
    out = torch.cat([torch.cat([r, q]).contiguous().view(torch.int64), c])
    if timed:
        events[1].record()
    return out


def summarize_partials(parts):
    """[world, 10] partial totals (partial_stats rows) -> the summary dict, reduced in rank order:
    the quantities the reference's scripts log per episode, as rates / means over all completed
    episodes -- hdqn.py:330-346 (reward = r1_accumulate, collision_rate, win_rate on the terminal
    observation) and main.py:221-228 (reward = the winner-filtered ep_reward, win on the
    pre-terminal observation) -- plus the ego-first rate (winner == 1) and the mean length."""
    import torch

    w = NUM_SUMS + NUM_COUNTS
    parts = parts.reshape(-1, w).cpu()
    r = parts[:, :NUM_SUMS].contiguous().view(torch.float64)
    c = parts[:, NUM_SUMS:].sum(0).tolist()
    sums = [0.0] * NUM_SUMS
    for row in r.tolist():
        sums = [a + b for a, b in zip(sums, row)]
    ep = max(c[0], 1)
    return {"completed": c[0], "mean_return_ego": sums[0] / ep, "mean_return_opp": sums[1] / ep,
            "mean_ep_reward_main": sums[2] / ep, "collision_rate": c[1] / ep, "ego_first_rate": c[2] / ep,
            "win_rate_main": c[4] / ep, "win_rate_hdqn": c[5] / ep, "mean_length": c[3] / ep,
            "mean_q_eval": sums[3] / ep}


def gather_episode_summary(returns, counts, group=None, timings=None):
    """All-gather every rank's 80-byte partial totals and reduce them: the global summary on
    every rank (the default collective of a sharded run). timings (a dict, optional) receives
    "reduce_ms" (this shard's reduction to its partial totals: HIP events right around its two
    launches on the GPU), "reduce_wall_ms" (the same call on the host clock, synchronised: Python and launch
    overheads included) and "allgather_ms" (the collective alone; None without one, world size 1)."""
    import time

    import torch
    import torch.distributed as dist

    # synchronise only to time the two steps apart: otherwise stream order carries the reduction
    # into the collective, and summarize_partials' host copy waits for both
    sync = ((lambda: torch.cuda.synchronize(returns.device)) if returns.is_cuda and timings is not None
            else (lambda: None))  # noqa: E731
    events = None
    if timings is not None and returns.is_cuda:
        events = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    sync()
    t0 = time.perf_counter()
    part = partial_stats(returns, counts, events=events)
    sync()
    t1 = time.perf_counter()
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if timings is not None:
        timings["reduce_wall_ms"] = (t1 - t0) * 1e3
        timings["reduce_ms"] = events[0].elapsed_time(events[1]) if events else timings["reduce_wall_ms"]
        timings["allgather_ms"] = None
    if world == 1:
        return summarize_partials(part)
    out = all_gather_rows(part.reshape(1, -1), group)
    sync()
    if timings is not None:
        timings["allgather_ms"] = (time.perf_counter() - t1) * 1e3
    return summarize_partials(out)


def summarize(returns, counts):
    """The summary (summarize_partials) of one process's per-env statistics."""
    return summarize_partials(partial_stats(returns, counts))
