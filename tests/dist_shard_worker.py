"""One rank of the sharded-run GPU test (tests/test_gpu_distributed.py), launched by
torch.distributed.run with the gloo backend; every rank steps its own contiguous shard of the
global batch on cuda:0 (the test box has one GPU) exactly as bench.py's ranks do on their own
GPUs, then the statistics are gathered -- the 80-byte summary (the default collective) and the
per-env rows (opt-in) -- and rank 0 saves both with its shard bookkeeping.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        tests/dist_shard_worker.py GLOBAL_ENVS STEPS SEED OUT
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))


def main():
    n_global, steps, seed, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import torch
    import torch.distributed as dist

    from merging_gym import MergeVecEnv
    from merging_gym.distributed import gather_episode_stats, gather_episode_summary, shard

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    offset, count = shard(n_global, world, rank)
    env = MergeVecEnv(count, device="cuda:0", env_offset=offset)
    # the bench's mix: single steps, then fused rollouts continuing the same Philox stream
    for k in range(steps // 2):
        env.step_random(seed, step_idx=k)
    k = steps // 2
    while k < steps:
        T = min(16, steps - k)
        env.rollout_random(T, seed, first_step=k)
        k += T
    torch.cuda.synchronize()
    summary = gather_episode_summary(env.returns, env.counts)
    returns, counts = gather_episode_stats(env.returns, env.counts)
    p1 = [torch.empty(count, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(p1, env.p1.cpu())
    if rank == 0:
        torch.save({"summary": summary, "returns": returns.cpu(), "counts": counts.cpu(),
                    "p1": torch.cat(p1), "world": world}, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
