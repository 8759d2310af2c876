"""One-rank RCCL run for tests/test_gpu_distributed.py::test_rccl_device_gather: launched by
torch.distributed.run with the "nccl" backend (RCCL on ROCm) on the test box's one GPU, it steps a
MergeVecEnv and runs distributed.all_gather_rows -- the all_gather_into_tensor device branch every
rank of a sharded run takes for the 80-byte episode summary and the per-env rows -- on device
tensors, then saves what came back beside the local values.

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \\
        tests/dist_rccl_worker.py ENVS STEPS SEED OUT
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))


def main():
    n, steps, seed, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import torch
    import torch.distributed as dist

    from merging_gym import MergeVecEnv
    from merging_gym.distributed import all_gather_rows, pack_stats, partial_stats

    torch.cuda.set_device(0)
    dist.init_process_group("nccl")
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    env = MergeVecEnv(n, device="cuda:0")
    k = 0
    while k < steps:
        env.rollout_random(16, seed, first_step=k)
        k += 16
    part = partial_stats(env.returns, env.counts)
    got_part = all_gather_rows(part.reshape(1, -1))
    rows = pack_stats(env.returns, env.counts)
    got_rows = all_gather_rows(rows)
    torch.cuda.synchronize()
    assert got_part.is_cuda and got_rows.is_cuda
    torch.save({"part": part.cpu(), "got_part": got_part.cpu(), "rows": rows.cpu(), "got_rows": got_rows.cpu()}, out)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
