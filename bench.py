"""Benchmark: env-steps/s of the batched MergingEnv step on MI355X (BASELINE.json config 3/4).

    python bench.py [--gpus N --steps K --warmup W --envs E]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU)

With --gpus N > 1 and no launcher (no WORLD_SIZE in the environment) bench.py starts the N one-GPU
ranks itself as child processes, before anything in the parent touches HIP, and exits with the
worst rank's status; fewer visible GPUs than N is an error under RCCL. Every rank checks that its
process group (and one all-reduce over it) has exactly N ranks.

A step = one launch of mg_step_random over this rank's 2^20 envs: Philox actions for both
players drawn on the device, the full reference step (merging_env.py:138-195), autoreset,
episode statistics. Envs are sharded across ranks (rank r owns global envs [r E, (r+1) E),
Philox keyed by the global index), with no collective inside the timed loop; after it, one
RCCL all-gather of each rank's 80-byte statistics totals (timed separately).

Before the W warm-up steps the batch is burned in (--burn-in-launches untimed one-step launches
of the same kernel, optionally preceded by --burn-in steps of fused rollouts) so the timed window
sees the steady state: envs finishing every step, autoreset, final observations and statistics
writes. The burn-in runs the step kernel itself by default: after a rollout burn-in (VALU-heavy)
plus 48 step launches, a 20-launch window measured 26.2-26.4 us per launch against 25.1-25.6
after 1,072 step launches, the env state at the window being the same (tools/gpu_burnin_ab.sh,
profiles/r02/ab/burnin/).
The K timed launches are host launches (the host enqueues one in ~4 us, the kernel takes ~25),
or a HIP-graph replay with --graph 1.

Rank 0 prints ONE JSON line: value = env-steps/s over all ranks (max-over-ranks time),
roofline = algorithmic bytes per launch / mean kernel time (HIP events on the launch stream)
against the 8 TB/s HBM3E peak, size_2p22 = the same kernel at 2^22 envs (past the 256 MiB
Infinity Cache, N = 1 only), cpu_baseline = the CPU restatements on the host cores (rank 0, at every
world size, after the GPU legs; the other ranks wait at the closing barrier).
"""

from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))

# Algorithmic bytes per env-step of mg_step_random (DESIGN.md "Roofline"):
#   read  p1 v1 p2 v2 ret1 ret2 (6 x f64) + tf (u16)                      = 50
#   write the same state 50 + obs 10 x f32 40 + rew 2 x f32 8 + done 1 + coll 1
#         + actions 2 x i8 2                                            = 102
# (final_obs / episode-statistics writes happen only for the ~0.5 % of envs that finish
#  in a step and are not counted.)
BYTES_PER_ENV_STEP = 152
# SURVEY.md 8(d)'s count for device-drawn actions: fp32 returns (8 B, not 16, each way), no
# action write-back, separate done / winner bytes: 136 B. The 16-B fp64-return premium is this
# build's choice (r{1,2}_accumulate stay the reference's fp64 sums);
# roofline.frac_8d reports the line against 136 B.
BYTES_PER_ENV_STEP_8D = 136
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
KERNEL_NAME = "step_kernel<1, false>"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs", type=int, default=1 << 20, help="envs per GPU")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank) or gloo (multi-rank rehearsal, ranks may share a GPU)")
    ap.add_argument("--burn-in", type=int, default=0,
                    help="untimed steps as 16-step fused rollouts before the burn-in launches (faster "
                         "to run, but the window after them starts in the rollout kernel's regime)")
    ap.add_argument("--stagger", type=int, default=256,
                    help="before the burn-in, S one-step launches each followed by a reset of the envs with "
                         "index % S == j: first-episode phases spread over S steps instead of all envs "
                         "starting together (tools/size2_probe.py: the finishing rate, and with it the "
                         "per-launch time past the Infinity Cache, otherwise oscillates for thousands of steps)")
    ap.add_argument("--burn-in-launches", type=int, default=1072,
                    help="untimed one-step launches before the warm-up: the steady state (episodes "
                         "need >= 106 steps, the mean is ~210) reached by the timed kernel itself")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: replay the K timed launches from a HIP graph captured before the window "
                         "(at K = 20 host launches measured 1.04x event time on the wall, the graph's "
                         "first replay 1.04-1.07x: tools/window_probe.py)")
    ap.add_argument("--sync-spin", type=int, default=1,
                    help="1: hipDeviceScheduleSpin (synchronize spins instead of yielding the host thread)")
    ap.add_argument("--size2-envs", type=int, default=1 << 22,
                    help="envs of the post-Infinity-Cache leg (N = 1 only); 0 disables it")
    ap.add_argument("--size2-steps", type=int, default=100)
    ap.add_argument("--size2-when", choices=("first", "last"), default="last",
                    help="run the 2^22 leg after every other leg (default) or right after the step leg")
    ap.add_argument("--size2-prealloc", action="store_true",
                    help="allocate the 2^22 leg's env before the other legs, whenever it runs (A/B of where "
                         "its memory lands)")
    ap.add_argument("--gather", choices=("summary", "per-env"), default="summary",
                    help="statistics collective: 80-byte totals per rank, or every env's row")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="per CPU-baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-events", action="store_true", help="skip per-launch HIP events")
    ap.add_argument("--event-every", type=int, default=8,
                    help="time every k-th launch with dispatch-recorded events (arming costs host time)")
    ap.add_argument("--rollout-steps", type=int, default=16,
                    help="T of the fused rollout leg (mg_rollout_random); 0 disables it")
    ap.add_argument("--rollout-launches", type=int, default=200,
                    help="timed launches of the rollout leg (after --leg-warmup untimed ones)")
    ap.add_argument("--leg-warmup", type=int, default=60,
                    help="untimed launches before each rollout / Q-net / h-DQN leg: a compute-heavy kernel "
                         "after the memory-bound step leg first runs through a clock transient "
                         "(tools/rollout_sustain.py); 10 left part of it in the window: rollout 11.1 vs "
                         "10.5 us per step, config-5 ego 51.4-52.1 vs 49.6-49.7 (tools/gpu_legwarm_ab.sh)")
    ap.add_argument("--replay-stores", type=int, default=20,
                    help="timed mg_replay_store calls of the replay-memory leg; 0 disables it")
    ap.add_argument("--qnet-launches", type=int, default=40,
                    help="launches of the config-5 leg (fused epsilon-greedy DQN rollout); 0 disables it")
    return ap.parse_args()


def cpu_baseline(seconds: float, envs: int):
    """The CPU restatements on the host cores (oracle/cpu_baselines.py, run as a child process
    that never touches the GPU): the C oracle on every core of the affinity mask, the NumPy
    restatement at the GPU batch size on one core and one process per core, the scalar list-API
    env one process per core. `value` is the fastest all-core figure; all are reported."""
    import subprocess

    cmd = [sys.executable, os.path.join(ROOT, "oracle", "cpu_baselines.py"), "--seconds", str(seconds),
           "--envs", str(envs)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return {"error": out.stderr[-500:]}
    d = json.loads(out.stdout.strip().splitlines()[-1])
    legs = {"c_oracle": d["c_oracle"], "numpy_all_cores": d["numpy"].get("all_cores", d["numpy"]["one_core"]),
            "scalar_per_core": d["scalar"]}
    best = max(legs, key=lambda k: legs[k]["value"])
    c = d["cores"]
    cores = legs[best].get("threads", legs[best].get("procs"))
    return {"value": legs[best]["value"], "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{best}: {legs[best]['sample']}; host affinity {c['affinity']} cores, cgroup CPU quota "
                      f"{c['cgroup_quota']}",
            "host_cores": c,
            "legs": {"c_oracle_all_affinity_threads": d["c_oracle"],
                     "numpy_2p20_one_core": d["numpy"]["one_core"],
                     "numpy_2p20_all_cores": d["numpy"].get("all_cores"),
                     "scalar_list_api_per_core": d["scalar"]},
            "workload": "Philox actions for both players, autoreset (scalar: host random actions, reset "
                        "on done); oracle/merge_oracle.c, oracle/merge_numpy.py, oracle/merge_oracle.py"}


def load_pmc(envs: int, kernel: str = "step"):
    """HBM traffic per launch from the committed rocprofv3 PMC summary (profiles/), if any: the
    step kernel's, or with kernel="rollout" the 16-step random rollout's."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        row = d.get("by_envs", {}).get(str(envs))
        if row is None and int(d.get("envs", -1)) == envs:
            row = d
        if row is not None and kernel != "step":
            row = row.get(kernel)
        return None if row is None else row.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def load_pmc_replay(envs: int, T: int):
    """HBM bytes of one replay store (the scan, group-scan and write kernels) from the committed
    rocprofv3 PMC summary (tools/profile_pmc_replay.py -> profiles/pmc_replay.json), if it was
    measured on this workload shape."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_replay.json")) as f:
            d = json.load(f)
        w = d["workload"]
        return d["store_hbm_bytes"] if (w["envs"], w["T"]) == (envs, T) else None
    except (OSError, ValueError, KeyError):
        return None


def load_valu():
    """Per-kernel VALU-issue figures from the committed rocprofv3 summary (tools/pmc_valu.sh +
    tools/valu_summary.py -> profiles/valu_busy.json): VALUBusy = VALU issue cycles of every SIMD
    over the kernel's GPU time, the ceiling of a kernel whose arithmetic, not its bytes, sets
    the pace."""
    try:
        with open(os.path.join(ROOT, "profiles", "valu_busy.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    out = {}
    for k, v in d.items():
        if not isinstance(v, dict) or "insts_per_64_env_steps" not in v:
            continue  # the file's notes and comparisons ("source", "round4_valu_before_after")
        ins = v.get("insts_per_64_env_steps", {})
        out[k] = {"valu_busy_frac": v.get("VALUBusy", 0.0) / 100.0,
                  "valu_insts_per_lane_step": ins.get("valu", 0.0),  # wave instructions per 64 env-steps
                  "fp64_share_of_valu": v.get("fp64_share_of_valu"),
                  "source": "profiles/valu_busy.json (rocprofv3 --pmc VALUBusy + SQ_INSTS_VALU*, 2^20 envs)"}
        if "mfma_busy_frac" in v:  # rocprofv3's MfmaUtil: matrix-pipe busy cycles / (GPU cycles x SIMDs)
            out[k]["mfma_busy_frac"] = v["mfma_busy_frac"]
            out[k]["mfma_bf16_flops_per_env_step"] = v.get("mfma_bf16_flops_per_env_step")
            out[k]["lds_bank_conflict_frac"] = v.get("lds_bank_conflict_frac")
            out[k]["source"] += " + MfmaUtil, SQ_INSTS_VALU_MFMA_MOPS_BF16, SQ_LDS_BANK_CONFLICT"
    return out


def stagger(env, S: int, seed: int, first_step: int, torch) -> int:
    """S untimed one-step launches, after launch j a reset of the envs with index % S == j; returns
    the next step index (see --stagger)."""
    if S <= 0:
        return first_step
    phase = torch.arange(env.num_envs, device=env.device) % S
    for j in range(S):
        env.step_random(seed, step_idx=first_step + j)
        env.reset(phase == j)
    return first_step + S


def burn_in(env, steps: int, seed: int, first_step: int) -> int:
    """Untimed fused rollouts until `steps` env-steps have passed; returns the next step index."""
    k = first_step
    while k - first_step < steps:
        T = min(16, steps - (k - first_step))
        env.rollout_random(T, seed, first_step=k, final_observation=False, won_mask=False)
        k += T
    return k


def capture_steps(step, first: int, count: int, torch):
    """The `count` launches step(first), ..., step(first + count - 1) captured into one HIP graph
    (torch.cuda.CUDAGraph over torch's capture stream, which MergeVecEnv launches on); replaying
    it runs exactly those launches. Capture executes nothing."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(first, first + count):
            step(k)
    return g


def size2_env(args, torch):
    from merging_gym import MergeVecEnv

    return MergeVecEnv(args.size2_envs, device=torch.device("cuda", torch.cuda.current_device()), autoreset=True,
                       final_observation=True, episode_stats=True)


def size2_leg(args, torch, env=None):
    """The step kernel past the Infinity Cache: --size2-envs envs (638 MB of state and outputs per
    step at 2^22 > 256 MiB), burned in to the steady state, --size2-steps launches timed with HIP
    events on the launch stream. env: one allocated earlier (--size2-prealloc)."""
    E = args.size2_envs
    prealloc = env is not None
    if env is None:
        env = size2_env(args, torch)
    k = burn_in(env, args.burn_in, args.seed, stagger(env, args.stagger, args.seed, 0, torch))
    env.clear_statistics()  # ahead of the burn-in launches (see the main leg)
    for _ in range(max(5, args.burn_in_launches)):
        env.step_random(args.seed, step_idx=k)
        k += 1
    # One event pair per window of 20 launches, averaged over all of them, with the host's enqueue
    # time of each window beside it. Rounds 2-3 saw the first window slow (one ~7 ms stall in r03e;
    # 109 vs 98-103 us per launch in the r03 driver run) and timed a rehearsal window first. The
    # causes, measured in round 4 ("The 2^22 first window"): (1) per-launch
    # times follow the number of envs finishing in the launch (~1 us per 1,000 finishes past the
    # Infinity Cache, tools/size2_probe.py), which oscillates for thousands of steps when every env
    # starts its first episode together -- --stagger spreads those starts; (2) the statistics clear
    # (any form of it) is followed by ~200 launches of up to +6 % (tools/size2_probe2.py) -- it now
    # runs before the burn-in launches; (3) a synchronize before the first window leaves the GPU idle
    # while the host resumes (386 us in the r04f trace) -- the windows follow the burn-in launches in
    # the same queue, so the events bracket queued kernel work only.
    win = 20
    nwin = max(1, args.size2_steps // win)
    gc.disable()
    rehearsal_us = None
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(nwin + 1)]
    host = []
    evs[0].record()  # behind the burn-in launches still in the queue: no idle gap before the window
    for w in range(nwin):
        h0 = time.perf_counter()
        for j in range(win):
            env.step_random(args.seed, step_idx=k + w * win + j)
        evs[w + 1].record()
        host.append(round((time.perf_counter() - h0) * 1e3, 3))
    torch.cuda.synchronize()
    gc.enable()
    win_us = [round(evs[w].elapsed_time(evs[w + 1]) / win * 1e3, 1) for w in range(nwin)]
    kernel_ms = evs[0].elapsed_time(evs[-1]) / (nwin * win)
    arena = env._arena.data_ptr() if env._arena is not None else env.p1.data_ptr()
    achieved = BYTES_PER_ENV_STEP * E / (kernel_ms * 1e-3) / 1e9
    frac_8d = BYTES_PER_ENV_STEP_8D * E / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
    completed = int(env.counts[:, 0].sum())
    del env
    torch.cuda.empty_cache()
    return {"envs": E, "steps": nwin * win, "burn_in_steps": args.burn_in + max(5, args.burn_in_launches),
            "when": args.size2_when, "preallocated": prealloc,
            "kernel_ms": kernel_ms, "window_us": win_us, "window_host_enqueue_ms": host,
            "rehearsal_window_us": rehearsal_us, "arena_addr": hex(arena),
            "value": E / (kernel_ms * 1e-3), "unit": "env-steps/s", "achieved": achieved, "peak": HBM_PEAK_GBPS,
            "unit_bw": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "frac_8d": frac_8d, "traffic": load_pmc(E),
            "episodes_completed": completed, "episodes_counted_since": "the clear before the burn-in launches"}


def rollout_leg(env, args, world, dist, torch):
    """The fused T-step kernel (mg_rollout_random): same per-step work and outputs, the env's
    state read and written once per launch. Algorithmic bytes per env-step:
    52 (obs 40 + rew 8 + done 1 + coll 1 + actions 2) + 100 / T (state in and out)."""
    T, L, E = args.rollout_steps, args.rollout_launches, env.num_envs
    k = 10_000_000
    for _ in range(max(1, args.leg_warmup)):
        env.rollout_random(T, args.seed, first_step=k, final_observation=False, won_mask=False)
        k += T
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    ev0.record()
    for j in range(L):
        env.rollout_random(T, args.seed, first_step=k, final_observation=False, won_mask=False)
        k += T
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / L
    t = torch.tensor([elapsed], dtype=torch.float64,
                     device="cpu" if args.dist_backend != "nccl" else env.device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    bytes_per_env_step = 52.0 + 100.0 / T
    achieved = bytes_per_env_step * E * T / (kernel_ms * 1e-3) / 1e9
    return {"kernel": "rollout_kernel", "steps_per_launch": T, "launches": L,
            "value": world * E * T * L / float(t[0]), "unit": "env-steps/s",
            "ms_per_step": float(t[0]) / (L * T) * 1e3, "kernel_ms_mean": kernel_ms,
            "bytes_per_env_step": bytes_per_env_step, "achieved": achieved, "peak": HBM_PEAK_GBPS,
            "unit_bw": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
            "traffic": load_pmc(E, "rollout") if T == 16 else None,
            "traffic_note": "HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, profiles/pmc_traffic.json); "
                            "the algorithmic bytes leave out the statistics records (32 B read per env per "
                            "launch)"}


QNET_USEFUL_FLOP = 2 * (10 * 200 + 200 * 100 + 100 * 5)      # one Net forward, main.py:30-47
# The reference evaluates a net only on choose_action's / choose_goal's greedy branch
# (np.random.randn() <= EPISILO: P = Phi(0.7), main.py:105, hdqn.py:86, :170) plus once per finished
# episode for the logged q_eval (main.py:221, hdqn.py:330). Round 5: useful FLOPs count exactly those
# forwards (the kernels since round 5 compute only them, and the counts below come from the leg's
# own episodes and goal breaks); rounds 1-4 counted one forward per net per env-step.


def p_greedy():
    from merging_gym.policy import greedy_threshold

    return greedy_threshold() / 2.0 ** 32
# MFMAs issued per 64-env forward (ABI 19). The 16x16 forward (self-play / other-net opponents,
# h-DQN): layer 1 14 x 32x32x16, layers 2 and 3 (196 + 16) x 16x16x32. The 32x32 forward (config 5
# without a net opponent): 132 x 32x32x16 (padded tiles, all-padding k-blocks skipped).
QNET_MFMA32_FLOP = 14 * 32 * 32 * 16 * 2
QNET_MFMA16_FLOP = 212 * 16 * 16 * 32 * 2
QNET_MFMA_FLOP = (QNET_MFMA32_FLOP + QNET_MFMA16_FLOP) // 64  # per env, 16x16 forward
QNET32_MFMA_FLOP = 132 * 32 * 32 * 16 * 2 // 64              # per env, 32x32 forward
MFMA_BF16_PEAK_TFLOPS = 2500.0                                 # MI355X dense bf16
# what the matrix pipe sustains on all 1,024 SIMDs, one wave per SIMD, nothing else running
# (register operands, tools/micro/qfwd_probe.hip, profiles/r03/qfwd_probe_16x16.txt): 32x32x16
# 2.07 PF, 16x16x32 2.33 PF; the 16x16 forward's mix of the two at those rates
MFMA32_BF16_SUSTAINED_TFLOPS = 2068.0
MFMA_BF16_SUSTAINED_TFLOPS = round((QNET_MFMA32_FLOP + QNET_MFMA16_FLOP) /
                                   (QNET_MFMA32_FLOP / MFMA32_BF16_SUSTAINED_TFLOPS + QNET_MFMA16_FLOP / 2330.0), 1)


def qnet_leg(env, args, world, dist, torch, opponent):
    """BASELINE config 5: the reference's epsilon-greedy DQN (weights: the checkpoint
    human_player.py:68 loads, tests/golden/dqn_checkpoints.npz) fused with the env step."""
    import numpy as np

    from merging_gym.policy import QNet

    f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    qnet = QNet.from_state_dict({k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l1/")},
                                device=env.device)
    label = opponent
    if opponent == "other":  # main.py's default Strategy_OP "L1": another trained DQN (:161-168)
        opponent = QNet.from_state_dict({k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l3/")},
                                        device=env.device)
    T, L, E = args.rollout_steps, args.qnet_launches, env.num_envs
    k = 20_000_000
    # the leg's own episodes (main.py's logged quantities, q_eval included): cleared ahead of the
    # warm-up launches, since a clear just before the window slows the launches after it (main leg)
    env.clear_statistics()
    for _ in range(max(1, args.leg_warmup)):
        env.rollout_qnet(T, qnet, args.seed, opponent=opponent, first_step=k, final_observation=False,
                         won_mask=False)
        k += T
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    ev0.record()
    for j in range(L):
        env.rollout_qnet(T, qnet, args.seed, opponent=opponent, first_step=k, final_observation=False,
                         won_mask=False)
        k += T
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / L
    nets = 2 if label in ("self", "other") else 1
    # the instances without a net opponent run the 32x32 forward (qnet32_mlp), the others the 16x16 one
    mfma_flop, sustained = ((QNET32_MFMA_FLOP, MFMA32_BF16_SUSTAINED_TFLOPS) if nets == 1
                            else (QNET_MFMA_FLOP, MFMA_BF16_SUSTAINED_TFLOPS))
    per_s = E * T / (kernel_ms * 1e-3)
    summ = env.episode_summary()  # untimed: mg_stats_reduce over the warm-up and timed launches' records
    ep_rate = summ["completed"] / (E * T * (L + max(1, args.leg_warmup)))  # episodes per env-step
    # forwards the reference runs per env-step: the ego's greedy branch + q_eval once per episode,
    # the opponent's greedy branch (self / other net)
    fwd = p_greedy() * nets + ep_rate
    # BASELINE config 5: greedy-action agreement with the reference's fp32 Net on the CPU
    # (main.py:30-47, re-declared here with torch) over the envs' current observations
    sample = env.observe()[: 1 << 16].clone()
    greedy_gpu = qnet.forward(sample).argmax(1).cpu()
    w = {k.split("/", 1)[1]: torch.from_numpy(f[k]) for k in f.files if k.startswith("l1/")}
    x = sample.cpu()
    h = torch.relu(x @ w["fc1.weight"].T + w["fc1.bias"])
    h = torch.relu(h @ w["fc2.weight"].T + w["fc2.bias"])
    greedy_cpu = (h @ w["out.weight"].T + w["out.bias"]).argmax(1)
    return {"episodes": {k: summ[k] for k in ("completed", "mean_q_eval", "mean_ep_reward_main", "win_rate_main",
                                               "collision_rate")},
            "q_eval_logged_as": "eval_net(state)[action] on each episode's last input and action (main.py:221)",
            "kernel": "qnet_rollout_ws_kernel<%s>" % {"none": "0, false", "uniform": "1, false", "self": "2, true",
                                                      "other": "3, true"}[label],
            "opponent": label if label != "other" else "other net (main.py Strategy_OP L1; checkpoint l3)",
            "steps_per_launch": T, "launches": L, "dtype": "bf16 (fp32 accumulate)",
            "value": world * E * T * L / elapsed, "unit": "env-steps/s",
            "ms_per_step": elapsed / (L * T) * 1e3, "kernel_ms_mean": kernel_ms,
            "reference_forwards_per_env_step": fwd,
            "forwards_rule": ("P(greedy) = Phi(0.7) per net per env-step (main.py:105) + one per finished episode "
                              "(q_eval, main.py:221)"),
            "useful_tflops": fwd * QNET_USEFUL_FLOP * per_s / 1e12,
            "forward": "32x32" if nets == 1 else "16x16",
            "mfma_tflops_if_every_forward_ran": nets * mfma_flop * per_s / 1e12,
            "peak_tflops": MFMA_BF16_PEAK_TFLOPS,
            "frac_useful": fwd * QNET_USEFUL_FLOP * per_s / 1e12 / MFMA_BF16_PEAK_TFLOPS,
            "sustained_tflops": sustained,
            "greedy_agreement_vs_fp32_cpu": float((greedy_gpu == greedy_cpu).double().mean()),
            "agreement_sample": int(x.shape[0])}


HDQN_META_FLOP = 2 * (10 * 200 + 200 * 100 + 100 * 3)   # Goal_DQN's meta-net (hdqn.py:38-55, 10 -> 3)
HDQN_LOWER_FLOP = 2 * (11 * 200 + 200 * 100 + 100 * 5)  # HDQN's lower-level net on [goal] + state (11 -> 5)


def hdqn_useful_flop(p, brk, ep, opponent_nets):
    """bf16 FLOPs per env-step of the forwards hdqn.py runs (greedy branches only): the ego's
    choose_goal on every next state (:303) and again at each new outer iteration (:283: after a
    goal break on the same state, after an episode end on the reset one), its choose_action every
    step (:292), the episode's q_eval (:330); with a net opponent its choose_action every step (:300)
    and its choose_goal at each outer iteration (:285). brk: outer iterations per env-step (goal
    breaks and episode ends, :322), ep: episodes per env-step."""
    meta = p * (1.0 + brk) + ep
    lower = p
    if opponent_nets:
        meta += p * brk
        lower += p
    return meta * HDQN_META_FLOP + lower * HDQN_LOWER_FLOP


def hdqn_leg(env, args, world, dist, torch):
    """hdqn.py's acting loop (scripts/hdqn.py:280-323) fused with the env step (mg_rollout_hdqn):
    per env-step Goal_DQN's meta-net (10 -> 3) on the next state and the lower-level Net
    (11 -> 5) on the goal state, both bf16 MFMA, L0 opponent. No h-DQN checkpoint ships with the
    reference, so the nets are seeded draws with torch.nn.Linear's default (signed) initialisation,
    U(-1/sqrt(in), 1/sqrt(in)) for weights and biases -- as the GPU tests use: their choices vary
    from env to env (hdqn.py:41-47's uniform(0, 1) weights pick one action for > 90 % of inputs,
    tests/test_hdqn_test_nets.py, which would measure an almost constant policy). The goal-break
    rate (the share of env-steps that end an inner loop, :322) is reported beside it."""
    import numpy as np

    from merging_gym.policy import NUM_GOALS, QNet

    # seed 15: the L0 leg's episodes mix collisions and ego wins (seed 0, rounds 2-5, gave a lower net
    # that picks speed 10 for 97 % of states: every ego trailed the L0 car, collision and win rates
    # 0.0). Chosen on the CPU from 40 seeds with the oracle and the bf16-emulated nets: collision
    # rate 0.195, ego first 0.90 over 3,000 episodes (h-DQN bench nets).
    rng = np.random.default_rng(15)

    def net(i, o):
        sd = {}
        for name, (a, b) in zip(("fc1", "fc2", "out"), [(200, i), (100, 200), (o, 100)]):
            sd[f"{name}.weight"] = rng.uniform(-b ** -0.5, b ** -0.5, (a, b)).astype(np.float32)
            sd[f"{name}.bias"] = rng.uniform(-b ** -0.5, b ** -0.5, a).astype(np.float32)
        return QNet.from_state_dict(sd, device=env.device)

    meta, lower = net(10, NUM_GOALS), net(11, 5)
    T, L, E = args.rollout_steps, args.qnet_launches, env.num_envs
    k = 40_000_000
    env.clear_statistics()  # the leg's own episodes (hdqn.py's logged quantities), ahead of the warm-up
    for _ in range(max(1, args.leg_warmup)):
        env.rollout_hdqn(T, meta, lower, args.seed, first_step=k, final_observation=False)
        k += T
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    ev0.record()
    for j in range(L):
        env.rollout_hdqn(T, meta, lower, args.seed, first_step=k, final_observation=False)
        k += T
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / L
    per_s = E * T / (kernel_ms * 1e-3)
    summ = env.episode_summary()  # untimed: the warm-up and timed launches' episodes (mg_stats_reduce)
    episodes = {k: summ[k] for k in ("completed", "mean_q_eval", "mean_return_ego", "win_rate_hdqn", "collision_rate")}
    ep_rate = summ["completed"] / (E * T * (L + max(1, args.leg_warmup)))
    # untimed: one launch with Goal_DQN's columns, for the inner-loop break rate (:322)
    tr = env.rollout_hdqn(T, meta, lower, args.seed, first_step=k, final_observation=False, goal_memory=True)
    k += T
    nb = tr["no_break"].cpu().numpy()  # [T, ceil(E/64)] bits: set where the step did not end the inner loop
    cont = int(np.unpackbits(nb.view(np.uint8), bitorder="little").reshape(T, -1)[:, :E].sum())
    break_rate = 1.0 - cont / (T * E)
    greedy_goal_spread = torch.bincount(tr["next_goal"].flatten().to(torch.int64), minlength=NUM_GOALS)
    greedy_goal_spread = (greedy_goal_spread.double() / greedy_goal_spread.sum()).tolist()

    # with hdqn.py's lower-level memory (HDQN.store_transition, :316, every transition): the
    # store fused into the launch vs the rollout followed by mg_replay_store from its outputs
    from merging_gym import ReplayRing

    ring = ReplayRing(1 << 24, device=env.device, goal=True)
    Lr = max(1, L // 2)

    def timed(fn):
        nonlocal k
        fn()
        k += T
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(Lr):
            fn()
            k += T
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / Lr

    obs0 = env.observe().clone()
    fused_ms = timed(lambda: env.rollout_hdqn(T, meta, lower, args.seed, first_step=k, ring=ring))

    def separate():
        tr = env.rollout_hdqn(T, meta, lower, args.seed, first_step=k)
        ring.store_rollout(obs0, tr, skip_ego_won=False, goal=tr["goal"], next_goal=tr["next_goal"],
                           reward=tr["reward"])
    separate_ms = timed(separate)
    del ring
    torch.cuda.empty_cache()
    # Strategy_OP "selfplay" (hdqn.py:262-264): the same nets also act for the opponent, on the
    # swapped state (its lower net every step, its meta-net at each outer-loop iteration)
    for _ in range(2):
        env.rollout_hdqn(T, meta, lower, args.seed, opponent="self", first_step=k, final_observation=False)
        k += T
    self_ms = timed(lambda: env.rollout_hdqn(T, meta, lower, args.seed, opponent="self", first_step=k,
                                             final_observation=False))
    self_per_s = E * T / (self_ms * 1e-3)
    # any other Strategy_OP (hdqn.py:265-268): the opponent's own Goal_DQN + HDQN from another
    # checkpoint; four nets exceed one CU's LDS, so the kernel reads the opponent's from L2
    meta_op, lower_op = net(10, NUM_GOALS), net(11, 5)
    env.hdqn_goal_op = None  # fresh opponent goals for the other nets
    for _ in range(2):
        env.rollout_hdqn(T, meta, lower, args.seed, opponent=(meta_op, lower_op), first_step=k,
                         final_observation=False)
        k += T
    other_ms = timed(lambda: env.rollout_hdqn(T, meta, lower, args.seed, opponent=(meta_op, lower_op),
                                              first_step=k, final_observation=False))
    other_per_s = E * T / (other_ms * 1e-3)
    p = p_greedy()
    l0_flop = hdqn_useful_flop(p, break_rate, ep_rate, False)
    self_flop = hdqn_useful_flop(p, break_rate, ep_rate, True)  # the L0 leg's break / episode rates
    return {"kernel": "hdqn_rollout_kernel<0>", "opponent": "none", "steps_per_launch": T, "launches": L,
            "selfplay": {"kernel": "hdqn_rollout_kernel<2>", "kernel_ms_mean": self_ms,
                         "env_steps_per_s": self_per_s, "useful_tflops": self_flop * self_per_s / 1e12,
                         "frac_useful": self_flop * self_per_s / 1e12 / MFMA_BF16_PEAK_TFLOPS},
            "other_checkpoint": {"kernel": "hdqn_rollout_kernel<3>", "kernel_ms_mean": other_ms,
                                 "env_steps_per_s": other_per_s,
                                 "frac_useful": self_flop * other_per_s / 1e12 / MFMA_BF16_PEAK_TFLOPS,
                                 "note": "opponent nets read from global memory (L2, fragment-major copies), not LDS"},
            "useful_flop_rule": ("hdqn.py's forwards, greedy branches only (P = Phi(0.7)): ego meta-net per next state "
                                 "and per outer iteration, ego lower net per step, q_eval per episode; a net opponent "
                                 "adds its lower net per step and its meta-net per outer iteration (break and "
                                 "episode rates of the L0 leg)"),
            "useful_flop_per_env_step": {"L0": l0_flop, "selfplay_other": self_flop},
            "with_goal_ring": {"fused_store_ms_per_launch": fused_ms, "rollout_then_replay_store_ms": separate_ms,
                               "fused_env_steps_per_s": E * T / (fused_ms * 1e-3),
                               "separate_env_steps_per_s": E * T / (separate_ms * 1e-3),
                               "ring_capacity": 1 << 24},
            "dtype": "bf16 (fp32 accumulate)", "value": world * E * T * L / elapsed, "unit": "env-steps/s",
            "ms_per_step": elapsed / (L * T) * 1e3, "kernel_ms_mean": kernel_ms,
            "useful_tflops": l0_flop * per_s / 1e12, "peak_tflops": MFMA_BF16_PEAK_TFLOPS,
            "frac_useful": l0_flop * per_s / 1e12 / MFMA_BF16_PEAK_TFLOPS,
            "episodes_per_env_step": ep_rate,
            "nets": ("seeded (numpy default_rng(15)), torch.nn.Linear default init U(-1/sqrt(in), 1/sqrt(in)) "
                     "(signed); the seed gives episodes with collisions and ego wins"),
            "goal_break_rate_per_step": break_rate, "next_goal_share": greedy_goal_spread,
            "episodes": episodes,
            "q_eval_logged_as": "meta_eval_net(state)[goal] on each episode's terminal state and its goal (hdqn.py:330)"}


def replay_algorithmic_bytes(n, T, kept, done_rows, capacity):
    """Bytes mg_replay_store must move at minimum: every obs row once (40) + the trajectory's
    interleaved (a1, a2, done, collision) word (4: a and done are read from it) + won bits (read by
    both kernels, 2 x 1/8); per stored transition r (4) + the 88-byte row written; the terminal
    observation of done rows (40); obs_first once per env (40). When one store appends more than
    the ring holds, only the newest `capacity` rows are written (the rest would be overwritten
    within the same store), so only those count."""
    written = min(kept, capacity)
    frac = written / kept if kept else 0.0
    return n * T * (40 + 4 + 0.25) + written * (4 + 88) + done_rows * frac * 40 + n * 40


def replay_leg(env, args, torch):
    """BASELINE section 8(f) rank 3: the device replay memory. A config-5 rollout (T steps of the
    fused DQN policy) is appended to a 2^24-row ring (DQN.store_transition, main.py:115-119,
    with the :209 filter) by mg_replay_store -- count, scan, write kernels, timed together with
    events on the stream they run on -- then a 128-row minibatch is drawn (main.py:130)."""
    import numpy as np

    from merging_gym import ReplayRing
    from merging_gym.policy import QNet

    f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    qnet = QNet.from_state_dict({k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l1/")},
                                device=env.device)
    T, E, L = args.rollout_steps, env.num_envs, args.replay_stores
    obs0 = env.observe().clone()
    traj = env.rollout_qnet(T, qnet, args.seed, first_step=30_000_000)
    ring = ReplayRing(1 << 24, device=env.device)
    for _ in range(2):
        ring.store_rollout(obs0, traj)
    torch.cuda.synchronize()
    c0 = ring.memory_counter
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * L)]
    for j in range(L):
        ev[2 * j].record()
        ring.store_rollout(obs0, traj)
        ev[2 * j + 1].record()
    torch.cuda.synchronize()
    kept = (ring.memory_counter - c0) / L
    ms = sum(ev[2 * j].elapsed_time(ev[2 * j + 1]) for j in range(L)) / L
    nbytes = replay_algorithmic_bytes(E, T, kept, int(traj["done"].sum().item()), ring.capacity)
    achieved = nbytes / (ms * 1e-3) / 1e9
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for j in range(100):
        ring.sample_rows(128, seed=args.seed, draw=j)
    e.record()
    torch.cuda.synchronize()
    traffic = load_pmc_replay(E, T)
    return {"kernels": "replay_scan_kernel + replay_group_scan_kernel + replay_write_kernel",
            "transitions_per_store": T * E, "stored_per_store": kept, "capacity": 1 << 24,
            "value": kept / (ms * 1e-3), "unit": "transitions/s", "ms_per_store": ms,
            "bytes_per_store": nbytes, "achieved": achieved,
            "peak": HBM_PEAK_GBPS, "unit_bw": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
            # bytes L2 really moves for the store (PMC): the write blocks re-read the observation row
            # before their 2-step chunk (Replay memory), ~1.16x the algorithmic bytes
            "traffic": traffic, "frac_traffic": None if traffic is None else traffic / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "sample_128_us": s.elapsed_time(e) / 100 * 1e3}


def dropin_leg(seed: int):
    """BASELINE config 1: merging_gym.make('merging-v0') single env, 500 step() calls with
    uniform random actions for both players, reset on done. Three steps on the same action
    sequence: the drop-in's default host backend (mg_host_step: the kernels' own step functions
    compiled for the CPU, one ctypes call per step), its GPU backend (a batch of one env in the
    step kernel: one launch + one stream sync per step, the kernel reading the actions from and
    writing its 168-byte record to pinned host memory), and the pure-Python restatement of the
    reference's step (oracle.PyMergeEnv, numpy sin/cos + the QP solved per car-step) -- the
    reference itself measured 5,090 steps/s in the survey container. The
    host and GPU backends must return the same values (checked here on every step)."""
    import numpy as np

    import merging_gym

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import merge_oracle

    rng = np.random.default_rng(seed)
    acts = rng.integers(0, 5, (500, 2)).tolist()
    out, trace = {}, {}
    for name, env in (("host_dropin", merging_gym.make("merging-v0")),
                      ("gpu_dropin", merging_gym.make("merging-v0", backend="gpu")),
                      ("cpu_python_port", merge_oracle.PyMergeEnv())):
        env.reset()
        env.step(0, 0)
        env.reset()
        episodes, rows = 0, []
        t0 = time.perf_counter()
        for a1, a2 in acts:
            row = env.step(a1, a2)
            rows.append(row)
            if row[2]:
                env.reset()
                episodes += 1
        dt = time.perf_counter() - t0
        trace[name] = rows
        out[name] = {"steps_per_s": 500 / dt, "us_per_step": dt / 500 * 1e6, "episodes_finished": episodes}
    out["host_equals_gpu"] = trace["host_dropin"] == trace["gpu_dropin"]
    out["default_backend"] = merging_gym.make("merging-v0").backend
    out["workload"] = "config 1: one env, 500 random-action step() calls, reset on done (list API)"
    return out


def _native_build_info():
    from merging_gym import _native

    return _native.build_info()


DEVICE_COUNT_ENV = "MG_BENCH_DEVICE_COUNT"   # overrides the probe (tests of the launch decision)
SELF_LAUNCH_ENV = "MG_BENCH_SELF_LAUNCHED"  # set in the ranks a self-launch starts


def visible_gpu_count() -> int:
    """GPUs the ranks could use, counted in a child process (torch.cuda.device_count() there), so that
    the launching process itself never imports torch or loads HIP before it starts the ranks."""
    if DEVICE_COUNT_ENV in os.environ:
        return int(os.environ[DEVICE_COUNT_ENV])
    import subprocess

    out = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                         capture_output=True, text=True, timeout=900)
    if out.returncode != 0:
        raise SystemExit(f"bench.py: counting GPUs failed (rc {out.returncode}): {out.stderr[-400:]}")
    return int(out.stdout.strip().splitlines()[-1])


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(args, environ, ngpu: int, port: int) -> list:
    """The environment of each rank of a self-launch (--gpus N > 1 without a launcher's WORLD_SIZE):
    the variables torchrun would set, one GPU per rank. Under RCCL (backend nccl) every rank needs a
    GPU of its own, so fewer than N visible GPUs is an error; a gloo rehearsal may share them."""
    n = args.gpus
    if ngpu < 1:
        raise SystemExit(f"bench.py --gpus {n}: no GPU visible")
    if args.dist_backend == "nccl" and ngpu < n:
        raise SystemExit(f"bench.py --gpus {n}: only {ngpu} GPU(s) visible; RCCL needs one per rank "
                         "(--dist-backend gloo rehearses N ranks on fewer GPUs)")
    out = []
    for r in range(n):
        e = dict(environ)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **{SELF_LAUNCH_ENV: "1"})
        out.append(e)
    return out


def self_launch(args, argv, popen=None, script=None) -> int:
    """Start N one-GPU ranks of this script (same arguments) as child processes and wait for them:
    rank 0 prints the JSON line on the shared stdout; when a rank fails the others are stopped. Returns
    the worst exit status (the first nonzero one in rank order). Runs before anything in this process
    imports torch or loads HIP, and replaces no process (children only)."""
    import signal
    import subprocess

    popen = popen or subprocess.Popen
    envs = rank_envs(args, os.environ, visible_gpu_count(), free_port())
    cmd = [sys.executable, "-u", script or os.path.abspath(__file__), *argv]
    procs = [popen(cmd, env=e) for e in envs]

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    first_bad = None
    stopped_at = None
    try:
        rcs = [None] * len(procs)
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
                    if rcs[i] not in (None, 0) and first_bad is None:
                        first_bad = rcs[i]
                        print(f"bench.py: rank {i} exited with {rcs[i]}; stopping the others", file=sys.stderr)
                        stop()  # a failed rank would leave the others at a barrier
                        stopped_at = time.time()
            if stopped_at is not None and time.time() - stopped_at > 30:
                for p in procs:  # a rank that ignored SIGTERM for 30 s (stuck in a collective)
                    if p.poll() is None:
                        p.kill()
                stopped_at = None
            time.sleep(0.05)
    finally:
        signal.signal(signal.SIGTERM, old)
        stop()
    if first_bad is None:
        return 0
    return first_bad if first_bad > 0 else 128 - first_bad  # killed by signal s: 128 + s, as a shell reports


def sync_spin(local_rank=None):
    """hipDeviceScheduleSpin for this rank's device, before the HIP context exists: a synchronize
    then spins on the host instead of yielding, so the host thread that issues the timed launches
    is awake when the window opens (tools/window_probe.py). The flags belong to the calling
    thread's current device, so a rank first makes its own device current (device LOCAL_RANK mod
    the visible count, as main() picks it below; rank r > 0 would otherwise set device 0's)."""
    import ctypes

    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return None
    if local_rank is not None:
        count = ctypes.c_int(0)
        if hip.hipGetDeviceCount(ctypes.byref(count)) != 0 or count.value < 1:
            return None
        if hip.hipSetDevice(ctypes.c_int(local_rank % count.value)) != 0:
            return None
    return hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's 1-GPU form (python3 bench.py --gpus N) asked for N GPUs: start N ranks here,
        # before this process touches HIP (sync_spin below already does)
        sys.exit(self_launch(args, sys.argv[1:]))
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} under a launcher with WORLD_SIZE={env_world}")
    launcher = ("self" if os.environ.get(SELF_LAUNCH_ENV) == "1" else "external") if env_world > 1 else None
    local = int(os.environ.get("LOCAL_RANK", "0"))
    spin_rc = sync_spin(local if env_world > 1 else None) if args.sync_spin else None
    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    if env_world > 1 and args.dist_backend == "nccl" and local >= ndev:
        raise SystemExit(f"rank with LOCAL_RANK {local}: only {ndev} GPU(s) visible (RCCL needs one per rank)")
    device = torch.device("cuda", local % max(ndev, 1) if env_world > 1 else 0)
    torch.cuda.set_device(device)
    backend = None
    coll_ranks = None
    if env_world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.dist_backend)
        backend = dist.get_backend()
        # the rank count the collective itself sees: one all-reduce of a 1 per rank over the
        # process group (RCCL over xGMI under "nccl"), outside every timed region
        one = torch.ones(1, dtype=torch.int64, device=device if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(one)
        coll_ranks = int(one.item())
    # the rank count and rank the process group reports (RCCL under backend "nccl" on ROCm)
    world = dist.get_world_size() if env_world > 1 else 1
    rank = dist.get_rank() if env_world > 1 else 0
    if world != args.gpus or (coll_ranks is not None and coll_ranks != args.gpus):
        raise SystemExit(f"bench.py --gpus {args.gpus}: process group of {world} ranks, all-reduce saw {coll_ranks}")
    host_coll = world > 1 and args.dist_backend != "nccl"

    from merging_gym import MergeVecEnv

    E = args.envs
    env = MergeVecEnv(E, device=device, autoreset=True, env_offset=rank * E,
                      final_observation=True, episode_stats=True)
    step = lambda k: env.step_random(args.seed, opponent_random=True, step_idx=k)  # noqa: E731

    # steady state first: every env past its first episodes, some finishing at every step
    k0 = burn_in(env, args.burn_in, args.seed, stagger(env, args.stagger, args.seed, 0, torch))
    # the statistics are cleared here, ahead of the burn-in launches, not just before the window: any
    # clear is followed by ~200 launches of up to +6 % per launch (a transient after the different
    # kernel, not the record writes: tools/size2_probe2.py, DESIGN.md section 4 "The 2^22 first
    # window"), so the episodes reported below are those completed since this point
    env.clear_statistics()
    launches_since_clear = args.burn_in_launches + args.warmup + args.steps
    for k in range(k0, k0 + args.burn_in_launches):
        step(k)
    k0 += args.burn_in_launches
    # The W warm-up launches run inside a rehearsal of the timed window (synchronize, event
    # pair, launches, event record, synchronize, elapsed time): the first such window of a
    # process pays one-time host costs -- 55-65 us before its first launch and a 30-40 us stall
    # inside, +15 % on a 20-launch window, 0 in the following ones (tools/window_probe2.py,
    # profiles/r02/window_probe2.json)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wev0, wev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    wev0.record()
    for k in range(k0, k0 + args.warmup):
        step(k)
    wev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wev0.elapsed_time(wev1)
    k0 += args.warmup
    graph = capture_steps(step, k0, args.steps, torch) if args.graph else None
    torch.cuda.synchronize()

    # Timed region: K launches back to back (one graph replay, or K host launches), bracketed by
    # a barrier + synchronize, with one HIP event pair recorded on the stream the kernels run on
    # (torch's current stream). Average launch duration = region / K (launch gaps included).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gc.disable()  # no collector pause inside the window
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    if graph is not None:
        graph.replay()
    else:
        for k in range(k0, k0 + args.steps):
            step(k)
    ev1.record()
    host_ms = (time.perf_counter() - t0) * 1e3 / args.steps  # host enqueue time per launch
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    k0 += args.steps
    completed_since_clear = int(env.counts[:, 0].sum())
    del graph

    # untimed: per-dispatch durations (events written by the dispatch packets themselves,
    # hipExtLaunchKernel via mg_time_next_launch) for a sample of launches, for reference
    dispatch_ms = None
    if not args.no_events:
        from merging_gym.profiling import KernelTimer

        nsamp = max(1, min(64, args.steps // max(1, args.event_every)))
        timer = KernelTimer(nsamp)
        for j in range(nsamp):
            timer.arm(j)
            step(k0 + j)
        torch.cuda.synchronize()
        durs = timer.durations_ms()
        dispatch_ms = sum(durs) / len(durs)
        timer.close()
        k0 += nsamp

    t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device="cpu" if host_coll else device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kernel_ms_max = float(t[0]), float(t[1])

    # episode statistics (every episode completed since the clear before the burn-in launches), the quantities the
    # reference's scripts log: each rank reduces its shard on the device to 80 bytes of totals,
    # which one RCCL all-gather (xGMI) brings to every rank, outside the timed loop. The device
    # reduction and the collective are timed apart; at world size 1 there is no collective.
    from merging_gym.distributed import (NUM_COUNTS, NUM_RETURNS, PARTIAL_BYTES, gather_episode_stats,
                                         gather_episode_summary, summarize)

    timings = {}
    torch.cuda.synchronize()
    if world > 1 and args.gather == "per-env":
        g0 = time.perf_counter()
        rows = gather_episode_stats(env.returns, env.counts)
        torch.cuda.synchronize()
        timings["allgather_ms"] = (time.perf_counter() - g0) * 1e3
        g0 = time.perf_counter()
        episodes = summarize(*rows)
        timings["reduce_ms"] = (time.perf_counter() - g0) * 1e3
        payload = E * (NUM_RETURNS + NUM_COUNTS // 2) * 8
    else:
        episodes = gather_episode_summary(env.returns, env.counts, timings=timings)
        payload = PARTIAL_BYTES if world > 1 else 0
    episodes["mean_q_eval"] = None  # random actions: no Q-net evaluates them (main.py:221 logs a DQN's value)
    episodes.update(allgather_ms=timings.get("allgather_ms"), reduce_ms=timings.get("reduce_ms"),
                    reduce_wall_ms=timings.get("reduce_wall_ms"),
                    reduce_how=("mg_stats_reduce, fixed order (64 B of records per env): reduce_ms = HIP events "
                                "around its two launches, reduce_wall_ms = the Python call on the host clock"),
                    allgather_bytes_per_rank=payload,
                    completed_rank0=completed_since_clear,
                    counted_since=(f"the statistics clear before the burn-in launches: {launches_since_clear} launches "
                                   "(burn-in, warm-up, timed window)"),
                    logged_as=("mean_return_ego / win_rate_hdqn: hdqn.py:312, :342 (terminal observation); "
                               "mean_ep_reward_main / win_rate_main: main.py:209-211, :225 (winner-filtered "
                               "reward, pre-terminal observation); ego_first_rate: winner == 1"))

    # the step kernel past the Infinity Cache, after every other leg by default. Rounds 2-3 saw it
    # 2.2-2.6x slower there in one 100-launch window; per-window timing (r03e) showed a one-time
    # ~7 ms stall inside the first 20 launches, the rest at full speed and every arena placement
    # equal (tools/placement_probe.py): with the collector off and one rehearsal window, first /
    # last / last with the env allocated before the legs measure 104.9 / 105.0 / 105.2 us (r03h)
    size2 = None
    do_size2 = world == 1 and args.size2_envs > 0 and args.size2_envs != E
    env2 = size2_env(args, torch) if do_size2 and args.size2_prealloc else None
    if do_size2 and args.size2_when == "first":
        size2 = size2_leg(args, torch, env2)
        env2 = None

    rollout = None
    if args.rollout_steps > 0:
        rollout = rollout_leg(env, args, world, dist, torch)
    replay = None
    if args.replay_stores > 0 and args.rollout_steps > 0:
        replay = replay_leg(env, args, torch)

    qnet = None
    if args.qnet_launches > 0 and args.rollout_steps > 0:
        qnet = [qnet_leg(env, args, world, dist, torch, opp) for opp in ("none", "self", "other")]

    hdqn = None
    if args.qnet_launches > 0 and args.rollout_steps > 0:
        hdqn = hdqn_leg(env, args, world, dist, torch)

    if do_size2 and args.size2_when == "last":
        size2 = size2_leg(args, torch, env2)
        env2 = None

    total_env_steps = world * E * args.steps
    value = total_env_steps / elapsed
    # the CPU baseline and the config-1 drop-in leg run on rank 0 after every rank's GPU legs, at any
    # world size (north_star: the reference-style step timed on the box's host cores in the same run);
    # the other ranks wait at the closing barrier. The child process never touches a GPU.
    cpu = dropin = None
    if world > 1:
        dist.barrier()
    if rank == 0 and not args.no_cpu_baseline:
        dropin = dropin_leg(args.seed)
        cpu = cpu_baseline(args.cpu_seconds, E)
        cpu["ran_while"] = ("the other ranks wait at the closing barrier" if world > 1 else "alone")
    if rank == 0:
        achieved = BYTES_PER_ENV_STEP * E / (kernel_ms * 1e-3) / 1e9 if kernel_ms else None
        # all ranks' bytes over the slowest rank's mean launch: the whole node against world x peak
        achieved_agg = world * BYTES_PER_ENV_STEP * E / (kernel_ms_max * 1e-3) / 1e9 if kernel_ms_max else None
        pmc = load_pmc(E)
        line = {
            "metric": "env-steps/sec at batch=2^20; achieved HBM GB/s vs peak; 1/2/4/8-GPU scaling",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "dist": {"backend": backend, "world_size": world, "rank_printing": rank,
                     "launcher_world_size": env_world, "launcher": launcher, "collective_ranks": coll_ranks,
                     "gpus_requested": args.gpus},
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (deterministic reset, Philox4x32-10 uniform actions for both players)",
            "config": {"workload": (("config 3/4: " if E == 1 << 20 else "")
                                    + f"{E:,} envs per MI355X, device-drawn random actions, "
                                    "autoreset, episode statistics"),
                       "envs_per_gpu": E, "global_envs": world * E,
                       "parallelism": f"dp{world} (env shards, no per-step collective)"},
            "burn_in_steps": args.burn_in + args.burn_in_launches,
            "build": _native_build_info(),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBPS) if achieved else None,
                         "traffic": pmc, "kernel": KERNEL_NAME,
                         "bytes_per_env_step": BYTES_PER_ENV_STEP,
                         "frac_8d": (BYTES_PER_ENV_STEP_8D * E / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
                                     if kernel_ms else None),
                         "bytes_per_env_step_8d": BYTES_PER_ENV_STEP_8D,
                         "bytes_note": ("frac: this layout's 152 B (fp64 returns 16 B each way, the action "
                                        "write-back 2 B, done / collision / actions as one 4-B record); "
                                        "frac_8d: SURVEY.md 8(d)'s 136 B (fp32 returns)"),
                         "kernel_ms_mean": kernel_ms, "kernel_ms_mean_max_rank": kernel_ms_max,
                         "achieved_aggregate": achieved_agg,
                         "frac_aggregate": (achieved_agg / (world * HBM_PEAK_GBPS)) if achieved_agg else None,
                         "aggregate_rule": "world x bytes per launch / the slowest rank's mean launch, vs world x peak",
                         "timing": ("HIP events recorded on the launch stream around the K timed launches "
                                    f"({'one HIP-graph replay' if args.graph else 'K host launches'}), / K"),
                         "kernel_ms_dispatch_sample": dispatch_ms, "host_enqueue_ms_per_launch": host_ms,
                         "host_sync": "spin" if spin_rc == 0 else "default",
                         "wall_over_kernel": (elapsed / args.steps * 1e3) / kernel_ms if kernel_ms else None,
                         "traffic_rule": "2 x FETCH_SIZE + WRITE_SIZE per launch, profiles/pmc_traffic.json"},
            "episodes": episodes,
        }
        valu = load_valu()
        if rollout is not None:
            if "rollout_kernel" in valu:  # VALU-issue roofline of the rollout (VALU, not HBM, bound)
                rollout["valu_roofline"] = valu["rollout_kernel"]
            line["rollout"] = rollout
        if replay is not None:
            line["replay"] = replay
        if qnet is not None:
            line["qnet_policy"] = qnet
        if hdqn is not None:
            if "hdqn_rollout" in valu:
                hdqn["valu"] = valu["hdqn_rollout"]
            for key, sub in (("hdqn_rollout<2>", "selfplay"), ("hdqn_rollout<3>", "other_checkpoint")):
                if key in valu and isinstance(hdqn.get(sub), dict):
                    hdqn[sub]["valu"] = valu[key]
            line["hdqn_policy"] = hdqn
        if qnet is not None:  # opponents none / self / other: kernel instances 0 / 2 / 3
            for leg, key in zip(qnet, ("qnet_rollout", "qnet_rollout<2>", "qnet_rollout<3>")):
                if key in valu:
                    leg["valu"] = valu[key]
        if size2 is not None:
            line["size_2p22"] = size2
        if cpu is not None:
            line["dropin_single_env"] = dropin
            line["cpu_baseline"] = cpu
        line["stagger"] = {"value": args.stagger, "statistics_cleared": "before the burn-in launches",
                           "note": "--stagger 0 reproduces the round-3 start (every env's first episode together)"}
        # the full record on an earlier line (not JSON by itself), then the compact JSON line the
        # driver parses: it keeps only the last ~8 KB of the output
        print("bench detail: " + json.dumps(line), flush=True)
        print(json.dumps(compact_line(line)), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def compact_line(line):
    """The bench contract's ONE JSON line, kept under ~6 KB: every leg's value, roofline fraction,
    mean kernel time and traffic; the per-leg details (VALU counters, episode statistics, notes) are
    on the earlier "bench detail:" line."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "dist", "build", "stagger")
    out = {k: line[k] for k in keep if k in line}
    rf = line["roofline"]
    out["roofline"] = {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel",
                                             "bytes_per_env_step", "frac_8d", "kernel_ms_mean",
                                             "kernel_ms_mean_max_rank", "achieved_aggregate", "frac_aggregate")}
    cb = line.get("cpu_baseline")
    if cb is not None:
        out["cpu_baseline"] = ({"error": cb["error"][-300:]} if "error" in cb else
                               {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "sample", "ran_while")})
    legs = {}
    ep = line.get("episodes") or {}
    legs["step_episodes"] = {k: ep.get(k) for k in ("completed", "collision_rate", "win_rate_hdqn", "allgather_ms",
                                                   "reduce_ms")}
    if "size_2p22" in line:
        z = line["size_2p22"]
        legs["size_2p22"] = {k: z.get(k) for k in ("envs", "value", "kernel_ms", "frac", "frac_8d", "traffic")}
    if "rollout" in line:
        z = line["rollout"]
        legs["rollout"] = {k: z.get(k) for k in ("kernel", "value", "kernel_ms_mean", "bytes_per_env_step", "frac",
                                                "traffic")}
    if "replay" in line:
        z = line["replay"]
        legs["replay"] = {k: z.get(k) for k in ("value", "unit", "ms_per_store", "frac", "traffic", "frac_traffic",
                                               "sample_128_us")}
    for z in line.get("qnet_policy") or []:
        legs["qnet_" + z["opponent"].split(" ")[0]] = {
            k: z.get(k) for k in ("kernel", "value", "kernel_ms_mean", "frac_useful", "reference_forwards_per_env_step",
                                  "greedy_agreement_vs_fp32_cpu")}
        legs["qnet_" + z["opponent"].split(" ")[0]]["q_eval_mean"] = z["episodes"]["mean_q_eval"]
    h = line.get("hdqn_policy")
    if h is not None:
        legs["hdqn_L0"] = {"kernel": h["kernel"], "value": h["value"], "kernel_ms_mean": h["kernel_ms_mean"],
                           "frac_useful": h["frac_useful"], "goal_break_rate": h["goal_break_rate_per_step"],
                           "episodes": h["episodes"]["completed"], "collision_rate": h["episodes"]["collision_rate"],
                           "win_rate_hdqn": h["episodes"]["win_rate_hdqn"]}
        for key, name in (("selfplay", "hdqn_self"), ("other_checkpoint", "hdqn_other")):
            z = h[key]
            legs[name] = {"kernel": z["kernel"], "env_steps_per_s": z["env_steps_per_s"],
                          "kernel_ms_mean": z["kernel_ms_mean"], "frac_useful": z["frac_useful"]}
        legs["hdqn_goal_ring"] = {k: h["with_goal_ring"][k] for k in ("fused_env_steps_per_s",
                                                                     "separate_env_steps_per_s")}
    d = line.get("dropin_single_env")
    if d is not None:
        legs["dropin_single_env_us_per_step"] = {k: d[k]["us_per_step"] for k in ("host_dropin", "gpu_dropin",
                                                                                   "cpu_python_port")}
    out["legs"] = legs
    out["detail"] = "the full record is the 'bench detail:' line above"
    return out


if __name__ == "__main__":
    main()
