"""In-process A/B of libmerging_hip.so build variants (cdna_hip_programming.md §5.4 rule 24).

    python tools/ab_kernels.py merging-gym_amd/variants/lib_*.so [--envs N] [--rounds R]

Every variant library is loaded into the same process and run on the same GPU in interleaved
rounds; kernel time per launch comes from events recorded by the dispatch packet
(mg_time_next_launch). Reports the median / min per variant for the step kernel
(mg_step_random) and the fused rollout (mg_rollout_random, T steps per launch).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from merging_gym import _native as nat  # noqa: E402  (struct definitions)


def bind(path):
    lib = ctypes.CDLL(path)
    PP, SP, OP, STP = (ctypes.POINTER(nat.Params), ctypes.POINTER(nat.State), ctypes.POINTER(nat.Outputs),
                       ctypes.POINTER(nat.Stats))
    P = ctypes.c_void_p
    lib.mg_params_default.argtypes = [PP]
    lib.mg_reset.argtypes = [PP, SP, P, OP, ctypes.c_int64, P]
    lib.mg_step_random.argtypes = [PP, SP, P, P, OP, STP, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                   ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint32, P]
    lib.mg_rollout_random.argtypes = [PP, SP, ctypes.POINTER(nat.Traj), STP, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_uint32, P]
    lib.mg_time_next_launch.argtypes = [P, P]
    lib.mg_qnet_packed_bytes.restype = ctypes.c_size_t
    lib.mg_qnet_pack.argtypes = [P] * 6 + [ctypes.c_int32, ctypes.c_int32, P, P]
    lib.mg_rollout_qnet.argtypes = [PP, SP, ctypes.POINTER(nat.Traj), STP, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32, P, ctypes.c_int32,
                                    ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint64, P, ctypes.c_uint32, P]
    return lib


class Bed:
    """State + outputs for one variant (separate buffers so variants do not share cache lines)."""

    def __init__(self, lib, n, T):
        self.lib, self.n, self.T = lib, n, T
        dev = "cuda"
        f = lambda: torch.empty(n, dtype=torch.float64, device=dev)  # noqa: E731
        self.t = [f() for _ in range(6)] + [torch.empty(n, dtype=torch.int16, device=dev)]
        self.obs = torch.empty((n, 10), device=dev)
        self.rew = torch.empty((n, 2), device=dev)
        self.done = torch.empty(n, dtype=torch.uint8, device=dev)
        self.coll = torch.empty(n, dtype=torch.uint8, device=dev)
        self.fobs = torch.empty((n, 10), device=dev)
        self.a = torch.empty((2, n), dtype=torch.int8, device=dev)
        self.ep_stats = torch.zeros((n, 8), dtype=torch.float64, device=dev)  # mg_episode_stats [n], 64 B each
        self.tobs = torch.empty((T, n, 10), device=dev)
        self.trew = torch.empty((T, n, 2), device=dev)
        self.tdone = torch.empty((T, n), dtype=torch.uint8, device=dev)
        self.tcoll = torch.empty((T, n), dtype=torch.uint8, device=dev)
        self.ta = torch.empty((2, T, n), dtype=torch.int8, device=dev)
        self.params = nat.Params()
        lib.mg_params_default(ctypes.byref(self.params))
        self.params.angle0 = float(np.arctan2(1000, 30000))
        self.state = nat.State(*(x.data_ptr() for x in self.t))
        self.out = nat.Outputs(self.obs.data_ptr(), self.rew.data_ptr(), self.done.data_ptr(),
                               self.coll.data_ptr(), None,
                               None if os.environ.get("MG_AB_NOFOBS") == "1" else self.fobs.data_ptr(), None, None)
        self.stats = (nat.Stats() if os.environ.get("MG_AB_NOSTATS") == "1"
                      else nat.Stats(self.ep_stats.data_ptr()))
        self.twon = torch.zeros((T, (n + 63) // 64), dtype=torch.int64, device=dev)
        won = self.twon.data_ptr() if os.environ.get("MG_AB_WON") == "1" else None
        self.traj = nat.Traj(self.tobs.data_ptr(), self.trew.data_ptr(), self.tdone.data_ptr(),
                             self.tcoll.data_ptr(), self.ta[0].data_ptr(), self.ta[1].data_ptr(), None, won)
        if os.environ.get("MG_AB_FLAGS") == "1":  # interleaved (a1, a2, done, coll) per env-step
            self.tflags = torch.empty((T, n, 4), dtype=torch.uint8, device=dev)
            self.traj = nat.Traj(self.tobs.data_ptr(), self.trew.data_ptr(), None, None, None, None, None, won,
                                 self.tflags.data_ptr())
        self.k = 0
        assert lib.mg_reset(ctypes.byref(self.params), ctypes.byref(self.state), None, None, n, None) == 0

    def step(self, ev=None):
        if ev:
            self.lib.mg_time_next_launch(*ev)
        rc = self.lib.mg_step_random(ctypes.byref(self.params), ctypes.byref(self.state), self.a[0].data_ptr(),
                                     self.a[1].data_ptr(), ctypes.byref(self.out), ctypes.byref(self.stats),
                                     self.n, 0, 5, self.k, 1, 1, torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        self.k += 1

    def pack_net(self, weights, attr="net"):
        ts = [torch.as_tensor(weights[k]).cuda().contiguous() for k in
              ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "out.weight", "out.bias")]
        setattr(self, attr + "_src", ts)
        net = torch.empty(self.lib.mg_qnet_packed_bytes(), dtype=torch.uint8, device="cuda")
        assert self.lib.mg_qnet_pack(*(t.data_ptr() for t in ts), 10, 5, net.data_ptr(), None) == 0
        setattr(self, attr, net)

    def qrollout(self, opp, ev=None):
        if ev:
            self.lib.mg_time_next_launch(*ev)
        thr = 3255688812  # round(Phi(0.7) * 2^32)
        rc = self.lib.mg_rollout_qnet(ctypes.byref(self.params), ctypes.byref(self.state), ctypes.byref(self.traj),
                                      ctypes.byref(self.stats), self.n, 0, 5, self.k, self.T, self.net.data_ptr(), 5,
                                      thr, opp, thr, self.opp_net.data_ptr() if opp == 3 else None, 1,
                                      torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        self.k += self.T

    def rollout(self, ev=None):
        if ev:
            self.lib.mg_time_next_launch(*ev)
        rc = self.lib.mg_rollout_random(ctypes.byref(self.params), ctypes.byref(self.state),
                                        ctypes.byref(self.traj), ctypes.byref(self.stats), self.n, 0, 5, self.k,
                                        self.T, 1, 1, torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        self.k += self.T


class Events:
    def __init__(self, n):
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        self.hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        self.ev = []
        for _ in range(n):
            a, b = ctypes.c_void_p(), ctypes.c_void_p()
            self.hip.hipEventCreate(ctypes.byref(a))
            self.hip.hipEventCreate(ctypes.byref(b))
            self.ev.append((a, b))

    def ms(self, k):
        v = ctypes.c_float()
        self.hip.hipEventElapsedTime(ctypes.byref(v), *self.ev[k])
        return v.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--rollouts", type=int, default=4)
    ap.add_argument("--warm", type=int, default=200, help="single steps before timing (1000+: steady state)")
    ap.add_argument("--qnet", action="store_true", help="A/B the fused Q-net rollout instead")
    ap.add_argument("--replay", action="store_true", help="A/B mg_replay_store instead")
    a = ap.parse_args()
    if a.qnet:
        return main_qnet(a)
    if a.replay:
        return main_replay(a)
    beds = {os.path.basename(p): Bed(bind(p), a.envs, a.T) for p in a.libs}
    ev = Events(max(a.steps, a.rollouts))
    res = {k: {"step": [], "rollout": [], "step_wall": [], "rollout_wall": []} for k in beds}
    import time
    for b in beds.values():  # warm up (and get into mixed episode phases)
        for _ in range(a.warm):
            b.step()
        b.rollout()
    torch.cuda.synchronize()
    for r in range(a.rounds):
        order = list(beds) if r % 2 == 0 else list(reversed(beds))
        for name in order:
            b = beds[name]
            for j in range(a.steps):
                b.step(ev.ev[j])
            torch.cuda.synchronize()
            res[name]["step"] += [ev.ms(j) for j in range(a.steps)]
            for j in range(a.rollouts):
                b.rollout(ev.ev[j])
            torch.cuda.synchronize()
            res[name]["rollout"] += [ev.ms(j) / a.T for j in range(a.rollouts)]
            # back-to-back wall clock (no events): kernel + launch boundary
            t0 = time.perf_counter()
            for j in range(a.steps):
                b.step()
            torch.cuda.synchronize()
            res[name]["step_wall"].append((time.perf_counter() - t0) / a.steps * 1e3)
            t0 = time.perf_counter()
            for j in range(a.rollouts):
                b.rollout()
            torch.cuda.synchronize()
            res[name]["rollout_wall"].append((time.perf_counter() - t0) / (a.rollouts * a.T) * 1e3)
    out = {}
    for name, d in res.items():
        s, ro = d["step"], d["rollout"]
        out[name] = {"step_us_median": 1e3 * statistics.median(s), "step_us_min": 1e3 * min(s),
                     "step_TBps": 152 * a.envs / (statistics.median(s) * 1e-3) / 1e12,
                     "rollout_us_per_step_median": 1e3 * statistics.median(ro),
                     "rollout_us_per_step_min": 1e3 * min(ro),
                     "rollout_TBps": (52 + 100 / a.T) * a.envs / (statistics.median(ro) * 1e-3) / 1e12,
                     "step_wall_us_median": 1e3 * statistics.median(d["step_wall"]),
                     "rollout_wall_us_per_step_median": 1e3 * statistics.median(d["rollout_wall"])}
        print(f"{name:24s} step {out[name]['step_us_median']:7.2f} us (min {out[name]['step_us_min']:6.2f}, "
              f"{out[name]['step_TBps']:.2f} TB/s)   rollout {out[name]['rollout_us_per_step_median']:6.2f} us/step "
              f"(min {out[name]['rollout_us_per_step_min']:6.2f}, {out[name]['rollout_TBps']:.2f} TB/s)  "
              f"wall: step {out[name]['step_wall_us_median']:6.2f} rollout {out[name]['rollout_wall_us_per_step_median']:6.2f}",
              flush=True)
    print(json.dumps({"envs": a.envs, "T": a.T, "results": out}))


def main_qnet(a):
    import time

    f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    w = {k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l1/")}
    w3 = {k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l3/")}  # main.py Strategy_OP "L1"
    beds = {os.path.basename(p): Bed(bind(p), a.envs, a.T) for p in a.libs}
    for b in beds.values():
        b.pack_net(w)
        b.pack_net(w3, "opp_net")
        for _ in range(a.warm):
            b.step()
    ev = Events(a.rollouts)
    res = {k: {0: [], 2: [], 3: []} for k in beds}
    torch.cuda.synchronize()
    for r in range(a.rounds):
        order = list(beds) if r % 2 == 0 else list(reversed(beds))
        for name in order:
            b = beds[name]
            for opp in (0, 2, 3):
                for j in range(a.rollouts):
                    b.qrollout(opp, ev.ev[j])
                torch.cuda.synchronize()
                res[name][opp] += [ev.ms(j) / a.T for j in range(a.rollouts)]
    for name, d in res.items():
        print(f"{name:24s} qnet(none) {1e3 * statistics.median(d[0]):7.2f} us/step   "
              f"qnet(self) {1e3 * statistics.median(d[2]):7.2f} us/step   "
              f"qnet(other) {1e3 * statistics.median(d[3]):7.2f} us/step", flush=True)


def main_replay(a):
    """mg_replay_store of one rollout's trajectory (T x envs transitions, made once with the
    default library) into a 2^24-row ring, per variant; events on the current stream."""
    from merging_gym import MergeVecEnv

    env = MergeVecEnv(a.envs, device="cuda")
    for k in range(230):
        env.step_random(5, step_idx=k)
    obs0 = env.observe().clone()
    traj = env.rollout_random(a.T, 5, first_step=230)
    ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    tr = nat.Transitions(ptr(obs0), ptr(traj["obs"]), ptr(traj["final_observation"]), None,
                         ptr(traj["rew"]), None, ptr(traj["won_mask"]), None, None, None, ptr(traj["flags"]))
    cap = 1 << 24
    beds = {}
    for p in a.libs:
        lib = ctypes.CDLL(p)
        lib.mg_replay_scratch_bytes.argtypes = [ctypes.c_int64, ctypes.c_int32]
        lib.mg_replay_scratch_bytes.restype = ctypes.c_size_t
        lib.mg_replay_store.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                        ctypes.POINTER(nat.Transitions), ctypes.c_int64, ctypes.c_int32,
                                        ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        nbytes = lib.mg_replay_scratch_bytes(a.envs, a.T)
        beds[os.path.basename(p)] = (lib, torch.zeros((cap, 22), device="cuda"),
                                     torch.zeros(1, dtype=torch.int64, device="cuda"),
                                     torch.zeros(nbytes // 8 + 1, dtype=torch.int64, device="cuda"), nbytes)

    def store(b):
        lib, ring, ctr, scr, nbytes = b
        rc = lib.mg_replay_store(ring.data_ptr(), ctr.data_ptr(), cap, 22, ctypes.byref(tr), a.envs, a.T, 1,
                                 scr.data_ptr(), nbytes, torch.cuda.current_stream().cuda_stream)
        assert rc == 0

    for b in beds.values():
        store(b)
    torch.cuda.synchronize()
    res = {k: [] for k in beds}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.rollouts)]
    for r in range(a.rounds):
        for name in (list(beds) if r % 2 == 0 else list(reversed(beds))):
            for j in range(a.rollouts):
                ev[2 * j].record()
                store(beds[name])
                ev[2 * j + 1].record()
            torch.cuda.synchronize()
            res[name] += [ev[2 * j].elapsed_time(ev[2 * j + 1]) for j in range(a.rollouts)]
    kept = int(beds[next(iter(beds))][2].item()) // (1 + a.rounds * a.rollouts)
    for name, d in res.items():
        print(f"{name:28s} store {1e3 * statistics.median(d):8.1f} us (min {1e3 * min(d):8.1f})  "
              f"{kept / (statistics.median(d) * 1e-3):.3e} transitions/s", flush=True)


if __name__ == "__main__":
    main()
