"""Phase clocks of the config-5 kernel (tools/clk_variant.py q5 / q5base builds): per phase, the
working time of the Q-net waves (0-3) and of the env waves (4-7) from the phase start to their
closing barrier, the phase length, and the median time of the k-th forward of a phase, averaged
over blocks 0..63 and the middle phases of a 16-step launch at 2^20 envs with the bench's
checkpoints (l1 ego; opponents none / self / l3).

    python tools/clk_probe_qnet.py tools/variants/lib_clk_*.so
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))

import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from merging_gym import MergeVecEnv, _native  # noqa: E402
from merging_gym.policy import QNet  # noqa: E402

libs = {os.path.basename(p): _native._load(p) for p in sys.argv[1:]}
env = MergeVecEnv(1 << 20, device="cuda", final_observation=False)
k = 1_000_000
for _ in range(100):
    env.rollout_random(16, 7, first_step=k)
    k += 16
f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
for name, lib in libs.items():
    _native.lib = lib
    nets = {key: QNet.from_state_dict({n.split("/", 1)[1]: f[n] for n in f.files if n.startswith(key + "/")},
                                      device="cuda") for key in ("l1", "l3")}
    lib.mg_debug_clocks.argtypes = [ctypes.c_void_p]
    for leg, opp in (("none", "none"), ("self", "self"), ("other", nets["l3"])):
        for _ in range(4):
            env.rollout_qnet(16, nets["l1"], 5, opponent=opp, first_step=k, final_observation=False)
            k += 16
        torch.cuda.synchronize()
        buf = np.zeros(64 * 8 * 64 * 16, np.uint32)
        assert lib.mg_debug_clocks(buf.ctypes.data) == 0
        c = buf.reshape(64, 8, 64, 16).astype(np.int64)
        ph = range(6, 30)
        q_work = np.mean([(c[:, w, p, 1] - c[:, w, p, 0]) for w in range(4) for p in ph])
        e_work = np.mean([(c[:, w, p, 1] - c[:, w, p, 0]) for w in range(4, 8) for p in ph])
        length = np.mean([(c[:, 0, p + 1, 0] - c[:, 0, p, 0]) for p in ph])
        qmax = np.mean([np.max(c[:, 0:4, p, 1] - c[:, 0:4, p, 0], axis=1) for p in ph])
        print(f"{name:20s} {leg:5s}  phase {length:8.0f}  Q work {q_work:8.0f} (max of 4 {qmax:8.0f})  env work {e_work:8.0f}"
              "  (s_memtime cycles)", flush=True)
        per_wave = [np.mean([(c[:, w, p, 1] - c[:, w, p, 0]) for p in ph]) for w in range(4)]
        print("    Q work per wave " + " ".join(f"{x:7.0f}" for x in per_wave), flush=True)
        marks = []
        for s_ in range(6):
            d = np.concatenate([(c[:, w, p, 8 + s_] - c[:, w, p, 2 + s_]) for w in range(4) for p in ph])
            ok = (d > 0) & (d < 1e6)
            if ok.mean() > 0.05:
                marks.append(f"fwd{s_} {np.median(d[ok]):6.0f} ({100 * ok.mean():.0f}%)")
        if marks:
            print("    " + "  ".join(marks), flush=True)
