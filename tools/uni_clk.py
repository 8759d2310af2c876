"""Per-wave clocks inside the uniform-wave config-5 kernel (tools/variants/qnet_uniform_waves.patch),
a diagnostic build, never shipped: blocks 0..63 stamp s_memtime around each step's forward and
step, and s_memrealtime (100 MHz) at the first and last step, into a device array that
mg_debug_clocks copies out. Answers whether a 64-env forward takes the stand-alone
micro-benchmark's cycles (tools/micro/qfwd32_waves.hip: 8,333 per wave with two waves per SIMD)
inside the rollout kernel, and at what clock.

    python tools/uni_clk.py build        # here: writes tools/variants/lib_uniclk{,_fwd}.so
    python tools/uni_clk.py run          # on the GPU box
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "merging-gym_amd", "csrc", "merging_hip.hip")
PATCH = os.path.join(ROOT, "tools", "variants", "qnet_uniform_waves.patch")

HDR = '''
__device__ unsigned g_mg_clk[64 * 8 * 64 * 16];
#define MG_CLK(ev) do { if (blockIdx.x < 64 && (threadIdx.x & 63) == 0 && t < 64) \\
  g_mg_clk[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 64 + t) * 16 + (ev)] = static_cast<unsigned>(__builtin_amdgcn_s_memtime()); } while (0)
#define MG_RT(ev) do { if (blockIdx.x < 64 && (threadIdx.x & 63) == 0 && t < 64) \\
  g_mg_clk[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 64 + t) * 16 + (ev)] = static_cast<unsigned>(__builtin_amdgcn_s_memrealtime()); } while (0)
extern "C" int mg_debug_clocks(void* dst) { return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_mg_clk), sizeof(g_mg_clk)); }
'''

EDITS = [
    ("  for (int t = 0; t < R.num_steps; ++t) {\n    // park the env's state",
     "  for (int t = 0; t < R.num_steps; ++t) {\n    MG_CLK(0); MG_RT(12);\n    // park the env's state"),
    ("    qnet32_forward(lds_net, wt, 0, false, q);  // every read of the wave's rows precedes the writes below\n",
     "    MG_CLK(2);\n    qnet32_forward(lds_net, wt, 0, false, q);  // every read of the wave's rows precedes the writes below\n"
     "    asm volatile(\"\" :: \"v\"(q[0]), \"v\"(q[1]), \"v\"(q[2]), \"v\"(q[3]), \"v\"(q[4]));\n    MG_CLK(8);\n"),
    ("    store_won_mask(R.T.won_mask, won[0], t, R.n, wbase, wrows);\n    wave_store_obs_n<1>(wt, r,",
     "    MG_CLK(3);\n    store_won_mask(R.T.won_mask, won[0], t, R.n, wbase, wrows);\n    wave_store_obs_n<1>(wt, r,"),
]
# forward only: the step replaced by a copy of q into the observation (as the noS A/B variant)
FWD_ONLY = ("""    qnet_policy_step_n<OPP, 1, CHECKED>(R, e, r, wbase + lane, live, t, greedy1, greedy2, won, qr, keep, pend, un,
                                        nullptr, nullptr);""",
            """    won[0] = false; for (int k = 0; k < kObs; ++k) r[0].o[k] = q[k % 5] * 0.5f + static_cast<float>(greedy1[0]); (void)un;""")


def build():
    src = subprocess.run(["git", "-C", ROOT, "show", "HEAD:merging-gym_amd/csrc/merging_hip.hip"],
                         capture_output=True, text=True, check=True).stdout
    tmp = os.path.join(ROOT, "merging-gym_amd", "csrc", ".uniclk_base.hip")
    open(tmp, "w").write(src)
    # apply the patch to the copy: patch(1) reads the unified diff
    subprocess.run(["patch", "-s", tmp, PATCH], check=True)
    base = open(tmp).read()
    os.remove(tmp)
    anchor = "constexpr int kQUniThreads = 512;"
    assert anchor in base
    for name, fwd_only in (("uniclk", False), ("uniclk_fwd", True)):
        s = base.replace(anchor, HDR + anchor, 1)
        for old, new in EDITS:
            assert s.count(old) == 1, old
            s = s.replace(old, new)
        if fwd_only:
            assert s.count(FWD_ONLY[0]) == 1
            s = s.replace(FWD_ONLY[0], FWD_ONLY[1])
        path = os.path.join(ROOT, "merging-gym_amd", "csrc", f".{name}.hip")
        open(path, "w").write(s)
        out = os.path.join(ROOT, "tools", "variants", f"lib_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-ffp-contract=off", "-fno-fast-math", "-w", "-DMG_SRC_SHA=\"uniclk\"",
                        "-I", os.path.join(ROOT, "include"), "-o", out, path], check=True)
        os.remove(path)
        print(out)


def run():
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import ab_kernels as ab

    f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
    w = {k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l1/")}
    for name in ("uniclk", "uniclk_fwd"):
        lib = ab.bind(os.path.join(ROOT, "tools", "variants", f"lib_{name}.so"))
        lib.mg_debug_clocks.argtypes = [ctypes.c_void_p]
        bed = ab.Bed(lib, 1 << 20, 16)
        bed.pack_net(w)
        bed.opp_net = bed.net
        for _ in range(2400):  # ~2 s of back-to-back launches before the stamped one (the guide's clock check)
            bed.qrollout(0)
        torch.cuda.synchronize()
        bed.qrollout(0)
        torch.cuda.synchronize()
        c = np.zeros(64 * 8 * 64 * 16, dtype=np.uint32)
        assert lib.mg_debug_clocks(c.ctypes.data) == 0
        c = c.reshape(64, 8, 64, 16).astype(np.int64)[:, :, :16]  # 16 steps per launch
        fwd = (c[..., 8] - c[..., 2]) & 0xffffffff
        it = (c[:, :, 1:, 0] - c[:, :, :-1, 0]) & 0xffffffff
        tail = (c[..., 3] - c[..., 8]) & 0xffffffff
        cyc = (c[:, :, 15, 0] - c[:, :, 0, 0]) & 0xffffffff
        rt = (c[:, :, 15, 12] - c[:, :, 0, 12]) & 0xffffffff
        clock = np.median(cyc / np.maximum(rt, 1)) * 0.1  # GHz (s_memrealtime ticks at 100 MHz)
        print(f"{name}: per wave: forward median {np.median(fwd):.0f} cycles, step + q-row / argmax "
              f"{np.median(tail):.0f}, whole iteration {np.median(it):.0f}; clock {clock:.3f} GHz; "
              f"per SIMD (2 waves) per 64 envs {np.median(it) / 2:.0f} cycles", flush=True)


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else run()
