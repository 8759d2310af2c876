"""Chunk-level clocks of the persistent uniform-wave config-5 kernel (a diagnostic build,
tools/variants/lib_pclk.so from tools/uni_build_pclk.py, never shipped): per wave of blocks 0..63 and per 512-env chunk it
walks, s_memtime at the chunk start, after the env load, after the T-step loop and after the
env store, and s_memrealtime (100 MHz) at the chunk start and end.

    python tools/uni_chunk_clk.py tools/variants/lib_pclk.so
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ab_kernels as ab  # noqa: E402

f = np.load(os.path.join(ROOT, "tests", "golden", "dqn_checkpoints.npz"))
w = {k.split("/", 1)[1]: f[k] for k in f.files if k.startswith("l1/")}
lib = ab.bind(sys.argv[1])
lib.mg_debug_clocks.argtypes = [ctypes.c_void_p]
bed = ab.Bed(lib, 1 << 20, 16)
bed.pack_net(w)
bed.opp_net = bed.net
ev = ab.Events(1)
for _ in range(2400):  # ~2 s of back-to-back launches first
    bed.qrollout(0)
torch.cuda.synchronize()
bed.qrollout(0, ev.ev[0])
torch.cuda.synchronize()
launch_us = ev.ms(0) * 1e3
c = np.zeros(64 * 8 * 64 * 16, dtype=np.uint32)
assert lib.mg_debug_clocks(c.ctypes.data) == 0
c = c.reshape(64, 8, 64, 16).astype(np.int64)[:, :, 32:40]  # chunk slots (8 chunks per block at 2^20)
d = lambda a, b: (c[..., b] - c[..., a]) & 0xffffffff  # noqa: E731
load, loop, store, chunk = d(0, 1), d(1, 2), d(2, 3), d(0, 3)
rt_chunk = d(12, 13)
clock = np.median(chunk / np.maximum(rt_chunk, 1)) * 0.1
gap = (c[:, :, 1:, 12] - c[:, :, :-1, 13]) & 0xffffffff  # realtime ticks between one chunk's end and the next's start
span = (c[:, :, 7, 13] - c[:, :, 0, 12]) & 0xffffffff
print(f"launch {launch_us:.1f} us (16 steps); clock {clock:.3f} GHz")
print(f"per wave per chunk, median cycles: env load {np.median(load):.0f}, 16-step loop {np.median(loop):.0f} "
      f"({np.median(loop) / 16:.0f} per step), env store {np.median(store):.0f}; chunk {np.median(chunk):.0f}")
print(f"between chunks (realtime): median {np.median(gap) * 10:.0f} ns; block span, first chunk start to last end: "
      f"median {np.median(span) / 100:.1f} us, max {np.max(span) / 100:.1f} us (the launch {launch_us:.1f})")
xcd = np.arange(64) % 8
bspan = span.max(axis=1) / 100  # us, slowest wave of each block
bcyc = ((c[:, :, 7, 3] - c[:, :, 0, 0]) & 0xffffffff).max(axis=1)
bclk = bcyc / np.maximum(((c[:, :, 7, 13] - c[:, :, 0, 12]) & 0xffffffff).max(axis=1), 1) * 0.1
for x in range(8):
    m = xcd == x
    print(f"XCD {x}: block span median {np.median(bspan[m]):.1f} us (min {bspan[m].min():.1f}, max {bspan[m].max():.1f}), "
          f"cycles median {np.median(bcyc[m]) / 1e6:.3f} M, clock {np.median(bclk[m]):.3f} GHz")
