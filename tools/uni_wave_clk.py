"""Per-wave occupancy of the persistent uniform-wave config-5 kernel with work items (a
diagnostic build, tools/variants/lib_dclk.so from tools/uni_build_dclk.py, never shipped): for each wave of blocks 0..63 the
realtime (100 MHz) at kernel entry, at its first item and at its exit, and the s_memtime cycles it
spent inside items, against the launch's own event time.

    python tools/uni_wave_clk.py tools/variants/lib_dclk.so
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
for _ in range(2400):
    bed.qrollout(0)
torch.cuda.synchronize()
bed.qrollout(0, ev.ev[0])
torch.cuda.synchronize()
launch_us = ev.ms(0) * 1e3
c = np.zeros(64 * 8 * 64 * 16, dtype=np.uint32)
assert lib.mg_debug_clocks(c.ctypes.data) == 0
c = c.reshape(64, 8, 64, 16).astype(np.int64)[:, :, 0]
u = lambda x: x & 0xffffffff  # noqa: E731
t_entry = c[..., 12]
t0 = t_entry.min()
entry_us = u(t_entry - t0) / 100
first_us = u(c[..., 13] - t0) / 100
exit_us = u(c[..., 14] - t0) / 100
cyc = u(c[..., 2] - c[..., 0])
clock = np.median(cyc / np.maximum(u(c[..., 14] - c[..., 12]), 1)) * 0.1
busy_us = c[..., 3] / (clock * 1e3)
print(f"launch {launch_us:.1f} us; clock {clock:.3f} GHz; items per wave: min {c[..., 4].min()}, median "
      f"{np.median(c[..., 4]):.0f}, max {c[..., 4].max()}")
print(f"kernel entry (from the first block's): median {np.median(entry_us):.1f} us, max {entry_us.max():.1f}")
print(f"first item starts: median {np.median(first_us):.1f} us; wave exits: median {np.median(exit_us):.1f}, "
      f"min {exit_us.min():.1f}, max {exit_us.max():.1f}")
print(f"busy inside items per wave: median {np.median(busy_us):.1f} us, min {busy_us.min():.1f}, max {busy_us.max():.1f}")
blk_exit = exit_us.max(axis=1)
print(f"block exits: median {np.median(blk_exit):.1f}, min {blk_exit.min():.1f}, max {blk_exit.max():.1f}; "
      f"within-block spread of wave exits: median {np.median(blk_exit - exit_us.min(axis=1)):.1f} us")
