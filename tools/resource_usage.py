"""Per-kernel register / LDS / occupancy table of libmerging_hip (hipcc -Rpass-analysis).

    python tools/resource_usage.py [extra hipcc flags...]

Compiles merging-gym_amd/csrc/merging_hip.hip for gfx950 into a throw-away object and prints
one line per kernel: VGPRs, AGPRs, SGPRs, spills, scratch, LDS and the occupancy hipcc reports.
"""

from __future__ import annotations

import re
import subprocess
import sys
import tempfile
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "merging-gym_amd", "csrc", "merging_hip.hip")
FIELDS = ("VGPRs", "AGPRs", "SGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
          "Occupancy [waves/SIMD]", "LDS Size [bytes/block]")


def main(argv):
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off", "-fno-fast-math", "-I", os.path.join(ROOT, "include"), "-o",
               os.path.join(td, "x.so"), SRC, "-Rpass-analysis=kernel-resource-usage", *argv]
        out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode:
        sys.stderr.write(out.stderr)
        return out.returncode
    rows, cur = [], None
    for line in out.stderr.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    short = lambda s: re.sub(r"_ZN12_GLOBAL__N_1\d+", "", s)[:48]  # noqa: E731
    print(f"{'kernel':48s} " + " ".join(f"{f.split(' ')[0][:6]:>6s}" for f in FIELDS))
    for r in rows:
        print(f"{short(r['name']):48s} " + " ".join(f"{r.get(f, '-'):>6s}" for f in FIELDS))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
