"""Build libmerging_hip.so in-tree: `python -m merging_gym.build`.

hipcc --offload-arch=gfx950, -ffp-contract=off (the step's fp64 arithmetic must not be
fused: positions and arrival tests are compared bit-for-bit with the reference's floats).
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)            # merging-gym_amd/
REPO = os.path.dirname(ROOT)           # repository root (include/)
SRC = os.path.join(ROOT, "csrc", "merging_hip.hip")
INCLUDE = os.path.join(REPO, "include")
OUT = os.path.join(PKG, "libmerging_hip.so")

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off", "-fno-fast-math", "-Wall"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise FileNotFoundError("hipcc not found (ROCm not installed?)")


def build(force: bool = False, verbose: bool = False) -> str:
    deps = [SRC, os.path.join(INCLUDE, "merging_hip.h"), __file__]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    tmp = OUT + ".tmp"
    cmd = [hipcc(), *HIPCC_FLAGS, "-I", INCLUDE, "-o", tmp, SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
