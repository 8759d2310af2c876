"""Build libmerging_hip.so in-tree: `python -m merging_gym.build`.

hipcc --offload-arch=gfx950, -ffp-contract=off (the step's fp64 arithmetic must not be
fused: positions and arrival tests are compared bit-for-bit with the reference's floats).
The library carries the sha256 of the source, header and flags it was built from (mg_build_info);
build() recompiles when that differs from the tree's, and merging_gym._native refuses (or rebuilds)
a stale in-tree library at import.
"""

from __future__ import annotations

import hashlib
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


HEADER = os.path.join(INCLUDE, "merging_hip.h")


def source_sha(src: str = SRC, header: str = HEADER) -> str:
    """sha256 (first 16 hex digits) of the kernel source, the C-ABI header and the compiler flags:
    embedded in the library (mg_build_info "src <sha>") so a build can be matched to its tree."""
    h = hashlib.sha256()
    for path in (src, header):
        with open(path, "rb") as f:
            h.update(f.read())
    h.update(" ".join(HIPCC_FLAGS).encode())
    return h.hexdigest()[:16]


def embedded_sha(lib_path: str) -> str | None:
    """The source sha a built library carries (mg_build_info's "src <sha>"), read from its bytes
    without loading it; None for a library built before round 5."""
    try:
        with open(lib_path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(b"; src ")
    return data[i + 6:i + 22].decode("ascii", "replace") if i >= 0 else None


def is_current(lib_path: str = OUT, sha: str | None = None) -> bool:
    """The library at lib_path was built from this tree's source and header (by content, not mtime)."""
    return embedded_sha(lib_path) == (sha or source_sha())


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile OUT unless it is current. Several processes may get here at once (the ranks of a
    multi-rank launch, each importing a stale library): an fcntl lock next to OUT serialises them,
    the current-check is repeated under it so only the first one compiles, and each compile writes
    its own temporary file, moved into place atomically."""
    import fcntl
    import tempfile

    sha = source_sha()
    if not force and os.path.exists(OUT) and is_current(OUT, sha):
        return OUT
    with open(OUT + ".lock", "a+") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            if not force and os.path.exists(OUT) and is_current(OUT, sha):
                return OUT  # another process built it while this one waited
            fd, tmp = tempfile.mkstemp(prefix=".libmerging_hip.", suffix=".so.tmp", dir=PKG)
            os.close(fd)
            try:
                cmd = [hipcc(), *HIPCC_FLAGS, f'-DMG_SRC_SHA="{sha}"', "-I", INCLUDE, "-o", tmp, SRC]
                if verbose:
                    print(" ".join(cmd), file=sys.stderr)
                subprocess.check_call(cmd)
                os.chmod(tmp, 0o755)
                os.replace(tmp, OUT)
            finally:
                if os.path.exists(tmp):
                    os.unlink(tmp)
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
