"""Build provenance (CPU): libmerging_hip.so carries the sha256 of the source, header and flags it
was built from (mg_build_info "src <sha>", merging_gym/build.py), build() recompiles when the tree's
differs, and the package refuses or rebuilds a stale in-tree library at import."""
import os

import pytest

from merging_gym import _native, build


def test_loaded_library_matches_this_tree():
    info = _native.build_info()
    assert f"src {build.source_sha()}" in info, (info, build.source_sha())
    assert build.is_current(build.OUT)


def test_touching_the_source_makes_the_library_stale(tmp_path):
    src, hdr, lib = tmp_path / "k.hip", tmp_path / "k.h", tmp_path / "lib.so"
    src.write_text("__global__ void k() {}\n")
    hdr.write_text("#define X 1\n")
    sha = build.source_sha(str(src), str(hdr))
    lib.write_bytes(b"\x7fELF...clang; ABI 20; gfx950, -ffp-contract=off; src " + sha.encode() + b"\x00rest")
    assert build.embedded_sha(str(lib)) == sha
    assert build.is_current(str(lib), build.source_sha(str(src), str(hdr)))
    src.write_text("__global__ void k() { }\n")  # one byte more: another source
    assert not build.is_current(str(lib), build.source_sha(str(src), str(hdr)))
    hdr.write_text("#define X 2\n")
    assert build.source_sha(str(src), str(hdr)) != sha


def test_a_library_without_a_source_sha_is_stale(tmp_path):
    lib = tmp_path / "old.so"
    lib.write_bytes(b"\x7fELF... ABI 20; gfx950, -ffp-contract=off\x00")  # a round-4 build
    assert build.embedded_sha(str(lib)) is None
    assert not build.is_current(str(lib))
    assert build.embedded_sha(str(tmp_path / "missing.so")) is None


@pytest.mark.skipif(not os.path.exists(build.OUT), reason="library not built")
def test_build_skips_a_current_library():
    before = os.path.getmtime(build.OUT)
    assert build.build() == build.OUT  # current by content: no hipcc run
    assert os.path.getmtime(build.OUT) == before


_RACE = r"""
import os, sys
sys.path.insert(0, {pkgroot!r})
from merging_gym import build
build.OUT = os.path.join({d!r}, "libmerging_hip.so")
build.PKG = {d!r}
print(build.build())
"""


def test_concurrent_builds_compile_once(tmp_path):
    """N ranks importing a stale library used to run hipcc into one shared `.tmp` path.
    build() now holds an fcntl lock next to the library, re-checks it under the lock and writes a
    per-process temporary file: four processes racing on a stale library run the compiler once and
    leave an intact library (a stand-in compiler that takes a second and logs each run)."""
    import subprocess
    import sys

    d = tmp_path / "pkg"
    d.mkdir()
    (d / "libmerging_hip.so").write_bytes(b"stale, no source sha")
    log = tmp_path / "runs.log"
    fake = tmp_path / "hipcc"
    fake.write_text("#!/usr/bin/env python3\nimport sys, time\n"
                    f"open({str(log)!r}, 'a').write('run\\n')\n"
                    "time.sleep(1.0)\n"
                    "args = sys.argv[1:]\nout = args[args.index('-o') + 1]\n"
                    "sha = [a for a in args if a.startswith('-DMG_SRC_SHA=')][0].split('=', 1)[1].strip('\"')\n"
                    "open(out, 'wb').write(b'ELF; src ' + sha.encode() + b'\\x00built')\n")
    fake.chmod(0o755)
    pkgroot = os.path.dirname(os.path.dirname(os.path.abspath(build.__file__)))
    env = dict(os.environ, HIPCC=str(fake))
    code = _RACE.format(pkgroot=pkgroot, d=str(d))
    procs = [subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
             for _ in range(4)]
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-400:] for o in outs]
    assert log.read_text().count("run") == 1
    assert build.embedded_sha(str(d / "libmerging_hip.so")) == build.source_sha()
    assert not [f for f in os.listdir(d) if f.endswith(".tmp")]
