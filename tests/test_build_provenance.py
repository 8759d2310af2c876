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
