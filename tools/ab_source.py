"""Build an A/B variant of libmerging_hip.so from an edited copy of the source (the shipped
source has no compile-time knobs): each argument after the name is `old=>new`, a literal text
replacement that must match exactly once (`old=>>new`: every occurrence).

    python tools/ab_source.py ahead6 'kQGlobalAhead = 3;=>kQGlobalAhead = 6;'
    -> tools/variants/lib_ahead6.so (same flags as merging_gym/build.py)
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
from merging_gym import build  # noqa: E402


def main(argv):
    name, edits = argv[0], argv[1:]
    src = open(build.SRC).read()
    for e in edits:
        every = "=>>" in e  # `old=>>new`: replace every occurrence (at least one)
        old, new = e.split("=>>" if every else "=>", 1)
        n = src.count(old)
        if n == 0 or (n != 1 and not every):
            raise SystemExit(f"{name}: '{old}' matches {n} times")
        src = src.replace(old, new)
    os.makedirs(os.path.join(ROOT, "tools", "variants"), exist_ok=True)
    out = os.path.join(ROOT, "tools", "variants", f"lib_{name}.so")
    with tempfile.NamedTemporaryFile("w", suffix=".hip", dir=os.path.dirname(build.SRC), delete=False) as f:
        f.write(src)
        tmp = f.name
    try:
        subprocess.check_call([build.hipcc(), *build.HIPCC_FLAGS, "-I", build.INCLUDE, "-o", out, tmp])
    finally:
        os.unlink(tmp)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1:])
