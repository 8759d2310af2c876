"""A recording stand-in for pygame 2.1.2 (test infrastructure only).

Neither this image nor the GPU box has pygame. The UI parity tests run the reference's
MergeEnv UI methods (merging_env.py:83-108, :241-395) against this package, run the build's
merging_gym UI against it too, and compare the two call logs: every surface, fill, blit,
draw primitive, text, display update and wait, with its arguments.

Only the pieces those methods touch exist. Rect(center=...) follows pygame 2.1.2 (a float
centre goes through a C (int) cast, x = cx - w // 2), Vector2 is fp64 with rotate(0) the
identity, as in tests/golden/gen_golden.py's non-recording stand-in.
"""

from . import display, draw, event, font, key, locals, math, surfarray, time  # noqa: F401
from ._rec import LOG, Rect, Surface, clear, record  # noqa: F401
from .locals import *  # noqa: F401,F403


def init():
    record("init")
    return (6, 0)


def quit():  # noqa: A001 - pygame's name
    record("quit")
