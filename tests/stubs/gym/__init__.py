"""A stand-in for gym 0.20.0 (test infrastructure only; gym is in neither this image nor the
GPU box). It carries the pieces merging_gym's registration and the reference's callers use:
`gym.make(id)` returning an env whose `.unwrapped` is the env itself (scripts/hdqn.py:26,
main.py:20, human_player.py:27), the registry behind `gym.envs.registration.register`
(merging_gym/__init__.py:3-11 in the reference), and `gym.error.Error`, which gym 0.20 raises
when an id is registered twice."""

from . import error, spaces  # noqa: F401
from .core import Env  # noqa: F401
from .envs.registration import make, register, registry, spec  # noqa: F401
