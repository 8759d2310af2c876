"""merging_gym for MI355X: the two-player on-ramp merging env, stepped by a HIP kernel.

Drop-in for the reference package (merging_gym/__init__.py:1-11): importing it registers
gym id "merging_env-v0" (plus the alias "merging-v0" and "merging_env_extend-v0") when gym
is importable. Without gym, `merging_gym.make(id)` builds the same envs.
"""

from .envs import MergeEnv, MergeEnvExtend, MergeVecEnv

__all__ = ["MergeEnv", "MergeEnvExtend", "MergeVecEnv", "ReplayRing", "make", "ENV_IDS"]


def __getattr__(name):  # ReplayRing loads the native library on first use only
    if name == "ReplayRing":
        from .replay import ReplayRing

        return ReplayRing
    raise AttributeError(name)

ENV_IDS = {
    "merging_env-v0": "merging_gym.envs:MergeEnv",
    "merging-v0": "merging_gym.envs:MergeEnv",
    "merging_env_extend-v0": "merging_gym.envs:MergeEnvExtend",
}


def register_with_gym(registration=None):
    """Register ENV_IDS with gym (merging_gym/__init__.py:3-11 in the reference). Runs at import
    when gym is importable; an id gym already holds (a re-import) is skipped, and any other
    failure propagates. Returns the ids registered by this call."""
    if registration is None:
        from gym.envs import registration
    known = getattr(registration.registry, "env_specs", registration.registry)  # gym 0.20 / >= 0.26
    added = []
    for env_id, entry in ENV_IDS.items():
        if env_id in known:
            continue
        registration.register(id=env_id, entry_point=entry)
        added.append(env_id)
    return added


try:
    import gym as _gym  # noqa: F401
except ImportError:  # this image has no gym: merging_gym.make() builds the same envs
    _gym = None
if _gym is not None:
    register_with_gym()


def make(env_id: str, **kwargs):
    """gym.make stand-in: `merging_gym.make("merging_env-v0")`."""
    import importlib

    try:
        entry = ENV_IDS[env_id]
    except KeyError:
        raise KeyError(f"unknown env id {env_id!r}; known: {sorted(ENV_IDS)}") from None
    mod, attr = entry.split(":")
    return getattr(importlib.import_module(mod), attr)(**kwargs)
