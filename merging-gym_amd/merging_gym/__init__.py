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

try:  # pragma: no cover - gym is not installed in this image
    from gym.envs.registration import register as _register

    for _id, _entry in ENV_IDS.items():
        try:
            _register(id=_id, entry_point=_entry)
        except Exception:  # noqa: BLE001 - already registered
            pass
except Exception:  # noqa: BLE001
    pass


def make(env_id: str, **kwargs):
    """gym.make stand-in: `merging_gym.make("merging_env-v0")`."""
    import importlib

    try:
        entry = ENV_IDS[env_id]
    except KeyError:
        raise KeyError(f"unknown env id {env_id!r}; known: {sorted(ENV_IDS)}") from None
    mod, attr = entry.split(":")
    return getattr(importlib.import_module(mod), attr)(**kwargs)
