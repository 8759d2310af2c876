"""gym 0.20's EnvRegistry: register() refuses an id twice with gym.error.Error; make() imports
the "module:attr" entry point and calls it with the kwargs."""

import importlib

from .. import error


class EnvSpec:
    def __init__(self, id, entry_point, kwargs=None):
        self.id, self.entry_point, self._kwargs = id, entry_point, dict(kwargs or {})

    def make(self, **kwargs):
        mod, attr = self.entry_point.split(":")
        return getattr(importlib.import_module(mod), attr)(**{**self._kwargs, **kwargs})


class EnvRegistry:
    def __init__(self):
        self.env_specs = {}

    def register(self, id, **kwargs):
        if id in self.env_specs:
            raise error.Error(f"Cannot re-register id: {id}")
        self.env_specs[id] = EnvSpec(id, **kwargs)

    def spec(self, id):
        return self.env_specs[id]

    def make(self, id, **kwargs):
        return self.spec(id).make(**kwargs)


registry = EnvRegistry()


def register(id, **kwargs):
    return registry.register(id, **kwargs)


def make(id, **kwargs):
    return registry.make(id, **kwargs)


def spec(id):
    return registry.spec(id)
