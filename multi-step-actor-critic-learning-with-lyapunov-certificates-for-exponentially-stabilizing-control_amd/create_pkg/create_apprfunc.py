"""create_apprfunc (RL/create_pkg/create_apprfunc.py:39-66): registry key `<module>_<Class>`."""
import importlib
import os

from ..utils.MyRL_path import apprfunc_path
from .registry import Registry

_PKG = __package__.rsplit(".", 1)[0]
registry = Registry("apprfunc")
for _f in sorted(os.listdir(apprfunc_path)):
    if _f.endswith(".py") and not _f.startswith("_") and _f != "base.py":
        _mod = importlib.import_module(f"{_PKG}.apprfunc.{_f[:-3]}")
        for _cls in _mod.__all__:
            registry.register(f"{_f[:-3]}_{_cls}", getattr(_mod, _cls))


def create_apprfunc(**kwargs):
    key = kwargs["apprfunc"].lower() + "_" + kwargs["name"]
    if key not in registry.specs:
        raise KeyError(f"No registered apprfunc with id: {kwargs['apprfunc'].lower()}_{kwargs['name']}")
    return registry.build(key, **kwargs)
