"""create_sampler (RL/create_pkg/create_sampler.py:33-80): trainer/sampler/<name>.py -> <Name>."""
from ..utils.MyRL_path import sampler_path, underline2camel
from .registry import Registry

_PKG = __package__.rsplit(".", 1)[0]
registry = Registry("sampler")
registry.discover(sampler_path, f"{_PKG}.trainer.sampler", underline2camel)


def create_sampler(**kwargs):
    name = kwargs["sampler_name"]
    sampler = registry.build(name, **kwargs)
    print(name, "created successfully!")
    return sampler
