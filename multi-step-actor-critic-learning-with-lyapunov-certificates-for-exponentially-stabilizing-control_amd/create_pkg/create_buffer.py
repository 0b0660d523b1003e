"""create_buffer (RL/create_pkg/create_buffer.py:33-66): None for on-policy trainers."""
from ..utils.MyRL_path import buffer_path, underline2camel
from .registry import Registry

_PKG = __package__.rsplit(".", 1)[0]
registry = Registry("buffer")
registry.discover(buffer_path, f"{_PKG}.trainer.buffer", underline2camel)


def create_buffer(**kwargs):
    name = kwargs.get("buffer_name", None)
    spec = registry.get(name)
    trainer = kwargs.get("trainer", spec.kwargs.get("trainer"))
    if trainer is None or trainer.startswith("on"):
        print("No buffer for on-policy trainer! return None")
        return None
    buf = registry.build(name, **kwargs)
    print(name, "created successfully")
    return buf
