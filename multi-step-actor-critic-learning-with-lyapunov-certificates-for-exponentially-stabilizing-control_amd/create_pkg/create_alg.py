"""create_alg / create_approx_contrainer (RL/create_pkg/create_alg.py:38-97).
Each algorithm/<name>.py exports <NAME> and ApproxContainer."""
from ..utils.MyRL_path import algorithm_path
from .registry import Registry

_PKG = __package__.rsplit(".", 1)[0]
registry = Registry("algorithm")
registry.discover(algorithm_path, f"{_PKG}.algorithm", lambda stem: stem.upper(),
                  extra_fn=lambda mod: {"approx_container_cls": getattr(mod, "ApproxContainer")})

_TRAINER_PREFIXES = ("off_serial", "nstep_off_serial", "on_serial", "on_sync")


def create_alg(**kwargs):
    algorithm = kwargs["algorithm"]
    spec = registry.get(algorithm)
    trainer = kwargs.get("trainer", spec.kwargs.get("trainer"))
    if trainer is not None and not trainer.startswith(_TRAINER_PREFIXES):
        raise RuntimeError(f"trainer {trainer} can not recognized")
    alg = registry.build(algorithm, **kwargs)
    print(algorithm, "algorithm created successfully!")
    return alg


def create_approx_contrainer(algorithm: str, **kwargs):
    spec = registry.get(algorithm)
    cls = spec.extra.get("approx_container_cls")
    if not callable(cls):
        raise RuntimeError(f"{algorithm} registered but approx_container_cls is not specified")
    merged = dict(spec.kwargs)
    merged.update(kwargs)
    return cls(**merged)


create_approx_container = create_approx_contrainer
