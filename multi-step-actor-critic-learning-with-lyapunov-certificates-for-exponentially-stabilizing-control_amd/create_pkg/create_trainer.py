"""create_trainer (RL/create_pkg/create_trainer.py:34-62): trainer/<x>trainer.py -> <X>Trainer."""
from ..utils.MyRL_path import trainer_path, underline2camel
from .registry import Registry

_PKG = __package__.rsplit(".", 1)[0]
registry = Registry("trainer")
registry.discover(trainer_path, f"{_PKG}.trainer", underline2camel, file_filter=lambda f: f.endswith("trainer.py"))


def create_trainer(alg, sampler, buffer, evaluator, **kwargs):
    name = kwargs["trainer"]
    spec = registry.get(name)
    if name.startswith(("off", "nstep_off")):
        trainer = registry.build(name, alg, sampler, buffer, evaluator, **kwargs)
    elif name.startswith("on"):
        trainer = registry.build(name, alg, sampler, evaluator, **kwargs)
    else:
        raise RuntimeError(f"trainer {spec.name} not recognized")
    print(name, "created successfully!")
    return trainer
