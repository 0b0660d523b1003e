"""create_evaluator (RL/create_pkg/create_evaluator.py:33-51)."""
from ..trainer.evaluator import Evaluator
from .registry import Registry

registry = Registry("evaluator")
registry.register("evaluator", Evaluator)


def create_evaluator(evaluator_name: str, **kwargs):
    ev = registry.build(evaluator_name, **kwargs)
    print(evaluator_name, "created successfully!")
    return ev
