"""Shared plugin-registry machinery behind create_alg / create_sampler / create_buffer /
create_trainer / create_apprfunc / create_evaluator.

Discovery rule is the reference's: every `<name>.py` in a plugin directory (not starting with
"_", not base.py) registers under `<name>` with entry point `underline2camel(<name>)`
(RL/create_pkg/create_sampler.py:33-42, create_buffer.py:33-41, create_trainer.py:34-39); the
algorithms export `<NAME>` + `ApproxContainer` (create_alg.py:38-47). Unknown ids raise
KeyError("No registered <kind> with id: ..."), non-callable entries RuntimeError.
"""
from __future__ import annotations

import importlib
import os
from dataclasses import dataclass, field
from typing import Callable, Dict


@dataclass
class Spec:
    name: str
    entry_point: Callable
    extra: dict = field(default_factory=dict)
    kwargs: dict = field(default_factory=dict)


class Registry:
    def __init__(self, kind: str):
        self.kind = kind
        self.specs: Dict[str, Spec] = {}

    def register(self, name, entry_point, extra=None, **kwargs):
        self.specs[name] = Spec(name, entry_point, extra or {}, kwargs)

    def get(self, name) -> Spec:
        spec = self.specs.get(name)
        if spec is None:
            raise KeyError(f"No registered {self.kind} with id: {name}")
        return spec

    def discover(self, directory, package, entry_name, file_filter=None, extra_fn=None):
        for fname in sorted(os.listdir(directory)):
            if not fname.endswith(".py") or fname.startswith("_") or fname == "base.py":
                continue
            if file_filter is not None and not file_filter(fname):
                continue
            stem = fname[:-3]
            mod = importlib.import_module(f"{package}.{stem}")
            ep = getattr(mod, entry_name(stem), None)
            if ep is None:
                continue
            self.register(stem, ep, extra_fn(mod) if extra_fn else None)

    def build(self, key, /, *args, **kwargs):
        spec = self.get(key)
        merged = dict(spec.kwargs)
        merged.update(kwargs)
        if not callable(spec.entry_point):
            raise RuntimeError(f"{spec.name} registered but entry_point is not specified")
        return spec.entry_point(*args, **merged)
