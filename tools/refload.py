"""Loader for the reference's env / sampler code WITHOUT its absent third-party dependency.

Test-infrastructure only (used by tools/gen_golden.py in the build container; the reference
never travels to the GPU box). gymnasium is not installed here and is NOT stood in for: the
module-level numpy code and the env methods are compiled from the reference source text with
`ast` and executed on a data-only `self`. The only values supplied from outside the reference's
own statements are the Box bounds, which are evaluated from the reference's own `spaces.Box(...)`
argument expressions and cast to the declared dtype (what Box stores).
"""
from __future__ import annotations

import ast
import random
import sys
import types

import numpy as np

REF = "/root/reference"


def _is_gym_import(node):
    if isinstance(node, ast.Import):
        return any(a.name.split(".")[0] == "gymnasium" for a in node.names)
    if isinstance(node, ast.ImportFrom):
        return (node.module or "").split(".")[0] == "gymnasium"
    return False


def _is_box_call(v):
    return (isinstance(v, ast.Call) and isinstance(v.func, ast.Attribute) and v.func.attr == "Box"
            and isinstance(v.func.value, ast.Name) and v.func.value.id == "spaces")


class RefModule:
    """Module namespace + the env class's methods, compiled from the reference source."""

    def __init__(self, relpath, class_name):
        self.path = f"{REF}/{relpath}"
        src = open(self.path).read()
        self.tree = ast.parse(src)
        if REF not in sys.path:
            sys.path.insert(0, REF)
        modname = "ref_" + class_name
        module = types.ModuleType(modname)
        sys.modules[modname] = module  # dataclasses look their module up in sys.modules
        self.ns = module.__dict__
        self.ns.update({"np": np, "random": random})
        self.cls_node = None
        for node in self.tree.body:
            if _is_gym_import(node):
                continue
            if isinstance(node, ast.ClassDef) and node.name == class_name:
                self.cls_node = node
                continue
            exec(compile(ast.Module(body=[node], type_ignores=[]), self.path, "exec"), self.ns)
        assert self.cls_node is not None, class_name
        self.methods = {}
        self.class_attrs = []
        for item in self.cls_node.body:
            if isinstance(item, ast.FunctionDef):
                exec(compile(ast.Module(body=[item], type_ignores=[]), self.path, "exec"), self.ns)
                self.methods[item.name] = self.ns.pop(item.name)
            elif isinstance(item, (ast.Assign, ast.AnnAssign)):
                self.class_attrs.append(item)

    def method_node(self, name):
        for item in self.cls_node.body:
            if isinstance(item, ast.FunctionDef) and item.name == name:
                return item
        raise KeyError(name)

    def make(self, **init_kwargs):
        """Build an env object: bind methods, set class attributes, run __init__ statements."""
        obj = types.SimpleNamespace()
        for name, fn in self.methods.items():
            if name != "__init__":
                setattr(obj, name, types.MethodType(fn, obj))
        loc = dict(self.ns)
        for st in self.class_attrs:
            cls_ns = {}
            exec(compile(ast.Module(body=[st], type_ignores=[]), self.path, "exec"), dict(loc), cls_ns)
            for k, v in cls_ns.items():
                setattr(obj, k, v)
        init = self.method_node("__init__")
        loc["self"] = obj
        args = init.args.args[1:]
        defaults = init.args.defaults
        for a, d in zip(args[len(args) - len(defaults):], defaults):
            loc[a.arg] = eval(compile(ast.Expression(d), self.path, "eval"), loc)
        loc.update(init_kwargs)
        skipped = []
        for st in init.body:
            if isinstance(st, ast.Assign) and _is_box_call(st.value):
                call = st.value
                kw = {k.arg: eval(compile(ast.Expression(k.value), self.path, "eval"), loc) for k in call.keywords}
                dt = kw.get("dtype", np.float32)
                low = np.asarray(kw["low"]).astype(dt)
                high = np.asarray(kw["high"]).astype(dt)
                box = types.SimpleNamespace(low=low, high=high, shape=low.shape, dtype=np.dtype(dt))
                tgt = st.targets[0]
                assert isinstance(tgt, ast.Attribute)
                setattr(obj, tgt.attr, box)
                continue
            src = ast.unparse(st)
            if src.startswith("super()"):
                skipped.append(src)
                continue
            exec(compile(ast.Module(body=[st], type_ignores=[]), self.path, "exec"), loc)
        obj._skipped_init = skipped
        return obj

    def run_statements(self, method, obj, skip_pred, local_extra=None):
        """Execute a method body statement by statement, skipping those `skip_pred(src)` marks."""
        node = self.method_node(method)
        loc = dict(self.ns)
        loc["self"] = obj
        if local_extra:
            loc.update(local_extra)
        cache = self.__dict__.setdefault("_stmt_cache", {})
        for st in node.body:
            hit = cache.get(id(st))
            if hit is None:  # unparse + compile once per statement (the timing calibration resets often)
                src = ast.unparse(st)
                if isinstance(st, ast.Return):
                    code = compile(ast.Expression(st.value), self.path, "eval")
                else:
                    code = compile(ast.Module(body=[st], type_ignores=[]), self.path, "exec")
                hit = cache[id(st)] = (src, code, isinstance(st, ast.Return))
            src, code, is_ret = hit
            if skip_pred(src):
                continue
            if is_ret:
                return eval(code, loc)
            exec(code, loc)
        return None


ENV_FILES = {
    "VanderPol": ("RL/env/VanderPol.py", "vanderpol"),
    "Pendulum": ("RL/env/Pendulum.py", "pendulum"),
    "DuctedFan": ("RL/env/DuctedFan.py", "ductedfan"),
    "TwoLink": ("RL/env/TwoLink.py", "twolink"),
    "SingleTrackCar": ("RL/env/SingleTrackCar.py", "singletrackcar"),
    "QuadTracking": ("RL/env/QuadTracking.py", "quadtracking"),
}


def load_env(name):
    rel, cls = ENV_FILES[name]
    return RefModule(rel, cls)
