"""Import alias for the engine package.

The package lives in the directory
`multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-control_amd/`
(not a valid Python identifier). `import msacl_amd` loads it under this name; every submodule
(`msacl_amd.create_pkg.create_sampler`, ...) then resolves through the package's __path__.
"""
import importlib.util
import os
import sys

PACKAGE_DIR = os.path.join(
    os.path.dirname(os.path.abspath(__file__)),
    "multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-control_amd",
)
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(PACKAGE_DIR, "__init__.py"), submodule_search_locations=[PACKAGE_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
