"""CPU: the C-ABI library loads, exports every symbol include/msacl_hip.h declares, and its
host-only entry (mh_env_info) agrees with the oracle's spaces. No compute call needs a GPU."""
import ctypes
import os
import re

import numpy as np

import msacl_amd._native as N
from oracle import envs as OE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "msacl_hip.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\*|void)\s+(mh_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(N.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(N.exported_symbols()) == syms


def test_abi_version_and_errors():
    L = N.lib()
    assert L.mh_abi_version() == 1
    info = N.EnvInfo()
    assert L.mh_env_info(42, ctypes.byref(info)) == -1
    assert b"unknown env id" in L.mh_last_error()
    h = ctypes.c_void_p()
    assert L.mh_env_create(0, 0, 0, ctypes.byref(h)) == -1  # num_envs out of range: no device touched
    assert L.mh_rollout_step(None, None, None, None, None, None, None, None, None, None) == -1


def test_env_info_matches_oracle_spaces():
    for name, cls in OE.ENVS.items():
        i = N.env_info(name)
        assert (i.obs_dim, i.act_dim) == (cls.obs_dim, cls.act_dim)
        np.testing.assert_array_equal(np.array(i.obs_low[:i.obs_dim], np.float32), cls.obs_low)
        np.testing.assert_array_equal(np.array(i.obs_high[:i.obs_dim], np.float32), cls.obs_high)
        np.testing.assert_array_equal(np.array(i.act_low[:i.act_dim], np.float32), cls.act_low)
        np.testing.assert_array_equal(np.array(i.act_high[:i.act_dim], np.float32), cls.act_high)
        assert i.max_step == 1000
        assert i.record_floats % 4 == 0 and i.record_floats >= 2 * i.obs_dim + i.act_dim + 4
