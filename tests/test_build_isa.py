"""CPU: static checks on the built gfx950 code object of the fused horizon sampler.

csrc/Makefile compiles sample_fused.hip with -fno-slp-vectorize: with the env step's scalar f32
code SLP-vectorised into packed-FP32 instructions (v_pk_mul / v_pk_add / v_pk_fma _f32) running on
the env waves beside the policy waves' MFMAs, QuadTracking produced run-to-run different results in
lanes 48-63 (tools/probes/variants_det.sh). The guard must not rest on the flag
alone. Since round 5 the policy pass has no packed-f32 arithmetic either (its split / rescale
pairs are scalar: beside MFMAs a v_pk_fma_f32 costs ~22 cycles more than two v_fma_f32), so no
k_sample_fused<Env> may contain a single packed-f32 instruction.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-"
                   "control_amd", "csrc", "build", "sample_fused.o")
LLVM = "/opt/rocm/lib/llvm/bin"
ENVS = ("VanderPol", "Pendulum", "DuctedFan", "TwoLink", "SingleTrackCar", "QuadTracking")


def _disassemble(tmp_path):
    if not os.path.exists(OBJ):
        pytest.skip("sample_fused.o not built (make -C csrc)")
    for tool in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump"):
        if not os.path.exists(os.path.join(LLVM, tool)) and shutil.which(tool) is None:
            pytest.skip(f"{tool} not available")
    fat, co = str(tmp_path / "fatbin.bin"), str(tmp_path / "gfx950.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", OBJ, str(tmp_path / "o.o")], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--input={fat}", f"--output={co}", "--unbundle"], check=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout


def test_env_step_code_of_the_fused_kernel_is_not_packed(tmp_path):
    asm = _disassemble(tmp_path)
    counts, name = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if m:
            name = m.group(1)
            continue
        if name and "k_sample_fused" in name and re.search(r"\bv_pk_(mul|add|fma)_f32\b", line):
            counts[name] = counts.get(name, 0) + 1
    per_env = {e: sum(c for n, c in counts.items() if e in n) for e in ENVS}
    assert any("k_sample_fused" in n for n in _kernels(asm)), "no k_sample_fused in the code object"
    assert all(v == 0 for v in per_env.values()), f"packed-f32 code in the fused kernel: {per_env}"


def _kernels(asm):
    return [m.group(1) for m in re.finditer(r"^[0-9a-f]+ <(.*)>:", asm, re.M)]
