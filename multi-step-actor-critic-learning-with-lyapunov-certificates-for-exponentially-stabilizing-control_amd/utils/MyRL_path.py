"""Package paths and the registry naming rule (mirrors RL/utils/MyRL_path.py:1-21)."""
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
algorithm_path = os.path.join(PKG_ROOT, "algorithm")
apprfunc_path = os.path.join(PKG_ROOT, "apprfunc")
trainer_path = os.path.join(PKG_ROOT, "trainer")
sampler_path = os.path.join(trainer_path, "sampler")
buffer_path = os.path.join(trainer_path, "buffer")


def underline2camel(s: str, first_upper: bool = False) -> str:
    """`nstep_off_sampler` -> `NstepOffSampler`; with first_upper the first word is upper-cased
    whole (`msacl_x` -> `MSACLX`)."""
    words = s.split("_")
    head = words.pop(0).upper() if first_upper else ""
    return head + "".join(w[:1].upper() + w[1:] for w in words)
