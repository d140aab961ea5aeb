"""The drop-in preamble: point the reference's hot-path module names at this package.

`scripts/prfl/train_prfl.py` and `scripts/pavrm/train_pavrm.py` import the Wan DiT, the reward
head, the UniPC sampler and the FSDP helpers from `diffusers_lite.*` (train_prfl.py:29-97,
train_pavrm.py:28-74).  `install()` registers this package's modules under those names in
`sys.modules` before the driver's imports run, so the driver resolves them here and everything
else (VAE, T5, CLIP, communication, model_utils, ...) from the reference package as before.
Each module listed in `MODULE_MAP` exports every top-level name its reference module defines
(checked against the reference's sources by tests/test_host.py::test_dropin_*).
"""
import importlib
import sys

MODULE_MAP = {
    "diffusers_lite.wan.modules.model": "prfl_amd.model",
    "diffusers_lite.wan.modules.attention": "prfl_amd.attention",
    "diffusers_lite.wan.utils.fm_solvers_unipc": "prfl_amd.schedulers",
    "diffusers_lite.utils.network": "prfl_amd.network",
    "diffusers_lite.utils.fsdp_utils": "prfl_amd.fsdp_utils",
    "diffusers_lite.utils.load": "prfl_amd.fsdp_utils",
}


def install(modules=None):
    """Register the replacements in `sys.modules` (or in the dict `modules`); returns the
    mapping {reference name: module object}.  Call it before importing the driver."""
    target = sys.modules if modules is None else modules
    done = {}
    for ref_name, ours in MODULE_MAP.items():
        mod = importlib.import_module(ours)
        target[ref_name] = mod
        done[ref_name] = mod
    return done
