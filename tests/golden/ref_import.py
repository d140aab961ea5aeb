"""Import the reference hot-path modules on a GPU-less host (fixture generation only).

Used ONLY by ``make_golden.py`` in the build container, where ``/root/reference`` exists.
Nothing on the GPU box imports this file.

What is substituted, and why none of it changes arithmetic:

* ``diffusers`` is not installed.  The reference uses it only for base classes and config
  bookkeeping (``ModelMixin``, ``ConfigMixin``/``register_to_config``, ``SchedulerMixin``,
  ``SchedulerOutput``, ``BaseOutput``, ``deprecate``, ``logging``, ``KarrasDiffusionSchedulers``,
  ``FP32LayerNorm``).  The stubs below record constructor arguments into ``self.config`` the way
  diffusers does and otherwise are plain ``nn.Module``/``object``.
* ``easydict``/``ftfy`` are imported by non-hot-path config modules; stubbed as dict/identity.
* ``flash_attn`` (third-party, `requirements.txt:16`, README pins 2.5.0) is absent.  Its
  published algorithm — softmax(q·kᵀ·d^-½)·v with bf16 inputs, fp32 softmax, keys ≥ k_len
  masked, bf16 output — is restated by ``sdpa_flash_attention`` and swapped in at the reference
  call site ``model.flash_attention`` (`attention.py:24-130`).
* The reference wraps fp32 islands in ``torch.cuda.amp.autocast(dtype=torch.float32)``
  (`model.py:339,347,354,386,590`) and disables autocast for RoPE (`model.py:35,60`).  On a CPU
  host the CUDA autocast context does not govern CPU autocast, so ``model.amp`` is re-pointed
  at a shim that applies the same context to the CPU autocast state.  With that, CPU bf16
  autocast reproduces the CUDA precision flow (bf16 GEMMs with fp32 accumulate, fp32 islands).
"""
import enum
import inspect
import os
import sys
import types
from dataclasses import dataclass

import torch
import torch.nn as nn

REF = os.environ.get("PRFL_REFERENCE", "/root/reference")


def _stub_module(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


class _Config(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def register_to_config(init):
    sig = inspect.signature(init)

    def wrapped(self, *args, **kwargs):
        bound = sig.bind(self, *args, **kwargs)
        bound.apply_defaults()
        cfg = {k: v for k, v in bound.arguments.items() if k != "self"}
        self.config = _Config(cfg)
        init(self, *args, **kwargs)

    return wrapped


class ConfigMixin:
    def register_to_config(self, **kwargs):
        if not hasattr(self, "config"):
            self.config = _Config()
        self.config.update(kwargs)


class ModelMixin(nn.Module):
    pass


class SchedulerMixin:
    pass


@dataclass
class SchedulerOutput:
    prev_sample: torch.Tensor


class BaseOutput:
    pass


class KarrasDiffusionSchedulers(enum.Enum):
    pass


class _Logger:
    def get_logger(self, *a, **k):
        import logging
        return logging.getLogger("ref")


class FP32LayerNorm(nn.LayerNorm):
    def forward(self, x):
        return nn.functional.layer_norm(x.float(), self.normalized_shape, None if self.weight is None
                                        else self.weight.float(), None if self.bias is None
                                        else self.bias.float(), self.eps).to(x.dtype)


class _AmpShim:
    """`torch.cuda.amp` stand-in whose autocast governs the CPU autocast state."""

    @staticmethod
    def autocast(enabled=True, dtype=torch.bfloat16, cache_enabled=True):
        if dtype not in (torch.bfloat16, torch.float16):
            # CUDA autocast(dtype=float32) == "run listed ops in fp32"; on CPU that is
            # autocast disabled (every op then runs in its input dtype, fp32 here).
            return torch.autocast("cpu", enabled=False)
        return torch.autocast("cpu", dtype=dtype, enabled=enabled)


def sdpa_flash_attention(q, k, v, q_lens=None, k_lens=None, dropout_p=0., softmax_scale=None,
                         q_scale=None, causal=False, window_size=(-1, -1), deterministic=False,
                         dtype=torch.bfloat16, version=None):
    """Restatement of flash_attn varlen semantics used at `attention.py:96-127`."""
    out_dtype = q.dtype
    b, lq, lk = q.size(0), q.size(1), k.size(1)
    with torch.autocast("cpu", enabled=False):
        qb = q.to(dtype).float()
        kb = k.to(dtype).float()
        vb = v.to(dtype).float()
        if q_scale is not None:
            qb = qb * q_scale
        scale = softmax_scale if softmax_scale is not None else qb.size(-1) ** -0.5
        s = torch.einsum("blnd,bmnd->bnlm", qb, kb) * scale
        if k_lens is not None:
            mask = torch.arange(lk).view(1, 1, 1, lk) >= k_lens.view(b, 1, 1, 1).to(torch.long)
            s = s.masked_fill(mask, float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("bnlm,bmnd->blnd", p, vb)
        if q_lens is not None:
            qmask = torch.arange(lq).view(1, lq, 1, 1) >= q_lens.view(b, 1, 1, 1).to(torch.long)
            o = o.masked_fill(qmask, 0.0)
    return o.to(dtype).to(out_dtype)


def import_reference():
    """Returns (model_mod, network_mod, unipc_mod, fm_mod)."""
    if REF not in sys.path:
        sys.path.insert(0, REF)
    _stub_module("diffusers")
    _stub_module("diffusers.configuration_utils", ConfigMixin=ConfigMixin,
                 register_to_config=register_to_config)
    _stub_module("diffusers.models")
    _stub_module("diffusers.models.modeling_utils", ModelMixin=ModelMixin)
    _stub_module("diffusers.models.normalization", FP32LayerNorm=FP32LayerNorm)
    _stub_module("diffusers.schedulers")
    _stub_module("diffusers.schedulers.scheduling_utils", SchedulerMixin=SchedulerMixin,
                 SchedulerOutput=SchedulerOutput,
                 KarrasDiffusionSchedulers=KarrasDiffusionSchedulers)
    _stub_module("diffusers.utils", BaseOutput=BaseOutput, logging=_Logger(),
                 deprecate=lambda *a, **k: None, is_scipy_available=lambda: False)
    _stub_module("diffusers.utils.torch_utils", randn_tensor=torch.randn)
    _stub_module("easydict", EasyDict=dict)
    _stub_module("ftfy", fix_text=lambda s: s)
    # bare packages: skip wan/__init__ and wan/modules/__init__ (t5.py:478 touches CUDA)
    for pkg in ("diffusers_lite.wan", "diffusers_lite.wan.modules", "diffusers_lite.wan.utils"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(REF, *pkg.split("."))]
        sys.modules[pkg] = m
    import importlib
    model_mod = importlib.import_module("diffusers_lite.wan.modules.model")
    model_mod.flash_attention = sdpa_flash_attention
    model_mod.amp = _AmpShim
    network_mod = importlib.import_module("diffusers_lite.utils.network")
    unipc_mod = importlib.import_module("diffusers_lite.wan.utils.fm_solvers_unipc")
    fm_mod = importlib.import_module("diffusers_lite.schedulers.scheduling_flow_match_discrete")
    diff_utils = importlib.import_module("diffusers_lite.utils.diffusion_utils")
    return model_mod, network_mod, unipc_mod, fm_mod, diff_utils
