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
  published FA2 algorithm — forward softmax(q·kᵀ·d^-½)·v with bf16 inputs, fp32 softmax, P
  rounded to bf16 for P·V, keys ≥ k_len masked, bf16 output; backward with D = rowsum(dO∘O) taken
  from the bf16 output — is restated by ``sdpa_flash_attention`` and swapped in at the reference
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


class _FlashAttnRestated(torch.autograd.Function):
    """flash_attn (FA2) published algorithm on [B, L, N, D] fp32 copies of bf16 q/k/v:
    forward  P = exp(s - rowmax) (bf16 for the P.V product), l = sum of fp32 P, O = bf16(P.V / l)
    backward dV = P^T dO, dP = dO V^T, D = rowsum(dO * O) with the bf16 O, dS = P (dP - D),
             dQ = scale dS K, dK = scale dS^T Q   (FA2 paper Alg. 2; flash_attn/flash_bwd_*)"""

    @staticmethod
    def forward(ctx, q, k, v, k_len, scale):
        bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
        qb, kb, vb = bf(q), bf(k), bf(v)
        s = torch.einsum("blnd,bmnd->bnlm", qb, kb) * scale
        if k_len is not None:
            lk = k.shape[1]
            mask = torch.arange(lk).view(1, 1, 1, lk) >= k_len.view(-1, 1, 1, 1).to(torch.long)
            s = s.masked_fill(mask, float("-inf"))
        m = s.amax(-1, keepdim=True)
        p = torch.exp(s - m)
        l = p.sum(-1, keepdim=True)
        o = bf(torch.einsum("bnlm,bmnd->blnd", bf(p), vb) / l.permute(0, 2, 1, 3))
        ctx.save_for_backward(qb, kb, vb, o, p / l)
        ctx.scale = scale
        return o

    @staticmethod
    def backward(ctx, do):
        qb, kb, vb, o, P = ctx.saved_tensors
        do = do.to(torch.bfloat16).float()
        dv = torch.einsum("bnlm,blnd->bmnd", P, do)
        dp = torch.einsum("blnd,bmnd->bnlm", do, vb)
        delta = (do * o).sum(-1).permute(0, 2, 1).unsqueeze(-1)
        ds = P * (dp - delta)
        dq = torch.einsum("bnlm,bmnd->blnd", ds, kb) * ctx.scale
        dk = torch.einsum("bnlm,blnd->bmnd", ds, qb) * ctx.scale
        return dq, dk, dv, None, None


def sdpa_flash_attention(q, k, v, q_lens=None, k_lens=None, dropout_p=0., softmax_scale=None,
                         q_scale=None, causal=False, window_size=(-1, -1), deterministic=False,
                         dtype=torch.bfloat16, version=None):
    """Restatement of flash_attn varlen semantics used at `attention.py:96-127`."""
    assert not causal and dropout_p == 0 and q_lens is None
    out_dtype = q.dtype
    with torch.autocast("cpu", enabled=False):
        if q_scale is not None:
            q = q * q_scale
        scale = softmax_scale if softmax_scale is not None else q.size(-1) ** -0.5
        o = _FlashAttnRestated.apply(q.float(), k.float(), v.float(), k_lens, scale)
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
