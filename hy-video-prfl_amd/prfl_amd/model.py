"""Wan2.1 DiT with the reference's module tree, names and call signatures, running the MI355X
kernels.  Drop-in for `diffusers_lite/wan/modules/model.py` (WanModel `:413-729`,
WanAttentionBlock `:280-359`): identical state-dict keys, so Wan2.1 checkpoints load unchanged,
and identical forward signatures, so scripts/prfl and scripts/pavrm drive it as they drive the
reference.

What runs where:
  * every WanAttentionBlock  -> the fused, checkpointed `prfl::wan_block` custom op
    (prfl_amd/custom_ops.py, prfl_amd/block.py)
  * patch / text / image embeddings (bf16 Linear under autocast) -> `prfl::linear_bf16`
  * fp32 islands the reference keeps in fp32 (time embedding MLP on [B, 256]; Head's
    LayerNorm + 5120->64 Linear; unpatchify) -> small fp32 torch ops on the GPU (< 0.1 % of the
    step's FLOPs).
"""
import json
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import block as B
from . import ops
from . import sp as SP
from .linear import linear_bf16

__all__ = ["WanModel", "WanAttentionBlock", "WanRMSNorm", "WanLayerNorm", "rope_params",
           "rope_apply", "sinusoidal_embedding_1d", "pad_freqs"]

T5_CONTEXT_TOKEN_NUMBER = 512
FIRST_LAST_FRAME_CONTEXT_TOKEN_NUMBER = 257 * 2


def sinusoidal_embedding_1d(dim, position):
    """model.py:22-32 — float64 [cos | sin] embedding of the timestep."""
    half = dim // 2
    p = position.to(torch.float64)
    ang = torch.outer(p, torch.pow(10000, -torch.arange(half, dtype=torch.float64, device=p.device)
                                   .div(half)))
    return torch.cat([torch.cos(ang), torch.sin(ang)], dim=1)


def rope_params(max_seq_len, dim, theta=10000):
    """model.py:36-43 — complex128 [max_seq_len, dim/2]."""
    f = torch.outer(torch.arange(max_seq_len, dtype=torch.float64),
                    1.0 / torch.pow(theta, torch.arange(0, dim, 2, dtype=torch.float64).div(dim)))
    return torch.polar(torch.ones_like(f), f)


def pad_freqs(original_tensor, target_len):
    """model.py:45-58: extend per-token rotations [S, n, d] to `target_len` rows with unit
    multipliers (the sequence-parallel tail).  The reference's diagnostic print reads `pad_size`
    before assigning it, so its padding branch raises; the intended padding is returned here."""
    s, a, b = original_tensor.shape
    pad = original_tensor.new_ones(max(target_len - s, 0), a, b)
    return torch.cat([original_tensor, pad], dim=0)


def rope_apply(x, grid_sizes, freqs):
    """model.py:61-103.  On the HIP path RoPE is fused into RMSNorm (prfl_rms_rope_fwd_pos);
    this standalone form (fp64, as the reference) serves the attention sub-modules.  Under
    sequence parallelism x holds this rank's s tokens, rotated by their positions
    [rank * s, (rank + 1) * s) in the whole sequence, unit multipliers past the grid
    (model.py:89-96)."""
    b, s, n, d = x.shape
    c = d // 2
    st = SP.current()
    row0 = st.rank * s if st is not None else 0
    fs = freqs.to(x.device).split([c - 2 * (c // 3), c // 3, c // 3], dim=1)
    out = []
    for i, (f, h, w) in enumerate(grid_sizes.tolist()):
        L = f * h * w
        fi = torch.cat([fs[0][:f].view(f, 1, 1, -1).expand(f, h, w, -1),
                        fs[1][:h].view(1, h, 1, -1).expand(f, h, w, -1),
                        fs[2][:w].view(1, 1, w, -1).expand(f, h, w, -1)], dim=-1).reshape(L, 1, -1)
        fi = pad_freqs(fi, row0 + s)[row0:row0 + s]           # rows past the grid: unit
        n_rot = max(0, min(s, L - row0))
        xi = torch.view_as_complex(x[i, :n_rot].to(torch.float64).reshape(n_rot, n, -1, 2))
        out.append(torch.cat([torch.view_as_real(xi * fi[:n_rot]).flatten(2),
                              x[i, n_rot:].to(torch.float64)]))
    return torch.stack(out).float()


class WanRMSNorm(nn.Module):
    """model.py:106-122.  Inside a block the kernel prfl_rms_rope_fwd_pos computes it; standalone
    calls use the same fp32 formula."""

    def __init__(self, dim, eps=1e-5):
        super().__init__()
        self.dim, self.eps = dim, eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)).type_as(x) * self.weight


class WanLayerNorm(nn.LayerNorm):
    """model.py:125-135 (fp32 LayerNorm, result in the input dtype)."""

    def __init__(self, dim, eps=1e-6, elementwise_affine=False):
        super().__init__(dim, elementwise_affine=elementwise_affine, eps=eps)

    def forward(self, x):
        return super().forward(x.float()).type_as(x)


class _Attn(nn.Module):
    """The reference attention modules (`model.py:138-271`): same parameters and forward
    signatures.  Inside a WanAttentionBlock their math runs fused (prfl_amd/block.py, one
    `prfl::wan_block` op per block); called on their own they compose the custom ops with the
    reference's cast points: `prfl::linear_bf16` projections (autocast bf16 Linear), WanRMSNorm
    (fp32, rounded to bf16, x fp32 weight), rope_apply (fp64) and `prfl::flash_attention`."""

    def __init__(self, dim, num_heads, window_size=(-1, -1), qk_norm=True, eps=1e-6, img=False):
        super().__init__()
        assert dim % num_heads == 0
        self.dim, self.num_heads, self.head_dim = dim, num_heads, dim // num_heads
        self.window_size, self.qk_norm, self.eps = window_size, qk_norm, eps
        self.q, self.k, self.v, self.o = (nn.Linear(dim, dim) for _ in range(4))
        self.norm_q = WanRMSNorm(dim, eps=eps) if qk_norm else nn.Identity()
        self.norm_k = WanRMSNorm(dim, eps=eps) if qk_norm else nn.Identity()
        if img:
            self.k_img = nn.Linear(dim, dim)
            self.v_img = nn.Linear(dim, dim)
            self.norm_k_img = WanRMSNorm(dim, eps=eps) if qk_norm else nn.Identity()

    def _proj(self, name, x):
        lin = getattr(self, name)
        return linear_bf16(x, lin.weight, lin.bias)

    def _heads(self, t):
        return t.view(t.shape[0], -1, self.num_heads, self.head_dim)

    def _kv(self, ctx, k="k", v="v", nk="norm_k"):
        return self._heads(getattr(self, nk)(self._proj(k, ctx))), self._heads(self._proj(v, ctx))

    def _qkv(self, x, ctx):
        return (self._heads(self.norm_q(self._proj("q", x))),) + self._kv(ctx)


class WanSelfAttention(_Attn):
    def forward(self, x, seq_lens, grid_sizes, freqs):
        """model.py:163-201; under sequence parallelism q/k/v go to (all tokens, this rank's
        heads) and the output back, each exchange with its inverse as backward (sp.py)."""
        from .attention import flash_attention
        q, k, v = self._qkv(x, x)
        q, k = rope_apply(q, grid_sizes, freqs), rope_apply(k, grid_sizes, freqs)
        st = SP.current()
        if st is not None:
            q, k, v = (SP.all_to_all_4d(t, st, True) for t in (q, k, v))
        a = flash_attention(q, k, v, k_lens=seq_lens, window_size=self.window_size)
        if st is not None:
            a = SP.all_to_all_4d(a, st, False)
        return self._proj("o", a.flatten(2))


class WanT2VCrossAttention(_Attn):
    def forward(self, x, context, context_lens):
        """model.py:206-226."""
        from .attention import flash_attention
        q, k, v = self._qkv(x, context)
        return self._proj("o", flash_attention(q, k, v, k_lens=context_lens).flatten(2))


class WanI2VCrossAttention(_Attn):
    def __init__(self, dim, num_heads, window_size=(-1, -1), qk_norm=True, eps=1e-6):
        super().__init__(dim, num_heads, window_size, qk_norm, eps, img=True)

    def forward(self, x, context, context_lens):
        """model.py:244-271: the leading context tokens are the image (CLIP) tokens."""
        from .attention import flash_attention
        n_img = context.shape[1] - T5_CONTEXT_TOKEN_NUMBER
        ctx_img, ctx = context[:, :n_img], context[:, n_img:]
        q, k, v = self._qkv(x, ctx)
        ki, vi = self._kv(ctx_img, "k_img", "v_img", "norm_k_img")
        img_x = flash_attention(q, ki, vi, k_lens=None)
        out = flash_attention(q, k, v, k_lens=context_lens)
        return self._proj("o", out.flatten(2) + img_x.flatten(2))


WAN_CROSSATTENTION_CLASSES = {"t2v_cross_attn": WanT2VCrossAttention,
                              "i2v_cross_attn": WanI2VCrossAttention}

_ROPE_CACHE = {}


def _rope_table(freqs, device):
    key = (id(freqs), str(device))
    t = _ROPE_CACHE.get(key)
    if t is None:
        t = ops.rope_table(freqs, device)
        _ROPE_CACHE.clear()
        _ROPE_CACHE[key] = t
    return t


class WanAttentionBlock(nn.Module):
    """model.py:280-359.  forward() is one fused, activation-checkpointed HIP autograd node."""

    fp8_gemm = 0        # config C5's fp8 path (WanModel.set_fp8_gemm); the reference is bf16-only
    self_checkpointing = True   # forward is already the per-block checkpoint (fsdp_utils.py)
    stash_attn = True           # may keep its attention output for the backward (block.py)

    def __init__(self, cross_attn_type, dim, ffn_dim, num_heads, window_size=(-1, -1),
                 qk_norm=True, cross_attn_norm=False, eps=1e-6):
        super().__init__()
        assert qk_norm and cross_attn_norm, "the Wan2.1 14B/1.3B configs use qk_norm and norm3"
        self.dim, self.ffn_dim, self.num_heads = dim, ffn_dim, num_heads
        self.window_size, self.qk_norm, self.cross_attn_norm, self.eps = (window_size, qk_norm,
                                                                         cross_attn_norm, eps)
        self.i2v = cross_attn_type == "i2v_cross_attn"
        self.norm1 = WanLayerNorm(dim, eps)
        self.self_attn = WanSelfAttention(dim, num_heads, window_size, qk_norm, eps)
        self.norm3 = WanLayerNorm(dim, eps, elementwise_affine=True)
        self.cross_attn = WAN_CROSSATTENTION_CLASSES[cross_attn_type](dim, num_heads, (-1, -1),
                                                                      qk_norm, eps)
        self.norm2 = WanLayerNorm(dim, eps)
        self.ffn = nn.Sequential(nn.Linear(dim, ffn_dim), nn.GELU(approximate="tanh"),
                                 nn.Linear(ffn_dim, dim))
        self.modulation = nn.Parameter(torch.randn(1, 6, dim) / dim ** 0.5)
        self._names = B.param_names(self.i2v)

    def _param(self, name):
        """Parameter by attribute path, not named_parameters(): under FSDP (use_orig_params
        False, as `train_prfl.py:361` wraps it) the block's parameters are plain tensor views
        of the all-gathered flat parameter during forward / backward."""
        obj = self
        for part in name.split("."):
            obj = getattr(obj, part)
        return obj

    def forward(self, x, e, seq_lens, grid_sizes, freqs, context, context_lens):
        assert e.dtype == torch.float32
        assert context_lens is None, "cross-attention keys are unmasked in the reference (model.py:597)"
        with torch.autocast("cuda", enabled=False):
            em = self.modulation + e                                   # model.py:340
            P = {n: self._param(n) for n in self._names}
            st = SP.current()
            if st is not None and self.num_heads % st.size:
                raise ValueError(f"sequence parallelism: {self.num_heads} heads do not split over "
                                 f"sp_size {st.size}")
            meta = B.Meta(self.num_heads, [tuple(g) for g in grid_sizes.tolist()],
                          [int(s) for s in seq_lens.tolist()], _rope_table(freqs, x.device),
                          self.i2v, self.eps, fp8=self.fp8_gemm, sp=st)
            ctx = context if context.dtype == torch.bfloat16 else context.to(torch.bfloat16)
            return B.block_apply(P, x.contiguous(), em.contiguous(), ctx.contiguous(), meta,
                                 allow_keep=self.stash_attn)


class Head(nn.Module):
    """model.py:362-389 (fp32)."""

    def __init__(self, dim, out_dim, patch_size, eps=1e-6):
        super().__init__()
        self.dim, self.out_dim, self.patch_size, self.eps = dim, out_dim, patch_size, eps
        self.norm = WanLayerNorm(dim, eps)
        self.head = nn.Linear(dim, math.prod(patch_size) * out_dim)
        self.modulation = nn.Parameter(torch.randn(1, 2, dim) / dim ** 0.5)

    def forward(self, x, e):
        with torch.autocast("cuda", enabled=False):
            e = (self.modulation + e.unsqueeze(1)).chunk(2, dim=1)
            h = F.layer_norm(x.float(), (self.dim,), eps=self.eps) * (1 + e[1]) + e[0]
            return F.linear(h, self.head.weight, self.head.bias)


class MLPProj(nn.Module):
    """model.py:392-410 (CLIP image tokens -> context)."""

    def __init__(self, in_dim, out_dim, flf_pos_emb=False):
        super().__init__()
        self.proj = nn.Sequential(nn.LayerNorm(in_dim), nn.Linear(in_dim, in_dim), nn.GELU(),
                                  nn.Linear(in_dim, out_dim), nn.LayerNorm(out_dim))
        if flf_pos_emb:
            self.emb_pos = nn.Parameter(torch.zeros(1, FIRST_LAST_FRAME_CONTEXT_TOKEN_NUMBER, 1280))

    def forward(self, image_embeds):
        with torch.autocast("cuda", enabled=False):
            if hasattr(self, "emb_pos"):
                bs, n, d = image_embeds.shape
                image_embeds = image_embeds.view(-1, 2 * n, d) + self.emb_pos
            p = self.proj
            h = F.layer_norm(image_embeds.float(), p[0].normalized_shape, p[0].weight, p[0].bias,
                             p[0].eps)
            h = linear_bf16(h, p[1].weight, p[1].bias)
            h = F.gelu(h)                                            # bf16 in, bf16 out
            h = linear_bf16(h, p[3].weight, p[3].bias)
            return F.layer_norm(h.float(), p[4].normalized_shape, p[4].weight, p[4].bias, p[4].eps)


class WanModel(nn.Module):
    """model.py:413-729 — Wan2.1 diffusion backbone (t2v / i2v / flf2v)."""

    ignore_for_config = ["patch_size", "cross_attn_norm", "qk_norm", "text_dim", "window_size"]
    _no_split_modules = ["WanAttentionBlock"]
    enable_teacache = False
    config_name = "config.json"

    def __init__(self, model_type="t2v", patch_size=(1, 2, 2), text_len=512, in_dim=16, dim=2048,
                 ffn_dim=8192, freq_dim=256, text_dim=4096, out_dim=16, num_heads=16,
                 num_layers=32, window_size=(-1, -1), qk_norm=True, cross_attn_norm=True,
                 eps=1e-6):
        super().__init__()
        assert model_type in ["t2v", "i2v", "flf2v"]
        self.config = dict(model_type=model_type, patch_size=tuple(patch_size), text_len=text_len,
                           in_dim=in_dim, dim=dim, ffn_dim=ffn_dim, freq_dim=freq_dim,
                           text_dim=text_dim, out_dim=out_dim, num_heads=num_heads,
                           num_layers=num_layers, window_size=tuple(window_size), qk_norm=qk_norm,
                           cross_attn_norm=cross_attn_norm, eps=eps)
        self.model_type = model_type
        self.patch_size, self.text_len, self.in_dim, self.dim = tuple(patch_size), text_len, in_dim, dim
        self.ffn_dim, self.freq_dim, self.text_dim, self.out_dim = ffn_dim, freq_dim, text_dim, out_dim
        self.num_heads, self.num_layers, self.window_size = num_heads, num_layers, window_size
        self.qk_norm, self.cross_attn_norm, self.eps = qk_norm, cross_attn_norm, eps

        self.patch_embedding = nn.Conv3d(in_dim, dim, kernel_size=patch_size, stride=patch_size)
        self.text_embedding = nn.Sequential(nn.Linear(text_dim, dim), nn.GELU(approximate="tanh"),
                                            nn.Linear(dim, dim))
        self.time_embedding = nn.Sequential(nn.Linear(freq_dim, dim), nn.SiLU(), nn.Linear(dim, dim))
        self.time_projection = nn.Sequential(nn.SiLU(), nn.Linear(dim, dim * 6))
        cat = "t2v_cross_attn" if model_type == "t2v" else "i2v_cross_attn"
        self.blocks = nn.ModuleList([
            WanAttentionBlock(cat, dim, ffn_dim, num_heads, window_size, qk_norm, cross_attn_norm,
                              eps) for _ in range(num_layers)])
        self.head = Head(dim, out_dim, patch_size, eps)
        assert (dim % num_heads) == 0 and (dim // num_heads) % 2 == 0
        d = dim // num_heads
        # plain attribute, not a buffer (model.py:518)
        self.freqs = torch.cat([rope_params(1024, d - 4 * (d // 6)), rope_params(1024, 2 * (d // 6)),
                                rope_params(1024, 2 * (d // 6))], dim=1)
        if model_type in ("i2v", "flf2v"):
            self.img_emb = MLPProj(1280, dim, flf_pos_emb=model_type == "flf2v")
        self.init_weights()

    def set_fp8_gemm(self, on=True, attn=False, keep_bf16=B.C5_KEEP_BF16):
        """Config C5 (`train_prfl_i2v_720`, "fp8 MFMA path"): every block's large forward
        projections — QKV, self-attn O, cross-attn q/o, FFN in/out — run as per-row e4m3 operands
        on the block-scaled fp8 MFMA; the backward GEMMs stay bf16 (straight-through).  With
        `attn` the L x L self-attention forward runs on the e4m3 MFMA too (ops.attn_fwd_fp8).
        Held to an fp32 truth (k x the bf16 path's error), not to the reference (bf16-only).
        `keep_bf16` names projections of block.PROJ that stay bf16: by default the
        cross-attention q / o (block.C5_KEEP_BF16: they carry most of the e4m3 error; with them
        bf16 the block's update is 2.5 % from the fp32 truth instead of 5.3 %);
        `keep_bf16=()` puts all six on e4m3.
        The e4m3 weights are quantised from the fp32 masters: a model whose block weights were
        stored in bf16 (train.store_frozen_bf16) is refused."""
        if on and any(p.dtype != torch.float32 for blk in self.blocks for p in blk.parameters()):
            raise ValueError("set_fp8_gemm: block weights must be fp32 masters (quantised per pass)")
        code = B.fp8_code(2 if attn else 1, keep_bf16) if on else 0
        for blk in self.blocks:
            blk.fp8_gemm = code
        return self

    # ---------------------------------------------------------------- checkpoint I/O --------
    @classmethod
    def from_config(cls, config):
        cfg = dict(config)
        keep = set(cls.__init__.__code__.co_varnames[1:cls.__init__.__code__.co_argcount])
        return cls(**{k: v for k, v in cfg.items() if k in keep})

    @classmethod
    def from_pretrained(cls, path, allow_missing=(), **kw):
        """Loads a diffusers-format directory: config.json + *.safetensors (sharded or not),
        as written by `utils/model_utils.py:70-125` and the Wan2.1 releases.  A checkpoint that
        leaves parameters unset (wrong model type, truncated shard) raises instead of silently
        keeping their random init; `allow_missing` lists key prefixes that may be absent."""
        from safetensors.torch import load_file
        with open(os.path.join(path, "config.json")) as f:
            model = cls.from_config(json.load(f))
        files = sorted(x for x in os.listdir(path) if x.endswith(".safetensors"))
        sd = {}
        for fn in files:
            sd.update(load_file(os.path.join(path, fn)))
        missing, unexpected = model.load_state_dict(sd, strict=False)
        if unexpected:
            raise RuntimeError(f"unexpected keys in checkpoint: {unexpected[:8]}")
        missing = [k for k in missing if not any(k.startswith(a) for a in allow_missing)]
        if missing:
            raise RuntimeError(f"{len(missing)} parameters missing from checkpoint {path}: "
                               f"{missing[:8]}")
        return model

    def save_pretrained(self, path, max_shard_bytes=5 * 1024 ** 3):
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        cfg = dict(self.config, _class_name="WanModel")
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(cfg, f, indent=2)
        shard, size, idx = {}, 0, 0
        sd = {k: v.detach().cpu().contiguous() for k, v in self.state_dict().items()}
        names = list(sd)
        for i, k in enumerate(names):
            shard[k] = sd[k]
            size += sd[k].numel() * sd[k].element_size()
            if size >= max_shard_bytes or i == len(names) - 1:
                save_file(shard, os.path.join(path, f"diffusion_pytorch_model-{idx:05d}.safetensors"))
                shard, size, idx = {}, 0, idx + 1

    # ---------------------------------------------------------------- forward ---------------
    def _embed(self, x, t, context, seq_len, clip_fea, y):
        if self.model_type in ("i2v", "flf2v"):
            assert clip_fea is not None and y is not None
        if y is not None:
            x = [torch.cat([u, v], dim=0) for u, v in zip(x, y)]
        pt, ph, pw = self.patch_size
        wpe = self.patch_embedding.weight.flatten(1)        # [dim, Cin*pt*ph*pw]
        toks, grids = [], []
        for u in x:
            c, f, h, w = u.shape
            g = (f // pt, h // ph, w // pw)
            p = u.view(c, g[0], pt, g[1], ph, g[2], pw).permute(1, 3, 5, 0, 2, 4, 6)
            p = p.reshape(g[0] * g[1] * g[2], c * pt * ph * pw)
            toks.append(linear_bf16(p, wpe, self.patch_embedding.bias))  # Conv3d k=s (model.py:578)
            grids.append(g)
        grid_sizes = torch.tensor(grids, dtype=torch.long)
        seq_lens = torch.tensor([u.shape[0] for u in toks], dtype=torch.long)
        assert seq_lens.max() <= seq_len
        xb = torch.stack([torch.cat([u, u.new_zeros(seq_len - u.shape[0], u.shape[1])]) for u in toks])
        with torch.autocast("cuda", enabled=False):           # fp32 island (model.py:590-594)
            s = sinusoidal_embedding_1d(self.freq_dim, t).float()
            te = self.time_embedding
            e = F.linear(F.silu(F.linear(s, te[0].weight, te[0].bias)), te[2].weight, te[2].bias)
            e0 = F.linear(F.silu(e), self.time_projection[1].weight, self.time_projection[1].bias)
            e0 = e0.unflatten(1, (6, self.dim))
        ctx = torch.stack([torch.cat([u, u.new_zeros(self.text_len - u.size(0), u.size(1))])
                           for u in context])
        ctx = linear_bf16(ctx, self.text_embedding[0].weight, self.text_embedding[0].bias, gelu=True)
        ctx = linear_bf16(ctx, self.text_embedding[2].weight, self.text_embedding[2].bias)
        if clip_fea is not None:
            ctx = torch.cat([self.img_emb(clip_fea).to(torch.bfloat16), ctx], dim=1)
        return xb, e, e0, ctx, grid_sizes, seq_lens, grids

    def forward(self, x, t, context, seq_len, clip_fea=None, y=None, cond_flag=False,
                output_features=False, selected_layers=[20, 30, 40]):
        """model.py:534-681.  Under the reference's sequence parallelism (its `parallel_states`
        initialised with sp_size > 1, or `prfl_amd.sp.set_group`) each rank runs the blocks on
        its seq_len / sp_size tokens (model.py:618-619) and the features / head output are
        all-gathered along the sequence (model.py:663-676), exactly as the reference."""
        xb, e, e0, ctx, grid_sizes, seq_lens, grids = self._embed(x, t, context, seq_len,
                                                                 clip_fea, y)
        st = SP.current()
        h = xb
        if st is not None:
            s = SP.split_len(xb.shape[1], st)
            h = xb.narrow(1, st.rank * s, s)                 # torch.chunk(x, sp, 1)[rank]
        feats = []
        for index, block in enumerate(self.blocks):
            h = block(h, e0, seq_lens, grid_sizes, self.freqs, ctx, None)
            if output_features and index + 1 in selected_layers:
                feats.append(SP.gather_seq(h, st) if st is not None else h)
        if output_features:
            return feats
        out = self.head(h, e)
        if st is not None:
            out = SP.gather_seq(out, st)
        return [u.float() for u in self.unpatchify(out, grid_sizes, self.out_dim)]

    def unpatchify(self, x, grid_sizes, c):
        out = []
        for u, v in zip(x, grid_sizes.tolist()):
            u = u[: math.prod(v)].view(*v, *self.patch_size, c)
            u = torch.einsum("fhwpqrc->cfphqwr", u)
            out.append(u.reshape(c, *[i * j for i, j in zip(v, self.patch_size)]))
        return out

    def init_weights(self):
        """model.py:707-729."""
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
        nn.init.xavier_uniform_(self.patch_embedding.weight.flatten(1))
        for m in list(self.text_embedding.modules()) + list(self.time_embedding.modules()):
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, std=.02)
        nn.init.zeros_(self.head.head.weight)
