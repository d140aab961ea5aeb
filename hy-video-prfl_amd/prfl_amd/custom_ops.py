"""The operator boundary of the MI355X path: ``torch.library`` custom ops in the ``prfl``
namespace, each with a schema, a fake (meta) implementation and a registered autograd formula,
whose CUDA (= HIP) implementations call the C ABI of ``libprfl_hip.so`` (include/prfl_hip.h).

| op                               | replaces (reference)                                        |
|----------------------------------|-------------------------------------------------------------|
| prfl::wan_block (+ _backward)    | WanAttentionBlock.forward under the per-block non-reentrant |
|                                  | checkpoint (`model.py:320-359`, `fsdp_utils.py:17-50`)      |
| prfl::linear_bf16 (+ _backward)  | autocast `nn.Linear` / Conv3d patch embed (`model.py:578`,  |
|                                  | `:598-607`, `network.py:80` in-projection)                  |
| prfl::flash_attention (+ _bwd)   | `flash_attention` (`attention.py:24-130`)                   |
| prfl::query_pool (+ _backward)   | the 1-query `nn.MultiheadAttention` core (`network.py:80`)  |
| prfl::unipc_step (+ _backward)   | `FlowUniPCMultistepScheduler.step`'s element-wise body      |
|                                  | (`fm_solvers_unipc.py:350-626`)                              |

Because these are dispatcher ops, autograd sees ordinary nodes: `torch.utils.checkpoint`
(non-reentrant, as `apply_fsdp_checkpointing` installs it) recomputes them, FSDP's
all-gathered parameter views flow in as plain tensor arguments, and FX / fake-tensor tracing
sees their schemas.  Only CUDA implementations are registered: a CPU tensor raises
NotImplementedError from the dispatcher (there is no CPU fallback anywhere on the product path).
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import block as B
from . import ops
from . import sp as SP
from .ops import BF16

F32 = torch.float32


def _empty(like, dtype=None):
    return like.new_empty((0,), dtype=dtype or like.dtype)


# ============================================================ fused WanAttentionBlock ======
def _meta(num_heads, grid, seq_lens, rope_tab, i2v, eps, fp8, sp=0):
    g = [tuple(grid[i:i + 3]) for i in range(0, len(grid), 3)]
    return B.Meta(num_heads, g, list(seq_lens), rope_tab, i2v, eps, fp8=fp8, sp=SP.lookup(sp))


@torch.library.custom_op("prfl::wan_block", mutates_args=(), device_types="cuda")
def wan_block(x: Tensor, e: Tensor, context: Tensor, params: List[Tensor], num_heads: int,
              grid: List[int], seq_lens: List[int], rope_tab: Tensor, i2v: bool, eps: float,
              fp8: int, keep_attn: bool, sp: int = 0) -> Tuple[Tensor, Tensor, Tensor]:
    """fp8: block.fp8_code -- bits 0-1 0 bf16, 1 e4m3 forward projections, 2 also the e4m3
    self-attention forward (config C5, block.Meta), from bit 2 the projections kept bf16; sp: 0
    or the prfl_amd.sp handle of the sequence-parallel group (Ulysses, block.Meta.sp).  x [B, L, C] (fp32, or bf16 for block 0), e [B, 6, C] fp32 (modulation + e0), context
    [B, Lc, C] bf16, params in block.param_names(i2v) order, grid = flattened (F, H, W) per
    sample.  Returns (out fp32 [B, L, C], kept self-attention output bf16 [B, L, C] and LSE fp32
    [B, H, L] when keep_attn, else empty).  sp: a sequence-parallel group handle (prfl_amd.sp;
    0 = none): x then holds this rank's tokens and the self-attention runs Ulysses-sharded, the
    kept output / LSE being the head-sharded ones in the same shapes."""
    meta = _meta(num_heads, grid, seq_lens, rope_tab, i2v, eps, fp8, sp)
    P = dict(zip(B.param_names(i2v), params))
    W = B.BF16Weights(P, fp8=fp8, need_bf16=False)
    outs, aos, lses = [], [], []
    for b in range(x.shape[0]):
        o, S = B.block_forward_one(P, W, x[b], e[b], context[b], meta, b, save=False,
                                   keep_attn=keep_attn)
        outs.append(o)
        if keep_attn:
            aos.append(S["attn"][0])
            lses.append(S["attn"][1])
    # one sample (every PRFL / PAVRM step): a view of the fresh per-sample buffers instead of a
    # stacked copy (1.5 GB of fp32 per 720p block forward, ~0.3 ms each)
    cat = (lambda ts: ts[0].unsqueeze(0)) if len(outs) == 1 else torch.stack
    out = cat(outs)
    if keep_attn:
        return out, cat(aos), cat(lses)
    return out, _empty(x, BF16), _empty(x, F32)


@wan_block.register_fake
def _(x, e, context, params, num_heads, grid, seq_lens, rope_tab, i2v, eps, fp8, keep_attn, sp=0):
    Bn, L, C = x.shape
    out = x.new_empty((Bn, L, C), dtype=F32)
    if keep_attn:
        return out, x.new_empty((Bn, L, C), dtype=BF16), x.new_empty((Bn, num_heads, L), dtype=F32)
    return out, _empty(x, BF16), _empty(x, F32)


@torch.library.custom_op("prfl::wan_block_backward", mutates_args=(), device_types="cuda")
def wan_block_backward(dout: Tensor, x: Tensor, e: Tensor, context: Tensor, params: List[Tensor],
                       ao: Tensor, lse: Tensor, num_heads: int, grid: List[int],
                       seq_lens: List[int], rope_tab: Tensor, i2v: bool, eps: float, fp8: int,
                       want_w: bool, want_ctx: bool, sp: int = 0) -> List[Tensor]:
    """Recompute the block forward (reusing a kept (ao, lse) when given), then the backward
    chain.  Returns [dx (x.dtype), de fp32, dctx (context.dtype or empty), *dparams (param
    dtype, or empty when not want_w)]."""
    meta = _meta(num_heads, grid, seq_lens, rope_tab, i2v, eps, fp8, sp)
    names = B.param_names(i2v)
    P = dict(zip(names, params))
    W = B.BF16Weights(P, fp8=fp8)
    G = {}
    dxs, des, dcs = [], [], []
    kept = ao.numel() > 0
    for b in range(x.shape[0]):
        _, S = B.block_forward_one(P, W, x[b], e[b], context[b], meta, b, save=True,
                                   attn=(ao[b], lse[b]) if kept else None)
        d = dout[b].to(F32).contiguous().clone()
        dx, de, dc = B.block_backward_one(P, W, x[b], e[b], context[b], meta, b, S, d, G,
                                          want_w=want_w)
        del S
        dxs.append(dx)
        des.append(de)
        dcs.append(dc)
    cat = (lambda ts: ts[0].unsqueeze(0)) if len(dxs) == 1 else torch.stack
    res = [cat(dxs).to(x.dtype), cat(des), cat(dcs).to(context.dtype) if want_ctx else _empty(context)]
    for n, p in zip(names, params):
        res.append(G[n].to(p.dtype) if want_w else _empty(p))
    return res


@wan_block_backward.register_fake
def _(dout, x, e, context, params, ao, lse, num_heads, grid, seq_lens, rope_tab, i2v, eps, fp8,
      want_w, want_ctx, sp=0):
    res = [torch.empty_like(x), e.new_empty(e.shape, dtype=F32),
           torch.empty_like(context) if want_ctx else _empty(context)]
    return res + [torch.empty_like(p) if want_w else _empty(p) for p in params]


def _wan_block_setup(ctx, inputs, output):
    x, e, context, params, num_heads, grid, seq_lens, rope_tab, i2v, eps, fp8, keep, sp = inputs
    _, ao, lse = output
    ctx.mark_non_differentiable(ao, lse)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(x, e, context, rope_tab, ao, lse, *params)
    ctx.args = (num_heads, list(grid), list(seq_lens), i2v, eps, fp8, sp)
    ctx.req = (x.requires_grad, e.requires_grad, context.requires_grad,
               [p.requires_grad for p in params])


def _wan_block_bwd(ctx, dout, _dao, _dlse):
    x, e, context, rope_tab, ao, lse, *params = ctx.saved_tensors
    nh, grid, seq_lens, i2v, eps, fp8, sp = ctx.args
    rx, re, rc, rp = ctx.req
    if ao.numel():                      # the kept (ao, lse) die with this node (block.py)
        B.credit_attn_stash(B.stash_bytes(ao, lse))
    # one entry per argument the caller passed (a trailing `sp` left at its default is not one)
    tail = (None,) * (len(ctx.needs_input_grad) - 4)
    if dout is None:
        return (None,) * 3 + ([None] * len(params),) + tail
    res = wan_block_backward(dout.contiguous(), x, e, context, params, ao, lse, nh, grid,
                             seq_lens, rope_tab, i2v, eps, fp8, any(rp), rc, sp)
    dps = [d if r else None for d, r in zip(res[3:], rp)]
    return (res[0] if rx else None, res[1] if re else None, res[2] if rc else None, dps) + tail


wan_block.register_autograd(_wan_block_bwd, setup_context=_wan_block_setup)


# ================================================================= bf16 Linear ==========
def _pad_rows(t, mult=8):
    """zero-pad dim 0 to a multiple of `mult` (GEMM N extents must be multiples of 8)."""
    n = t.shape[0]
    if n % mult == 0:
        return t
    out = torch.zeros((n + mult - 1) // mult * mult, *t.shape[1:], dtype=t.dtype, device=t.device)
    out[:n] = t
    return out


def _gelu_grad(x):
    k_beta, k_kappa = 0.7978845608028654, 0.044715
    t = torch.tanh(k_beta * (x + k_kappa * x * x * x))
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k_beta * (1 + 3 * k_kappa * x * x)


@torch.library.custom_op("prfl::linear_bf16", mutates_args=(), device_types="cuda")
def linear_bf16(x: Tensor, w: Tensor, b: Optional[Tensor], gelu: bool) -> Tuple[Tensor, Tensor]:
    """y = bf16(bf16(x) @ bf16(w)^T + bf16(b)) [GELU(tanh) fused]: the autocast nn.Linear.
    Returns (y bf16 [..., N], pre-activation bf16 [M, N] when gelu, else empty)."""
    shp = x.shape
    xb = x.reshape(-1, shp[-1]).to(BF16).contiguous()
    N = w.shape[0]
    wb = _pad_rows(ops.cast_bf16(w))
    bb = _pad_rows(ops.cast_bf16(b)) if b is not None else None
    if gelu:
        pre = torch.empty(xb.shape[0], wb.shape[0], dtype=BF16, device=x.device)
        y = ops.linear(xb, wb, bb, ops.EPI_GELU, aux=pre)
    else:
        pre = _empty(xb)
        y = ops.linear(xb, wb, bb)
    if y.shape[1] != N:
        y = y[:, :N].contiguous()
        pre = pre[:, :N].contiguous() if gelu else pre
    return y.view(*shp[:-1], N), pre


@linear_bf16.register_fake
def _(x, w, b, gelu):
    M = x.numel() // x.shape[-1]
    y = x.new_empty((*x.shape[:-1], w.shape[0]), dtype=BF16)
    return y, (x.new_empty((M, w.shape[0]), dtype=BF16) if gelu else _empty(x, BF16))


@torch.library.custom_op("prfl::linear_bf16_backward", mutates_args=(), device_types="cuda")
def linear_bf16_backward(dy: Tensor, x: Tensor, w: Tensor, pre: Tensor, need_dx: bool,
                         need_dw: bool, need_db: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """dX = dY W (bf16, returned in x.dtype), dW = dY^T X (fp32), db = colsum(dY) (fp32)."""
    N = w.shape[0]
    dy2 = dy.reshape(-1, N).to(BF16).contiguous()
    if pre.numel():      # d(pre-activation) = bf16(dy * gelu'(pre)); small (text tokens only)
        dy2 = (dy2.float() * _gelu_grad(pre.float())).to(BF16)
    wb = _pad_rows(ops.cast_bf16(w))
    if wb.shape[0] != N:   # out_features not a multiple of 8 (e.g. the reward MLP's fc3)
        dyp = torch.zeros(dy2.shape[0], wb.shape[0], dtype=BF16, device=dy2.device)
        dyp[:, :N] = dy2
        dy2 = dyp
    dx = ops.linear_dx(dy2, wb).view(x.shape).to(x.dtype) if need_dx else _empty(x)
    dw = ops.linear_dw(dy2, x.reshape(-1, x.shape[-1]).to(BF16).contiguous())[:N].contiguous() \
        if need_dw else _empty(w, F32)
    db = ops.colsum(dy2)[:N].contiguous() if need_db else _empty(w, F32)
    return dx, dw, db


@linear_bf16_backward.register_fake
def _(dy, x, w, pre, need_dx, need_dw, need_db):
    return (torch.empty_like(x) if need_dx else _empty(x),
            w.new_empty(w.shape, dtype=F32) if need_dw else _empty(w, F32),
            w.new_empty((w.shape[0],), dtype=F32) if need_db else _empty(w, F32))


def _linear_setup(ctx, inputs, output):
    x, w, b, gelu = inputs
    _, pre = output
    ctx.mark_non_differentiable(pre)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(x, w, pre)
    ctx.req = (x.requires_grad, w.requires_grad, b is not None and b.requires_grad)
    ctx.b_dtype = b.dtype if b is not None else None


def _linear_bwd(ctx, dy, _dpre):
    x, w, pre = ctx.saved_tensors
    rx, rw, rb = ctx.req
    if dy is None:
        return None, None, None, None
    dx, dw, db = linear_bf16_backward(dy.contiguous(), x, w, pre, rx, rw, rb)
    return (dx if rx else None, dw.to(w.dtype) if rw else None,
            db.to(ctx.b_dtype) if rb else None, None)


linear_bf16.register_autograd(_linear_bwd, setup_context=_linear_setup)


# ============================================================ flash_attention API ========
@torch.library.custom_op("prfl::flash_attention", mutates_args=(), device_types="cuda")
def flash_attention(q: Tensor, k: Tensor, v: Tensor, k_lens: Optional[List[int]],
                    scale: float) -> Tuple[Tensor, Tensor]:
    """q [B, Lq, N, 128], k/v [B, Lk, N, 128] (any float dtype; computed in bf16) ->
    (o bf16 [B, Lq, N, 128], lse2 fp32 [B, N, Lq]); keys >= k_lens[b] masked."""
    Bn, Lq, N, D = q.shape
    Lk = k.shape[1]
    if D != 128 or k.shape[2] != N:
        raise ValueError("prfl::flash_attention: head_dim 128 and Nq == Nk")
    qb = q.to(BF16).reshape(Bn, Lq, N * D).contiguous()
    kb = k.to(BF16).reshape(Bn, Lk, N * D).contiguous()
    vb = v.to(BF16).reshape(Bn, Lk, N * D).contiguous()
    o = torch.empty(Bn, Lq, N * D, dtype=BF16, device=q.device)
    lses = []
    for b in range(Bn):
        kl = Lk if k_lens is None else int(k_lens[b])
        _, lse = ops.attn_fwd(qb[b], kb[b], vb[b], N, k_len=kl, out=o[b], scale=scale)
        lses.append(lse)
    return o.view(Bn, Lq, N, D), torch.stack(lses)


@flash_attention.register_fake
def _(q, k, v, k_lens, scale):
    Bn, Lq, N, D = q.shape
    return q.new_empty((Bn, Lq, N, D), dtype=BF16), q.new_empty((Bn, N, Lq), dtype=F32)


@torch.library.custom_op("prfl::flash_attention_backward", mutates_args=(), device_types="cuda")
def flash_attention_backward(do: Tensor, q: Tensor, k: Tensor, v: Tensor, o: Tensor, lse: Tensor,
                             k_lens: Optional[List[int]], scale: float) -> Tuple[Tensor, Tensor, Tensor]:
    Bn, Lq, N, D = q.shape
    Lk = k.shape[1]
    qb = q.to(BF16).reshape(Bn, Lq, N * D).contiguous()
    kb = k.to(BF16).reshape(Bn, Lk, N * D).contiguous()
    vb = v.to(BF16).reshape(Bn, Lk, N * D).contiguous()
    ob = o.reshape(Bn, Lq, N * D)
    dob = do.to(BF16).reshape(Bn, Lq, N * D).contiguous()
    dq, dk, dv = torch.empty_like(qb), torch.empty_like(kb), torch.empty_like(vb)
    for b in range(Bn):
        kl = Lk if k_lens is None else int(k_lens[b])
        ops.attn_bwd(qb[b], kb[b], vb[b], ob[b], dob[b], lse[b], N, k_len=kl, dq=dq[b], dk=dk[b],
                     dv=dv[b], scale=scale)
    return (dq.view(q.shape).to(q.dtype), dk.view(k.shape).to(k.dtype),
            dv.view(v.shape).to(v.dtype))


@flash_attention_backward.register_fake
def _(do, q, k, v, o, lse, k_lens, scale):
    return torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)


def _fa_setup(ctx, inputs, output):
    q, k, v, k_lens, scale = inputs
    o, lse = output
    ctx.mark_non_differentiable(lse)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(q, k, v, o, lse)
    ctx.k_lens, ctx.scale = k_lens, scale


def _fa_bwd(ctx, do, _dlse):
    q, k, v, o, lse = ctx.saved_tensors
    if do is None:
        return None, None, None, None, None
    dq, dk, dv = flash_attention_backward(do.contiguous(), q, k, v, o, lse, ctx.k_lens, ctx.scale)
    return dq, dk, dv, None, None


flash_attention.register_autograd(_fa_bwd, setup_context=_fa_setup)


# ================================================= single-query pooling (reward head) ====
@torch.library.custom_op("prfl::query_pool", mutates_args=(), device_types="cuda")
def query_pool(q: Tensor, kv: Tensor, num_heads: int, scale: float) -> Tuple[Tensor, Tensor, Tensor]:
    """softmax(q k^T * scale) v per head for ONE query per sample: q [N, E] bf16, kv [N, L, 2E]
    bf16 (k | v, the MHA in-projection output) -> (o bf16 [N, E], lse2 fp32 [N, H], o32 fp32
    [N, E]: o before its bf16 rounding, kept for the backward's D)."""
    return ops.query_pool_fwd(q.contiguous(), kv, num_heads, scale)


@query_pool.register_fake
def _(q, kv, num_heads, scale):
    return (q.new_empty(q.shape, dtype=BF16), q.new_empty((q.shape[0], num_heads), dtype=F32),
            q.new_empty(q.shape, dtype=F32))


@torch.library.custom_op("prfl::query_pool_backward", mutates_args=(), device_types="cuda")
def query_pool_backward(do: Tensor, q: Tensor, kv: Tensor, o32: Tensor, lse: Tensor,
                        num_heads: int, scale: float) -> Tuple[Tensor, Tensor]:
    """(dq fp32 [N, E], dkv bf16 [N, L, 2E])."""
    return ops.query_pool_bwd(do.to(BF16).contiguous(), q.contiguous(), kv, o32, lse, num_heads,
                              scale)


@query_pool_backward.register_fake
def _(do, q, kv, o32, lse, num_heads, scale):
    return q.new_empty(q.shape, dtype=F32), torch.empty_like(kv)


def _qp_setup(ctx, inputs, output):
    q, kv, num_heads, scale = inputs
    o, lse, o32 = output
    ctx.mark_non_differentiable(lse, o32)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(q, kv, o32, lse)
    ctx.args = (num_heads, scale)


def _qp_bwd(ctx, do, _dlse, _do32):
    q, kv, o32, lse = ctx.saved_tensors
    if do is None:
        return None, None, None, None
    dq, dkv = query_pool_backward(do.contiguous(), q, kv, o32, lse, *ctx.args)
    return dq.to(q.dtype), dkv, None, None


query_pool.register_autograd(_qp_bwd, setup_context=_qp_setup)


# ====================================================================== UniPC step =======
@torch.library.custom_op("prfl::unipc_step", mutates_args=(), device_types="cuda")
def unipc_step(model_output: Tensor, sample: Tensor, last_sample: Optional[Tensor],
               hist1: Optional[Tensor], hist2: Optional[Tensor], coef: List[float],
               corr_order: int, pred_order: int) -> Tuple[Tensor, Tensor, Tensor]:
    """Fused FlowUniPC update (csrc/unipc.hip): (m_t fp32, corrected sample bf16 — empty when
    corr_order == 0, the caller keeps `sample` — , prev_sample bf16)."""
    m_t, sample_c, prev = ops.unipc_step_fwd(sample, model_output, last_sample, hist1, hist2,
                                             coef, corr_order, pred_order)
    return m_t, (sample_c if corr_order else _empty(sample)), prev


@unipc_step.register_fake
def _(model_output, sample, last_sample, hist1, hist2, coef, corr_order, pred_order):
    return (sample.new_empty(sample.shape, dtype=F32),
            torch.empty_like(sample) if corr_order else _empty(sample), torch.empty_like(sample))


@torch.library.custom_op("prfl::unipc_step_backward", mutates_args=(), device_types="cuda")
def unipc_step_backward(grad_prev: Tensor, coef: List[float], corr_order: int,
                        pred_order: int) -> Tensor:
    return ops.unipc_step_bwd(grad_prev, coef, corr_order, pred_order)


@unipc_step_backward.register_fake
def _(grad_prev, coef, corr_order, pred_order):
    return grad_prev.new_empty(grad_prev.shape, dtype=F32)


def _unipc_setup(ctx, inputs, output):
    mo, sample, last, h1, h2, coef, corr, pred = inputs
    m_t, sample_c, prev = output
    ctx.mark_non_differentiable(sample_c)
    ctx.set_materialize_grads(False)
    ctx.args = (list(coef), corr, pred)


def _unipc_bwd(ctx, g_mt, g_sc, g_prev):
    if g_mt is not None:
        raise NotImplementedError("fused UniPC step: gradient through the stored m_t history")
    gmo = unipc_step_backward(g_prev.contiguous(), *ctx.args) if g_prev is not None else None
    return gmo, None, None, None, None, None, None, None


unipc_step.register_autograd(_unipc_bwd, setup_context=_unipc_setup)


def unipc_update(model_output, sample, last_sample, hist1, hist2, coef, corr_order, pred_order):
    """(m_t, corrected sample, prev_sample) of one FlowUniPC step; differentiable w.r.t.
    model_output only — the one input that carries the reward gradient at train_prfl.py:734
    (the sample comes out of the no-grad rollout)."""
    for t in (sample, last_sample, hist1, hist2):
        if t is not None and t.requires_grad and torch.is_grad_enabled():
            raise NotImplementedError("fused UniPC step differentiates w.r.t. model_output only")
    m_t, sample_c, prev = unipc_step(model_output, sample, last_sample, hist1, hist2,
                                     [float(c) for c in coef], int(corr_order), int(pred_order))
    return m_t, (sample_c if corr_order else sample), prev
