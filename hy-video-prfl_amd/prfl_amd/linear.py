"""Autocast-equivalent bf16 Linear on the HIP GEMM, as an autograd node.

Forward: y = bf16(bf16(x) @ bf16(W)^T + bf16(b)) [optionally GELU(tanh) fused, as in the
text embedding `model.py:499-501`].  Backward: dX = dY @ W (bf16), dW = dY^T @ X (fp32),
db = colsum(dY) — the grads autocast's bf16 F.linear produces, accumulated in fp32.
"""
import torch

from . import ops
from .ops import BF16


class LinearBF16Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, gelu):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        xb = x2 if x2.dtype == BF16 else x2.to(BF16)
        xb = xb.contiguous()
        wb = _pad_rows(ops.cast_bf16(w))
        bb = _pad_rows(ops.cast_bf16(b)) if b is not None else None
        if gelu:
            pre = torch.empty(xb.shape[0], w.shape[0], dtype=BF16, device=x.device)
            y = ops.linear(xb, wb, bb, ops.EPI_GELU, aux=pre)
        else:
            pre = None
            y = ops.linear(xb, wb, bb)
        ctx.save_for_backward(xb, w, pre)
        ctx.has_bias = b is not None
        ctx.x_dtype = x.dtype
        ctx.shp = shp
        if y.shape[1] != w.shape[0]:
            y = y[:, :w.shape[0]].contiguous()
            pre = pre[:, :w.shape[0]] if pre is not None else None
        return y.view(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        xb, w, pre = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        dy2 = (dy2 if dy2.dtype == BF16 else dy2.to(BF16)).contiguous()
        N = w.shape[0]
        wb = _pad_rows(ops.cast_bf16(w))
        if pre is not None:  # d(pre-activation) = bf16(dy * gelu'(pre)); small (text tokens only)
            dy2 = (dy2.float() * _gelu_grad(pre[:, :N].float())).to(BF16)
        if wb.shape[0] != N:   # out_features not a multiple of 8 (e.g. the reward MLP's fc3)
            dyp = torch.zeros(dy2.shape[0], wb.shape[0], dtype=BF16, device=dy2.device)
            dyp[:, :N] = dy2
            dy2 = dyp
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = ops.linear_dx(dy2, wb).view(ctx.shp).to(ctx.x_dtype)
        if ctx.needs_input_grad[1]:
            dw = ops.linear_dw(dy2, xb)[:N]
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = ops.colsum(dy2)[:N]
        return dx, dw, db, None


def _pad_rows(t, mult=8):
    """zero-pad dim 0 to a multiple of `mult` (GEMM N extents must be multiples of 8)."""
    n = t.shape[0]
    if n % mult == 0:
        return t
    out = torch.zeros((n + mult - 1) // mult * mult, *t.shape[1:], dtype=t.dtype, device=t.device)
    out[:n] = t
    return out


def _gelu_grad(x):
    k_beta = 0.7978845608028654
    k_kappa = 0.044715
    inner = k_beta * (x + k_kappa * x * x * x)
    t = torch.tanh(inner)
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k_beta * (1 + 3 * k_kappa * x * x)


def linear_bf16(x, w, b=None, gelu=False):
    return LinearBF16Fn.apply(x, w, b, gelu)
