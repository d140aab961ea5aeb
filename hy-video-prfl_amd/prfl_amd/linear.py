"""Autocast-equivalent bf16 Linear on the HIP GEMM (the `prfl::linear_bf16` custom op).

Forward: y = bf16(bf16(x) @ bf16(W)^T + bf16(b)) [optionally GELU(tanh) fused, as in the
text embedding `model.py:499-501`].  Backward (`prfl::linear_bf16_backward`): dX = dY @ W (bf16),
dW = dY^T @ X (fp32), db = colsum(dY) — the grads autocast's bf16 F.linear produces, accumulated
in fp32.
"""
from . import custom_ops


def linear_bf16(x, w, b=None, gelu=False):
    return custom_ops.linear_bf16(x, w, b, bool(gelu))[0]
