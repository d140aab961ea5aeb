"""`flash_attention` drop-in (`wan/modules/attention.py:24-130`) on the HIP kernels, through the
`prfl::flash_attention` custom op (forward + registered backward).

q [B, Lq, Nq, 128], k/v [B, Lk, Nk, 128] (Nq == Nk), any float dtype -> bf16 compute, output in
q's dtype; `k_lens` masks keys per sample; causal / dropout / sliding windows are not used by
Wan training and are rejected.
"""
import torch

from . import custom_ops

__all__ = ["flash_attention", "attention"]        # attention.py:18-21


def flash_attention(q, k, v, q_lens=None, k_lens=None, dropout_p=0., softmax_scale=None,
                    q_scale=None, causal=False, window_size=(-1, -1), deterministic=False,
                    dtype=torch.bfloat16, version=None):
    if causal or dropout_p or tuple(window_size) != (-1, -1) or q_lens is not None:
        raise NotImplementedError("Wan training uses non-causal, full-window, dropout-free attention")
    if q_scale is not None:
        q = q * q_scale
    out_dtype = q.dtype
    scale = softmax_scale if softmax_scale is not None else q.shape[-1] ** -0.5
    kl = None if k_lens is None else [int(x) for x in k_lens.tolist()]
    return custom_ops.flash_attention(q, k, v, kl, float(scale))[0].to(out_dtype)


attention = flash_attention
