"""`flash_attention` drop-in (`wan/modules/attention.py:24-130`) on the HIP kernels, through the
`prfl::flash_attention` custom op (forward + registered backward).

q [B, Lq, Nq, 128], k/v [B, Lk, Nk, 128] (Nq == Nk), any float dtype -> bf16 compute, output in
q's dtype; `k_lens` masks keys per sample.  `q_lens` is accepted as the reference accepts it:
its varlen output is unflattened to [B, Lq] (`attention.py:110,127`), which only succeeds when
every q_lens[b] == Lq, so a shorter length raises here as it does there.  Lengths given as a list
or a host tensor cost no device sync; a device tensor costs one (the reference's `u[:v]` slicing
syncs on the same values).  Causal / dropout / sliding windows are not used by Wan training and
are rejected; `deterministic` is always honoured (the backward has no atomics); `version` is
ignored.
"""
import torch

from . import custom_ops

__all__ = ["flash_attention", "attention"]        # attention.py:18-21

_HALF = (torch.float16, torch.bfloat16)


def _lens(x, n, full, what, lo=0):
    if x is None:
        return None
    vals = [int(t) for t in (x.tolist() if torch.is_tensor(x) else x)]
    if len(vals) != n:
        raise ValueError(f"{what} has {len(vals)} entries for a batch of {n}")
    if any(t < lo or t > full for t in vals):
        raise ValueError(f"{what} {vals} outside [{lo}, {full}]")
    return vals


def flash_attention(q, k, v, q_lens=None, k_lens=None, dropout_p=0., softmax_scale=None,
                    q_scale=None, causal=False, window_size=(-1, -1), deterministic=False,
                    dtype=torch.bfloat16, version=None):
    assert dtype in _HALF                                   # attention.py:53
    if causal or dropout_p or tuple(window_size) != (-1, -1):
        raise NotImplementedError("Wan training uses non-causal, full-window, dropout-free attention")
    b, lq, lk, out_dtype = q.shape[0], q.shape[1], k.shape[1], q.dtype
    ql = _lens(q_lens, b, lq, "q_lens")
    if ql is not None and any(t != lq for t in ql):
        # attention.py:69,110: cat(u[:v]) holds sum(q_lens) rows, unflatten(0, (b, lq)) needs b * lq
        raise RuntimeError(f"q_lens {ql}: the varlen output of {sum(ql)} rows cannot be "
                           f"unflattened to ({b}, {lq})")
    kl = _lens(k_lens, b, lk, "k_lens", lo=1)
    if q_scale is not None:                                 # attention.py:59-86: half, to v's, scale
        vd = v.dtype if v.dtype in _HALF else dtype
        q = (q if q.dtype in _HALF else q.to(dtype)).to(vd) * q_scale
    scale = softmax_scale if softmax_scale is not None else q.shape[-1] ** -0.5
    return custom_ops.flash_attention(q, k, v, kl, float(scale))[0].to(out_dtype)


attention = flash_attention
