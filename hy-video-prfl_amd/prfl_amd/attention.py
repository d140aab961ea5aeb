"""`flash_attention` drop-in (`wan/modules/attention.py:24-130`) on the HIP kernels.

q [B, Lq, Nq, 128], k/v [B, Lk, Nk, 128] (Nq == Nk), any float dtype -> bf16 compute, output in
q's dtype; `k_lens` masks keys per sample; causal / dropout / sliding windows are not used by
Wan training and are rejected.  Differentiable (prfl_attn_bwd).
"""
import torch

from . import ops

BF16 = torch.bfloat16


class FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, k_lens, scale):
        B, Lq, N, D = q.shape
        Lk = k.shape[1]
        assert D == 128 and k.shape[2] == N, "head_dim 128, Nq == Nk"
        qb = q.to(BF16).reshape(B, Lq, N * D).contiguous()
        kb = k.to(BF16).reshape(B, Lk, N * D).contiguous()
        vb = v.to(BF16).reshape(B, Lk, N * D).contiguous()
        o = torch.empty(B, Lq, N * D, dtype=BF16, device=q.device)
        lses = []
        for b in range(B):
            kl = Lk if k_lens is None else int(k_lens[b])
            _, lse = ops.attn_fwd(qb[b], kb[b], vb[b], N, k_len=kl, out=o[b], scale=scale)
            lses.append(lse)
        ctx.save_for_backward(qb, kb, vb, o, torch.stack(lses))
        ctx.k_lens, ctx.scale, ctx.shape = k_lens, scale, (B, Lq, Lk, N, D)
        ctx.dtypes = (q.dtype, k.dtype, v.dtype)
        return o.view(B, Lq, N, D)

    @staticmethod
    def backward(ctx, do):
        qb, kb, vb, o, lse = ctx.saved_tensors
        B, Lq, Lk, N, D = ctx.shape
        dob = do.to(BF16).reshape(B, Lq, N * D).contiguous()
        dq, dk, dv = torch.empty_like(qb), torch.empty_like(kb), torch.empty_like(vb)
        for b in range(B):
            kl = Lk if ctx.k_lens is None else int(ctx.k_lens[b])
            ops.attn_bwd(qb[b], kb[b], vb[b], o[b], dob[b], lse[b], N, k_len=kl, dq=dq[b],
                         dk=dk[b], dv=dv[b], scale=ctx.scale)
        shp = lambda t, L: t.view(B, L, N, D)  # noqa: E731
        return (shp(dq, Lq).to(ctx.dtypes[0]), shp(dk, Lk).to(ctx.dtypes[1]),
                shp(dv, Lk).to(ctx.dtypes[2]), None, None)


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
    return FlashAttnFn.apply(q, k, v, kl, scale).to(out_dtype)


attention = flash_attention
