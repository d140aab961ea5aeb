"""GPU fp32 checker for a whole WanAttentionBlock forward + backward at real geometry.

TEST INFRASTRUCTURE.  The CPU oracle (`oracle/wan_oracle.py`) restates the reference block with its
autocast cast points, but its autograd attention materialises the L x L scores (40 heads x
32 760^2 fp32 = 172 GB at 480p x 81f).  This module runs the SAME `wan_oracle.block_forward` on the
GPU in fp32 with one substitution: the attention is `ChunkedFlashAttention`, the oracle's FA2
numerics (`wan_oracle._FlashAttention`: bf16 q / k / v, P rounded to bf16 for P.V while the
normaliser sums fp32 P, bf16 output; backward dV = P^T dO, D = rowsum(dO * bf16 O), dS = P (dP - D))
computed over query chunks with the probabilities recomputed from the saved LSE in the backward,
so nothing L x L is ever held.  `tests/test_gpu_configs.py` validates this checker against the CPU
oracle at L = 4 200 in the same test before trusting it at L = 32 760.
"""
import contextlib

import torch

from oracle import wan_oracle as O


class ChunkedFlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, k_len, scale, chunk):
        # q [1, Lq, N, D], k / v [1, Lk, N, D] (fp32 values)
        qb, kb, vb = O.bf(q[0]).transpose(0, 1), O.bf(k[0]).transpose(0, 1), O.bf(v[0]).transpose(0, 1)
        N, Lq, D = qb.shape
        Lk = kb.shape[1]
        o = torch.empty(N, Lq, D, device=q.device)
        lse = torch.empty(N, Lq, 1, device=q.device)
        for c0 in range(0, Lq, chunk):
            cs = slice(c0, min(Lq, c0 + chunk))
            s = torch.bmm(qb[:, cs], kb.transpose(1, 2)).mul_(scale)
            if k_len is not None and int(k_len) < Lk:
                s[:, :, int(k_len):] = float("-inf")
            m = s.amax(-1, keepdim=True)
            p = s.sub_(m).exp_()
            l = p.sum(-1, keepdim=True)
            o[:, cs] = O.bf(torch.bmm(O.bf(p), vb) / l)
            lse[:, cs] = m + torch.log(l)
            del s, p
        ctx.save_for_backward(qb, kb, vb, o, lse)
        ctx.k_len, ctx.scale, ctx.chunk = k_len, scale, chunk
        return o.transpose(0, 1).unsqueeze(0)

    @staticmethod
    def backward(ctx, do):
        qb, kb, vb, o, lse = ctx.saved_tensors
        scale, chunk, k_len = ctx.scale, ctx.chunk, ctx.k_len
        N, Lq, D = qb.shape
        Lk = kb.shape[1]
        dob = O.bf(do[0]).transpose(0, 1)
        delta = (dob * o).sum(-1, keepdim=True)
        dq = torch.empty_like(qb)
        dk = torch.zeros_like(kb)
        dv = torch.zeros_like(vb)
        for c0 in range(0, Lq, chunk):
            cs = slice(c0, min(Lq, c0 + chunk))
            s = torch.bmm(qb[:, cs], kb.transpose(1, 2)).mul_(scale)
            if k_len is not None and int(k_len) < Lk:
                s[:, :, int(k_len):] = float("-inf")
            P = s.sub_(lse[:, cs]).exp_()
            dv += torch.bmm(P.transpose(1, 2), dob[:, cs])
            dp = torch.bmm(dob[:, cs], vb.transpose(1, 2))
            ds = P.mul_(dp.sub_(delta[:, cs]))
            del dp
            dq[:, cs] = torch.bmm(ds, kb) * scale
            dk += torch.bmm(ds.transpose(1, 2), qb[:, cs]) * scale
            del ds
        t = lambda x: x.transpose(0, 1).unsqueeze(0)  # noqa: E731
        return t(dq), t(dk), t(dv), None, None, None


def chunked_attention(chunk=512):
    def attention(q, k, v, k_len=None, scale=None, q_chunk=None):
        sc = scale if scale is not None else q.shape[-1] ** -0.5
        return ChunkedFlashAttention.apply(q.float(), k.float(), v.float(), k_len, sc, chunk)
    return attention


@contextlib.contextmanager
def oracle_on(device, chunk=512):
    """The oracle's module-level helpers create tensors without a device: run them under the
    default device, with the chunked attention swapped in."""
    saved = O.attention
    O.attention = chunked_attention(chunk)
    try:
        with torch.device(device):
            yield
    finally:
        O.attention = saved


def block_grads(P, pre, x, e, ctx, grid, seq_len, nh, up, device="cuda", i2v=False, chunk=512):
    """wan_oracle.block_forward + backward of sum(out * up) on `device` in fp32.  Returns
    (out, dx, {param name: grad}) on the host."""
    Pd = {k: v.detach().to(device).float().requires_grad_(True) for k, v in P.items()
          if k.startswith(pre)}
    xd = x.detach().to(device).requires_grad_(True)
    with oracle_on(device, chunk):
        out = O.block_forward(Pd, pre, xd, e.to(device), torch.tensor([grid], device=device),
                              O.rope_freqs(128).to(device), ctx.to(device).float(), nh,
                              seq_len=seq_len, i2v=i2v)
        (out * up.to(device)).sum().backward()
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize()
    G = {k[len(pre):]: v.grad.detach().cpu() for k, v in Pd.items() if v.grad is not None}
    res = out.detach().cpu(), xd.grad.detach().cpu(), G
    del Pd, xd, out
    if torch.device(device).type == "cuda":
        torch.cuda.empty_cache()
    return res
