"""CPU stand-ins for the C-ABI wrappers of `prfl_amd.ops` and the `prfl::` custom ops — TEST
INFRASTRUCTURE ONLY, installed in spawned test processes (never in the product, which registers
CUDA kernels only and raises on a CPU tensor).

They let the multi-rank CPU tests (gloo) run the product's own host logic — the fused block's
forward / backward chain in `prfl_amd/block.py`, its sequence-parallel exchange (`prfl_amd/sp.py`),
the custom-op plumbing and WanModel — with each kernel replaced by a torch fp32 restatement of the
same contract (include/prfl_hip.h: the bf16 rounding points of each entry, the log2-unit q of the
*_l2q attention entries, the row offset of prfl_rms_rope_*_pos).  What such a test checks is the
host side (shapes, offsets, exchanges, accumulation), not the HIP kernels, whose parity the GPU
suite holds against the oracle.
"""
import math

import torch

BF16, F32 = torch.bfloat16, torch.float32
EPI_BF16, EPI_GELU, EPI_RESID, EPI_F32, EPI_DGELU = range(5)
LN2 = math.log(2.0)


def bf(x):
    return x.to(BF16).to(F32)


def _gelu(x):
    return 0.5 * x * (1 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))


def _gelu_grad(x):
    k, a = 0.7978845608028654, 0.044715
    t = torch.tanh(k * (x + a * x ** 3))
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k * (1 + 3 * a * x * x)


def _put(out, val):
    if out is None:
        return val
    out.copy_(val)
    return out


# ------------------------------------------------------------------------------- GEMMs ------
def _mm(a, b):
    """fp64 products rounded once to fp32: a row's result does not depend on how the rows are
    partitioned (sequence-parallel ranks vs one process), so the multi-rank tests compare the
    host logic, not BLAS blocking."""
    return (a.double() @ b.double()).float()


def _epi(acc, epilogue, bias, gate, res, aux, out, accumulate=False):
    if epilogue == EPI_F32:
        if accumulate:
            out.add_(acc)
            return out
        return _put(out, acc)
    y = acc + (bias.float() if bias is not None else 0)
    if epilogue == EPI_BF16:
        return _put(out, y.to(BF16))
    if epilogue == EPI_GELU:
        pre = bf(y)
        if aux is not None:
            aux.copy_(pre.to(BF16))
        return _put(out, _gelu(pre).to(BF16))
    if epilogue == EPI_RESID:
        yb = bf(y)
        if aux is not None:
            aux.copy_(yb.to(BF16))
        g = gate.float() if gate is not None else 1.0
        return _put(out, res.float() + yb * g)
    if epilogue == EPI_DGELU:
        return _put(out, (bf(acc) * _gelu_grad(aux.float())).to(BF16))
    raise ValueError(epilogue)


def gemm(a, b, c, M, N, K, a_kmajor=True, b_kmajor=True, epilogue=EPI_BF16, bias=None, gate=None,
         res=None, aux=None, accumulate=False, tile=0):
    A = a.float() if a_kmajor else a.float().t()          # [M, K]
    Bm = b.float() if b_kmajor else b.float().t()         # [N, K]
    return _epi(_mm(A[:M, :K], Bm[:N, :K].t()), epilogue, bias, gate, res, aux, c, accumulate)


def linear(x, w, bias=None, epilogue=EPI_BF16, out=None, gate=None, res=None, aux=None, tile=0):
    return _epi(_mm(x, w.t()), epilogue, bias, gate, res, aux, out)


def linear_t(x, wt, bias=None, epilogue=EPI_BF16, out=None, gate=None, res=None, aux=None):
    return _epi(_mm(x, wt), epilogue, bias, gate, res, aux, out)


def linear_dx(dy, w, out=None, epilogue=EPI_BF16, aux=None):
    return _epi(_mm(dy, w), epilogue, None, None, None, aux, out)


def linear_dw(dy, x, out=None, accumulate=False):
    return _epi(_mm(dy.t(), x), EPI_F32, None, None, None, None, out, accumulate)


def cast_bf16(src, dst=None):
    v = src.to(BF16)
    return v if dst is None else dst.view(src.shape).copy_(v)


def cast_bf16_t(w, dst=None):
    return _put(dst, w.t().to(BF16))


def colsum(x, out=None, accumulate=False):
    s = x.double().sum(0).float()
    if out is not None and accumulate:
        return out.add_(s)
    return _put(out, s)


def gate_bwd(dx, y, gate, dy_out=None, want_gate=True, want_bias=True):
    g = gate.float() if gate is not None else 1.0
    dy = (dx.float() * g).to(BF16)
    dy_out = _put(dy_out, dy)
    dgate = (dx.double() * y.double()).sum(0).float() if (want_gate and y is not None) else None
    dbias = dy.double().sum(0).float() if want_bias else None
    return dy_out, dgate, dbias


# ------------------------------------------------------------------------------- norms ------
def ln_mod_fwd(x, scale=None, shift=None, w=None, b=None, eps=1e-6, out=None):
    xf = x.float()
    mean = xf.mean(-1)
    rstd = torch.rsqrt(((xf - mean[:, None]) ** 2).mean(-1) + eps)
    xh = (xf - mean[:, None]) * rstd[:, None]
    if w is None:
        if x.dtype == BF16:
            xh = bf(xh)
        y = xh * (1 + scale.float()) + shift.float()
    else:
        y = xh * w.float() + (b.float() if b is not None else 0)
    return _put(out, y.to(BF16)), mean, rstd


def ln_mod_bwd(dy, x, mean, rstd, dx, scale=None, w=None, accumulate=True):
    xf, d = x.float(), dy.float()
    xh = (xf - mean[:, None]) * rstd[:, None]
    xu = bf(xh) if (w is None and x.dtype == BF16) else xh
    gg = d * (w.float() if w is not None else 1 + scale.float())
    m1 = gg.mean(-1, keepdim=True)
    m2 = (gg * xh).mean(-1, keepdim=True)
    o = rstd[:, None] * (gg - m1 - xh * m2)
    if accumulate:
        dx.add_(o)
    else:
        dx.copy_(o)
    return (d.double() * xu).sum(0).float(), d.double().sum(0).float()


def _rope_cs(rope_tab, grid, row0, L, C):
    """per (row, pair) (cos, sin) [L, C/2] and the rotated-row mask, as rope_pos / rope_index."""
    F_, H_, W_ = grid
    rows = torch.arange(L) + row0
    rot = rows < F_ * H_ * W_
    pf, ph, pw = rows // (H_ * W_), (rows // W_) % H_, rows % W_
    pair = torch.arange(C // 2) % 64
    idx = torch.where(pair < 22, pf[:, None], torch.where(pair < 43, ph[:, None], pw[:, None]))
    idx = idx.clamp(max=1023)
    tab = rope_tab.float().view(1024, 64, 2)
    cs = tab[idx, pair[None, :].expand(L, -1)]
    return cs[..., 0], cs[..., 1], rot


def rms_rope_fwd(x, w, eps=1e-6, rope_tab=None, grid=(0, 0, 0), out=None, out_scale=1.0, row0=0):
    L, C = x.shape
    xf = x.float()
    rstd = torch.rsqrt((xf * xf).mean(-1) + eps)
    y = bf(xf * rstd[:, None]) * w.float()
    if rope_tab is not None and grid[0] * grid[1] * grid[2] > 0:
        c, s, rot = _rope_cs(rope_tab, grid, row0, L, C)
        a, b2 = y[:, 0::2], y[:, 1::2]
        yr = torch.stack([a * c - b2 * s, a * s + b2 * c], dim=-1).flatten(1)
        y = torch.where(rot[:, None], yr, y)
    return _put(out, (y * out_scale).to(BF16)), rstd


def rms_rope_bwd(dout, x, rstd, w, rope_tab=None, grid=(0, 0, 0), dx=None, out_scale=1.0, row0=0):
    L, C = x.shape
    g = dout.float() * out_scale
    if rope_tab is not None and grid[0] * grid[1] * grid[2] > 0:
        c, s, rot = _rope_cs(rope_tab, grid, row0, L, C)
        ga, gb = g[:, 0::2], g[:, 1::2]
        gr = torch.stack([ga * c + gb * s, gb * c - ga * s], dim=-1).flatten(1)
        g = torch.where(rot[:, None], gr, g)
    xh = x.float() * rstd[:, None]
    d = bf(g * w.float())
    m = (d * xh).mean(-1, keepdim=True)
    out = (rstd[:, None] * (d - xh * m)).to(BF16)
    return _put(dx, out), (g.double() * bf(xh)).sum(0).float()


# ---------------------------------------------------------------------------- attention -----
def _scores(q, k, nh, k_len, scale, q_log2):
    Lq, Lk = q.shape[0], k.shape[0]
    qh = q.float().view(Lq, nh, 128).transpose(0, 1)
    kh = k.float().view(Lk, nh, 128).transpose(0, 1)
    s2 = _mm(qh, kh.transpose(1, 2))                       # [H, Lq, Lk]
    if not q_log2:
        s2 = s2 * (scale * 1.4426950408889634)
    if k_len is not None and k_len < Lk:
        s2[:, :, k_len:] = float("-inf")
    return s2, qh, kh


def attn_fwd(q, k, v, num_heads, k_len=None, out=None, scale=None, q_log2=False):
    sc = scale if scale is not None else 1 / math.sqrt(128)
    Lq, Lk = q.shape[0], k.shape[0]
    k_len = Lk if k_len is None else int(k_len)
    s2, _, _ = _scores(q, k, num_heads, k_len, sc, q_log2)
    m = s2.amax(-1, keepdim=True)
    p = torch.exp2(s2 - m)
    l = p.sum(-1, keepdim=True)
    vh = v.float().view(Lk, num_heads, 128).transpose(0, 1)
    o = _mm(bf(p), vh) / l                                  # [H, Lq, 128]
    lse = (m + torch.log2(l)).squeeze(-1)
    return _put(out, o.transpose(0, 1).reshape(Lq, -1).to(BF16)), lse


def attn_bwd(q, k, v, o, do, lse, num_heads, k_len=None, dq=None, dk=None, dv=None, scale=None,
             q_log2=False):
    sc = scale if scale is not None else 1 / math.sqrt(128)
    Lq, Lk = q.shape[0], k.shape[0]
    k_len = Lk if k_len is None else int(k_len)
    s2, qh, kh = _scores(q, k, num_heads, k_len, sc, q_log2)
    P = torch.exp2(s2 - lse[:, :, None])
    vh = v.float().view(Lk, num_heads, 128).transpose(0, 1)
    doh = do.float().view(Lq, num_heads, 128).transpose(0, 1)
    oh = o.float().view(Lq, num_heads, 128).transpose(0, 1)
    dvh = _mm(P.transpose(1, 2), doh)
    dp = _mm(doh, vh.transpose(1, 2))
    D = (doh * oh).sum(-1, keepdim=True)
    ds = P * (dp - D)
    f = LN2 if q_log2 else sc                # d S / d(q.k): ln 2 in log2 units, else the scale
    dqh = _mm(ds, kh) * f
    dkh = _mm(ds.transpose(1, 2), qh) * f
    res = []
    for t, buf, L in ((dqh, dq, Lq), (dkh, dk, Lk), (dvh, dv, Lk)):
        res.append(_put(buf, t.transpose(0, 1).reshape(L, -1).to(BF16)))
    return tuple(res)


OPS_FUNCS = ["gemm", "linear", "linear_t", "linear_dx", "linear_dw", "cast_bf16", "cast_bf16_t",
             "colsum", "gate_bwd", "ln_mod_fwd", "ln_mod_bwd", "rms_rope_fwd", "rms_rope_bwd",
             "attn_fwd", "attn_bwd"]


def install():
    """Point prfl_amd.ops' wrappers at the CPU stand-ins and register CPU kernels for the
    prfl:: custom ops (the product's own Python implementations for wan_block /
    wan_block_backward, torch restatements for linear_bf16 / flash_attention)."""
    import sys
    from prfl_amd import custom_ops, ops
    me = sys.modules[__name__]
    for n in OPS_FUNCS:
        setattr(ops, n, getattr(me, n))
    lib = torch.library
    lib.register_kernel("prfl::wan_block", "cpu", custom_ops.wan_block._init_fn)
    lib.register_kernel("prfl::wan_block_backward", "cpu", custom_ops.wan_block_backward._init_fn)

    def linear_cpu(x, w, b, gelu):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(BF16).float()
        y = _mm(x2, w.to(BF16).float().t()) + (b.to(BF16).float() if b is not None else 0)
        pre = bf(y)
        out = _gelu(pre) if gelu else pre
        return (out.to(BF16).view(*shp[:-1], w.shape[0]),
                pre.to(BF16) if gelu else x.new_empty((0,), dtype=BF16))

    def linear_bwd_cpu(dy, x, w, pre, need_dx, need_dw, need_db):
        N = w.shape[0]
        dy2 = dy.reshape(-1, N).to(BF16).float()
        if pre.numel():
            dy2 = bf(dy2 * _gelu_grad(pre.float()))
        x2 = x.reshape(-1, x.shape[-1]).to(BF16).float()
        dx = _mm(dy2, w.to(BF16).float()).to(BF16).view(x.shape).to(x.dtype) if need_dx \
            else x.new_empty((0,))
        dw = _mm(dy2.t(), x2) if need_dw else w.new_empty((0,), dtype=F32)
        db = dy2.double().sum(0).float() if need_db else w.new_empty((0,), dtype=F32)
        return dx, dw, db

    def fa_cpu(q, k, v, k_lens, scale):
        Bn, Lq, N, D = q.shape
        Lk = k.shape[1]
        os_, ls = [], []
        for b in range(Bn):
            kl = Lk if k_lens is None else int(k_lens[b])
            o, lse = attn_fwd(q[b].reshape(Lq, -1), k[b].reshape(Lk, -1), v[b].reshape(Lk, -1), N,
                              k_len=kl, scale=scale)
            os_.append(o.view(Lq, N, D))
            ls.append(lse)
        return torch.stack(os_), torch.stack(ls)

    def fa_bwd_cpu(do, q, k, v, o, lse, k_lens, scale):
        Bn, Lq, N, D = q.shape
        Lk = k.shape[1]
        r = [], [], []
        for b in range(Bn):
            kl = Lk if k_lens is None else int(k_lens[b])
            g = attn_bwd(q[b].reshape(Lq, -1), k[b].reshape(Lk, -1), v[b].reshape(Lk, -1),
                         o[b].reshape(Lq, -1), do[b].reshape(Lq, -1), lse[b], N, k_len=kl,
                         scale=scale)
            for lst, t, L in zip(r, g, (Lq, Lk, Lk)):
                lst.append(t.view(L, N, D))
        return (torch.stack(r[0]).to(q.dtype), torch.stack(r[1]).to(k.dtype),
                torch.stack(r[2]).to(v.dtype))

    lib.register_kernel("prfl::linear_bf16", "cpu", linear_cpu)
    lib.register_kernel("prfl::linear_bf16_backward", "cpu", linear_bwd_cpu)
    lib.register_kernel("prfl::flash_attention", "cpu", fa_cpu)
    lib.register_kernel("prfl::flash_attention_backward", "cpu", fa_bwd_cpu)
