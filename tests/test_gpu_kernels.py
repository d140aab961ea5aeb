"""Per-kernel parity on the MI355X: HIP C-ABI kernels vs the CPU oracle / fp32 references.

Tolerances (bf16 operands, fp32 accumulate): GEMM rel-L2 <= 2e-3 vs an fp32 GEMM of the same
bf16 operands (bf16 output rounding is 2^-9); attention / norms rel-L2 <= 5e-3 fwd, 2e-2 bwd
(SURVEY.md §8c tolerances).
"""
import math

import pytest
import torch

from oracle import wan_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def ops():
    from prfl_amd import ops as _ops
    return _ops


def bf(t):
    return t.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 384, 192), (105, 512, 256),
                                   (1000, 640, 144), (48, 15360, 5120), (2300, 3072, 512),
                                   (4096, 5120, 1024)])
def test_gemm_forward_epilogues(ops, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N)
    a = bf(torch.randn(M, K, generator=g)).to(DEV)
    w = bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV)
    bias = bf(torch.randn(N, generator=g) * 0.1).to(DEV)
    ref = a.float() @ w.float().t() + bias.float()
    out = ops.linear(a, w, bias)
    assert rel(out, ref) < 3e-3
    # GELU epilogue with pre-activation store
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    act = ops.linear(a, w, bias, ops.EPI_GELU, aux=pre)
    assert rel(pre, ref) < 3e-3
    assert rel(act, torch.nn.functional.gelu(pre.float(), approximate="tanh")) < 3e-3
    # gated fp32 residual: res + bf16(acc+b)*gate
    res = torch.randn(M, N, generator=g).to(DEV)
    gate = (torch.randn(N, generator=g) * 0.5).to(DEV)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    o = ops.linear(a, w, bias, ops.EPI_RESID, gate=gate, res=res, aux=y)
    assert rel(o, res + ref * gate) < 3e-3
    assert torch.equal(o, res + y.float() * gate)


def _tile_diff(a, b, tile=256):
    """[(tile_m, tile_n, quadrant, n_bad)] of the output elements where a != b."""
    bad = (a != b)
    if bad.dim() == 1:
        bad = bad[None]
    idx = bad.nonzero()
    out = {}
    for m, n in idx[:4096].tolist():
        key = (m // tile, n // tile, (m % tile) // (tile // 2), (n % tile) // (tile // 2))
        out[key] = out.get(key, 0) + 1
    return sorted(out.items())[:16]


# (M, N, K): the round-1 failing shape, then the 720p x 81f block projections (L = 73 920):
# fused QKV, o-proj / FFN-down with the gated residual, FFN-up with GELU
_CROSS_SHAPES = [(4096, 5120, 1024), (73920, 15360, 5120), (73920, 5120, 5120),
                 (73920, 13824, 5120), (73920, 5120, 13824)]


@pytest.mark.parametrize("M,N,K", _CROSS_SHAPES)
def test_gemm_tiles_bit_identical_forward(ops, M, N, K):
    """The four-wave 256x256 kernel (tile 256), the 8-wave staggered-ring kernel (tile 512) and
    the 128x128 kernel sum every element in the same k order (t, then the two 32-deep k-steps),
    so every epilogue must agree bit for bit.  A
    mismatch names the 256-tiles / quadrants that differ; comparing y = aux with the residual
    output separates an accumulator (ring / barrier) fault from an epilogue fault."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
    bias = (torch.randn(N, generator=g, device=DEV) * 0.1).to(torch.bfloat16)
    res = torch.randn(M, N, generator=g, device=DEV)
    gate = torch.randn(N, generator=g, device=DEV) * 0.5
    outs = {}
    for tile in (128, 256, 512):
        y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        o = ops.linear(a, w, bias, ops.EPI_RESID, gate=gate, res=res, aux=y, tile=tile)
        assert torch.equal(o, res + y.float() * gate), f"tile {tile}: residual epilogue"
        pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        act = ops.linear(a, w, bias, ops.EPI_GELU, aux=pre, tile=tile)
        outs[tile] = dict(bf16=ops.linear(a, w, bias, tile=tile), y=y, o=o, pre=pre, act=act,
                          f32=ops.linear(a, w, None, ops.EPI_F32, tile=tile))
        torch.cuda.synchronize()
    for key in outs[128]:
        for t in (256, 512):
            x128, xt = outs[128][key], outs[t][key]
            assert torch.equal(x128, xt), (t, key, _tile_diff(x128, xt))
    # residual output aliasing its input (the block's in-place x += o-proj * gate)
    xr = res.clone()
    ops.linear(a, w, bias, ops.EPI_RESID, out=xr, gate=gate, res=xr)
    assert torch.equal(xr, outs[256]["o"])
    # and one check against an independent fp32 GEMM of the same bf16 operands
    rows = torch.arange(0, M, max(1, M // 257), device=DEV)
    ref = a[rows].float() @ w.float().t()
    assert rel(outs[256]["f32"][rows], ref) < 1e-5


@pytest.mark.parametrize("M,N,K", [(5120, 13824, 73920), (5120, 5120, 32760), (13824, 5120, 4096)])
def test_gemm_tiles_bit_identical_weight_grad(ops, M, N, K):
    """dW = dY^T X (both operands MN-major, ds_read_b64_tr_b16 path) and dX = dY W: 128 vs 256
    (four-wave) vs 512 (8-wave) tile.  K = 32760 (480p tokens, K % 64 = 56) takes the bulk + tail split on the 256 path, so
    there only the fp32 reference check applies."""
    g = torch.Generator(device=DEV).manual_seed(M * 3 + N)
    dy = torch.randn(K, M, generator=g, device=DEV).to(torch.bfloat16)
    x = torch.randn(K, N, generator=g, device=DEV).to(torch.bfloat16)
    dws = [ops.linear_dw(dy, x, out=torch.empty(M, N, device=DEV)) for _ in range(1)]
    ref_rows = torch.arange(0, M, 97, device=DEV)
    ref = dy[:, ref_rows].float().t() @ x.float()
    assert rel(dws[0][ref_rows], ref) < 1e-5
    if K % 64 == 0:
        d128 = torch.empty(M, N, device=DEV)
        ops.gemm(dy, x, d128, M, N, K, False, False, ops.EPI_F32, tile=128)
        for t in (256, 512):
            dt_ = torch.empty(M, N, device=DEV)
            ops.gemm(dy, x, dt_, M, N, K, False, False, ops.EPI_F32, tile=t)
            assert torch.equal(d128, dt_), (t, _tile_diff(d128, dt_))
        assert torch.equal(d128, dws[0])
    # dX[K, N] = dY[K, M] @ W[M, N]: B MN-major
    w = (torch.randn(M, N, generator=g, device=DEV) / math.sqrt(M)).to(torch.bfloat16)
    outs = []
    for tile in (128, 256, 512):
        dx = torch.empty(K, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(dy, w, dx, K, N, M, True, False, ops.EPI_BF16, tile=tile)
        outs.append(dx)
    for o_ in outs[1:]:
        assert torch.equal(outs[0], o_), _tile_diff(outs[0], o_)


@pytest.mark.parametrize("M,N,K", [(256, 384, 128), (105, 256, 296), (1000, 136, 520),
                                   (3072, 2048, 3072), (3000, 2048, 3072)])
def test_gemm_backward_layouts(ops, M, N, K):
    """dX = dY W (N-major B) and dW = dY^T X (both MN-major): the ds_read_b64_tr_b16 paths."""
    g = torch.Generator().manual_seed(N)
    dy = bf(torch.randn(M, N, generator=g)).to(DEV)
    w = bf(torch.randn(N, K, generator=g)).to(DEV)
    x = bf(torch.randn(M, K, generator=g)).to(DEV)
    dx = ops.linear_dx(dy, w)
    assert rel(dx, dy.float() @ w.float()) < 3e-3
    dw = ops.linear_dw(dy, x)
    assert rel(dw, dy.float().t() @ x.float()) < 1e-4
    ops.linear_dw(dy, x, out=dw, accumulate=True)
    assert rel(dw, 2 * (dy.float().t() @ x.float())) < 1e-4
    pre = bf(torch.randn(M, K, generator=g)).to(DEV)
    dg = ops.linear_dx(dy, w, epilogue=ops.EPI_DGELU, aux=pre)
    p = pre.float().requires_grad_(True)
    torch.nn.functional.gelu(p, approximate="tanh").backward(bf(dy.float() @ w.float()).float())
    assert rel(dg, p.grad) < 5e-3


@pytest.mark.parametrize("M,N,K", [(4096, 1536, 512), (73920, 5120, 5120), (2000, 768, 1280),
                                   (300, 512, 384)])
def test_linear_transposed_weight_bit_identical(ops, M, N, K):
    """The forward projections on the transposed weight (ops.cast_bf16_t + ops.linear_t: W^T as
    an MN-major operand, block.BF16Weights) against linear() on the K-major weight: outputs and
    aux bit-identical for the bf16 / GELU / gated-residual (fp32 and bf16 residual) epilogues,
    incl. the 128-tile fallback (M, K off the 256 grid); the transposing cast vs torch's."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    w32 = torch.randn(N, K, generator=g, device=DEV) * 0.02
    x = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    bias = (torch.randn(N, generator=g, device=DEV) * 0.1).to(torch.bfloat16)
    wt = ops.cast_bf16_t(w32)
    assert torch.equal(wt, w32.t().to(torch.bfloat16))
    wk = ops.cast_bf16(w32)
    assert torch.equal(ops.linear_t(x, wt, bias), ops.linear(x, wk, bias))
    a0, a1 = (torch.empty(M, N, dtype=torch.bfloat16, device=DEV) for _ in range(2))
    assert torch.equal(ops.linear_t(x, wt, bias, ops.EPI_GELU, aux=a0),
                       ops.linear(x, wk, bias, ops.EPI_GELU, aux=a1))
    assert torch.equal(a0, a1)
    gate = torch.randn(N, generator=g, device=DEV)
    for res in (torch.randn(M, N, generator=g, device=DEV),
                torch.randn(M, N, generator=g, device=DEV).to(torch.bfloat16)):
        y0 = ops.linear_t(x, wt, bias, ops.EPI_RESID, gate=gate, res=res, aux=a0)
        y1 = ops.linear(x, wk, bias, ops.EPI_RESID, gate=gate, res=res, aux=a1)
        assert torch.equal(y0, y1) and torch.equal(a0, a1)


def test_gemm_identity_asymmetric(ops):
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    n = 128
    a = torch.eye(n, dtype=torch.bfloat16, device=DEV)
    b = bf(torch.arange(n * n, dtype=torch.float32).view(n, n) % 97).to(DEV)
    out = ops.linear(a, b)
    assert torch.equal(out.float(), b.float().t())


@pytest.mark.parametrize("Lq,Lk,H,klen", [(128, 128, 1, 128), (200, 333, 2, 333), (105, 512, 2, 20),
                                          (1000, 1000, 3, 937)])
def test_attention_fwd_bwd(ops, Lq, Lk, H, klen):
    g = torch.Generator().manual_seed(Lq + Lk)
    C = H * 128
    q = bf(torch.randn(Lq, C, generator=g) * 1.5)
    k = bf(torch.randn(Lk, C, generator=g) * 1.5)
    v = bf(torch.randn(Lk, C, generator=g))
    o, lse = ops.attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), H, k_len=klen)
    qr = q.float().view(1, Lq, H, 128).requires_grad_(True)
    kr = k.float().view(1, Lk, H, 128).requires_grad_(True)
    vr = v.float().view(1, Lk, H, 128).requires_grad_(True)
    ref = O.attention(qr, kr, vr, k_len=klen if klen < Lk else None)
    assert rel(o, ref.reshape(Lq, C)) < 5e-3
    do = bf(torch.randn(Lq, C, generator=g))
    ref.backward(do.float().view(1, Lq, H, 128))
    dq, dk, dv = ops.attn_bwd(q.to(DEV), k.to(DEV), v.to(DEV), o, do.to(DEV), lse, H, k_len=klen)
    assert rel(dq, qr.grad.reshape(Lq, C)) < 2e-2
    assert rel(dk, kr.grad.reshape(Lk, C)) < 2e-2
    assert rel(dv, vr.grad.reshape(Lk, C)) < 2e-2
    if klen < Lk:
        assert dk[klen:].abs().max().item() == 0 and dv[klen:].abs().max().item() == 0


SL2 = 1.4426950408889634 / math.sqrt(128)     # softmax_scale * log2(e), head_dim 128


def _l2q(q):
    """The *_l2q attention operand of a bf16 q: q2 = bf16(q * scale * log2 e) (what the fused
    block's rms_rope_fwd writes), and the fp32 q that q2 represents exactly (q2 / (scale log2 e)),
    the input of the reference computation."""
    q2 = (q.float() * SL2).to(torch.bfloat16)
    return q2, q2.float() / SL2


@pytest.mark.parametrize("Lq,Lk,H,klen", [(200, 333, 2, 333), (105, 512, 2, 20),
                                          (300, 512, 2, 512), (700, 1024, 1, 960),
                                          (4200, 4200, 2, 4133), (4111, 5000, 1, 4500)])
def test_attention_log2_q_vs_oracle(ops, Lq, Lk, H, klen):
    """The q-in-log2-units entries (prfl_attn_fwd_l2q_ws / prfl_attn_bwd_l2q_ws: S accumulators
    starting at the running max, one v_exp per score; the fused block's path) on the short-KV
    (cross-attention) and long-KV (self-attention) instantiations vs the CPU oracle on the
    q they represent; dq is the gradient w.r.t. the pre-scaled q (x scale log2 e = the oracle's)."""
    g = torch.Generator().manual_seed(Lq * 7 + Lk)
    C = H * 128
    q2, qe = _l2q(bf(torch.randn(Lq, C, generator=g) * 1.5))
    k = bf(torch.randn(Lk, C, generator=g) * 1.5)
    v = bf(torch.randn(Lk, C, generator=g))
    o, lse = ops.attn_fwd(q2.to(DEV), k.to(DEV), v.to(DEV), H, k_len=klen, q_log2=True)
    qr = qe.view(1, Lq, H, 128).clone().requires_grad_(True)
    kr = k.float().view(1, Lk, H, 128).requires_grad_(True)
    vr = v.float().view(1, Lk, H, 128).requires_grad_(True)
    ref = O.attention(qr, kr, vr, k_len=klen if klen < Lk else None)
    assert rel(o, ref.reshape(Lq, C)) < 5e-3
    lref = _lse2_ref(qe, k, H, klen, 1 / math.sqrt(128))
    assert (lse.cpu() - lref).abs().max().item() < 1e-3
    do = bf(torch.randn(Lq, C, generator=g))
    ref.backward(do.float().view(1, Lq, H, 128))
    dq, dk, dv = ops.attn_bwd(q2.to(DEV), k.to(DEV), v.to(DEV), o, do.to(DEV), lse, H, k_len=klen,
                              q_log2=True)
    assert rel(dq.float() * SL2, qr.grad.reshape(Lq, C)) < 2e-2
    assert rel(dk, kr.grad.reshape(Lk, C)) < 2e-2
    assert rel(dv, vr.grad.reshape(Lk, C)) < 2e-2
    if klen < Lk:
        assert dk[klen:].abs().max().item() == 0 and dv[klen:].abs().max().item() == 0


@pytest.mark.parametrize("l2", [True, False])
def test_attention_log2_q_extreme_rows(ops, l2):
    """Rows whose scores all sit near -250 log2 units (exp2 of them underflows fp32) and rows with
    scores in the hundreds plus one spike: the log2-q forward starts each row from its first
    tile's max (the accumulators hold S - m), so neither underflows to an empty row nor
    overflows; vs fp64 on the same bf16 operands."""
    L, H = 4200, 1
    C = H * 128
    g = torch.Generator().manual_seed(3)
    base = torch.randn(C, generator=g)
    k = bf(base + 0.1 * torch.randn(L, C, generator=g))       # every key ~ base
    v = bf(torch.randn(L, C, generator=g))
    q = torch.randn(L, C, generator=g) * 0.05
    bb = k.float().mean(0)
    q[:64] += -bb / bb.norm() ** 2 * 250.0 / SL2               # scores ~ -250 +- a few
    n = k[4000].float() - bb
    q[64:128] += n / n.norm() ** 2 * 300.0 / SL2               # key 4000 stands out by ~300
    q2 = (q * SL2).to(torch.bfloat16)
    if l2:
        o, lse = ops.attn_fwd(q2.to(DEV), k.to(DEV), v.to(DEV), H, q_log2=True)
        s = q2[:128].double() @ k.double().t()                 # scores in log2 units
    else:                                                      # the plain entry, same extremes
        q1 = q.to(torch.bfloat16)
        o, lse = ops.attn_fwd(q1.to(DEV), k.to(DEV), v.to(DEV), H)
        s = q1[:128].double() @ k.double().t() * SL2
    assert s[:64].max() < -200
    exact = torch.softmax(s * math.log(2.0), -1) @ v.double()
    assert torch.isfinite(o.float()).all() and torch.isfinite(lse).all()
    assert rel(o[:128].cpu(), exact) < 5e-3
    lref = torch.logsumexp(s * math.log(2.0), -1) / math.log(2.0)
    assert (lse[0, :128].cpu().double() - lref).abs().max().item() < 1e-2


def _lse2_ref(q, k, H, klen, scale):
    """log2-domain row LSE of softmax(q k^T * scale) over keys < klen; q/k bf16 [L, H*128]."""
    Lq, Lk = q.shape[0], k.shape[0]
    qh = q.float().view(Lq, H, 128).transpose(0, 1)
    kh = k.float().view(Lk, H, 128).transpose(0, 1)
    s = torch.bmm(qh, kh.transpose(1, 2))[:, :, :klen] * scale
    return torch.logsumexp(s, -1) / math.log(2.0)


@pytest.mark.parametrize("Lq,Lk,H,klen", [(4200, 4200, 2, 4133), (4133, 4133, 1, 4133),
                                          (1000, 4100, 2, 4097), (4111, 5000, 1, 4500)])
def test_attention_long_kv_vs_oracle(ops, Lq, Lk, H, klen):
    """The production self-attention instantiation (Lk >= 4096 -> attn_fwd_kernel<false, ATTN_FWD_SCHED, 3, QS>,
    the L x L forward of every block) and both backward kernels vs the CPU oracle: L not a
    multiple of 96 or 256 (the clamped last K/V tile, partial query tiles), k_len < Lk."""
    g = torch.Generator().manual_seed(Lq * 3 + Lk)
    C = H * 128
    q = bf(torch.randn(Lq, C, generator=g) * 1.5)
    k = bf(torch.randn(Lk, C, generator=g) * 1.5)
    v = bf(torch.randn(Lk, C, generator=g))
    o, lse = ops.attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), H, k_len=klen)
    qr = q.float().view(1, Lq, H, 128).requires_grad_(True)
    kr = k.float().view(1, Lk, H, 128).requires_grad_(True)
    vr = v.float().view(1, Lk, H, 128).requires_grad_(True)
    ref = O.attention(qr, kr, vr, k_len=klen if klen < Lk else None)
    assert rel(o, ref.reshape(Lq, C)) < 5e-3
    lref = _lse2_ref(q, k, H, klen, 1 / math.sqrt(128))
    assert (lse.cpu() - lref).abs().max().item() < 1e-3
    do = bf(torch.randn(Lq, C, generator=g))
    ref.backward(do.float().view(1, Lq, H, 128))
    dq, dk, dv = ops.attn_bwd(q.to(DEV), k.to(DEV), v.to(DEV), o, do.to(DEV), lse, H, k_len=klen)
    assert rel(dq, qr.grad.reshape(Lq, C)) < 2e-2
    assert rel(dk, kr.grad.reshape(Lk, C)) < 2e-2
    assert rel(dv, vr.grad.reshape(Lk, C)) < 2e-2
    if klen < Lk:
        assert dk[klen:].abs().max().item() == 0 and dv[klen:].abs().max().item() == 0


def _attention_ref_gpu(q, k, v, do, H, scale, chunk=4096):
    """fp32 FA2-numerics reference (oracle/_FlashAttention restated in query chunks on the GPU
    for full-size L): P rounded to bf16 for P.V, the normaliser sums fp32 P, bf16 output,
    D = rowsum(dO * bf16 O)."""
    L, C = q.shape
    Lk = k.shape[0]
    o = torch.empty(L, C, dtype=torch.bfloat16, device=DEV)
    lse2 = torch.empty(H, L, device=DEV)
    dq = torch.empty(L, C, device=DEV)
    dk = torch.zeros(Lk, C, device=DEV)
    dv = torch.zeros(Lk, C, device=DEV)
    for h in range(H):
        sl = slice(h * 128, (h + 1) * 128)
        kh, vh = k[:, sl].float(), v[:, sl].float()
        for c0 in range(0, L, chunk):
            cs = slice(c0, min(L, c0 + chunk))
            qh, doh = q[cs, sl].float(), do[cs, sl].float()
            s = (qh @ kh.t()) * scale
            m = s.amax(-1, keepdim=True)
            p = torch.exp(s - m)
            l = p.sum(-1, keepdim=True)
            oh = ((p.to(torch.bfloat16).float() @ vh) / l).to(torch.bfloat16)
            o[cs, sl] = oh
            lse2[h, cs] = ((m + torch.log(l)) / math.log(2.0)).squeeze(-1)
            P = p / l
            del p, s
            dv[:, sl] += P.t() @ doh
            dp = doh @ vh.t()
            delta = (doh * oh.float()).sum(-1, keepdim=True)
            ds = P * (dp - delta)
            del P, dp
            dq[cs, sl] = (ds @ kh) * scale
            dk[:, sl] += (ds.t() @ qh) * scale
            del ds
    return o, lse2, dq, dk, dv


@pytest.mark.parametrize("L,H,l2", [(32760, 2, False), (73920, 1, False), (73920, 1, True)])
def test_attention_full_size_vs_reference(ops, L, H, l2):
    """Self-attention at the real token counts (480p x 81f: L = 32 760, L % 96 = 24, L % 256 =
    248; 720p x 81f: L = 73 920) against an fp32 GPU restatement of the FA2 numerics; the
    forward rows are also checked against an fp64 CPU computation over all keys."""
    g = torch.Generator(device=DEV).manual_seed(L)
    C = H * 128
    q = torch.randn(L, C, generator=g, device=DEV).to(torch.bfloat16)
    k = torch.randn(L, C, generator=g, device=DEV).to(torch.bfloat16)
    v = torch.randn(L, C, generator=g, device=DEV).to(torch.bfloat16)
    do = torch.randn(L, C, generator=g, device=DEV).to(torch.bfloat16)
    scale = 1 / math.sqrt(128)
    if l2:       # the fused block's path: q in log2 units; references on the q it represents
        q2, q = _l2q(q)
        o, lse = ops.attn_fwd(q2, k, v, H, q_log2=True)
        dq, dk, dv = ops.attn_bwd(q2, k, v, o, do, lse, H, q_log2=True)
        dq = dq.float() * SL2
    else:
        o, lse = ops.attn_fwd(q, k, v, H)
        dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, H)
    ro, rlse, rdq, rdk, rdv = _attention_ref_gpu(q, k, v, do, H, scale)
    assert rel(o, ro) < 5e-3
    assert (lse - rlse).abs().max().item() < 1e-3
    assert rel(dq, rdq) < 2e-2 and rel(dk, rdk) < 2e-2 and rel(dv, rdv) < 2e-2
    rows = torch.randperm(L, generator=torch.Generator().manual_seed(1))[:64].sort().values
    qc = q[rows.to(DEV)].double().cpu().view(64, H, 128).transpose(0, 1)
    kc = k.double().cpu().view(L, H, 128).transpose(0, 1)
    vc = v.double().cpu().view(L, H, 128).transpose(0, 1)
    p = torch.softmax(torch.bmm(qc, kc.transpose(1, 2)) * scale, -1)
    exact = torch.bmm(p, vc).transpose(0, 1).reshape(64, C)
    assert rel(o[rows.to(DEV)], exact) < 5e-3


def test_attention_split_tail(ops):
    """Split tails of the long-KV attention (prfl_attn_fwd_ws / prfl_attn_bwd_ws): L = 8100
    (ragged last query tile), k_len = 8000 < Lk, 9 heads -> 288 units on 256 CUs, so the last 32
    units (head 8) run as 8 shares each + merge, forward and backward.  Units outside the tail are bit-identical to the unsplit
    launch; the tail rows match it to rounding and match an fp64 computation over all keys."""
    from prfl_amd import _lib
    L, H, klen = 8100, 9, 8000
    C = H * 128
    if (torch.cuda.get_device_properties(0).multi_processor_count != 256
            or _lib.load().prfl_attn_fwd_ws_bytes(1, L, L, H, klen) == 0):
        pytest.skip("the tail layout below assumes MI355X's 256 CUs")
    g = torch.Generator(device=DEV).manual_seed(11)
    q, k, v = (torch.randn(L, C, generator=g, device=DEV).to(torch.bfloat16) for _ in range(3))
    o, lse = ops.attn_fwd(q, k, v, H, k_len=klen)             # split tail
    o1 = torch.empty_like(o)
    lse1 = torch.empty_like(lse)
    _lib.call("prfl_attn_fwd", _lib.ptr(q), _lib.I64(C), _lib.I64(0), _lib.ptr(k), _lib.I64(C),
              _lib.I64(0), _lib.ptr(v), _lib.I64(C), _lib.I64(0), _lib.ptr(o1), _lib.I64(C),
              _lib.I64(0), _lib.ptr(lse1), _lib.I64(1), _lib.I64(L), _lib.I64(L), _lib.I64(H),
              _lib.I64(klen), _lib.F32(128 ** -0.5), _lib.stream_ptr())   # no workspace: unsplit
    tail = slice(8 * 128, 9 * 128)
    assert torch.equal(o[:, :8 * 128], o1[:, :8 * 128]) and torch.equal(lse[:8], lse1[:8])
    assert not torch.equal(o[:, tail], o1[:, tail])          # the tail did take the split path
    # the key shares round P to bf16 against their own row max: on random data O is a
    # cancelling sum whose P-rounding noise is ~2^-9 relative in either form (so ~2.8e-3 between
    # the two); both are held to the same bar against the exact result below
    assert rel(o[:, tail], o1[:, tail]) < 5e-3
    assert (lse[8] - lse1[8]).abs().max().item() < 1e-4
    rows = torch.cat([torch.arange(0, 40), torch.arange(L - 60, L)])
    qc = q[rows.to(DEV), tail].double().cpu()
    kc, vc = k[:klen, tail].double().cpu(), v[:klen, tail].double().cpu()
    s = qc @ kc.t() / math.sqrt(128)
    exact = torch.softmax(s, -1) @ vc
    assert rel(o[rows.to(DEV), tail], exact) < 5e-3
    assert rel(o1[rows.to(DEV), tail], exact) < 5e-3
    lse_exact = torch.logsumexp(s, -1) / math.log(2.0)
    assert (lse[8, rows.to(DEV)].double().cpu() - lse_exact).abs().max().item() < 1e-3
    # backward (prfl_attn_bwd_ws): dK/dV units are 256-key tiles (32 per head, head 8 = the
    # tail, split over query tiles), dQ units 256-query tiles (head 8 split over key tiles);
    # same forward output for both so only the backward's tail handling differs
    if _lib.load().prfl_attn_bwd_ws_bytes(1, L, L, H, klen) == 0:
        return
    do = torch.randn(L, C, generator=g, device=DEV).to(torch.bfloat16)
    dq, dk, dv = ops.attn_bwd(q, k, v, o1, do, lse1, H, k_len=klen)     # split tails
    dq1, dk1, dv1 = (torch.empty_like(q) for _ in range(3))
    delta = torch.empty(H, L, device=DEV)
    _lib.call("prfl_attn_bwd", *[_lib.ptr(t) if torch.is_tensor(t) else _lib.I64(t) for t in (
        q, C, 0, k, C, 0, v, C, 0, o1, C, 0, do, C, 0, lse1, delta, dq1, C, 0, dk1, C, 0, dv1, C,
        0, 1, L, L, H, klen)], _lib.F32(128 ** -0.5), _lib.stream_ptr())       # unsplit
    for x, x1 in ((dq, dq1), (dk, dk1), (dv, dv1)):
        assert torch.equal(x[:, :8 * 128], x1[:, :8 * 128])
        assert not torch.equal(x[:, tail], x1[:, tail])
        assert rel(x[:, tail], x1[:, tail]) < 2e-3        # fp32 partial sums, one bf16 rounding
    assert torch.equal(dk[klen:], torch.zeros_like(dk[klen:]))
    assert torch.equal(dv[klen:], torch.zeros_like(dv[klen:]))
    _, _, rdq, rdk, rdv = _attention_ref_gpu(q[:, tail], k[:klen, tail], v[:klen, tail],
                                             do[:, tail], 1, 128 ** -0.5)
    assert rel(dq[:, tail], rdq) < 2e-2
    assert rel(dk[:klen, tail], rdk) < 2e-2 and rel(dv[:klen, tail], rdv) < 2e-2


def _vt_image(v, H):
    """torch restatement of prfl_attn_v_to_vt for one sample: v [Lk, H*128] -> [H][Lkp/8][128][8],
    chunk 2j + h holding keys 16j + 4h + (0, 1, 2, 3, 8, 9, 10, 11), zero past Lk (Lkp = Lk
    rounded up to 96)"""
    Lk = v.shape[0]
    lkp = (Lk + 95) // 96 * 96
    vp = torch.zeros(lkp, H, 128, dtype=v.dtype, device=v.device)
    vp[:Lk] = v.view(Lk, H, 128)
    perm = torch.tensor([0, 1, 2, 3, 8, 9, 10, 11, 4, 5, 6, 7, 12, 13, 14, 15], device=v.device)
    x = vp.view(lkp // 16, 16, H, 128)[:, perm]                  # [j][h*8 + slot][H][d]
    return x.view(lkp // 8, 8, H, 128).permute(2, 0, 3, 1).contiguous()


@pytest.mark.parametrize("Lq,Lk,H,klen,B", [(4200, 4200, 2, 4133, 1), (4111, 5000, 1, 4500, 1),
                                            (1000, 4100, 3, 4097, 2), (8100, 8100, 9, 8000, 1)])
def test_attention_vt_bit_identical(ops, Lq, Lk, H, klen, B):
    """The VT forward (prfl_attn_v_to_vt + prfl_attn_fwd_l2q_vt_ws: V^T fragments as one
    ds_read_b128 from a key-chunked transposed image) against the row-major l2q forward: the
    same operand values in the same k-slot order, so O and the LSE are bit-identical, including
    ragged Lk (not a multiple of 96), k_len < Lk, two samples (sample strides) and the split-KV
    tail (L = 8100, 9 heads); the transpose itself vs its torch restatement."""
    from prfl_amd import _lib
    C = H * 128
    g = torch.Generator(device=DEV).manual_seed(Lq + Lk + B)
    q2 = (torch.randn(B, Lq, C, generator=g, device=DEV) * 1.5 * SL2).to(torch.bfloat16)
    k = (torch.randn(B, Lk, 3 * C, generator=g, device=DEV) * 1.5).to(torch.bfloat16)[:, :, :C]
    v = torch.randn(B, Lk, 2 * C, generator=g, device=DEV).to(torch.bfloat16)[:, :, C:]  # strided
    lkp = (Lk + 95) // 96 * 96
    nb = _lib.load().prfl_attn_vt_bytes(B, Lk, H)
    assert nb == B * H * lkp * 128 * 2
    vt = torch.full((nb // 2,), float("nan"), dtype=torch.bfloat16, device=DEV)
    _lib.call("prfl_attn_v_to_vt", _lib.ptr(v), _lib.I64(2 * C), _lib.I64(Lk * 2 * C), _lib.ptr(vt),
              _lib.I64(B), _lib.I64(Lk), _lib.I64(H), _lib.stream_ptr())
    for b in range(B):
        assert torch.equal(vt.view(B, H, lkp // 8, 128, 8)[b], _vt_image(v[b], H))
    wsb = _lib.load().prfl_attn_fwd_ws_bytes(B, Lq, Lk, H, klen)
    ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=DEV)
    outs = []
    for use_vt in (False, True):
        o = torch.empty(B, Lq, C, dtype=torch.bfloat16, device=DEV)
        lse = torch.empty(B, H, Lq, device=DEV)
        qk = (_lib.ptr(q2), _lib.I64(C), _lib.I64(Lq * C), _lib.ptr(k), _lib.I64(3 * C), _lib.I64(Lk * 3 * C))
        tail = (_lib.ptr(o), _lib.I64(C), _lib.I64(Lq * C), _lib.ptr(lse), _lib.I64(B), _lib.I64(Lq),
                _lib.I64(Lk), _lib.I64(H), _lib.I64(klen), _lib.ptr(ws), _lib.I64(wsb), _lib.stream_ptr())
        if use_vt:
            _lib.call("prfl_attn_fwd_l2q_vt_ws", *qk, _lib.ptr(vt), *tail)
        else:
            _lib.call("prfl_attn_fwd_l2q_ws", *qk, _lib.ptr(v), _lib.I64(2 * C), _lib.I64(Lk * 2 * C), *tail)
        outs.append((o, lse))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    # the ops-level path the fused block takes (ATTN_VT) against the row-major entry
    o3, lse3 = ops.attn_fwd(q2[0], k[0], v[0], H, k_len=klen, q_log2=True)
    assert torch.equal(o3, outs[0][0][0]) and torch.equal(lse3, outs[0][1][0])
    # short KV has no VT instantiation: the entry refuses it
    with pytest.raises(RuntimeError):
        _lib.call("prfl_attn_fwd_l2q_vt_ws", _lib.ptr(q2), _lib.I64(C), _lib.I64(0), _lib.ptr(k),
                  _lib.I64(3 * C), _lib.I64(0), _lib.ptr(vt), _lib.ptr(outs[0][0]), _lib.I64(C),
                  _lib.I64(0), _lib.ptr(outs[0][1]), _lib.I64(1), _lib.I64(Lq), _lib.I64(512),
                  _lib.I64(H), _lib.I64(512), _lib.ptr(None), _lib.I64(0), _lib.stream_ptr())


@pytest.mark.parametrize("Lq,Lk,H,klen", [(4200, 4200, 2, 4133), (4111, 5000, 1, 4500),
                                          (8100, 8100, 9, 8000)])
def test_attention_kt_backward_bit_identical(ops, Lq, Lk, H, klen):
    """The KT backward (prfl_attn_bwd_l2q_kt_ws: the dQ kernel's K^T fragments from K's VT image,
    one ds_read_b128 each) against the row-major l2q backward: dq, dk, dv bit-identical, incl.
    ragged Lk, k_len < Lk and the split tails (L = 8100, 9 heads)."""
    from prfl_amd import ops as O_
    g = torch.Generator(device=DEV).manual_seed(Lq * 5 + Lk)
    C = H * 128
    q2 = (torch.randn(Lq, C, generator=g, device=DEV) * 1.5 * SL2).to(torch.bfloat16)
    k = (torch.randn(Lk, C, generator=g, device=DEV) * 1.5).to(torch.bfloat16)
    v = torch.randn(Lk, C, generator=g, device=DEV).to(torch.bfloat16)
    do = torch.randn(Lq, C, generator=g, device=DEV).to(torch.bfloat16)
    o, lse = ops.attn_fwd(q2, k, v, H, k_len=klen, q_log2=True)
    got = []
    saved = O_.ATTN_KT
    try:
        for kt in (False, True):
            O_.ATTN_KT = kt
            got.append(ops.attn_bwd(q2, k, v, o, do, lse, H, k_len=klen, q_log2=True))
    finally:
        O_.ATTN_KT = saved
    for a, b in zip(*got):
        assert torch.equal(a, b)


def test_attention_rescale_spike(ops):
    """Force the online-softmax rescale: one key gets a huge score in a late tile (rule 26)."""
    L, C = 256, 128
    g = torch.Generator().manual_seed(3)
    q = torch.randn(L, C, generator=g) * 0.1
    k = torch.randn(L, C, generator=g) * 0.1
    k[200] = q[5] * 60.0
    q, k = bf(q), bf(k)
    v = bf(torch.randn(L, C, generator=g))
    o, _ = ops.attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), 1)
    ref = O.attention(q.float().view(1, L, 1, C), k.float().view(1, L, 1, C), v.float().view(1, L, 1, C))
    assert rel(o, ref.reshape(L, C)) < 5e-3


@pytest.mark.parametrize("C,x_bf16,affine", [(256, False, False), (256, True, False),
                                             (5120, False, False), (5120, False, True)])
def test_ln_mod(ops, C, x_bf16, affine):
    L = 77
    g = torch.Generator().manual_seed(C)
    x = torch.randn(L, C, generator=g) * 2 + 0.3
    if x_bf16:
        x = bf(x)
    sc = torch.randn(C, generator=g) * 0.1
    sh = torch.randn(C, generator=g) * 0.1
    w = 1 + torch.randn(C, generator=g) * 0.1
    bb = torch.randn(C, generator=g) * 0.1
    xr = x.float().requires_grad_(True)
    scr, shr = sc.clone().requires_grad_(True), sh.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), bb.clone().requires_grad_(True)
    if affine:
        ref = O.layer_norm(xr, 1e-6, wr, br)
        out, mean, rstd = ops.ln_mod_fwd(x.to(DEV), w=w.to(DEV), b=bb.to(DEV))
    else:
        ref = O.layer_norm(xr, 1e-6, in_bf16=x_bf16) * (1 + scr) + shr
        out, mean, rstd = ops.ln_mod_fwd(x.to(DEV), scale=sc.to(DEV), shift=sh.to(DEV))
    assert rel(out, O.bf(ref)) < 3e-3
    dy = bf(torch.randn(L, C, generator=g))
    ref.backward(dy.float())
    dx = torch.zeros(L, C, device=DEV)
    if affine:
        d0, d1 = ops.ln_mod_bwd(dy.to(DEV), x.to(DEV), mean, rstd, dx, w=w.to(DEV))
        assert rel(d0, wr.grad) < 5e-3 and rel(d1, br.grad) < 5e-3
    else:
        d0, d1 = ops.ln_mod_bwd(dy.to(DEV), x.to(DEV), mean, rstd, dx, scale=sc.to(DEV))
        assert rel(d0, scr.grad) < 5e-3 and rel(d1, shr.grad) < 5e-3
    assert rel(dx, xr.grad) < 5e-3


@pytest.mark.parametrize("rope", [True, False])
@pytest.mark.parametrize("osc", [1.0, 1.4426950408889634 / math.sqrt(128)])
def test_rms_rope(ops, rope, osc):
    """RMSNorm (+ RoPE) vs the oracle; osc = the out_scale that writes q in log2 units for the
    *_l2q attention entries (the backward scales the incoming gradient by it)."""
    C, H = 256, 2
    grid = (3, 5, 7)
    L = 112   # 105 rotated + 7 pass-through rows
    g = torch.Generator().manual_seed(11)
    x = bf(torch.randn(L, C, generator=g) * 3)
    w = 1 + torch.randn(C, generator=g) * 0.1
    freqs = O.rope_freqs(128)
    tab = ops.rope_table(freqs, DEV) if rope else None
    out, rstd = ops.rms_rope_fwd(x.to(DEV), w.to(DEV), 1e-6, tab, grid if rope else (0, 0, 0),
                                 out_scale=osc)
    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    n = O.rms_norm(xr, wr)
    if rope:
        n = O.rope_apply(n.view(1, L, H, 128), torch.tensor([grid]), freqs).view(L, C)
    n = n * osc
    assert rel(out, O.bf(n)) < 3e-3
    do = bf(torch.randn(L, C, generator=g))
    n.backward(do.float())
    dx, dw = ops.rms_rope_bwd(do.to(DEV), x.to(DEV), rstd, w.to(DEV), tab,
                              grid if rope else (0, 0, 0), out_scale=osc)
    assert rel(dx, xr.grad) < 1e-2
    assert rel(dw, wr.grad) < 5e-3


def test_adamw_matches_torch(ops):
    g = torch.Generator().manual_seed(5)
    p = torch.randn(10007, generator=g)
    grads = [torch.randn(10007, generator=g) for _ in range(3)]
    ref = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=5e-6, betas=(0.9, 0.999), weight_decay=0.01, eps=1e-8,
                            foreach=False)
    pd, m, v = p.to(DEV), torch.zeros(10007, device=DEV), torch.zeros(10007, device=DEV)
    for step, gr in enumerate(grads, 1):
        ref.grad = gr.clone()
        opt.step()
        ops.adamw_(pd, gr.to(DEV), m, v, 5e-6, 0.9, 0.999, 1e-8, 0.01, step)
    assert (pd.cpu() - ref.detach()).abs().max().item() < 1e-6


def test_adamw_host_state_streaming_is_bit_exact(ops):
    """AdamW with moments in pinned host memory (streamed through the HBM ring) == on-device."""
    from prfl_amd.optim import AdamW
    g = torch.Generator().manual_seed(6)
    shapes = [(3000,), (257, 33), (5,), (1024, 64), (7, 11)]      # more tensors than ring slots
    base = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) for s in shapes] for _ in range(3)]
    a = [b.clone().to(DEV).requires_grad_(True) for b in base]
    b = [x.clone().to(DEV).requires_grad_(True) for x in base]
    oa, ob = AdamW(a), AdamW(b, state_on_host=True)
    for gs in grads:
        for pa, pb, gr in zip(a, b, gs):
            pa.grad, pb.grad = gr.to(DEV), gr.to(DEV)
        oa.step()
        ob.step()
    torch.cuda.synchronize()
    for pa, pb in zip(a, b):
        assert torch.equal(pa, pb)
    for pa, pb in zip(a, b):
        assert torch.equal(oa.state[pa][0].flatten().cpu(), ob.state[pb][0])
        assert torch.equal(oa.state[pa][1].flatten().cpu(), ob.state[pb][1])


def test_adamw_overlapped_update_is_bit_exact(ops):
    """overlap=True (update on a side stream, readers ordered by per-parameter events installed
    as forward pre-hooks) == the synchronous update, with host-streamed and device moments."""
    from prfl_amd.optim import AdamW

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = torch.nn.Linear(16, 64)
            self.blocks = torch.nn.ModuleList([torch.nn.Linear(64, 64) for _ in range(5)])
            self.head = torch.nn.Linear(64, 3)

        def forward(self, x):
            x = self.emb(x)
            for b in self.blocks:
                x = torch.tanh(b(x))
            return self.head(x)

    torch.manual_seed(0)
    ref = Toy().to(DEV)
    x = torch.randn(32, 16, device=DEV)
    for host in (False, True, 0.4):      # 0.4: the streamed tail (last blocks + head), rest in HBM
        a, b = Toy().to(DEV), Toy().to(DEV)
        a.load_state_dict(ref.state_dict())
        b.load_state_dict(ref.state_dict())
        oa = AdamW(list(a.parameters()), lr=1e-2, state_on_host=host)
        ob = AdamW(list(b.parameters()), lr=1e-2, state_on_host=host, overlap=True, ring_slots=2)
        ob.attach(b)
        assert ob.params[0] is b.emb.weight and ob.params[-1] is b.head.bias
        if host == 0.4:
            hp = ob._host_params()
            assert b.head.bias in hp and b.emb.weight not in hp and 0 < len(hp) < len(ob.params)
        for it in range(4):
            la, lb = a(x).square().mean(), b(x).square().mean()   # b's forward waits per block
            assert torch.equal(la, lb), (host, it)
            la.backward()
            lb.backward()
            oa.step()
            ob.step()
            assert len(ob._ready) == len(ob.params)
            oa.zero_grad()
            ob.zero_grad()
        ob.synchronize()
        for pa, pb in zip(a.parameters(), b.parameters()):
            assert torch.equal(pa, pb), host


def test_sumsq_scale(ops):
    x = torch.randn(100003, device=DEV)
    out = torch.zeros(1, device=DEV)
    ops.sumsq_(x, out)
    assert abs(out.item() / (x.double() ** 2).sum().item() - 1) < 1e-4
    f = torch.tensor([0.5], device=DEV)
    y = x.clone()
    ops.scale_(y, f)
    assert torch.equal(y, x * 0.5)


@pytest.mark.parametrize("P,N", [(1155, 5120), (7, 64), (33, 13824), (1, 4), (64, 6)])
def test_colsum_reduce(ops, P, N):
    """[P][N] partial column sums -> [N] (bias / LN-affine gradients), fresh and accumulating."""
    g = torch.Generator(device=DEV).manual_seed(P * N)
    part = torch.randn(P, N, generator=g, device=DEV)
    ref = part.double().sum(0)
    out = ops.colsum_reduce(part)
    assert (out.double() - ref).abs().max().item() <= 1e-5 * max(1.0, ref.abs().max().item())
    base = torch.randn(N, generator=g, device=DEV)
    out2 = base.clone()
    ops.colsum_reduce(part, out=out2, accumulate=True)
    assert (out2.double() - (ref + base.double())).abs().max().item() <= 1e-4


def test_adamw_zero_grad_in_step_is_bit_exact(ops):
    """step(zero_grad=True) (the update kernel zeroes each gradient once read, buffers kept) ==
    step() + zero_grad(): identical parameters over several steps with the next gradient
    accumulated by autograd into the zeroed buffer behind attach()'s forward pre-hook, overlapped,
    with device and host-streamed moments; the gradient tensors are the same storage throughout."""
    from prfl_amd.optim import AdamW
    g = torch.Generator().manual_seed(8)
    shapes = [(3000,), (257, 33), (5,), (1024, 64)]
    base = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) for s in shapes] for _ in range(4)]

    class Holder(torch.nn.Module):
        def __init__(self, ts):
            super().__init__()
            self.ps = torch.nn.ParameterList([torch.nn.Parameter(t) for t in ts])

        def forward(self, gs):                     # d/dp sum(p * g) = g, accumulated into .grad
            return sum((p * gr).sum() for p, gr in zip(self.ps, gs))

    for host in (False, True):
        a = [x.clone().to(DEV).requires_grad_(True) for x in base]
        hb = Holder([x.clone().to(DEV) for x in base])
        b = list(hb.ps)
        oa = AdamW(a, lr=1e-2, state_on_host=host)
        ob = AdamW(b, lr=1e-2, state_on_host=host, overlap=True, ring_slots=2)
        ob.attach(hb, groups=[])                   # the forward waits for every pending update
        ptrs = None
        for gs in grads:
            for pa, gr in zip(a, gs):
                pa.grad = gr.to(DEV)
            hb([gr.to(DEV) for gr in gs]).backward()
            oa.step()
            oa.zero_grad()
            ob.step(zero_grad=True)
            ob.wait()
            assert all(bool((pb.grad == 0).all()) for pb in b)
            p2 = [pb.grad.data_ptr() for pb in b]
            assert ptrs is None or p2 == ptrs
            ptrs = p2
        ob.synchronize()
        for pa, pb in zip(a, b):
            assert torch.equal(pa, pb), host


def test_adamw_zero_grad_skips_untouched_like_set_to_none(ops):
    """The reference's optimizer.zero_grad() sets gradients to None, and AdamW then skips a
    parameter that gets no gradient in the next window (no weight decay, no moment decay).
    step(zero_grad=True) keeps the buffers zeroed instead; a buffer it zeroed that autograd has
    not accumulated into since is skipped the same way.  A toy model whose block 1 is
    bypassed in every other window: the overlapped, hook-ordered step(zero_grad=True) (attach) is
    bit-identical to step() + zero_grad(set_to_none=True) with the same kernel, and both follow
    torch.optim.AdamW; without the skip (the round-4 behaviour) the bypassed block drifts."""
    from prfl_amd.optim import AdamW

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = torch.nn.Linear(16, 64)
            self.blocks = torch.nn.ModuleList([torch.nn.Linear(64, 64) for _ in range(3)])
            self.head = torch.nn.Linear(64, 3)

        def forward(self, x, skip=()):
            x = self.emb(x)
            for i, b in enumerate(self.blocks):
                if i not in skip:
                    x = torch.tanh(b(x))
            return self.head(x)

    torch.manual_seed(0)
    models = [Toy().to(DEV) for _ in range(4)]
    for m in models[1:]:
        m.load_state_dict(models[0].state_dict())
    ref, a, b, c = models
    x = torch.randn(32, 16, device=DEV)
    topt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=0.01, foreach=False)
    oa = AdamW(list(a.parameters()), lr=1e-3)
    ob = AdamW(list(b.parameters()), lr=1e-3, overlap=True)
    ob.attach(b)
    oc = AdamW(list(c.parameters()), lr=1e-3)
    for it in range(6):
        skip = (1,) if it % 2 else ()
        for m in models:
            m(x, skip).square().mean().backward()
        topt.step()
        topt.zero_grad(set_to_none=True)
        oa.step()
        oa.zero_grad()                          # set_to_none: block 1 skipped in odd windows
        ob.step(zero_grad=True)
        oc._zeroed.clear()                      # round 4: every zeroed buffer updated
        oc.step(zero_grad=True)
    ob.synchronize()
    torch.cuda.synchronize()
    for (n, pr), pa, pb, pc in zip(ref.named_parameters(), a.parameters(), b.parameters(),
                                   c.parameters()):
        assert torch.equal(pa, pb), n
        assert rel(pa, pr) <= 1e-3, (n, rel(pa, pr))   # kernel vs torch rounding through 6 steps
    # round-4 semantics: the bypassed block decays in the windows it sat out (and the model drifts)
    assert rel(c.blocks[1].weight, a.blocks[1].weight) > 1e-4


def test_adamw_overlap_zero_grad_requires_attach(ops):
    """The refusal comes before any counter moves: after attach() the retried step
    is the first one, with the bias correction of step 1."""
    from prfl_amd.optim import AdamW
    m = torch.nn.Module()
    m.blocks = torch.nn.ModuleList([torch.nn.Linear(8, 8, bias=False).to(DEV)])
    p = m.blocks[0].weight
    p.grad = torch.ones_like(p)
    opt = AdamW([p], overlap=True)
    with pytest.raises(RuntimeError, match="attach"):
        opt.step(zero_grad=True)
    assert opt.step_count == 0 and not opt._pstep and not opt._zeroed
    twin = p.detach().clone().requires_grad_(True)
    twin.grad = torch.ones_like(twin)
    ref = AdamW([twin])
    opt.attach(m)
    opt.step(zero_grad=True)
    ref.step()
    opt.synchronize()
    assert opt.step_count == 1 and torch.equal(p, twin)
