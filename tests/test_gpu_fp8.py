"""fp8 path (config C5, `train_prfl_i2v_720` "fp8 MFMA path"): per-row e4m3 quantisation and the
block-scaled fp8 MFMA GEMM (csrc/gemm.hip) on the MI355X.

Bars: quantisation bit-exact vs torch's float8_e4m3fn cast of the same scaled values; the GEMM
exact on integer data (every product and partial sum representable) and within fp32 summation
order + the bf16 output rounding (rel-L2 <= 3e-3) on random data, including every 720p x 81f
projection shape of the block (M = 73 920); an fp8 linear against the bf16 linear of the same
operands within the SURVEY §8c fp8 tolerance (rel-L2 <= 5e-2); the real-width I2V block on the
fp8 path at L = 4 200 against the oracle's fp32 truth, held to k = 16 times the bf16 path's
error against that same truth (see test_block_fp8_vs_fp32_truth)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
FP8 = torch.float8_e4m3fn


def rel(a, b):
    a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("M,K,dt", [(7, 5120, torch.bfloat16), (300, 13824, torch.bfloat16),
                                    (64, 1024, torch.float32), (3, 8, torch.float32)])
def test_quant_rows_fp8_matches_torch_cast(M, K, dt):
    from prfl_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M * K)
    x = (torch.randn(M, K, generator=g, device=DEV) * torch.rand(M, 1, generator=g, device=DEV) * 9)
    x = x.to(dt)
    x[0, :] = 0                                            # an all-zero row: scale 1, q = 0
    q, s = ops.quant_rows_fp8(x)
    # fp32 IEEE divisions as the kernel does them (tensor / tensor on the CPU: no reciprocal
    # rewrite), then the scaled values cast by torch
    amax = x.float().abs().amax(1).cpu()
    c448 = torch.full_like(amax, 448.0)
    ref_s = torch.where(amax > 0, amax / c448, torch.ones_like(amax))
    inv = torch.where(amax > 0, c448 / amax, torch.ones_like(amax))
    ref_q = (x.float().cpu() * inv[:, None]).to(FP8)
    q = q.cpu()
    assert torch.equal(s.cpu(), ref_s)
    bad = (q.view(torch.uint8) != ref_q.view(torch.uint8)).sum().item()
    assert bad == 0, f"{bad} of {q.numel()} e4m3 codes differ"


def test_gemm_fp8_exact_on_integers_asymmetric():
    """A = I-like integer pattern against an ASYMMETRIC B: catches any row/col or k-map error."""
    from prfl_amd import ops
    M, N, K = 512, 768, 384
    g = torch.Generator().manual_seed(0)
    a = torch.randint(-3, 4, (M, K), generator=g).float()
    b = (torch.arange(N)[:, None] * 7 + torch.arange(K)[None, :] * 3) % 9 - 4
    b = b.float()
    sa = torch.full((M,), 0.5)
    sb = torch.linspace(0.25, 2.0, N)
    out = ops.linear_fp8(a.to(FP8).to(DEV), sa.to(DEV), b.to(FP8).to(DEV), sb.to(DEV),
                         out=torch.empty(M, N, dtype=torch.float32, device=DEV),
                         epilogue=ops.EPI_RESID, res=torch.zeros(M, N, device=DEV))
    # RESID stores res + bf16(y) * gate: the linear output is rounded to bf16 as under autocast
    ref = ((a @ b.T) * (sa[:, None] * sb[None, :])).to(torch.bfloat16).float()
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("M,N,K", [(1000, 1536, 5120), (4096, 5120, 13824), (333, 260, 256)])
def test_gemm_fp8_random_epilogues(M, N, K):
    from prfl_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=DEV) / K ** 0.5)
    bias = (0.1 * torch.randn(N, generator=g, device=DEV)).to(torch.bfloat16)
    xq, xs = ops.quant_rows_fp8(x)
    wq, ws = ops.quant_rows_fp8(w)
    deq = (xq.float() * xs[:, None]) @ (wq.float() * ws[:, None]).T
    y = ops.linear_fp8(xq, xs, wq, ws, bias)
    assert rel(y.float(), (deq + bias.float()).to(torch.bfloat16).float()) < 3e-3
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    act = ops.linear_fp8(xq, xs, wq, ws, bias, epilogue=ops.EPI_GELU, aux=pre)
    ref_pre = (deq + bias.float()).to(torch.bfloat16).float()
    assert rel(pre.float(), ref_pre) < 3e-3
    assert rel(act.float(), torch.nn.functional.gelu(ref_pre, approximate="tanh")) < 3e-3
    res = torch.randn(M, N, generator=g, device=DEV)
    gate = torch.randn(N, generator=g, device=DEV)
    o = ops.linear_fp8(xq, xs, wq, ws, bias, epilogue=ops.EPI_RESID, res=res, gate=gate)
    assert rel(o, res + ref_pre * gate) < 3e-3
    # the fp8 path against the bf16 path of the same operands (SURVEY §8c fp8 tolerance)
    yb = ops.linear(x, w.to(torch.bfloat16), bias)
    assert rel(y.float(), yb.float()) < 5e-2


def _rel_gpu(a, b, rows=8192):
    """rel-L2 of two large [M, N] device tensors, reduced on the device in fp64 row blocks."""
    num = torch.zeros((), dtype=torch.float64, device=a.device)
    den = torch.zeros((), dtype=torch.float64, device=a.device)
    for i in range(0, a.shape[0], rows):
        x, y = a[i:i + rows].double(), b[i:i + rows].double()
        num += (x - y).pow(2).sum()
        den += y.pow(2).sum()
        del x, y
    return (num.sqrt() / den.sqrt()).item()


@pytest.mark.parametrize("N,K", [(15360, 5120), (5120, 5120), (13824, 5120), (5120, 13824)])
def test_gemm_fp8_720p_shapes(N, K):
    """The fp8 GEMM at every 720p x 81f forward-projection shape of config C5 (M = 73 920 tokens;
    fused QKV 15360 x 5120, O / cross q / cross o 5120 x 5120, FFN in 13824 x 5120, FFN out
    5120 x 13824) against the product of the dequantised operands computed in fp32 on the same
    device (torch.matmul, allow_tf32 off): within fp32 summation order + the bf16 output rounding."""
    from prfl_amd import ops
    assert not torch.backends.cuda.matmul.allow_tf32
    M = 73920
    g = torch.Generator(device=DEV).manual_seed(N + K)
    x = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, generator=g, device=DEV) / K ** 0.5
    bias = (0.1 * torch.randn(N, generator=g, device=DEV)).to(torch.bfloat16)
    xq, xs = ops.quant_rows_fp8(x)
    del x
    wq, ws = ops.quant_rows_fp8(w)
    y = ops.linear_fp8(xq, xs, wq, ws, bias)
    torch.cuda.synchronize()
    wd = (wq.float() * ws[:, None]).T.contiguous()
    ref = torch.empty(M, N, dtype=torch.float32, device=DEV)
    for i in range(0, M, 16384):        # dequantised A rows in blocks (fp32 A would be 4 GB)
        a = xq[i:i + 16384].float() * xs[i:i + 16384, None]
        torch.matmul(a, wd, out=ref[i:i + 16384])
        ref[i:i + 16384] += bias.float()
        del a
    r = _rel_gpu(y, ref.to(torch.bfloat16))
    assert r < 3e-3, r
    assert torch.isfinite(y).all()


def _block_update(P, names, x, e, ctx, grid, up, i2v, fp8):
    from oracle import wan_oracle as O
    from prfl_amd import block as B
    from prfl_amd import ops
    L = x.shape[1]
    Pd = {n: P["b." + n].to(DEV).requires_grad_(True) for n in names}
    xd = x.to(DEV).requires_grad_(True)
    meta = B.Meta(40, [grid], [L], ops.rope_table(O.rope_freqs(128), DEV), i2v, fp8=fp8)
    out = B.block_apply(Pd, xd, e.to(DEV), ctx.to(DEV), meta)
    (out * up.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    return ((out.detach() - xd.detach()).cpu(), xd.grad.cpu(),
            {n: p.grad.cpu() for n, p in Pd.items()})


def test_block_fp8_vs_fp32_truth():
    """Config C5's fp8 path on the real-width I2V block (C = 5120, 40 heads, F = 13 824, 257
    image + 512 text context tokens) at L = 4 200 (3 x 35 x 40: the production long-KV attention
    kernels), against the oracle.

    Reference points, all on the same weights and inputs: the oracle with the reference's bf16
    cast points (`wan_oracle.block_forward`, = the reference under autocast) and the oracle's
    fp32 TRUTH (every cast point removed: fp32 operands everywhere, unrounded attention).
    Criterion: err(fp8 path vs truth) <= k * err(bf16 path vs truth), k = 16, for
    the block's residual update, the input gradient and the projection-weight gradients, plus an
    absolute cap of 1e-1.  Why k = 16: it is the unit-roundoff ratio of the two operand formats
    (e4m3 keeps 3 mantissa bits, bf16 7: 2^-4 vs 2^-8), i.e. the fp8 path may sit as far from the
    truth as one e4m3 rounding of its GEMM operands sits from one bf16 rounding.  Measured on this
    block (GPU run r3a): 4.5x (dx) to 9.8x (FFN-out weight grad), update 8.4x = 5.3 % vs 0.62 %
    — the e4m3 mantissa, not the kernel: per-row scales leave no operand subnormal, so block
    scaling cannot lower it.  A broken fp8 kernel (wrong scale, lost k-block) is >= 100 % off,
    > 160x.  The bf16 path itself is also held to the oracle (<= 1e-2).  The same bound holds with
    the C5 self-attention forward (int8 Q.K^T, e4m3 P.V) on as well (block.Meta fp8 = 2):
    measured within 5 % of the projections-only errors on every tensor (GPU run r3i).  Round 6:
    config C5's default keeps the cross-attention q / o projections bf16 (block.C5_KEEP_BF16),
    which holds the update to SURVEY §8c's absolute 5e-2 as well (2.5 % measured)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from shapes import block_shapes, seeded_params
    from oracle import wan_oracle as O
    from prfl_amd import block as B
    torch.set_num_threads(16)
    C, Fd, nh, i2v = 5120, 13824, 40, True
    P = seeded_params(block_shapes("b.", C, Fd, i2v), prefix="fp8t.")
    names = B.param_names(i2v)
    grid = (3, 35, 40)
    L = grid[0] * grid[1] * grid[2]
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1, L, C, generator=g)
    e0 = torch.randn(1, 6, C, generator=g) * 0.1
    e = e0 + P["b.modulation"]
    ctx = torch.randn(1, 512 + 257, C, generator=g).to(torch.bfloat16)
    up = torch.randn(1, L, C, generator=g)
    c5 = B.fp8_code(2, B.C5_KEEP_BF16)     # config C5's default: cross-attention q / o bf16
    hip = {fp8: _block_update(P, names, x, e, ctx, grid, up, i2v, fp8) for fp8 in (0, 1, 2, c5)}

    def oracle(truth):
        saved = O.bf
        if truth:
            O.bf = lambda t: t
        try:
            Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
            xr = x.clone().requires_grad_(True)
            ref = O.block_forward(Pr, "b.", xr, e0, torch.tensor([grid]), O.rope_freqs(128),
                                  ctx.float(), nh, seq_len=L, i2v=i2v)
            (ref * up).sum().backward()
            return ((ref - x).detach(), xr.grad, {n: Pr["b." + n].grad for n in names})
        finally:
            O.bf = saved
    truth = oracle(True)
    ref16 = oracle(False)
    keys = ["update", "dx", "self_attn.q.weight", "self_attn.o.weight", "cross_attn.q.weight",
            "cross_attn.o.weight", "ffn.0.weight", "ffn.2.weight"]

    def errs(res, against):
        d, gx, G = res
        td, tgx, tG = against
        out = {"update": rel(d, td), "dx": rel(gx, tgx)}
        out.update({n: rel(G[n], tG[n]) for n in keys[2:]})
        return out
    e16, e8, eor = errs(hip[0], truth), errs(hip[1], truth), errs(ref16, truth)
    e8a = errs(hip[2], truth)
    e8d = errs(hip[c5], truth)
    e16_vs_oracle = errs(hip[0], ref16)
    print("vs truth: bf16 path", {k: round(v, 4) for k, v in e16.items()})
    print("vs truth: fp8 path ", {k: round(v, 4) for k, v in e8.items()})
    print("vs truth: fp8+attn ", {k: round(v, 4) for k, v in e8a.items()})
    print("vs truth: oracle   ", {k: round(v, 4) for k, v in eor.items()})
    print("fp8 / bf16 ratio   ", {k: round(e8[k] / e16[k], 2) for k in keys})
    print("fp8+attn / bf16    ", {k: round(e8a[k] / e16[k], 2) for k in keys})
    print("vs truth: C5 default", {k: round(v, 4) for k, v in e8d.items()})
    for k in keys:
        assert e8[k] <= 16 * e16[k] and e8[k] <= 1e-1, (k, e8[k], e16[k])
        assert e8a[k] <= 16 * e16[k] and e8a[k] <= 1e-1, (k, e8a[k], e16[k])
        assert e8d[k] <= 16 * e16[k] and e8d[k] <= 1e-1, (k, e8d[k], e16[k])
    # SURVEY §8c's fp8 tolerance, met by the default C5 path (round 6: 2.5 % measured; every
    # projection on e4m3, the 5.3 % above, does not meet it: test_c5_per_projection_error_table)
    assert e8d["update"] <= 5e-2 and e8d["dx"] <= 5e-2, e8d
    assert e16_vs_oracle["update"] < 1e-2 and e16_vs_oracle["dx"] < 3e-2, e16_vs_oracle




def test_c5_per_projection_error_table():
    """which e4m3 operand sets config C5's per-block error?  The real-width I2V
    block of test_block_fp8_vs_fp32_truth (C = 5120, 40 heads, F = 13 824, 257 + 512 context
    tokens, L = 4 200), run with e4m3 on ONE forward projection at a time (QKV, self-attn o,
    cross q, cross o, FFN up, FFN down; every other GEMM bf16), with only the int8 / e4m3
    self-attention forward, with everything (the C5 path), and with everything but the largest
    contributor(s) kept bf16 (block.fp8_code); each against the oracle's fp32 truth.  Relative
    errors add in quadrature (independent roundings), so the table says what keeping a
    projection bf16 buys.  Asserted: every single-operand error sits between the bf16 path's and
    the full C5 path's; the table is printed for the record (profiles/r06_c5_projection_table.log)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from shapes import block_shapes, seeded_params
    from oracle import wan_oracle as O
    from prfl_amd import block as B
    torch.set_num_threads(16)
    C, Fd, nh, i2v = 5120, 13824, 40, True
    P = seeded_params(block_shapes("b.", C, Fd, i2v), prefix="fp8t.")
    names = B.param_names(i2v)
    grid = (3, 35, 40)
    L = grid[0] * grid[1] * grid[2]
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1, L, C, generator=g)
    e0 = torch.randn(1, 6, C, generator=g) * 0.1
    e = e0 + P["b.modulation"]
    ctx = torch.randn(1, 512 + 257, C, generator=g).to(torch.bfloat16)
    up = torch.randn(1, L, C, generator=g)
    saved = O.bf
    O.bf = lambda t: t                       # the fp32 truth: every cast point removed
    try:
        Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
        xr = x.clone().requires_grad_(True)
        ref = O.block_forward(Pr, "b.", xr, e0, torch.tensor([grid]), O.rope_freqs(128),
                              ctx.float(), nh, seq_len=L, i2v=i2v)
        (ref * up).sum().backward()
        truth = ((ref - x).detach(), xr.grad)
    finally:
        O.bf = saved
    del Pr, ref

    def err(code):
        d, gx, _ = _block_update(P, names, x, e, ctx, grid, up, i2v, code)
        return rel(d, truth[0]), rel(gx, truth[1])

    rows = {"bf16": err(0), "C5 (all e4m3 + attention)": err(B.fp8_code(2))}
    for pj in B.PROJ:
        rows[f"only {pj}"] = err(B.fp8_code(1, [q for q in B.PROJ if q != pj]))
    rows["only attention"] = err(B.fp8_code(2, B.PROJ))
    singles = sorted(B.PROJ, key=lambda pj: -rows[f"only {pj}"][0])
    for k in (1, 2):
        keep = singles[:k]
        rows[f"C5 with {'+'.join(keep)} bf16"] = err(B.fp8_code(2, keep))
    print("C5 per-projection error vs the fp32 truth (update, dx):")
    for k, (u, dx) in rows.items():
        print(f"  {k:34s} update {u:.4f}  dx {dx:.4f}")
    quad = (sum(rows[f"only {pj}"][0] ** 2 for pj in B.PROJ) + rows["only attention"][0] ** 2) ** 0.5
    print(f"  quadrature sum of the singles: update {quad:.4f}")
    b16, full = rows["bf16"][0], rows["C5 (all e4m3 + attention)"][0]
    for pj in B.PROJ:
        assert b16 <= rows[f"only {pj}"][0] <= 1.05 * full, (pj, rows[f"only {pj}"], b16, full)


def test_fp8_error_across_a_block_chain():
    """Does config C5's per-block error compound over depth?  Four real-width I2V blocks (C =
    5120, 40 heads, independent weights) chained at L = 4 200, no grad: after every block the
    cumulative residual update x_k - x_0 of the fp8 path (e4m3 projections AND the int8 / e4m3
    self-attention forward, block.Meta fp8 = 2) and of the bf16 path, both against the oracle's
    fp32 truth chain (every cast point removed).  Held to the single-block rule at every depth
    (fp8 <= 16 x bf16 and <= 1e-1), and to NO compounding: the fp8 chain's error after four
    blocks stays within 1.5 x its error after one (the e4m3 roundings of different blocks are
    independent, so the relative error of the summed update does not grow with depth; a
    compounding bias would).  VERDICT r03 weak #8: 'nothing measures what 5 % per block does
    across 40 blocks'."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from shapes import block_shapes, seeded_params
    from oracle import wan_oracle as O
    from prfl_amd import block as B
    from prfl_amd import ops
    torch.set_num_threads(16)
    C, Fd, nh, i2v, depth = 5120, 13824, 40, True, 4
    grid = (3, 35, 40)
    L = grid[0] * grid[1] * grid[2]
    names = B.param_names(i2v)
    g = torch.Generator().manual_seed(21)
    x0 = torch.randn(1, L, C, generator=g)
    ctx = torch.randn(1, 512 + 257, C, generator=g).to(torch.bfloat16)
    rope = ops.rope_table(O.rope_freqs(128), DEV)
    xs = {"truth": x0.clone(), 0: x0.to(DEV), 2: x0.to(DEV)}
    errs = {0: [], 2: []}
    saved = O.bf
    for k in range(depth):
        P = seeded_params(block_shapes("b.", C, Fd, i2v), prefix=f"fp8chain{k}.")
        e0 = torch.randn(1, 6, C, generator=g) * 0.1
        O.bf = lambda t: t
        try:
            with torch.no_grad():
                xs["truth"] = O.block_forward(P, "b.", xs["truth"], e0, torch.tensor([grid]),
                                              O.rope_freqs(128), ctx.float(), nh, seq_len=L, i2v=i2v)
        finally:
            O.bf = saved
        Pd = {n: P["b." + n].to(DEV) for n in names}
        e = (e0 + P["b.modulation"]).to(DEV)
        for fp8 in (0, 2):
            meta = B.Meta(nh, [grid], [L], rope, i2v, fp8=fp8)
            with torch.no_grad():
                xs[fp8] = B.block_apply(Pd, xs[fp8], e, ctx.to(DEV), meta)
        del Pd, P
        upd_t = xs["truth"] - x0
        for fp8 in (0, 2):
            errs[fp8].append(rel((xs[fp8] - x0.to(DEV)).cpu(), upd_t))
    print("cumulative-update error vs the fp32 truth per depth: bf16", [round(v, 4) for v in errs[0]],
          "fp8", [round(v, 4) for v in errs[2]])
    for k in range(depth):
        assert errs[2][k] <= 16 * errs[0][k] and errs[2][k] <= 1e-1, (k, errs[2][k], errs[0][k])
        assert errs[0][k] < 1e-2, (k, errs[0][k])
    assert errs[2][-1] <= 1.5 * errs[2][0], errs[2]


# ------------------------------------------------- low-precision self-attention forward (C5) --
def _quant_ref(q, k, v, H, klen=None):
    """The kernel's quantisation restated in torch (prfl_attn_fwd_fp8's prologue): Q int8 per
    (token, head) and K int8 per (128-key tile, head), each amax / 127, round to nearest even;
    V e4m3 per (head, channel), amax / 448; the K / V scales over the keys < klen only (masked
    keys are quantised to 0).  Returns the DEQUANTISED fp32 operands [H, L, 128]."""
    Lq, Lk = q.shape[0], k.shape[0]
    klen = Lk if klen is None else klen
    if klen < Lk:
        k, v = k.clone(), v.clone()
        k[klen:] = 0
        v[klen:] = 0
    qh = q.float().view(Lq, H, 128).transpose(0, 1)
    kh = k.float().view(Lk, H, 128).transpose(0, 1)
    vh = v.float().view(Lk, H, 128).transpose(0, 1)
    c127 = torch.tensor(127.0, device=q.device)
    c448 = torch.tensor(448.0, device=q.device)

    def qi8(x, amax):
        inv = torch.where(amax > 0, c127 / amax, torch.zeros_like(amax))
        return torch.round(x * inv) * torch.where(amax > 0, amax / c127, torch.ones_like(amax))
    kt = torch.zeros(H, (Lk + 127) // 128 * 128, 128, device=q.device)
    kt[:, :Lk] = kh
    kam = kt.view(H, -1, 128 * 128).abs().amax(-1)                       # [H, tiles]
    kam = kam.repeat_interleave(128, 1)[:, :Lk, None]
    vam = vh.abs().amax(1, keepdim=True)
    vinv = torch.where(vam > 0, c448 / vam, torch.zeros_like(vam))
    return (qi8(qh, qh.abs().amax(-1, keepdim=True)), qi8(kh, kam),
            (vh * vinv).to(FP8).float() * (vam / c448))


def _attn64(qh, kh, vh, klen, scale, rows=None):
    """fp64 softmax attention of [H, L, 128] operands over keys < klen (query rows `rows`) ->
    (o [Lq', H*128], lse2 [H, Lq'])."""
    if rows is not None:
        qh = qh[:, rows]
    s = torch.bmm(qh.double(), kh[:, :klen].double().transpose(1, 2)) * scale
    lse = torch.logsumexp(s, -1)
    o = torch.bmm(torch.softmax(s, -1), vh[:, :klen].double())
    return o.transpose(0, 1).reshape(qh.shape[1], -1), lse / torch.log(torch.tensor(2.0)).double()


@pytest.mark.parametrize("Lq,Lk,H,klen", [(4200, 4200, 16, 4133), (1000, 4100, 2, 4097),
                                          (300, 777, 2, 777), (4111, 5000, 1, 4500)])
def test_attn_fp8_vs_dequantised_fp64(Lq, Lk, H, klen):
    """The C5 attention forward (int8 Q.K^T, e4m3 P.V) against fp64 attention over the same
    QUANTISED operands (the prologue restated in torch): isolates the kernel (k-slot maps of both
    products, the transposed and key-permuted V image, the folded per-token / per-tile / per-
    channel scales, masking, the split-KV tail: 4200 x 16 heads = 272 query-tile units on 256
    CUs) from the rounding of Q, K, V itself.  Left: the e4m3 rounding of P and fp32
    accumulation: O within 2.5e-2 rel-L2 (measured 1.7-2.0e-2; a swapped key or channel is
    ~1.4).  The scores are exact (integer products, i32 sums), but the row sums come out of the
    P.V MFMA over the e4m3-ROUNDED P (the normaliser then matches the numerator's weights), so the
    log2 LSE carries that rounding: within 5e-2 (measured <= 2.7e-2, i.e. <= 1.9 % in the sum;
    a lost key tile or a wrong scale is >= 1)."""
    from prfl_amd import ops
    g = torch.Generator(device=DEV).manual_seed(Lq * 7 + Lk)
    C = H * 128
    q = (torch.randn(Lq, C, generator=g, device=DEV) * 1.5).to(torch.bfloat16)
    k = (torch.randn(Lk, C, generator=g, device=DEV) * 1.5).to(torch.bfloat16)
    v = torch.randn(Lk, C, generator=g, device=DEV)
    v = (v * torch.linspace(0.1, 3.0, C, device=DEV)).to(torch.bfloat16)   # uneven channel scales
    scale = 128 ** -0.5
    o, lse = ops.attn_fwd_fp8(q, k, v, H, k_len=klen)
    torch.cuda.synchronize()
    qd, kd, vd = _quant_ref(q, k, v, H, klen)
    ro, rlse = _attn64(qd, kd, vd, klen, scale)
    assert torch.isfinite(o).all()
    r = rel(o, ro)
    print(f"vs dequantised fp64: O rel-L2 {r:.3e}, max |dLSE2| {(lse.double() - rlse).abs().max().item():.2e}")
    assert r < 2.5e-2, r
    assert (lse.double() - rlse).abs().max().item() < 5e-2


@pytest.mark.parametrize("Lq,Lk,klen", [(1000, 4100, 3990), (600, 777, 700)])
def test_attn_fp8_masked_keys_set_no_scale(Lq, Lk, klen):
    """Keys at or past k_len (padding) set none of the C5 quantisation scales: with
    the padding rows 1000 x larger than the valid keys, the output and LSE are bit-identical to
    those of zero padding, and match fp64 attention over the operands quantised from the valid
    keys alone."""
    from prfl_amd import ops
    H = 2
    g = torch.Generator(device=DEV).manual_seed(Lk + klen)
    C = H * 128
    # operands as test_attn_fp8_vs_dequantised_fp64 draws them (its 2.5e-2 bound is the e4m3
    # rounding of P for that score spread)
    q = (torch.randn(Lq, C, generator=g, device=DEV) * 1.5).to(torch.bfloat16)
    k = (torch.randn(Lk, C, generator=g, device=DEV) * 1.5).to(torch.bfloat16)
    v = torch.randn(Lk, C, generator=g, device=DEV)
    v = (v * torch.linspace(0.1, 3.0, C, device=DEV)).to(torch.bfloat16)
    k0, v0 = k.clone(), v.clone()
    k0[klen:] = 0
    v0[klen:] = 0
    kb, vb = k0.clone(), v0.clone()
    kb[klen:] = 1000 * torch.randn(Lk - klen, C, generator=g, device=DEV).to(torch.bfloat16)
    vb[klen:] = 1000 * torch.randn(Lk - klen, C, generator=g, device=DEV).to(torch.bfloat16)
    o0, l0 = ops.attn_fwd_fp8(q, k0, v0, H, k_len=klen)
    ob, lb = ops.attn_fwd_fp8(q, kb, vb, H, k_len=klen)
    torch.cuda.synchronize()
    assert torch.isfinite(ob).all()
    assert torch.equal(o0, ob) and torch.equal(l0, lb)
    qd, kd, vd = _quant_ref(q, kb, vb, H, klen)
    ro, _ = _attn64(qd, kd, vd, klen, 128 ** -0.5)
    assert rel(ob, ro) < 2.5e-2, rel(ob, ro)


@pytest.mark.parametrize("L,H", [(4200, 16), (73920, 1)])
def test_attn_fp8_vs_fp64_truth(L, H):
    """fp32-truth rule of config C5 (as for the fp8 block): err(C5 attention
    vs fp64 attention of the bf16 operands) <= k * err(bf16 attention vs the same) on sampled
    query rows, incl. the 720p x 81f token count (73 920 keys).  k = 24: the P.V product rounds
    BOTH of its operands to e4m3 (P and V, independent roundings, unit roundoff 2^-4 each) where
    the bf16 kernel rounds one (P, 2^-8): sqrt(2) x 16 = 22.6, rounded up.  Zero-mean random V
    is the worst case for a relative error (|O| is small while each rounding error is not);
    measured 17.3x (4 200 keys, 16 heads) and 19.4x (73 920 keys), 4.0-4.4 % vs 0.23 %; the
    kernel alone against the dequantised operands is test_attn_fp8_vs_dequantised_fp64."""
    from prfl_amd import ops
    g = torch.Generator(device=DEV).manual_seed(L + H)
    C = H * 128
    q = (torch.randn(L, C, generator=g, device=DEV) * 1.5).to(torch.bfloat16)
    k = (torch.randn(L, C, generator=g, device=DEV) * 1.5).to(torch.bfloat16)
    v = torch.randn(L, C, generator=g, device=DEV).to(torch.bfloat16)
    scale = 128 ** -0.5
    o8, _ = ops.attn_fwd_fp8(q, k, v, H)
    o16, _ = ops.attn_fwd(q, k, v, H)
    rows = torch.randperm(L, generator=torch.Generator().manual_seed(3))[:256].sort().values.to(DEV)
    tr, _ = _attn64(*(x.float().view(L, H, 128).transpose(0, 1) for x in (q, k, v)), L, scale,
                    rows=rows)
    e8, e16 = rel(o8[rows], tr), rel(o16[rows], tr)
    print(f"attn C5 vs truth {e8:.3e}, bf16 vs truth {e16:.3e}, ratio {e8 / e16:.2f}")
    assert e8 <= 24 * e16, (e8, e16)
    assert e8 < 6e-2


def test_c5_reward_gradient_direction_vs_bf16_and_truth():
    """what config C5's fp8 path does to the gradient PRFL trains on.  The
    generator piece of the reward backward (`train_prfl.py:703-830`: one grad-enabled generator
    step at t_mid, then the differentiable UniPC step, with a fixed upstream d(stepped)) at real
    width (I2V, C = 5120, 40 heads, F = 13 824, 2 blocks + embeddings + head, 257 CLIP tokens) and
    L = 4 200 (latent [16, 3, 70, 80]), mid_timestep 0, on three paths with the same weights and
    inputs: the bf16 path, the fp8 path (set_fp8_gemm(True, attn=True): e4m3 projections, int8 /
    e4m3 self-attention forward, bf16 backward), and the oracle's fp32 TRUTH (wan_oracle's model
    with every cast point removed, run on the GPU by tests/gpu_block_checker.py, + the oracle's
    UniPC step).  Per parameter: rel-L2 and cosine of the fp8 gradient vs the truth and vs the
    bf16 gradient; the whole gradient's cosine.  Bounds: see the asserts."""
    import math
    import os
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import gpu_block_checker as GC
    from tolerance import key_path_scale
    from oracle import wan_oracle as O
    from prfl_amd.model import WanModel
    from prfl_amd.schedulers import FlowUniPCMultistepScheduler
    from prfl_amd.train import batch2list, list2batch
    torch.manual_seed(5)
    with torch.device(DEV):
        gen = WanModel(model_type="i2v", in_dim=36, num_layers=2, dim=5120, ffn_dim=13824,
                       freq_dim=256, text_dim=4096, out_dim=16, num_heads=40)
        torch.nn.init.normal_(gen.head.head.weight, std=0.02)   # random-init trap
    Fl, Hl, Wl = 3, 70, 80
    L = Fl * (Hl // 2) * (Wl // 2)
    g = torch.Generator(device=DEV).manual_seed(4200)
    lat = torch.randn(1, 16, Fl, Hl, Wl, generator=g, device=DEV).to(torch.bfloat16)
    text = (0.08 * torch.randn(1, 126, 4096, generator=g, device=DEV)).to(torch.bfloat16)
    clip = torch.randn(1, 257, 1280, generator=g, device=DEV).to(torch.bfloat16)
    cond = torch.randn(1, 16, Fl, Hl, Wl, generator=g, device=DEV).to(torch.bfloat16)
    mask = torch.zeros(1, 4, Fl, Hl, Wl, device=DEV, dtype=torch.bfloat16)
    mask[:, :, :1] = 1
    cond = torch.cat([mask, cond], dim=1)
    up = torch.randn(1, 16, Fl, Hl, Wl, generator=g, device=DEV)
    names = [n for n, _ in gen.named_parameters()]

    def ours(fp8):
        gen.set_fp8_gemm(fp8, attn=fp8)
        for p in gen.parameters():
            p.grad = None
        sch = FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1,
                                          use_dynamic_shifting=False)
        sch.set_timesteps(num_inference_steps=40, device=DEV, shift=5.0)
        t = sch.timesteps[0]
        npred = list2batch(gen(x=batch2list(lat), t=t.reshape(1), context=batch2list(text),
                               seq_len=L, clip_fea=clip, y=batch2list(cond)))
        stepped = sch.step(npred, t, lat, return_dict=False)[0]
        (stepped.float() * up).sum().backward()
        torch.cuda.synchronize()
        return {n: p.grad.detach().float().cpu() for n, p in gen.named_parameters()}, int(t)

    g16, t0 = ours(False)
    g8, _ = ours(True)
    gen.set_fp8_gemm(False)
    # the fp32 truth: the oracle's model on the GPU with every bf16 cast point removed
    cfg = dict(dim=5120, num_heads=40, model_type="i2v", freq_dim=256, text_len=512, out_dim=16,
               num_layers=2)
    Pd = {n: p.detach().float().clone().requires_grad_(True) for n, p in gen.named_parameters()}
    saved = O.bf
    O.bf = lambda t: t
    try:
        with GC.oracle_on(DEV):
            out = O.model_forward(Pd, cfg, [lat[0].float()], torch.tensor([t0], device=DEV),
                                  [text[0].float()], L, clip_fea=clip.float(),
                                  y_list=[cond[0].float()])
            sch = O.UniPCOracle(40, 5.0)
            stepped = sch.step(out[0], t0, lat[0].float())
            (stepped * up[0]).sum().backward()
    finally:
        O.bf = saved
    torch.cuda.synchronize()
    gt = {n: Pd[n].grad.detach().float().cpu() for n in names}
    del Pd, out, stepped

    def cos(a, b):
        a, b = a.double().flatten(), b.double().flatten()
        return (a @ b / (a.norm() * b.norm()).clamp_min(1e-300)).item()
    gnp = {"grad/" + n: v.numpy() for n, v in gt.items()}
    rows = []
    for n in names:
        if key_path_scale(gnp, n) is not None or gt[n].norm() == 0:
            continue                       # cancellation-dominated key-side directions
        rows.append((n, rel(g8[n], gt[n]), rel(g16[n], gt[n]), cos(g8[n], gt[n]),
                     cos(g16[n], gt[n]), cos(g8[n], g16[n])))
    cat = lambda d: torch.cat([d[n].flatten() for n in names])  # noqa: E731
    whole = {"fp8 vs truth": cos(cat(g8), cat(gt)), "bf16 vs truth": cos(cat(g16), cat(gt)),
             "fp8 vs bf16": cos(cat(g8), cat(g16)),
             "fp8 rel vs truth": rel(cat(g8), cat(gt)), "bf16 rel vs truth": rel(cat(g16), cat(gt))}
    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
    print("whole-gradient", {k: round(v, 5) for k, v in whole.items()})
    print("per-parameter (%d): fp8 rel vs truth median %.4f max %.4f | bf16 median %.4f max %.4f | "
          "fp8 cos vs truth min %.5f | fp8 cos vs bf16 min %.5f" % (
              len(rows), med([r[1] for r in rows]), max(r[1] for r in rows),
              med([r[2] for r in rows]), max(r[2] for r in rows), min(r[3] for r in rows),
              min(r[5] for r in rows)))
    for r in sorted(rows, key=lambda r: -r[1])[:12]:
        print("  %-40s fp8 rel %.4f (bf16 %.4f)  cos fp8/truth %.5f  bf16/truth %.5f  fp8/bf16 %.5f"
              % r)
    assert all(math.isfinite(v) for r in rows for v in r[1:])
    # bf16 path: the parity bar of every other gradient test
    assert whole["bf16 rel vs truth"] < 3e-2 and whole["bf16 vs truth"] > 0.999, whole
    # fp8 path: the C5 rule of test_block_fp8_vs_fp32_truth on the whole gradient (<= 16 x the
    # bf16 path's error and <= 1e-1) and the direction kept: cosine to the truth >= 0.99
    assert whole["fp8 rel vs truth"] <= 16 * whole["bf16 rel vs truth"], whole
    assert whole["fp8 rel vs truth"] <= 1e-1 and whole["fp8 vs truth"] >= 0.99, whole
    for n, e8, e16, c8, c16, c816 in rows:
        assert e8 <= max(16 * e16, 2e-2) and c8 >= 0.95, (n, e8, e16, c8)
