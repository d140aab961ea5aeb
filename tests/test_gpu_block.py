"""Fused WanAttentionBlock (HIP path) vs the oracle and the reference golden fixtures.

Tolerances: block output rel-L2 <= 1e-2, input / parameter grads rel-L2 <= 3e-2.
"""
import numpy as np
import pytest
import torch

import seeded
from shapes import block_shapes, seeded_params
from tolerance import key_path_scale
from oracle import wan_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu().flatten()
    b = torch.as_tensor(b).detach().double().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def run_block(P, x, e, ctx, grid, seq_len, nh, i2v, up):
    from prfl_amd import block as B
    from prfl_amd import ops
    mod = P["blocks.0.modulation"]
    names = [n for n in B.param_names(i2v)]
    Pd = {n: P["blocks.0." + n].detach().to(DEV).requires_grad_(True) for n in names}
    xd = x.detach().to(DEV).requires_grad_(True)
    e0d = e.detach().to(DEV).requires_grad_(True)
    modd = mod.detach().to(DEV).requires_grad_(True)
    ctxd = ctx.detach().to(DEV).to(torch.bfloat16).requires_grad_(True)
    meta = B.Meta(nh, [grid], [seq_len], ops.rope_table(O.rope_freqs(128), DEV), i2v)
    out = B.block_apply(Pd, xd, modd + e0d, ctxd, meta)
    (out * up.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    return out, xd.grad, e0d.grad, modd.grad, ctxd.grad, {n: p.grad for n, p in Pd.items()}


@pytest.mark.parametrize("i2v,x_bf16", [(False, False), (True, False), (False, True)])
def test_toy_block_vs_oracle(i2v, x_bf16):
    dim, ffn, nh = 256, 512, 2
    P = seeded_params(block_shapes("blocks.0.", dim, ffn, i2v), prefix="tb.")
    L, Lc = 105, (512 if not i2v else 769)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(1, L, dim, generator=g)
    if x_bf16:
        x = x.to(torch.bfloat16)
    e = torch.randn(1, 6, dim, generator=g) * 0.1
    ctx = torch.randn(1, Lc, dim, generator=g).to(torch.bfloat16)
    up = torch.randn(1, L, dim, generator=g)
    grid = (3, 5, 7)
    out, dx, de, dmod, dctx, G = run_block(P, x, e, ctx, grid, L, nh, i2v, up)
    # oracle
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    xr = (x.clone() if x_bf16 else x.clone()).requires_grad_(True)
    er = e.clone().requires_grad_(True)
    cr = ctx.float().requires_grad_(True)
    ref = O.block_forward(Pr, "blocks.0.", xr, er, torch.tensor([grid]), O.rope_freqs(128), cr,
                          nh, seq_len=L, i2v=i2v)
    (ref * up).sum().backward()
    assert rel(out, ref) < 1e-2, rel(out, ref)
    assert rel(dx.float(), xr.grad.float()) < 3e-2, rel(dx.float(), xr.grad.float())
    assert rel(de, er.grad) < 3e-2, rel(de, er.grad)
    assert rel(dmod, Pr["blocks.0.modulation"].grad) < 3e-2
    assert rel(dctx.float(), cr.grad) < 3e-2, rel(dctx.float(), cr.grad)
    for n, gr in G.items():
        r = rel(gr, Pr["blocks.0." + n].grad)
        scale = key_path_scale({"grad/" + k: v.grad.numpy() for k, v in Pr.items()
                                if v.grad is not None}, "blocks.0." + n)
        if scale is not None:   # cancellation-dominated key-side directions (tolerance.py)
            assert (gr.cpu() - Pr["blocks.0." + n].grad).norm() < 3e-2 * scale, n
        else:
            assert r < 3e-2, (n, r)


@pytest.mark.parametrize("tag", ["t2v", "i2v"])
def test_real_width_block_vs_reference(golden, tag):
    """14B block (C=5120, 40 heads, F=13824), L=48, against the reference's own outputs."""
    g = golden("real_block_" + tag)
    i2v = tag == "i2v"
    P = seeded_params(block_shapes("blocks.0.", 5120, 13824, i2v))
    L, Lc = 48, (512 if not i2v else 769)
    x = torch.from_numpy(seeded.randn("blk.x", (1, L, 5120)))
    e = torch.from_numpy(seeded.randn("blk.e", (1, 6, 5120), 0.1))
    ctx = torch.from_numpy(seeded.randn("blk.ctx" + tag, (1, Lc, 5120))).to(torch.bfloat16)
    up = torch.from_numpy(seeded.randn("blk.up" + tag, (1, L, 5120)))
    out, dx, de, dmod, dctx, G = run_block(P, x, e, ctx, tuple(g["grid"][0]), L, 40, i2v, up)
    assert rel(out, g["out"]) < 1e-2, rel(out, g["out"])
    assert rel(dx, g["dx"]) < 3e-2, rel(dx, g["dx"])
    assert rel(de, g["de"]) < 3e-2, rel(de, g["de"])
    assert abs(dctx.double().norm().item() / float(g["dctx_norm"]) - 1) < 3e-2
    for k, v in g.items():
        if k.startswith("gnorm/") and not k.endswith("modulation"):
            n = k[6:]
            gn = G[n].double().norm().item()
            gp = (G[n].double().cpu().flatten() * torch.from_numpy(
                seeded.randn("proj:" + n, (G[n].numel(),))).double()).sum().item()
            scale = key_path_scale(g, n)
            if scale is not None:   # cancellation-dominated key-side directions (tolerance.py)
                assert abs(gn - float(v)) < 3e-2 * scale, (n, gn, float(v))
                assert abs(gp - float(g["gproj/" + n])) < 5e-2 * scale, n
                continue
            assert abs(gn / float(v) - 1) < 3e-2, (n, gn, float(v))
            assert abs(gp - float(g["gproj/" + n])) < 5e-2 * float(v), (n, gp, float(g["gproj/" + n]))
    assert abs(dmod.double().norm().item() / float(g["gnorm/modulation"]) - 1) < 3e-2


def test_real_width_block_long_L_vs_oracle():
    """14B block (C = 5120, 40 heads, F = 13 824) at L = 4 200 (3 x 35 x 40 tokens: L >= 4096
    selects the production self-attention kernels, L % 96 = 72, L % 256 = 104), with the
    attention-output stash on (the backward reuses the forward's kept (ao, lse)), vs the CPU
    oracle: output, input / modulation / context gradients and every parameter gradient."""
    from prfl_amd import block as B
    torch.set_num_threads(16)
    P = seeded_params(block_shapes("blocks.0.", 5120, 13824, False), prefix="long.")
    grid = (3, 35, 40)
    L, Lc = 4200, 512
    g = torch.Generator().manual_seed(7)
    x = torch.randn(1, L, 5120, generator=g)
    e = torch.randn(1, 6, 5120, generator=g) * 0.1
    ctx = torch.randn(1, Lc, 5120, generator=g).to(torch.bfloat16)
    up = torch.randn(1, L, 5120, generator=g)
    try:
        B.set_attn_stash_budget(1 << 30)
        out, dx, de, dmod, dctx, G = run_block(P, x, e, ctx, grid, L, 40, False, up)
    finally:
        B.set_attn_stash_budget(0)
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    xr, er = x.clone().requires_grad_(True), e.clone().requires_grad_(True)
    cr = ctx.float().requires_grad_(True)
    ref = O.block_forward(Pr, "blocks.0.", xr, er, torch.tensor([grid]), O.rope_freqs(128), cr,
                          40, seq_len=L)
    (ref * up).sum().backward()
    assert rel(out, ref) < 1e-2, rel(out, ref)
    assert rel(dx, xr.grad) < 3e-2, rel(dx, xr.grad)
    assert rel(de, er.grad) < 3e-2, rel(de, er.grad)
    assert rel(dmod, Pr["blocks.0.modulation"].grad) < 3e-2
    assert rel(dctx.float(), cr.grad) < 3e-2
    grads = {"grad/" + k: v.grad.numpy() for k, v in Pr.items() if v.grad is not None}
    for n, gr in G.items():
        refg = Pr["blocks.0." + n].grad
        scale = key_path_scale(grads, "blocks.0." + n)
        if scale is not None:
            assert (gr.cpu() - refg).norm() < 3e-2 * scale, n
        else:
            assert rel(gr, refg) < 3e-2, (n, rel(gr, refg))


@pytest.mark.parametrize("L,grid", [(105, (3, 5, 7)), (4200, (3, 35, 40))])
def test_attention_stash_is_bit_identical(L, grid):
    """Keeping the self-attention output/LSE for the backward (block.set_attn_stash_budget)
    gives bit-identical outputs and gradients to the plain checkpoint recompute (L = 4 200 runs
    the production long-KV attention kernels)."""
    from prfl_amd import block as B
    from prfl_amd import ops
    dim, ffn, nh = 256, 512, 2
    P = seeded_params(block_shapes("blocks.0.", dim, ffn, False), prefix="stash.")
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, L, dim, generator=g)
    e = torch.randn(1, 6, dim, generator=g) * 0.1 + P["blocks.0.modulation"]
    ctx = torch.randn(1, 512, dim, generator=g).to(torch.bfloat16)
    up = torch.randn(1, L, dim, generator=g)
    res = []
    try:
        for budget in (0, 1 << 30):
            B.set_attn_stash_budget(budget)
            Pd = {n: P["blocks.0." + n].to(DEV).requires_grad_(True) for n in B.param_names(False)}
            xd = x.to(DEV).requires_grad_(True)
            meta = B.Meta(nh, [grid], [L], ops.rope_table(O.rope_freqs(128), DEV), False)
            out = B.block_apply(Pd, xd, e.to(DEV), ctx.to(DEV), meta)
            if budget:          # the forward took its stash from the budget ...
                assert B._STASH["left"] == budget - (L * dim * 2 + nh * L * 4)
            (out * up.to(DEV)).sum().backward()
            # ... and the backward gave it back (no trainer reset needed between steps)
            assert B._STASH["left"] == budget
            res.append([out.detach(), xd.grad] + [p.grad for p in Pd.values()])
    finally:
        B.set_attn_stash_budget(0)
    assert all(torch.equal(a, b) for a, b in zip(*res))


def test_c1_block_forward_480p49f_vs_oracle():
    """Config C1 (`pre_480`): one 14B WanAttentionBlock forward at 480p x 49f — L = 20 280
    tokens, grid 13 x 30 x 52 (SURVEY §8 geometry), inputs as SURVEY §8d C1 (x ~ N(0,1) fp32,
    e0 ~ 0.1 N(0,1), 512 text tokens ~ N(0,1)).  The oracle computes 1 024 output rows spread over
    the sequence (first / last rows included) with keys and values from all 20 280 tokens
    (wan_oracle.block_forward(rows=...)); block output rel-L2 <= 1e-2."""
    from prfl_amd import block as B
    from prfl_amd import ops
    torch.set_num_threads(16)
    P = seeded_params(block_shapes("blocks.0.", 5120, 13824, False), prefix="c1.")
    grid = (13, 30, 52)
    L = 13 * 30 * 52
    g = torch.Generator().manual_seed(20280)
    x = torch.randn(1, L, 5120, generator=g)
    e = torch.randn(1, 6, 5120, generator=g) * 0.1
    ctx = torch.randn(1, 512, 5120, generator=g).to(torch.bfloat16)
    names = B.param_names(False)
    Pd = {n: P["blocks.0." + n].to(DEV) for n in names}
    meta = B.Meta(40, [grid], [L], ops.rope_table(O.rope_freqs(128), DEV), False)
    with torch.no_grad():
        out = B.block_apply(Pd, x.to(DEV), (P["blocks.0.modulation"] + e).to(DEV), ctx.to(DEV),
                            meta).cpu()
    rows = torch.cat([torch.arange(0, 16), torch.linspace(16, L - 17, 992).long(),
                      torch.arange(L - 16, L)])
    with torch.no_grad():
        ref = O.block_forward(P, "blocks.0.", x, e, torch.tensor([grid]), O.rope_freqs(128),
                              ctx.float(), 40, seq_len=L, rows=rows)
    assert torch.isfinite(out).all()
    assert rel(out[:, rows], ref) < 1e-2, rel(out[:, rows], ref)
