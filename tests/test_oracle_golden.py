"""Pin the oracle (CPU restatement) to the reference's own outputs (golden fixtures).

The fixtures were produced by running the reference modules (tests/golden/make_golden.py).  These
tests run on CPU only; they are what makes the oracle trustworthy as the GPU parity checker.
"""
import numpy as np
import pytest
import torch

import seeded
from shapes import TOY, block_shapes, model_shapes, qa_shapes, mlp_shapes, seeded_params
from tolerance import key_path_scale
from oracle import wan_oracle as O

torch.set_num_threads(8)


def rel(a, b):
    a = torch.as_tensor(a, dtype=torch.float64).flatten()
    b = torch.as_tensor(b, dtype=torch.float64).flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_rope_exact(golden):
    g = golden("ops")
    freqs = O.rope_freqs(128)
    assert np.array_equal(torch.view_as_real(freqs).numpy(), g["freqs_real"])
    out = O.rope_apply(torch.from_numpy(g["rope_x"]), torch.from_numpy(g["rope_grid"]), freqs)
    assert np.array_equal(out.numpy(), g["rope_out"])


def test_norms_exact(golden):
    g = golden("ops")
    x = torch.from_numpy(g["rms_x"]).to(torch.bfloat16)
    out = O.rms_norm(x, torch.from_numpy(g["rms_w"]))
    assert np.array_equal(out.numpy(), g["rms_out"])
    xl = torch.from_numpy(g["ln_x"])
    assert np.allclose(O.layer_norm(xl).numpy(), g["ln_out"], atol=1e-6)
    assert np.array_equal(O.layer_norm(xl.to(torch.bfloat16), in_bf16=True).numpy(),
                          g["ln_out_bf16in"])
    out = O.layer_norm(xl, 1e-6, torch.from_numpy(g["ln_aff_w"]), torch.from_numpy(g["ln_aff_b"]))
    assert np.allclose(out.numpy(), g["ln_aff_out"], atol=1e-5)


def _toy_params(model_type):
    return seeded_params(model_shapes(TOY, model_type), prefix="toy.")


@pytest.mark.parametrize("model_type", ["t2v", "i2v"])
def test_toy_model_fwd_bwd(golden, model_type):
    g = golden("toy_" + model_type)
    P = {k: v.requires_grad_(True) for k, v in _toy_params(model_type).items()}
    cfg = dict(TOY, model_type=model_type)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    kw = {}
    if model_type == "i2v":
        kw = dict(y_list=[torch.from_numpy(g["y"])], clip_fea=torch.from_numpy(g["clip"]))
    out = O.model_forward(P, cfg, [x], torch.from_numpy(g["t"]), [torch.from_numpy(g["ctx"])],
                          105, **kw)[0]
    assert rel(out, g["out"]) < 2e-3, rel(out, g["out"])
    (out * torch.from_numpy(g["upstream"])).sum().backward()
    assert rel(x.grad, g["dx"]) < 2e-2, rel(x.grad, g["dx"])
    checked = 0
    for k, v in g.items():
        if k.startswith("grad/"):
            n = k[5:]
            r = rel(P[n].grad, v)
            scale = key_path_scale(g, n)
            if scale is not None:
                assert (P[n].grad.flatten() - torch.from_numpy(v)).norm().item() < 3e-2 * scale, n
            else:
                assert r < 3e-2, (n, r)
            checked += 1
        elif k.startswith("gnorm/"):
            n = k[6:]
            gn = P[n].grad.double().norm().item()
            assert abs(gn - float(v)) / max(float(v), 1e-30) < 3e-2, (n, gn, float(v))
            checked += 1
    assert checked > 20
    feats = O.model_forward({k: v.detach() for k, v in P.items()}, cfg, [x.detach()],
                            torch.from_numpy(g["t"]), [torch.from_numpy(g["ctx"])], 105,
                            output_features=True, selected_layers=[1], **kw)
    assert rel(feats[0], g["feat1"]) < 2e-3


@pytest.mark.parametrize("tag", ["t2v", "i2v"])
@pytest.mark.slow
def test_real_width_block(golden, tag):
    """One 14B block (C=5120, 40 heads, F=13824) at L=48: oracle vs reference fwd + grads."""
    g = golden("real_block_" + tag)
    P = seeded_params(block_shapes("blocks.0.", 5120, 13824, tag == "i2v"))
    P = {k: v.requires_grad_(True) for k, v in P.items()}
    L, Lc = 48, (512 if tag == "t2v" else 769)
    x = torch.from_numpy(seeded.randn("blk.x", (1, L, 5120))).requires_grad_(True)
    e = torch.from_numpy(seeded.randn("blk.e", (1, 6, 5120), 0.1)).requires_grad_(True)
    ctx = torch.from_numpy(seeded.randn("blk.ctx" + tag, (1, Lc, 5120))).to(torch.bfloat16).float()
    ctx.requires_grad_(True)
    out = O.block_forward(P, "blocks.0.", x, e, torch.from_numpy(g["grid"]), O.rope_freqs(128),
                          ctx, 40, seq_len=L, i2v=(tag == "i2v"))
    assert rel(out, g["out"]) < 1e-3, rel(out, g["out"])
    up = torch.from_numpy(seeded.randn("blk.up" + tag, (1, L, 5120)))
    (out * up).sum().backward()
    assert rel(x.grad, g["dx"]) < 2e-2, rel(x.grad, g["dx"])
    assert rel(e.grad, g["de"]) < 2e-2, rel(e.grad, g["de"])
    assert abs(ctx.grad.double().norm().item() / float(g["dctx_norm"]) - 1) < 2e-2
    for k, v in g.items():
        if k.startswith("gnorm/"):
            n = k[6:]
            gn = P["blocks.0." + n].grad.double().norm().item()
            assert abs(gn - float(v)) / max(float(v), 1e-30) < 3e-2, (n, gn, float(v))


def test_reward_head(golden):
    g = golden("reward_head")
    QA = seeded_params(qa_shapes(5120), prefix="qa.")
    ML = seeded_params(mlp_shapes(5120), prefix="mlp.")
    P = {"qa." + k: v for k, v in QA.items()}
    P.update({"mlp." + k: v for k, v in ML.items()})
    feat = torch.from_numpy(g["feat"]).requires_grad_(True)
    pooled = O.query_attention(P, "qa.", feat)
    assert rel(pooled.flatten(), g["pooled"].flatten()) < 2e-3
    r = O.mlp_reward(P, "mlp.", pooled)
    assert abs(r.item() - float(g["reward"].item())) < 1e-2
    loss = O.prfl_hinge(r)
    assert abs(loss.item() - float(g["loss"])) < 2e-3
    loss.backward()
    assert rel(feat.grad, g["dfeat"]) < 5e-2, rel(feat.grad, g["dfeat"])


def test_unipc_trajectory(golden):
    g = golden("schedulers")
    sch = O.UniPCOracle(40, 5.0)
    assert np.array_equal(sch.timesteps.numpy(), g["unipc_timesteps"])
    assert np.array_equal(sch.sigmas.numpy(), g["unipc_sigmas"])
    lat = torch.from_numpy(g["unipc_lat0"]).to(torch.bfloat16).view(1, 16, 3, 10, 14)
    for i in range(6):
        mo = torch.from_numpy(g["unipc_model_outputs"][i])
        lat = sch.step(mo, sch.timesteps[i], lat)
        assert lat.dtype == torch.bfloat16
        d = (lat.float() - torch.from_numpy(g["unipc_traj"][i])).abs().max().item()
        assert d <= 2 ** -6 * max(1.0, np.abs(g["unipc_traj"][i]).max()), (i, d)
    mo = torch.from_numpy(g["unipc_mo6"]).requires_grad_(True)
    prev = sch.step(mo, sch.timesteps[6], lat)
    assert rel(prev.float().detach(), g["unipc_prev6"]) < 1e-2
    (prev.float() * torch.from_numpy(g["unipc_w"])).sum().backward()
    assert rel(mo.grad, g["unipc_dmo6"]) < 1e-2


def test_flowmatch(golden):
    g = golden("schedulers")
    ts, sig = O.flowmatch_sigmas(1000, 5.0)
    assert np.array_equal(ts.numpy(), g["fm_timesteps"])
    assert np.allclose(sig.numpy(), g["fm_sigmas"], atol=1e-7)


def test_oracle_row_subset_and_chunked_attention_match_full():
    """The checker shortcuts used at C1's L = 20 280: block_forward(rows=...) equals the rows
    of the full forward, and the no-grad chunked attention equals the autograd FA2 path."""
    import torch
    from oracle import wan_oracle as O
    from shapes import block_shapes, seeded_params
    P = seeded_params(block_shapes("b.", 256, 512), prefix="rows.")
    g = torch.Generator().manual_seed(4)
    L = 3 * 5 * 7 + 3
    x = torch.randn(1, L, 256, generator=g)
    e = torch.randn(1, 6, 256, generator=g) * 0.1
    ctx = torch.randn(1, 512, 256, generator=g).to(torch.bfloat16).float()
    grid, fr = torch.tensor([[3, 5, 7]]), O.rope_freqs(128)
    with torch.no_grad():
        full = O.block_forward(P, "b.", x, e, grid, fr, ctx, 2, seq_len=105)
        rows = torch.tensor([0, 1, 50, 104, 105, L - 1])
        sub = O.block_forward(P, "b.", x, e, grid, fr, ctx, 2, seq_len=105, rows=rows)
    assert torch.allclose(sub, full[:, rows], rtol=1e-5, atol=1e-5)
    q, k, v = (torch.randn(1, 70, 2, 128, generator=g) for _ in range(3))
    with torch.no_grad():
        a = O.attention(q, k, v, k_len=50, q_chunk=16)
    b = O._FlashAttention.apply(q, k, v, 50, 128 ** -0.5)
    assert (a - b).abs().max().item() <= 2 ** -8 * b.abs().max().item()


@pytest.mark.parametrize("i2v", [False, True])
def test_gpu_block_checker_matches_oracle_on_cpu(i2v):
    """tests/gpu_block_checker.py (the oracle's block with a query-chunked FA2 attention, the
    checker of test_gpu_configs.py's real-geometry gradient test) run on the CPU at toy width
    equals the oracle's own autograd: output exactly, input gradient and every parameter gradient
    to fp32 rounding (the key bias, cancellation-dominated, to 5e-3)."""
    import gpu_block_checker as GC
    from shapes import block_shapes, seeded_params
    P = seeded_params(block_shapes("blocks.0.", 256, 512, i2v), prefix="chk.")
    L, grid = 105, (3, 5, 7)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(1, L, 256, generator=g)
    e = torch.randn(1, 6, 256, generator=g) * 0.1
    ctx = torch.randn(1, 769 if i2v else 512, 256, generator=g).to(torch.bfloat16)
    up = torch.randn(1, L, 256, generator=g)
    co, cdx, cG = GC.block_grads(P, "blocks.0.", x, e, ctx, grid, L, 2, up, device="cpu", i2v=i2v,
                                 chunk=32)
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    xr = x.clone().requires_grad_(True)
    ref = O.block_forward(Pr, "blocks.0.", xr, e, torch.tensor([grid]), O.rope_freqs(128),
                          ctx.float(), 2, seq_len=L, i2v=i2v)
    (ref * up).sum().backward()
    r = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert torch.equal(co, ref.detach())
    assert r(cdx, xr.grad) < 1e-4
    for k, v in Pr.items():
        if v.grad is not None:
            assert r(cG[k[len("blocks.0."):]], v.grad) < 5e-3, k
