"""Ulysses sequence parallelism of the fused block on the MI355X (VERDICT r05 "next" #1): ranks
sharing cuda:0, each holding seq_len / P tokens of one real-width 14B block (C = 5120, 40 heads,
F = 13 824) at L = 4 200, run the HIP path with the head-sharded self-attention (40 / P heads over
all 4 200 keys, `prfl_rms_rope_*_pos` at the rank's row offset); rank 0 runs the same block
unsharded as the reference.  The exchange is gloo's all-to-all staged through host memory (RCCL
refuses two ranks on one device) — the same `prfl_amd.sp` calls the RCCL path makes.

Held (reference semantics, `model.py:183-196`, `communication.py:40-160`): the gathered output
and input gradient vs the unsharded block; d(modulation), d(context) and every parameter gradient
summed over the ranks vs the unsharded block's (context-side parameters and d(context) at bf16
resolution: each rank's partial is a bf16 attention-backward output, as in the reference's SP);
the attention stash (kept head-sharded (O, LSE)) bit-identical to the recompute.  The host logic
is also held at fp32 exactness (fp64 stand-in kernels, world 4, whole model) by
tests/test_sp_gloo.py."""
import os
import traceback

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CTX_PARTS = ("cross_attn.k.", "cross_attn.v.", "cross_attn.norm_k.", "cross_attn.k_img.",
             "cross_attn.v_img.", "cross_attn.norm_k_img.")


def _rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _setup(i2v):
    from shapes import block_shapes, seeded_params
    C, F, nh, L = 5120, 13824, 40, 4200
    P = seeded_params(block_shapes("blocks.0.", C, F, i2v), prefix="spb.")
    g = torch.Generator().manual_seed(21)
    x = torch.randn(1, L, C, generator=g)
    e = torch.randn(1, 6, C, generator=g) * 0.1
    ctx = (torch.randn(1, 769 if i2v else 512, C, generator=g) * 0.5).to(torch.bfloat16)
    up = torch.randn(1, L, C, generator=g)
    return P, x, e, ctx, up, (6, 20, 35), nh


def _run_block(P, x, e, ctx, up, grid, nh, i2v, L, st, keep):
    from oracle import wan_oracle as O
    from prfl_amd import block as B
    from prfl_amd import ops
    names = B.param_names(i2v)
    Pd = {n: P["blocks.0." + n].cuda().requires_grad_(True) for n in names}
    xd = x.cuda().requires_grad_(True)
    ed = e.cuda().requires_grad_(True)
    modd = P["blocks.0.modulation"].cuda().requires_grad_(True)
    cd = ctx.cuda().requires_grad_(True)
    meta = B.Meta(nh, [grid], [L], ops.rope_table(O.rope_freqs(128), "cuda"), i2v, sp=st)
    B.set_attn_stash_budget(int(1e10) if keep else 0)
    out = B.block_apply(Pd, xd, modd + ed, cd, meta)
    (out * up.cuda()).sum().backward()
    B.set_attn_stash_budget(0)
    torch.cuda.synchronize()
    return (out.detach(), xd.grad, ed.grad, modd.grad, cd.grad,
            {n: p.grad for n, p in Pd.items()})


def _worker(rank, world, port, i2v, out_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hy-video-prfl_amd"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        out_q.put((rank, _run(rank, world, i2v)))
    except Exception:
        out_q.put((rank, "error:" + traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def _run(rank, world, i2v):
    import torch.distributed as dist
    from prfl_amd import sp
    P, x, e, ctx, up, grid, nh = _setup(i2v)
    L = x.shape[1]
    st = sp.set_group(None)
    s = L // world
    rows = slice(rank * s, (rank + 1) * s)
    got = _run_block(P, x[:, rows], e, ctx, up[:, rows], grid, nh, i2v, L, st, keep=False)
    kept = _run_block(P, x[:, rows], e, ctx, up[:, rows], grid, nh, i2v, L, st, keep=True)
    stash_exact = all(torch.equal(a, b) for a, b in zip(got[:5], kept[:5])) and \
        all(torch.equal(got[5][n], kept[5][n]) for n in got[5])
    del kept
    out = sp.all_gather_seq(got[0].cpu(), st)
    dx = sp.all_gather_seq(got[1].cpu(), st)
    sums = [got[2].cpu(), got[3].cpu(), got[4].float().cpu()] + [got[5][n].cpu() for n in sorted(got[5])]
    for t in sums:
        dist.all_reduce(t)
    names = sorted(got[5])
    del got
    torch.cuda.empty_cache()
    dist.barrier()
    rep = {"stash_exact": stash_exact}
    if rank == 0:
        sp.set_group(False)
        ref = _run_block(P, x, e, ctx, up, grid, nh, i2v, L, None, keep=False)
        rep["out"] = _rel(out, ref[0].cpu())
        rep["dx"] = _rel(dx, ref[1].cpu())
        rep["de"] = _rel(sums[0], ref[2].cpu())
        rep["dmod"] = _rel(sums[1], ref[3].cpu())
        rep["dctx"] = _rel(sums[2], ref[4].float().cpu())
        worst, worst_ctx = 0.0, 0.0
        G = {n: g.cpu() for n, g in ref[5].items()}
        for n, g in zip(names, sums[3:]):
            r = _rel(g, G[n])
            if n.endswith(("k.bias", "k_img.bias")):       # key-side: on the value path's scale
                vb = n.replace("k.bias", "v.bias").replace("k_img.bias", "v_img.bias")
                r = (g - G[n]).double().norm().item() / G[vb].double().norm().item()
            if any(p in n for p in CTX_PARTS):
                worst_ctx = max(worst_ctx, r)
            elif r > worst:
                worst, rep["worst"] = r, n
        rep["param"], rep["param_ctx"] = worst, worst_ctx
    dist.barrier()
    return rep


@pytest.mark.parametrize("world,i2v", [(2, False), (4, True)])
def test_sp_block_ranks_on_one_gpu_vs_unsharded(world, i2v):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + (os.getpid() + world) % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, i2v, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    rep = res[0]
    print(f"SP {world} ({'i2v' if i2v else 't2v'}): {rep}")
    assert all(res[r]["stash_exact"] for r in range(world))
    # a GEMM / RMSNorm row is computed identically whatever the partition; the attention grid
    # (40 / P heads) takes a different split-KV tail (flash-decoding merge order), and the
    # cross-rank sums add partials in another order: bf16 flips downstream of those, and the
    # column sums (d gate, d modulation, norm3) cancel heavily.  Measured at P = 2 (t2v): out /
    # dx 2.2e-4, d e 2.6e-3, worst parameter 4.2e-3, context side 4.8e-3; at P = 4 (i2v) out / dx
    # bit-identical, parameters 4.4e-7, context side 4.0e-3 (profiles/r06_gputest_sp.log) — all
    # an order below the 3e-2 bound that holds the unsharded block to the oracle
    assert rep["out"] < 1e-3 and rep["dx"] < 1e-3, rep
    assert rep["de"] < 1e-2 and rep["dmod"] < 1e-2, rep
    assert rep["param"] < 1e-2, rep
    assert rep["param_ctx"] < 2e-2 and rep["dctx"] < 2e-2, rep
    for p in procs:
        assert p.exitcode == 0
