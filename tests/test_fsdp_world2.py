"""FSDP FULL_SHARD at world size 2 around the drop-in WanModel (VERDICT r04 "missing" #3): the
reference drivers' multi-GPU mode (`train_prfl.py:346-374`, `fsdp_utils.py:66-122`), which the GPU
suite can only exercise at world 1, where FSDP falls back to NO_SHARD.

Two gloo ranks on the CPU wrap a toy WanModel exactly as the drivers do (`get_dit_fsdp_kwargs(m,
"full")`: FULL_SHARD, fp32 MixedPrecision, auto-wrap on WanAttentionBlock, flat parameters;
`apply_fsdp_checkpointing` with and without the fused blocks wrapped) and run one forward /
backward on a different sample per rank.  The ops keep their product plumbing — the `prfl::`
custom-op schemas, their registered autograd formulas and fakes, the block's parameter views
taken from FSDP's all-gathered flat parameters — but their kernels are CPU stand-ins registered
in the spawned ranks only: the oracle's fp32 block forward (its autograd for the backward op) and
its bf16 linear.  So this checks the FSDP composition (parameter sharding / all-gather around the
op, the gradient reduce-scatter into the shards, checkpoint recompute through the op), not the
HIP kernels, whose parity the GPU suite holds.  Reference: the same model unwrapped in one process
on both samples, loss halved per sample (FSDP averages over ranks)."""
import concurrent.futures
import os
import traceback

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _register_cpu_standins():
    """CPU kernels for prfl::wan_block / _backward and prfl::linear_bf16 / _backward (test
    infrastructure: the product registers CUDA kernels only and raises on a CPU tensor)."""
    from oracle import wan_oracle as O
    from prfl_amd import block as B
    from prfl_amd.custom_ops import _gelu_grad

    bf16, f32 = torch.bfloat16, torch.float32

    def oracle_block(x, e, context, params, num_heads, grid, seq_lens, rope_tab, i2v, eps):
        P = {"b." + n: p for n, p in zip(B.param_names(i2v), params)}
        P["b.modulation"] = torch.zeros(1, 6, x.shape[-1])   # e already holds modulation + e0
        freqs = torch.view_as_complex(rope_tab.double().contiguous())
        g = torch.tensor(grid, dtype=torch.int64).view(-1, 3)
        assert x.shape[0] == 1 and len(seq_lens) == 1
        return O.block_forward(P, "b.", x, e, g, freqs, context.float(), num_heads,
                               seq_len=seq_lens[0], i2v=i2v, eps=eps)

    def wan_block_cpu(x, e, context, params, num_heads, grid, seq_lens, rope_tab, i2v, eps, fp8,
                      keep_attn):
        with torch.no_grad():
            out = oracle_block(x, e, context, params, num_heads, grid, seq_lens, rope_tab, i2v, eps)
        return out.float().contiguous(), x.new_empty((0,), dtype=bf16), x.new_empty((0,), dtype=f32)

    def wan_block_bwd_cpu(dout, x, e, context, params, ao, lse, num_heads, grid, seq_lens,
                          rope_tab, i2v, eps, fp8, want_w, want_ctx):
        ins = [x.detach().clone().requires_grad_(), e.detach().clone().requires_grad_(),
               context.detach().float().requires_grad_()]
        ps = [p.detach().clone().requires_grad_() for p in params]

        def vjp():
            # on a fresh thread: a custom op's kernel runs below the autograd dispatch key
            # (thread-local), where the oracle would record no graph
            with torch.enable_grad():
                out = oracle_block(ins[0], ins[1], ins[2], ps, num_heads, grid, seq_lens,
                                   rope_tab, i2v, eps)
                return torch.autograd.grad(out, ins + ps, dout.float(), allow_unused=True)

        with concurrent.futures.ThreadPoolExecutor(1) as ex:
            gs = ex.submit(vjp).result()
        gs = [torch.zeros_like(t) if g is None else g for g, t in zip(gs, ins + ps)]
        res = [gs[0].to(x.dtype), gs[1].float(),
               gs[2].to(context.dtype) if want_ctx else context.new_empty((0,))]
        return res + [g.to(p.dtype) if want_w else p.new_empty((0,)) for g, p in zip(gs[3:], params)]

    def linear_cpu(x, w, b, gelu):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).float()
        y = O.linear_bf16(x2, w.float(), None if b is None else b.float())
        if gelu:
            pre = y.to(bf16)
            y = O.gelu_tanh_bf16(y)
        else:
            pre = x.new_empty((0,), dtype=bf16)
        return y.to(bf16).view(*shp[:-1], w.shape[0]), pre

    def linear_bwd_cpu(dy, x, w, pre, need_dx, need_dw, need_db):
        N = w.shape[0]
        dy2 = dy.reshape(-1, N).to(bf16).float()
        if pre.numel():
            dy2 = (dy2 * _gelu_grad(pre.float())).to(bf16).float()
        wb = w.to(bf16).float()
        x2 = x.reshape(-1, x.shape[-1]).to(bf16).float()
        dx = (dy2 @ wb).to(bf16).view(x.shape).to(x.dtype) if need_dx else x.new_empty((0,))
        dw = (dy2.t() @ x2) if need_dw else w.new_empty((0,), dtype=f32)
        db = dy2.sum(0) if need_db else w.new_empty((0,), dtype=f32)
        return dx, dw, db

    torch.library.register_kernel("prfl::wan_block", "cpu", wan_block_cpu)
    torch.library.register_kernel("prfl::wan_block_backward", "cpu", wan_block_bwd_cpu)
    torch.library.register_kernel("prfl::linear_bf16", "cpu", linear_cpu)
    torch.library.register_kernel("prfl::linear_bf16_backward", "cpu", linear_bwd_cpu)


def _sample(rank):
    g = torch.Generator().manual_seed(40 + rank)
    x = torch.randn(16, 3, 10, 14, generator=g)
    ctx = torch.randn(20, 64, generator=g)
    up = torch.randn(16, 3, 10, 14, generator=g)
    return x, ctx, up


def _worker(rank, world, port, wrap_fused, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _run(rank, wrap_fused, out_q)
    except Exception:
        out_q.put((rank, "error", traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def _run(rank, wrap_fused, out_q):
    from torch.distributed.fsdp import FullyShardedDataParallel as FSDP
    from prfl_amd import fsdp_utils
    from prfl_amd.model import WanModel
    from shapes import TOY, model_shapes, seeded_params
    _register_cpu_standins()
    sd = seeded_params(model_shapes(TOY, "t2v"), prefix="toy.")
    m = WanModel(model_type="t2v", in_dim=16, **TOY)
    m.load_state_dict(sd)
    n_total = sum(p.numel() for p in m.parameters())
    # the drivers' kwargs; device_id is the CPU here (get_dit_fsdp_kwargs asks the current
    # CUDA device, which a CPU-only process does not have)
    cur = torch.cuda.current_device
    torch.cuda.current_device = lambda: torch.device("cpu")
    try:
        kw, ns = fsdp_utils.get_dit_fsdp_kwargs(m, "full")
    finally:
        torch.cuda.current_device = cur
    kw["device_id"] = torch.device("cpu")
    m = FSDP(m, **kw)
    fsdp_utils.apply_fsdp_checkpointing(m, ns, 1.0, wrap_fused=wrap_fused)
    n_local = sum(p.numel() for p in m.parameters())
    t = torch.tensor([700])
    x, ctx, up = _sample(rank)
    out = m(x=[x], t=t, context=[ctx], seq_len=105)[0]
    (out * up).sum().backward()
    gn = m.clip_grad_norm_(max_norm=1e9)
    torch.optim.SGD(m.parameters(), lr=1.0).step()      # p - g on the shards
    with FSDP.summon_full_params(m):
        got = {n.replace("_fsdp_wrapped_module.", "").replace("_checkpoint_wrapped_module.", ""):
               p.detach().clone().numpy() for n, p in m.named_parameters()}
    out_q.put((rank, out.detach().numpy(), float(gn), got, n_local, n_total))
    dist.barrier()


def _ref_worker(out_q):
    torch.set_num_threads(4)
    _register_cpu_standins()
    from prfl_amd.model import WanModel
    from shapes import TOY, model_shapes, seeded_params
    ref = WanModel(model_type="t2v", in_dim=16, **TOY)
    ref.load_state_dict(seeded_params(model_shapes(TOY, "t2v"), prefix="toy."))
    t = torch.tensor([700])
    outs = []
    for r in range(2):
        x, c, up = _sample(r)
        out = ref(x=[x], t=t, context=[c], seq_len=105)[0]
        outs.append(out.detach().numpy())
        ((out * up).sum() / 2).backward()
    gn = torch.nn.utils.clip_grad_norm_(ref.parameters(), max_norm=1e9)
    grads = {n: p.grad.detach().clone().numpy() for n, p in ref.named_parameters()
             if p.grad is not None}
    torch.optim.SGD(ref.parameters(), lr=1.0).step()
    out_q.put((outs, float(gn), {n: p.detach().numpy() for n, p in ref.named_parameters()}, grads))


@pytest.mark.parametrize("wrap_fused", [False, True])
def test_fsdp_full_shard_world2_composes_with_fused_block(wrap_fused):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() + int(wrap_fused)) % 200
    procs = [ctx.Process(target=_worker, args=(r, 2, port, wrap_fused, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for r in res:
        assert not (isinstance(r[1], str) and r[1] == "error"), r[2]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # FULL_SHARD really sharded: each rank holds about half of the parameters
    for _, _, _, _, n_local, n_total in res:
        assert n_local < 0.6 * n_total
    # the reference: the same model unwrapped, both samples in one (spawned: the CPU stand-ins
    # must not stay registered in this process) process, loss halved per sample
    rq = ctx.Queue()
    rp = ctx.Process(target=_ref_worker, args=(rq,))
    rp.start()
    ref_outs, gn_ref, ref_params, ref_grads = rq.get(timeout=300)
    rp.join(timeout=60)
    assert rp.exitcode == 0
    for r in range(2):
        assert torch.equal(torch.from_numpy(res[r][1]), torch.from_numpy(ref_outs[r])), f"rank {r} forward"
    assert abs(res[0][2] / gn_ref - 1) < 1e-5 and res[0][2] == res[1][2]
    # FSDP's reduce (each rank's gradient pre-divided by 2, then summed: exact) and the reference's
    # accumulation agree up to the order in which autograd sums a parameter's uses (the time
    # embedding feeds every block): held to 1e-5 of the gradient's scale plus the fp32 rounding of
    # p - g
    n_cmp, worst = 0, 0.0
    for n, pv in ref_params.items():
        if n not in ref_grads:
            continue
        p, g = torch.from_numpy(pv), torch.from_numpy(ref_grads[n])
        a = torch.from_numpy(res[0][3][n])
        assert torch.equal(a, torch.from_numpy(res[1][3][n])), n        # replicas agree
        err = (a - p).abs().max().item()
        scale = g.abs().max().item()
        assert err <= 1e-5 * scale + 2e-6 * max(1.0, p.abs().max().item()), (n, err, scale)
        worst = max(worst, err / max(scale, 1e-30))
        n_cmp += 1
    assert n_cmp > 30
    print(f"FSDP world 2 (wrap_fused={wrap_fused}): {n_cmp} parameters, worst |error| / max|grad| "
          f"{worst:.2e}")
