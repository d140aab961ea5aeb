"""FSDP FULL_SHARD at world size 2 with the HIP kernels (VERDICT r05 "missing" #3): the reference
drivers' multi-GPU mode (`train_prfl.py:346-374`, `fsdp_utils.py:66-122`) around the drop-in
WanModel, both ranks on cuda:0.  tests/test_fsdp_world2.py holds the same composition on the CPU
with stand-in kernels; here every op is the shipped `prfl::` HIP path (fused blocks, bf16 linears,
attention, norms) running on FSDP's all-gathered flat parameters, its gradients reduce-scattered
into the shards, `clip_grad_norm_` over the shards and an SGD step on them.

The collectives: RCCL refuses two ranks on one device, so the ranks run gloo, and the four calls
FSDP makes (`all_gather_into_tensor`, `reduce_scatter_tensor`, `all_reduce`, `all_gather`:
`_flat_param.py`, `_runtime_utils.py`, `fully_sharded_data_parallel.py`) are staged through host
memory for CUDA tensors in the spawned ranks only (test infrastructure; on a node each rank owns
its GPU and FSDP's own RCCL calls run).

Reference: the same model unwrapped in rank 0's process on both samples, the loss halved per
sample (FSDP's reduce-scatter averages over the ranks)."""
import os
import traceback

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _stage_collectives():
    import torch.distributed as dist
    ag, rs, ar, agl = (dist.all_gather_into_tensor, dist.reduce_scatter_tensor, dist.all_reduce,
                       dist.all_gather)

    def all_gather_into_tensor(out, inp, group=None, async_op=False):
        assert not async_op
        o = out.cpu()
        ag(o, inp.cpu(), group=group)
        out.copy_(o)

    def reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=None, async_op=False):
        assert not async_op
        o = out.cpu()
        rs(o, inp.cpu(), op=op, group=group)
        out.copy_(o)

    def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
        assert not async_op
        if not t.is_cuda:
            return ar(t, op=op, group=group)
        c = t.cpu()
        ar(c, op=op, group=group)
        t.copy_(c)

    def all_gather(outs, t, group=None, async_op=False):
        assert not async_op
        cs = [o.cpu() for o in outs]
        agl(cs, t.cpu(), group=group)
        for o, c in zip(outs, cs):
            o.copy_(c)

    dist.all_gather_into_tensor, dist.reduce_scatter_tensor = all_gather_into_tensor, reduce_scatter_tensor
    dist.all_reduce, dist.all_gather = all_reduce, all_gather


def _sample(rank):
    g = torch.Generator().manual_seed(40 + rank)
    x = torch.randn(16, 3, 10, 14, generator=g)
    ctx = torch.randn(20, 64, generator=g)
    up = torch.randn(16, 3, 10, 14, generator=g)
    return x, ctx, up


def _model():
    from prfl_amd.model import WanModel
    from shapes import TOY, model_shapes, seeded_params
    m = WanModel(model_type="t2v", in_dim=16, **TOY)
    m.load_state_dict(seeded_params(model_shapes(TOY, "t2v"), prefix="toy."))
    return m


def _worker(rank, world, port, wrap_fused, out_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hy-video-prfl_amd"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        out_q.put((rank, _run(rank, wrap_fused)))
    except Exception:
        out_q.put((rank, "error:" + traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def _run(rank, wrap_fused):
    import torch.distributed as dist
    from torch.distributed.fsdp import FullyShardedDataParallel as FSDP
    from prfl_amd import fsdp_utils
    _stage_collectives()
    m = _model()
    n_total = sum(p.numel() for p in m.parameters())
    kw, ns = fsdp_utils.get_dit_fsdp_kwargs(m, "full")       # the drivers' kwargs, device cuda:0
    m = FSDP(m, **kw)
    fsdp_utils.apply_fsdp_checkpointing(m, ns, 1.0, wrap_fused=wrap_fused)
    n_local = sum(p.numel() for p in m.parameters())
    t = torch.tensor([700], device="cuda")
    x, ctx, up = (v.cuda() for v in _sample(rank))
    out = m(x=[x], t=t, context=[ctx], seq_len=105)[0]
    (out * up).sum().backward()
    gn = float(m.clip_grad_norm_(max_norm=1e9))
    torch.optim.SGD(m.parameters(), lr=1.0).step()          # p - g on the shards
    with FSDP.summon_full_params(m):
        got = {n.replace("_fsdp_wrapped_module.", "").replace("_checkpoint_wrapped_module.", ""):
               p.detach().float().cpu().clone() for n, p in m.named_parameters()}
    rep = {"n_local": n_local, "n_total": n_total, "gn": gn}
    outs = [t_.cpu() for t_ in [out.detach().float()]]
    gathered = [torch.empty_like(outs[0]) for _ in range(2)]
    dist.all_gather(gathered, outs[0])
    names = sorted(got)
    flat = torch.cat([got[n].flatten() for n in names])
    other = [torch.empty_like(flat) for _ in range(2)]
    dist.all_gather(other, flat)
    rep["replicas_equal"] = torch.equal(other[0], other[1])
    del m
    torch.cuda.empty_cache()
    if rank == 0:
        ref = _model().cuda()
        ref_outs = []
        for r in range(2):
            xr, cr, ur = (v.cuda() for v in _sample(r))
            o = ref(x=[xr], t=t, context=[cr], seq_len=105)[0]
            ref_outs.append(o.detach().float().cpu())
            ((o * ur).sum() / 2).backward()
        grads = {n: p.grad.detach().float().cpu().clone() for n, p in ref.named_parameters()
                 if p.grad is not None}
        rep["gn_ref"] = float(torch.nn.utils.clip_grad_norm_(ref.parameters(), max_norm=1e9))
        torch.optim.SGD(ref.parameters(), lr=1.0).step()
        rep["out_exact"] = all(torch.equal(gathered[r], ref_outs[r]) for r in range(2))
        worst, n_cmp = 0.0, 0
        for n, p in ref.named_parameters():
            if n not in grads:
                continue
            a, b = got[n], p.detach().float().cpu()
            scale = grads[n].abs().max().item()
            err = (a - b).abs().max().item()
            worst = max(worst, err / max(scale, 1e-30))
            rep.setdefault("bad", [])
            if err > 1e-5 * scale + 2e-6 * max(1.0, b.abs().max().item()):
                rep["bad"].append((n, err, scale))
            n_cmp += 1
        rep["n_cmp"], rep["worst"] = n_cmp, worst
    dist.barrier()
    return rep


@pytest.mark.parametrize("wrap_fused", [False, True])
def test_fsdp_full_shard_two_ranks_one_gpu_hip_kernels(wrap_fused):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 34600 + (os.getpid() + int(wrap_fused)) % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, wrap_fused, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(res[r], str), res[r]
    rep = res[0]
    print(f"FSDP 2 ranks on cuda:0 (wrap_fused={wrap_fused}): n_cmp {rep['n_cmp']}, worst |error| / "
          f"max|grad| {rep['worst']:.2e}, grad norm {rep['gn']:.6g} vs {rep['gn_ref']:.6g}")
    for r in range(2):
        assert res[r]["n_local"] < 0.6 * res[r]["n_total"]          # really sharded
        assert res[r]["replicas_equal"]
    assert rep["out_exact"]                  # each rank's output = the unwrapped model's, bit for bit
    assert abs(rep["gn"] / rep["gn_ref"] - 1) < 1e-5 and res[1]["gn"] == rep["gn"]
    # measured: every updated parameter bit-identical to the unwrapped model's (the halved loss
    # halves every gradient exactly, and the one sum of the two samples' halves is the same add
    # either way; profiles/r06_gputest_fsdp.log); held to the CPU test's 1e-5 of the gradient scale
    assert rep["n_cmp"] > 30 and not rep["bad"], rep["bad"][:5]
    for p in procs:
        assert p.exitcode == 0
