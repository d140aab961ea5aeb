"""World-size-2 data-parallel exchange on CPU (gloo): GradReducer must produce the same
accumulated, averaged gradients as single-process training on the concatenated batch, and
broadcast_int must give every rank rank-0's mid_timestep (train_prfl.py:640-652)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp



def _to_torch(obj):
    """numpy payloads from the worker processes (sent by value: shared-memory tensor handles die
    with a worker that has already exited) -> torch."""
    import numpy as np
    if isinstance(obj, np.ndarray):
        return torch.from_numpy(obj)
    if isinstance(obj, dict):
        return {k: _to_torch(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_torch(v) for v in obj)
    return obj

def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from prfl_amd.dist import GradReducer, broadcast_int, all_reduce_mean
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(300, 300), torch.nn.ReLU(), torch.nn.Linear(300, 7))
    red = GradReducer(list(model.parameters()), small_numel=512)
    g = torch.Generator().manual_seed(100 + rank)
    for micro in range(3):                    # grad accumulation across micro-steps
        x = torch.randn(4, 300, generator=g)
        red.begin()
        model(x).pow(2).mean().backward()
        red.end()
    mid = broadcast_int(17 if rank == 0 else 3)
    loss = all_reduce_mean(torch.tensor([float(rank)]))
    out_q.put((rank, {n: p.grad.numpy().copy() for n, p in model.named_parameters()}, mid, loss.item()))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_reducer_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [_to_torch(q.get(timeout=120)) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda r: r[0])
    (_, g0, mid0, l0), (_, g1, mid1, l1) = res
    assert mid0 == mid1 == 17 and l0 == l1 == 0.5
    # reference: single process, average over ranks of each micro-step's grads, accumulated
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(300, 300), torch.nn.ReLU(), torch.nn.Linear(300, 7))
    gens = [torch.Generator().manual_seed(100 + r) for r in range(2)]
    for micro in range(3):
        for r in range(2):
            x = torch.randn(4, 300, generator=gens[r])
            (model(x).pow(2).mean() / 2).backward()
    for n, p in model.named_parameters():
        assert torch.allclose(g0[n], p.grad, atol=1e-6, rtol=1e-5), n
        assert torch.equal(g0[n], g1[n]), n


def _adamw_ref(p, g, m, v, lr, b1, b2, eps, wd, step):
    """torch.optim.AdamW update (the prfl_adamw kernel's contract) for the CPU test."""
    p.mul_(1 - lr * wd)
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    denom = (v / (1 - b2 ** step)).sqrt_().add_(eps)
    p.addcdiv_(m, denom, value=-lr / (1 - b1 ** step))


def _zero1_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from prfl_amd import optim
    optim.ops.adamw_ = _adamw_ref
    torch.manual_seed(0)
    ps = [torch.randn(s).requires_grad_(True) for s in [(64, 33), (1000,), (7,), (300, 3), (5, 5)]]
    opt = optim.AdamW(ps, lr=1e-2, shard=True)
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        for p in ps:
            p.grad = torch.randn(p.shape, generator=g)    # identical on both ranks (post all-reduce)
        opt.step()
    owned = sorted(i for i, p in enumerate(ps) if opt.owner[p] == rank)
    out_q.put((rank, [p.detach().numpy().copy() for p in ps], owned, len(opt.state)))
    dist.barrier()
    dist.destroy_process_group()


def test_zero1_adamw_gloo_world2():
    """ZeRO-1 AdamW: each rank holds half the moments; parameters equal the replicated update."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_zero1_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([_to_torch(q.get(timeout=120)) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, p0, own0, n0), (_, p1, own1, n1) = res
    assert sorted(own0 + own1) == list(range(5)) and not set(own0) & set(own1)
    assert n0 == len(own0) and n1 == len(own1)
    torch.manual_seed(0)
    ref = [torch.randn(s) for s in [(64, 33), (1000,), (7,), (300, 3), (5, 5)]]
    st = [(torch.zeros_like(p), torch.zeros_like(p)) for p in ref]
    g = torch.Generator().manual_seed(1)
    for step in range(1, 4):
        for p, (m, v) in zip(ref, st):
            _adamw_ref(p, torch.randn(p.shape, generator=g), m, v, 1e-2, 0.9, 0.999, 1e-8, 0.01, step)
    for a, b, r in zip(p0, p1, ref):
        assert torch.equal(a, b) and torch.equal(a, r)


class _DoneWork:
    def wait(self):
        return True


def _avg_worker(rank, world, port, out_q):
    """GradReducer's RCCL branch (ReduceOp.AVG, no host-side division) run over gloo: gloo has
    no AVG, so AVG is emulated as SUM followed by the division RCCL performs internally."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from prfl_amd import dist as pdist
    real = dist.all_reduce

    def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
        if op == dist.ReduceOp.AVG:
            real(t, op=dist.ReduceOp.SUM)
            t.div_(world)
            return _DoneWork() if async_op else None
        return real(t, op=op, async_op=async_op)
    pdist.dist.all_reduce = all_reduce
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(300, 300), torch.nn.ReLU(), torch.nn.Linear(300, 7))
    red = pdist.GradReducer(list(model.parameters()), small_numel=512)
    red.backend = "nccl"                       # take the RCCL code path
    assert red._op() == dist.ReduceOp.AVG
    g = torch.Generator().manual_seed(100 + rank)
    for micro in range(3):
        x = torch.randn(4, 300, generator=g)
        red.begin()
        model(x).pow(2).mean().backward()
        red.end()
    pdist.dist.all_reduce = real
    out_q.put((rank, {n: p.grad.numpy().copy() for n, p in model.named_parameters()}))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_reducer_rccl_branch_arithmetic_world2():
    """The AVG path: after end() every rank holds acc + avg(fresh) without dividing again."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    procs = [ctx.Process(target=_avg_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([_to_torch(q.get(timeout=120)) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, g0), (_, g1) = res
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(300, 300), torch.nn.ReLU(), torch.nn.Linear(300, 7))
    gens = [torch.Generator().manual_seed(100 + r) for r in range(2)]
    for micro in range(3):
        for r in range(2):
            x = torch.randn(4, 300, generator=gens[r])
            (model(x).pow(2).mean() / 2).backward()
    for n, p in model.named_parameters():
        assert torch.allclose(g0[n], p.grad, atol=1e-6, rtol=1e-5), n
        assert torch.equal(g0[n], g1[n]), n


def _guard_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from prfl_amd.train import guard_loss
    res = []
    # only rank 1's loss is NaN: both ranks skip (a lone skip would stall the grad all-reduce)
    res.append(guard_loss(torch.tensor(float("nan") if rank == 1 else 0.5)) is None)
    # both finite: neither skips; a large loss is clamped on its own rank only
    big = guard_loss(torch.tensor(3e6 if rank == 0 else 0.25))
    res.append(float(big))
    out_q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_nan_loss_skip_is_agreed_across_ranks_world2():
    """`train_prfl.py:800-811` under data parallelism: the NaN / Inf skip is taken by every rank
    when any rank's loss is bad; the |loss| > 1e6 clamp stays per rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 32500 + os.getpid() % 1000
    procs = [ctx.Process(target=_guard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, r0), (_, r1) = res
    assert r0[0] and r1[0]
    assert r0[1] == 1e6 and r1[1] == 0.25
