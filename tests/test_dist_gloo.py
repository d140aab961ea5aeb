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
    # a bucket of ~1500 elements: groups [(64, 33)], [(1000,), (7,), (300, 3)], [(5, 5)] -> every
    # element shard boundary falls inside a tensor somewhere
    opt = optim.AdamW(ps, lr=1e-2, shard=True, shard_bucket_numel=1500)
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        for p in ps:
            p.grad = torch.randn(p.shape, generator=g)    # identical on both ranks (post all-reduce)
        opt.step()
    owned = {i: opt._range[p] for i, p in enumerate(ps) if p in opt._range}
    out_q.put((rank, [p.detach().numpy().copy() for p in ps], owned, opt.state_bytes() // 8))
    dist.barrier()
    dist.destroy_process_group()


def test_zero1_adamw_gloo_world2():
    """ZeRO-1 AdamW (element shards of each group, one all-gather per group): each rank holds half
    the moments; parameters equal the replicated update bit for bit."""
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
    shapes = [(64, 33), (1000,), (7,), (300, 3), (5, 5)]
    numel = [int(torch.Size(s).numel()) for s in shapes]
    # every element owned by exactly one rank, moments only for the owned elements
    for i, n in enumerate(numel):
        cover = sorted([own0[i]] if i in own0 else []) + sorted([own1[i]] if i in own1 else [])
        assert sum(b - a for a, b in cover) == n, (i, cover)
    assert n0 + n1 == sum(numel) and abs(n0 - n1) <= 3
    assert any(i in own0 and i in own1 for i in range(5))      # a tensor split between ranks
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


# ---- world 4: the trainer's whole collective schedule, recorded per rank ---------------------
# RCCL (like NCCL) needs every rank to issue the same collectives in the same order: the
# GradReducer's all-reduces (post-accumulate hooks, in autograd's order, then the coalesced small
# tensors at end()), the guard's MAX flag, the loss averages, mid_timestep's broadcast and the
# ZeRO-1 per-group all-gathers from the optimizer step.  The toy modules below stand in for the
# HIP-backed WanModel (which has no CPU path) behind the same call signature; the compute ops the
# trainer calls directly (UniPC update, clip, AdamW) are swapped for their torch restatements.

class _ToyWan(torch.nn.Module):
    """WanModel's forward signature over a [16, F, H, W] latent; blocks of mixed sizes so the
    GradReducer takes both its per-tensor and its coalesced path."""

    def __init__(self, dim=32, n_blocks=3, head=True):
        super().__init__()
        self.patch = torch.nn.Linear(16, dim)
        self.text = torch.nn.Linear(4096, dim)
        self.time = torch.nn.Parameter(torch.zeros(dim))
        self.blocks = torch.nn.ModuleList(
            [torch.nn.Sequential(torch.nn.Linear(dim, 4 * dim), torch.nn.Tanh(),
                                 torch.nn.Linear(4 * dim, dim)) for _ in range(n_blocks)])
        self.head = torch.nn.Linear(dim, 16) if head else None

    def forward(self, x, t, context, seq_len, clip_fea=None, y=None, output_features=False,
                selected_layers=(2,)):
        u = x[0]
        c, f, h, w = u.shape
        tok = u.reshape(c, -1).t().float()
        hcur = self.patch(tok) + self.text(context[0].float().mean(0)) + \
            self.time * (t.float().reshape(()) / 1000)
        feats = []
        for i, b in enumerate(self.blocks):
            hcur = hcur + b(hcur)
            if output_features and i + 1 in selected_layers:
                feats.append(hcur.unsqueeze(0))
        if output_features:
            return feats
        return [self.head(hcur).t().reshape(c, f, h, w).to(u.dtype)]


class _ToyQA(torch.nn.Module):
    def __init__(self, dim=32):
        super().__init__()
        self.q = torch.nn.Linear(dim, dim)

    def forward(self, feats):
        return self.q(feats.mean(dim=(0, 2)))


_RECORDED = ("all_reduce", "broadcast", "all_gather_into_tensor")


def _record_collectives(log):
    real = {n: getattr(dist, n) for n in _RECORDED}

    def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
        log.append(("all_reduce", tuple(t.shape), str(t.dtype), str(op)))
        return real["all_reduce"](t, op=op, group=group, async_op=async_op)

    def broadcast(t, src=0, group=None, async_op=False):
        log.append(("broadcast", tuple(t.shape), str(t.dtype), int(src)))
        return real["broadcast"](t, src=src, group=group, async_op=async_op)

    def all_gather_into_tensor(out, inp, group=None, async_op=False):
        log.append(("all_gather_into_tensor", tuple(out.shape), str(out.dtype), tuple(inp.shape)))
        return real["all_gather_into_tensor"](out, inp, group=group, async_op=async_op)
    dist.all_reduce, dist.broadcast = all_reduce, broadcast
    dist.all_gather_into_tensor = all_gather_into_tensor
    return real


def _trainer_worker(rank, world, port, out_q):
    import random
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import wan_oracle as O
    from prfl_amd import optim
    from prfl_amd.schedulers import FlowUniPCMultistepScheduler
    from prfl_amd.train import PRFLTrainer
    FlowUniPCMultistepScheduler._update = staticmethod(O.unipc_update)
    optim.ops.adamw_ = _adamw_ref
    optim.ops.sumsq_ = lambda g, ss: ss.add_(g.double().square().sum().float())
    optim.ops.scale_ = lambda g, coef: g.mul_(coef)
    torch.manual_seed(0)                               # identical replicas on every rank
    gen, lrm = _ToyWan(), _ToyWan(n_blocks=2, head=False)
    lrm.requires_grad_(False)
    qa, mlp = _ToyQA(), torch.nn.Linear(32, 1)
    qa.requires_grad_(False)
    mlp.requires_grad_(False)
    tr = PRFLTrainer(gen, lrm, qa, mlp, lr=1e-3, grad_accum=2.0, inference_steps=6,
                     feature_layer=(2,), optimizer_shard=True, optimizer_overlap=True,
                     lrm_weights_bf16=False)
    tr.reducer.small_numel = 600                       # block weights reduce alone, biases coalesce
    log = []
    real = _record_collectives(log)
    random.seed(1000 + rank)                           # each rank draws its own mid: rank 0's wins
    g = torch.Generator().manual_seed(7 + rank)        # distinct data per rank
    latents = torch.randn(1, 16, 2, 4, 4, generator=g)
    text = torch.randn(1, 5, 4096, generator=g)
    mids = []
    for step in range(4):                              # two iterations, each SFT + reward; GA 2
        tr.sft_step(step, latents, text, 32, generator=g)
        mids.append(tr.reward_step(step, latents, text, 32, generator=g)["mid"])
    for n in _RECORDED:
        setattr(dist, n, real[n])
    opt = tr.optimizer
    mine = sum(b - a for a, b in opt._range.values())
    out_q.put((rank, log, mids, mine, len(opt._layout()),
               [p.detach().numpy().copy() for p in gen.parameters()], opt.state_bytes() // 8,
               sum(p.numel() for p in tr.params)))
    dist.barrier()
    dist.destroy_process_group()


def test_prfl_trainer_collective_sequence_identical_world4():
    """four ranks run two PRFL iterations (SFT + reward, gradient
    accumulation 2, ZeRO-1 with overlap=True) through PRFLTrainer; every rank must issue the
    identical collective sequence (op, shape, dtype, reduce-op / root), the replicas must stay
    identical, rank 0's mid_timestep must reach every rank, and ZeRO-1 must take one all-gather
    per parameter group (<= 60 per optimizer step) over balanced element shards."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 4
    port = 33500 + os.getpid() % 1000
    procs = [ctx.Process(target=_trainer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([_to_torch(q.get(timeout=300)) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    logs = [r[1] for r in res]
    assert len(logs[0]) > 40
    for r in range(1, world):
        assert logs[r] == logs[0], f"rank {r} diverges at collective " \
            f"{next(i for i, (a, b) in enumerate(zip(logs[r], logs[0])) if a != b)}"
    kinds = {e[0] for e in logs[0]}
    assert kinds == {"all_reduce", "broadcast", "all_gather_into_tensor"}
    # ZeRO-1: ONE all-gather per group (embeddings, each block, the head) per optimizer update —
    # two optimizer steps per iteration (SFT + reward at GA boundaries), two iterations — and
    # no per-tensor broadcast any more (the broadcasts left are mid_timestep's, shape (1,))
    n_groups = res[0][4]
    gathers = [e for e in logs[0] if e[0] == "all_gather_into_tensor"]
    assert len(gathers) == 2 * 2 * n_groups and n_groups <= 60
    assert all(e[1] == (1,) for e in logs[0] if e[0] == "broadcast")
    print(f"collectives over 2 iterations: {len(logs[0])} ({len(gathers)} ZeRO-1 all-gathers, "
          f"{n_groups} groups per optimizer step)")
    mids = [r[2] for r in res]
    assert all(m == mids[0] for m in mids)
    mine, total = [r[3] for r in res], res[0][7]
    assert sum(mine) == total and max(mine) - min(mine) <= n_groups, mine   # balanced shards
    assert sum(r[6] for r in res) == total            # each element's moments on exactly one rank
    for r in range(1, world):
        for a, b in zip(res[r][5], res[0][5]):
            assert torch.equal(a, b)
