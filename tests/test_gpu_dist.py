"""Two ranks on one MI355X (gloo for the collectives, both ranks on cuda:0): the data-parallel
optimizer path bench.py takes at N > 1 for 720p — ZeRO-1 sharded AdamW (element shards of each
attach() group, one all-gather per group) with host-resident moments streamed through HBM on side
streams, overlapped with the next forward (optim.py) — must give parameters bit-identical to the
replicated single-process update, on every rank."""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SHAPES = [(64, 33), (1000,), (7,), (300, 3), (5, 5), (128, 64)]



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

class _Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = torch.nn.Linear(16, 32)
        self.blocks = torch.nn.ModuleList([torch.nn.Linear(32, 32) for _ in range(3)])
        self.head = torch.nn.Linear(32, 2)

    def forward(self, x):
        x = self.emb(x)
        for b in self.blocks:
            x = torch.tanh(b(x))
        return self.head(x)


def _worker(rank, world, port, out_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hy-video-prfl_amd")]
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from prfl_amd.optim import AdamW
    torch.manual_seed(0)
    model = _Toy().cuda()
    opt = AdamW(list(model.parameters()), lr=1e-2, state_on_host=True, shard=True, overlap=True,
                ring_slots=2)
    opt.init_state()
    opt.attach(model)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(8, 16, device="cuda", generator=g)
    losses = []
    for _ in range(3):
        loss = model(x).square().mean()              # waits per block for the previous update
        losses.append(loss.item())
        loss.backward()                              # same data on both ranks: grads identical
        opt.step()
        opt.zero_grad()
    opt.synchronize()
    out_q.put((rank, [p.detach().cpu().numpy().copy() for p in model.parameters()], losses,
               opt.state_bytes() // 8))
    dist.barrier()
    dist.destroy_process_group()


def test_zero1_streamed_overlapped_adamw_two_ranks_one_gpu():
    from prfl_amd.optim import AdamW
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([_to_torch(q.get(timeout=150)) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, p0, l0, n0), (_, p1, l1, n1) = res
    # moments split between ranks: element shards of each group (emb, 3 blocks, head)
    assert n0 + n1 == sum(a.numel() for a in p0) and n0 > 0 and n1 > 0
    # replicated reference: same model, synchronous on-device AdamW, one process
    torch.manual_seed(0)
    model = _Toy().cuda()
    opt = AdamW(list(model.parameters()), lr=1e-2)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(8, 16, device="cuda", generator=g)
    ref_losses = []
    for _ in range(3):
        loss = model(x).square().mean()
        ref_losses.append(loss.item())
        loss.backward()
        opt.step()
        opt.zero_grad()
    torch.cuda.synchronize()
    assert l0 == l1 == ref_losses
    for a, b, r in zip(p0, p1, model.parameters()):
        assert torch.equal(a, b) and torch.equal(a, r.detach().cpu())


def _fused_worker(rank, world, port, out_q):
    """Each rank: the toy WanModel (fused prfl::wan_block blocks) on its own sample, GradReducer
    averaging the gradients across ranks during the backward, two accumulated micro-steps."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hy-video-prfl_amd"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from prfl_amd.dist import GradReducer
    model = _toy_wan()
    red = GradReducer([p for p in model.parameters() if p.requires_grad])
    for micro in range(2):
        x, ctx, up = _sample(rank, micro)
        red.begin()
        out = model(x=[x], t=torch.tensor([700], device="cuda"), context=[ctx], seq_len=105)[0]
        (out * up).sum().backward()
        red.end()
    torch.cuda.synchronize()
    out_q.put((rank, {n: p.grad.detach().cpu().numpy().copy() for n, p in model.named_parameters()
                      if p.grad is not None}))
    dist.barrier()
    dist.destroy_process_group()


def _toy_wan():
    from shapes import TOY, model_shapes, seeded_params
    from prfl_amd.model import WanModel
    m = WanModel(model_type="t2v", in_dim=16, **TOY)
    m.load_state_dict(seeded_params(model_shapes(TOY, "t2v"), prefix="toy."))
    return m.cuda()


def _sample(rank, micro):
    g = torch.Generator().manual_seed(1000 * rank + micro)
    return (torch.randn(16, 3, 10, 14, generator=g).cuda(), torch.randn(20, 64, generator=g).cuda(),
            torch.randn(16, 3, 10, 14, generator=g).cuda())


def test_grad_reducer_fused_blocks_two_ranks_one_gpu():
    """GradReducer with the fused block nodes (its post-accumulate-grad hooks fire as each fused
    block's backward returns): every rank ends with sum_micro mean_rank(grad), bit-identical
    across ranks and to the single-process reference that averages the per-rank gradients of
    each micro-step in the same order (gloo SUM of two tensors, then / 2)."""
    import sys
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 32500 + os.getpid() % 1000
    procs = [ctx.Process(target=_fused_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([_to_torch(q.get(timeout=200)) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, g0), (_, g1) = res
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    model = _toy_wan()
    acc = {}
    for micro in range(2):
        per_rank = []
        for r in range(2):
            model.zero_grad(set_to_none=True)
            x, ctx_, up = _sample(r, micro)
            out = model(x=[x], t=torch.tensor([700], device="cuda"), context=[ctx_], seq_len=105)[0]
            (out * up).sum().backward()
            per_rank.append({n: p.grad.detach().cpu().clone() for n, p in model.named_parameters()
                             if p.grad is not None})
        for n in per_rank[0]:
            avg = (per_rank[0][n] + per_rank[1][n]) / 2
            acc[n] = avg if n not in acc else acc[n] + avg
    assert set(acc) == set(g0) == set(g1) and len(acc) > 30
    for n in acc:
        assert torch.equal(g0[n], g1[n]), n
        # (2 acc + f0 + f1) / 2 vs acc + (f0 + f1) / 2: equal up to fp32 rounding of the sums
        scale = acc[n].abs().max().item()
        assert (g0[n] - acc[n]).abs().max().item() <= 4e-6 * scale + 1e-12, n


def _rccl_worker(port, out_q):
    """One rank over RCCL (backend "nccl") on cuda:0: GradReducer forced on at world size 1, so the
    exchange bench.py runs at N > 1 executes for real — post-accumulate-grad hooks on the fused
    blocks, async all_reduce(AVG) per large gradient, coalesced flat reduce of the small ones,
    copy-back — on the toy WanModel, two accumulated micro-steps."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hy-video-prfl_amd"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    from prfl_amd.dist import GradReducer
    model = _toy_wan()
    red = GradReducer([p for p in model.parameters() if p.requires_grad], small_numel=4096, min_world=1)
    assert red.backend == "nccl" and red.active and len(red.handles) > 30
    n_works = []
    for micro in range(2):
        x, ctx, up = _sample(0, micro)
        red.begin()
        out = model(x=[x], t=torch.tensor([700], device="cuda"), context=[ctx], seq_len=105)[0]
        (out * up).sum().backward()
        n_works.append(len(red.works) + (1 if red.small_pending else 0))
        red.end()
    torch.cuda.synchronize()
    out_q.put((n_works, {n: p.grad.detach().cpu().numpy().copy() for n, p in model.named_parameters()
                         if p.grad is not None}))
    dist.destroy_process_group()


def test_grad_reducer_rccl_one_rank():
    """The RCCL branch of GradReducer (AVG op, no division) executed on the GPU: gradients after
    two accumulated micro-steps equal the plain single-process accumulation bit for bit (an AVG
    over one rank is exact), and the hooks actually issued the collectives."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(port, q))
    p.start()
    n_works, g = _to_torch(q.get(timeout=200))
    p.join(timeout=60)
    assert all(n > 5 for n in n_works), n_works
    model = _toy_wan()
    for micro in range(2):
        x, ctx_, up = _sample(0, micro)
        out = model(x=[x], t=torch.tensor([700], device="cuda"), context=[ctx_], seq_len=105)[0]
        (out * up).sum().backward()
    torch.cuda.synchronize()
    ref = {n: p.grad.detach().cpu() for n, p in model.named_parameters() if p.grad is not None}
    assert set(ref) == set(g)
    for n in ref:
        assert torch.equal(g[n], ref[n]), n
