"""Two ranks on one MI355X (gloo for the collectives, both ranks on cuda:0): the data-parallel
optimizer path bench.py takes at N > 1 for 720p — ZeRO-1 sharded AdamW with host-resident moments
streamed through HBM on side streams, overlapped with the next forward (optim.py) — must give
parameters bit-identical to the replicated single-process update, on every rank."""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SHAPES = [(64, 33), (1000,), (7,), (300, 3), (5, 5), (128, 64)]


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
    out_q.put((rank, [p.detach().cpu().clone() for p in model.parameters()], losses,
               sum(1 for p in opt.state)))
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
    res = sorted([q.get(timeout=150) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, p0, l0, n0), (_, p1, l1, n1) = res
    assert n0 + n1 == len(p0) and n0 > 0 and n1 > 0          # moments split between ranks
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
