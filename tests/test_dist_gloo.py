"""World-size-2 data-parallel exchange on CPU (gloo): GradReducer must produce the same
accumulated, averaged gradients as single-process training on the concatenated batch, and
broadcast_int must give every rank rank-0's mid_timestep (train_prfl.py:640-652)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


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
    out_q.put((rank, {n: p.grad.clone() for n, p in model.named_parameters()}, mid, loss.item()))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_reducer_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
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
