"""Ulysses sequence parallelism through the WHOLE drop-in WanModel on the MI355X: two ranks
sharing cuda:0 run the toy T2V and I2V models (2 heads of 128, 2 blocks) with `prfl_amd.sp` on,
every op the shipped HIP path, and rank 0 runs the same model with SP off.  tests/test_sp_gloo.py
holds the host logic at world 4 with fp64 CPU stand-ins; tests/test_gpu_sp.py the fused block at
real width.  This one covers the model-level pieces on the GPU: the per-rank sequence chunk
(`model.py:618-619`), RoPE at the rank's offset over `pad_freqs` (`:89-96`, the padded case:
seq_len 256 > 240 tokens), the feature / head all-gathers (`:663-676`) and their autograd.

Held: the gathered output and features vs SP = 1, and summed over the ranks the input gradient
and every parameter gradient (context-side ones at bf16 resolution, as in tests/test_gpu_sp.py).
The exchange is gloo staged through host memory (RCCL refuses two ranks on one device)."""
import os
import traceback

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CTX_PARAMS = ("text_embedding.", "img_emb.")
CTX_PARTS = ("cross_attn.k.", "cross_attn.v.", "cross_attn.norm_k.", "cross_attn.k_img.",
             "cross_attn.v_img.", "cross_attn.norm_k_img.")


def _rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _inputs(model_type):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(16, 4, 12, 20, generator=g)            # grid (4, 6, 10): 240 tokens
    ctx = torch.randn(24, 64, generator=g)
    up = torch.randn(16, 4, 12, 20, generator=g)
    clip = torch.randn(1, 257, 1280, generator=g) if model_type == "i2v" else None
    y = torch.randn(20, 4, 12, 20, generator=g) if model_type == "i2v" else None
    return x, ctx, up, clip, y


def _model(model_type):
    from prfl_amd.model import WanModel
    from shapes import TOY
    torch.manual_seed(3)
    m = WanModel(model_type=model_type, in_dim=16 if model_type == "t2v" else 36, **TOY)
    with torch.no_grad():                 # the reference zero-inits the head: give it a gradient path
        m.head.head.weight.normal_(0, 0.02)
    return m.cuda()


def _step(m, model_type, seq_len):
    x, ctx, up, clip, y = (None if v is None else v.cuda() for v in _inputs(model_type))
    x = x.clone().requires_grad_()
    m.zero_grad(set_to_none=True)
    kw = dict(clip_fea=clip, y=[y] if y is not None else None)
    t = torch.tensor([700], device="cuda")
    out = m(x=[x], t=t, context=[ctx], seq_len=seq_len, **kw)[0]
    feats = m(x=[x], t=t, context=[ctx], seq_len=seq_len, output_features=True,
              selected_layers=[1, 2], **kw)
    g = torch.Generator().manual_seed(11)
    fup = [torch.randn(f.shape, generator=g).cuda() for f in feats]
    loss = (out * up).sum() + sum((f.float() * u).sum() for f, u in zip(feats, fup)) * 1e-2
    loss.backward()
    grads = {n: p.grad.detach().float().cpu() for n, p in m.named_parameters() if p.grad is not None}
    torch.cuda.synchronize()
    return (out.detach().float().cpu(), [f.detach().float().cpu() for f in feats],
            x.grad.detach().float().cpu(), grads)


def _worker(rank, world, port, model_type, seq_len, out_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hy-video-prfl_amd"), os.path.join(root, "tests", "golden")]
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        out_q.put((rank, _run(rank, model_type, seq_len)))
    except Exception:
        out_q.put((rank, "error:" + traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def _run(rank, model_type, seq_len):
    import torch.distributed as dist
    from prfl_amd import sp
    m = _model(model_type)
    st = sp.set_group(None)
    got = _step(m, model_type, seq_len)
    sp.set_group(False)
    dx = got[2].clone()
    dist.all_reduce(dx)
    names = sorted(got[3])
    sums = {n: got[3][n].clone() for n in names}
    for n in names:
        dist.all_reduce(sums[n])
    rep = {"n_param": len(names), "size": st.size}
    if rank == 0:
        ref = _step(m, model_type, seq_len)
        rep["out"] = _rel(got[0], ref[0])
        rep["feat"] = max(_rel(a, b) for a, b in zip(got[1], ref[1]))
        rep["dx"] = _rel(dx, ref[2])
        assert sorted(ref[3]) == names, "a parameter lost its gradient under SP"
        worst, worst_ctx = 0.0, 0.0
        for n in names:
            r = _rel(sums[n], ref[3][n])
            if n.endswith(("k.bias", "k_img.bias")):      # key-side: on the value path's scale
                vb = n.replace("k.bias", "v.bias").replace("k_img.bias", "v_img.bias")
                r = (sums[n] - ref[3][n]).double().norm().item() / ref[3][vb].double().norm().item()
            if n.startswith(CTX_PARAMS) or any(p in n for p in CTX_PARTS):
                worst_ctx = max(worst_ctx, r)
            elif r > worst:
                worst, rep["worst"] = r, n
        rep["param"], rep["param_ctx"] = worst, worst_ctx
    dist.barrier()
    return rep


@pytest.mark.parametrize("model_type,seq_len", [("t2v", 240), ("t2v", 256), ("i2v", 256)])
def test_sp_whole_model_two_ranks_one_gpu(model_type, seq_len):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 35700 + (os.getpid() * 3 + seq_len + len(model_type)) % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, model_type, seq_len, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(res[r], str), res[r]
    rep = res[0]
    print(f"SP 2 whole model ({model_type}, seq_len {seq_len}): {rep}")
    assert rep["size"] == 2 and rep["n_param"] > 40
    # per head the attention sees the same keys; the rank partition changes only the order of
    # the cross-rank gradient sums here (no split-KV tail at this size).  Measured: output,
    # features and dx bit-identical, parameters <= 4.7e-7, context side <= 6.1e-3
    # (profiles/r06_gputest_sp_model.log)
    assert rep["out"] < 1e-5 and rep["feat"] < 1e-5 and rep["dx"] < 1e-5, rep
    assert rep["param"] < 1e-5, rep
    assert rep["param_ctx"] < 2e-2, rep
    for p in procs:
        assert p.exitcode == 0
