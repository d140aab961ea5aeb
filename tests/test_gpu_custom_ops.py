"""The `prfl::` custom ops on the MI355X: torch.library.opcheck (schema, autograd registration,
fake tensors), the fused block under torch.utils.checkpoint and under the reference's FSDP
wrap + apply_fsdp_checkpointing (`train_prfl.py:346-374`, `fsdp_utils.py:23-122`), and the
single-query pooling kernel (`network.py:80`) against an fp32 reference."""
import math
import os
import socket

import pytest
import torch

from oracle import wan_oracle as O
from shapes import TOY, block_shapes, model_shapes, seeded_params

pytestmark = pytest.mark.gpu
DEV = "cuda"
OPCHECK = ("test_schema", "test_autograd_registration", "test_faketensor")


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu().flatten()
    b = torch.as_tensor(b).detach().double().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def cops():
    from prfl_amd import custom_ops
    return custom_ops


def _block_inputs(L=105, dim=256, req=True, prefix="cop."):
    from prfl_amd import block as B
    from prfl_amd import ops
    P = seeded_params(block_shapes("blocks.0.", dim, 2 * dim, False), prefix=prefix)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, L, dim, generator=g).to(DEV).requires_grad_(req)
    e = (torch.randn(1, 6, dim, generator=g) * 0.1 + P["blocks.0.modulation"]).to(DEV)
    ctx = torch.randn(1, 512, dim, generator=g).to(torch.bfloat16).to(DEV)
    params = [P["blocks.0." + n].to(DEV).requires_grad_(req) for n in B.param_names(False)]
    tab = ops.rope_table(O.rope_freqs(128), DEV)
    return x, e, ctx, params, tab


def test_opcheck_linear_and_attention(cops):
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(37, 64, generator=g, device=DEV, requires_grad=True)
    w = torch.randn(24, 64, generator=g, device=DEV, requires_grad=True)
    b = torch.randn(24, generator=g, device=DEV, requires_grad=True)
    for gelu in (False, True):
        torch.library.opcheck(torch.ops.prfl.linear_bf16.default, (x, w, b, gelu), test_utils=OPCHECK)
    q = torch.randn(1, 70, 2, 128, generator=g, device=DEV, requires_grad=True)
    k = torch.randn(1, 90, 2, 128, generator=g, device=DEV, requires_grad=True)
    v = torch.randn(1, 90, 2, 128, generator=g, device=DEV, requires_grad=True)
    torch.library.opcheck(torch.ops.prfl.flash_attention.default, (q, k, v, [61], 0.088),
                          test_utils=OPCHECK)
    qp = torch.randn(2, 256, generator=g, device=DEV).to(torch.bfloat16).requires_grad_(True)
    kv = torch.randn(2, 77, 512, generator=g, device=DEV).to(torch.bfloat16).requires_grad_(True)
    torch.library.opcheck(torch.ops.prfl.query_pool.default, (qp, kv, 8, 32 ** -0.5),
                          test_utils=OPCHECK)


def test_opcheck_wan_block(cops):
    x, e, ctx, params, tab = _block_inputs()
    for keep in (False, True):
        torch.library.opcheck(torch.ops.prfl.wan_block.default,
                              (x, e, ctx, params, 2, [3, 5, 7], [105], tab, False, 1e-6, 0, keep),
                              test_utils=OPCHECK)


def test_block_under_torch_checkpoint_is_bit_identical(cops):
    """The fused block wrapped in torch.utils.checkpoint (non-reentrant, the wrapper
    apply_fsdp_checkpointing installs) recomputes through the op and gives the same output and
    gradients, bit for bit, as the block alone."""
    from prfl_amd import block as B
    from torch.utils.checkpoint import checkpoint
    res = []
    for wrap in (False, True):
        x, e, ctx, params, tab = _block_inputs()
        names = B.param_names(False)
        meta = B.Meta(2, [(3, 5, 7)], [105], tab, False)
        P = dict(zip(names, params))
        f = lambda xx: B.block_apply(P, xx, e, ctx, meta)  # noqa: E731
        out = checkpoint(f, x, use_reentrant=False) if wrap else f(x)
        (out * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
        res.append([out.detach(), x.grad] + [p.grad for p in params])
    assert all(torch.equal(a, b) for a, b in zip(*res))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("wrap_fused", [False, True])
def test_fsdp_wrap_and_checkpointing_compose(wrap_fused):
    """The reference's model_init path on a toy WanModel: FSDP(FULL_SHARD, fp32 MixedPrecision,
    auto-wrap on WanAttentionBlock, use_orig_params False) + apply_fsdp_checkpointing, world size
    1 over RCCL (FSDP then runs NO_SHARD, still on flat parameters whose views feed the fused
    blocks), autocast bf16 forward, backward, transformer.clip_grad_norm_ — against the same
    model unwrapped."""
    import torch.distributed as dist
    from torch.distributed.fsdp import FullyShardedDataParallel as FSDP
    from prfl_amd.fsdp_utils import apply_fsdp_checkpointing, get_dit_fsdp_kwargs
    from prfl_amd.model import WanModel
    created = not dist.is_initialized()
    if created:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                                world_size=1, device_id=torch.device(DEV, 0))
    try:
        sd = seeded_params(model_shapes(TOY, "t2v"), prefix="toy.")
        ref = WanModel(model_type="t2v", in_dim=16, **TOY)
        ref.load_state_dict(sd)
        ref = ref.to(DEV)
        m = WanModel(model_type="t2v", in_dim=16, **TOY)
        m.load_state_dict(sd)
        kw, ns = get_dit_fsdp_kwargs(m, "full")
        m = FSDP(m, **kw)
        apply_fsdp_checkpointing(m, ns, 1.0, wrap_fused=wrap_fused)
        g = torch.Generator().manual_seed(4)
        x = torch.randn(16, 3, 10, 14, generator=g).to(DEV)
        ctx = torch.randn(20, 64, generator=g).to(DEV)
        t = torch.tensor([700], device=DEV)
        up = torch.randn(16, 3, 10, 14, generator=g).to(DEV)
        outs = []
        for model in (ref, m):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(x=[x], t=t, context=[ctx], seq_len=105)[0]
            (out * up).sum().backward()
            outs.append(out.detach())
        assert torch.equal(outs[0], outs[1])
        gn = m.clip_grad_norm_(max_norm=1e9)
        gn_ref = torch.nn.utils.clip_grad_norm_(ref.parameters(), max_norm=1e9)
        assert abs(gn.item() / gn_ref.item() - 1) < 1e-5
        # the gradients reach FSDP's flat parameters: one SGD step (lr 1: p - g, exact in fp32)
        # on both models, then compare the un-flattened parameters
        # (summon_full_params(with_grads=True) is unsupported with use_orig_params=False)
        for model in (ref, m):
            torch.optim.SGD(model.parameters(), lr=1.0).step()
        with FSDP.summon_full_params(m):
            got = {n.replace("_fsdp_wrapped_module.", "").replace("_checkpoint_wrapped_module.", ""): p
                   for n, p in m.named_parameters()}
            n_cmp = 0
            for n, p in ref.named_parameters():
                if p.grad is None:
                    continue
                assert torch.equal(got[n], p), n
                n_cmp += 1
            assert n_cmp > 30
    finally:
        if created:
            dist.destroy_process_group()


def _pool_ref(q, kv, H, scale):
    """fp32 restatement of the reference pooling under flash numerics (network.py:80):
    P rounded to bf16 for P.V, fp32 normaliser, bf16 output."""
    N, E = q.shape
    hd = E // H
    k = kv[:, :, :E].float().view(N, -1, H, hd)
    v = kv[:, :, E:].float().view(N, -1, H, hd)
    s = torch.einsum("nhd,nlhd->nhl", q.float().view(N, H, hd), k) * scale
    m = s.amax(-1, keepdim=True)
    p = torch.exp(s - m)
    l = p.sum(-1, keepdim=True)
    o = torch.einsum("nhl,nlhd->nhd", p.to(torch.bfloat16).float(), v) / l
    return o.reshape(N, E).to(torch.bfloat16), ((m + l.log()) / math.log(2)).squeeze(-1)


@pytest.mark.parametrize("N,L,E,H", [(1, 48, 5120, 8), (2, 4133, 5120, 8), (1, 73920, 5120, 8),
                                     (3, 105, 256, 8)])
def test_query_pool_vs_reference(cops, N, L, E, H):
    """prfl::query_pool forward (o, LSE) and backward (dq, dk, dv) vs an fp32 GPU restatement with
    autograd; the backward reference differentiates the same math (FA2: D from the bf16 O)."""
    g = torch.Generator(device=DEV).manual_seed(L + E)
    q = torch.randn(N, E, generator=g, device=DEV).to(torch.bfloat16)
    kv = torch.randn(N, L, 2 * E, generator=g, device=DEV).to(torch.bfloat16)
    do = torch.randn(N, E, generator=g, device=DEV).to(torch.bfloat16)
    scale = (E // H) ** -0.5
    o, lse, _ = cops.query_pool(q, kv, H, scale)
    ro, rlse = _pool_ref(q, kv, H, scale)
    assert rel(o, ro) < 5e-3 and (lse - rlse).abs().max().item() < 1e-3
    qr = q.float().requires_grad_(True)
    kvr = kv.float().requires_grad_(True)
    hd = E // H
    s = torch.einsum("nhd,nlhd->nhl", qr.view(N, H, hd), kvr[:, :, :E].view(N, L, H, hd)) * scale
    p = torch.softmax(s, -1)
    out = torch.einsum("nhl,nlhd->nhd", p, kvr[:, :, E:].view(N, L, H, hd)).reshape(N, E)
    out.backward(do.float())
    qg = q.clone().requires_grad_(True)
    kvg = kv.clone().requires_grad_(True)
    o2, _, _ = cops.query_pool(qg, kvg, H, scale)
    o2.backward(do)
    assert torch.equal(o2, o)
    assert rel(qg.grad, qr.grad) < 2e-2
    assert rel(kvg.grad[:, :, :E], kvr.grad[:, :, :E]) < 2e-2
    assert rel(kvg.grad[:, :, E:], kvr.grad[:, :, E:]) < 2e-2


def test_train_model_on_the_reward_mlp():
    """network.train_model on this package's reward MLP (bf16 GEMMs on the HIP op): the scores
    reach BCELoss in fp32 (the reference's fp32 nn.Linear MLP gives fp32), and it trains."""
    from prfl_amd.network import MLP, _scores, train_model
    torch.manual_seed(0)
    X = torch.randn(512, 64, device=DEV)
    y = (X[:, :1] > 0).float()
    m = MLP(64).to(DEV)
    assert _scores(m, "clf", X).dtype == torch.float32
    bce = torch.nn.functional.binary_cross_entropy
    before = bce(_scores(m, "clf", X), y).item()
    train_model(m, DEV, "clf", X, y, X, y, epochs=30, lr=3e-3, batch_size=128)
    after = bce(_scores(m, "clf", X), y).item()
    assert after < 0.7 * before, (before, after)
