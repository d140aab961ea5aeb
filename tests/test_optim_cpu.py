"""AdamW host logic on the CPU (the update kernel replaced by torch's AdamW formula, as in
tests/test_dist_gloo.py): which gradients count after step(zero_grad=True), and the
torch-compatible state_dict."""
import copy

import pytest
import torch

from test_dist_gloo import _adamw_ref


@pytest.fixture
def optim(monkeypatch):
    from prfl_amd import optim as O
    monkeypatch.setattr(O.ops, "adamw_", _adamw_ref)
    return O


@pytest.mark.parametrize("how", ["assign", "copy", "autograd", "untouched"])
def test_zeroed_buffer_counts_any_fresh_gradient(optim, how):
    """After step(zero_grad=True) a gradient that arrives WITHOUT autograd accumulation
    (`p.grad = g`, `p.grad.copy_(g)`, as FSDP / ZeRO code or hand-computed grads do) is applied;
    only a buffer nothing wrote since the zeroing is skipped (torch skips a None gradient)."""
    torch.manual_seed(0)
    p = torch.randn(5, 4, requires_grad=True)
    opt = optim.AdamW([p], lr=1e-2)
    p.grad = torch.randn(5, 4)
    opt.step(zero_grad=True)
    assert torch.count_nonzero(p.grad) == 0
    before = p.detach().clone()
    g = torch.randn(5, 4)
    if how == "assign":
        p.grad = g.clone()
    elif how == "copy":
        p.grad.copy_(g)
    elif how == "autograd":
        (p * g).sum().backward()
    opt.step(zero_grad=True)
    moved = not torch.equal(p.detach(), before)
    assert moved == (how != "untouched"), how
    assert opt._pstep[p] == (2 if how != "untouched" else 1)


def test_state_dict_is_torch_loadable_in_constructor_order(optim):
    """attach() re-sorts the update order; state_dict keys stay the constructor's indices, so a
    torch.optim.AdamW over the same parameter list continues the exact trajectory, and our
    load_state_dict restores an instance whose update order differs."""
    torch.manual_seed(1)

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.head = torch.nn.Linear(4, 3)
            self.blocks = torch.nn.ModuleList([torch.nn.Linear(4, 4) for _ in range(2)])
            self.emb = torch.nn.Linear(6, 4)

    m = M()
    params = list(m.parameters())                      # head first: attach() puts it last
    opt = optim.AdamW(params, lr=1e-2, weight_decay=0.05)
    opt.attach(m)
    assert [id(p) for p in opt.params] != [id(p) for p in params]
    for it in range(3):
        for p in params:
            p.grad = torch.randn(p.shape)
        opt.step()
    sd = opt.state_dict()
    assert sorted(sd["state"]) == list(range(len(params)))
    for i, p in enumerate(params):
        assert sd["state"][i]["exp_avg"].shape == p.shape
    # torch continues from our state
    twin = [p.detach().clone().requires_grad_(True) for p in params]
    topt = torch.optim.AdamW(twin, lr=1e-2, weight_decay=0.05, foreach=False)
    topt.load_state_dict(copy.deepcopy(sd))      # (torch keeps references, as ours hands out)
    # ours, restored into a fresh instance WITHOUT attach (other update order)
    twin2 = [p.detach().clone().requires_grad_(True) for p in params]
    opt2 = optim.AdamW(twin2, lr=1e-3)
    opt2.load_state_dict(sd)
    assert opt2.lr == 1e-2 and opt2.weight_decay == 0.05 and opt2.step_count == 3
    g = torch.Generator().manual_seed(9)
    grads = [torch.randn(p.shape, generator=g) for p in params]
    for ps, o in ((params, opt), (twin, topt), (twin2, opt2)):
        for p, gg in zip(ps, grads):
            p.grad = gg.clone()
        o.step()
    for a, b, c in zip(params, twin, twin2):
        assert torch.allclose(a, b, rtol=0, atol=1e-6)
        assert torch.equal(a.detach(), c.detach())
