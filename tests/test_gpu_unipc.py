"""Fused FlowUniPC step (csrc/unipc.hip) on the MI355X vs the reference trajectory fixtures and
the oracle's restatement of the element-wise chain.

Bar: bit-exact.  The kernel performs the reference's fp32 operations in the reference's order
with its bf16 rounding points (tests/golden/schedulers.npz was produced by the reference's own
FlowUniPCMultistepScheduler, fm_solvers_unipc.py:655-739, on the CPU).
"""
import pytest
import torch

from oracle import wan_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _sched():
    from prfl_amd.schedulers import FlowUniPCMultistepScheduler
    sch = FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1, use_dynamic_shifting=False)
    sch.set_timesteps(num_inference_steps=40, device=DEV, shift=5.0)
    return sch


def test_unipc_fused_trajectory_bit_exact(golden):
    g = golden("schedulers")
    sch = _sched()
    lat = torch.from_numpy(g["unipc_lat0"]).to(torch.bfloat16).view(1, 16, 3, 10, 14).to(DEV)
    for i in range(6):
        mo = torch.from_numpy(g["unipc_model_outputs"][i]).to(DEV)
        lat = sch.step(mo, sch.timesteps[i], lat, return_dict=False)[0]
        assert lat.dtype == torch.bfloat16 and lat.is_cuda
        assert torch.equal(lat.float().cpu(), torch.from_numpy(g["unipc_traj"][i])), i
    mo = torch.from_numpy(g["unipc_mo6"]).to(DEV).requires_grad_(True)
    prev = sch.step(mo, sch.timesteps[6], lat, return_dict=False)[0]
    assert torch.equal(prev.float().detach().cpu(), torch.from_numpy(g["unipc_prev6"]))
    (prev.float() * torch.from_numpy(g["unipc_w"]).to(DEV)).sum().backward()
    ref = torch.from_numpy(g["unipc_dmo6"])
    # the backward kernel replays torch autograd's op order and casts: bit-exact as well
    assert torch.equal(mo.grad.cpu(), ref), (mo.grad.cpu() - ref).abs().max()


@pytest.mark.parametrize("n", [7, 4096 + 3, 16 * 21 * 88 * 160])
def test_unipc_fused_vs_oracle_all_orders(n):
    """Every (corrector, predictor) order combination, ragged and full 720p latent sizes, against
    the oracle's torch chain on the CPU (forward and autograd backward): bit-exact."""
    from prfl_amd import custom_ops
    gen = torch.Generator().manual_seed(n)
    sample = torch.randn(n, generator=gen).to(torch.bfloat16)
    last = torch.randn(n, generator=gen).to(torch.bfloat16)
    mo = torch.randn(n, generator=gen)
    h1 = torch.randn(n, generator=gen)
    h2 = torch.randn(n, generator=gen)
    gp = torch.randn(n, generator=gen)
    coef = [0.83, 0.97, -0.11, 0.71, float(torch.tensor(0.62).bfloat16()),
            float(torch.tensor(0.47).bfloat16()), -0.09, 0.95, -0.13, 0.66, -0.12]
    for corr in (0, 1, 2):
        for pred in (1, 2):
            mo_c = mo.clone().requires_grad_(True)
            m_r, x_r, p_r = O.unipc_update(mo_c, sample, last if corr else None,
                                           h1, h2 if corr == 2 else None, coef, corr, pred)
            (p_r.float() * gp).sum().backward()
            mo_g = mo.to(DEV).requires_grad_(True)
            m_g, x_g, p_g = custom_ops.unipc_update(mo_g, sample.to(DEV), last.to(DEV) if corr else None,
                                           h1.to(DEV), h2.to(DEV) if corr == 2 else None, coef,
                                           corr, pred)
            (p_g.float() * gp.to(DEV)).sum().backward()
            assert torch.equal(m_g.detach().cpu(), m_r.detach()), (corr, pred)
            assert torch.equal(x_g.cpu(), x_r.detach()), (corr, pred)
            assert torch.equal(p_g.detach().cpu(), p_r.detach()), (corr, pred)
            d = (mo_g.grad.cpu() - mo_c.grad).abs().max().item()
            assert torch.equal(mo_g.grad.cpu(), mo_c.grad), (corr, pred, d)


def test_unipc_fused_rejects_bad_inputs():
    from prfl_amd import custom_ops
    s = torch.zeros(64, dtype=torch.bfloat16, device=DEV)
    mo = torch.zeros(64, device=DEV)
    with pytest.raises(NotImplementedError):
        custom_ops.unipc_update(mo.bfloat16(), s, None, None, None, [0.0] * 11, 0, 1)
    with pytest.raises(RuntimeError):
        custom_ops.unipc_update(mo, s, None, None, None, [0.0] * 11, 0, 2)   # order 2 needs history
    with pytest.raises(NotImplementedError):
        custom_ops.unipc_update(mo, s.float().requires_grad_(True).bfloat16(), None, None, None,
                       [0.0] * 11, 0, 1)
