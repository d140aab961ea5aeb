"""Diagnostic (GPU box): the fused UniPC step vs the oracle torch chain on CPU tensors and on GPU
tensors, on the toy PRFL chain's real step inputs (forward outputs and model-output grads)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_model as T  # noqa: E402
from oracle import wan_oracle as O  # noqa: E402
from prfl_amd import ops, custom_ops  # noqa: E402
from prfl_amd.schedulers import FlowUniPCMultistepScheduler  # noqa: E402

cache = {}


def golden(name):
    if name not in cache:
        cache[name] = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz")))
    return cache[name]


calls = []


def spy(mo, sample, last, h1, h2, coef, corr, pred):
    out = custom_ops.unipc_update(mo, sample, last, h1, h2, coef, corr, pred)
    cl = lambda t: None if t is None else t.detach().clone()  # noqa: E731
    calls.append((cl(mo), cl(sample), cl(last), cl(h1), cl(h2), coef, corr, pred,
                  [cl(o) for o in out], mo.requires_grad))
    return out


FlowUniPCMultistepScheduler._update = staticmethod(spy)
T.check_grads = lambda *a, **k: 99
try:
    T.test_toy_prfl_chain_vs_reference(golden)
except AssertionError as e:
    print("assert:", str(e)[:200])
for ci, (mo, s, last, h1, h2, coef, corr, pred, outs, rg) in enumerate(calls):
    print("call", ci, "corr", corr, "pred", pred, "grad", rg, "coef", coef)
    for dev in ("cpu", "cuda"):
        mv = lambda t: None if t is None else t.to(dev)  # noqa: E731
        mo_r = mo.to(dev).detach().clone().requires_grad_(True)
        ref = O.unipc_update(mo_r, mv(s), mv(last), mv(h1), mv(h2), coef, corr, pred)
        d = [(a.float().cpu() - b.detach().float().cpu()).abs().max().item() for a, b in zip(outs, ref)]
        gp = torch.randn(s.shape, generator=torch.Generator().manual_seed(ci)).to(dev)
        (ref[2].float() * gp).sum().backward()
        mo_f = mo.detach().clone().requires_grad_(True)
        o2 = custom_ops.unipc_update(mo_f, s, last, h1, h2, coef, corr, pred)
        (o2[2].float() * gp.cuda()).sum().backward()
        gd = (mo_f.grad.cpu() - mo_r.grad.cpu()).abs().max().item()
        print(f"   vs oracle on {dev}: fwd max|d| m_t {d[0]:.3e} x_c {d[1]:.3e} prev {d[2]:.3e}; "
              f"grad max|d| {gd:.3e} (|g| {mo_r.grad.abs().max().item():.3e})")
