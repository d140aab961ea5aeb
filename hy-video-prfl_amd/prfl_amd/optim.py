"""Optimizer-side pieces of the PRFL step on the HIP kernels.

* ``AdamW``           — torch.optim.AdamW semantics (`train_prfl.py:479-491`: lr 5e-6, betas
                        (0.9, 0.999), eps 1e-8, weight decay 0.01), fp32 state, one HBM-bound
                        kernel per parameter tensor (prfl_adamw).
* ``clip_grad_norm_`` — global L2 norm over all grads and in-place scaling by
                        min(1, max_norm/(norm+1e-6)) (`train_prfl.py:825,972`), with the clip
                        coefficient kept on the device (no host synchronisation).
"""
import torch

from . import ops


class AdamW:
    def __init__(self, params, lr=5e-6, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01):
        self.params = [p for p in params if p.requires_grad]
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.state = {}
        self.step_count = 0
        self.param_groups = [dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                  params=self.params)]

    @torch.no_grad()
    def step(self):
        self.step_count += 1
        lr = self.param_groups[0]["lr"]
        for p in self.params:
            if p.grad is None:
                continue
            st = self.state.get(p)
            if st is None:
                st = self.state[p] = (torch.zeros_like(p), torch.zeros_like(p))
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            ops.adamw_(p.data, g, st[0], st[1], lr, self.betas[0], self.betas[1], self.eps,
                       self.weight_decay, self.step_count)

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def state_bytes(self):
        return sum(2 * p.numel() * 4 for p in self.state)


@torch.no_grad()
def clip_grad_norm_(params, max_norm=1.0, eps=1e-6):
    """Returns the pre-clip total norm as a 0-dim device tensor (no host sync)."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return torch.zeros(())
    dev = grads[0].device
    ss = torch.zeros(1, dtype=torch.float32, device=dev)
    for g in grads:
        ops.sumsq_(g if g.is_contiguous() else g.contiguous(), ss)
    total = ss.sqrt()
    coef = torch.clamp(max_norm / (total + eps), max=1.0)
    for g in grads:
        ops.scale_(g, coef)
    return total[0]
