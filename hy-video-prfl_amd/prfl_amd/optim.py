"""Optimizer-side pieces of the PRFL step on the HIP kernels.

* ``AdamW``           — torch.optim.AdamW semantics (`train_prfl.py:479-491`: lr 5e-6, betas
                        (0.9, 0.999), eps 1e-8, weight decay 0.01), fp32 state, one HBM-bound
                        kernel per parameter tensor (prfl_adamw).  ``state_on_host=True`` keeps
                        exp_avg / exp_avg_sq (8 B/param, 114 GB for the 14B DiT) in pinned host
                        memory and streams them through a 3-slot HBM ring on two copy streams
                        (H2D of tensor i+1 and D2H of tensor i-1 overlap the kernel on tensor i):
                        the memory plan that fits 720p x 81f on one 288 GB GPU.
                        ``shard=True`` (data parallel, world > 1): ZeRO-1 — every rank keeps the
                        moments of, and updates, only the tensors it owns (size-balanced, the same
                        assignment on every rank), then each tensor is broadcast from its owner;
                        parameters stay bit-identical to the replicated update.
* ``clip_grad_norm_`` — global L2 norm over all grads and in-place scaling by
                        min(1, max_norm/(norm+1e-6)) (`train_prfl.py:825,972`), with the clip
                        coefficient kept on the device (no host synchronisation).
"""
import torch

from . import ops


class AdamW:
    def __init__(self, params, lr=5e-6, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                 state_on_host=False, ring_slots=3, shard=False):
        self.params = [p for p in params if p.requires_grad]
        self.shard = shard
        if shard:
            import torch.distributed as dist
            self.rank, self.world = dist.get_rank(), dist.get_world_size()
            loads = [0] * self.world
            self.owner = {}
            order = sorted(range(len(self.params)), key=lambda i: (-self.params[i].numel(), i))
            for i in order:
                r = min(range(self.world), key=lambda k: (loads[k], k))
                self.owner[self.params[i]] = r
                loads[r] += self.params[i].numel()
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.state = {}
        self.step_count = 0
        self.state_on_host = state_on_host
        self.ring_slots = ring_slots
        self._ring = None
        self.param_groups = [dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                  params=self.params)]

    def _state(self, p):
        st = self.state.get(p)
        if st is None:
            if self.state_on_host:
                st = (torch.zeros(p.numel(), dtype=torch.float32, pin_memory=True),
                      torch.zeros(p.numel(), dtype=torch.float32, pin_memory=True))
            else:
                st = (torch.zeros_like(p), torch.zeros_like(p))
            self.state[p] = st
        return st

    @torch.no_grad()
    def step(self):
        self.step_count += 1
        lr = self.param_groups[0]["lr"]
        live = [p for p in self.params if p.grad is not None]
        if self.shard:
            import torch.distributed as dist
            self._update([p for p in live if self.owner[p] == self.rank], lr)
            for p in live:
                dist.broadcast(p.data, src=self.owner[p])
            return
        self._update(live, lr)

    def _update(self, live, lr):
        if self.state_on_host:
            return self._step_streamed(live, lr)
        for p in live:
            m, v = self._state(p)
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            ops.adamw_(p.data, g, m, v, lr, self.betas[0], self.betas[1], self.eps,
                       self.weight_decay, self.step_count)

    def _step_streamed(self, live, lr):
        if not live:
            return
        dev = live[0].device
        nmax = max(p.numel() for p in live)
        if self._ring is None or self._ring[0].numel() < 2 * nmax:
            k = self.ring_slots
            self._ring = [torch.empty(2 * nmax, dtype=torch.float32, device=dev) for _ in range(k)]
            self._h2d = torch.cuda.Stream(device=dev)
            self._d2h = torch.cuda.Stream(device=dev)
            self._ev = [[torch.cuda.Event() for _ in range(3)] for _ in range(k)]  # h2d, kernel, d2h
            self._used = [False] * k
        main = torch.cuda.current_stream(dev)
        k = self.ring_slots
        for i, p in enumerate(live):
            j = i % k
            n = p.numel()
            m_h, v_h = self._state(p)
            buf = self._ring[j]
            m_d, v_d = buf[:n], buf[nmax:nmax + n]
            ev_h2d, ev_k, ev_d2h = self._ev[j]
            with torch.cuda.stream(self._h2d):
                if self._used[j]:
                    self._h2d.wait_event(ev_d2h)          # slot's previous tensor written back
                m_d.copy_(m_h, non_blocking=True)
                v_d.copy_(v_h, non_blocking=True)
                ev_h2d.record(self._h2d)
            main.wait_event(ev_h2d)
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            ops.adamw_(p.data, g, m_d.view_as(p), v_d.view_as(p), lr, self.betas[0], self.betas[1],
                       self.eps, self.weight_decay, self.step_count)
            ev_k.record(main)
            with torch.cuda.stream(self._d2h):
                self._d2h.wait_event(ev_k)
                m_h.copy_(m_d, non_blocking=True)
                v_h.copy_(v_d, non_blocking=True)
                ev_d2h.record(self._d2h)
            self._used[j] = True
        # the host state must be complete before anyone reads it; the ring before it is reused
        main.wait_stream(self._d2h)

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def state_bytes(self):
        return sum(2 * p.numel() * 4 for p in self.state)

    def state_dict(self):
        """Moments of the tensors this rank holds (host or device), by parameter index."""
        idx = {id(p): i for i, p in enumerate(self.params)}
        return {"step": self.step_count,
                "state": {idx[id(p)]: {"exp_avg": m.view_as(p), "exp_avg_sq": v.view_as(p)}
                          for p, (m, v) in self.state.items()}}


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
