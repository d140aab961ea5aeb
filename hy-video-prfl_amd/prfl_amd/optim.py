"""Optimizer-side pieces of the PRFL step on the HIP kernels.

* ``AdamW``           — torch.optim.AdamW semantics (`train_prfl.py:479-491`: lr 5e-6, betas
                        (0.9, 0.999), eps 1e-8, weight decay 0.01), fp32 state, one HBM-bound
                        kernel per parameter tensor (prfl_adamw).
    ``state_on_host`` keeps exp_avg / exp_avg_sq (8 B/param, 114 GB for the 14B DiT) in pinned
                      host memory and streams them through a small HBM ring: the memory plan that
                      fits 720p x 81f on one 288 GB GPU.  Both directions share ONE
                      copy stream: the host link moves 57 GB/s one way at a time but only
                      ~37 GB/s in total when H2D and D2H run concurrently (profiles/r01_pcie.txt).
                      A fraction f in (0, 1) streams only the moments of the LAST tensors in
                      update order (attach(): the last blocks a forward reads) covering f of the
                      parameters and keeps the rest in HBM: the 480p plan (C3), where the whole
                      stream (~4 s of PCIe per update) does not hide under a 480p rollout but a
                      fifth of it does, and frees 23 GB of HBM.
    ``overlap``       the update runs on a side stream and step() returns without making the
                      caller's stream wait.  Every parameter gets a ready event; ``attach(model)``
                      installs forward pre-hooks so the first forward that reads a parameter
                      (block by block) waits for exactly that parameter's update.  The streamed
                      update of block i thus runs under the forwards of blocks < i (the SFT
                      step's update hides under the reward step's no-grad rollout).  Results are
                      bit-identical to the synchronous update: same kernel, same inputs, and every
                      reader is ordered after the write.
    ``shard``         (data parallel, world > 1): ZeRO-1 — the tensors are grouped (attach(): the
                      embeddings, each block, the head) and each group, laid end to end, is cut
                      into `world` equal element shards; rank r keeps the moments of, and
                      updates, shard r of every group, then one all_gather_into_tensor per group
                      rebuilds it everywhere (~42 collectives per optimizer step for the 14B DiT
                      instead of one broadcast per tensor); parameters stay bit-identical to the
                      replicated update (AdamW is element-wise).
* ``clip_grad_norm_`` — global L2 norm over all grads and in-place scaling by
                        min(1, max_norm/(norm+1e-6)) (`train_prfl.py:825,972`), with the clip
                        coefficient kept on the device (no host synchronisation).
"""
import weakref

import torch

from . import ops


class AdamW:
    def __init__(self, params, lr=5e-6, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                 state_on_host=False, ring_slots=3, shard=False, overlap=False,
                 shard_bucket_numel=1 << 26):
        self.params = [p for p in params if p.requires_grad]
        self._orig = list(self.params)      # the caller's order: state_dict indices (attach re-sorts)
        self.shard = shard
        self.rank, self.world = 0, 1
        if shard:
            import torch.distributed as dist
            self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.shard_bucket_numel = shard_bucket_numel
        self._groups = None         # ZeRO-1 layout (lazy: attach() may still re-order)
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.state = {}             # param -> (exp_avg, exp_avg_sq) of this rank's range of it
        self.step_count = 0         # optimizer steps taken
        self._pstep = {}            # per-parameter update count (torch's state['step']): the bias
        #                             correction of a parameter that skipped a window lags behind
        self.state_on_host = state_on_host
        self.overlap = overlap
        self.ring_slots = ring_slots
        self.duplex = True          # D2H on its own copy stream (False: both directions on one)
        self._ring = None
        self._streams = None
        self._ready = {}            # param -> event (optimizer stream) after its final write
        self._hooks = []
        # step(zero_grad=True) keeps the gradient buffers (zeroed) where the reference's
        # optimizer.zero_grad() sets them to None.  A parameter whose buffer this optimizer zeroed
        # and that has received no gradient since is skipped, as torch.optim.AdamW skips a None
        # gradient (no weight decay, no moment decay).  "Received" is read off the buffer itself:
        # the zeroed buffer's identity and version counter are recorded, and autograd's in-place
        # accumulation, `p.grad.copy_(...)` or any in-place write bumps the version while
        # `p.grad = g` swaps the object — so gradients from hooks, FSDP / ZeRO code or hand-set
        # ones all count (the zeroing kernel itself writes below the version counter).
        self._zeroed = {}
        self.param_groups = [dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                  params=self.params)]

    def _fresh(self, p):
        z = self._zeroed.get(p)
        if z is None:
            return True
        ref, ver = z
        g = p.grad
        return ref() is not g or g._version != ver

    # ------------------------------------------------------------------ ZeRO-1 layout -----
    def _layout(self):
        """Groups of tensors in update order, each laid out end to end and cut into `world`
        equal element shards: rank r updates (and keeps the moments of) shard r of every group,
        then ONE all_gather_into_tensor per group rebuilds the group on every rank.  Groups are
        attach()'s (embeddings, each block, the head) or, unattached, consecutive tensors of
        >= shard_bucket_numel elements.  AdamW is element-wise, so every element gets exactly the
        update the replicated optimizer computes (same kernel, same per-tensor step count).
        Without sharding: one group of every tensor, all of it this rank's (no collective).

        self._groups = [(tensors, offsets, n, shard)]; self._range[p] = (a, b) (this rank's
        elements of p, absent if none)."""
        if self._groups is not None:
            return self._groups
        if not self.shard:
            lists = [list(self.params)]             # one group: the streamed ring runs end to end
        elif getattr(self, "_group_lists", None) is not None:
            lists = [g for g in self._group_lists if g]
        else:
            lists, cur, n = [], [], 0
            for p in self.params:
                cur.append(p)
                n += p.numel()
                if n >= self.shard_bucket_numel:
                    lists.append(cur)
                    cur, n = [], 0
            if cur:
                lists.append(cur)
        self._groups, self._range = [], {}
        for ts in lists:
            offs, n = [], 0
            for p in ts:
                offs.append(n)
                n += p.numel()
            sz = -(-n // self.world)
            lo, hi = self.rank * sz, min(n, (self.rank + 1) * sz)
            for p, o in zip(ts, offs):
                a, b = max(lo, o) - o, min(hi, o + p.numel()) - o
                if a < b:
                    self._range[p] = (a, b)
            self._groups.append((ts, offs, n, sz))
        return self._groups

    def _host_params(self):
        """The tensors whose moments live on the host: all (state_on_host True), none (False),
        or the shortest tail of self.params (update order) holding >= f of the parameters."""
        hp = getattr(self, "_host_set", None)
        if hp is None:
            f = self.state_on_host
            if f is True or f is False:
                hp = set(self.params) if f else set()
            else:
                f = float(f)
                if not 0.0 < f <= 1.0:
                    raise ValueError(f"state_on_host fraction must be in (0, 1], got {f}")
                need, hp = f * sum(p.numel() for p in self.params), set()
                for p in reversed(self.params):
                    if need <= 0:
                        break
                    hp.add(p)
                    need -= p.numel()
            self._host_set = hp
        return hp

    def _state(self, p):
        st = self.state.get(p)
        if st is None:
            self._layout()
            a, b = self._range[p]
            if p in self._host_params():
                st = (torch.zeros(b - a, dtype=torch.float32, pin_memory=True),
                      torch.zeros(b - a, dtype=torch.float32, pin_memory=True))
            else:
                st = (torch.zeros(b - a, dtype=torch.float32, device=p.device),
                      torch.zeros(b - a, dtype=torch.float32, device=p.device))
            self.state[p] = st
        return st

    def init_state(self):
        """Allocate the moments now (zeros, as torch.optim.AdamW's lazy first step does) instead
        of inside the first step: pinning 114 GB of host memory takes ~10 s, a one-time cost."""
        self._layout()
        for p in self.params:
            if p in self._range:
                self._state(p)

    # ------------------------------------------------------------------ ordering ----------
    def wait(self, params=None):
        """Make the current stream wait for the pending updates of `params` (default: all)."""
        if not self._ready:
            return
        ps = list(self._ready) if params is None else [p for p in params if p in self._ready]
        if not ps:
            return
        cur = torch.cuda.current_stream(ps[0].device)
        for p in ps:
            cur.wait_event(self._ready.pop(p))

    def synchronize(self):
        """All updates visible to the current stream and the host moments complete."""
        self.wait()
        if self._streams is not None:
            for s in self._streams:
                s.synchronize()

    def attach(self, model, groups=None):
        """Forward pre-hooks: each module in `groups` (default: every element of model.blocks,
        then model.head) waits for its own parameters' updates; `model` itself waits for the
        remaining ones (embeddings), which are therefore updated first: the update order becomes
        [rest, groups...] = the order in which a forward first reads them.  These are also the
        ZeRO-1 gather groups (one all-gather each per step)."""
        if groups is None:
            groups = list(model.blocks) + ([model.head] if getattr(model, "head", None) is not None
                                           else [])
        inner = {id(p) for g in groups for p in g.parameters()}
        rest = [p for p in model.parameters() if id(p) not in inner]
        order = {id(p): i for i, p in enumerate(rest + [p for g in groups for p in g.parameters()])}
        self.params.sort(key=lambda p: order.get(id(p), len(order)))
        if self.step_count:
            raise RuntimeError("attach() must precede the first step: the update order decides "
                               "the host-moment tail and the ZeRO-1 shards")
        reinit = bool(self.state)           # zero moments from init_state(): re-placed below
        self.state = {}
        self._host_set = None
        mine = {id(p) for p in self.params}
        lists = [[p for p in rest if id(p) in mine]] + \
            [[p for p in g.parameters() if id(p) in mine] for g in groups]
        placed = {id(p) for ts in lists for p in ts}
        lists.append([p for p in self.params if id(p) not in placed])
        self._group_lists = lists
        self._groups = None
        if reinit:
            self.init_state()
        self._hooks.append(model.register_forward_pre_hook(lambda m, a: self.wait(rest)))
        for g in groups:
            ps = list(g.parameters())
            self._hooks.append(g.register_forward_pre_hook(lambda m, a, ps=ps: self.wait(ps)))
        self._attached = True

    # ------------------------------------------------------------------ update ------------
    @torch.no_grad()
    def step(self, zero_grad=False):
        """One AdamW update of every parameter holding a gradient.  `zero_grad`: the update
        kernel also zeroes each gradient once read (= step() + zero_grad(set_to_none=False) in
        one pass): the gradient buffers stay allocated, so the next backward accumulates into
        them instead of allocating 4 B / parameter again while this update may still be reading
        the old ones on the side stream (which made the caching allocator reserve a second set)."""
        live = [p for p in self.params if p.grad is not None and self._fresh(p)]
        if (live and live[0].is_cuda and self.overlap and zero_grad
                and not getattr(self, "_attached", False)):
            # the next backward accumulates into buffers this update zeroes on the side stream:
            # only the forward pre-hooks of attach() order that write after the zeroing.  Checked
            # before any counter moves, so a caller may attach() and call step() again.
            raise RuntimeError("AdamW(overlap=True).step(zero_grad=True) needs attach(model) first")
        self.step_count += 1
        lr = self.param_groups[0]["lr"]
        for p in live:
            self._pstep[p] = self._pstep.get(p, 0) + 1
        self._step_live(live, lr, zero_grad)
        for p in live:                              # after every in-place write of this step
            if zero_grad:
                self._zeroed[p] = (weakref.ref(p.grad), p.grad._version)
            else:
                self._zeroed.pop(p, None)

    def _step_live(self, live, lr, zero_grad):
        if not live:
            return
        groups = self._layout()
        is_live = set(live)
        cuda = live[0].is_cuda
        if cuda:
            dev = live[0].device
            main = torch.cuda.current_stream(dev)
            if self._streams is None:
                self._streams = tuple(torch.cuda.Stream(device=dev) for _ in range(3))
            opt, cp, dn = self._streams
            self.wait(live)                         # a previous step still in flight
            opt.wait_stream(main)                   # grads (clipped) and params are final
        host = self._host_params()
        for ts, offs, n, sz in groups:
            glive = [p for p in ts if p in is_live]
            if not glive:
                continue
            units = [(p,) + self._range[p] for p in glive if p in self._range]
            if not cuda:                            # CPU (gloo tests): plain synchronous update
                self._update_cpu(units, lr)
                if zero_grad:
                    for p in glive:
                        p.grad.zero_()
                self._gather(ts, offs, n, sz, is_live)
                continue
            with torch.cuda.stream(opt):
                if zero_grad and self.shard:        # the elements another rank updates
                    for p in glive:
                        a, b = self._range.get(p, (0, 0))
                        g = p.grad.view(-1)
                        if a > 0:
                            g[:a].zero_()
                        if b < g.numel():
                            g[b:].zero_()
                # device-resident moments first, then the streamed ones: their first H2D copies
                # start on `cp` at once, beside the device updates
                done = self._update_device([u for u in units if u[0] not in host], lr, zero_grad)
                done.update(self._update_streamed([u for u in units if u[0] in host], lr, opt, cp,
                                                  dn if self.duplex else cp, zero_grad))
                if self.shard:
                    for p in glive:
                        if p in done:
                            opt.wait_event(done[p])
                    self._gather(ts, offs, n, sz, is_live)
                    ev = torch.cuda.Event()
                    ev.record(opt)
                    for p in glive:
                        self._ready[p] = ev
                else:
                    self._ready.update(done)
        if cuda:
            for p in live:                          # grads are read on the side stream
                p.grad.record_stream(opt)
            if not self.overlap:
                self.wait(live)

    def _gather(self, ts, offs, n, sz, is_live):
        """ZeRO-1: this rank's updated shard of the group -> every rank (one collective)."""
        if not self.shard:
            return
        import torch.distributed as dist
        dev = ts[0].device
        lo = self.rank * sz
        shard = torch.empty(sz, dtype=torch.float32, device=dev)
        for p, o in zip(ts, offs):
            r = self._range.get(p)
            if r is not None and p in is_live:      # (other slots: not read back below)
                shard[o + r[0] - lo:o + r[1] - lo].copy_(p.data.view(-1)[r[0]:r[1]])
        full = torch.empty(sz * self.world, dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(full, shard, async_op=True).wait()
        for p, o in zip(ts, offs):
            if p in is_live:
                p.data.view(-1).copy_(full[o:o + p.numel()])

    @staticmethod
    def _flat(t, a, b):
        return t.view(-1)[a:b]

    def _update_device(self, units, lr, zero_grad=False):
        done = {}
        for p, a, b in units:
            m, v = self._state(p)
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            ops.adamw_(self._flat(p.data, a, b), self._flat(g, a, b), m, v, lr, self.betas[0],
                       self.betas[1], self.eps, self.weight_decay, self._pstep[p],
                       zero_grad=zero_grad)
            if zero_grad and g is not p.grad:
                p.grad.zero_()
            ev = torch.cuda.Event()
            ev.record()
            done[p] = ev
        return done

    def _update_streamed(self, units, lr, opt, cp, dn, zero_grad=False):
        """Moments host -> ring -> kernel -> host with the two directions on two copy streams, so
        PCIe carries both at once (full duplex): `cp` H2D(0..k-1), then H2D(i+k) into the slot
        once D2H(i) on `dn` has drained it; `dn` D2H(i) after kernel(i) on `opt`.  (One stream for
        both directions ran them in turn: the last update of a run, which nothing hides, moved
        its moments at one direction's rate.)"""
        done = {}
        if not units:
            return done
        dev = units[0][0].device
        nmax = max(b - a for _, a, b in units)
        k = self.ring_slots
        if self._ring is None or self._ring[0].numel() < 2 * nmax:
            self._ring = [torch.empty(2 * nmax, dtype=torch.float32, device=dev) for _ in range(k)]
            for buf in self._ring:
                buf.record_stream(cp)
                buf.record_stream(dn)
        cap = self._ring[0].numel() // 2
        slots = [(buf[:cap], buf[cap:2 * cap]) for buf in self._ring]
        h2d_ev, d2h_ev = [None] * len(units), [None] * len(units)
        # the ring and the host moments are reused across steps and groups: every earlier D2H
        # (slot drained, host copy written) precedes this call's first H2D
        cp.wait_stream(dn)

        def h2d(i):
            p, a, b = units[i]
            m_h, v_h = self._state(p)
            m_d, v_d = slots[i % k]
            n = b - a
            with torch.cuda.stream(cp):
                if i >= k:
                    cp.wait_event(d2h_ev[i - k])
                m_d[:n].copy_(m_h, non_blocking=True)
                v_d[:n].copy_(v_h, non_blocking=True)
                h2d_ev[i] = torch.cuda.Event()
                h2d_ev[i].record(cp)

        for i in range(min(k, len(units))):
            h2d(i)
        for i, (p, a, b) in enumerate(units):
            n = b - a
            m_d, v_d = slots[i % k]
            opt.wait_event(h2d_ev[i])
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            ops.adamw_(self._flat(p.data, a, b), self._flat(g, a, b), m_d[:n], v_d[:n], lr,
                       self.betas[0], self.betas[1], self.eps, self.weight_decay, self._pstep[p],
                       zero_grad=zero_grad)
            if zero_grad and g is not p.grad:
                p.grad.zero_()
            ev = torch.cuda.Event()
            ev.record(opt)
            done[p] = ev
            m_h, v_h = self._state(p)
            with torch.cuda.stream(dn):
                dn.wait_event(ev)
                m_h.copy_(m_d[:n], non_blocking=True)
                v_h.copy_(v_d[:n], non_blocking=True)
                d2h_ev[i] = torch.cuda.Event()
                d2h_ev[i].record(dn)
            if i + k < len(units):
                h2d(i + k)
        return done

    def _update_cpu(self, units, lr):
        for p, a, b in units:
            m, v = self._state(p)
            ops.adamw_(self._flat(p.data, a, b), self._flat(p.grad, a, b), m, v, lr, self.betas[0],
                       self.betas[1], self.eps, self.weight_decay, self._pstep[p])

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None
        self._zeroed = {}

    def state_bytes(self):
        return sum(2 * m.numel() * 4 for m, _ in self.state.values())

    def state_dict(self):
        """torch.optim.AdamW's layout: per-parameter {"step", "exp_avg", "exp_avg_sq"} keyed by
        the index in the CONSTRUCTOR's parameter order (attach() re-sorts the update order, not
        these keys), one param group.  Unsharded every entry is torch-loadable; a ZeRO-1 rank
        holds its element range of some tensors: those entries carry "range" = (a, b) and flat
        moments (this class's load_state_dict reads them on a rank of the same layout)."""
        self.synchronize()
        idx = {id(p): i for i, p in enumerate(self._orig)}
        g = {k: v for k, v in self.param_groups[0].items() if k != "params"}
        g.update(params=list(range(len(self._orig))), amsgrad=False, maximize=False,
                 foreach=None, capturable=False, differentiable=False, fused=None)
        st = {}
        for p, (m, v) in self.state.items():
            a, b = self._range[p]
            whole = (a, b) == (0, p.numel())
            e = {"step": torch.tensor(float(self._pstep.get(p, 0))),
                 "exp_avg": m.view_as(p) if whole else m, "exp_avg_sq": v.view_as(p) if whole else v}
            if not whole:
                e["range"] = (a, b)
            st[idx[id(p)]] = e
        return {"state": st, "param_groups": [g], "prfl_step_count": self.step_count}

    def load_state_dict(self, sd):
        """Inverse of state_dict (also accepts torch.optim.AdamW's): moments copied into this
        optimizer's storage (host-pinned or HBM, as this instance places them)."""
        self.synchronize()
        self._layout()
        for i, e in sd["state"].items():
            p = self._orig[int(i)]
            if p not in self._range:
                continue
            a, b = self._range[p]
            if tuple(e.get("range", (0, p.numel()))) != (a, b):
                raise ValueError(f"state_dict entry {i}: element range {e.get('range')} does not "
                                 f"match this rank's {(a, b)} (different ZeRO-1 layout)")
            m, v = self._state(p)
            m.copy_(e["exp_avg"].reshape(-1))
            v.copy_(e["exp_avg_sq"].reshape(-1))
            self._pstep[p] = int(float(e["step"]))
        self.step_count = int(sd.get("prfl_step_count",
                                     max([self._pstep.get(p, 0) for p in self._orig] + [0])))
        g = sd["param_groups"][0]
        self.param_groups[0].update(lr=g["lr"], betas=tuple(g["betas"]), eps=g["eps"],
                                    weight_decay=g["weight_decay"])
        self.lr, self.betas, self.eps, self.weight_decay = (g["lr"], tuple(g["betas"]), g["eps"],
                                                            g["weight_decay"])


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
