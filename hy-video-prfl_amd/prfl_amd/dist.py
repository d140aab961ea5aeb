"""Data-parallel gradient exchange for the PRFL step (replaces FSDP FULL_SHARD + Ulysses SP of
`fsdp_utils.py:66-122` / `communication.py:40-160` with pure batch DP over RCCL/xGMI).

Every rank holds a full replica of the weights.
The reference reduces the FRESH gradient of every backward (FSDP reduce-scatters each micro-step,
no `no_sync`) and accumulates the reduced gradient.  Because the accumulated part is already
identical on every rank, avg_r(acc + fresh_r) = acc + avg_r(fresh_r): `GradReducer` lets autograd
accumulate in place into .grad and all-reduces the sum, which needs no second gradient buffer
(57 GB for the 14B DiT in fp32 - what makes the 720p step fit):

  during backward : a post-accumulate-grad hook fires per parameter as soon as its block's fused
                    backward node returns (reverse layer order) and launches an async all-reduce
                    on RCCL's stream -> communication overlaps the remaining blocks' backward
  after backward  : wait; average (gloo has no AVG)

Block gradients are 105-283 MB tensors, well past the point where a ring all-reduce is
bandwidth-bound on xGMI, so tensors are reduced individually (no flatten/copy buckets); the
small 1-D tensors (biases, norm weights) of a block are coalesced into one flat reduce.
"""
import torch
import torch.distributed as dist


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


class GradReducer:
    def __init__(self, params, small_numel=1 << 16, min_world=2):
        # min_world=1 hooks a one-rank process group too (exercises the exchange end to end on
        # a single device: the RCCL AVG over one rank is exact)
        self.params = [p for p in params if p.requires_grad]
        on = dist.is_available() and dist.is_initialized() and dist.get_world_size() >= min_world
        self.world = dist.get_world_size() if on else 1
        self.active = on
        self.small_numel = small_numel
        self.works = []
        self.small_pending = []
        self.backend = dist.get_backend() if on else None
        self.handles = []
        self.time_tail = False      # bench.py: HIP-event time of the exposed all-reduce tail
        self.tail_ms = []
        self._tail_ev = []
        if on:
            for p in self.params:
                self.handles.append(p.register_post_accumulate_grad_hook(self._hook))

    def _op(self):
        return dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM

    def _hook(self, p):
        if p.numel() <= self.small_numel:
            self.small_pending.append(p)
            if sum(q.numel() for q in self.small_pending) >= 8 * self.small_numel:
                self._flush_small()
            return
        self.works.append((dist.all_reduce(p.grad, op=self._op(), async_op=True), [p.grad]))

    def _flush_small(self):
        if not self.small_pending:
            return
        ps, self.small_pending = self.small_pending, []
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        w = dist.all_reduce(flat, op=self._op(), async_op=True)
        self.works.append((w, (flat, ps)))

    def begin(self):
        """Call before loss.backward() (kept for the driver's call pattern; nothing to stash)."""
        self.works = []

    def end(self):
        """Call after loss.backward(): completes the exchange."""
        ev0 = None
        if self.active and self.time_tail and torch.cuda.is_available():
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()                 # the backward's last kernel on the compute stream
        if self.active:
            self._flush_small()
            for w, payload in self.works:
                w.wait()
                if isinstance(payload, tuple):
                    flat, ps = payload
                    if self.backend != "nccl":
                        flat.div_(self.world)
                    off = 0
                    for p in ps:
                        n = p.numel()
                        p.grad.copy_(flat[off:off + n].view_as(p.grad))
                        off += n
                elif self.backend != "nccl":
                    payload[0].div_(self.world)
            self.works = []
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()                 # the stream has waited for every reduce of this backward
            self._tail_ev.append((ev0, ev1))

    def collect_tail_ms(self):
        """Exposed all-reduce tail of each timed backward (ms), then reset."""
        out = []
        for a, b in self._tail_ev:
            b.synchronize()
            out.append(a.elapsed_time(b))
        self._tail_ev = []
        self.tail_ms = out
        return out


def broadcast_int(v, src=0, device="cpu"):
    """`train_prfl.py:640-652`: rank 0 draws mid_timestep, every rank uses it."""
    if not is_dist():
        return int(v)
    t = torch.tensor([int(v)], dtype=torch.long, device=device)
    dist.broadcast(t, src=src)
    return int(t.item())


def all_reduce_max(t):
    if not is_dist():
        return t
    t = t.clone()
    dist.all_reduce(t, dist.ReduceOp.MAX)
    return t


def all_reduce_mean(t):
    if not is_dist():
        return t
    t = t.clone()
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, dist.ReduceOp.AVG)
    else:
        dist.all_reduce(t, dist.ReduceOp.SUM)
        t /= dist.get_world_size()
    return t
