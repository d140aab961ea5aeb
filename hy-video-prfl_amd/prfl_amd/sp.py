"""Ulysses sequence parallelism of the drop-in WanModel (the reference's `sp_size > 1` path).

What the reference does when `parallel_states.get_sequence_parallel_state()` is on
(`diffusers_lite/wan/modules/model.py`, `utils/communication.py`):

  * the padded token sequence [B, seq_len, C] is split into `sp_size` equal chunks and each rank
    of the group keeps its own (`model.py:618-619`);
  * RoPE rotates a rank's tokens by their positions in the whole sequence, unit multipliers past
    the video grid (`model.py:89-96`, `pad_freqs` `:45-58`);
  * around self-attention q/k/v go from (tokens of this rank, all heads) to (all tokens, this
    rank's heads) and the output back (`model.py:183-196`, `_all_to_all_4D`
    `communication.py:40-125`); the backward of each all-to-all is the inverse all-to-all
    (`SeqAllToAll4D` `:128-152`);
  * cross-attention, norms, FFN and the head work on the rank's tokens alone;
  * the selected features and the head output are all-gathered along the sequence; the backward
    of that gather keeps the rank's own slice of the gradient (`_AllGather` `:224-260`).

Here the self-attention exchange runs INSIDE the fused block (`block.py`, one `prfl::wan_block`
node): the QKV GEMM and RMSNorm+RoPE (at the rank's row offset, `prfl_rms_rope_fwd_pos`) work on
the rank's s = seq_len / P tokens, ONE all-to-all moves q, k and v together (a [P][s][3][C/P]
send image, so the received buffer is the full-sequence q | k | v of this rank's H/P heads as
row-strided views the attention kernels read in place), the HIP attention runs on H/P heads over
all seq_len keys, and one all-to-all returns the output.  The block's backward does the inverse:
d(out) to heads, the attention backward writes dq | dk | dv into one [S][3][C/P] buffer that is
already the send image of the return all-to-all.

The group comes from (1) `set_group()` of this module (the trainers, the tests) or else (2) the
reference's own `diffusers_lite.utils.parallel_states` module, if the driver has imported it and
initialised SP (`train_prfl.py:118`) — nothing is imported from the reference here.

Collectives are issued on the current stream's order (RCCL over xGMI with backend "nccl"); a
gloo group with device tensors stages them through host memory (two ranks sharing one GPU in
the GPU tests, where RCCL refuses a duplicate device).
"""
import sys

import torch
import torch.distributed as dist


class SPState:
    """One rank's view of its sequence-parallel group."""

    def __init__(self, group, rank, size):
        self.group, self.rank, self.size = group, int(rank), int(size)

    def __repr__(self):
        return f"SPState(rank={self.rank}, size={self.size})"


_EXPLICIT = {"state": None, "set": False}
_REGISTRY = {}


def set_group(group):
    """Use `group` (a torch.distributed process group, or None = the default group) as this
    process's sequence-parallel group; `set_group(False)` turns SP off again (and stops reading
    the reference's parallel_states)."""
    if group is False:
        _EXPLICIT.update(state=None, set=True)
        return None
    st = SPState(group, dist.get_rank(group), dist.get_world_size(group))
    _EXPLICIT.update(state=st if st.size > 1 else None, set=True)
    return _EXPLICIT["state"]


def clear():
    """Forget an explicit setting (fall back to the reference's parallel_states)."""
    _EXPLICIT.update(state=None, set=False)


def current():
    """The active SPState, or None when sequence parallelism is off."""
    if _EXPLICIT["set"]:
        return _EXPLICIT["state"]
    ps = sys.modules.get("diffusers_lite.utils.parallel_states")
    get = getattr(ps, "get_sequence_parallel_state", None)
    if callable(get) and get():
        info = ps.nccl_info
        if int(info.sp_size) > 1:
            return SPState(info.group, info.rank_within_group, info.sp_size)
    return None


def register(st):
    """An int handle for `st` (the custom-op schema carries plain ints); 0 = no SP."""
    if st is None:
        return 0
    key = id(st.group) if st.group is not None else -1
    _REGISTRY[key] = st
    return key if key != 0 else -1


def lookup(handle):
    if not handle:
        return None
    return _REGISTRY[handle]


def split_len(total, st):
    """Tokens per rank; the reference's all-to-all needs equal chunks (`communication.py:63-64`)."""
    if total % st.size:
        raise ValueError(f"sequence parallelism: seq_len {total} is not divisible by sp_size "
                         f"{st.size} (the reference's Ulysses all-to-all needs equal chunks)")
    return total // st.size


# ------------------------------------------------------------------------- collectives ------
def _staged(group):
    return dist.get_backend(group) == "gloo"


def all_to_all_(out, inp, st):
    """out[j] <- rank j's inp[rank] for contiguous [P, ...] buffers."""
    if _staged(st.group) and inp.is_cuda:
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), group=st.group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, group=st.group)
    return out


def all_gather_seq(x, st, dim=1):
    """[.., s, ..] of every rank concatenated along `dim` (no autograd)."""
    src = x.contiguous()
    if _staged(st.group) and src.is_cuda:
        parts = [torch.empty(src.shape, dtype=src.dtype) for _ in range(st.size)]
        dist.all_gather(parts, src.cpu(), group=st.group)
        return torch.cat(parts, dim=dim).to(x.device)
    parts = [torch.empty_like(src) for _ in range(st.size)]
    dist.all_gather(parts, src, group=st.group)
    return torch.cat(parts, dim=dim)


# ------------------------------------------ the fused block's self-attention exchange -------
def qkv_to_heads(q, k, v, st):
    """q, k, v [s, C] (row-strided views) of this rank's tokens -> the full-sequence q | k | v of
    this rank's C/P columns: one [S, 3, C/P] buffer, returned with its three [S, C/P] views."""
    s, C = q.shape
    P = st.size
    cg = C // P
    send = torch.empty(P, s, 3, cg, dtype=q.dtype, device=q.device)
    for i, t in enumerate((q, k, v)):
        send[:, :, i, :].copy_(t.view(s, P, cg).permute(1, 0, 2))
    recv = all_to_all_(torch.empty_like(send), send, st).view(P * s, 3, cg)
    return recv, recv[:, 0], recv[:, 1], recv[:, 2]


def heads_to_seq(a_full, st, out=None):
    """a_full [S, C/P] (contiguous: rank i's tokens are rows [i*s, (i+1)*s)) -> [s, C]."""
    S, cg = a_full.shape
    P = st.size
    s = S // P
    recv = all_to_all_(torch.empty_like(a_full), a_full.contiguous(), st).view(P, s, cg)
    if out is None:
        out = torch.empty(s, P * cg, dtype=a_full.dtype, device=a_full.device)
    out.view(s, P, cg).copy_(recv.permute(1, 0, 2))
    return out


def seq_to_heads(x, st):
    """x [s, C] -> [S, C/P] (the d(out) of the self-attention on its way to the attention
    backward: the inverse of heads_to_seq)."""
    s, C = x.shape
    P = st.size
    cg = C // P
    send = x.reshape(s, P, cg).permute(1, 0, 2).contiguous()
    return all_to_all_(torch.empty_like(send), send, st).view(P * s, cg)


def dqkv_to_seq(dqkv_full, st, dq_out, dk_out, dv_out):
    """dqkv_full [S, 3, C/P] (dq | dk | dv of this rank's heads) -> each rank's [s, C] pieces,
    written into dq_out / dk_out / dv_out (row-strided views)."""
    S, _, cg = dqkv_full.shape
    P = st.size
    s = S // P
    recv = all_to_all_(torch.empty_like(dqkv_full), dqkv_full, st).view(P, s, 3, cg)
    for i, o in enumerate((dq_out, dk_out, dv_out)):
        o.view(s, P, cg).copy_(recv[:, :, i, :].permute(1, 0, 2))   # row-strided views split fine


# ------------------------------------------------------- autograd forms (module level) ------
class _SeqAllToAll4D(torch.autograd.Function):
    """[B, s, N, D] (this rank's tokens, all heads) <-> [B, S, N/P, D] (all tokens, this rank's
    heads), `SeqAllToAll4D` of communication.py:128-160 (scatter 2 / gather 1 and back)."""

    @staticmethod
    def forward(ctx, x, st, to_heads):
        ctx.st, ctx.to_heads = st, to_heads
        return _a2a_4d(x, st, to_heads)

    @staticmethod
    def backward(ctx, g):
        return _a2a_4d(g.contiguous(), ctx.st, not ctx.to_heads), None, None


def _a2a_4d(x, st, to_heads):
    P = st.size
    if to_heads:
        B, s, N, D = x.shape
        send = x.reshape(B, s, P, N // P, D).permute(2, 1, 0, 3, 4).contiguous()  # [P, s, B, n, D]
        recv = all_to_all_(torch.empty_like(send), send, st)                      # [P(src), s, B, n, D]
        return recv.reshape(P * s, B, N // P, D).transpose(0, 1).contiguous()
    B, S, n, D = x.shape
    s = S // P
    send = x.reshape(B, P, s, n, D).permute(1, 3, 2, 0, 4).contiguous()           # [P, n, s, B, D]
    recv = all_to_all_(torch.empty_like(send), send, st)                          # [P(src), n, s, B, D]
    return recv.reshape(P * n, s, B, D).permute(2, 1, 0, 3).contiguous()


def all_to_all_4d(x, st, to_heads=True):
    return _SeqAllToAll4D.apply(x, st, to_heads)


class _GatherSeq(torch.autograd.Function):
    """all-gather along the sequence; backward keeps this rank's slice (`_AllGather`,
    communication.py:224-260: every rank computes the same loss on the gathered tensor)."""

    @staticmethod
    def forward(ctx, x, st, dim):
        ctx.st, ctx.dim, ctx.n = st, dim, x.shape[dim]
        return all_gather_seq(x, st, dim)

    @staticmethod
    def backward(ctx, g):
        return g.narrow(ctx.dim, ctx.st.rank * ctx.n, ctx.n), None, None


def gather_seq(x, st, dim=1):
    return _GatherSeq.apply(x, st, dim)
