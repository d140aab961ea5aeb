"""Tensor-level wrappers over the C ABI (shapes, strides and dtypes checked here).

All tensors are 2-D row-major views ``[rows, cols]`` with unit column stride; row strides are
passed through, so q/k/v slices of the fused QKV output need no copy.
"""
import math

import torch

from . import _lib
from ._lib import F32, I32, I64, P, call, ptr, stream_ptr

BF16 = torch.bfloat16
EPI_BF16, EPI_GELU, EPI_RESID, EPI_F32, EPI_DGELU = range(5)


def _ld(t):
    assert t.dim() == 2 and t.stride(1) == 1, (tuple(t.shape), t.stride())
    return t.stride(0)


def gemm(a, b, c, M, N, K, a_kmajor=True, b_kmajor=True, epilogue=EPI_BF16, bias=None,
         gate=None, res=None, aux=None, accumulate=False, tile=0):
    """C[m][n] = sum_k A(m,k) B(n,k) (+ epilogue); see include/prfl_hip.h.  tile: 0 = by shape,
    128 / 256 (four-wave) / 512 (8-wave 256 tile) = forced (prfl_gemm_bf16_tiled)."""
    _lib.require_gpu(a, b, c)
    assert a.dtype == BF16 and b.dtype == BF16
    assert bias is None or (bias.dtype == BF16 and bias.is_contiguous())
    assert gate is None or (gate.dtype == torch.float32 and gate.is_contiguous())
    call("prfl_gemm_bf16_tiled", ptr(a), I64(_ld(a)), I32(int(a_kmajor)), ptr(b), I64(_ld(b)),
         I32(int(b_kmajor)), ptr(c), I64(_ld(c)), I64(M), I64(N), I64(K), I32(epilogue),
         ptr(bias), ptr(gate), ptr(res), I64(_ld(res) if res is not None else 0),
         I32(int(res is not None and res.dtype == BF16)), ptr(aux),
         I64(_ld(aux) if aux is not None else 0), I32(int(accumulate)), I32(tile), stream_ptr())
    return c


def linear(x, w, bias=None, epilogue=EPI_BF16, out=None, gate=None, res=None, aux=None, tile=0):
    """y = x @ w^T (+bias) with x [M,K] bf16, w [N,K] bf16 (nn.Linear layout)."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        dt = torch.float32 if epilogue in (EPI_RESID, EPI_F32) else BF16
        out = torch.empty(M, N, dtype=dt, device=x.device)
    return gemm(x, w, out, M, N, K, True, True, epilogue, bias, gate, res, aux, tile=tile)


def linear_t(x, wt, bias=None, epilogue=EPI_BF16, out=None, gate=None, res=None, aux=None):
    """linear() on the transposed weight wt [K, N] (cast_bf16_t of the nn.Linear weight): the
    weight is then an MN-major GEMM operand; results bit-identical to linear(x, wt.t())."""
    M, K = x.shape
    N = wt.shape[1]
    if out is None:
        dt = torch.float32 if epilogue in (EPI_RESID, EPI_F32) else BF16
        out = torch.empty(M, N, dtype=dt, device=x.device)
    return gemm(x, wt, out, M, N, K, True, False, epilogue, bias, gate, res, aux)


def linear_dx(dy, w, out=None, epilogue=EPI_BF16, aux=None):
    """dX[M,K] = dY[M,N] @ W[N,K] (bf16 out; DGELU epilogue multiplies by gelu'(aux))."""
    M, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, dtype=BF16, device=dy.device)
    return gemm(dy, w, out, M, K, N, True, False, epilogue, aux=aux)


def linear_dw(dy, x, out=None, accumulate=False):
    """dW[N,K] = dY[M,N]^T @ X[M,K] in fp32 (accumulate=True adds into `out`)."""
    M, N = dy.shape
    K = x.shape[1]
    if out is None:
        out = torch.empty(N, K, dtype=torch.float32, device=dy.device)
    return gemm(dy, x, out, N, K, M, False, False, EPI_F32, accumulate=accumulate)


FP8 = torch.float8_e4m3fn   # OCP e4m3 (gfx950), not the MI300 fnuz variant


def quant_rows_fp8(x, q=None, scale=None):
    """Per-row e4m3 quantisation: scale[m] = amax_m / 448, q = e4m3(x * 448 / amax_m).
    x [M, K] bf16 or fp32 (row-strided), K % 8 == 0, K <= 16384."""
    _lib.require_gpu(x)
    M, K = x.shape
    if q is None:
        q = torch.empty(M, K, dtype=FP8, device=x.device)
    if scale is None:
        scale = torch.empty(M, dtype=torch.float32, device=x.device)
    assert x.dtype in (BF16, torch.float32) and q.dtype == FP8
    call("prfl_quant_rows_fp8", ptr(x), I32(int(x.dtype == torch.float32)), I64(_ld(x)), I64(M),
         I64(K), ptr(q), I64(_ld(q)), ptr(scale), stream_ptr())
    return q, scale


def linear_fp8(xq, xs, wq, ws, bias=None, epilogue=EPI_BF16, out=None, gate=None, res=None,
               aux=None):
    """y = (xs * xq) @ (ws * wq)^T (+bias, epilogue) on the block-scaled fp8 MFMA: xq [M,K],
    wq [N,K] e4m3 with per-row fp32 scales xs [M], ws [N]."""
    _lib.require_gpu(xq, wq)
    assert xq.dtype == FP8 and wq.dtype == FP8
    assert bias is None or (bias.dtype == BF16 and bias.is_contiguous())
    assert gate is None or (gate.dtype == torch.float32 and gate.is_contiguous())
    M, K = xq.shape
    N = wq.shape[0]
    if out is None:
        dt = torch.float32 if epilogue == EPI_RESID else BF16
        out = torch.empty(M, N, dtype=dt, device=xq.device)
    call("prfl_gemm_fp8", ptr(xq), I64(_ld(xq)), ptr(xs), ptr(wq), I64(_ld(wq)), ptr(ws),
         ptr(out), I64(_ld(out)), I64(M), I64(N), I64(K), I32(epilogue), ptr(bias), ptr(gate),
         ptr(res), I64(_ld(res) if res is not None else 0),
         I32(int(res is not None and res.dtype == BF16)), ptr(aux),
         I64(_ld(aux) if aux is not None else 0), stream_ptr())
    return out


def cast_bf16(src, dst=None):
    """fp32 -> bf16 (round to nearest even); dst may be a contiguous slice of a larger buffer.
    A weight already stored in bf16 (a frozen trunk, train.store_frozen_bf16) is returned as
    it is, or copied into dst: its bits are what the cast of its fp32 master would give."""
    _lib.require_gpu(src)
    src = src.contiguous()
    if src.dtype == BF16:
        if dst is None:
            return src
        assert dst.is_contiguous() and dst.numel() == src.numel()
        return dst.view(src.shape).copy_(src)
    if dst is None:
        dst = torch.empty(src.shape, dtype=BF16, device=src.device)
    assert dst.is_contiguous() and dst.numel() == src.numel()
    call("prfl_cast_f32_bf16", ptr(src), ptr(dst), I64(src.numel()), stream_ptr())
    return dst


def cast_bf16_t(w, dst=None):
    """fp32 nn.Linear weight w [N, K] -> bf16 w^T [K, N] (prfl_cast_f32_bf16_t); dst may be a
    column block of a wider row-major buffer (its row stride is dst.stride(0))."""
    _lib.require_gpu(w)
    w = w.contiguous()
    N, K = w.shape
    if dst is None:
        dst = torch.empty(K, N, dtype=BF16, device=w.device)
    assert dst.shape == (K, N) and dst.stride(1) == 1
    call("prfl_cast_f32_bf16_t", ptr(w), I64(N), I64(K), I64(K), ptr(dst), I64(dst.stride(0)),
         stream_ptr())
    return dst


def colsum_reduce(part, out=None, accumulate=False):
    P_, N = part.shape
    if out is None:
        out = torch.empty(N, dtype=torch.float32, device=part.device)
        accumulate = False
    call("prfl_colsum_reduce", ptr(part), I64(P_), I64(N), ptr(out), I32(int(accumulate)),
         stream_ptr())
    return out


def colsum(x, out=None, accumulate=False):
    """sum over rows of a bf16 [L, N] matrix -> fp32 [N]."""
    L, N = x.shape
    rp = call_int("prfl_colsum_rows_per_part")
    part = torch.empty((L + rp - 1) // rp, N, dtype=torch.float32, device=x.device)
    call("prfl_colsum_bf16", ptr(x), I64(_ld(x)), I64(L), I64(N), ptr(part), stream_ptr())
    return colsum_reduce(part, out, accumulate)


_int_cache = {}


def call_int(name):
    if name not in _int_cache:
        _int_cache[name] = getattr(_lib.load(), name)()
    return _int_cache[name]


def gate_bwd(dx, y, gate, dy_out=None, want_gate=True, want_bias=True):
    """x_out = x + y*gate: dy = bf16(dx*gate), d gate = sum dx*y, d bias = sum dy."""
    L, N = dx.shape
    rp = call_int("prfl_colsum_rows_per_part")
    nb = (L + rp - 1) // rp
    if dy_out is None:
        dy_out = torch.empty(L, N, dtype=BF16, device=dx.device)
    pg = torch.empty(nb, N, dtype=torch.float32, device=dx.device) if (want_gate and y is not None) else None
    pb = torch.empty(nb, N, dtype=torch.float32, device=dx.device) if want_bias else None
    call("prfl_gate_bwd", ptr(dx), I64(_ld(dx)), ptr(y), I64(_ld(y) if y is not None else 0),
         ptr(gate), I64(L), I64(N), ptr(dy_out), I64(_ld(dy_out)), ptr(pg), ptr(pb), stream_ptr())
    dgate = colsum_reduce(pg) if pg is not None else None
    dbias = colsum_reduce(pb) if pb is not None else None
    return dy_out, dgate, dbias


def ln_mod_fwd(x, scale=None, shift=None, w=None, b=None, eps=1e-6, out=None):
    """bf16(LN(x)*(1+scale)+shift) or bf16(LN(x)*w+b); returns (out, mean, rstd)."""
    L, C = x.shape
    if out is None:
        out = torch.empty(L, C, dtype=BF16, device=x.device)
    mean = torch.empty(L, dtype=torch.float32, device=x.device)
    rstd = torch.empty(L, dtype=torch.float32, device=x.device)
    call("prfl_ln_mod_fwd", ptr(x), I32(int(x.dtype == BF16)), I64(_ld(x)), I64(L), I64(C),
         ptr(scale), ptr(shift), ptr(w), ptr(b), F32(eps), ptr(out), I64(_ld(out)), ptr(mean),
         ptr(rstd), stream_ptr())
    return out, mean, rstd


def ln_mod_bwd(dy, x, mean, rstd, dx, scale=None, w=None, accumulate=True):
    """dx (+)= LN backward; returns (sum dy*xhat, sum dy) — (d scale, d shift) or (d w, d b)."""
    L, C = x.shape
    rp = call_int("prfl_norm_rows_per_part")
    nb = (L + rp - 1) // rp
    p0 = torch.empty(nb, C, dtype=torch.float32, device=x.device)
    p1 = torch.empty(nb, C, dtype=torch.float32, device=x.device)
    call("prfl_ln_mod_bwd", ptr(dy), I64(_ld(dy)), ptr(x), I32(int(x.dtype == BF16)), I64(_ld(x)),
         ptr(mean), ptr(rstd), I64(L), I64(C), ptr(scale), ptr(w), ptr(dx), I64(_ld(dx)),
         I32(int(accumulate)), ptr(p0), ptr(p1), stream_ptr())
    return colsum_reduce(p0), colsum_reduce(p1)


# softmax_scale * log2(e) of head_dim 128: the out_scale that turns norm_q's output into the q
# operand of the *_l2q attention entries (attn_fwd / attn_bwd with q_log2=True)
L2Q_SCALE = 1.4426950408889634 / math.sqrt(128)


def rms_rope_fwd(x, w, eps=1e-6, rope_tab=None, grid=(0, 0, 0), out=None, out_scale=1.0, row0=0):
    """bf16(rope(bf16(x * rsqrt(mean x^2 + eps)) * w) * out_scale); row r is token row0 + r of
    the grid (row0 > 0: a sequence-parallel rank's shard, model.py:89-96)."""
    L, C = x.shape
    if out is None:
        out = torch.empty(L, C, dtype=BF16, device=x.device)
    rstd = torch.empty(L, dtype=torch.float32, device=x.device)
    f, h, ww = grid
    call("prfl_rms_rope_fwd_pos", ptr(x), I64(_ld(x)), I64(L), I64(C), ptr(w), F32(eps),
         ptr(rope_tab), I64(f), I64(h), I64(ww), I64(row0), ptr(out), I64(_ld(out)), ptr(rstd),
         F32(out_scale), stream_ptr())
    return out, rstd


def rms_rope_bwd(dout, x, rstd, w, rope_tab=None, grid=(0, 0, 0), dx=None, out_scale=1.0, row0=0):
    """returns (dx bf16, d w fp32); out_scale and row0 as the forward's (dout is scaled by it)."""
    L, C = x.shape
    rp = call_int("prfl_norm_rows_per_part")
    p0 = torch.empty((L + rp - 1) // rp, C, dtype=torch.float32, device=x.device)
    if dx is None:
        dx = torch.empty(L, C, dtype=BF16, device=x.device)
    f, h, ww = grid
    call("prfl_rms_rope_bwd_pos", ptr(dout), I64(_ld(dout)), ptr(x), I64(_ld(x)), ptr(rstd),
         I64(L), I64(C), ptr(w), ptr(rope_tab), I64(f), I64(h), I64(ww), I64(row0), ptr(dx),
         I64(_ld(dx)), ptr(p0), F32(out_scale), stream_ptr())
    return dx, colsum_reduce(p0)


# the long-KV q_log2 forward reads V from its key-chunked transposed image (prfl_attn_v_to_vt +
# prfl_attn_fwd_l2q_vt_ws: one ds_read_b128 per V^T fragment; outputs bit-identical)
ATTN_VT = True     # 720p forward 84.11 -> 83.08 ms incl. the 0.29 ms transpose (profiles/r04_ab_attn_vt.txt)
# ... and (off) the long-KV q_log2 backward's dQ kernel its K^T fragments from K's VT image
# (prfl_attn_bwd_l2q_kt_ws; bit-identical, measured 0.3-0.5 % slower with the K transpose
# included: profiles/r04_ab_bwd_variants.txt)
ATTN_KT = False
VT_MIN_KEYS = 4096


def attn_fwd(q, k, v, num_heads, k_len=None, out=None, scale=None, q_log2=False):
    """q [Lq, H*128], k/v [Lk, H*128] (row-strided views) -> (o bf16 [Lq, H*128], lse2 [H, Lq]).
    q_log2: q is already multiplied by softmax_scale * log2(e) (rms_rope_fwd out_scale=L2Q_SCALE);
    scale is then unused (prfl_attn_fwd_l2q_ws; with Lk >= VT_MIN_KEYS and ATTN_VT, V is first
    rewritten into the VT layout and prfl_attn_fwd_l2q_vt_ws runs)."""
    Lq, C = q.shape
    Lk = k.shape[0]
    assert C == num_heads * 128, "head_dim must be 128"
    k_len = Lk if k_len is None else int(k_len)
    sc = scale if scale is not None else 1.0 / math.sqrt(128)
    if out is None:
        out = torch.empty(Lq, C, dtype=BF16, device=q.device)
    lse = torch.empty(num_heads, Lq, dtype=torch.float32, device=q.device)
    # scratch for the split-KV tail of long-KV launches (0 bytes when the grid has no tail)
    nb = _lib.load().prfl_attn_fwd_ws_bytes(1, Lq, Lk, num_heads, k_len)
    ws = torch.empty(nb, dtype=torch.uint8, device=q.device) if nb > 0 else None
    head = (ptr(q), I64(_ld(q)), I64(0), ptr(k), I64(_ld(k)), I64(0), ptr(v), I64(_ld(v)), I64(0),
            ptr(out), I64(_ld(out)), I64(0), ptr(lse), I64(1), I64(Lq), I64(Lk), I64(num_heads),
            I64(k_len))
    if q_log2 and ATTN_VT and Lk >= VT_MIN_KEYS:
        vt = attn_v_to_vt(v, num_heads)
        call("prfl_attn_fwd_l2q_vt_ws", *head[:6], ptr(vt), *head[9:], ptr(ws), I64(nb), stream_ptr())
    elif q_log2:
        call("prfl_attn_fwd_l2q_ws", *head, ptr(ws), I64(nb), stream_ptr())
    else:
        call("prfl_attn_fwd_ws", *head, F32(sc), ptr(ws), I64(nb), stream_ptr())
    return out, lse


def attn_v_to_vt(v, num_heads):
    """v [Lk, H*128] (row-strided view) -> its VT image (prfl_attn_v_to_vt), a flat bf16 tensor"""
    Lk = v.shape[0]
    nb = _lib.load().prfl_attn_vt_bytes(1, Lk, num_heads)
    vt = torch.empty(nb // 2, dtype=BF16, device=v.device)
    call("prfl_attn_v_to_vt", ptr(v), I64(_ld(v)), I64(0), ptr(vt), I64(1), I64(Lk), I64(num_heads),
         stream_ptr())
    return vt


def attn_fwd_fp8(q, k, v, num_heads, k_len=None, out=None, scale=None, q_log2=False):
    """attn_fwd on the block-scaled e4m3 MFMA (config C5 self-attention): same arguments and
    outputs; q/k/v are quantised inside the call into a scratch buffer (~3 bytes per element)."""
    Lq, C = q.shape
    Lk = k.shape[0]
    assert C == num_heads * 128, "head_dim must be 128"
    k_len = Lk if k_len is None else int(k_len)
    sc = scale if scale is not None else 1.0 / math.sqrt(128)
    if out is None:
        out = torch.empty(Lq, C, dtype=BF16, device=q.device)
    lse = torch.empty(num_heads, Lq, dtype=torch.float32, device=q.device)
    nb = _lib.load().prfl_attn_fwd_fp8_ws_bytes(1, Lq, Lk, num_heads, k_len)
    ws = torch.empty(nb, dtype=torch.uint8, device=q.device)
    head = (ptr(q), I64(_ld(q)), I64(0), ptr(k), I64(_ld(k)), I64(0), ptr(v), I64(_ld(v)), I64(0),
            ptr(out), I64(_ld(out)), I64(0), ptr(lse), I64(1), I64(Lq), I64(Lk), I64(num_heads),
            I64(k_len))
    if q_log2:
        call("prfl_attn_fwd_fp8_l2q", *head, ptr(ws), I64(nb), stream_ptr())
    else:
        call("prfl_attn_fwd_fp8", *head, F32(sc), ptr(ws), I64(nb), stream_ptr())
    return out, lse


def attn_bwd(q, k, v, o, do, lse, num_heads, k_len=None, dq=None, dk=None, dv=None, scale=None,
             q_log2=False):
    """Backward of attn_fwd; with q_log2 dq is the gradient w.r.t. the pre-scaled q."""
    Lq, C = q.shape
    Lk = k.shape[0]
    k_len = Lk if k_len is None else int(k_len)
    sc = scale if scale is not None else 1.0 / math.sqrt(128)
    dev = q.device
    dq = torch.empty(Lq, C, dtype=BF16, device=dev) if dq is None else dq
    dk = torch.empty(Lk, C, dtype=BF16, device=dev) if dk is None else dk
    dv = torch.empty(Lk, C, dtype=BF16, device=dev) if dv is None else dv
    delta = torch.empty(num_heads, Lq, dtype=torch.float32, device=dev)
    # scratch for the split tails of long-KV launches (0 bytes when the grids have no tail)
    nb = _lib.load().prfl_attn_bwd_ws_bytes(1, Lq, Lk, num_heads, k_len)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev) if nb > 0 else None
    head = (ptr(q), I64(_ld(q)), I64(0), ptr(k), I64(_ld(k)), I64(0), ptr(v), I64(_ld(v)), I64(0),
            ptr(o), I64(_ld(o)), I64(0), ptr(do), I64(_ld(do)), I64(0), ptr(lse), ptr(delta),
            ptr(dq), I64(_ld(dq)), I64(0), ptr(dk), I64(_ld(dk)), I64(0), ptr(dv), I64(_ld(dv)),
            I64(0), I64(1), I64(Lq), I64(Lk), I64(num_heads), I64(k_len))
    if q_log2 and ATTN_KT and Lk >= VT_MIN_KEYS:
        kt = attn_v_to_vt(k, num_heads)            # K in the VT layout for the dQ kernel
        call("prfl_attn_bwd_l2q_kt_ws", *head[:6], ptr(kt), *head[6:], ptr(ws), I64(nb), stream_ptr())
    elif q_log2:
        call("prfl_attn_bwd_l2q_ws", *head, ptr(ws), I64(nb), stream_ptr())
    else:
        call("prfl_attn_bwd_ws", *head, F32(sc), ptr(ws), I64(nb), stream_ptr())
    return dq, dk, dv


def query_pool_fwd(q, kv, num_heads, scale, nsplit=None):
    """Single-query attention pooling (csrc/pool.hip): q [N, E] bf16, kv [N, L, 2E] bf16 (k | v)
    -> (o bf16 [N, E], lse2 fp32 [N, H], o32 fp32 [N, E] = o before its bf16 rounding)."""
    _lib.require_gpu(q, kv)
    assert q.dtype == BF16 and kv.dtype == BF16 and kv.stride(2) == 1
    N, E = q.shape
    L = kv.shape[1]
    if nsplit is None:
        nsplit = call_int_args("prfl_query_pool_splits", I64(N), I64(L), I64(num_heads))
    hd = E // num_heads
    o = torch.empty(N, E, dtype=BF16, device=q.device)
    lse = torch.empty(N, num_heads, dtype=torch.float32, device=q.device)
    o32 = torch.empty(N, E, dtype=torch.float32, device=q.device)
    pm = torch.empty(N * num_heads * nsplit, dtype=torch.float32, device=q.device)
    pl = torch.empty_like(pm)
    po = torch.empty(N * num_heads * nsplit * hd, dtype=torch.float32, device=q.device)
    call("prfl_query_pool_fwd", ptr(q), I64(_ld(q)), ptr(kv), I64(kv.stride(1)), I64(kv.stride(0)),
         I64(N), I64(L), I64(num_heads), I64(E), F32(scale), ptr(o), I64(E), ptr(lse), ptr(o32),
         ptr(pm), ptr(pl), ptr(po), I64(nsplit), stream_ptr())
    return o, lse, o32


def query_pool_bwd(do, q, kv, o32, lse, num_heads, scale, nsplit=None):
    """-> (dq fp32 [N, E], dkv bf16 [N, L, 2E])."""
    N, E = q.shape
    L = kv.shape[1]
    if nsplit is None:
        nsplit = call_int_args("prfl_query_pool_splits", I64(N), I64(L), I64(num_heads))
    hd = E // num_heads
    dq = torch.empty(N, E, dtype=torch.float32, device=q.device)
    dkv = torch.empty(N, L, 2 * E, dtype=BF16, device=q.device)
    po = torch.empty(N * num_heads * nsplit * hd, dtype=torch.float32, device=q.device)
    call("prfl_query_pool_bwd", ptr(do), ptr(q), I64(_ld(q)), ptr(kv), I64(kv.stride(1)),
         I64(kv.stride(0)), ptr(o32), ptr(lse), I64(N), I64(L), I64(num_heads), I64(E), F32(scale),
         ptr(dq), I64(E), ptr(dkv), I64(2 * E), I64(L * 2 * E), ptr(po), I64(nsplit), stream_ptr())
    return dq, dkv


def call_int_args(name, *args):
    return getattr(_lib.load(), name)(*args)


def sumsq_(x, out):
    call("prfl_sumsq", ptr(x), I64(x.numel()), ptr(out), stream_ptr())


def scale_(x, factor):
    call("prfl_scale", ptr(x), I64(x.numel()), ptr(factor), stream_ptr())


def adamw_(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step, zero_grad=False):
    """One AdamW step on p (m, v: its moments); zero_grad also sets g to 0 once read."""
    for t in (p, g, m, v):
        assert t.is_contiguous() and t.dtype == torch.float32
    call("prfl_adamw_zero_grad" if zero_grad else "prfl_adamw", ptr(p), ptr(g), ptr(m), ptr(v),
         I64(p.numel()), F32(lr), F32(beta1), F32(beta2), F32(eps), F32(weight_decay), I64(step),
         stream_ptr())


def rope_table(freqs_complex, device):
    """complex freqs [1024, 64] (model.py:521-526) -> fp32 (cos, sin) table on device."""
    t = torch.view_as_real(freqs_complex.to(torch.complex128)).to(torch.float32).contiguous()
    return t.to(device)


def prof_enable(on=True):
    call("prfl_prof_enable", I32(int(on)))


def prof_collect():
    import ctypes
    n = _lib.NKID
    counts = (ctypes.c_int64 * n)()
    ms = (ctypes.c_double * n)()
    work = (ctypes.c_double * n)()
    call("prfl_prof_collect", ctypes.cast(counts, ctypes.c_void_p), ctypes.cast(ms, ctypes.c_void_p),
         ctypes.cast(work, ctypes.c_void_p), I32(n))
    return {k: dict(count=counts[i], ms=ms[i], work=work[i]) for k, i in _lib.KID.items()}


def prof_clock():
    """Effective shader clock of the self-attention forwards since the last call (MHz)."""
    import ctypes
    v = (ctypes.c_double * 3)()
    n = ctypes.c_int64()
    base = ctypes.addressof(v)
    call("prfl_prof_clock", P(base), P(base + 8), P(base + 16), P(ctypes.addressof(n)))
    return dict(mean_mhz=v[0], min_mhz=v[1], max_mhz=v[2], launches=n.value)


def _coef_array(coef):
    import ctypes
    assert len(coef) == 11
    return (ctypes.c_float * 11)(*[float(c) for c in coef])


def unipc_step_fwd(sample, model_output, last_sample, hist1, hist2, coef, corr_order, pred_order):
    """Fused FlowUniPC update (csrc/unipc.hip).  Returns (m_t fp32, sample_c bf16, prev bf16)."""
    import ctypes
    _lib.require_gpu(sample, model_output)
    if sample.dtype != torch.bfloat16 or model_output.dtype != torch.float32:
        raise NotImplementedError("fused UniPC step: bf16 sample and fp32 model output "
                                  "(the PRFL chain's dtypes, train_prfl.py:687-734)")
    n = sample.numel()
    for t in (model_output, last_sample, hist1, hist2):
        if t is not None and (t.numel() != n or not t.is_contiguous()):
            raise ValueError("fused UniPC step: operands must be contiguous with the sample's shape")
    sample = sample.contiguous()
    m_t = torch.empty(sample.shape, dtype=torch.float32, device=sample.device)
    prev = torch.empty_like(sample)
    sample_c = torch.empty_like(sample) if corr_order else sample
    cf = _coef_array(coef)
    call("prfl_unipc_step", ptr(sample), ptr(model_output), ptr(last_sample), ptr(hist1),
         ptr(hist2), ptr(m_t), ptr(sample_c) if corr_order else P(0), ptr(prev), I64(n),
         ctypes.cast(cf, ctypes.c_void_p), I32(corr_order), I32(pred_order), stream_ptr())
    return m_t, sample_c, prev


def unipc_step_bwd(grad_prev, coef, corr_order, pred_order):
    import ctypes
    g = grad_prev.to(torch.bfloat16).contiguous()
    out = torch.empty(g.shape, dtype=torch.float32, device=g.device)
    cf = _coef_array(coef)
    call("prfl_unipc_step_bwd", ptr(g), ptr(out), I64(g.numel()), ctypes.cast(cf, ctypes.c_void_p),
         I32(corr_order), I32(pred_order), stream_ptr())
    return out
