"""Fused WanAttentionBlock forward/backward on the HIP kernels (`model.py:280-359`).

The block is one autograd node (the ``prfl::wan_block`` custom op, custom_ops.py) that implements
the reference's non-reentrant
activation checkpoint (`fsdp_utils.py:17-50`, every block checkpointed): the forward keeps only the
block input; the backward re-runs the forward saving what the backward kernels need, then runs
the hand-written backward chain.  fp32 master weights are cast to bf16 once per pass into
transient buffers (q/k/v concatenated into one [3C, C] operand, so the QKV projection is a single
GEMM without changing any state-dict key).

Precision flow = the reference under bf16 autocast: LN/RMSNorm/modulation/gates
fp32, every Linear bf16 x bf16 -> fp32 accumulate -> bf16, RoPE applied in fp32 to the bf16-rounded
normalised q/k, residual stream fp32.
"""
import torch

from . import ops
from . import sp as SP
from .ops import BF16, EPI_BF16, EPI_GELU, EPI_RESID, EPI_DGELU

T5_CONTEXT_TOKEN_NUMBER = 512  # model.py:18

SA_NAMES = ["self_attn.q.weight", "self_attn.q.bias", "self_attn.k.weight", "self_attn.k.bias",
            "self_attn.v.weight", "self_attn.v.bias", "self_attn.o.weight", "self_attn.o.bias",
            "self_attn.norm_q.weight", "self_attn.norm_k.weight"]
CA_NAMES = ["norm3.weight", "norm3.bias", "cross_attn.q.weight", "cross_attn.q.bias",
            "cross_attn.k.weight", "cross_attn.k.bias", "cross_attn.v.weight", "cross_attn.v.bias",
            "cross_attn.o.weight", "cross_attn.o.bias", "cross_attn.norm_q.weight",
            "cross_attn.norm_k.weight"]
I2V_NAMES = ["cross_attn.k_img.weight", "cross_attn.k_img.bias", "cross_attn.v_img.weight",
             "cross_attn.v_img.bias", "cross_attn.norm_k_img.weight"]
FFN_NAMES = ["ffn.0.weight", "ffn.0.bias", "ffn.2.weight", "ffn.2.bias"]


def param_names(i2v):
    return SA_NAMES + CA_NAMES + (I2V_NAMES if i2v else []) + FFN_NAMES


# Attention-output stash (memory-for-time trade on top of the reference's per-block checkpoint):
# a block whose forward records a graph may keep its self-attention output and LSE (L*C*2 +
# H*L*4 bytes per sample) so the backward's recompute skips the L x L attention forward — the
# kernels are deterministic, so the recomputed and the kept tensors are bit-identical.  The budget
# bounds the bytes kept at any time: a forward takes `need` from it, the block's backward gives
# it back (custom_ops._wan_block_bwd), so any training loop — the reference drivers included —
# keeps using it step after step.  The trainers also reset it at the start of every step (a
# graph dropped without a backward never gives its bytes back).  0 (the default) keeps the pure
# checkpoint.  A block under an external torch.utils.checkpoint (apply_fsdp_checkpointing with
# wrap_fused) has `stash_attn` off: that recompute could otherwise decide differently.
_STASH = {"budget": 0, "left": 0}


def set_attn_stash_budget(nbytes):
    _STASH["budget"] = int(nbytes)
    _STASH["left"] = int(nbytes)


def reset_attn_stash():
    _STASH["left"] = _STASH["budget"]


def stash_bytes(ao, lse):
    return ao.numel() * ao.element_size() + lse.numel() * lse.element_size()


def credit_attn_stash(nbytes):
    _STASH["left"] = min(_STASH["budget"], _STASH["left"] + int(nbytes))


class Meta:
    """Non-tensor block arguments."""

    def __init__(self, num_heads, grid, seq_len, rope_tab, i2v, eps=1e-6, fp8=0, sp=None):
        self.num_heads = num_heads
        # Ulysses sequence parallelism (sp.SPState or None): x holds this rank's L tokens, the
        # rank's tokens start at position sp.rank * L of the padded sequence (sp.py)
        self.sp = sp
        # config C5 (WanModel.set_fp8_gemm): fp8 & 3 = 0 bf16; 1 e4m3 forward projections; 2 also
        # the e4m3 self-attention forward (ops.attn_fwd_fp8; its backward stays bf16 on that
        # forward's O/LSE); fp8 >> 2 = mask of projections kept bf16 (fp8_code)
        self.fp8 = int(fp8)
        self.fp8_mode = self.fp8 & 3
        self.grid = grid            # list of (F, H, W) per sample
        self.seq_len = seq_len      # list of valid key lengths per sample (k_lens)
        self.rope_tab = rope_tab    # fp32 [1024, 64, 2] device tensor
        self.i2v = i2v
        self.eps = eps


PROJ = ("qkv", "o", "cq", "co", "1", "2")   # the six forward projections the fp8 path quantises


def fp8_code(mode, keep_bf16=()):
    """The `fp8` integer of Meta / the prfl::wan_block op: mode 0 / 1 / 2 (block.Meta) plus the
    projections (names of PROJ) that stay bf16 while the others run e4m3 — the per-projection
    error study of config C5 (tests/test_gpu_fp8.py) and its bf16-kept option."""
    mask = 0
    for n in keep_bf16:
        mask |= 1 << PROJ.index(n)
    return int(mode) | (mask << 2)


# config C5's default (round 6): the cross-attention q / o projections stay bf16.  Measured on the
# real-width I2V block against the fp32 truth (profiles/r06_c5_projection_table.log), e4m3 on ONE
# operand at a time gives a residual-update error of 3.3 % (cross q), 3.4 % (cross o), 1.8 %
# (FFN up / down), 0.7 % (QKV, self o, the int8 / e4m3 attention: the bf16 path's own 0.6 %);
# all of them together 5.3 %, with cross q + o bf16 2.5 % (SURVEY §8c's 5e-2), for the
# bf16 cost of two C x C GEMMs per block forward
C5_KEEP_BF16 = ("cq", "co")


class BF16Weights:
    """bf16 copies of a block's Linear weights/biases for one forward or backward pass.

    With ``fp8`` the six large forward projections (QKV, O, cross q/o, FFN in/out) also get
    per-output-row e4m3 copies quantised straight from the fp32 masters (``self.q[name]`` =
    (codes, scales)); ``need_bf16=False`` (a no-grad forward on the fp8 path) skips their bf16
    casts — only the backward's dX GEMMs read those."""

    FP8_KEYS = {"qkv": None, "o": "self_attn.o", "cq": "cross_attn.q", "co": "cross_attn.o",
                "1": "ffn.0", "2": "ffn.2"}

    def __init__(self, P, fp8=0, need_bf16=True):
        g = P.__getitem__
        C = g("self_attn.q.weight").shape[0]
        dev = g("self_attn.q.weight").device
        code = int(fp8)
        keep = {n for i, n in enumerate(PROJ) if (code >> 2) >> i & 1}
        fp8 = (code & 3) > 0
        if keep:                 # some projections bf16 beside e4m3 ones: every bf16 copy cast
            need_bf16 = True
        self.fp8 = fp8
        self.q = {}
        # bf16 path: the six forward projections take their weight TRANSPOSED (self.t[name] =
        # W^T [K, N], cast straight from the fp32 master by ops.cast_bf16_t): an MN-major GEMM
        # operand, bit-identical results, 2-4 % faster forward GEMMs (profiles/r04_ab_gemm_wt.txt);
        # the K-major copies (self.w*) are cast only where a backward's dX GEMM reads them, and
        # there (need_bf16: the backward's recompute, 88 of the 928 block forwards of a 720p
        # iteration) the forward reuses them: no second copy of the block's weights at the peak
        self.t = {}
        if not fp8 and not need_bf16:
            f32 = lambda n: g(n).dtype == torch.float32  # noqa: E731  (bf16-stored: K-major path)
            wt = lambda n: ops.cast_bf16_t(g(n)) if f32(n) and g(n).shape[0] % 256 == 0 else None  # noqa: E731
            if C % 256 == 0 and all(f32(f"self_attn.{n}.weight") for n in "qkv"):
                self.t["qkv"] = torch.empty(C, 3 * C, dtype=BF16, device=dev)
                for i, n in enumerate("qkv"):
                    ops.cast_bf16_t(g(f"self_attn.{n}.weight"), self.t["qkv"][:, i * C:(i + 1) * C])
            for name, pre in self.FP8_KEYS.items():
                if pre is not None:
                    t = wt(pre + ".weight")
                    if t is not None:
                        self.t[name] = t
        big = need_bf16 or (not fp8 and len(self.t) < 6)
        if big:
            self.wqkv = torch.empty(3 * C, C, dtype=BF16, device=dev)
        self.bqkv = torch.empty(3 * C, dtype=BF16, device=dev)
        for i, n in enumerate("qkv"):
            if big:
                ops.cast_bf16(g(f"self_attn.{n}.weight"), self.wqkv[i * C:(i + 1) * C])
            ops.cast_bf16(g(f"self_attn.{n}.bias"), self.bqkv[i * C:(i + 1) * C])
        c = lambda n: ops.cast_bf16(g(n))  # noqa: E731
        cw = lambda n: c(n) if big else None  # noqa: E731
        self.wo, self.bo = cw("self_attn.o.weight"), c("self_attn.o.bias")
        for n in ("q", "k", "v", "o", "k_img", "v_img"):
            key = f"cross_attn.{n}.weight"
            if key in P:
                setattr(self, "wc" + n, cw(key) if n in ("q", "o") else c(key))
                setattr(self, "bc" + n, c(f"cross_attn.{n}.bias"))
        self.w1, self.b1 = cw("ffn.0.weight"), c("ffn.0.bias")
        self.w2, self.b2 = cw("ffn.2.weight"), c("ffn.2.bias")
        if fp8:
            for name, pre in self.FP8_KEYS.items():
                if name in keep:
                    continue
                if pre is None:     # q/k/v rows quantised into one [3C, C] operand
                    wq = torch.empty(3 * C, C, dtype=ops.FP8, device=dev)
                    ws = torch.empty(3 * C, dtype=torch.float32, device=dev)
                    for i, n in enumerate("qkv"):
                        ops.quant_rows_fp8(g(f"self_attn.{n}.weight"), wq[i * C:(i + 1) * C],
                                           ws[i * C:(i + 1) * C])
                    self.q[name] = (wq, ws)
                else:
                    self.q[name] = ops.quant_rows_fp8(g(pre + ".weight"))


def lin(W, name, x, **kw):
    """The block's forward projection `name` (qkv, o, cq, co, 1, 2) of x [M, K] bf16: on the fp8
    path x is quantised per row and the GEMM runs on the block-scaled fp8 MFMA, otherwise bf16."""
    wn = {"qkv": "qkv", "o": "o", "cq": "cq", "co": "co", "1": "1", "2": "2"}[name]
    bias = getattr(W, "b" + wn)
    if W.fp8 and name in W.q:
        xq, xs = ops.quant_rows_fp8(x)
        wq, ws = W.q[name]
        return ops.linear_fp8(xq, xs, wq, ws, bias, **kw)
    if name in W.t:
        return ops.linear_t(x, W.t[name], bias, **kw)
    return ops.linear(x, getattr(W, "w" + wn), bias, **kw)


def _split_ctx(ctx, i2v):
    if not i2v:
        return ctx, None
    n_img = ctx.shape[0] - T5_CONTEXT_TOKEN_NUMBER
    return ctx[n_img:], ctx[:n_img]


def block_forward_one(P, W, x, e, ctx, meta, b, save, attn=None, keep_attn=False):
    """One sample: x [L, C] (fp32, or bf16 for block 0), e [6, C] fp32, ctx [Lc, C] bf16.
    attn: a kept (ao, lse) of this sample's self-attention (skips the attention forward);
    keep_attn: return it in S["attn"] even when not saving for the backward."""
    g = P.__getitem__
    L, C = x.shape
    nh, eps = meta.num_heads, meta.eps
    S = {}
    # ---- self-attention (model.py:344-348) ----
    h1, m1, r1 = ops.ln_mod_fwd(x, scale=e[1], shift=e[0], eps=eps)
    qkv = lin(W, "qkv", h1)
    q_raw, k_raw, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    grid = meta.grid[b]
    # q leaves RMSNorm+RoPE already in log2 units (x softmax_scale * log2 e, one bf16 rounding as
    # before): the attention kernels then take one v_exp per score (ops.L2Q_SCALE, q_log2)
    st = meta.sp
    row0 = st.rank * L if st is not None else 0     # the rank's first token (model.py:89-96)
    qr, rq = ops.rms_rope_fwd(q_raw, g("self_attn.norm_q.weight"), eps, meta.rope_tab, grid,
                              out_scale=ops.L2Q_SCALE, row0=row0)
    kr, rk = ops.rms_rope_fwd(k_raw, g("self_attn.norm_k.weight"), eps, meta.rope_tab, grid,
                              row0=row0)
    fwd = ops.attn_fwd_fp8 if meta.fp8_mode >= 2 else ops.attn_fwd
    if st is None:
        if attn is not None:
            ao, lse = attn
        else:
            ao, lse = fwd(qr, kr, v, nh, k_len=meta.seq_len[b], q_log2=True)
        if keep_attn:
            S["attn"] = (ao, lse)
    else:
        # Ulysses: all tokens of this rank's nh / P heads (model.py:183-196); the kept output
        # is the head-sharded one, viewed in the [L, C] / [H, L] shapes of the unsharded stash
        P, Sq = st.size, st.size * L
        full = None
        if attn is None or save:
            full = SP.qkv_to_heads(qr, kr, v, st)
        if attn is not None:
            ao_full, lse = attn[0].view(Sq, C // P), attn[1].view(nh // P, Sq)
        else:
            ao_full, lse = fwd(full[1], full[2], full[3], nh // P, k_len=meta.seq_len[b],
                               q_log2=True)
        if keep_attn:
            S["attn"] = (ao_full.view(L, C), lse.view(nh, L))
        ao = SP.heads_to_seq(ao_full, st)
        if save:
            S.update(qkv_full=full[0], ao_full=ao_full)
    y1 = torch.empty(L, C, dtype=BF16, device=x.device) if save else None
    x1 = lin(W, "o", ao, epilogue=EPI_RESID, gate=e[2], res=x, aux=y1)
    if save:
        S.update(h1=h1, m1=m1, r1=r1, qkv=qkv, qr=qr, rq=rq, kr=kr, rk=rk, ao=ao, lse=lse, y1=y1,
                 x1=x1)
    else:
        del h1, qkv, qr, kr, ao
    # ---- cross-attention (model.py:352, :204-271) ----
    n3, m3, r3 = ops.ln_mod_fwd(x1, w=g("norm3.weight"), b=g("norm3.bias"), eps=eps)
    qc_raw = lin(W, "cq", n3)
    qc, rqc = ops.rms_rope_fwd(qc_raw, g("cross_attn.norm_q.weight"), eps, out_scale=ops.L2Q_SCALE)
    ctx_t, ctx_i = _split_ctx(ctx, meta.i2v)
    kc_raw = ops.linear(ctx_t, W.wck, W.bck)
    kc, rkc = ops.rms_rope_fwd(kc_raw, g("cross_attn.norm_k.weight"), eps)
    vc = ops.linear(ctx_t, W.wcv, W.bcv)
    ac, lsec = ops.attn_fwd(qc, kc, vc, nh, q_log2=True)
    if meta.i2v:
        ki_raw = ops.linear(ctx_i, W.wck_img, W.bck_img)
        ki, rki = ops.rms_rope_fwd(ki_raw, g("cross_attn.norm_k_img.weight"), eps)
        vi = ops.linear(ctx_i, W.wcv_img, W.bcv_img)
        ai, lsei = ops.attn_fwd(qc, ki, vi, nh, q_log2=True)
        acs = ac + ai          # fp32 sum of two bf16 outputs, rounded once (model.py:269)
    else:
        acs = ac
    x2 = x1 if not save else torch.empty_like(x1)
    lin(W, "co", acs, epilogue=EPI_RESID, out=x2, res=x1)
    if save:
        S.update(n3=n3, m3=m3, r3=r3, qc_raw=qc_raw, qc=qc, rqc=rqc, kc_raw=kc_raw, kc=kc, rkc=rkc,
                 vc=vc, ac=ac, lsec=lsec, acs=acs, x2=x2)
        if meta.i2v:
            S.update(ki_raw=ki_raw, ki=ki, rki=rki, vi=vi, ai=ai, lsei=lsei)
    # ---- FFN (model.py:353-355) ----
    h2, m2, r2 = ops.ln_mod_fwd(x2, scale=e[4], shift=e[3], eps=eps)
    fpre = torch.empty(L, W.w1.shape[0], dtype=BF16, device=x.device) if save else None
    fact = lin(W, "1", h2, epilogue=EPI_GELU, aux=fpre)
    y2 = torch.empty(L, C, dtype=BF16, device=x.device) if save else None
    out = torch.empty_like(x2) if save else x2
    lin(W, "2", fact, epilogue=EPI_RESID, out=out, gate=e[5], res=x2, aux=y2)
    if save:
        S.update(h2=h2, m2=m2, r2=r2, fpre=fpre, fact=fact, y2=y2)
    return out, S


def block_backward_one(P, W, x, e, ctx, meta, b, S, dout, G, want_w=True):
    """Backward of block_forward_one.  dout fp32 [L, C] (consumed/overwritten).  Parameter
    gradients are accumulated into the fp32 dict G (skipped entirely when want_w is False, e.g.
    for the frozen reward-model trunk); returns (dx fp32, de [6, C], dctx fp32)."""
    g = P.__getitem__
    L, C = x.shape
    nh, eps = meta.num_heads, meta.eps
    grid = meta.grid[b]
    de = [None] * 6

    def acc(name, val):
        if not want_w:
            return
        if G.get(name) is None:
            G[name] = val
        else:
            G[name].add_(val)

    def dw(name, dy, xin):
        if not want_w:
            return
        if G.get(name) is None:
            G[name] = ops.linear_dw(dy, xin)
        else:
            ops.linear_dw(dy, xin, out=G[name], accumulate=True)

    dx = dout
    # ---- FFN ----
    dy2, de[5], db2 = ops.gate_bwd(dx, S["y2"], e[5])
    acc("ffn.2.bias", db2)
    dw("ffn.2.weight", dy2, S["fact"])
    dfpre = ops.linear_dx(dy2, W.w2, epilogue=EPI_DGELU, aux=S["fpre"])
    del dy2
    dw("ffn.0.weight", dfpre, S["h2"])
    if want_w:
        acc("ffn.0.bias", ops.colsum(dfpre))
    dh2 = ops.linear_dx(dfpre, W.w1)
    del dfpre
    de[4], de[3] = ops.ln_mod_bwd(dh2, S["x2"], S["m2"], S["r2"], dx, scale=e[4])
    del dh2
    # ---- cross-attention ----
    dyc, _, dbco = ops.gate_bwd(dx, None, None, want_gate=False)
    acc("cross_attn.o.bias", dbco)
    dw("cross_attn.o.weight", dyc, S["acs"])
    dac = ops.linear_dx(dyc, W.wco)
    del dyc
    ctx_t, ctx_i = _split_ctx(ctx, meta.i2v)
    dqc, dkc, dvc = ops.attn_bwd(S["qc"], S["kc"], S["vc"], S["ac"], dac, S["lsec"], nh, q_log2=True)
    if meta.i2v:
        dqi, dki, dvi = ops.attn_bwd(S["qc"], S["ki"], S["vi"], S["ai"], dac, S["lsei"], nh,
                                     q_log2=True)
        dqc = dqc + dqi
    dqc_raw, dnq = ops.rms_rope_bwd(dqc, S["qc_raw"], S["rqc"], g("cross_attn.norm_q.weight"),
                                    out_scale=ops.L2Q_SCALE)
    acc("cross_attn.norm_q.weight", dnq)
    dw("cross_attn.q.weight", dqc_raw, S["n3"])
    if want_w:
        acc("cross_attn.q.bias", ops.colsum(dqc_raw))
    dn3 = ops.linear_dx(dqc_raw, W.wcq)
    dw3, db3 = ops.ln_mod_bwd(dn3, S["x1"], S["m3"], S["r3"], dx, w=g("norm3.weight"))
    acc("norm3.weight", dw3)
    acc("norm3.bias", db3)
    del dn3, dqc_raw
    dkc_raw, dnk = ops.rms_rope_bwd(dkc, S["kc_raw"], S["rkc"], g("cross_attn.norm_k.weight"))
    acc("cross_attn.norm_k.weight", dnk)
    dw("cross_attn.k.weight", dkc_raw, ctx_t)
    if want_w:
        acc("cross_attn.k.bias", ops.colsum(dkc_raw))
    dw("cross_attn.v.weight", dvc, ctx_t)
    if want_w:
        acc("cross_attn.v.bias", ops.colsum(dvc))
    dctx = torch.empty(ctx.shape, dtype=torch.float32, device=x.device)
    n_img = ctx.shape[0] - ctx_t.shape[0]
    dctx_t = dctx[n_img:]
    ops.gemm(dkc_raw, W.wck, dctx_t, ctx_t.shape[0], C, C, True, False, ops.EPI_F32)
    ops.gemm(dvc, W.wcv, dctx_t, ctx_t.shape[0], C, C, True, False, ops.EPI_F32, accumulate=True)
    if meta.i2v:
        dki_raw, dnki = ops.rms_rope_bwd(dki, S["ki_raw"], S["rki"],
                                         g("cross_attn.norm_k_img.weight"))
        acc("cross_attn.norm_k_img.weight", dnki)
        dw("cross_attn.k_img.weight", dki_raw, ctx_i)
        if want_w:
            acc("cross_attn.k_img.bias", ops.colsum(dki_raw))
        dw("cross_attn.v_img.weight", dvi, ctx_i)
        if want_w:
            acc("cross_attn.v_img.bias", ops.colsum(dvi))
        dctx_i = dctx[:n_img]
        ops.gemm(dki_raw, W.wck_img, dctx_i, n_img, C, C, True, False, ops.EPI_F32)
        ops.gemm(dvi, W.wcv_img, dctx_i, n_img, C, C, True, False, ops.EPI_F32, accumulate=True)
    # ---- self-attention ----
    dy1, de[2], dbo = ops.gate_bwd(dx, S["y1"], e[2])
    acc("self_attn.o.bias", dbo)
    dw("self_attn.o.weight", dy1, S["ao"])
    dao = ops.linear_dx(dy1, W.wo)
    del dy1
    qkv = S["qkv"]
    dqkv = torch.empty(L, 3 * C, dtype=BF16, device=x.device)
    st = meta.sp
    if st is None:
        row0 = 0
        dqr, dkr, _ = ops.attn_bwd(S["qr"], S["kr"], qkv[:, 2 * C:], S["ao"], dao, S["lse"], nh,
                                   k_len=meta.seq_len[b], dv=dqkv[:, 2 * C:], q_log2=True)
    else:
        # the inverse exchange: d(out) to this rank's heads, the attention backward over all
        # tokens into one [S, 3, C/P] dq | dk | dv image, back to this rank's tokens
        row0 = st.rank * L
        P = st.size
        dao_full = SP.seq_to_heads(dao, st)
        full = S["qkv_full"]
        dfull = torch.empty_like(full)
        ops.attn_bwd(full[:, 0], full[:, 1], full[:, 2], S["ao_full"], dao_full, S["lse"], nh // P,
                     k_len=meta.seq_len[b], dq=dfull[:, 0], dk=dfull[:, 1], dv=dfull[:, 2],
                     q_log2=True)
        del dao_full
        dqr = torch.empty(L, C, dtype=BF16, device=x.device)
        dkr = torch.empty(L, C, dtype=BF16, device=x.device)
        SP.dqkv_to_seq(dfull, st, dqr, dkr, dqkv[:, 2 * C:])
        del dfull
    del dao
    _, dnq = ops.rms_rope_bwd(dqr, qkv[:, :C], S["rq"], g("self_attn.norm_q.weight"),
                              meta.rope_tab, grid, dx=dqkv[:, :C], out_scale=ops.L2Q_SCALE,
                              row0=row0)
    _, dnk = ops.rms_rope_bwd(dkr, qkv[:, C:2 * C], S["rk"], g("self_attn.norm_k.weight"),
                              meta.rope_tab, grid, dx=dqkv[:, C:2 * C], row0=row0)
    acc("self_attn.norm_q.weight", dnq)
    acc("self_attn.norm_k.weight", dnk)
    del dqr, dkr
    for i, n in enumerate("qkv"):
        dw(f"self_attn.{n}.weight", dqkv[:, i * C:(i + 1) * C], S["h1"])
    if want_w:
        dbqkv = ops.colsum(dqkv)
        for i, n in enumerate("qkv"):
            acc(f"self_attn.{n}.bias", dbqkv[i * C:(i + 1) * C].clone())
    dh1 = ops.gemm(dqkv, W.wqkv, torch.empty(L, C, dtype=BF16, device=x.device), L, C, 3 * C,
                   True, False, EPI_BF16)
    del dqkv
    de[1], de[0] = ops.ln_mod_bwd(dh1, x, S["m1"], S["r1"], dx, scale=e[1])
    return dx, torch.stack(de), dctx


def block_apply(P, x, e, context, meta, allow_keep=True):
    """The fused, checkpointed block through the `prfl::wan_block` custom op (its backward is
    `prfl::wan_block_backward`).  P: name -> fp32 parameter (the block's, without
    'modulation'); x [B, L, C], e [B, 6, C] fp32 (modulation + e0), context [B, Lc, C] bf16.

    The self-attention output / LSE is kept for the backward only when this forward records a
    graph (grad mode on and some input requires grad) and the per-step stash budget has room."""
    from . import custom_ops
    params = [P[n] for n in param_names(meta.i2v)]
    L, C = x.shape[1], x.shape[2]
    need = x.shape[0] * (L * C * 2 + meta.num_heads * L * 4)
    records = torch.is_grad_enabled() and (x.requires_grad or e.requires_grad or
                                           context.requires_grad or
                                           any(p.requires_grad for p in params))
    keep = allow_keep and records and _STASH["left"] >= need
    if keep:
        _STASH["left"] -= need
    grid = [int(v) for g in meta.grid for v in g]
    out, _, _ = custom_ops.wan_block(x, e, context, params, int(meta.num_heads), grid,
                                     [int(v) for v in meta.seq_len], meta.rope_tab, bool(meta.i2v),
                                     float(meta.eps), int(meta.fp8), keep, SP.register(meta.sp))
    return out
