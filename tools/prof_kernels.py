"""Dev probe: isolated hot kernels at the 480p x 81f shapes (L = 32760, C = 5120, 40 heads),
for rocprofv3 counter runs.  usage: python tools/prof_kernels.py [attn|attn_fp8|gemm|attn_bwd] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd import ops  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "attn"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
L, C, NH, F = int(os.environ.get("PRFL_PROF_L", 32760)), 5120, 40, 13824
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
if which == "attn_fp8":
    # config C5 self-attention forward (prologue + attn_fwd_lp_kernel)
    qkv = torch.randn(L, 3 * C, device=dev, generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    fl = 4 * L * L * C
    for i in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.time()
        ops.attn_fwd_fp8(q, k, v, NH)
        torch.cuda.synchronize()
        dt = time.time() - t0
        print(f"attn_fp8 {dt*1e3:.2f} ms  {fl/dt/1e12:.0f} TF/s", flush=True)
elif which in ("attn", "attn_bwd", "attn_l2q", "attn_bwd_l2q"):
    # *_l2q: the fused block's path (q in log2 units, prfl_attn_*_l2q entries)
    l2 = which.endswith("_l2q")
    which = which.replace("_l2q", "")
    qkv = torch.randn(L, 3 * C, device=dev, generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    if l2:
        q = (q.float() * ops.L2Q_SCALE).to(torch.bfloat16)
    o, lse = ops.attn_fwd(q, k, v, NH, q_log2=l2)
    do = torch.randn(L, C, device=dev, generator=g).to(torch.bfloat16)
    fl = 4 * L * L * C
    for i in range(reps):
        torch.cuda.synchronize()
        t0 = time.time()
        if which == "attn":
            ops.attn_fwd(q, k, v, NH, out=o, q_log2=l2)
        else:
            ops.attn_bwd(q, k, v, o, do, lse, NH, q_log2=l2)
        torch.cuda.synchronize()
        dt = time.time() - t0
        print(f"{which} {dt*1e3:.2f} ms  {fl*(1 if which=='attn' else 2.5)/dt/1e12:.0f} TF/s", flush=True)
    ops.prof_enable(True)
    if which == "attn":
        ops.attn_fwd(q, k, v, NH, out=o, q_log2=l2)
    else:
        ops.attn_bwd(q, k, v, o, do, lse, NH, q_log2=l2)
    torch.cuda.synchronize()
    ops.prof_enable(False)
    for kname, d in ops.prof_collect().items():
        if d["count"]:
            print(f"  {kname}: {d['ms']:.2f} ms  {d['work'] / (d['ms'] * 1e-3) / 1e12:.0f} TF/s", flush=True)
elif which == "ln":
    # LN + AdaLN modulate forward at L tokens (fp32 residual in, bf16 out), and the affine norm3
    x = torch.randn(L, C, device=dev, generator=g)
    sc, sh = 0.1 * torch.randn(C, device=dev, generator=g), 0.1 * torch.randn(C, device=dev, generator=g)
    for name, kw in (("mod", dict(scale=sc, shift=sh)), ("affine", dict(w=1 + sc, b=sh))):
        y, m, r = ops.ln_mod_fwd(x, **kw)
        torch.cuda.synchronize()
        t0 = time.time()
        for i in range(reps):
            ops.ln_mod_fwd(x, out=y, **kw)
        torch.cuda.synchronize()
        dt = (time.time() - t0) / reps
        ck = (y.double().sum().item(), y.double().abs().sum().item(), m.double().sum().item(),
              r.double().sum().item())
        print(f"ln_mod_fwd {name} {L}x{C}: {dt*1e3:.3f} ms  {L*C*6/dt/1e9:.0f} GB/s  checksum {ck}",
              flush=True)
elif which == "gemm720":
    # one dispatch per GEMM of a 720p block's forward + backward (the bench's shapes), for PMC runs
    Lq = L
    shapes = [("qkv", Lq, 3 * C, C), ("o", Lq, C, C), ("ffn1", Lq, F, C), ("ffn2", Lq, C, F)]
    for name, M, N, K in shapes:
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        for i in range(reps):
            torch.cuda.synchronize()
            t0 = time.time()
            y = ops.linear(x, w)
            torch.cuda.synchronize()
            dt = time.time() - t0
            print(f"gemm fwd {name} {M}x{N}x{K} {dt*1e3:.2f} ms  {2*M*N*K/dt/1e12:.0f} TF/s", flush=True)
        dy = (torch.randn(M, N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        for i in range(reps):
            torch.cuda.synchronize()
            t0 = time.time()
            ops.linear_dx(dy, w)
            torch.cuda.synchronize()
            dt = time.time() - t0
            print(f"gemm dx  {name} {M}x{K}x{N} {dt*1e3:.2f} ms  {2*M*N*K/dt/1e12:.0f} TF/s", flush=True)
            torch.cuda.synchronize()
            t0 = time.time()
            ops.linear_dw(dy, x)
            torch.cuda.synchronize()
            dt = time.time() - t0
            print(f"gemm dw  {name} {N}x{K}x{M} {dt*1e3:.2f} ms  {2*M*N*K/dt/1e12:.0f} TF/s", flush=True)
        del x, w, y, dy
elif which == "gemmepi":
    # the fused-epilogue forward GEMMs of a 720p block (o-proj gated residual, FFN-up GELU with
    # the pre-activation store, FFN-down gated residual), one dispatch each per rep, for PMC runs
    for name, N, K, epi in (("o_resid", C, C, ops.EPI_RESID), ("ffn1_gelu", F, C, ops.EPI_GELU),
                            ("ffn2_resid", C, F, ops.EPI_RESID)):
        x = torch.randn(L, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        aux = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
        if epi == ops.EPI_RESID:
            res = torch.randn(L, N, device=dev, generator=g)
            gate = torch.randn(N, device=dev, generator=g)
            kw = dict(gate=gate, res=res, aux=aux)
        else:
            kw = dict(aux=aux)
        for i in range(reps):
            torch.cuda.synchronize()
            t0 = time.time()
            ops.linear(x, w, None, epi, **kw)
            torch.cuda.synchronize()
            dt = time.time() - t0
            print(f"gemm {name} {L}x{N}x{K} {dt*1e3:.2f} ms  {2*L*N*K/dt/1e12:.0f} TF/s", flush=True)
        del x, w, aux, kw
elif which == "gemm720t":
    # the SHIPPED GEMMs of a 720p block, one dispatch each per rep, for PMC runs: forward on the
    # W^T image (gemm4w_kernel<true,false,EPI>: QKV +bias, o-proj / FFN-down gated residual,
    # FFN-up GELU), dX (gemm4w_kernel<true,false,EPI_BF16>), dW (gemm4x_kernel<false,false,F32>)
    for name, N, K, epi in (("qkv", 3 * C, C, ops.EPI_BF16), ("o_resid", C, C, ops.EPI_RESID),
                            ("ffn1_gelu", F, C, ops.EPI_GELU), ("ffn2_resid", C, F, ops.EPI_RESID)):
        x = torch.randn(L, K, device=dev, generator=g).to(torch.bfloat16)
        w32 = torch.randn(N, K, device=dev, generator=g) * 0.02
        wt, w = ops.cast_bf16_t(w32), w32.to(torch.bfloat16)
        bias = (0.02 * torch.randn(N, device=dev, generator=g)).to(torch.bfloat16)
        aux = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
        kw = {}
        if epi == ops.EPI_RESID:
            res = torch.randn(L, N, device=dev, generator=g)
            kw = dict(gate=torch.randn(N, device=dev, generator=g), res=res, aux=aux, out=res)
        elif epi == ops.EPI_GELU:
            kw = dict(aux=aux)
        dy = (torch.randn(L, N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        for i in range(reps):
            for pas, fn in (("fwd", lambda: ops.linear_t(x, wt, bias, epi, **kw)),
                            ("dx", lambda: ops.linear_dx(dy, w)), ("dw", lambda: ops.linear_dw(dy, x))):
                torch.cuda.synchronize()
                t0 = time.time()
                fn()
                torch.cuda.synchronize()
                dt = time.time() - t0
                print(f"gemm {pas} {name} {L}x{N}x{K} {dt*1e3:.2f} ms  {2*L*N*K/dt/1e12:.0f} TF/s",
                      flush=True)
        del x, w32, wt, w, aux, kw, dy
elif which == "gemmcmp":
    # the QKV forward GEMM through prfl_gemm and through torch.matmul (hipBLASLt), same operands:
    # PMC comparison of MFMA busy, clock (GRBM_GUI_ACTIVE / 8 / wall) and instruction mix
    x = torch.randn(L, C, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(3 * C, C, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    y = torch.empty(L, 3 * C, device=dev, dtype=torch.bfloat16)
    tile = int(os.environ.get("PRFL_GEMM_TILE", 0))
    for i in range(reps):
        ops.linear(x, w, out=y, tile=tile)
        torch.matmul(x, w.t(), out=y)
    torch.cuda.synchronize()
    print("gemmcmp done", flush=True)
elif which == "gemmfwd":
    # the forward projections of one block at L tokens (the rollout's hot GEMMs), bf16 epilogue
    for (N, K, name) in [(3 * C, C, "qkv"), (C, C, "o/cq/co"), (F, C, "ffn1"), (C, F, "ffn2")]:
        x = torch.randn(L, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        y = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
        ops.linear(x, w, out=y)
        torch.cuda.synchronize()
        t0 = time.time()
        for i in range(reps):
            ops.linear(x, w, out=y)
        torch.cuda.synchronize()
        dt = (time.time() - t0) / reps
        print(f"gemm {name} {L}x{N}x{K} {dt*1e3:.2f} ms  {2*L*N*K/dt/1e12:.0f} TF/s", flush=True)
        # the fp8 path (C5): per-row quantisation of x + block-scaled fp8 MFMA GEMM
        wq, ws = ops.quant_rows_fp8(w)
        xq, xs = ops.quant_rows_fp8(x)
        ops.linear_fp8(xq, xs, wq, ws, out=y)
        torch.cuda.synchronize()
        t0 = time.time()
        for i in range(reps):
            ops.linear_fp8(xq, xs, wq, ws, out=y)
        torch.cuda.synchronize()
        dt8 = (time.time() - t0) / reps
        t0 = time.time()
        for i in range(reps):
            ops.quant_rows_fp8(x, xq, xs)
        torch.cuda.synchronize()
        dtq = (time.time() - t0) / reps
        print(f"  fp8 {dt8*1e3:.2f} ms  {2*L*N*K/dt8/1e12:.0f} TF/s;  quant x {dtq*1e3:.2f} ms "
              f"({L*K*3/dtq/1e9:.0f} GB/s)", flush=True)
        del x, w, y, wq, xq
else:
    x = torch.randn(L, C, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(F, C, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    dy = (torch.randn(L, F, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    cases = {"fwd": lambda: ops.linear(x, w), "dx": lambda: ops.linear_dx(dy, w),
             "dw": lambda: ops.linear_dw(dy, x)}
    # spot check against torch on a 256-row slice of the output
    y = ops.linear(x, w).float()
    ref = x[:256].float() @ w.float().t()
    print("fwd rel err", ((y[:256] - ref).norm() / ref.norm()).item())
    dx = ops.linear_dx(dy, w).float()
    ref = dy[:256].float() @ w.float()
    print("dx rel err", ((dx[:256] - ref).norm() / ref.norm()).item())
    dw = ops.linear_dw(dy, x)
    ref = dy[:, :256].float().t() @ x.float()
    print("dw rel err", ((dw[:256] - ref).norm() / ref.norm()).item(), flush=True)
    for name, fn in cases.items():
        for i in range(reps):
            torch.cuda.synchronize()
            t0 = time.time()
            fn()
            torch.cuda.synchronize()
            dt = time.time() - t0
            print(f"gemm {name} {L}x{F}x{C} {dt*1e3:.2f} ms  {2*L*F*C/dt/1e12:.0f} TF/s", flush=True)
