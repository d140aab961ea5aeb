"""Dev probe: the 720p block GEMMs through prfl_gemm (ops.linear / linear_dx / linear_dw) next to
torch.matmul (hipBLASLt) on the same operands, interleaved, HIP events on the current stream.
    python tools/gemm_vs_blaslt.py [reps]
Prints per shape and pass the median ms and TF/s of both and the ratio; the torch column is a
ceiling reference only (the product path never calls it).  The forward rows run the shipped path
(ops.linear_t on the W^T weight image, with the block's epilogues: +bias, gated residual on the
o / FFN-down shapes, GELU + pre-activation on FFN-up) against hipBLASLt's plain x @ W^T."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
L, C, F = int(os.environ.get("PRFL_PROF_L", 73920)), 5120, 13824
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def timeit(fn):
    ts = []
    for i in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


for name, N, K in [("qkv", 3 * C, C), ("o", C, C), ("ffn1", F, C), ("ffn2", C, F)]:
    x = torch.randn(L, K, device=dev, generator=g).to(torch.bfloat16)
    w32 = torch.randn(N, K, device=dev, generator=g) * 0.02
    w = w32.to(torch.bfloat16)
    wt = ops.cast_bf16_t(w32)                      # the shipped forward's W^T operand
    bias = (0.02 * torch.randn(N, device=dev, generator=g)).to(torch.bfloat16)
    dy = (torch.randn(L, N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    y = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
    aux = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
    res = torch.randn(L, N, device=dev, generator=g)
    gate = torch.randn(N, device=dev, generator=g)
    dx = torch.empty(L, K, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(N, K, device=dev)                 # prfl accumulates dW in fp32
    dwb = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    fl = 2 * L * N * K
    blaslt_fwd = lambda: torch.matmul(x, w.t(), out=y)  # noqa: E731
    cases = [("fwd W^T +bias", lambda: ops.linear_t(x, wt, bias, out=y), blaslt_fwd)]
    if name in ("o", "ffn2"):      # the block's gated-residual projections (x + y * gate, y kept)
        cases.append(("fwd W^T resid", lambda: ops.linear_t(x, wt, bias, ops.EPI_RESID, out=res,
                                                            gate=gate, res=res, aux=aux), blaslt_fwd))
    if name == "ffn1":             # FFN-up: GELU + the pre-activation kept for the backward
        cases.append(("fwd W^T gelu", lambda: ops.linear_t(x, wt, bias, ops.EPI_GELU, out=y, aux=aux),
                      blaslt_fwd))
    cases += [("dx", lambda: ops.linear_dx(dy, w, out=dx), lambda: torch.matmul(dy, w, out=dx)),
              ("dw", lambda: ops.linear_dw(dy, x, out=dw), lambda: torch.matmul(dy.t(), x, out=dwb))]
    for pas, ours, ref in cases:
        a, b = timeit(ours), timeit(ref)
        print(f"{name:5s} {pas:14s} M={L} N={N} K={K}: prfl {a:7.2f} ms {fl / a / 1e9:5.0f} TF/s | "
              f"hipBLASLt {b:7.2f} ms {fl / b / 1e9:5.0f} TF/s | prfl/blaslt time {a / b:.3f}",
              flush=True)
    del x, w, w32, wt, dy, y, aux, res, dx, dw, dwb
