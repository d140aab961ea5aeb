"""Is the gated-residual epilogue's cost chip-bandwidth-bound or per-CU latency-bound?
    python tools/gemm_epi_probe.py [lib.so ...]
The forward GEMM on W^T (gemm4w_kernel, K = 5120) on grids of 32 ... 256 tiles (one tile per CU
at most: every tile's epilogue runs at the same moment) and of 5 760 tiles (the 720p o-projection):
plain (bf16 out) vs gated residual (fp32 residual in, fp32 out, bf16 aux out).  Per-tile excess
time constant in the tile count = latency-bound per CU; growing with it = the chip's bandwidth."""
import os
import statistics
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd import ops  # noqa: E402


def timeit(fn, reps=30):
    ts = []
    for _ in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts[3:])


K = 5120
g = torch.Generator(device="cuda").manual_seed(0)
for tm, tn in ((8, 4), (8, 8), (16, 8), (16, 16), (288, 20)):
    M, N = 256 * tm, 256 * tn
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    wt = (torch.randn(K, N, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    gate = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, N, device="cuda", generator=g)
    out_b = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    out_f = torch.empty(M, N, device="cuda")
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    reps = 30 if tm * tn <= 256 else 8
    def run(epi, out, **kw):   # tile 256 forced: gemm4w_kernel on every grid
        return lambda: ops.gemm(x, wt, out, M, N, K, True, False, epi, tile=256, **kw)
    t_plain = timeit(run(ops.EPI_BF16, out_b), reps)
    t_gelu = timeit(run(ops.EPI_GELU, out_b, aux=aux), reps)
    t_res = timeit(run(ops.EPI_RESID, out_f, gate=gate, res=res, aux=aux), reps)
    # attribution: fp32 output alone, the residual without its bf16 y output, a bf16 residual,
    # the in-place residual (out = res, as the block runs it)
    t_f32 = timeit(run(ops.EPI_F32, out_f), reps)
    t_noaux = timeit(run(ops.EPI_RESID, out_f, gate=gate, res=res), reps)
    res16 = res.to(torch.bfloat16)
    t_r16 = timeit(run(ops.EPI_RESID, out_f, gate=gate, res=res16, aux=aux), reps)
    t_inpl = timeit(run(ops.EPI_RESID, res, gate=gate, res=res, aux=aux), reps)
    nt = tm * tn
    waves = -(-nt // 256)
    d = lambda t: (t - t_plain) * 1e3 / waves  # noqa: E731
    print(f"tiles {nt:5d} ({waves:2d} waves): plain {t_plain * 1e3:7.1f} us; extra per wave of tiles: "
          f"GELU {d(t_gelu):5.1f}, resid {d(t_res):5.1f}, fp32 out {d(t_f32):5.1f}, resid w/o y "
          f"{d(t_noaux):5.1f}, bf16 residual {d(t_r16):5.1f}, in place {d(t_inpl):5.1f} us", flush=True)
    del x, wt, res, out_b, out_f, aux, res16
