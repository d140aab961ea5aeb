"""Dev probe: does the K-major operand's 64-B DMA row run cost the four-wave GEMM its issue slots?
The same product C = X W^T at the 720p forward shapes with X as a K-major operand (token-major
[L, K]: 16 rows x 64 B per 1-KiB LDS-DMA piece of a 32-deep slice) and as an MN-major operand
(X^T [K, L]: 4 rows x 256 B per piece), W on the W^T image (MN-major) in both; same kernel
(gemm4w_kernel<A_KC, false, EPI_BF16>), same k order (outputs bit-identical), interleaved reps.
    python tools/gemm_run_probe.py [reps]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
# L = 73 728 = 288 x 256: an MN-major A needs whole 256-row tiles (720p: 73 920)
L, C, F = int(os.environ.get("PRFL_PROF_L", 73728)), 5120, 13824
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
for name, N, K in [("qkv", 3 * C, C), ("o", C, C), ("ffn1", F, C), ("ffn2", C, F)]:
    x = torch.randn(L, K, device=dev, generator=g).to(torch.bfloat16)
    xt = x.t().contiguous()
    wt = (torch.randn(K, N, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    ya = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
    yb = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
    runs = {"A K-major": lambda: ops.gemm(x, wt, ya, L, N, K, True, False),
            "A MN-major": lambda: ops.gemm(xt, wt, yb, L, N, K, False, False)}
    ts = {k: [] for k in runs}
    for r in range(reps + 1):
        for k, fn in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts[k].append(e0.elapsed_time(e1))
    fl = 2 * L * N * K
    print(f"{name:5s} M={L} N={N} K={K}: " + " | ".join(
        f"{k} {statistics.median(v):.3f} ms {fl / statistics.median(v) / 1e9:.0f} TF/s"
        for k, v in ts.items()) + f" | identical {torch.equal(ya, yb)}", flush=True)
    del x, xt, wt, ya, yb
