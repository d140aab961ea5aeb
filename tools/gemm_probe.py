"""Dev probe: where the 256x256 GEMM's time goes at the 720p QKV shape (M=73920, N=15360,
K=5120).  Interleaved variants on random bf16 data:
  full    : the real operands (A 757 MB, B 157 MB)
  smallA  : A rows overlapping (lda = 64: every row distinct, 9.5 MB footprint, L2/MALL-resident)
  smallAB : both operands overlapping (lda = ldb = 64)
  kx4     : K = 20480 (prologue / epilogue amortised 4x; TF/s compared)
    python tools/gemm_probe.py [reps]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
M, N, K = 73920, 15360, 5120
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def rnd(n, s=1.0):
    return (torch.randn(n, device=dev, generator=g) * s).to(torch.bfloat16)


A = rnd(M * K).view(M, K)
B = rnd(N * K, 0.02).view(N, K)
As = torch.as_strided(rnd(M * 64 + K), (M, K), (64, 1))
Bs = torch.as_strided(rnd(N * 64 + K, 0.02), (N, K), (64, 1))
M4 = M // 4
A4 = torch.as_strided(A, (M4, 4 * K), (4 * K, 1))
B4 = torch.as_strided(rnd(N * 4 * K, 0.02), (N, 4 * K), (4 * K, 1))
C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
C4 = torch.empty(M4, N, device=dev, dtype=torch.bfloat16)
cases = {
    "full": (lambda: ops.gemm(A, B, C, M, N, K), 2 * M * N * K),
    "smallA": (lambda: ops.gemm(As, B, C, M, N, K), 2 * M * N * K),
    "smallAB": (lambda: ops.gemm(As, Bs, C, M, N, K), 2 * M * N * K),
    "kx4": (lambda: ops.gemm(A4, B4, C4, M4, N, 4 * K), 2 * M4 * N * 4 * K),
}
times = {k: [] for k in cases}
for r in range(reps + 1):
    for name, (fn, fl) in cases.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if r:
            times[name].append(e0.elapsed_time(e1))
for name, (fn, fl) in cases.items():
    t = statistics.median(times[name])
    print(f"{name:8s} {t:7.2f} ms  {fl / t / 1e9:5.0f} TF/s", flush=True)
