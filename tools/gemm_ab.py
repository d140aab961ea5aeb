"""Dev A/B: the 720p block GEMMs through two prfl_gemm kernels (tile codes, e.g. 0 = shipped
dispatch, 4 = four-wave 256x256), interleaved, HIP events; checks bit-identical outputs.
    python tools/gemm_ab.py [tileA] [tileB] [reps]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd import ops  # noqa: E402

ta = int(sys.argv[1]) if len(sys.argv) > 1 else 0
tb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
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
    w = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    dy = (torch.randn(L, N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    outs = {t: (torch.empty(L, N, device=dev, dtype=torch.bfloat16),
                torch.empty(L, K, device=dev, dtype=torch.bfloat16),
                torch.empty(N, K, device=dev)) for t in (ta, tb)}
    fl = 2 * L * N * K
    passes = {
        "fwd": lambda t: ops.gemm(x, w, outs[t][0], L, N, K, True, True, tile=t),
        "dx": lambda t: ops.gemm(dy, w, outs[t][1], L, K, N, True, False, tile=t),
        "dw": lambda t: ops.gemm(dy, x, outs[t][2], N, K, L, False, False, ops.EPI_F32, tile=t),
    }
    for pas, fn in passes.items():
        a, b = timeit(lambda: fn(ta)), timeit(lambda: fn(tb))
        i = {"fwd": 0, "dx": 1, "dw": 2}[pas]
        same = torch.equal(outs[ta][i], outs[tb][i])
        err = ((outs[ta][i].float() - outs[tb][i].float()).abs().max().item())
        print(f"{name:5s} {pas:3s}: tile{ta} {a:7.2f} ms {fl / a / 1e9:5.0f} TF/s | tile{tb} {b:7.2f} ms "
              f"{fl / b / 1e9:5.0f} TF/s | A/B time {a / b:.3f} | bit-identical {same} (max diff {err:.3g})",
              flush=True)
    del x, w, dy, outs
