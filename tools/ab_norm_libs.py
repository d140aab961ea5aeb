"""Dev A/B of builds of the RMSNorm+RoPE forward in ONE process, interleaved:
    python tools/ab_norm_libs.py <lib1.so> <lib2.so> ... [--reps 10]
prfl_rms_rope_fwd_scaled at the 720p self-attention q shape (L = 73 920 rows of a [L, 3C] QKV output,
C = 5120, 3-D RoPE over the 21 x 44 x 80 grid, out_scale = scale * log2 e), HIP events on the
launch stream; prints medians, GB/s (read 2 B + write 2 B per element) and the largest output
difference vs the first build in bf16 ulps."""
import argparse
import ctypes
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402

P, I64, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float
SIG = [P, I64, I64, I64, P, F32, P, I64, I64, I64, P, I64, P, F32, P]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    libs = []
    for p in a.libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        lib.prfl_rms_rope_fwd_scaled.argtypes, lib.prfl_rms_rope_fwd_scaled.restype = SIG, ctypes.c_int
        libs.append(lib)
    from prfl_amd import ops
    from prfl_amd.model import _rope_table, rope_params
    F, Hg, Wg, C = 21, 44, 80, 5120
    L = F * Hg * Wg
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(L, 3 * C, device=dev, generator=g).to(torch.bfloat16)
    w = 1 + 0.1 * torch.randn(C, device=dev, generator=g)
    d = 128
    freqs = torch.cat([rope_params(1024, d - 4 * (d // 6)), rope_params(1024, 2 * (d // 6)),
                       rope_params(1024, 2 * (d // 6))], dim=1)
    tab = _rope_table(freqs, dev)
    outs = [torch.empty(L, C, device=dev, dtype=torch.bfloat16) for _ in libs]
    rstd = [torch.empty(L, device=dev) for _ in libs]
    st = torch.cuda.current_stream().cuda_stream
    sc = 1.4426950408889634 / math.sqrt(128)
    ts = [[] for _ in libs]
    for r in range(a.reps + 1):
        for i, lib in enumerate(libs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.prfl_rms_rope_fwd_scaled(qkv.data_ptr(), 3 * C, L, C, w.data_ptr(), 1e-6, tab.data_ptr(),
                                       F, Hg, Wg, outs[i].data_ptr(), C, rstd[i].data_ptr(), sc, st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            if r:
                ts[i].append(e0.elapsed_time(e1))
    meds = [statistics.median(t) for t in ts]
    byt = L * C * 4
    ulp = [((o.view(torch.int16).int() - outs[0].view(torch.int16).int()).abs().max().item()) for o in outs]
    print("rms_rope_fwd 720p q: " + " | ".join(f"lib{i} {m:.3f} ms {byt / m / 1e6:.0f} GB/s (max {u} ulp)"
                                             for i, (m, u) in enumerate(zip(meds, ulp))), flush=True)


if __name__ == "__main__":
    main()
