"""Dev A/B of builds of the row-norm kernels in ONE process, interleaved (MI355X guide rule 24):
    python tools/ab_norms.py <lib1.so> <lib2.so> ... [--reps 10]
At the 720p shapes of the fused block (L = 73 920, C = 5120):
  rms_fwd  prfl_rms_rope_fwd_pos on the q slice of a [L, 3C] QKV output, 3-D RoPE, log2 out_scale
           (bytes: read 2 + write 2 per element)
  rms_bwd  prfl_rms_rope_bwd_pos of the same (read dout 2 + x 2, write dx 2; the d w partial rows)
  ln_fwd   prfl_ln_mod_fwd on the fp32 residual stream with (scale, shift) (read 4 + write 2)
  ln_bwd   prfl_ln_mod_bwd of the same, accumulating into an fp32 dx (read dy 2 + x 4 + dx 4, write
           dx 4, accumulated over the repetitions; the two partial column-sum rows)
HIP events on the launch stream; prints medians, GB/s and the largest output difference vs the
first build (bf16 ulps; rstd / partial sums relative)."""
import argparse
import ctypes
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402

P, I64, I32, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
SIGS = {
    "prfl_rms_rope_fwd_pos": [P, I64, I64, I64, P, F32, P, I64, I64, I64, I64, P, I64, P, F32, P],
    "prfl_rms_rope_bwd_pos": [P, I64, P, I64, P, I64, I64, P, P, I64, I64, I64, I64, P, I64, P, F32, P],
    "prfl_ln_mod_fwd": [P, I32, I64, I64, I64, P, P, P, P, F32, P, I64, P, P, P],
    "prfl_ln_mod_bwd": [P, I64, P, I32, I64, P, P, I64, I64, P, P, P, I64, I32, P, P, P],
}


def ulps(a, b):
    return (a.view(torch.int16).int() - b.view(torch.int16).int()).abs().max().item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    libs = []
    for p in a.libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        for n, sig in SIGS.items():
            getattr(lib, n).argtypes, getattr(lib, n).restype = sig, ctypes.c_int
        libs.append(lib)
    from prfl_amd.model import _rope_table, rope_params
    F, Hg, Wg, C = 21, 44, 80, 5120
    L = F * Hg * Wg
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(L, 3 * C, device=dev, generator=g).to(torch.bfloat16)
    dq = torch.randn(L, C, device=dev, generator=g).to(torch.bfloat16)
    w = 1 + 0.1 * torch.randn(C, device=dev, generator=g)
    xres = torch.randn(L, C, device=dev, generator=g)
    sc_, sh_ = 0.1 * torch.randn(C, device=dev, generator=g), 0.1 * torch.randn(C, device=dev, generator=g)
    d = 128
    freqs = torch.cat([rope_params(1024, d - 4 * (d // 6)), rope_params(1024, 2 * (d // 6)),
                       rope_params(1024, 2 * (d // 6))], dim=1)
    tab = _rope_table(freqs, dev)
    n = len(libs)
    o_rf = [torch.empty(L, C, device=dev, dtype=torch.bfloat16) for _ in libs]
    rstd = [torch.empty(L, device=dev) for _ in libs]
    o_rb = [torch.empty(L, C, device=dev, dtype=torch.bfloat16) for _ in libs]
    part = [torch.empty((L + 31) // 32, C, device=dev) for _ in libs]
    o_ln = [torch.empty(L, C, device=dev, dtype=torch.bfloat16) for _ in libs]
    mean_ln = [torch.empty(L, device=dev) for _ in libs]
    rstd_ln = [torch.empty(L, device=dev) for _ in libs]
    dyl = torch.randn(L, C, device=dev, generator=g).to(torch.bfloat16)
    dxl = [torch.zeros(L, C, device=dev) for _ in libs]
    p0l = [torch.empty((L + 31) // 32, C, device=dev) for _ in libs]
    p1l = [torch.empty((L + 31) // 32, C, device=dev) for _ in libs]
    st = torch.cuda.current_stream().cuda_stream
    osc = 1.4426950408889634 / math.sqrt(128)

    def run(i, which):
        lib = libs[i]
        if which == "rms_fwd":
            return lib.prfl_rms_rope_fwd_pos(qkv.data_ptr(), 3 * C, L, C, w.data_ptr(), 1e-6, tab.data_ptr(),
                                             F, Hg, Wg, 0, o_rf[i].data_ptr(), C, rstd[i].data_ptr(), osc, st)
        if which == "rms_bwd":
            return lib.prfl_rms_rope_bwd_pos(dq.data_ptr(), C, qkv.data_ptr(), 3 * C, rstd[0].data_ptr(), L, C,
                                             w.data_ptr(), tab.data_ptr(), F, Hg, Wg, 0, o_rb[i].data_ptr(), C,
                                             part[i].data_ptr(), osc, st)
        if which == "ln_fwd":
            return lib.prfl_ln_mod_fwd(xres.data_ptr(), 0, C, L, C, sc_.data_ptr(), sh_.data_ptr(), None, None,
                                       1e-6, o_ln[i].data_ptr(), C, mean_ln[i].data_ptr(), rstd_ln[i].data_ptr(), st)
        return lib.prfl_ln_mod_bwd(dyl.data_ptr(), C, xres.data_ptr(), 0, C, mean_ln[0].data_ptr(),
                                   rstd_ln[0].data_ptr(), L, C, sc_.data_ptr(), None, dxl[i].data_ptr(), C, 1,
                                   p0l[i].data_ptr(), p1l[i].data_ptr(), st)

    byts = {"rms_fwd": L * C * 4, "rms_bwd": L * C * 6, "ln_fwd": L * C * 6, "ln_bwd": L * C * 14}
    for which in ("rms_fwd", "rms_bwd", "ln_fwd", "ln_bwd"):
        ts = [[] for _ in libs]
        for r in range(a.reps + 1):
            for i in range(n):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = run(i, which)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, (which, rc)
                if r:
                    ts[i].append(e0.elapsed_time(e1))
        meds = [statistics.median(t) for t in ts]
        if which == "rms_fwd":
            diff = [f"{ulps(o_rf[i], o_rf[0])} ulp, rstd {((rstd[i] - rstd[0]).abs() / rstd[0]).max().item():.1e}"
                    for i in range(n)]
        elif which == "rms_bwd":
            diff = [f"{ulps(o_rb[i], o_rb[0])} ulp, dw {((part[i].sum(0) - part[0].sum(0)).norm() / part[0].sum(0).norm()).item():.1e}"
                    for i in range(n)]
        elif which == "ln_fwd":
            diff = [f"{ulps(o_ln[i], o_ln[0])} ulp" for i in range(n)]
        else:
            diff = [f"dx {((dxl[i] - dxl[0]).norm() / dxl[0].norm()).item():.1e}, d scale "
                    f"{((p0l[i].sum(0) - p0l[0].sum(0)).norm() / p0l[0].sum(0).norm()).item():.1e}" for i in range(n)]
        print(f"{which} 720p: " + " | ".join(
            f"lib{i} {m:.3f} ms {byts[which] / m / 1e6:.0f} GB/s ({dd})" for i, (m, dd) in enumerate(zip(meds, diff))),
            flush=True)


if __name__ == "__main__":
    main()
