"""Dev A/B of several builds of the GEMM in ONE process, interleaved (guide §5.4 rule 24):
    python tools/ab_gemm_libs.py <tile> <lib1.so> <lib2.so> ... [--reps R] [--shapes qkv,ffn2]
Each build is called through prfl_gemm_bf16_tiled with the given tile code on the 720p block
GEMMs (fwd, dX, dW); prints per-build medians and checks all builds' outputs are bit-identical."""
import argparse
import ctypes
import os
import statistics

import torch

P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
SIG = [P, I64, I32, P, I64, I32, P, I64, I64, I64, I64, I32, P, P, P, I64, I32, P, I64, I32, I32, P]


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.prfl_gemm_bf16_tiled.argtypes, lib.prfl_gemm_bf16_tiled.restype = SIG, ctypes.c_int
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tile", type=int)
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shapes", default="qkv,o,ffn1,ffn2")
    ap.add_argument("--passes", default="fwd,dx,dw")
    ap.add_argument("--tiles", default=None, help="per-lib tile codes, comma separated")
    ap.add_argument("--bias", action="store_true", help="the forward passes on W^T with a bf16 bias (the "
                    "block's projections all have one)")
    a = ap.parse_args()
    libs = [load(p) for p in a.libs]
    tiles = [int(t) for t in a.tiles.split(",")] if a.tiles else [a.tile] * len(libs)
    tile_of = {id(lib): t for lib, t in zip(libs, tiles)}
    L, C, F = 73920, 5120, 13824
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    shapes = {"qkv": (3 * C, C), "o": (C, C), "ffn1": (F, C), "ffn2": (C, F)}
    for name in a.shapes.split(","):
        N, K = shapes[name]
        x = torch.randn(L, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        dy = (torch.randn(L, N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        outs = [dict(fwd=torch.empty(L, N, device=dev, dtype=torch.bfloat16),
                     dx=torch.empty(L, K, device=dev, dtype=torch.bfloat16),
                     dw=torch.empty(N, K, device=dev)) for _ in libs]
        fl = 2 * L * N * K

        wt = w.t().contiguous()     # [K, N]: the weight as an MN-major B operand

        def call(lib, o, pas):
            if pas.endswith("_t"):    # forward passes on the transposed weight (MN-major B)
                # residna_t: the gated residual without the saved y (the no-grad rollout's form)
                epi = {"fwd_t": 0, "gelu_t": 1, "resid_t": 2, "residna_t": 2}[pas]
                rc = lib.prfl_gemm_bf16_tiled(x.data_ptr(), K, 1, wt.data_ptr(), N, 0, o.data_ptr(), N, L, N, K,
                                              epi, bias.data_ptr() if a.bias else None,
                                              gate.data_ptr() if epi == 2 else None,
                                              res.data_ptr() if epi == 2 else None, N, 0,
                                              aux.data_ptr() if epi and pas != "residna_t" else None, N, 0,
                                              tile_of[id(lib)], st)
                assert rc == 0, rc
                return
            if pas == "fwd":   # y[L,N] = x[L,K] w[N,K]^T
                args = (x.data_ptr(), K, 1, w.data_ptr(), K, 1, o.data_ptr(), N, L, N, K, 0)
            elif pas == "dx":  # dx[L,K] = dy[L,N] w[N,K]
                args = (dy.data_ptr(), N, 1, w.data_ptr(), K, 0, o.data_ptr(), K, L, K, N, 0)
            elif pas == "gelu":   # FFN-up: GELU epilogue, pre-activation to aux
                rc = lib.prfl_gemm_bf16_tiled(x.data_ptr(), K, 1, w.data_ptr(), K, 1, o.data_ptr(), N, L, N, K, 1,
                                              None, None, None, 0, 0, aux.data_ptr(), N, 0, tile_of[id(lib)], st)
                assert rc == 0, rc
                return
            elif pas == "resid":  # o-proj / FFN-down: x + bf16(y) * gate (fp32), y to aux
                rc = lib.prfl_gemm_bf16_tiled(x.data_ptr(), K, 1, w.data_ptr(), K, 1, o.data_ptr(), N, L, N, K, 2,
                                              None, gate.data_ptr(), res.data_ptr(), N, 0, aux.data_ptr(), N, 0,
                                              tile_of[id(lib)], st)
                assert rc == 0, rc
                return
            elif pas == "dgelu":  # FFN-up backward: dX through the GELU derivative of aux
                rc = lib.prfl_gemm_bf16_tiled(dy.data_ptr(), N, 1, w.data_ptr(), K, 0, o.data_ptr(), K, L, K, N, 4,
                                              None, None, None, 0, 0, pre_k.data_ptr(), K, 0,
                                              tile_of[id(lib)], st)
                assert rc == 0, rc
                return
            elif pas == "dwacc":  # weight grad accumulated into fp32 .grad
                rc = lib.prfl_gemm_bf16_tiled(dy.data_ptr(), N, 0, x.data_ptr(), K, 0, o.data_ptr(), K, N, K, L, 3,
                                              None, None, None, 0, 0, None, 0, 1, tile_of[id(lib)], st)
                assert rc == 0, rc
                return
            else:              # dw[N,K] = dy^T x (fp32)
                args = (dy.data_ptr(), N, 0, x.data_ptr(), K, 0, o.data_ptr(), K, N, K, L, 3)
            rc = lib.prfl_gemm_bf16_tiled(*args, None, None, None, 0, 0, None, 0, 0, tile_of[id(lib)], st)
            assert rc == 0, rc

        gate = torch.randn(N, device=dev, generator=g)
        bias = (torch.randn(N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        res = torch.randn(L, N, device=dev, generator=g)
        aux = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
        pre_k = torch.randn(L, K, device=dev, generator=g).to(torch.bfloat16)
        for o in outs:
            o["dgelu"] = torch.empty(L, K, device=dev, dtype=torch.bfloat16)
            o["gelu"] = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
            o["resid"] = torch.empty(L, N, device=dev)
            o["dwacc"] = torch.zeros(N, K, device=dev)
            o["fwd_t"] = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
            o["gelu_t"] = torch.empty(L, N, device=dev, dtype=torch.bfloat16)
            o["resid_t"] = torch.empty(L, N, device=dev)
            o["residna_t"] = torch.empty(L, N, device=dev)
        for pas in a.passes.split(","):
            ts = [[] for _ in libs]
            for r in range(a.reps + 1):
                for i, lib in enumerate(libs):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    call(lib, outs[i][pas], pas)
                    e1.record()
                    torch.cuda.synchronize()
                    if r:
                        ts[i].append(e0.elapsed_time(e1))
            same = all(torch.equal(outs[0][pas], o[pas]) for o in outs[1:]) if pas != "dwacc" else "n/a"
            if same is False:      # different MFMA shapes round differently: report how far
                r0 = outs[0][pas].float()
                same = "rel " + ",".join(f"{((o[pas].float() - r0).norm() / r0.norm()).item():.1e}"
                                         for o in outs[1:])
            meds = [statistics.median(t) for t in ts]
            print(f"{name:5s} {pas:3s}: " + " | ".join(f"lib{i} {m:6.2f} ms {fl / m / 1e9:5.0f} TF/s"
                                                       for i, m in enumerate(meds))
                  + f" | identical {same}", flush=True)
        for pa, pb in (("fwd", "fwd_t"), ("gelu", "gelu_t"), ("resid", "resid_t")):
            if pa in a.passes.split(",") and pb in a.passes.split(","):
                print(f"{name:5s} {pa} vs {pb}: identical {torch.equal(outs[0][pa], outs[0][pb])}", flush=True)
        del x, w, dy, outs


if __name__ == "__main__":
    main()
