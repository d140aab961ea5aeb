"""A/B of two builds of the attention kernels in ONE process, interleaved (guide §5.4 rule 24):
    python tools/ab_attn.py <libA.so> <libB.so> [L] [rounds]
Times prfl_attn_fwd / prfl_attn_bwd at L tokens, 40 heads (720p: L = 73 920) with HIP events on
the launch stream, checks that both builds give bit-identical outputs, and prints per-round
times and the medians."""
import ctypes
import os
import statistics
import sys

import torch

P, I64, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float
FWD = [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, I64, I64, I64, F32, P]
BWD = [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, P, P, I64, I64, P, I64,
       I64, P, I64, I64, I64, I64, I64, I64, I64, F32, P]


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.prfl_attn_fwd.argtypes, lib.prfl_attn_fwd.restype = FWD, ctypes.c_int
    lib.prfl_attn_bwd.argtypes, lib.prfl_attn_bwd.restype = BWD, ctypes.c_int
    lib.has_ws = hasattr(lib, "prfl_attn_fwd_ws")
    if lib.has_ws:   # split-KV tail builds: forward with a caller-owned workspace
        lib.prfl_attn_fwd_ws.argtypes, lib.prfl_attn_fwd_ws.restype = FWD[:-1] + [P, I64, P], ctypes.c_int
        lib.prfl_attn_fwd_ws_bytes.argtypes = [I64] * 5
        lib.prfl_attn_fwd_ws_bytes.restype = I64
    if hasattr(lib, "prfl_attn_fwd_fp8"):
        lib.prfl_attn_fwd_fp8.argtypes, lib.prfl_attn_fwd_fp8.restype = FWD[:-1] + [P, I64, P], ctypes.c_int
        lib.prfl_attn_fwd_fp8_ws_bytes.argtypes = [I64] * 5
        lib.prfl_attn_fwd_fp8_ws_bytes.restype = I64
    lib.has_l2q = hasattr(lib, "prfl_attn_fwd_l2q_ws")
    if lib.has_l2q:   # q in log2 units (the fused block's path): no scale argument
        lib.prfl_attn_fwd_l2q_ws.argtypes = FWD[:-2] + [P, I64, P]
        lib.prfl_attn_fwd_l2q_ws.restype = ctypes.c_int
        lib.prfl_attn_bwd_l2q_ws.argtypes = BWD[:-2] + [P, I64, P]
        lib.prfl_attn_bwd_l2q_ws.restype = ctypes.c_int
    lib.has_vt = hasattr(lib, "prfl_attn_fwd_l2q_vt_ws")
    if lib.has_vt:    # V in the key-chunked transposed layout (round 4)
        lib.prfl_attn_fwd_l2q_vt_ws.argtypes = FWD[:6] + [P] + FWD[9:-2] + [P, I64, P]
        lib.prfl_attn_fwd_l2q_vt_ws.restype = ctypes.c_int
        lib.prfl_attn_v_to_vt.argtypes, lib.prfl_attn_v_to_vt.restype = [P, I64, I64, P, I64, I64, I64, P], ctypes.c_int
        lib.prfl_attn_vt_bytes.argtypes, lib.prfl_attn_vt_bytes.restype = [I64] * 3, I64
    lib.has_kt = hasattr(lib, "prfl_attn_bwd_l2q_kt_ws")
    if lib.has_kt:
        lib.prfl_attn_bwd_l2q_kt_ws.argtypes = BWD[:6] + [P] + BWD[6:-2] + [P, I64, P]
        lib.prfl_attn_bwd_l2q_kt_ws.restype = ctypes.c_int
    if hasattr(lib, "prfl_attn_bphase_read"):
        lib.prfl_attn_bphase_read.argtypes, lib.prfl_attn_bphase_read.restype = [P], ctypes.c_int
    lib.has_bws = hasattr(lib, "prfl_attn_bwd_ws")
    if lib.has_bws:
        lib.prfl_attn_bwd_ws.argtypes, lib.prfl_attn_bwd_ws.restype = BWD[:-1] + [P, I64, P], ctypes.c_int
        lib.prfl_attn_bwd_ws_bytes.argtypes = [I64] * 5
        lib.prfl_attn_bwd_ws_bytes.restype = I64
    return lib


def main():
    libs = [load(sys.argv[1]), load(sys.argv[2])]
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 73920
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    H, C = 40, 5120
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(L, 3 * C, generator=g, device=dev).to(torch.bfloat16)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    do = torch.randn(L, C, generator=g, device=dev).to(torch.bfloat16)
    outs = []
    for _ in libs:
        outs.append(dict(o=torch.empty(L, C, dtype=torch.bfloat16, device=dev),
                         lse=torch.empty(H, L, device=dev), delta=torch.empty(H, L, device=dev),
                         dq=torch.empty(L, C, dtype=torch.bfloat16, device=dev),
                         dk=torch.empty(L, C, dtype=torch.bfloat16, device=dev),
                         dv=torch.empty(L, C, dtype=torch.bfloat16, device=dev)))
    sc = 128 ** -0.5
    st = torch.cuda.current_stream().cuda_stream

    def fwd(lib, b):
        rc = lib.prfl_attn_fwd(q.data_ptr(), 3 * C, 0, k.data_ptr(), 3 * C, 0, v.data_ptr(), 3 * C, 0,
                               b["o"].data_ptr(), C, 0, b["lse"].data_ptr(), 1, L, L, H, L, sc, st)
        assert rc == 0

    def bwd(lib, b):
        rc = lib.prfl_attn_bwd(q.data_ptr(), 3 * C, 0, k.data_ptr(), 3 * C, 0, v.data_ptr(), 3 * C, 0,
                               b["o"].data_ptr(), C, 0, do.data_ptr(), C, 0, b["lse"].data_ptr(),
                               b["delta"].data_ptr(), b["dq"].data_ptr(), C, 0, b["dk"].data_ptr(), C, 0,
                               b["dv"].data_ptr(), C, 0, 1, L, L, H, L, sc, st)
        assert rc == 0

    times = {(i, w): [] for i in range(2) for w in ("fwd", "bwd")}
    for r in range(rounds + 1):
        for i, lib in enumerate(libs):
            for w, fn in (("fwd", fwd), ("bwd", bwd)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn(lib, outs[i])
                e1.record()
                torch.cuda.synchronize()
                if r:
                    times[(i, w)].append(e0.elapsed_time(e1))
        if r:
            print(f"round {r}: " + "  ".join(f"{'AB'[i]}-{w} {times[(i, w)][-1]:.2f} ms"
                                           for i in range(2) for w in ("fwd", "bwd")), flush=True)
    same = all(torch.equal(outs[0][n], outs[1][n]) for n in ("o", "lse", "dq", "dk", "dv"))
    fl = {"fwd": 4 * L * L * C, "bwd": 14 * L * L * C}
    for w in ("fwd", "bwd"):
        ma, mb = statistics.median(times[(0, w)]), statistics.median(times[(1, w)])
        print(f"{w}: A median {ma:.2f} ms ({fl[w] / ma / 1e9:.0f} TF/s)  B median {mb:.2f} ms "
              f"({fl[w] / mb / 1e9:.0f} TF/s)  A/B time {ma / mb:.4f}")
    print("bit-identical outputs:", same)


if __name__ == "__main__":
    main()
