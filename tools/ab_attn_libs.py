"""Dev A/B of N builds of the attention kernels in ONE process, interleaved (guide §5.4 rule 24):
    python tools/ab_attn_libs.py <lib1.so> <lib2.so> ... [--L 73920] [--reps 6] [--bwd]
prfl_attn_fwd (and with --bwd prfl_attn_bwd) at L tokens, 40 heads, HIP events on the launch
stream; prints per-build medians and whether all builds' outputs are bit-identical."""
import argparse
import statistics

import torch

from ab_attn import load


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--L", type=int, default=73920)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--lk", type=int, default=0, help="key count (cross-attention: 512); default L")
    ap.add_argument("--fp8", action="store_true", help="time prfl_attn_fwd_fp8 (config C5) instead")
    ap.add_argument("--qs", default="", help="comma list of lib indices built with ATTN_QS=1: they "
                    "get q pre-scaled by softmax_scale * log2(e) (rounded to bf16 once)")
    ap.add_argument("--phases", action="store_true", help="libs built with ATTN_PHASETIME=1: after the "
                    "timing, one more forward and the per-wave phase cycles of its first 64 workgroups")
    ap.add_argument("--bphases", action="store_true", help="libs built with ATTN_PHASETIME=1: after the "
                    "timing, one more backward and the per-wave phase cycles of the dK/dV and dQ kernels' "
                    "first 64 workgroups")
    ap.add_argument("--vt", default="", help="comma list of lib indices to run through the VT entry "
                    "(prfl_attn_v_to_vt + prfl_attn_fwd_l2q_vt_ws, the transpose inside the timing)")
    a = ap.parse_args()
    libs = [load(p) for p in a.libs]
    L, H, C = a.L, 40, 5120
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(L, 3 * C, generator=g, device=dev).to(torch.bfloat16)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    Lk = a.lk or L
    k, v = k[:Lk], v[:Lk]
    do = torch.randn(L, C, generator=g, device=dev).to(torch.bfloat16)
    outs = [dict(o=torch.empty(L, C, dtype=torch.bfloat16, device=dev), lse=torch.empty(H, L, device=dev),
                 delta=torch.empty(H, L, device=dev), dq=torch.empty(L, C, dtype=torch.bfloat16, device=dev),
                 dk=torch.empty(L, C, dtype=torch.bfloat16, device=dev),
                 dv=torch.empty(L, C, dtype=torch.bfloat16, device=dev)) for _ in libs]
    sc = 128 ** -0.5
    st = torch.cuda.current_stream().cuda_stream
    qs_libs = {int(i) for i in a.qs.split(",") if i}
    qsc = qkv[:, :C].float().mul(sc * 1.4426950408889634).to(torch.bfloat16).contiguous()

    def fwd(lib, b):
        qq = (qsc.data_ptr(), C, 0) if b.get("qs") else (q.data_ptr(), 3 * C, 0)
        args = (*qq, k.data_ptr(), 3 * C, 0, v.data_ptr(), 3 * C, 0,
                b["o"].data_ptr(), C, 0, b["lse"].data_ptr(), 1, L, Lk, H, Lk, sc)
        if a.fp8:
            nb = lib.prfl_attn_fwd_fp8_ws_bytes(1, L, L, H, L)
            if "ws8" not in b or b["ws8"].numel() < nb:
                b["ws8"] = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
            assert lib.prfl_attn_fwd_fp8(*args, b["ws8"].data_ptr(), nb, st) == 0
        elif lib.has_ws:
            nb = lib.prfl_attn_fwd_ws_bytes(1, L, Lk, H, Lk)
            if "ws" not in b or b["ws"].numel() < nb:
                b["ws"] = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
            if b.get("vt"):
                nv = lib.prfl_attn_vt_bytes(1, Lk, H)
                if "vtb" not in b:
                    b["vtb"] = torch.empty(nv, dtype=torch.uint8, device=dev)
                assert lib.prfl_attn_v_to_vt(v.data_ptr(), 3 * C, 0, b["vtb"].data_ptr(), 1, Lk, H, st) == 0
                assert lib.prfl_attn_fwd_l2q_vt_ws(*args[:6], b["vtb"].data_ptr(), *args[9:-1],
                                                   b["ws"].data_ptr(), nb, st) == 0
            elif b.get("qs") and lib.has_l2q:
                assert lib.prfl_attn_fwd_l2q_ws(*args[:-1], b["ws"].data_ptr(), nb, st) == 0
            else:
                assert lib.prfl_attn_fwd_ws(*args, b["ws"].data_ptr(), nb, st) == 0
        else:
            assert lib.prfl_attn_fwd(*args, st) == 0

    def bwd(lib, b):
        # ATTN_BWD_QS builds: q pre-scaled, gradient scale ln 2 (dK = ln2 * dS^T q')
        qq = (qsc.data_ptr(), C, 0) if b.get("qs") else (q.data_ptr(), 3 * C, 0)
        gsc = 0.6931471805599453 if b.get("qs") else sc
        args = (*qq, k.data_ptr(), 3 * C, 0, v.data_ptr(), 3 * C, 0,
                b["o"].data_ptr(), C, 0, do.data_ptr(), C, 0, b["lse"].data_ptr(),
                b["delta"].data_ptr(), b["dq"].data_ptr(), C, 0, b["dk"].data_ptr(), C, 0,
                b["dv"].data_ptr(), C, 0, 1, L, L, H, L, gsc)
        if lib.has_bws:
            nb = lib.prfl_attn_bwd_ws_bytes(1, L, L, H, L)
            if "bws" not in b or b["bws"].numel() < nb:
                b["bws"] = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
            if b.get("vt") and lib.has_kt:     # VT libs also take the KT backward
                nv = lib.prfl_attn_vt_bytes(1, L, H)
                if "ktb" not in b:
                    b["ktb"] = torch.empty(nv, dtype=torch.uint8, device=dev)
                assert lib.prfl_attn_v_to_vt(k.data_ptr(), 3 * C, 0, b["ktb"].data_ptr(), 1, L, H, st) == 0
                assert lib.prfl_attn_bwd_l2q_kt_ws(*args[:6], b["ktb"].data_ptr(), *args[6:-1],
                                                   b["bws"].data_ptr(), nb, st) == 0
            elif b.get("qs") and lib.has_l2q:
                assert lib.prfl_attn_bwd_l2q_ws(*args[:-1], b["bws"].data_ptr(), nb, st) == 0
            else:
                assert lib.prfl_attn_bwd_ws(*args, b["bws"].data_ptr(), nb, st) == 0
        else:
            assert lib.prfl_attn_bwd(*args, st) == 0

    for i in qs_libs:
        outs[i]["qs"] = True
    for i in {int(i) for i in a.vt.split(",") if i}:
        assert i in qs_libs, "the VT entry takes q in log2 units"
        outs[i]["vt"] = True
    for i in sorted(j for j in range(len(libs)) if outs[j].get("vt")):   # the transpose alone
        lib = libs[i]
        vtb = torch.empty(lib.prfl_attn_vt_bytes(1, Lk, H), dtype=torch.uint8, device=dev)
        ts = []
        for r in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert lib.prfl_attn_v_to_vt(v.data_ptr(), 3 * C, 0, vtb.data_ptr(), 1, Lk, H, st) == 0
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        m = statistics.median(ts)
        print(f"v_to_vt lib{i}: {m:.3f} ms ({2 * Lk * C * 2 / m / 1e6:.0f} GB/s)", flush=True)
    work = [("fwd", fwd, 4 * L * Lk * C)] + ([("bwd", bwd, 10 * L * L * C)] if a.bwd else [])
    for w, fn, fl in work:
        ts = [[] for _ in libs]
        for r in range(a.reps + 1):
            for i, lib in enumerate(libs):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn(lib, outs[i])
                e1.record()
                torch.cuda.synchronize()
                if r:
                    ts[i].append(e0.elapsed_time(e1))
        meds = [statistics.median(t) for t in ts]
        keys = ("o", "lse") if w == "fwd" else ("dq", "dk", "dv")
        same = all(torch.equal(outs[0][n], o[n]) for o in outs[1:] for n in keys)
        print(f"{w}: " + " | ".join(f"lib{i} {m:.2f} ms {fl / m / 1e9:.0f} TF/s" for i, m in enumerate(meds))
              + f" | identical {same}", flush=True)
        if w == "fwd" and not same:
            # accuracy of every build vs an exact fp64 softmax attention on sampled rows / heads
            rows = torch.linspace(0, L - 1, 48, device=dev).long()
            errs = [[] for _ in libs]
            for h in (0, 17, 39):
                sl = slice(h * 128, (h + 1) * 128)
                qq, kk, vv = q[rows, sl].double(), k[:, sl].double(), v[:, sl].double()
                ref = torch.softmax(qq @ kk.T * sc, -1) @ vv
                for i in range(len(libs)):
                    o = outs[i]["o"][rows, sl].double()
                    errs[i].append(((o - ref).norm() / ref.norm()).item())
            print("fwd rel-L2 vs fp64 (48 rows x 3 heads): " +
                  " | ".join(f"lib{i} {max(e):.2e}" for i, e in enumerate(errs)), flush=True)
    if a.bphases:
        print_bphases(libs, outs, bwd)
    if a.phases:
        import ctypes
        names = ("X (S + P.V MFMAs)", "X vmcnt", "barrier 1", "Y prefetch+tail", "Y vmcnt", "barrier 2",
                 "Y DMA issue", "Y mask/exp/sum", "Y pack")
        for i, lib in enumerate(libs):
            if not hasattr(lib, "prfl_attn_phase_read"):
                continue
            buf = (ctypes.c_ulonglong * 128)()
            lib.prfl_attn_phase_read(buf)          # clear
            fwd(lib, outs[i])
            torch.cuda.synchronize()
            assert lib.prfl_attn_phase_read(buf) == 0
            for wv in range(8):
                n = max(buf[wv * 16 + 15], 1)
                tot = sum(buf[wv * 16 + k] for k in range(9))
                print(f"lib{i} wave {wv}: " + ", ".join(f"{names[k]} {buf[wv * 16 + k] / n / 1e3:.1f}k "
                      f"({100 * buf[wv * 16 + k] / max(tot, 1):.1f}%)" for k in range(9))
                      + f" | {n} workgroups", flush=True)


def print_bphases(libs, outs, bwd):
    import ctypes
    names = {0: ("S/dP chain", "softmax", "DMA issue", "pack", "dV/dK chain", "tile vmcnt", "barrier"),
             1: ("S/dP chain", "softmax", "pack", "DMA issue", "dQ chain", "tile vmcnt", "barrier")}
    for i, lib in enumerate(libs):
        if not hasattr(lib, "prfl_attn_bphase_read"):
            continue
        buf = (ctypes.c_ulonglong * 256)()
        lib.prfl_attn_bphase_read(buf)             # clear
        bwd(lib, outs[i])
        torch.cuda.synchronize()
        assert lib.prfl_attn_bphase_read(buf) == 0
        for kern, kname in ((0, "dK/dV"), (1, "dQ")):
            for wv in range(8):
                base = (kern * 8 + wv) * 16
                n = max(buf[base + 15], 1)
                tot = sum(buf[base + k] for k in range(7))
                print(f"lib{i} {kname} wave {wv}: " + ", ".join(
                    f"{names[kern][k]} {buf[base + k] / n / 1e3:.1f}k ({100 * buf[base + k] / max(tot, 1):.1f}%)"
                    for k in range(7)) + f" | total {tot / n / 1e3:.1f}k cycles, {n} workgroups", flush=True)


if __name__ == "__main__":
    main()
