"""Dev timing of the e4m3 self-attention forward (ops.attn_fwd_fp8) against the bf16 forward
(ops.attn_fwd) at L tokens x 40 heads in ONE process, interleaved; per-kernel HIP-event times
from the library's own profiler (prologue = quantisation kernels, main = attn_fwd_fp8_kernel)
and the two outputs' rel-L2 against an fp64 computation on sampled rows.
    python tools/ab_attn_fp8.py [--L 73920] [--reps 5]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hy-video-prfl_amd"))
from prfl_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=73920)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    L, H, C = a.L, 40, 5120
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(L, 3 * C, generator=g, device=dev).to(torch.bfloat16)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    flop = 4.0 * H * 128 * L * L
    t = {"bf16": [], "fp8": [], "fp8_main": [], "fp8_prologue": []}
    outs = {}
    for r in range(a.reps + 1):
        for name, fn in (("bf16", ops.attn_fwd), ("fp8", ops.attn_fwd_fp8)):
            torch.cuda.synchronize()
            ops.prof_enable(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            outs[name] = fn(q, k, v, H)[0]
            e1.record()
            torch.cuda.synchronize()
            ops.prof_enable(False)
            p = ops.prof_collect()
            if r == 0:
                continue
            t[name].append(e0.elapsed_time(e1))
            if name == "fp8":
                t["fp8_main"].append(p["attn_fwd_fp8"]["ms"])
                t["fp8_prologue"].append(p["eltwise"]["ms"])
    for k_, v_ in t.items():
        ms = statistics.median(v_)
        print(f"{k_:13s} {ms:8.2f} ms  {flop / ms / 1e9:7.1f} TF/s  (reps {['%.2f' % x for x in v_]})")
    rows = torch.randperm(L, generator=torch.Generator().manual_seed(1))[:128].sort().values.to(dev)
    qc = q[rows].double().view(-1, H, 128).transpose(0, 1)
    kc = k.double().view(L, H, 128).transpose(0, 1)
    vc = v.double().view(L, H, 128).transpose(0, 1)
    ex = []
    for h in range(H):
        s = torch.softmax(qc[h] @ kc[h].T * 128 ** -0.5, -1)
        ex.append(s @ vc[h])
    ex = torch.stack(ex).transpose(0, 1).reshape(-1, C)
    for name, o in outs.items():
        d = o[rows].double()
        print(f"{name}: rel-L2 vs fp64 on 128 rows = {((d - ex).norm() / ex.norm()).item():.3e}")


if __name__ == "__main__":
    main()
