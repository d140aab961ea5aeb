"""Dev A/B: the streamed AdamW update (moments in pinned host memory, HBM ring) with both copy
directions on one stream vs on two (AdamW.duplex), one process, interleaved:
    python tools/ab_adamw_stream.py [--gb 4] [--reps 4]
--gb: GB of fp32 parameters (moments: 2x that on the host, each moved H2D and D2H per step)."""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd.optim import AdamW  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    n_t = 16
    per = int(a.gb * 1e9 / 4 / n_t)
    g = torch.Generator(device="cuda").manual_seed(0)
    params = [torch.randn(per, device="cuda", generator=g).requires_grad_(True) for _ in range(n_t)]
    for p in params:
        p.grad = torch.randn(per, device="cuda", generator=g) * 1e-3
    opt = AdamW(params, lr=1e-4, state_on_host=True)
    moved = 2 * 2 * 4 * per * n_t / 1e9                   # m, v each way
    ts = {True: [], False: []}
    for r in range(a.reps + 1):
        for duplex in (False, True):
            opt.duplex = duplex
            torch.cuda.synchronize()
            t0 = time.time()
            opt.step()
            opt.synchronize()
            dt = time.time() - t0
            if r:
                ts[duplex].append(dt)
    for duplex in (False, True):
        m = statistics.median(ts[duplex])
        print(f"duplex={duplex}: {m * 1e3:.1f} ms per step, {moved / m:.1f} GB/s of moments "
              f"(H2D + D2H), {a.gb:.1f} GB of parameters", flush=True)


if __name__ == "__main__":
    main()
