"""Thread scaling of the bench's CPU baseline (config C1 on the oracle, test infrastructure):
    python tools/cpu_scaling.py 8 16
one 14B block forward at 480p x 49f per thread count; prints seconds and the speed-up."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import bench  # noqa: E402
from oracle import wan_oracle as O  # noqa: E402


def main():
    counts = [int(t) for t in sys.argv[1:]] or [8, 16]
    P, x, e0, ctx = bench.c1_inputs("cpu")
    base = None
    print(f"host: {bench.cpu_model()}, nproc {os.cpu_count()}, cores per socket "
          f"{bench.cores_per_socket()}", flush=True)
    for t in counts:
        torch.set_num_threads(t)
        t0 = time.time()
        with torch.no_grad():
            O.block_forward(P, "b.", x, e0, torch.tensor([bench.C1_GRID]), O.rope_freqs(128), ctx.float(),
                            bench.NH, seq_len=bench.C1_L)
        dt = time.time() - t0
        base = base or (dt, t)
        print(f"threads {t:3d}: {dt:6.1f} s  speed-up vs {base[1]} threads {base[0] / dt:.2f} "
              f"(linear {t / base[1]:.2f})", flush=True)


if __name__ == "__main__":
    main()
