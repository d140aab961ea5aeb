"""Dev probe: self-attention forward rate vs operand layout / data at L tokens (40 heads, D=128).
  strided : q, k, v column slices of one [L, 3C] tensor (ld = 3C), raw N(0,1)
  sep     : q, k contiguous [L, C] copies (ld = C), v strided (the block's layout), raw N(0,1)
  rms     : as sep, q/k through the block's RMSNorm + 3-D RoPE kernel (the block's data)
  corr    : as rms, but every token = 0.8 * a shared per-channel vector + 0.6 * noise (tokens
            correlated the way hidden states become after a few blocks; same per-element scale)
  sharp   : as rms with q scaled by 8 (peaked softmax: most P entries underflow to 0)
usage: PRFL_PROF_L=73920 [PRFL_PROF_WARM_S=seconds] python tools/attn_layout_probe.py [reps]
PRFL_PROF_FILL_GB allocates (and touches) that much HBM before the operands, as the bench's
resident model state does.  PRFL_PROF_GAP_S idles the GPU that long before each timed launch.  PRFL_PROF_WARM_S keeps the GPU busy on the first case for that long before anything is timed."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
L, C, NH = int(os.environ.get("PRFL_PROF_L", 73920)), 5120, 40
grid = {73920: (21, 44, 80), 32760: (21, 30, 52)}.get(L, (1, 1, L))
dev = "cuda"
_fill = [torch.ones(int(2e9), dtype=torch.uint8, device=dev)
         for _ in range(int(float(os.environ.get("PRFL_PROF_FILL_GB", "0")) / 2))]
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(L, 3 * C, device=dev, generator=g).to(torch.bfloat16)
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]


def _freqs(dim):   # model.py:36-43 rope_params, max_len 1024, theta 1e4
    f = 1.0 / torch.pow(10000.0, torch.arange(0, dim, 2, dtype=torch.float64) / dim)
    return torch.polar(torch.ones(1024, dim // 2, dtype=torch.float64),
                       torch.outer(torch.arange(1024, dtype=torch.float64), f))


tab = ops.rope_table(torch.cat([_freqs(44), _freqs(42), _freqs(42)], dim=1), dev)
w = torch.ones(C, device=dev)
qr, _ = ops.rms_rope_fwd(q, w, 1e-6, tab, grid)
kr, _ = ops.rms_rope_fwd(k, w, 1e-6, tab, grid)
common = torch.randn(1, 3 * C, device=dev, generator=g)
qkvc = (0.8 * common + 0.6 * torch.randn(L, 3 * C, device=dev, generator=g)).to(torch.bfloat16)
qc, _ = ops.rms_rope_fwd(qkvc[:, :C], w, 1e-6, tab, grid)
kc, _ = ops.rms_rope_fwd(qkvc[:, C:2 * C], w, 1e-6, tab, grid)
cases = {"strided": (q, k, v), "sep": (q.contiguous(), k.contiguous(), v), "rms": (qr, kr, v),
         "corr": (qc, kc, qkvc[:, 2 * C:]), "sharp": ((qr.float() * 8).to(torch.bfloat16), kr, v)}
# sink: corr with key 0 scaled x4, so every row's max sits in the first key tile (no rescale
# after it) and every other probability underflows towards 0
kcs = kc.clone()
kcs[0] = (kcs[0].float() * 4).to(torch.bfloat16)
cases["sink"] = (qc, kcs, qkvc[:, 2 * C:])
fl = 4 * L * L * C
warm_s = float(os.environ.get("PRFL_PROF_WARM_S", "0"))
gap_s = float(os.environ.get("PRFL_PROF_GAP_S", "0"))
if warm_s > 0:
    o, _ = ops.attn_fwd(q, k, v, NH)
    t0 = time.time()
    while time.time() - t0 < warm_s:
        ops.attn_fwd(q, k, v, NH, out=o)
        torch.cuda.synchronize()
for name, (a, b, c) in cases.items():
    o, lse = ops.attn_fwd(a, b, c, NH)
    torch.cuda.synchronize()
    ts = []
    for i in range(reps):
        if gap_s > 0:
            time.sleep(gap_s)
        t0 = time.time()
        ops.attn_fwd(a, b, c, NH, out=o)
        torch.cuda.synchronize()
        ts.append(time.time() - t0)
    dt = min(ts)
    print(f"L={L} {name:8s} {dt*1e3:.2f} ms  {fl/dt/1e12:.0f} TF/s", flush=True)
