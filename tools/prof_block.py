"""Dev probe: one 14B WanAttentionBlock forward + backward at 480p x 81f (L = 32760) on the HIP
path, with per-kernel HIP-event timing (prfl_prof hooks).  Synthetic random weights."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd import block as B, ops  # noqa: E402
from oracle import wan_oracle as O  # noqa: E402  (rope table only)

L = int(os.environ.get("PROBE_L", 32760))
grid = (21, 30, 52) if L == 32760 else (1, 1, L)
C, F, NH = 5120, 13824, 40
dev = "cuda"
torch.manual_seed(0)
P = {}
for n in B.param_names(False):
    if n.endswith("weight") and ("norm" in n):
        P[n] = (1 + 0.1 * torch.randn(C, device=dev)).requires_grad_(True)
    elif n.endswith("bias"):
        shape = (F,) if n == "ffn.0.bias" else (C,)
        P[n] = (0.02 * torch.randn(shape, device=dev)).requires_grad_(True)
    else:
        shape = (F, C) if n == "ffn.0.weight" else ((C, F) if n == "ffn.2.weight" else (C, C))
        P[n] = (torch.randn(shape, device=dev) / shape[1] ** 0.5).requires_grad_(True)
x = torch.randn(1, L, C, device=dev).requires_grad_(True)
e = (0.1 * torch.randn(1, 6, C, device=dev)).requires_grad_(True)
ctx = torch.randn(1, 512, C, device=dev).to(torch.bfloat16)
meta = B.Meta(NH, [grid], [L], ops.rope_table(O.rope_freqs(128), dev), False)


def step():
    out = B.block_apply(P, x, e, ctx, meta)
    out.backward(torch.ones_like(out) * 1e-3)


step()
torch.cuda.synchronize()
for p in P.values():
    p.grad = None
ops.prof_enable(True)
t0 = time.time()
step()
torch.cuda.synchronize()
dt = time.time() - t0
ops.prof_enable(False)
st = ops.prof_collect()
blk = 8 * L * C * C + 4 * L * L * C + 4 * L * C * C + 4 * 512 * C * C + 4 * L * 512 * C + 4 * L * C * F
print(f"L={L}: block fwd+bwd wall {dt*1e3:.1f} ms (algorithmic 3x fwd = {3*blk/1e12:.1f} TF; "
      f"incl. recompute 4x -> {4*blk/dt/1e12:.0f} TF/s executed)")
for k, v in st.items():
    if v["count"]:
        ms = v["ms"]
        unit = "GB/s" if k in ("ln", "rms", "eltwise", "adamw") else "TF/s"
        scale = 1e9 if unit == "GB/s" else 1e12
        print(f"  {k:15s} n={v['count']:4d} total {ms:8.2f} ms  avg {ms/v['count']:8.3f} ms  "
              f"{v['work']/(ms*1e-3)/scale:8.1f} {unit}")
