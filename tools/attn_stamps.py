"""Dev probe: phase shares of the self-attention forward from the stamped diagnostic build
(prfl_attn_fwd_stamped): per wave, cycles in {MFMA phase X, barrier after X, softmax phase Y,
barrier after Y}, summed over the key tiles.  usage: python tools/attn_stamps.py [L]"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
from prfl_amd._lib import I64, F32, call, ptr, stream_ptr  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
C, H = 5120, 40
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(L, 3 * C, device="cuda", generator=g).to(torch.bfloat16)
o = torch.empty(L, C, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(H, L, device="cuda")
st = torch.zeros(16 * 8 * 4, dtype=torch.int64, device="cuda")
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
for _ in range(2):
    call("prfl_attn_fwd_stamped", ptr(q), I64(3 * C), ptr(k), I64(3 * C), ptr(v), I64(3 * C),
         ptr(o), I64(C), ptr(lse), I64(L), I64(H), F32(1 / math.sqrt(128)), ptr(st), stream_ptr())
torch.cuda.synchronize()
s = st.view(16, 8, 4).double()
ntile = (L + 63) // 64 + 1
print(f"L={L}: cycles per tile, mean over 16 workgroups (head 0); X = MFMA phase, Y = softmax phase")
for w in range(8):
    m = s[:, w].mean(0) / ntile
    tot = m.sum().item()
    print(f" wave {w}: X {m[0]:7.0f}  wait {m[1]:6.0f}  Y {m[2]:7.0f}  wait {m[3]:6.0f}  total {tot:7.0f}"
          f"   (32 MFMA = 1024 cyc -> MFMA share {1024 / tot:.2f})")
