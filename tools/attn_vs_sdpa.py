"""Dev probe: prfl self-attention (ops.attn_fwd / attn_bwd) next to torch's
scaled_dot_product_attention (the ROCm build's flash backend) at the 720p shape, same random
operands, interleaved, HIP events.  The torch column is a ceiling reference only.
    python tools/attn_vs_sdpa.py [L] [reps]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.nn.attention import SDPBackend, sdpa_kernel  # noqa: E402
from prfl_amd import ops  # noqa: E402

# never the math backend (an L x L score matrix per head would not fit)
sdpa_kernel([SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION]).__enter__()

L = int(sys.argv[1]) if len(sys.argv) > 1 else 73920
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
H, D = 40, 128
C = H * D
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(L, 3 * C, generator=g, device=dev).to(torch.bfloat16)
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
do = torch.randn(L, C, generator=g, device=dev).to(torch.bfloat16)
qt, kt, vt = (t.view(L, H, D).transpose(0, 1).unsqueeze(0).contiguous() for t in (q, k, v))
dot = do.view(L, H, D).transpose(0, 1).unsqueeze(0).contiguous()
o, lse = ops.attn_fwd(q, k, v, H)


def timeit(fn):
    ts = []
    for i in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


fl = 4 * L * L * C
print("sdpa backends:", torch.backends.cuda.flash_sdp_enabled(), torch.backends.cuda.mem_efficient_sdp_enabled(),
      flush=True)
a = timeit(lambda: ops.attn_fwd(q, k, v, H, out=o))
with torch.no_grad():
    b = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt))
print(f"fwd L={L}: prfl {a:.2f} ms {fl / a / 1e9:.0f} TF/s | sdpa {b:.2f} ms {fl / b / 1e9:.0f} TF/s", flush=True)
ref = F.scaled_dot_product_attention(qt[:, :2], kt[:, :2], vt[:, :2])[0].transpose(0, 1).reshape(L, 2 * D)
print("fwd heads 0-1 max |prfl - sdpa|:", (o[:, :2 * D].float() - ref.float()).abs().max().item(), flush=True)
a = timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, H))
qr, kr, vr = (t.clone().requires_grad_(True) for t in (qt, kt, vt))
out = F.scaled_dot_product_attention(qr, kr, vr)
b = timeit(lambda: torch.autograd.grad(out, (qr, kr, vr), dot, retain_graph=True))
print(f"bwd L={L}: prfl {a:.2f} ms {2.5 * fl / a / 1e9:.0f} TF/s | sdpa {b:.2f} ms {2.5 * fl / b / 1e9:.0f} TF/s",
      flush=True)
