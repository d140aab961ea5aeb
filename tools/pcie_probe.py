"""Dev probe: host<->HBM copy bandwidth with pinned buffers (the streamed-AdamW path)."""
import time
import torch

n = 256 * 1024 * 1024 // 4 * 2          # 512 MB fp32
h = torch.empty(n, dtype=torch.float32, pin_memory=True)
h2 = torch.empty(n, dtype=torch.float32, pin_memory=True)
d = torch.empty(n, dtype=torch.float32, device="cuda")
d2 = torch.empty(n, dtype=torch.float32, device="cuda")
print("pinned:", h.is_pinned(), flush=True)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
for name, fn in [("h2d", lambda: d.copy_(h, non_blocking=True)),
                 ("d2h", lambda: h.copy_(d, non_blocking=True))]:
    for _ in range(2):
        torch.cuda.synchronize(); t = time.time(); fn(); torch.cuda.synchronize()
    print(f"{name} {n * 4 / (time.time() - t) / 1e9:.1f} GB/s", flush=True)
torch.cuda.synchronize(); t = time.time()
with torch.cuda.stream(s1):
    d.copy_(h, non_blocking=True)
with torch.cuda.stream(s2):
    h2.copy_(d2, non_blocking=True)
torch.cuda.synchronize()
print(f"concurrent h2d+d2h {2 * n * 4 / (time.time() - t) / 1e9:.1f} GB/s total", flush=True)
