"""Dev probe: host<->HBM copy rate for the streamed-AdamW pattern (many ~283 MB pinned tensors,
large total footprint, one copy stream alternating directions) vs a small footprint."""
import os
import time
import torch

print("nproc", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)), flush=True)
for p in ["/sys/class/drm/card0/device/numa_node", "/sys/class/drm/card1/device/numa_node"]:
    if os.path.exists(p):
        print(p, open(p).read().strip(), flush=True)
try:
    print(open("/sys/devices/system/node/online").read().strip(), "numa nodes online", flush=True)
except OSError:
    pass
n = 70_778_880                     # ffn.0.weight numel (13824 x 5120)
cnt = int(os.environ.get("PROBE_TENSORS", 48))     # 48 x 283 MB = 13.6 GB per moment set
t0 = time.time()
hm = [torch.zeros(n, dtype=torch.float32, pin_memory=True) for _ in range(cnt)]
print(f"pinned alloc+zero {cnt * n * 4 / 1e9:.1f} GB in {time.time() - t0:.1f} s", flush=True)
ring = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(3)]
cp = torch.cuda.Stream()


def run(label, idx, alternate=True):
    torch.cuda.synchronize()
    t = time.time()
    with torch.cuda.stream(cp):
        for j, i in enumerate(idx):
            ring[j % 3].copy_(hm[i], non_blocking=True)
            if alternate and j >= 1:
                hm[idx[j - 1]].copy_(ring[(j - 1) % 3], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.time() - t
    nbytes = len(idx) * n * 4 * (2 if alternate else 1) - (n * 4 if alternate else 0)
    print(f"{label}: {nbytes / dt / 1e9:.1f} GB/s ({nbytes / 1e9:.1f} GB in {dt:.2f} s)", flush=True)


run("small footprint h2d only (1 tensor x16)", [0] * 16, alternate=False)
run("large footprint h2d only", list(range(cnt)), alternate=False)
run("small footprint alternating", [0, 1] * 8)
run("large footprint alternating", list(range(cnt)))
run("large footprint alternating again", list(range(cnt)))
