"""Diagnostic (GPU box): per-parameter grad rel-L2 of the toy PRFL chain vs the reference golden,
with the fused UniPC kernel and with the oracle's torch-op chain (on the GPU) in its place."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402

import test_gpu_model as T  # noqa: E402
from oracle import wan_oracle as O  # noqa: E402
from prfl_amd.schedulers import FlowUniPCMultistepScheduler  # noqa: E402

cache = {}


def golden(name):
    if name not in cache:
        cache[name] = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz")))
    return cache[name]


def report(g, named, prefix_key="grad/", tol=0):
    rs = sorted(((T.rel(named[k[5:]].grad, v), k[5:]) for k, v in g.items() if k.startswith("grad/")),
                reverse=True)
    for r, n in rs[:3]:
        print(f"   {r:.4f} {n}")
    return 99


T.check_grads = report
F = FlowUniPCMultistepScheduler._update
for name, upd in (("torch-ops", O.unipc_update), ("fused", F), ("torch-ops", O.unipc_update), ("fused", F)):
    FlowUniPCMultistepScheduler._update = staticmethod(upd)
    print(name)
    try:
        T.test_toy_prfl_chain_vs_reference(golden)
    except AssertionError as e:
        print("  assert:", str(e)[:200])
