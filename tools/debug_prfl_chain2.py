"""Diagnostic (GPU box): toy PRFL reward step, d loss / d model_output through the fused UniPC
step vs through the oracle's torch chain, same inputs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tests", "golden")]
import copy  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_model as T  # noqa: E402
from oracle import wan_oracle as O  # noqa: E402
from prfl_amd.network import MLP, QueryAttention, forward_mlp  # noqa: E402
from prfl_amd.schedulers import FlowUniPCMultistepScheduler  # noqa: E402
from prfl_amd.train import build_lrm, batch2list, list2batch  # noqa: E402
from shapes import qa_shapes, mlp_shapes, seeded_params  # noqa: E402

DEV = "cuda"
g = dict(np.load(os.path.join(ROOT, "tests", "golden", "toy_prfl.npz")))
gen = T.toy_model("t2v")
lrm = build_lrm(T.toy_model("t2v"), [0])
qa = QueryAttention(256, 1, 8, 0., return_type="query")
qa.load_state_dict(seeded_params(qa_shapes(256), prefix="tqa."))
mlp = MLP(256)
mlp.load_state_dict(seeded_params(mlp_shapes(256), prefix="tmlp."))
qa, mlp = qa.to(DEV).requires_grad_(False), mlp.to(DEV).requires_grad_(False)
sch = FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1, use_dynamic_shifting=False)
sch.set_timesteps(num_inference_steps=40, device=DEV, shift=5.0)
ts = sch.timesteps
ctx = torch.from_numpy(g["ctx"]).to(DEV).to(torch.bfloat16)
latent = torch.from_numpy(g["noise"]).to(DEV).to(torch.bfloat16)
mid = int(g["mid"])
with torch.no_grad():
    for i in range(mid):
        npred = list2batch(gen(x=batch2list(latent), t=torch.tensor([ts[i]], device=DEV),
                               context=batch2list(ctx), seq_len=105))
        latent = sch.step(npred, ts[i], latent, return_dict=False)[0]
npred = list2batch(gen(x=batch2list(latent), t=torch.tensor([ts[mid]], device=DEV),
                       context=batch2list(ctx), seq_len=105))
print("npred", npred.shape, npred.dtype, npred.is_contiguous(), "golden npred rel", T.rel(npred, g["npred"]))
res = {}
for name, upd in (("fused", FlowUniPCMultistepScheduler._update), ("oracle", O.unipc_update)):
    s2 = copy.copy(sch)
    s2._update = upd
    mo = npred.detach().clone().requires_grad_(True)
    prev = s2.step(mo, ts[mid], latent, return_dict=False)[0]
    feats = list2batch(lrm(x=batch2list(prev), t=torch.tensor([ts[mid + 1]], device=DEV),
                           context=batch2list(ctx), seq_len=105, output_features=True,
                           selected_layers=[1]))
    r = forward_mlp(mlp, qa(feats))
    loss = 0.1 * torch.relu(-r.squeeze() + 2).mean() / 5.0
    gprev, = torch.autograd.grad(loss, prev, retain_graph=True)
    gmo, = torch.autograd.grad(loss, mo)
    res[name] = (prev.detach(), loss.item(), gprev, gmo)
    print(name, "loss", loss.item(), "stepped rel", T.rel(prev, g["stepped"]), "|gprev|", gprev.norm().item(),
          "|gmo|", gmo.norm().item(), gprev.dtype)
a, b = res["fused"], res["oracle"]
print("prev max|d|", (a[0].float() - b[0].float()).abs().max().item())
print("gprev rel", T.rel(a[2], b[2]), "gmo rel", T.rel(a[3], b[3]))
