"""Debug: GPU toy I2V WanModel grads vs the CPU oracle, per parameter."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd"), os.path.join(ROOT, "tests", "golden")]
import numpy as np, torch
from shapes import TOY, model_shapes, seeded_params
from oracle import wan_oracle as O
from prfl_amd.model import WanModel
g = dict(np.load(os.path.join(ROOT, "tests/golden/toy_i2v.npz")))
m = WanModel(model_type="i2v", in_dim=36, **TOY)
sd = seeded_params(model_shapes(TOY, "i2v"), prefix="toy.")
m.load_state_dict(sd); m = m.cuda()
x = torch.from_numpy(g["x"]).cuda().requires_grad_(True)
y = torch.from_numpy(g["y"]).cuda(); clip = torch.from_numpy(g["clip"]).cuda()
out = m(x=[x], t=torch.from_numpy(g["t"]).cuda(), context=[torch.from_numpy(g["ctx"]).cuda()], seq_len=105, y=[y], clip_fea=clip)[0]
(out * torch.from_numpy(g["upstream"]).cuda()).sum().backward()
P = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
xr = torch.from_numpy(g["x"]).requires_grad_(True)
ref = O.model_forward(P, dict(TOY, model_type="i2v"), [xr], torch.from_numpy(g["t"]), [torch.from_numpy(g["ctx"])], 105, y_list=[torch.from_numpy(g["y"])], clip_fea=torch.from_numpy(g["clip"]))[0]
(ref * torch.from_numpy(g["upstream"])).sum().backward()
def rel(a, b): a = a.detach().double().cpu().flatten(); b = b.detach().double().cpu().flatten(); return ((a-b).norm()/b.norm()).item()
print("out", rel(out, ref), "dx", rel(x.grad, xr.grad))
for n, p in m.named_parameters():
    r = rel(p.grad, P[n].grad)
    flag = " <<<" if r > 0.03 else ""
    print(f"{n:45s} {r:.4f}{flag}")
    if "k_img.weight" in n and r > 0.03:
        d = (p.grad.cpu() - P[n].grad).abs()
        print("   row err (first/last 4):", d.sum(1)[:4].tolist(), d.sum(1)[-4:].tolist())
        print("   col err (first/last 4):", d.sum(0)[:4].tolist(), d.sum(0)[-4:].tolist())
