"""Model-level parity on the MI355X: WanModel (toy width, T2V + I2V), the reward head at real
width, the toy PRFL reward chain and SFT step — all against the reference's golden fixtures."""
import numpy as np
import pytest
import torch

import seeded
from shapes import TOY, model_shapes, qa_shapes, mlp_shapes, seeded_params
from tolerance import key_path_scale

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu().flatten()
    b = torch.as_tensor(b).detach().double().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def toy_model(model_type, prefix="toy."):
    from prfl_amd.model import WanModel
    m = WanModel(model_type=model_type, in_dim=16 if model_type == "t2v" else 36, **TOY)
    sd = seeded_params(model_shapes(TOY, model_type), prefix=prefix)
    m.load_state_dict(sd)
    return m.to(DEV)


def check_grads(g, named, prefix_key="grad/", tol=3e-2):
    n_checked = 0
    for k, v in g.items():
        if k.startswith(prefix_key):
            n = k[len(prefix_key):]
            gr = named[n].grad
            gk = {k2[len(prefix_key):] if k2.startswith(prefix_key) else k2: v2 for k2, v2 in g.items()}
            scale = key_path_scale({("grad/" + k2): v2 for k2, v2 in gk.items()}, n)
            if scale is not None:
                assert (gr.cpu().flatten() - torch.from_numpy(v)).norm().item() < tol * scale, n
            else:
                assert rel(gr, v) < tol, (n, rel(gr, v))
            n_checked += 1
    return n_checked


@pytest.mark.parametrize("model_type", ["t2v", "i2v"])
def test_toy_wanmodel_vs_reference(golden, model_type):
    g = golden("toy_" + model_type)
    m = toy_model(model_type)
    x = torch.from_numpy(g["x"]).to(DEV).requires_grad_(True)
    kw = {}
    if model_type == "i2v":
        kw = dict(y=[torch.from_numpy(g["y"]).to(DEV)], clip_fea=torch.from_numpy(g["clip"]).to(DEV))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(x=[x], t=torch.from_numpy(g["t"]).to(DEV), context=[torch.from_numpy(g["ctx"]).to(DEV)],
                seq_len=105, **kw)[0]
    assert out.dtype == torch.float32 and tuple(out.shape) == tuple(g["out"].shape)
    assert rel(out, g["out"]) < 1e-2, rel(out, g["out"])
    (out * torch.from_numpy(g["upstream"]).to(DEV)).sum().backward()
    assert rel(x.grad, g["dx"]) < 3e-2, rel(x.grad, g["dx"])
    named = dict(m.named_parameters())
    assert check_grads(g, named) > 20
    feats = m(x=[x.detach()], t=torch.from_numpy(g["t"]).to(DEV),
              context=[torch.from_numpy(g["ctx"]).to(DEV)], seq_len=105, output_features=True,
              selected_layers=[1], **kw)
    assert rel(feats[0], g["feat1"]) < 1e-2


def test_reward_head_vs_reference(golden):
    from prfl_amd.network import MLP, QueryAttention, forward_mlp
    g = golden("reward_head")
    qa = QueryAttention(5120, 1, 8, 0., return_type="query")
    qa.load_state_dict(seeded_params(qa_shapes(5120), prefix="qa."))
    mlp = MLP(5120)
    mlp.load_state_dict(seeded_params(mlp_shapes(5120), prefix="mlp."))
    qa, mlp = qa.to(DEV), mlp.to(DEV)
    feat = torch.from_numpy(g["feat"]).to(DEV).requires_grad_(True)
    pooled = qa(feat)
    # SURVEY §8c per-op bound (5e-3): the bf16 output roundings of o and of out_proj alone are
    # ~1.1e-3 each; the split-L kernel rounds P against the running max (flash numerics)
    assert rel(pooled, g["pooled"]) < 5e-3, rel(pooled, g["pooled"])
    r = forward_mlp(mlp, pooled)
    loss = 0.1 * torch.relu(-r.squeeze() + 2).mean()
    assert abs(loss.item() - float(g["loss"])) < 2e-3
    loss.backward()
    assert rel(feat.grad, g["dfeat"]) < 5e-2, rel(feat.grad, g["dfeat"])
    named = {**{k: v for k, v in qa.named_parameters()}, **{k: v for k, v in mlp.named_parameters()}}
    for k, v in g.items():
        if k.startswith("grad/"):
            n = k[5:]
            assert rel(named[n].grad, v) < 5e-2, (n, rel(named[n].grad, v))


def test_toy_prfl_chain_vs_reference(golden):
    """Reward step of train_prfl.py:585-835 with a toy generator/LRM, mid_timestep = 3."""
    from prfl_amd.network import MLP, QueryAttention, forward_mlp
    from prfl_amd.schedulers import FlowUniPCMultistepScheduler, FlowMatchDiscreteScheduler
    from prfl_amd.train import build_lrm, batch2list, list2batch
    g = golden("toy_prfl")
    gen = toy_model("t2v")
    lrm = build_lrm(toy_model("t2v"), [0])
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
    assert rel(latent, g["rollout"]) < 2e-2, rel(latent, g["rollout"])
    npred = list2batch(gen(x=batch2list(latent), t=torch.tensor([ts[mid]], device=DEV),
                           context=batch2list(ctx), seq_len=105))
    latent = sch.step(npred, ts[mid], latent, return_dict=False)[0]
    # the fused UniPC step follows the reference's own op semantics: 2.4e-4 here (torch ops on
    # the GPU, with CUDA's fp32 left scalars and reciprocal division, land at 2.9e-3)
    assert rel(latent, g["stepped"]) < 1e-3, rel(latent, g["stepped"])
    feats = list2batch(lrm(x=batch2list(latent), t=torch.tensor([ts[mid + 1]], device=DEV),
                           context=batch2list(ctx), seq_len=105, output_features=True,
                           selected_layers=[1]))
    assert rel(feats, g["feat"]) < 3e-2, rel(feats, g["feat"])
    r = forward_mlp(mlp, qa(feats))
    loss = 0.1 * torch.relu(-r.squeeze() + 2).mean() / 5.0
    assert abs(loss.item() - float(g["loss"])) < 2e-3 * abs(float(g["loss"])) + 1e-4
    loss.backward()
    named = dict(gen.named_parameters())
    # The gradients through the whole chain are pinned piece by piece on the reference's own
    # inputs in test_prfl_reward_chain_split_vs_reference: the reward MLP's ReLUs switch at
    # bf16 resolution, so two whole-chain bf16 runs land several % apart by construction; here:
    # every generator parameter received a finite, non-zero gradient.
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in named.values())
    assert sum(int(p.grad.abs().sum() > 0) for p in named.values()) > 20
    # SFT flow-matching step
    gen.zero_grad()
    fm = FlowMatchDiscreteScheduler(shift=5.0)
    fm.set_timesteps(1000, dtype=torch.int64)
    idx = int(g["sft_idx"])
    x0 = torch.from_numpy(g["x0"]).to(DEV).to(torch.bfloat16)
    noise = torch.from_numpy(g["sft_noise"]).to(DEV).to(torch.bfloat16)
    sigma = fm.sigmas[[idx]].float().view(1, 1, 1, 1, 1).to(DEV)
    assert torch.equal(fm.timesteps[[idx]], torch.from_numpy(g["sft_timestep"]))
    noisy = fm.add_noise(x0, noise, sigma)
    pred = list2batch(gen(x=batch2list(noisy), t=fm.timesteps[[idx]].to(DEV), context=batch2list(ctx),
                          seq_len=105))
    sft_loss = torch.mean((pred.float() - fm.get_train_target(x0, noise).float()) ** 2) / 5.0
    assert abs(sft_loss.item() / float(g["sft_loss"]) - 1) < 1e-2
    sft_loss.backward()
    assert check_grads(g, named, prefix_key="sft:grad/", tol=3e-2) > 20


def summary_errors(g, prefix, named):
    """{param: error} of our gradients vs a `make_golden.grads_of` summary stored under
    `prefix`: rel-L2 of full small tensors (key-side biases against their weight's gradient scale,
    tolerance.key_path_scale), and for large ones the worst of the leading values' rel-L2, the
    norm ratio and the seeded projection's difference over the norm."""
    strip = {k[len(prefix):]: v for k, v in g.items() if k.startswith(prefix)}
    errs = {}
    for k, v in strip.items():
        kind, _, n = k.partition("/")
        if kind not in ("grad", "ghead") or n not in named:
            continue
        gr = named[n].grad.detach().float().cpu().flatten()
        if kind == "grad":
            scale = key_path_scale(strip, n)
            errs[n] = ((gr - torch.from_numpy(v)).norm().item() / scale if scale is not None
                       else rel(gr, v))
        else:
            nrm = float(strip["gnorm/" + n])
            r = torch.from_numpy(seeded.randn("proj:" + n, (gr.numel(),))).double()
            errs[n] = max(rel(gr[:v.size], v), abs(gr.double().norm().item() / nrm - 1),
                          abs((gr.double() * r).sum().item() - float(strip["gproj/" + n])) / nrm)
    return errs


def _inject_unipc_state(sch, g, pre):
    """The reference scheduler's state before the grad-enabled step (make_golden._unipc_state)."""
    for j in range(2):
        k = f"{pre}state:mo{j}"
        if k in g:
            t = torch.from_numpy(g[k]).to(DEV)
            sch.model_outputs[j] = t.to(torch.bfloat16) if bool(g[k + ":bf16"]) else t
    if pre + "state:last" in g:
        t = torch.from_numpy(g[pre + "state:last"]).to(DEV)
        sch.last_sample = t.to(torch.bfloat16) if bool(g[pre + "state:last:bf16"]) else t
    sch.lower_order_nums = int(g[pre + "state:lon"])
    sch.this_order = int(g[pre + "state:this_order"])
    if int(g[pre + "state:step_index"]) >= 0:
        sch._step_index = int(g[pre + "state:step_index"])


@pytest.mark.parametrize("mid", [0, 3])
def test_prfl_reward_chain_split_vs_reference(golden, mid):
    """The PRFL reward backward (`train_prfl.py:703-830`) pinned piece by piece on the
    reference's own inputs (make_golden.case_toy_prfl_split), so no piece inherits the bf16
    noise of the pieces before it:

    * head (MLP + sigmoid + hinge) from the reference's pooled feature: reward and d(pooled)
      vs the reference;
    * trunk (1-block LRM + QueryAttention) from the reference's stepped bf16 latent with the
      reference's d(pooled) upstream: pooled and d(stepped) vs the reference AND vs the fp32
      truth of the same piece;
    * generator (grad-enabled step at t_mid + the fused differentiable UniPC step) from the
      reference's pre-step latent and scheduler state with the reference's d(stepped) upstream:
      stepped latent and every generator gradient vs the reference and vs the fp32 truth.

    Bounds: SURVEY §8c's 3e-2 for gradients, 1e-2 for forward values.  mid 0 has no rollout
    (order-1 step, no corrector); mid 3 runs the corrector and the order-2 predictor on the
    reference's history."""
    from prfl_amd.network import MLP, QueryAttention, forward_mlp
    from prfl_amd.schedulers import FlowUniPCMultistepScheduler
    from prfl_amd.train import build_lrm, batch2list, list2batch
    g = golden("toy_prfl_split")
    pre = f"m{mid}:"
    gen = toy_model("t2v")
    lrm = build_lrm(toy_model("t2v"), [0])
    qa = QueryAttention(256, 1, 8, 0., return_type="query")
    qa.load_state_dict(seeded_params(qa_shapes(256), prefix="tqa."))
    mlp = MLP(256)
    mlp.load_state_dict(seeded_params(mlp_shapes(256), prefix="tmlp."))
    qa, mlp = qa.to(DEV).requires_grad_(False), mlp.to(DEV).requires_grad_(False)
    ctx = torch.from_numpy(g["ctx"]).to(DEV).to(torch.bfloat16)
    T = lambda k: torch.from_numpy(g[pre + k]).to(DEV)  # noqa: E731
    report = {}
    # head
    p = T("pooled").requires_grad_(True)
    r = forward_mlp(mlp, p)
    loss = 0.1 * torch.relu(-r.squeeze() + 2).mean() / 5.0
    loss.backward()
    want = float(g[pre + "reward"].reshape(-1)[0])
    assert abs(r.item() - want) < 2e-3, (r.item(), want)
    report["head d(pooled) vs ref"] = rel(p.grad, g[pre + "dpool"])
    report["head d(pooled) vs truth (ref: %.4f)" % rel(g[pre + "dpool"], g[pre + "t32:dpool"])] = \
        rel(p.grad, g[pre + "t32:dpool"])
    assert report["head d(pooled) vs ref"] < 3e-2, report
    # trunk
    leaf = T("stepped").to(torch.bfloat16).requires_grad_(True)
    feats = list2batch(lrm(x=batch2list(leaf), t=T("t1").view(1), context=batch2list(ctx),
                           seq_len=105, output_features=True, selected_layers=[1]))
    pooled = qa(feats)
    assert rel(pooled, g[pre + "pooled"]) < 1e-2, rel(pooled, g[pre + "pooled"])
    pooled.backward(T("dpool"))
    report["trunk d(stepped) vs ref"] = rel(leaf.grad, g[pre + "dstep"])
    report["trunk d(stepped) vs truth (ref: %.4f)" % rel(g[pre + "dstep"], g[pre + "t32:dstep"])] \
        = rel(leaf.grad, g[pre + "t32:dstep"])
    assert max(v for k, v in report.items() if k.startswith("trunk")) < 3e-2, report
    # generator
    sch = FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1, use_dynamic_shifting=False)
    sch.set_timesteps(num_inference_steps=40, device=DEV, shift=5.0)
    _inject_unipc_state(sch, g, pre)
    t_mid = T("t_mid").view(1)
    lat = T("pre").to(torch.bfloat16)
    npred = list2batch(gen(x=batch2list(lat), t=t_mid, context=batch2list(ctx), seq_len=105))
    assert rel(npred, g[pre + "npred"]) < 1e-2, rel(npred, g[pre + "npred"])
    stepped = sch.step(npred, t_mid[0], lat, return_dict=False)[0]
    assert stepped.dtype == torch.bfloat16
    report["gen stepped vs ref"] = rel(stepped, g[pre + "stepped"])
    assert report["gen stepped vs ref"] < 1e-2, report
    stepped.backward(T("dstep").to(torch.bfloat16))
    named = dict(gen.named_parameters())
    e_ref = summary_errors(g, pre, named)
    e_t32 = summary_errors(g, pre + "t32:", named)
    med = lambda d: sorted(d.values())[len(d) // 2]  # noqa: E731
    worst = sorted(e_ref.items(), key=lambda kv: -kv[1])[:3]
    report.update({"gen grads vs ref: median": med(e_ref), "worst": worst,
                   "gen grads vs truth: median": med(e_t32), "max": max(e_t32.values())})
    print(report)
    assert len(e_ref) > 60 and len(e_t32) == len(e_ref)
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in named.values())
    assert max(e_ref.values()) < 3e-2, report
    assert max(e_t32.values()) < 3e-2, report


def _summary_pairs(g, prefix, ours):
    """(name, ours, reference-side key suffix) over a fixture summary (make_golden._summ): full
    small tensors and the leading values of large ones."""
    for k in g:
        if k.startswith(prefix + "full/") or k.startswith(prefix + "head/"):
            kind, n = k[len(prefix):].split("/", 1)
            o = ours[n].detach().float().cpu().flatten()
            yield n, (o if kind == "full" else o[:g[k].size]), k


def _as_grads_of(g, prefix):
    """A `make_golden._summ` summary under `prefix` in `grads_of` naming (for summary_errors)."""
    ren = {"full": "grad", "head": "ghead", "norm": "gnorm", "proj": "gproj"}
    out = {}
    for k, v in g.items():
        if k.startswith(prefix):
            kind, _, n = k[len(prefix):].partition("/")
            if kind in ren:
                out[ren[kind] + "/" + n] = v
    return out


class _Grads:
    def __init__(self, t):
        self.grad = t


@pytest.mark.parametrize("fixture", ["toy_prfl_trainer", "toy_prfl_trainer_mid0"])
def test_prfl_trainer_two_iterations_vs_reference(golden, fixture):
    """PRFLTrainer over two iterations with gradient_accumulation_steps = 2 vs
    the reference's `train_step` + `train_step_refl` run on the same toy models, draws and mids
    (make_golden.case_toy_prfl_trainer; mids (2, 1), and (0, 0): no rollout): iteration 0
    accumulates (the reward gradient lands on the clipped SFT gradient), iteration 1 is the
    boundary where BOTH steps call AdamW.
    Per backward: loss, reward, pre-clip grad norm.  The SFT step's fresh gradient of every
    parameter vs the reference's (3e-2, as the toy-model test).  The reward step's fresh
    gradient is NOT compared here: the reward MLP's ReLUs switch at bf16 resolution, so whole-
    chain bf16 runs — the reference's own, one ulp apart in the initial noise — land 1-12 %
    apart (the fixture's floor:* arrays); test_prfl_reward_chain_split_vs_reference pins every
    piece of that backward on the reference's own inputs instead.
    Per optimizer step: our update vs torch.optim.AdamW on our clipped gradients (exact), and vs
    the reference's update (norm, sign agreement)."""
    from prfl_amd.network import MLP, QueryAttention
    from prfl_amd.schedulers import FlowMatchDiscreteScheduler
    from prfl_amd.train import PRFLTrainer, build_lrm
    g = golden(fixture)
    ga, lr = float(g["ga"]), float(g["lr"])
    gen = toy_model("t2v")
    lrm = build_lrm(toy_model("t2v"), [0])
    qa = QueryAttention(256, 1, 8, 0., return_type="query")
    qa.load_state_dict(seeded_params(qa_shapes(256), prefix="tqa."))
    mlp = MLP(256)
    mlp.load_state_dict(seeded_params(mlp_shapes(256), prefix="tmlp."))
    qa, mlp = qa.to(DEV).requires_grad_(False), mlp.to(DEV).requires_grad_(False)
    tr = PRFLTrainer(gen, lrm, qa, mlp, lr=lr, grad_accum=ga, feature_layer=(1,))
    named = {n: p for n, p in gen.named_parameters() if p.requires_grad}
    rec = {}
    begin, end, ostep = tr.reducer.begin, tr.reducer.end, tr.optimizer.step

    def hook_begin():
        tr.optimizer.wait()
        rec["before"] = {n: p.grad.clone() if p.grad is not None else torch.zeros_like(p)
                         for n, p in named.items()}
        begin()

    def hook_end():
        end()
        rec["fresh"] = {n: p.grad - rec["before"][n] for n, p in named.items()}

    def hook_step(**kw):
        tr.optimizer.wait()
        rec["clipped"] = {n: p.grad.clone() for n, p in named.items()}
        rec["p0"] = {n: p.detach().clone() for n, p in named.items()}
        ostep(**kw)
        tr.optimizer.wait()
        rec["upd"] = {n: p.detach() - rec["p0"][n] for n, p in named.items()}
    tr.reducer.begin, tr.reducer.end, tr.optimizer.step = hook_begin, hook_end, hook_step
    ctx = torch.from_numpy(seeded.randn("trainer.ctx", (1, 20, 64))).to(DEV).to(torch.bfloat16)
    x0 = torch.from_numpy(seeded.randn("trainer.x0", (1, 16, 3, 10, 14))).to(DEV).to(torch.bfloat16)
    fm = FlowMatchDiscreteScheduler(shift=5.0)
    fm.set_timesteps(1000, dtype=torch.int64)
    torch_opt, torch_params = None, None
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    report = {}
    for step in (0, 1):
        for phase in ("sft", "rwd"):
            tag = f"it{step}:{phase}"
            rec.pop("upd", None)
            if phase == "sft":
                noise = torch.from_numpy(seeded.randn(f"trainer.sft_noise.{step}", (1, 16, 3, 10, 14)))
                out = tr.sft_step(step, x0, ctx, 105, noise=noise.to(DEV).to(torch.bfloat16),
                                  timestep=fm.timesteps[[int(g["sft_idx"][step])]].to(DEV))
                assert abs(float(out["loss"]) / float(g[tag + ":loss"]) - 1) < 1e-2, tag
            else:
                noise = torch.from_numpy(seeded.randn(f"trainer.rwd_noise.{step}", (1, 16, 3, 10, 14)))
                out = tr.reward_step(step, x0, ctx, 105, mid_timestep=int(g["mid"][step]),
                                     noise=noise.to(DEV).to(torch.bfloat16))
                assert abs(float(out["reward"]) - float(g[tag + ":reward"])) < 3e-3, tag
                assert abs(float(out["loss"]) - float(g[tag + ":loss"])) < \
                    2e-3 * abs(float(g[tag + ":loss"])) + 1e-4, tag
            report[tag + ":grad_norm/ref"] = float(out["grad_norm"]) / float(g[tag + ":grad_norm"])
            # fresh gradient of this backward: vs the reference (SFT) and vs the fp32 truth
            fresh = {n: _Grads(t) for n, t in rec["fresh"].items()}
            e_ref = summary_errors(_as_grads_of(g, tag + ":fresh:"), "", fresh)
            e_t32 = summary_errors(_as_grads_of(g, "t32:" + tag + ":fresh:"), "", fresh)
            assert len(e_ref) > 60 and len(e_t32) == len(e_ref)
            report[tag + ":vs ref med/max"] = (med(e_ref.values()), max(e_ref.values()))
            report[tag + ":vs truth med (ref runs: %.4f-%.4f)" % (
                min(g[f"floor:{tag}:med"]), max(g[f"floor:{tag}:med"]))] = med(e_t32.values())
            assert all(torch.isfinite(t).all() for t in rec["fresh"].values()), tag
            if phase == "sft":
                worst = sorted(e_ref.items(), key=lambda kv: -kv[1])[:3]
                assert max(e_ref.values()) < 3e-2, (tag, worst)
                assert abs(report[tag + ":grad_norm/ref"] - 1) < 1e-2, (tag, report)
            else:
                assert sum(int(t.abs().sum() > 0) for t in rec["fresh"].values()) > 60, tag
            # optimizer steps: only at the boundary iteration, in both steps
            assert ("upd" in rec) == (step == 1), tag
            if step == 1:
                if torch_opt is None:
                    torch_params = {n: rec["p0"][n].clone().requires_grad_(True) for n in named}
                    torch_opt = torch.optim.AdamW(list(torch_params.values()), lr=lr,
                                                  betas=(0.9, 0.999), weight_decay=0.01, eps=1e-8)
                with torch.no_grad():
                    for n, p in torch_params.items():
                        p.copy_(rec["p0"][n])
                        p.grad = rec["clipped"][n].clone()
                torch_opt.step()
                for n, p in torch_params.items():
                    d_ours, d_torch = rec["upd"][n], p.detach() - rec["p0"][n]
                    tol = 1e-3 * lr + 4 * torch.finfo(torch.float32).eps * rec["p0"][n].abs()
                    assert bool(((d_ours - d_torch).abs() <= tol).all()), (tag, n)
                agree = []
                for n, o, k in _summary_pairs(g, tag + ":upd:", rec["upd"]):
                    agree.append(float((torch.sign(o) == torch.sign(torch.from_numpy(g[k])))
                                       .double().mean()))
                for k in g:
                    if k.startswith(tag + ":upd:norm/"):
                        n = k[len(tag + ":upd:norm/"):]
                        assert abs(rec["upd"][n].double().norm().item() / float(g[k]) - 1) < 2e-3, \
                            (tag, n)
                # the reference's own bf16 run agrees in sign with the truth on >= 98.8 % per tensor
                assert min(agree) >= 0.97 and sum(agree) / len(agree) >= 0.99, (tag, min(agree))
    print(fixture, report)
    assert tr.optimizer.step_count == 2


def test_prfl_trainer_skips_nan_loss():
    """`train_prfl.py:800-807`: a NaN / Inf reward loss skips backward and optimizer step (even
    at an accumulation boundary) and reports loss 0 / grad_norm 0."""
    from prfl_amd.network import MLP, QueryAttention
    from prfl_amd.train import PRFLTrainer, build_lrm
    gen = toy_model("t2v")
    lrm = build_lrm(toy_model("t2v"), [0])
    qa = QueryAttention(256, 1, 8, 0., return_type="query").to(DEV).requires_grad_(False)
    mlp = MLP(256).to(DEV).requires_grad_(False)
    with torch.no_grad():
        mlp.fc3.bias.fill_(float("nan"))
    tr = PRFLTrainer(gen, lrm, qa, mlp, grad_accum=1.0, feature_layer=(1,))
    lat = torch.randn(1, 16, 3, 10, 14, device=DEV).to(torch.bfloat16)
    ctx = torch.randn(1, 20, 64, device=DEV).to(torch.bfloat16)
    before = {n: p.detach().clone() for n, p in gen.named_parameters()}
    b = tr.reward_step(0, lat, ctx, 105, mid_timestep=1)
    torch.cuda.synchronize()
    assert b.get("skipped") and float(b["loss"]) == 0.0 and b["grad_norm"] == 0
    assert tr.optimizer.step_count == 0
    assert all(p.grad is None for p in gen.parameters())
    assert all(torch.equal(before[n], p) for n, p in gen.named_parameters())


def test_prfl_trainer_iteration_runs():
    """One SFT + reward iteration through PRFLTrainer (optimizer step included)."""
    from prfl_amd.network import MLP, QueryAttention
    from prfl_amd.train import PRFLTrainer, build_lrm
    gen = toy_model("t2v")
    lrm = build_lrm(toy_model("t2v"), [0])
    qa = QueryAttention(256, 1, 8, 0., return_type="query").to(DEV).requires_grad_(False)
    mlp = MLP(256).to(DEV).requires_grad_(False)
    tr = PRFLTrainer(gen, lrm, qa, mlp, grad_accum=1.0, feature_layer=(1,))
    before = {n: p.detach().clone() for n, p in gen.named_parameters()}
    lat = torch.randn(1, 16, 3, 10, 14, device=DEV).to(torch.bfloat16)
    ctx = torch.randn(1, 20, 64, device=DEV).to(torch.bfloat16)
    a = tr.sft_step(0, lat, ctx, 105)
    b = tr.reward_step(0, lat, ctx, 105, mid_timestep=2)
    torch.cuda.synchronize()
    assert torch.isfinite(a["loss"]) and torch.isfinite(b["loss"])
    assert float(a["grad_norm"]) > 0 and float(b["grad_norm"]) > 0
    moved = sum(int(not torch.equal(before[n], p)) for n, p in gen.named_parameters())
    assert moved > 50 and tr.optimizer.step_count == 2   # SFT and reward both stepped


def test_flash_attention_api():
    from prfl_amd.attention import flash_attention
    from oracle import wan_oracle as O
    g = torch.Generator().manual_seed(9)
    q = torch.randn(2, 70, 2, 128, generator=g)
    k = torch.randn(2, 90, 2, 128, generator=g)
    v = torch.randn(2, 90, 2, 128, generator=g)
    out = flash_attention(q.to(DEV), k.to(DEV), v.to(DEV), k_lens=torch.tensor([90, 41]))
    assert out.dtype == torch.float32
    for b, kl in enumerate([90, 41]):
        ref = O.attention(q[b:b + 1], k[b:b + 1], v[b:b + 1], k_len=kl if kl < 90 else None)
        assert rel(out[b:b + 1], ref) < 5e-3
    # full q_lens (the only lengths the reference's unflatten accepts) change nothing; k_lens as
    # a device tensor or a list give the same result; q_scale multiplies the bf16 q (attention.py:86)
    out2 = flash_attention(q.to(DEV), k.to(DEV), v.to(DEV), q_lens=torch.tensor([70, 70], device=DEV),
                           k_lens=torch.tensor([90, 41], device=DEV))
    assert torch.equal(out2, out)
    out3 = flash_attention(q.to(DEV), k.to(DEV), v.to(DEV), k_lens=[90, 41], q_scale=0.5)
    ref3 = flash_attention(q.to(DEV).to(torch.bfloat16) * 0.5, k.to(DEV), v.to(DEV), k_lens=[90, 41])
    assert torch.equal(out3, ref3.float())


def test_toy_pavrm_steps_vs_reference(golden):
    """Two PAVRM 'ce' steps (train_pavrm.py:671-920) through PAVRMTrainer vs the reference run
    of make_golden.case_toy_pavrm: features, probability, BCE loss, every trunk / QueryAttention /
    MLP gradient and the transformer grad norm (clip_grad_norm_ over the trunk only) of both
    steps (the second on AdamW-updated weights).  The update itself is checked against
    torch.optim.AdamW with the reference's three parameter groups, given our clipped grads."""
    from prfl_amd.network import MLP, QueryAttention
    from prfl_amd.train import PAVRMTrainer
    g = golden("toy_pavrm")
    lrm = toy_model("t2v")
    lrm.blocks = torch.nn.ModuleList(list(lrm.blocks))
    del lrm.head
    lrm.head = None
    qa = QueryAttention(256, 1, 8, 0., return_type="query")
    qa.load_state_dict(seeded_params(qa_shapes(256), prefix="pqa."))
    mlp = MLP(256)
    mlp.load_state_dict(seeded_params(mlp_shapes(256), prefix="pmlp."))
    qa, mlp = qa.to(DEV), mlp.to(DEV)
    tr = PAVRMTrainer(lrm, qa, mlp, feature_layer=(2,))
    assert tr.opt_trunk.lr == tr.opt_head.lr == 1e-6          # learning_rate_mlp unset (CE)
    named = {**dict(lrm.named_parameters()), **{"qa." + k: v for k, v in qa.named_parameters()},
             **{"mlp." + k: v for k, v in mlp.named_parameters()}}
    ctx = torch.from_numpy(g["ctx"]).to(DEV).to(torch.bfloat16)
    grads = {}
    orig_step = {}

    def capture(opt, tag):          # grads as the optimizer sees them (after the trunk clip)
        f = opt.step

        def step(**kw):
            grads[tag] = [p.grad.detach().clone() for p in opt.params]
            orig_step[tag] = [p.detach().clone() for p in opt.params]
            f(**kw)
        opt.step = step
    capture(tr.opt_trunk, "trunk")
    capture(tr.opt_head, "head")
    ref_states = {}
    for s in range(2):
        x0 = torch.from_numpy(g[f"s{s}:x0"]).to(DEV).to(torch.bfloat16)
        noise = torch.from_numpy(g[f"s{s}:noise"]).to(DEV).to(torch.bfloat16)
        t = tr.fm.timesteps[[int(g[f"s{s}:idx"])]].to(DEV)
        label = torch.tensor([float(g[f"s{s}:label"])], device=DEV)
        # raw (pre-clip) grads: record them in a backward hook of the reducer's end()
        raw = {}
        end = tr.reducer.end

        def end_hook():
            end()
            for n, p in named.items():
                if p.grad is not None:
                    raw[n] = p.grad.detach().clone()
        tr.reducer.end = end_hook
        out = tr.step(x0, ctx, 105, label, noise=noise, timestep=t)
        tr.reducer.end = end
        assert abs(float(out["prob"].flatten()[0]) - float(g[f"s{s}:prob"].flatten()[0])) < 3e-3
        assert abs(float(out["loss"]) / float(g[f"s{s}:loss"]) - 1) < 1e-2
        assert abs(float(out["grad_norm"]) / float(g[f"s{s}:grad_norm"]) - 1) < 3e-2
        # gradients vs the fp32 truth of the same step (unrounded attention, no autocast,
        # make_golden._toy_pavrm_fp32_truth), next to the reference's own bf16 run: the BCE
        # gradient at p ~ 0.5 through 8-head pooling over both blocks is ill-conditioned in bf16
        # (the reference's own run is 7 % / 14 % off the truth at the median at steps 0 / 1)
        ours, refs = {}, {}
        for k, v in g.items():
            if not k.startswith(f"s{s}:") or ":t32:" in k or "grad/" not in k:
                continue
            key = k[len(f"s{s}:"):]
            pre, n = key.split("grad/")
            truth = g[f"s{s}:t32:{pre}grad/{n}"]
            ours[pre + n] = rel(raw[pre + n], truth)
            refs[pre + n] = rel(v, truth)
        assert len(ours) > 30
        med = lambda d: sorted(d.values())[len(d) // 2]  # noqa: E731
        worst = sorted(ours.items(), key=lambda kv: -kv[1])[:5]
        # ours within 1 % of the reference's own median distance (both are bf16 draws around the
        # truth at ~7 %; round 5 measured ratio 1.0002 at step 0 and 0.073 at step 1, where the
        # reference's own run sits 14 % off the truth; the kernels are deterministic, so the gate
        # was tightened from round 3's 1.05; a broken kernel lands at many x)
        print(f"PAVRM toy step {s}: median distance to the fp32 truth ours {med(ours):.4e}, "
              f"reference {med(refs):.4e}, ratio {med(ours) / med(refs):.4f}")
        assert med(ours) <= 1.01 * med(refs), (s, med(ours), med(refs), worst)
        if s == 0:
            # same weights and inputs as the reference: every tensor within 1.5x its worst error
            assert max(ours.values()) <= 1.5 * max(refs.values()), (s, worst, max(refs.values()))
        # at step 1 the weights already differ from the reference's by AdamW's first update,
        # which is ~lr * sign(grad) per element: where the bf16 gradients disagree in sign the
        # weights differ by 2e-6, and block 0's cross-attention gradients (near-uniform attention
        # over 492 identical padded text tokens) amplify that, so only the median is held there
        # the update: torch.optim.AdamW (reference groups) on the same clipped grads
        for tag, opt in (("trunk", tr.opt_trunk), ("head", tr.opt_head)):
            ps = [p.clone().requires_grad_(True) for p in orig_step[tag]]
            ref = torch.optim.AdamW(ps, lr=1e-6, betas=(0.9, 0.999), weight_decay=0.01, eps=1e-8)
            if s == 1:
                ref.load_state_dict(ref_states[tag])
            for p, gr in zip(ps, grads[tag]):
                p.grad = gr
            ref.step()
            moved = 0.0
            for p, q, p0 in zip(ps, opt.params, orig_step[tag]):
                # updates compared, not parameters: one AdamW step moves an element by ~lr, so
                # a bound tied to |p| could not see a skipped update
                d_ref, d_ours = p.detach() - p0, q.detach() - p0
                tol = 1e-3 * 1e-6 + 4 * torch.finfo(torch.float32).eps * p0.abs()
                assert bool(((d_ours - d_ref).abs() <= tol).all())
                moved = max(moved, d_ref.abs().max().item())
            # the step did move the parameters by ~lr (tensors whose gradients are far below
            # AdamW's eps move by much less: lr * |g| / (|g| + eps))
            assert moved > 0.5e-6, (tag, moved)
            ref_states[tag] = ref.state_dict()
