"""Generate the golden parity fixtures from the REFERENCE implementation (build container only).

    python tests/golden/make_golden.py          # writes tests/golden/*.npz

Runs the reference modules from /root/reference (imported via ``ref_import.py``) on CPU under
``torch.autocast("cpu", bfloat16)``, which with the amp shim reproduces the CUDA autocast precision
flow of the training scripts (`train_prfl.py:686,723,762`).  Weights and inputs come from
``seeded.py``.  The fixtures hold inputs and outputs only (data); the GPU box regenerates the
same weights from ``seeded.py``.  Each case cites the reference lines it exercises.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import seeded  # noqa: E402
from ref_import import import_reference  # noqa: E402

torch.set_num_threads(8)
M, NET, UNIPC, FM, DU = import_reference()
AC = dict(device_type="cpu", dtype=torch.bfloat16)

TOY = dict(dim=256, ffn_dim=512, freq_dim=256, text_dim=64, num_heads=2, num_layers=2,
           out_dim=16, text_len=512)
TOY_LATENT = (16, 3, 10, 14)     # -> grid (3,5,7), L=105 (not a multiple of any tile)


def np32(t):
    return t.detach().float().cpu().numpy()


def load_seeded(module, seed=seeded.BASE_SEED, prefix=""):
    shapes = [(k, tuple(v.shape)) for k, v in module.state_dict().items()]
    sd = seeded.make_state_dict([(prefix + k, s) for k, s in shapes], seed)
    sd = {k[len(prefix):]: torch.from_numpy(v) for k, v in sd.items()}
    module.load_state_dict(sd)
    return module


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: (v if isinstance(v, np.ndarray) else np.asarray(v))
                                 for k, v in arrs.items()})
    print("wrote", path, f"{os.path.getsize(path)/1e6:.2f} MB")


def grads_of(module, keep_full=True, head=256, full_max=70000):
    """Full grads for small params; for large ones: norm, first `head` values and a projection
    onto a seeded random vector (`gproj`), which pins every element at O(1/sqrt(n)) weight."""
    out = {}
    for n, p in module.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().float().flatten()
        if keep_full and g.numel() <= full_max:
            out["grad/" + n] = g.numpy()
        else:
            r = torch.from_numpy(seeded.randn("proj:" + n, (g.numel(),)))
            out["gnorm/" + n] = np.float64(g.double().norm().item())
            out["ghead/" + n] = g[:head].numpy()
            out["gproj/" + n] = np.float64((g.double() * r.double()).sum().item())
    return out


# ----------------------------------------------------------------------------------------------
def case_ops():
    """rope_apply (`model.py:61-103`), WanRMSNorm (`:106-122`), WanLayerNorm (`:125-135`)."""
    d = 128
    freqs = torch.cat([M.rope_params(1024, d - 4 * (d // 6)), M.rope_params(1024, 2 * (d // 6)),
                       M.rope_params(1024, 2 * (d // 6))], dim=1)
    x = torch.from_numpy(seeded.randn("rope.x", (1, 112, 2, d)))
    grid = torch.tensor([[3, 5, 7]])
    rope = M.rope_apply(x, grid, freqs)                       # 105 rotated + 7 pass-through rows
    rms = load_seeded(M.WanRMSNorm(256, eps=1e-6), prefix="rms.norm_q.")
    xr = torch.from_numpy(seeded.randn("rms.x", (1, 40, 256), 3.0)).to(torch.bfloat16)
    rms_out = rms(xr)                                          # bf16 * fp32 weight -> fp32
    ln = M.WanLayerNorm(256, 1e-6)
    ln_aff = load_seeded(M.WanLayerNorm(256, 1e-6, elementwise_affine=True), prefix="ln.norm3.")
    xl = torch.from_numpy(seeded.randn("ln.x", (1, 40, 256), 2.0)) + 0.5
    save("ops", freqs_real=np.ascontiguousarray(torch.view_as_real(freqs).numpy()),
         rope_x=np32(x), rope_grid=grid.numpy(), rope_out=np32(rope),
         rms_x=np32(xr), rms_w=np32(rms.weight), rms_out=np32(rms_out),
         ln_x=np32(xl), ln_out=np32(ln(xl)), ln_out_bf16in=np32(ln(xl.to(torch.bfloat16))),
         ln_aff_w=np32(ln_aff.weight), ln_aff_b=np32(ln_aff.bias), ln_aff_out=np32(ln_aff(xl)))


def _toy_model(model_type):
    torch.manual_seed(0)
    in_dim = 16 if model_type == "t2v" else 36
    m = M.WanModel(model_type=model_type, in_dim=in_dim, **TOY)
    m.__class__.enable_teacache = False
    return load_seeded(m, prefix="toy.")


def case_toy_model(model_type):
    """WanModel.forward/backward end to end (`model.py:534-705`), T2V and I2V."""
    m = _toy_model(model_type)
    x = torch.from_numpy(seeded.randn(model_type + ".x", TOY_LATENT)).requires_grad_(True)
    ctx = torch.from_numpy(seeded.randn(model_type + ".ctx", (20, TOY["text_dim"])))
    t = torch.tensor([700])
    L = 3 * 5 * 7
    kw = {}
    extra = {}
    if model_type == "i2v":
        y = torch.from_numpy(seeded.randn("i2v.y", (20,) + TOY_LATENT[1:]))
        clip = torch.from_numpy(seeded.randn("i2v.clip", (1, 257, 1280)))
        kw = dict(y=[y], clip_fea=clip)
        extra = dict(y=np32(y), clip=np32(clip))
    with torch.autocast(**AC):
        out = m(x=[x], t=t, context=[ctx], seq_len=L, **kw)[0]
    w = torch.from_numpy(seeded.randn(model_type + ".w", tuple(out.shape)))
    (out * w).sum().backward()
    # LRM feature tap (`model.py:656-670`, `train_prfl.py:762-767`)
    m.zero_grad()
    with torch.autocast(**AC):
        feats = m(x=[x.detach()], t=t, context=[ctx], seq_len=L, output_features=True,
                  selected_layers=[1], **kw)
    save("toy_" + model_type, x=np32(x), ctx=np32(ctx), t=t.numpy(), out=np32(out),
         upstream=np32(w), dx=np32(x.grad), feat1=np32(feats[0]), **extra,
         **{k: v for k, v in _saved_grads.items()})


_saved_grads = {}


def case_toy_model_with_grads(model_type):
    m = _toy_model(model_type)
    global _saved_grads
    x = torch.from_numpy(seeded.randn(model_type + ".x", TOY_LATENT)).requires_grad_(True)
    ctx = torch.from_numpy(seeded.randn(model_type + ".ctx", (20, TOY["text_dim"])))
    t = torch.tensor([700])
    kw = {}
    if model_type == "i2v":
        kw = dict(y=[torch.from_numpy(seeded.randn("i2v.y", (20,) + TOY_LATENT[1:]))],
                  clip_fea=torch.from_numpy(seeded.randn("i2v.clip", (1, 257, 1280))))
    with torch.autocast(**AC):
        out = m(x=[x], t=t, context=[ctx], seq_len=105, **kw)[0]
    w = torch.from_numpy(seeded.randn(model_type + ".w", tuple(out.shape)))
    (out * w).sum().backward()
    _saved_grads = grads_of(m)


def _real_block(kind):
    blk = M.WanAttentionBlock(kind, 5120, 13824, 40, (-1, -1), True, True, 1e-6)
    return load_seeded(blk, prefix="blocks.0.")


def case_real_block(kind):
    """One 14B WanAttentionBlock fwd/bwd at real width (C=5120, 40 heads, F=13824), L=48."""
    tag = "t2v" if kind.startswith("t2v") else "i2v"
    blk = _real_block(kind)
    d = 128
    freqs = torch.cat([M.rope_params(1024, d - 4 * (d // 6)), M.rope_params(1024, 2 * (d // 6)),
                       M.rope_params(1024, 2 * (d // 6))], dim=1)
    L, Lc = 48, (512 if tag == "t2v" else 769)
    x = torch.from_numpy(seeded.randn("blk.x", (1, L, 5120))).requires_grad_(True)
    e = torch.from_numpy(seeded.randn("blk.e", (1, 6, 5120), 0.1)).requires_grad_(True)
    ctx = torch.from_numpy(seeded.randn("blk.ctx" + tag, (1, Lc, 5120))).to(torch.bfloat16)
    ctx.requires_grad_(True)
    grid = torch.tensor([[2, 4, 6]])
    with torch.autocast(**AC):
        out = blk(x, e, torch.tensor([L]), grid, freqs, ctx, None)
    up = torch.from_numpy(seeded.randn("blk.up" + tag, (1, L, 5120)))
    (out * up).sum().backward()
    # inputs are regenerated from seeded.py on the GPU box (names above); dctx is summarised
    g = ctx.grad.detach().float().flatten()
    r = torch.from_numpy(seeded.randn("proj:dctx", (g.numel(),)))
    save("real_block_" + tag, grid=grid.numpy(), out=np32(out), dx=np32(x.grad), de=np32(e.grad),
         dctx_head=np32(ctx.grad[0, :8]), dctx_norm=np.float64(g.double().norm().item()),
         dctx_proj=np.float64((g.double() * r.double()).sum().item()),
         **grads_of(blk, keep_full=False))


def case_reward_head():
    """QueryAttention + MLP + sigmoid + PRFL hinge (`network.py:8-152`, `train_prfl.py:780-798`)."""
    qa = NET.QueryAttention(feature_dim=5120, num_queries=1, num_heads=8, dropout=0.,
                            return_type="query")
    load_seeded(qa, prefix="qa.")
    mlp = load_seeded(NET.MLP(5120), prefix="mlp.")
    feats = torch.from_numpy(seeded.randn("qa.feat", (1, 1, 48, 5120), 1.0)).requires_grad_(True)
    with torch.autocast(**AC):
        pooled = qa(feats)                                   # 4-D path (`network.py:65-69`)
        r = NET.forward_mlp(mlp, pooled)
        loss = 0.1 * torch.relu(-r.squeeze() + 2).mean()
    loss.backward()
    save("reward_head", feat=np32(feats), pooled=np32(pooled), reward=np32(r), loss=np32(loss),
         dfeat=np32(feats.grad), **{k: v for k, v in grads_of(qa).items()}, **grads_of(mlp))


def case_schedulers():
    """FlowUniPCMultistepScheduler (`fm_solvers_unipc.py`) and FlowMatchDiscreteScheduler."""
    sch = UNIPC.FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1,
                                            use_dynamic_shifting=False)
    sch.set_timesteps(num_inference_steps=40, device="cpu", shift=5.0)
    ts = sch.timesteps.clone()
    sig = sch.sigmas.clone()
    lat = torch.from_numpy(seeded.randn("unipc.lat", (1, 16, 3, 10, 14))).to(torch.bfloat16)
    traj, outs = [], []
    for i in range(6):
        mo = torch.from_numpy(seeded.randn(f"unipc.mo{i}", (1, 16, 3, 10, 14)))
        outs.append(np32(mo))
        lat = sch.step(mo, ts[i], lat, return_dict=False)[0]
        traj.append(np32(lat))
    # differentiable step (the reward gradient path, `train_prfl.py:733-735`)
    mo = torch.from_numpy(seeded.randn("unipc.mo6", (1, 16, 3, 10, 14))).requires_grad_(True)
    prev = sch.step(mo, ts[6], lat, return_dict=False)[0]
    w = torch.from_numpy(seeded.randn("unipc.w", (1, 16, 3, 10, 14)))
    (prev.float() * w).sum().backward()
    fm = FM.FlowMatchDiscreteScheduler(shift=5.0)
    fm.set_timesteps(1000, dtype=torch.int64)
    torch.manual_seed(7)
    t_s, s_s = fm.get_train_timestep_and_sigma(weighting_scheme="uniform", batch_size=1,
                                               n_dim=5)
    save("schedulers", unipc_timesteps=ts.numpy(), unipc_sigmas=sig.numpy(),
         unipc_lat0=np32(torch.from_numpy(seeded.randn("unipc.lat", (1, 16, 3, 10, 14)))
                         .to(torch.bfloat16)),
         unipc_model_outputs=np.stack(outs), unipc_traj=np.stack(traj), unipc_mo6=np32(mo),
         unipc_prev6=np32(prev), unipc_w=np32(w), unipc_dmo6=np32(mo.grad),
         fm_sigmas=fm.sigmas.numpy(), fm_timesteps=fm.timesteps.numpy(),
         fm_sample_t=t_s.numpy(), fm_sample_sigma=np32(s_s))


def case_toy_prfl():
    """Toy PRFL reward step + SFT step, restating `train_prfl.py:585-835` and `:900-977`."""
    gen = _toy_model("t2v")
    lrm = _toy_model("t2v")
    lrm.blocks = torch.nn.ModuleList([lrm.blocks[0]])      # trainable_blocks [0] (`:241-254`)
    del lrm.head
    lrm.head = None
    for p in lrm.parameters():
        p.requires_grad_(False)
    qa = load_seeded(NET.QueryAttention(256, 1, 8, 0., return_type="query"), prefix="tqa.")
    mlp = load_seeded(NET.MLP(256), prefix="tmlp.")
    for p in list(qa.parameters()) + list(mlp.parameters()):
        p.requires_grad_(False)
    sch = UNIPC.FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1,
                                            use_dynamic_shifting=False)
    sch.set_timesteps(num_inference_steps=40, device="cpu", shift=5.0)
    ts = sch.timesteps
    ctx = torch.from_numpy(seeded.randn("prfl.ctx", (1, 20, TOY["text_dim"]))).to(torch.bfloat16)
    latent = torch.from_numpy(seeded.randn("prfl.noise", (1,) + TOY_LATENT)).to(torch.bfloat16)
    mid = 3
    L = 105
    with torch.no_grad():
        for i in range(mid):
            with torch.autocast(**AC):
                npred = DU.list2batch(gen(x=DU.batch2list(latent), t=torch.tensor([ts[i]]),
                                          context=DU.batch2list(ctx), seq_len=L))
                latent = sch.step(npred, ts[i], latent, return_dict=False)[0]
    roll = latent.clone()
    with torch.autocast(**AC):
        npred = DU.list2batch(gen(x=DU.batch2list(latent), t=torch.tensor([ts[mid]]),
                                  context=DU.batch2list(ctx), seq_len=L))
    latent = sch.step(npred, ts[mid], latent, return_dict=False)[0]
    with torch.autocast(**AC):
        feats = DU.list2batch(lrm(x=DU.batch2list(latent), t=torch.tensor([ts[mid + 1]]),
                                  context=DU.batch2list(ctx), seq_len=L, output_features=True,
                                  selected_layers=[1]))
        r = NET.forward_mlp(mlp, qa(feats))
        loss = 0.1 * torch.relu(-r.squeeze() + 2).mean()
    loss = loss / 5.0
    loss.backward()
    g_reward = grads_of(gen)
    # SFT flow-matching step (`:900-971`), fixed draw
    gen.zero_grad()
    fm = FM.FlowMatchDiscreteScheduler(shift=5.0)
    fm.set_timesteps(1000, dtype=torch.int64)
    x0 = torch.from_numpy(seeded.randn("sft.x0", (1,) + TOY_LATENT)).to(torch.bfloat16)
    noise = torch.from_numpy(seeded.randn("sft.noise", (1,) + TOY_LATENT)).to(torch.bfloat16)
    idx = 613
    timestep = fm.timesteps[[idx]]
    sigma = fm.sigmas[[idx]].float().view(1, 1, 1, 1, 1)
    noisy = fm.add_noise(x0, noise, sigma)
    with torch.autocast(**AC):
        pred = DU.list2batch(gen(x=DU.batch2list(noisy), t=timestep, context=DU.batch2list(ctx),
                                 seq_len=L))
    target = fm.get_train_target(x0, noise)
    sft_loss = torch.mean((pred.float() - target.float()) ** 2) / 5.0
    sft_loss.backward()
    g_sft = {"sft:" + k: v for k, v in grads_of(gen).items()}
    save("toy_prfl", ctx=np32(ctx), noise=np32(torch.from_numpy(
        seeded.randn("prfl.noise", (1,) + TOY_LATENT)).to(torch.bfloat16)), mid=np.int64(mid),
        rollout=np32(roll), npred=np32(npred), stepped=np32(latent), feat=np32(feats),
        reward=np32(r), loss=np32(loss), x0=np32(x0), sft_noise=np32(noise), sft_idx=np.int64(idx),
        sft_timestep=fm.timesteps[[idx]].numpy(), sft_sigma=np32(sigma), sft_pred=np32(pred),
        sft_loss=np32(sft_loss), **g_reward, **g_sft)


SPLIT_MIDS = (0, 3)


def _unipc_state(sch):
    """The reference scheduler's state before a step: what the grad-enabled step reads."""
    st = {"state:lon": np.int64(sch.lower_order_nums), "state:this_order": np.int64(getattr(sch, "this_order", 1)),
          "state:step_index": np.int64(-1 if sch.step_index is None else sch.step_index)}
    for j, mo in enumerate(sch.model_outputs):
        if mo is not None:
            st[f"state:mo{j}"] = np32(mo)
            st[f"state:mo{j}:bf16"] = np.bool_(mo.dtype == torch.bfloat16)
    if sch.last_sample is not None:
        st["state:last"] = np32(sch.last_sample)
        st["state:last:bf16"] = np.bool_(sch.last_sample.dtype == torch.bfloat16)
    return st


def _toy_prfl_models():
    gen = _toy_model("t2v")
    lrm = _toy_model("t2v")
    lrm.blocks = torch.nn.ModuleList([lrm.blocks[0]])
    del lrm.head
    lrm.head = None
    for p in lrm.parameters():
        p.requires_grad_(False)
    qa = load_seeded(NET.QueryAttention(256, 1, 8, 0., return_type="query"), prefix="tqa.")
    mlp = load_seeded(NET.MLP(256), prefix="tmlp.")
    for p in list(qa.parameters()) + list(mlp.parameters()):
        p.requires_grad_(False)
    return gen, lrm, qa, mlp


def _lrm_pool(lrm, qa, stepped, t1, ctx, ac):
    """LRM feature tap + QueryAttention (`train_prfl.py:745-790`) from a leaf copy of the stepped
    latent: (leaf, pooled)."""
    leaf = stepped.detach().clone().requires_grad_(True)
    with torch.autocast(**ac):
        feats = DU.list2batch(lrm(x=DU.batch2list(leaf), t=t1, context=DU.batch2list(ctx),
                                  seq_len=105, output_features=True, selected_layers=[1]))
        pooled = qa(feats)
    return leaf, pooled


def _mlp_hinge(mlp, pooled, ac):
    """MLP + sigmoid + hinge / GA (`train_prfl.py:791-798`, GA 5) from a leaf copy of the
    pooled feature: (loss, reward, d loss / d pooled)."""
    p = pooled.detach().clone().requires_grad_(True)
    with torch.autocast(**ac):
        r = NET.forward_mlp(mlp, p)
        loss = 0.1 * torch.relu(-r.squeeze() + 2).mean()
    loss = loss / 5.0
    loss.backward()
    return loss, r, p.grad


def case_toy_prfl_split():
    """The reward chain of `train_prfl.py:703-830` cut at the pooled feature and at the stepped
    latent, so each piece is pinned on the reference's own inputs, without the bf16 noise of the
    pieces before it:

    * head: MLP + sigmoid + hinge from the reference's pooled feature -> d(pooled).  This is the
      one non-smooth piece: its ReLUs switch for units within a bf16 ulp of zero, which is what
      makes whole-chain bf16 runs land 1-8 % apart (the reference's own bf16 head is 4.6-7.5 %
      from its fp32 evaluation on the same input);
    * trunk: LRM + QueryAttention backward from the reference's stepped bf16 latent with the
      reference's d(pooled) upstream -> d(stepped) (smooth: the reference is 0.5 % from the fp32
      truth here);
    * generator: the grad-enabled generator step + differentiable UniPC step from the
      reference's pre-step latent and scheduler state, back-propagating the reference's
      d(stepped) -> every generator gradient.

    Cutting does not change the reference's arithmetic: the gradients reaching the pooled feature
    and the bf16 stepped latent are the same tensors as in the uncut backward.  Each piece also
    has its fp32 truth on the same inputs.  Two mids: 0 (no rollout, order-1 step, no corrector)
    and 3 (corrector + order-2 predictor from the rollout's history)."""
    ctx = torch.from_numpy(seeded.randn("prfl.ctx", (1, 20, TOY["text_dim"]))).to(torch.bfloat16)
    out = {"ctx": np32(ctx)}
    no_ac = dict(AC, enabled=False)
    for mid in SPLIT_MIDS:
        pre = f"m{mid}:"
        gen, lrm, qa, mlp = _toy_prfl_models()
        sch = UNIPC.FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1,
                                                use_dynamic_shifting=False)
        sch.set_timesteps(num_inference_steps=40, device="cpu", shift=5.0)
        ts = sch.timesteps
        latent = torch.from_numpy(seeded.randn("prfl.noise", (1,) + TOY_LATENT)).to(torch.bfloat16)
        with torch.no_grad():
            for i in range(mid):
                with torch.autocast(**AC):
                    npred = DU.list2batch(gen(x=DU.batch2list(latent), t=torch.tensor([ts[i]]),
                                              context=DU.batch2list(ctx), seq_len=105))
                    latent = sch.step(npred, ts[i], latent, return_dict=False)[0]
        state = _unipc_state(sch)
        pre_lat = latent.clone()
        with torch.autocast(**AC):
            npred = DU.list2batch(gen(x=DU.batch2list(latent), t=torch.tensor([ts[mid]]),
                                      context=DU.batch2list(ctx), seq_len=105))
        stepped = sch.step(npred, ts[mid], latent, return_dict=False)[0]
        t1 = torch.tensor([ts[mid + 1]])
        leaf, pooled = _lrm_pool(lrm, qa, stepped, t1, ctx, AC)
        loss, r, dpool = _mlp_hinge(mlp, pooled, AC)
        pooled.backward(dpool)                                   # the trunk piece
        dstep = leaf.grad
        stepped.backward(dstep)                                  # the generator piece
        g_gen = grads_of(gen, head=4096, full_max=4096)
        # fp32 truths of each piece on the same inputs and upstream gradients
        saved = M.flash_attention
        M.flash_attention = _exact_attention
        try:
            gen32, lrm32, qa32, mlp32 = _toy_prfl_models()
            _, r32, dpool32 = _mlp_hinge(mlp32, pooled.float(), no_ac)
            leaf32, pooled32 = _lrm_pool(lrm32, qa32, stepped.float(), t1, ctx.float(), no_ac)
            pooled32.backward(dpool.float())
            dstep32 = leaf32.grad
            sch32 = UNIPC.FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1,
                                                      use_dynamic_shifting=False)
            sch32.set_timesteps(num_inference_steps=40, device="cpu", shift=5.0)
            sch32.model_outputs = [None if k not in state else torch.from_numpy(state[k])
                                   for k in ("state:mo0", "state:mo1")]
            sch32.last_sample = (torch.from_numpy(state["state:last"]) if "state:last" in state
                                 else None)
            sch32.lower_order_nums = int(state["state:lon"])
            sch32.this_order = int(state["state:this_order"])
            if int(state["state:step_index"]) >= 0:
                sch32._step_index = int(state["state:step_index"])
            npred32 = DU.list2batch(gen32(x=DU.batch2list(pre_lat.float()),
                                          t=torch.tensor([ts[mid]]),
                                          context=DU.batch2list(ctx.float()), seq_len=105))
            stepped32 = sch32.step(npred32, ts[mid], pre_lat.float(), return_dict=False)[0]
            stepped32.backward(dstep.float())
            g_gen32 = grads_of(gen32, head=4096, full_max=4096)
        finally:
            M.flash_attention = saved
        e = lambda a, b: ((a.float() - b).norm() / b.norm()).item()  # noqa: E731
        print(f"mid {mid}: reward {r.item():.5f} (truth {r32.item():.5f}); reference vs truth: "
              f"d(pooled) {e(dpool, dpool32):.4f}, d(stepped) {e(dstep, dstep32):.4f}")
        out.update({pre + "pre": np32(pre_lat), pre + "npred": np32(npred),
                    pre + "stepped": np32(stepped), pre + "t_mid": np.int64(ts[mid]),
                    pre + "t1": np.int64(ts[mid + 1]), pre + "loss": np32(loss),
                    pre + "reward": np32(r), pre + "pooled": np32(pooled),
                    pre + "dpool": np32(dpool), pre + "dstep": np32(dstep),
                    pre + "t32:dpool": np32(dpool32), pre + "t32:dstep": np32(dstep32),
                    pre + "t32:reward": np32(r32),
                    **{pre + k: v for k, v in state.items()},
                    **{pre + k: v for k, v in g_gen.items()},
                    **{pre + "t32:" + k: v for k, v in g_gen32.items()}})
    save("toy_prfl_split", **out)


def case_toy_pavrm():
    """Toy PAVRM training step with the 'ce' loss, restating `train_pavrm.py:671-920` on the
    reference modules: `model_init` (`:200-235`: embeddings frozen, trainable_blocks kept, head
    dropped), `optimizer_init` (`:459-506`: ONE AdamW over three parameter groups — transformer,
    MLP, QueryAttention — all at `learning_rate` because the CE configs leave
    `learning_rate_mlp` commented out, `train_pavrm_t2v_480.yaml:61-62`), then per step: noise at
    a fixed timestep, 8-block-style feature tap, 4-D QueryAttention pooling (`:793-800`, the
    sp_size > 1 branch our DP run takes), sigmoid MLP, BCE (`:869`), the pre-backward clip that
    sees no gradients (`:883-889`), backward, `transformer.clip_grad_norm_(1.0)` over the
    transformer grads only (`:899`), optimizer.step, zero_grad.  Two steps, so the second one
    runs on AdamW-updated weights with non-zero moments."""
    lrm = _toy_model("t2v")
    for name in ("patch_embedding", "text_embedding", "time_embedding", "time_projection"):
        for p in getattr(lrm, name).parameters():
            p.requires_grad_(False)
    for blk in lrm.blocks:                                   # trainable_blocks [0, 1]
        for p in blk.parameters():
            p.requires_grad_(True)
    del lrm.head
    lrm.head = None
    qa = load_seeded(NET.QueryAttention(256, 1, 8, 0., return_type="query"), prefix="pqa.")
    mlp = load_seeded(NET.MLP(256), prefix="pmlp.")
    tparams = [p for p in lrm.parameters() if p.requires_grad]
    opt = torch.optim.AdamW([{"params": tparams, "lr": 1e-6},
                             {"params": list(mlp.parameters()), "lr": 1e-6},
                             {"params": list(qa.parameters()), "lr": 1e-6}],
                            betas=(0.9, 0.999), weight_decay=0.01, eps=1e-8)
    fm = FM.FlowMatchDiscreteScheduler(shift=5.0)
    fm.set_timesteps(1000, dtype=torch.int64)
    crit = torch.nn.BCELoss()
    ctx = torch.from_numpy(seeded.randn("pavrm.ctx", (1, 20, TOY["text_dim"]))).to(torch.bfloat16)
    out = {"ctx": np32(ctx)}
    for s, (idx, label) in enumerate(((613, 1.0), (287, 0.0))):
        x0 = torch.from_numpy(seeded.randn(f"pavrm.x0.{s}", (1,) + TOY_LATENT)).to(torch.bfloat16)
        noise = torch.from_numpy(seeded.randn(f"pavrm.noise.{s}", (1,) + TOY_LATENT)).to(torch.bfloat16)
        timestep = fm.timesteps[[idx]]
        sigma = fm.sigmas[[idx]].float().view(1, 1, 1, 1, 1)
        noisy = fm.add_noise(x0, noise, sigma)
        with torch.autocast(**AC):
            feats = DU.list2batch(lrm(x=DU.batch2list(noisy), t=timestep, context=DU.batch2list(ctx),
                                      seq_len=105, output_features=True, selected_layers=[2]))
            pooled = qa(feats)
            prob = NET.forward_mlp(mlp, pooled)
        lab = torch.tensor([label])
        loss = crit(prob.squeeze().float(), lab.squeeze().float())
        states = [{k: v.detach().clone() for k, v in m.state_dict().items()} for m in (lrm, qa, mlp)]
        out.update(_toy_pavrm_fp32_truth(s, states, noisy, fm.timesteps[[idx]], ctx, lab))
        loss.backward()
        g = {f"s{s}:" + k: v for k, v in grads_of(lrm).items()}
        g.update({f"s{s}:qa." + k: v for k, v in grads_of(qa).items()})
        g.update({f"s{s}:mlp." + k: v for k, v in grads_of(mlp).items()})
        gn = torch.nn.utils.clip_grad_norm_(tparams, max_norm=1.0)
        opt.step()
        opt.zero_grad()
        out.update({f"s{s}:x0": np32(x0), f"s{s}:noise": np32(noise), f"s{s}:idx": np.int64(idx),
                    f"s{s}:label": np.float32(label), f"s{s}:feat": np32(feats),
                    f"s{s}:prob": np32(prob), f"s{s}:loss": np32(loss),
                    f"s{s}:grad_norm": np32(gn), **g})
    save("toy_pavrm", **out)


def _summ(tensors, head=1024, full_max=4096):
    """Per-tensor summary of a {name: tensor} dict: full values for small tensors; for large ones
    the first `head` values, the L2 norm and the projection onto a seeded random vector."""
    out = {}
    for n, g in tensors.items():
        g = g.detach().float().flatten()
        if g.numel() <= full_max:
            out["full/" + n] = g.numpy()
        else:
            r = torch.from_numpy(seeded.randn("proj:" + n, (g.numel(),)))
            out["head/" + n] = g[:head].numpy()
            out["norm/" + n] = np.float64(g.double().norm().item())
            out["proj/" + n] = np.float64((g.double() * r.double()).sum().item())
    return out


TRAINER_GA = 2.0          # gradient_accumulation_steps (the configs' 5.0, shortened to 2)
TRAINER_LR = 5e-6         # train_prfl_t2v_480.yaml optimizer.learning_rate
TRAINER_SFT_IDX = (613, 287)
TRAINER_MID = (2, 1)


def _bump_ulps(t, name, n=8):
    """t (bf16-valued) with n seeded elements moved by one bf16 ulp: a perturbation at the
    resolution of the bf16 state, to sample the chain's own bf16 noise floor."""
    flat = t.to(torch.bfloat16).flatten().clone()
    idx = torch.from_numpy((np.abs(seeded.randn(name, (n,))) * 1e6).astype(np.int64) % flat.numel())
    bits = flat.view(torch.int16)
    sign = torch.from_numpy(np.sign(seeded.randn(name + ".s", (n,)))).to(torch.int16)
    bits[idx] += sign
    return bits.view(torch.bfloat16).view(t.shape).to(t.dtype)


def _trainer_run(truth, perturb=None, mids=TRAINER_MID):
    """Two PRFL iterations (step 0, then step 1 = an optimizer-step boundary for
    gradient_accumulation_steps 2) restating `train_prfl.py` on the reference modules:
    `train_step` (`:900-980`: flow-matching SFT loss / GA, backward, `clip_grad_norm_(1.0)`,
    AdamW step + zero_grad when (step+1) % GA == 0) then `train_step_refl` (`:585-846`: UniPC
    rollout to `mid`, grad-enabled generator step, differentiable UniPC step, frozen 1-block LRM
    + QueryAttention + MLP, hinge, NaN/Inf check and clamp `:800-811`, loss / GA, backward onto
    the SFT step's accumulated grads, clip, AdamW step at the boundary).  AdamW = `optimizer_init`
    (`:479-491`: all generator parameters, lr 5e-6, betas (0.9, 0.999), wd 0.01, eps 1e-8).
    `truth`: the same run in fp32 without autocast, with unrounded attention and fp32 latents:
    the values the bf16 runs approximate.  Records per backward the fresh gradient increment,
    the clipped norm, the losses, and each optimizer step's parameter update."""
    ac = dict(AC, enabled=not truth)
    saved = M.flash_attention
    if truth:
        M.flash_attention = _exact_attention
    try:
        gen = _toy_model("t2v")
        lrm = _toy_model("t2v")
        lrm.blocks = torch.nn.ModuleList([lrm.blocks[0]])
        del lrm.head
        lrm.head = None
        for p in lrm.parameters():
            p.requires_grad_(False)
        qa = load_seeded(NET.QueryAttention(256, 1, 8, 0., return_type="query"), prefix="tqa.")
        mlp = load_seeded(NET.MLP(256), prefix="tmlp.")
        for p in list(qa.parameters()) + list(mlp.parameters()):
            p.requires_grad_(False)
        params = [p for p in gen.parameters() if p.requires_grad]
        named = {n: p for n, p in gen.named_parameters() if p.requires_grad}
        opt = torch.optim.AdamW(params, lr=TRAINER_LR, betas=(0.9, 0.999), weight_decay=0.01,
                                eps=1e-8)
        fm = FM.FlowMatchDiscreteScheduler(shift=5.0)
        fm.set_timesteps(1000, dtype=torch.int64)
        sch = UNIPC.FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1,
                                                use_dynamic_shifting=False)
        lat_dt = torch.float32 if truth else torch.bfloat16
        ctx = torch.from_numpy(seeded.randn("trainer.ctx", (1, 20, TOY["text_dim"]))) \
            .to(torch.bfloat16).to(lat_dt)
        x0 = torch.from_numpy(seeded.randn("trainer.x0", (1,) + TOY_LATENT)).to(torch.bfloat16) \
            .to(lat_dt)
        L = 105
        out = {}

        def backward_and_step(loss, step, tag):
            before = {n: (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p))
                      for n, p in named.items()}
            loss.backward()
            fresh = {n: p.grad.detach() - before[n] for n, p in named.items()}
            out.update({f"{tag}:fresh:" + k: v for k, v in _summ(fresh).items()})
            gn = torch.nn.utils.clip_grad_norm_(params, max_norm=1.0)
            out[f"{tag}:grad_norm"] = np.float64(gn.item())
            if (step + 1) % TRAINER_GA == 0:
                p0 = {n: p.detach().clone() for n, p in named.items()}
                opt.step()
                opt.zero_grad()
                upd = {n: p.detach() - p0[n] for n, p in named.items()}
                out.update({f"{tag}:upd:" + k: v for k, v in _summ(upd).items()})

        for step in (0, 1):
            # ---- train_step (SFT) ----
            noise = torch.from_numpy(seeded.randn(f"trainer.sft_noise.{step}", (1,) + TOY_LATENT)) \
                .to(torch.bfloat16).to(lat_dt)
            idx = TRAINER_SFT_IDX[step]
            timestep = fm.timesteps[[idx]]
            sigma = fm.sigmas[[idx]].float().view(1, 1, 1, 1, 1)
            noisy = fm.add_noise(x0, noise, sigma)
            with torch.autocast(**ac):
                pred = DU.list2batch(gen(x=DU.batch2list(noisy), t=timestep,
                                         context=DU.batch2list(ctx), seq_len=L))
            target = fm.get_train_target(x0, noise)
            weighting = fm.get_train_loss_weighting(sigma)
            loss = torch.mean(weighting.float() * (pred.float() - target.float()) ** 2)
            loss = loss / TRAINER_GA
            out[f"it{step}:sft:loss"] = np.float64(loss.item())
            backward_and_step(loss, step, f"it{step}:sft")
            # ---- train_step_refl (reward) ----
            sch.set_timesteps(num_inference_steps=40, device="cpu", shift=5.0)
            ts = sch.timesteps
            latent = torch.from_numpy(seeded.randn(f"trainer.rwd_noise.{step}", (1,) + TOY_LATENT)) \
                .to(torch.bfloat16).to(lat_dt)
            if perturb is not None:
                latent = _bump_ulps(latent, f"trainer.perturb.{perturb}.{step}")
            mid = mids[step]
            with torch.no_grad():
                for i in range(mid):
                    with torch.autocast(**ac):
                        npred = DU.list2batch(gen(x=DU.batch2list(latent), t=torch.tensor([ts[i]]),
                                                  context=DU.batch2list(ctx), seq_len=L))
                        latent = sch.step(npred, ts[i], latent, return_dict=False)[0]
            with torch.autocast(**ac):
                npred = DU.list2batch(gen(x=DU.batch2list(latent), t=torch.tensor([ts[mid]]),
                                          context=DU.batch2list(ctx), seq_len=L))
            latent = sch.step(npred, ts[mid], latent, return_dict=False)[0]
            with torch.autocast(**ac):
                feats = DU.list2batch(lrm(x=DU.batch2list(latent), t=torch.tensor([ts[mid + 1]]),
                                          context=DU.batch2list(ctx), seq_len=L,
                                          output_features=True, selected_layers=[1]))
                r = NET.forward_mlp(mlp, qa(feats))
                loss = 0.1 * torch.relu(-r.squeeze() + 2).mean()
                assert torch.isfinite(loss) and abs(loss.item()) <= 1e6
            out[f"it{step}:rwd:reward"] = np.float64(r.item())
            loss = loss / TRAINER_GA
            out[f"it{step}:rwd:loss"] = np.float64(loss.item())
            backward_and_step(loss, step, f"it{step}:rwd")
        return out
    finally:
        M.flash_attention = saved


def _fresh_err_stats(run, t32, tag):
    """(median, max) over parameters of the rel-L2 of a run's fresh gradient vs the truth's."""
    errs = []
    for k, v in run.items():
        if k.startswith(tag + ":fresh:") and ("/full/" in k.replace(":fresh:", "/") or
                                              "/head/" in k.replace(":fresh:", "/")):
            t = t32[k]
            errs.append(float(np.linalg.norm(v - t) / max(np.linalg.norm(t), 1e-30)))
    errs.sort()
    return errs[len(errs) // 2], errs[-1]


TRAINER_PERTURB = 8


def case_toy_prfl_trainer(mids=TRAINER_MID, name="toy_prfl_trainer"):
    """PRFLTrainer parity: the reference run, its fp32 truth, and the reference's
    own bf16 noise floor through the reward chain: TRAINER_PERTURB more reference runs whose
    reward-step initial noise differs by one bf16 ulp in 8 elements (the chain's MLP ReLUs switch
    at bf16 resolution, case_toy_prfl_split, so one bf16 run's distance to the truth is a draw
    from this spread, not a fixed number).  `mids` = the reward steps' mid_timestep per
    iteration; the `_mid0` fixture runs both iterations without a rollout."""
    ref = _trainer_run(truth=False, mids=mids)
    t32 = _trainer_run(truth=True, mids=mids)
    tags = [f"it{s}:{p}" for s in (0, 1) for p in ("sft", "rwd")]
    floor = {t: [] for t in tags}
    for i in range(TRAINER_PERTURB):
        run = _trainer_run(truth=False, perturb=i, mids=mids)
        for t in tags:
            floor[t].append(_fresh_err_stats(run, t32, t))
    extra = {}
    for t in tags:
        extra[f"floor:{t}:med"] = np.asarray([m for m, _ in floor[t]])
        extra[f"floor:{t}:max"] = np.asarray([x for _, x in floor[t]])
        print(t, "reference runs' median err vs truth:", np.round(extra[f"floor:{t}:med"], 4),
              "max:", np.round(extra[f"floor:{t}:max"], 4))
    save(name, ga=np.float64(TRAINER_GA), lr=np.float64(TRAINER_LR),
         sft_idx=np.asarray(TRAINER_SFT_IDX), mid=np.asarray(mids), **ref,
         **{"t32:" + k: v for k, v in t32.items()}, **extra)


def _exact_attention(q, k, v, q_lens=None, k_lens=None, dropout_p=0., softmax_scale=None,
                     q_scale=None, causal=False, window_size=(-1, -1), deterministic=False,
                     dtype=None, version=None):
    """Unrounded attention in the inputs' dtype (fp32) for the truth run."""
    if q_scale is not None:
        q = q * q_scale
    scale = softmax_scale if softmax_scale is not None else q.size(-1) ** -0.5
    s = torch.einsum("blnd,bmnd->bnlm", q, k) * scale
    if k_lens is not None:
        lk = k.shape[1]
        s = s.masked_fill(torch.arange(lk).view(1, 1, 1, lk) >= k_lens.view(-1, 1, 1, 1), float("-inf"))
    return torch.einsum("bnlm,bmnd->blnd", torch.softmax(s, -1), v)


def _toy_pavrm_fp32_truth(step, states, noisy, timestep, ctx, label):
    """Step `step` of case_toy_pavrm from the same weights and inputs without autocast, all fp32,
    with unrounded attention: the gradients the bf16 runs approximate (fp32 rounding ~1e-7 vs
    bf16's ~4e-3).  The GPU test holds our error to this truth next to the reference's own."""
    saved = M.flash_attention
    M.flash_attention = _exact_attention
    try:
        lrm = _toy_model("t2v")
        del lrm.head
        lrm.head = None
        qa = NET.QueryAttention(256, 1, 8, 0., return_type="query")
        mlp = NET.MLP(256)
        for m, st in zip((lrm, qa, mlp), states):
            m.load_state_dict(st)
        for name in ("patch_embedding", "text_embedding", "time_embedding", "time_projection"):
            for p in getattr(lrm, name).parameters():
                p.requires_grad_(False)
        feats = DU.list2batch(lrm(x=DU.batch2list(noisy.float()), t=timestep,
                                  context=DU.batch2list(ctx.float()), seq_len=105,
                                  output_features=True, selected_layers=[2]))
        prob = NET.forward_mlp(mlp, qa(feats))
        loss = torch.nn.BCELoss()(prob.squeeze(), label.squeeze().float())
        loss.backward()
        pre = f"s{step}:t32:"
        g = {pre + k: v for k, v in grads_of(lrm).items()}
        g.update({pre + "qa." + k: v for k, v in grads_of(qa).items()})
        g.update({pre + "mlp." + k: v for k, v in grads_of(mlp).items()})
        g[pre + "prob"] = np.float64(prob.item())
        return g
    finally:
        M.flash_attention = saved


if __name__ == "__main__":
    which = sys.argv[1:] or ["ops", "toy", "real", "head", "sched", "prfl", "pavrm", "trainer", "trainer0", "split"]
    if "trainer" in which:
        case_toy_prfl_trainer()
    if "trainer0" in which:
        case_toy_prfl_trainer(mids=(0, 0), name="toy_prfl_trainer_mid0")
    if "split" in which:
        case_toy_prfl_split()
    if "pavrm" in which:
        case_toy_pavrm()
    if "ops" in which:
        case_ops()
    if "toy" in which:
        for mt in ("t2v", "i2v"):
            case_toy_model_with_grads(mt)
            case_toy_model(mt)
    if "real" in which:
        case_real_block("t2v_cross_attn")
        case_real_block("i2v_cross_attn")
    if "head" in which:
        case_reward_head()
    if "sched" in which:
        case_schedulers()
    if "prfl" in which:
        case_toy_prfl()
