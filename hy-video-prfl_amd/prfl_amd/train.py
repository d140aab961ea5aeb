"""PRFL / PAVRM training steps on the MI355X path.

Restates the per-iteration logic of the reference drivers (which cannot travel to the GPU box):
  * ``sft_step``     — `scripts/prfl/train_prfl.py:900-1034` (flow-matching SFT loss)
  * ``reward_step``  — `scripts/prfl/train_prfl.py:585-898`  (no-grad UniPC rollout to a random
                       mid timestep, one grad-enabled generator step, one differentiable UniPC
                       step, frozen latent reward model + QueryAttention + MLP, hinge loss)
  * ``pavrm_step``   — `scripts/pavrm/train_pavrm.py:671-920` (BCE reward-model training)
  * ``build_lrm``    — `train_prfl.py:217-266` (first `trainable_blocks` of a Wan model, no head)
Optimizer semantics kept: loss / gradient_accumulation_steps, clip_grad_norm_(1.0) on the
accumulated grads every micro-step, optimizer.step() when (step+1) % accum == 0 in BOTH steps
(the reward step's gradient accumulates onto the SFT step's: no zero_grad between them).
Failure handling kept (`train_prfl.py:800-811`, `train_pavrm.py:874-880`): a NaN / Inf loss skips
the backward and the optimizer step and reports loss 0 / grad_norm 0; |loss| > 1e6 is clamped
(zero gradient).  Under data parallelism the skip is agreed across ranks (one MAX all-reduce of
the flag): a rank that skipped alone would leave the others waiting in the gradient all-reduce.
"""
import random

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import block as _block
from .dist import GradReducer, all_reduce_max, all_reduce_mean, broadcast_int, is_dist
from .network import forward_mlp
from .optim import AdamW, clip_grad_norm_
from .schedulers import FlowMatchDiscreteScheduler, FlowUniPCMultistepScheduler


def batch2list(batch):
    return [item for item in batch]


def list2batch(lst):
    return torch.stack(lst)


def build_lrm(model, trainable_blocks=range(8)):
    """Latent reward model trunk: keep blocks[trainable_blocks], drop the head, freeze all
    (the reference leaves requires_grad=True on the kept blocks but never optimises them)."""
    keep = set(trainable_blocks)
    model.blocks = nn.ModuleList([b for i, b in enumerate(model.blocks) if i in keep])
    if hasattr(model, "head"):
        del model.head
        model.head = None
    for p in model.parameters():
        p.requires_grad_(False)
    return model


def store_frozen_bf16(model):
    """Keep a frozen model's block Linear weights in bf16 (a memory plan step, §f-1): the fused
    block casts every Linear weight to bf16 before its GEMM anyway (autocast, `model.py`), and a
    bf16 copy made once holds exactly those bits, so outputs are bit-identical while the PRFL
    reward model's 8-block trunk takes 5.6 GB instead of 11.2 at 14B width.  Norm weights,
    biases and modulation stay fp32 (the kernels read them in fp32).  Refuses trainable weights,
    and blocks on config C5's fp8 path: there the e4m3 codes and per-row scales are quantised from
    the fp32 master every pass (block.BF16Weights), and quantising from a bf16 copy instead would
    change the amax and round twice — the C5 trunk stays fp32.  Swaps `p.data` in
    place on the caller's model (PRFLTrainer(lrm_weights_bf16=False) leaves it alone)."""
    for blk in model.blocks:
        if getattr(blk, "fp8_gemm", 0):
            raise ValueError("store_frozen_bf16: fp8 blocks quantise from the fp32 master")
        for name, p in blk.named_parameters():
            if p.dim() == 2 and name.endswith(".weight"):
                if p.requires_grad:
                    raise ValueError(f"store_frozen_bf16: {name} is trainable")
                p.data = p.data.to(torch.bfloat16)
    return model


def guard_loss(loss):
    """`train_prfl.py:800-811` / `train_pavrm.py:874-880`: None for a NaN / Inf loss (the caller
    skips backward and optimizer step), the loss clamped to [-1e6, 1e6] when |loss| > 1e6 (whose
    gradient is then zero, as torch.clamp's), else the loss unchanged.  One host read of the
    flags, as the reference's `loss.item()`; the NaN flag is the MAX over data-parallel ranks."""
    d = loss.detach().float()
    bad, big = (bool(v) for v in torch.stack([~torch.isfinite(d), d.abs() > 1e6]).tolist())
    if is_dist():
        bad = bool(all_reduce_max(torch.tensor([float(bad)], device=d.device)).item())
    if bad:
        return None
    if big:                                  # the clamp itself stays per rank, as the reference's
        return torch.clamp(loss, -1e6, 1e6)
    return loss


class PRFLTrainer:
    def __init__(self, transformer, lrm, query_attention, mlp, lr=5e-6, weight_decay=0.01,
                 grad_accum=5.0, flow_shift=5.0, inference_steps=40, feature_layer=(8,),
                 max_grad_norm=1.0, optimizer_state_on_host=False, optimizer_shard=False,
                 optimizer_overlap=True, lrm_weights_bf16=True):
        self.transformer, self.lrm, self.qa, self.mlp = transformer, lrm, query_attention, mlp
        if (lrm_weights_bf16 and not any(p.requires_grad for p in lrm.parameters())
                and not any(getattr(b, "fp8_gemm", 0) for b in lrm.blocks)):
            store_frozen_bf16(lrm)            # frozen bf16 reward trunk: bit-identical, half the bytes
        params = [p for p in transformer.parameters() if p.requires_grad]
        self.params = params
        self.optimizer = AdamW(params, lr=lr, weight_decay=weight_decay,
                               state_on_host=optimizer_state_on_host, shard=optimizer_shard,
                               overlap=optimizer_overlap)
        if optimizer_overlap:
            # each block's forward waits for its own parameters' update (optim.py): the SFT
            # step's optimizer update streams under the reward step's rollout
            self.optimizer.attach(transformer)
        self.optimizer.init_state()          # after attach: a host-moment fraction is a tail in update order
        self.reducer = GradReducer(params)
        self.grad_accum = grad_accum
        self.inference_steps = inference_steps
        self.feature_layer = list(feature_layer)
        self.max_grad_norm = max_grad_norm
        self.flow_shift = flow_shift
        self.fm = FlowMatchDiscreteScheduler(shift=flow_shift)
        self.fm.set_timesteps(1000, dtype=torch.int64)
        self.unipc = FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1,
                                                 use_dynamic_shifting=False)

    def _guard(self, loss):
        return guard_loss(loss)

    def _backward_and_step(self, loss, step):
        self.reducer.begin()
        loss.backward()
        self.reducer.end()
        grad_norm = clip_grad_norm_(self.params, self.max_grad_norm)
        if (step + 1) % self.grad_accum == 0:
            self.optimizer.step(zero_grad=True)       # step + zero_grad (buffers kept)
        return grad_norm

    def _kw(self, latent, text_states, seq_len, image_embeds, cond):
        return dict(context=batch2list(text_states), seq_len=seq_len, clip_fea=image_embeds,
                    y=batch2list(cond) if cond is not None else None)

    def sft_step(self, step, latents, text_states, seq_len, image_embeds=None, cond=None,
                 generator=None, noise=None, timestep=None):
        """train_prfl.py:900-980.  `noise` / `timestep` (a value of the 1000-step schedule's
        `timesteps`) replace the random draws when given."""
        _block.reset_attn_stash()
        bsz = latents.shape[0]
        if noise is None:
            noise = torch.randn(latents.shape, generator=generator, dtype=latents.dtype,
                                device=latents.device)
        if timestep is None:
            timestep, sigma = self.fm.get_train_timestep_and_sigma(
                weighting_scheme="uniform", batch_size=bsz, device=latents.device,
                n_dim=latents.ndim)
        else:
            sigma = self.fm.get_train_sigma(timestep, n_dim=latents.ndim, device=latents.device)
        noisy = self.fm.add_noise(latents, noise, sigma)
        pred = list2batch(self.transformer(x=batch2list(noisy), t=timestep,
                                           **self._kw(noisy, text_states, seq_len, image_embeds,
                                                      cond)))
        target = self.fm.get_train_target(latents, noise)
        loss = torch.mean((pred.float() - target.float()) ** 2) / self.grad_accum
        grad_norm = self._backward_and_step(loss, step)
        return dict(loss=all_reduce_mean(loss.detach()), grad_norm=grad_norm)

    def reward_step(self, step, latents, text_states, seq_len, image_embeds=None, cond=None,
                    mid_timestep=None, generator=None, noise=None):
        """train_prfl.py:585-846.  `noise` replaces the initial latent's random draw
        (`randn_like(latents)`, `:637`) when given."""
        _block.reset_attn_stash()
        sch = self.unipc
        sch.set_timesteps(num_inference_steps=self.inference_steps, device=latents.device,
                          shift=self.flow_shift)
        timesteps = sch.timesteps
        if noise is None:
            latent = torch.randn(latents.shape, generator=generator, dtype=latents.dtype,
                                 device=latents.device)
        else:
            latent = noise.to(latents.dtype)
        if mid_timestep is None:
            mid_timestep = random.randint(0, self.inference_steps - 2)
        mid = broadcast_int(mid_timestep, device=latents.device)
        kw = self._kw(latent, text_states, seq_len, image_embeds, cond)
        dev = latents.device
        with torch.no_grad():                                          # :665-699
            for i in range(mid):
                t = timesteps[i]
                pred = list2batch(self.transformer(x=batch2list(latent), t=t.reshape(1),
                                                   **kw))
                latent = sch.step(pred, t, latent, return_dict=False)[0]
        t_mid = timesteps[mid]                                         # :708-735
        pred = list2batch(self.transformer(x=batch2list(latent), t=t_mid.reshape(1),
                                           **kw))
        latent = sch.step(pred, t_mid, latent, return_dict=False)[0]
        t1 = timesteps[mid + 1]                                        # :745-798
        feats = list2batch(self.lrm(x=batch2list(latent), t=t1.reshape(1),
                                    output_features=True, selected_layers=self.feature_layer,
                                    **kw))
        reward = forward_mlp(self.mlp, self.qa(feats))
        loss = 0.1 * F.relu(-reward.squeeze() + 2).mean()
        loss = self._guard(loss)                                       # :800-811
        if loss is None:
            return dict(loss=torch.tensor(0.0), grad_norm=0, mid=mid, reward=reward.detach(),
                        skipped=True)
        loss = loss / self.grad_accum
        grad_norm = self._backward_and_step(loss, step)
        return dict(loss=all_reduce_mean(loss.detach().float()), grad_norm=grad_norm, mid=mid,
                    reward=reward.detach())


class PAVRMTrainer:
    """train_pavrm.py:671-920 with loss 'ce': BCE(sigmoid(MLP(QA(features))), label).

    Optimizer = `optimizer_init` (`train_pavrm.py:459-506`): the transformer's trainable blocks at
    `lr`; the MLP and QueryAttention at `lr_head` = `learning_rate_mlp` when the config sets it,
    else `lr` (the CE configs leave it commented out, `train_pavrm_t2v_480.yaml:61-62`).  One
    AdamW over the three groups is the same update as one AdamW per group (AdamW is per
    parameter).  Clipping = `transformer.clip_grad_norm_(1.0)` after backward (`:899`) over the
    transformer grads only; the pre-backward clip of `:883-889` runs on parameters whose grads
    were cleared by the previous `zero_grad`, so it clips nothing and is not restated."""

    def __init__(self, lrm, query_attention, mlp, lr=1e-6, lr_head=None, weight_decay=0.01,
                 flow_shift=5.0, feature_layer=(8,), max_grad_norm=1.0):
        self.lrm, self.qa, self.mlp = lrm, query_attention, mlp
        for p in lrm.parameters():
            p.requires_grad_(False)
        for blk in lrm.blocks:                       # trainable blocks (train_pavrm.py:215-235)
            for p in blk.parameters():
                p.requires_grad_(True)
        for m in (query_attention, mlp):
            for p in m.parameters():
                p.requires_grad_(True)
        self.trunk_params = [p for p in lrm.parameters() if p.requires_grad]
        self.head_params = list(mlp.parameters()) + list(query_attention.parameters())
        lr_head = lr if lr_head is None else lr_head
        self.opt_trunk = AdamW(self.trunk_params, lr=lr, weight_decay=weight_decay)
        self.opt_head = AdamW(self.head_params, lr=lr_head, weight_decay=weight_decay)
        self.reducer = GradReducer(self.trunk_params + self.head_params)
        self.fm = FlowMatchDiscreteScheduler(shift=flow_shift)
        self.fm.set_timesteps(1000, dtype=torch.int64)
        self.feature_layer = list(feature_layer)
        self.max_grad_norm = max_grad_norm

    def step(self, latents, text_states, seq_len, label, image_embeds=None, cond=None,
             generator=None, noise=None, timestep=None):
        """One PAVRM step; `noise` / `timestep` (values of the 1000-step schedule's `timesteps`,
        as `train_pavrm.py:721-728` passes them) replace the random draws when given."""
        _block.reset_attn_stash()
        bsz = latents.shape[0]
        if noise is None:
            noise = torch.randn(latents.shape, generator=generator, dtype=latents.dtype,
                                device=latents.device)
        if timestep is None:
            timestep, sigma = self.fm.get_train_timestep_and_sigma(
                weighting_scheme="uniform", batch_size=bsz, device=latents.device,
                n_dim=latents.ndim)
        else:
            sigma = self.fm.get_train_sigma(timestep, n_dim=latents.ndim, device=latents.device)
        noisy = self.fm.add_noise(latents, noise, sigma)
        feats = list2batch(self.lrm(x=batch2list(noisy), t=timestep, context=batch2list(text_states),
                                    seq_len=seq_len, clip_fea=image_embeds,
                                    y=batch2list(cond) if cond is not None else None,
                                    output_features=True, selected_layers=self.feature_layer))
        out = forward_mlp(self.mlp, self.qa(feats))
        loss = F.binary_cross_entropy(out.squeeze().float(), label.squeeze().float())
        loss = guard_loss(loss)                                        # train_pavrm.py:874-880
        if loss is None:
            return dict(loss=torch.tensor(0.0), grad_norm=0, prob=out.detach(), skipped=True)
        self.reducer.begin()
        loss.backward()
        self.reducer.end()
        grad_norm = clip_grad_norm_(self.trunk_params, self.max_grad_norm)
        self.opt_trunk.step(zero_grad=True)
        self.opt_head.step(zero_grad=True)
        return dict(loss=all_reduce_mean(loss.detach()), grad_norm=grad_norm, prob=out.detach())
