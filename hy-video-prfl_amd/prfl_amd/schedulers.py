"""Flow-matching samplers used by the PRFL step (host logic; the tensors stay on the GPU).

* FlowUniPCMultistepScheduler — bh2 UniPC, order 2, x0-prediction, as configured by
  `train_prfl.py:413-415, :633` (`wan/utils/fm_solvers_unipc.py`, itself diffusers v0.31.0's UniPC
  adapted to flow matching).  The host computes the step's scalar coefficients exactly as the
  reference does (0-dim fp32 tensors, rhos cast to bf16); the element-wise body — model-output
  conversion, UniC corrector and UniP predictor — is ONE fused HIP kernel (`prfl::unipc_step`,
  csrc/unipc.hip), bit-identical to the reference's torch chain and differentiable w.r.t. the
  model output, through which the reward gradient flows (`train_prfl.py:734`).
* FlowMatchDiscreteScheduler — training-time sigma/timestep sampling, add_noise, target
  (`schedulers/scheduling_flow_match_discrete.py`).
"""
from types import SimpleNamespace

import numpy as np
import torch

from . import custom_ops


class FlowUniPCMultistepScheduler:
    order = 1

    def __init__(self, num_train_timesteps=1000, solver_order=2, prediction_type="flow_prediction",
                 shift=1.0, use_dynamic_shifting=False, predict_x0=True, solver_type="bh2",
                 lower_order_final=True, disable_corrector=(), final_sigmas_type="zero", **_):
        if prediction_type != "flow_prediction" or solver_type != "bh2" or not predict_x0:
            raise NotImplementedError("PRFL uses flow_prediction + bh2 + predict_x0")
        if use_dynamic_shifting:
            raise NotImplementedError("dynamic shifting is not used by PRFL")
        self.config = SimpleNamespace(num_train_timesteps=num_train_timesteps,
                                      solver_order=solver_order, shift=shift,
                                      lower_order_final=lower_order_final,
                                      final_sigmas_type=final_sigmas_type,
                                      use_dynamic_shifting=False)
        self.disable_corrector = list(disable_corrector)
        a = np.linspace(1, 1 / num_train_timesteps, num_train_timesteps)[::-1].copy()
        s = torch.from_numpy(1.0 - a).to(torch.float32)
        s = shift * s / (1 + (shift - 1) * s)
        self.sigmas = s
        self.timesteps = s * num_train_timesteps
        self.sigma_min, self.sigma_max = s[-1].item(), s[0].item()
        self.num_inference_steps = None
        self._reset()

    def _reset(self):
        self.model_outputs = [None] * self.config.solver_order
        self.timestep_list = [None] * self.config.solver_order
        self.lower_order_nums = 0
        self.last_sample = None
        self._step_index = None
        self._begin_index = None
        self.this_order = 1

    @property
    def step_index(self):
        return self._step_index

    def set_begin_index(self, begin_index=0):
        self._begin_index = begin_index

    def set_timesteps(self, num_inference_steps=None, device=None, sigmas=None, mu=None, shift=None):
        if sigmas is None:
            sigmas = np.linspace(self.sigma_max, self.sigma_min, num_inference_steps + 1).copy()[:-1]
        shift = self.config.shift if shift is None else shift
        sigmas = shift * sigmas / (1 + (shift - 1) * sigmas)
        timesteps = sigmas * self.config.num_train_timesteps
        self.sigmas = torch.from_numpy(np.concatenate([sigmas, [0.0]]).astype(np.float32))
        self.timesteps = torch.from_numpy(timesteps).to(device=device, dtype=torch.int64)
        self.num_inference_steps = len(timesteps)
        self._reset()

    @staticmethod
    def _lambda(sigma):
        return torch.log(1 - sigma) - torch.log(sigma)

    def _coeffs(self, sig_t, sig_s0):
        alpha_t = 1 - sig_t
        h = self._lambda(sig_t) - self._lambda(sig_s0)
        hh = -h
        return alpha_t, h, hh, torch.expm1(hh), torch.expm1(hh)   # h_phi_1, B_h (bh2)

    def _init_step_index(self, timestep):
        if self._begin_index is not None:
            self._step_index = self._begin_index
            return
        t = timestep.to(self.timesteps.device) if torch.is_tensor(timestep) else timestep
        idx = (self.timesteps == t).nonzero()
        self._step_index = idx[1 if len(idx) > 1 else 0].item()

    def _corrector_coef(self):
        """UniC-p scalars (fm_solvers_unipc.py:486-626) as the reference computes them: 0-dim
        fp32 host tensors; the solved rhos are cast to the sample dtype (bf16, :612)."""
        i, order = self._step_index, self.this_order
        sig_t, sig_s0 = self.sigmas[i], self.sigmas[i - 1]
        alpha_t, h, hh, h_phi_1, B_h = self._coeffs(sig_t, sig_s0)
        r, c1, aBh = sig_t / sig_s0, alpha_t * h_phi_1, alpha_t * B_h
        if order == 1:
            return [r, c1, 1.0, 0.0, torch.tensor(0.5, dtype=torch.bfloat16), aBh], 1
        rk = (self._lambda(self.sigmas[i - 2]) - self._lambda(sig_s0)) / h
        hpk = h_phi_1 / hh - 1
        b1 = hpk / B_h
        b2 = (hpk / hh - 0.5) * 2 / B_h
        R = torch.stack([torch.stack([torch.ones(()), torch.ones(())]),
                         torch.stack([rk, torch.ones(())])])
        rhos = torch.linalg.solve(R, torch.stack([b1, b2])).to(torch.bfloat16)
        return [r, c1, rk, rhos[0], rhos[-1], aBh], 2

    def _predictor_coef(self):
        """UniP-p scalars (fm_solvers_unipc.py:350-484)."""
        i = self._step_index
        sig_t, sig_s0 = self.sigmas[i + 1], self.sigmas[i]
        alpha_t, h, hh, h_phi_1, B_h = self._coeffs(sig_t, sig_s0)
        rk = 1.0
        if self.this_order == 2:
            rk = (self._lambda(self.sigmas[i - 1]) - self._lambda(sig_s0)) / h
        return [sig_t / sig_s0, alpha_t * h_phi_1, rk, alpha_t * B_h], self.this_order

    # the fused element-wise update (csrc/unipc.hip); tests swap in the oracle's restatement
    _update = staticmethod(custom_ops.unipc_update)

    def step(self, model_output, timestep, sample, return_dict=True, generator=None):
        if self.num_inference_steps is None:
            raise ValueError("call set_timesteps first")
        if self._step_index is None:
            self._init_step_index(timestep)
        i = self._step_index
        corr_c, corr = [0.0] * 6, 0
        if i > 0 and (i - 1) not in self.disable_corrector and self.last_sample is not None:
            corr_c, corr = self._corrector_coef()
        order = self.config.solver_order
        if self.config.lower_order_final:
            order = min(order, len(self.timesteps) - i)
        this_order = min(order, self.lower_order_nums + 1)
        self.this_order = this_order
        pred_c, pred = self._predictor_coef()
        coef = [float(c) for c in [self.sigmas[i]] + corr_c + pred_c]
        h1, h2 = self.model_outputs[-1], self.model_outputs[-2]
        m_t, sample_c, prev = self._update(model_output, sample,
                                           self.last_sample if corr else None,
                                           h1 if (corr or pred == 2) else None,
                                           h2 if corr == 2 else None, coef, corr, pred)
        self.model_outputs = self.model_outputs[1:] + [m_t]
        self.timestep_list = self.timestep_list[1:] + [timestep]
        self.last_sample = sample_c
        self.lower_order_nums = min(self.lower_order_nums + 1, self.config.solver_order)
        self._step_index += 1
        return (prev,) if not return_dict else SimpleNamespace(prev_sample=prev)


class FlowMatchDiscreteScheduler:
    order = 1

    def __init__(self, num_train_timesteps=1000, shift=1.0, sigma_max=1.0, reverse=True,
                 solver="euler"):
        self.config = SimpleNamespace(num_train_timesteps=num_train_timesteps, shift=shift,
                                      reverse=reverse, solver=solver)
        self.sigma_max = sigma_max
        s = torch.linspace(sigma_max, 0, num_train_timesteps + 1)
        self.sigmas = s if reverse else s.flip(0)
        self.timesteps = (self.sigmas[:-1] * num_train_timesteps).to(torch.float32)
        self._step_index = None

    def set_timesteps(self, num_inference_steps, device=None, dtype=torch.float32):
        self.num_inference_steps = num_inference_steps
        s = torch.linspace(self.sigma_max, 0, num_inference_steps + 1)
        s = (self.config.shift * s) / (1 + (self.config.shift - 1) * s)
        if not self.config.reverse:
            s = 1 - s
        self.sigmas = s
        self.timesteps = (s[:-1] * self.config.num_train_timesteps).to(dtype=dtype, device=device)
        self._step_index = None

    def get_train_timestep_and_sigma(self, weighting_scheme="logit_normal", batch_size=1,
                                     logit_mean=0.0, logit_std=1.0, device="cpu", generator=None,
                                     n_dim=4):
        if weighting_scheme == "logit_normal":
            u = torch.sigmoid(torch.normal(mean=logit_mean, std=logit_std, size=(batch_size,),
                                           generator=generator))
        else:
            u = torch.rand(size=(batch_size,), generator=generator)
        idx = (u * self.config.num_train_timesteps).long()
        t = self.timesteps[idx].to(device=device)
        sigma = self.sigmas[idx].to(device=device, dtype=torch.float32)
        while sigma.dim() < n_dim:
            sigma = sigma.unsqueeze(-1)
        return t, sigma

    def get_train_sigma(self, timestep, n_dim=4, device="cpu", dtype=torch.float32):
        if isinstance(timestep, float):
            timestep = torch.tensor([timestep], dtype=dtype)
        sig = self.sigmas.to(device, dtype=dtype)
        sch = self.timesteps.to(device)
        idx = [(sch == t).nonzero()[0].item() for t in timestep.to(device)]
        s = sig[idx].flatten()
        while s.dim() < n_dim:
            s = s.unsqueeze(-1)
        return s

    def add_noise(self, original_samples, noise, sigma):
        return (1 - sigma) * original_samples + sigma * noise

    def get_train_target(self, original_samples, noise):
        return noise - original_samples

    def get_train_loss_weighting(self, sigma):
        return torch.ones_like(sigma)

    def get_x0(self, model_output, sample, sigma_t):
        return sample + model_output.to(torch.float32) * (torch.zeros_like(sigma_t) - sigma_t)

    def step(self, model_output, timestep, sample, return_dict=True):
        if self._step_index is None:
            idx = (self.timesteps == timestep).nonzero()
            self._step_index = idx[1 if len(idx) > 1 else 0].item()
        sample = sample.to(torch.float32)
        dt = self.sigmas[self._step_index + 1] - self.sigmas[self._step_index]
        prev = sample + model_output.to(torch.float32) * dt
        self._step_index += 1
        return (prev,) if not return_dict else SimpleNamespace(prev_sample=prev)
