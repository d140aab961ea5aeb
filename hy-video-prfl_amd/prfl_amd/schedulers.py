"""Flow-matching samplers used by the PRFL step (host logic; the tensors stay on the GPU).

* FlowUniPCMultistepScheduler — bh2 UniPC, order 2, x0-prediction, as configured by
  `train_prfl.py:413-415, :633` (`wan/utils/fm_solvers_unipc.py`, itself diffusers v0.31.0's UniPC
  adapted to flow matching).  The reward gradient flows through one `step` (`train_prfl.py:734`),
  so every update here is plain differentiable tensor arithmetic with the reference's dtype
  behaviour: the sample stays in its own dtype (bf16 in PRFL) and scalar coefficients are 0-dim
  fp32 tensors, so `sigma_t/sigma_s0 * x` is rounded to bf16 exactly as in the reference.
* FlowMatchDiscreteScheduler — training-time sigma/timestep sampling, add_noise, target
  (`schedulers/scheduling_flow_match_discrete.py`).
"""
from types import SimpleNamespace

import numpy as np
import torch


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

    def _corrector(self, m_t, x_t):
        """UniC-p (fm_solvers_unipc.py:486-626)."""
        i, order = self._step_index, self.this_order
        m0, x = self.model_outputs[-1], self.last_sample
        sig_t, sig_s0 = self.sigmas[i], self.sigmas[i - 1]
        alpha_t, h, hh, h_phi_1, B_h = self._coeffs(sig_t, sig_s0)
        x_t_ = sig_t / sig_s0 * x - alpha_t * h_phi_1 * m0
        if order == 1:
            rho_last = torch.tensor(0.5, dtype=x.dtype)
            corr = 0
        else:
            rk = (self._lambda(self.sigmas[i - 2]) - self._lambda(sig_s0)) / h
            D1 = (self.model_outputs[-2] - m0) / rk
            hpk = h_phi_1 / hh - 1
            b1 = hpk / B_h
            b2 = (hpk / hh - 0.5) * 2 / B_h
            R = torch.stack([torch.stack([torch.ones(()), torch.ones(())]),
                             torch.stack([rk, torch.ones(())])])
            rhos = torch.linalg.solve(R, torch.stack([b1, b2])).to(x.dtype)
            corr = rhos[0] * D1
            rho_last = rhos[-1]
        return (x_t_ - alpha_t * B_h * (corr + rho_last * (m_t - m0))).to(x.dtype)

    def _predictor(self, x):
        """UniP-p (fm_solvers_unipc.py:350-484)."""
        i, m0 = self._step_index, self.model_outputs[-1]
        sig_t, sig_s0 = self.sigmas[i + 1], self.sigmas[i]
        alpha_t, h, hh, h_phi_1, B_h = self._coeffs(sig_t, sig_s0)
        x_t_ = sig_t / sig_s0 * x - alpha_t * h_phi_1 * m0
        if self.this_order == 2:
            rk = (self._lambda(self.sigmas[i - 1]) - self._lambda(sig_s0)) / h
            D1 = (self.model_outputs[-2] - m0) / rk
            x_t_ = x_t_ - alpha_t * B_h * (torch.tensor(0.5, dtype=x.dtype) * D1)
        return x_t_.to(x.dtype)

    def step(self, model_output, timestep, sample, return_dict=True, generator=None):
        if self.num_inference_steps is None:
            raise ValueError("call set_timesteps first")
        if self._step_index is None:
            self._init_step_index(timestep)
        # sigmas stay on the host as 0-dim fp32 scalars (as in the reference): scalar x device
        # tensor keeps the sample dtype and needs no host<->device traffic
        i = self._step_index
        m_t = sample - self.sigmas[i] * model_output                # convert_model_output (:321)
        if i > 0 and (i - 1) not in self.disable_corrector and self.last_sample is not None:
            sample = self._corrector(m_t, sample)
        self.model_outputs = self.model_outputs[1:] + [m_t]
        self.timestep_list = self.timestep_list[1:] + [timestep]
        order = self.config.solver_order
        if self.config.lower_order_final:
            order = min(order, len(self.timesteps) - i)
        self.this_order = min(order, self.lower_order_nums + 1)
        self.last_sample = sample
        prev = self._predictor(sample)
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
