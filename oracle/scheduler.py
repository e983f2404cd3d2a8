"""DPM-Solver++ (multistep, order 2, midpoint, v-prediction, final sigma 0).

Restates vibevoice/schedule/dpm_solver.py as constructed at
vibevoice/modular/modeling_vibevoice.py:138-142
(num_train_timesteps=1000, beta_schedule="cosine", prediction_type="v_prediction",
all other arguments at their defaults, dpm_solver.py:203-227).
"""
import math

import numpy as np
import torch


def cosine_alphas_cumprod(num_train_timesteps=1000, max_beta=0.999):
    """betas_for_alpha_bar(cosine) (dpm_solver.py:28-83) -> cumprod(1-beta) (:252-253)."""
    def abar(t):
        return math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2
    betas = [min(1 - abar((i + 1) / num_train_timesteps) / abar(i / num_train_timesteps), max_beta)
             for i in range(num_train_timesteps)]
    betas = torch.tensor(betas, dtype=torch.float32)
    return torch.cumprod(1.0 - betas, dim=0)


class DPMSolverPP:
    """Stateful restatement of DPMSolverMultistepScheduler for this config.

    algorithm_type "dpmsolver++" (the model's, modeling_vibevoice.py:138-142) or
    "sde-dpmsolver++" (gradio_demo.py:114-118; "squaredcos_cap_v2" is the same
    cosine betas, dpm_solver.py:239-241).  The SDE variant takes the step's
    fp32 noise explicitly (step()'s variance_noise, :985-989)."""

    def __init__(self, num_train_timesteps=1000, algorithm_type="dpmsolver++"):
        if algorithm_type not in ("dpmsolver++", "sde-dpmsolver++"):
            raise NotImplementedError(algorithm_type)
        self.algorithm_type = algorithm_type
        self.T = num_train_timesteps
        self.alphas_cumprod = cosine_alphas_cumprod(num_train_timesteps)
        ac = self.alphas_cumprod
        alpha_t, sigma_t = torch.sqrt(ac), torch.sqrt(1 - ac)
        self.lambda_t = torch.log(alpha_t) - torch.log(sigma_t)         # :263

    def set_timesteps(self, num_inference_steps):
        """dpm_solver.py:321-423 with timestep_spacing="linspace", no karras/lu."""
        clipped = torch.searchsorted(torch.flip(self.lambda_t, [0]), -float("inf"))
        last = int((self.T - clipped).numpy().item())                   # :354-355
        ts = (np.linspace(0, last - 1, num_inference_steps + 1)
              .round()[::-1][:-1].copy().astype(np.int64))              # :359-364
        sig = (((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5).numpy()
        sig = np.interp(ts, np.arange(0, len(sig)), sig)                 # :397
        self.sigmas = torch.from_numpy(np.concatenate([sig, [0.0]]).astype(np.float32))  # :401-410
        self.timesteps = torch.from_numpy(ts)
        self.model_outputs = [None, None]                                # :415-418
        self.lower_order_nums = 0
        self.step_index = 0                                              # :923-933 (unique ts)

    @staticmethod
    def _alpha_sigma(sigma):
        a = 1 / ((sigma ** 2 + 1) ** 0.5)                                # :483-487
        return a, sigma * a

    def step(self, v, sample, noise=None):
        """step() dpm_solver.py:935-1022; `v` and `sample` share a dtype.

        The dtype flow is the reference's: x0 = alpha*sample - sigma*v runs in
        the sample dtype (:581-584); the update upcasts `sample` to fp32 (:993)
        but every coefficient x (bf16 tensor) product stays bf16 (0-dim fp32
        tensors do not promote); the result is cast back (:1014).
        """
        i, S = self.step_index, len(self.timesteps)
        lower_final = i == S - 1                                         # :978-982 (sigmas zero)
        a_s, s_s = self._alpha_sigma(self.sigmas[i])
        x0 = a_s * sample - s_s * v                                      # :581-584
        self.model_outputs = [self.model_outputs[1], x0]
        x = sample.to(torch.float32)
        sig_t, sig_s0 = self.sigmas[i + 1], self.sigmas[i]
        a_t, s_t = self._alpha_sigma(sig_t)
        a_0, s_0 = self._alpha_sigma(sig_s0)
        lam_t = torch.log(a_t) - torch.log(s_t)
        lam_0 = torch.log(a_0) - torch.log(s_0)
        h = lam_t - lam_0
        sde = self.algorithm_type == "sde-dpmsolver++"
        if sde:
            assert noise is not None
            noise = noise.to(torch.float32)
        if self.lower_order_nums < 1 or lower_final:                     # :1003-1004, :669-677
            if sde:                                                      # :680-686
                out = ((s_t / s_0 * torch.exp(-h)) * x + (a_t * (1 - torch.exp(-2.0 * h))) * x0
                       + s_t * torch.sqrt(1.0 - torch.exp(-2 * h)) * noise)
            else:
                out = (s_t / s_0) * x - (a_t * (torch.exp(-h) - 1.0)) * x0
        else:                                                            # :738-764
            a_1, s_1 = self._alpha_sigma(self.sigmas[i - 1])
            lam_1 = torch.log(a_1) - torch.log(s_1)
            r0 = (lam_0 - lam_1) / h
            m0, m1 = self.model_outputs[1], self.model_outputs[0]
            d1 = (1.0 / r0) * (m0 - m1)
            if sde:                                                      # :785-793 (midpoint)
                out = ((s_t / s_0 * torch.exp(-h)) * x + (a_t * (1 - torch.exp(-2.0 * h))) * m0
                       + 0.5 * (a_t * (1 - torch.exp(-2.0 * h))) * d1
                       + s_t * torch.sqrt(1.0 - torch.exp(-2 * h)) * noise)
            else:
                out = ((s_t / s_0) * x - (a_t * (torch.exp(-h) - 1.0)) * m0
                       - 0.5 * (a_t * (torch.exp(-h) - 1.0)) * d1)
        if self.lower_order_nums < 2:
            self.lower_order_nums += 1
        self.step_index += 1
        return out.to(v.dtype)
