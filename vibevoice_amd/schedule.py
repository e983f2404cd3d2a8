"""Host-side DPM-Solver++ tables for the device sampler.

The reference builds DPMSolverMultistepScheduler(num_train_timesteps=1000,
beta_schedule="cosine", prediction_type="v_prediction") (modeling_vibevoice.py:
138-142) and calls set_timesteps(S) + step() per denoising step
(modeling_vibevoice_inference.py:714-724).  Every scalar of step() is a 0-dim
float32 torch tensor computed on the CPU (dpm_solver.py:295, 423), so this
module evaluates the same scalar expressions with torch float32 scalars and
hands the per-step coefficients to the HIP kernel (k_cfg_dpm), which applies
the tensor part with the reference's bf16/fp32 rounding points.

Per step s (8 floats): alpha_s, sigma_s   (x0 = alpha_s*x - sigma_s*v, :581-584)
                       c_x, c_d0, c_d1, inv_r0, order, 0
  order 1 (:669-677):  x' = c_x*x - c_d0*x0
  order 2 (:738-764):  x' = c_x*x - c_d0*x0 - c_d1*(inv_r0*(x0 - x0_prev))
"""
import math

import numpy as np
import torch

SUPPORTED_ALGORITHMS = ("dpmsolver++",)


def _cosine_alphas_cumprod(T=1000, max_beta=0.999):
    """betas_for_alpha_bar("cosine") (dpm_solver.py:28-83) and cumprod (:252-253)."""
    f = lambda t: math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2  # noqa: E731
    betas = torch.tensor([min(1 - f((i + 1) / T) / f(i / T), max_beta) for i in range(T)], dtype=torch.float32)
    return torch.cumprod(1.0 - betas, dim=0)


class Schedule:
    def __init__(self, num_train_timesteps=1000, algorithm_type="dpmsolver++"):
        if algorithm_type not in SUPPORTED_ALGORITHMS:
            raise NotImplementedError(f"algorithm_type {algorithm_type!r} (supported: {SUPPORTED_ALGORITHMS})")
        self.T = num_train_timesteps
        self.ac = _cosine_alphas_cumprod(num_train_timesteps)
        lam = torch.log(torch.sqrt(self.ac)) - torch.log(torch.sqrt(1 - self.ac))
        self.lambda_t = lam

    def timesteps_sigmas(self, steps):
        """set_timesteps, linspace spacing, final sigma 0 (dpm_solver.py:349-410)."""
        clipped = torch.searchsorted(torch.flip(self.lambda_t, [0]), -float("inf"))
        last = int((self.T - clipped).numpy().item())
        ts = np.linspace(0, last - 1, steps + 1).round()[::-1][:-1].copy().astype(np.int64)
        sig = (((1 - self.ac) / self.ac) ** 0.5).numpy()
        sig = np.interp(ts, np.arange(0, len(sig)), sig)
        sig = np.concatenate([sig, [0.0]]).astype(np.float32)
        return torch.from_numpy(ts), torch.from_numpy(sig)

    def coefficients(self, steps):
        ts, sig = self.timesteps_sigmas(steps)

        def a_s(s):
            a = 1 / ((s ** 2 + 1) ** 0.5)
            return a, s * a

        rows = []
        for i in range(steps):
            a0, s0 = a_s(sig[i])
            at, st = a_s(sig[i + 1])
            lam_t = torch.log(at) - torch.log(st)
            lam_0 = torch.log(a0) - torch.log(s0)
            h = lam_t - lam_0
            c_d0 = at * (torch.exp(-h) - 1.0)
            order = 1 if (i == 0 or i == steps - 1) else 2      # lower_order_nums / final (:978-1006)
            inv_r0 = c_d1 = torch.tensor(0.0)
            if order == 2:
                a1, s1 = a_s(sig[i - 1])
                lam_1 = torch.log(a1) - torch.log(s1)
                r0 = (lam_0 - lam_1) / h
                inv_r0 = 1.0 / r0
                c_d1 = 0.5 * c_d0
            rows.append([float(a0), float(s0), float(st / s0), float(c_d0), float(c_d1), float(inv_r0), float(order),
                         0.0])
        return ts, np.array(rows, dtype=np.float32)

    def timestep_features(self, steps, dim=256, max_period=10000):
        """TimestepEmbedder.timestep_embedding of the bf16-cast timesteps
        (modular_vibevoice_diffusion_head.py:66-88; the cast is :720)."""
        ts, _ = self.timesteps_sigmas(steps)
        t = ts.to(torch.bfloat16)
        half = dim // 2
        freqs = torch.exp(-math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half)
        args = t[:, None].float() * freqs[None]
        return torch.cat([torch.cos(args), torch.sin(args)], dim=-1).to(torch.bfloat16)
