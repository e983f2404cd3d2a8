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
                       c_x, c_d0, c_d1, inv_r0, order, c_n
  order 1 (:669-686):  x' = c_x*x - c_d0*x0                                 [+ c_n*noise]
  order 2 (:738-793):  x' = c_x*x - c_d0*x0 - c_d1*(inv_r0*(x0 - x0_prev))  [+ c_n*noise]
algorithm_type "dpmsolver++" (the model's, modeling_vibevoice.py:138-142) or
"sde-dpmsolver++" (gradio_demo.py:114-118, swapped in through
model.model.noise_scheduler = ....from_config(config, algorithm_type=...)): the
SDE variant adds c_n * noise with fp32 noise drawn per step on the device
generator (step(), :985-987); c_n = 0 for the ODE solver.
"""
import math

import numpy as np
import torch

SUPPORTED_ALGORITHMS = ("dpmsolver++", "sde-dpmsolver++")
# beta schedules with the same betas (dpm_solver.py:239-241)
SUPPORTED_BETAS = ("cosine", "squaredcos_cap_v2")


def _cosine_alphas_cumprod(T=1000, max_beta=0.999):
    """betas_for_alpha_bar("cosine") (dpm_solver.py:28-83) and cumprod (:252-253)."""
    f = lambda t: math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2  # noqa: E731
    betas = torch.tensor([min(1 - f((i + 1) / T) / f(i / T), max_beta) for i in range(T)], dtype=torch.float32)
    return torch.cumprod(1.0 - betas, dim=0)


class _Config(dict):
    """The scheduler's `config` (diffusers FrozenDict-like: keys and attributes)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None


class Schedule:
    """The model's DPMSolverMultistepScheduler as far as the loop uses it
    (model.model.noise_scheduler).  Only the configurations the reference's
    callers build are accepted; anything else raises."""

    def __init__(self, num_train_timesteps=1000, algorithm_type="dpmsolver++", beta_schedule="cosine",
                 prediction_type="v_prediction", solver_order=2, solver_type="midpoint", lower_order_final=True,
                 final_sigmas_type="zero", **unused):
        if algorithm_type not in SUPPORTED_ALGORITHMS:
            raise NotImplementedError(f"algorithm_type {algorithm_type!r} (supported: {SUPPORTED_ALGORITHMS})")
        if beta_schedule not in SUPPORTED_BETAS:
            raise NotImplementedError(f"beta_schedule {beta_schedule!r} (supported: {SUPPORTED_BETAS})")
        if (prediction_type, solver_order, solver_type, lower_order_final, final_sigmas_type) != \
                ("v_prediction", 2, "midpoint", True, "zero"):
            raise NotImplementedError("only the model's solver configuration (v_prediction, order 2, midpoint, "
                                      "lower_order_final, final sigma 0) is implemented")
        self.algorithm_type = algorithm_type
        self.config = _Config(num_train_timesteps=num_train_timesteps, algorithm_type=algorithm_type,
                              beta_schedule=beta_schedule, prediction_type=prediction_type, solver_order=solver_order,
                              solver_type=solver_type, lower_order_final=lower_order_final,
                              final_sigmas_type=final_sigmas_type)
        self.T = num_train_timesteps
        self.ac = _cosine_alphas_cumprod(num_train_timesteps)
        lam = torch.log(torch.sqrt(self.ac)) - torch.log(torch.sqrt(1 - self.ac))
        self.lambda_t = lam

    @classmethod
    def from_config(cls, config, **overrides):
        """ConfigMixin.from_config: the config's arguments with `overrides` on top."""
        return cls(**{**dict(config), **overrides})

    @property
    def sde(self):
        return self.algorithm_type == "sde-dpmsolver++"

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
            if self.sde:     # :680-686 / :785-793, scalar expressions in the reference's order
                c_x = st / s0 * torch.exp(-h)
                c_d0 = -(at * (1 - torch.exp(-2.0 * h)))
                c_n = st * torch.sqrt(1.0 - torch.exp(-2 * h))
            else:
                c_x = st / s0
                c_d0 = at * (torch.exp(-h) - 1.0)
                c_n = torch.tensor(0.0)
            order = 1 if (i == 0 or i == steps - 1) else 2      # lower_order_nums / final (:978-1006)
            inv_r0 = c_d1 = torch.tensor(0.0)
            if order == 2:
                a1, s1 = a_s(sig[i - 1])
                lam_1 = torch.log(a1) - torch.log(s1)
                r0 = (lam_0 - lam_1) / h
                inv_r0 = 1.0 / r0
                c_d1 = -(0.5 * (at * (1 - torch.exp(-2.0 * h)))) if self.sde else 0.5 * c_d0
            rows.append([float(a0), float(s0), float(c_x), float(c_d0), float(c_d1), float(inv_r0), float(order),
                         float(c_n)])
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
