"""Diffusion head + CFG sampling loop (oracle).

Restates vibevoice/modular/modular_vibevoice_diffusion_head.py and
VibeVoiceForConditionalGenerationInference.sample_speech_tokens
(vibevoice/modular/modeling_vibevoice_inference.py:712-725).
`sd` is the head's state dict (keys relative to `model.prediction_head.`).
"""
import math

import torch
import torch.nn.functional as F

from .scheduler import DPMSolverPP


def rms_norm(x, eps, weight=None):
    """RMSNorm (modular_vibevoice_diffusion_head.py:31-38): fp32 normalise,
    cast back, then multiply by the weight in the input dtype."""
    y = x.float()
    y = (y * torch.rsqrt(y.pow(2).mean(-1, keepdim=True) + eps)).type_as(x)
    return y * weight if weight is not None else y


def timestep_freq(t, dim=256, max_period=10000):
    """TimestepEmbedder.timestep_embedding (:66-88): cos||sin, cast to t.dtype."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(0, half, dtype=torch.float32, device=t.device) / half)
    args = t[:, None].float() * freqs[None]
    return torch.cat([torch.cos(args), torch.sin(args)], dim=-1).to(t.dtype)


def head_forward(sd, noisy, t, cond, n_layers, eps=1e-5):
    """VibeVoiceDiffusionHead.forward (:254-280)."""
    x = F.linear(noisy, sd["noisy_images_proj.weight"])
    tf = timestep_freq(t)
    temb = F.linear(F.silu(F.linear(tf, sd["t_embedder.mlp.0.weight"])), sd["t_embedder.mlp.2.weight"])
    c = F.linear(cond, sd["cond_proj.weight"]) + temb
    sc = F.silu(c)
    for i in range(n_layers):                                           # HeadLayer.forward :158-161
        p = f"layers.{i}."
        shift, scale, gate = F.linear(sc, sd[p + "adaLN_modulation.1.weight"]).chunk(3, dim=-1)
        h = rms_norm(x, eps, sd[p + "norm.weight"]) * (1 + scale) + shift
        h = F.linear(F.silu(F.linear(h, sd[p + "ffn.gate_proj.weight"])) * F.linear(h, sd[p + "ffn.up_proj.weight"]),
                     sd[p + "ffn.down_proj.weight"])                     # FeedForwardNetwork :116-123
        x = x + gate * h
    shift, scale = F.linear(sc, sd["final_layer.adaLN_modulation.1.weight"]).chunk(2, dim=-1)
    x = rms_norm(x, eps) * (1 + scale) + shift                            # FinalLayer :184-188
    return F.linear(x, sd["final_layer.linear.weight"])


def sample_speech_tokens(sd, cond, neg_cond, noise, steps, cfg_scale, n_layers, eps=1e-5,
                         return_trace=False, sde_noise=None):
    """sample_speech_tokens (:712-725).

    `noise` is the [2n, latent] draw the reference makes with the CPU generator
    (:716, torch.randn(...).to(condition)); pass it already in the model dtype.
    Only rows [:n] influence the result; all 2n rows are stepped as in the
    reference so the trace matches.
    """
    # sde_noise: [steps, 2n, latent] fp32, the per-step draws step() makes for
    # sde-dpmsolver++ (dpm_solver.py:985-987)
    sched = DPMSolverPP(algorithm_type="sde-dpmsolver++" if sde_noise is not None else "dpmsolver++")
    sched.set_timesteps(steps)
    condition = torch.cat([cond, neg_cond], dim=0)
    speech = noise.clone()
    n = cond.shape[0]
    trace = []
    for si, t in enumerate(sched.timesteps):
        half = speech[:n]
        combined = torch.cat([half, half], dim=0)
        eps_ = head_forward(sd, combined, t.repeat(2 * n).to(device=combined.device, dtype=combined.dtype), condition, n_layers, eps)
        c_eps, u_eps = torch.split(eps_, n, dim=0)
        half_eps = u_eps + cfg_scale * (c_eps - u_eps)
        speech = sched.step(torch.cat([half_eps, half_eps], dim=0), speech,
                            None if sde_noise is None else sde_noise[si])
        if return_trace:
            trace.append(speech[:n].clone())
    return (speech[:n], trace) if return_trace else speech[:n]
