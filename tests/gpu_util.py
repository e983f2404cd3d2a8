"""Helpers for the GPU parity tests (run on the MI355X box)."""
import torch


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    assert a.numel() == b.numel(), (a.shape, b.shape)   # no silent broadcasting
    a = a.reshape(b.shape)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def max_rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def cos(a, b):
    a, b = a.float().cpu().reshape(-1), b.float().cpu().reshape(-1)
    return torch.nn.functional.cosine_similarity(a, b, dim=0).item()
