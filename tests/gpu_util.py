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


def kv_synthetic(eng, slots, p0, p1, seed=0):
    """Diagnostic (vibevoice_hip_diag.h vv_kv_synthetic): deterministic
    pseudo-random K/V at positions [p0, p1) of `slots` of engine `eng`."""
    import ctypes
    from vibevoice_amd import _lib
    s = torch.cuda.current_stream()
    _lib.check(_lib.lib().vv_kv_synthetic(eng.h, slots.shape[0], ctypes.c_void_p(slots.data_ptr()), int(p0), int(p1),
                                          int(seed) & 0xffffffff, ctypes.c_void_p(s.cuda_stream)), "kv_synthetic")
