"""A small engine whose workspaces the kernel-level GPU tests borrow."""
from tiny import tiny_config
from vibevoice_amd.engine import Engine
from vibevoice_amd.weights import synthetic_state_dict

_ENG = None


def tiny_engine():
    global _ENG
    if _ENG is None:
        cfg = tiny_config()
        sd = synthetic_state_dict(cfg, seed=0, device="cpu", mode="test", with_acoustic_encoder=False)
        _ENG = Engine(cfg, sd, "cuda", max_batch=2, max_ctx=64)
    return _ENG
