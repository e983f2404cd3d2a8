"""Golden-vector harness: imports the READ-ONLY reference at /root/reference.

Test infrastructure only, and only in the build container (the reference does
not exist on the GPU box).  Nothing in the product, the GPU tests, smoke() or
bench.py imports this module; its only job is to run the reference's own
sub-modules so `make_golden.py` can write small .npz fixtures.

The container's package set differs from the reference's pins
(transformers 5.15 vs 4.51.3, no diffusers), so four harness-side shims are
installed before import:
  1. a stub `diffusers` exposing ConfigMixin / register_to_config /
     SchedulerMixin / SchedulerOutput / deprecate / randn_tensor
     (config plumbing only; the scheduler arithmetic is the reference's own);
  2. `_LazyAutoMapping.register(..., exist_ok=True)` (5.15 ships classes whose
     names collide with the reference's AutoModel.register calls);
  3. alias `transformers.models.qwen2.tokenization_qwen2_fast`;
  4. `tie_weights(*a, **k)` tolerance for 5.15's post_init signature.
"""
import inspect
import sys
import types
from dataclasses import dataclass

import torch

REF = "/root/reference"


def _install_diffusers_stub():
    if "diffusers" in sys.modules:
        return
    d = types.ModuleType("diffusers")
    cu = types.ModuleType("diffusers.configuration_utils")
    ut = types.ModuleType("diffusers.utils")
    tu = types.ModuleType("diffusers.utils.torch_utils")
    sc = types.ModuleType("diffusers.schedulers")
    su = types.ModuleType("diffusers.schedulers.scheduling_utils")

    class _Cfg(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

    class ConfigMixin:
        def register_to_config(self, **kw):
            if not hasattr(self, "config"):
                self.config = _Cfg()
            self.config.update(kw)

    def register_to_config(init):
        sig = inspect.signature(init)

        def wrapped(self, *args, **kwargs):
            bound = sig.bind(self, *args, **kwargs)
            bound.apply_defaults()
            cfg = _Cfg({k: v for k, v in bound.arguments.items() if k != "self"})
            self.config = cfg
            init(self, *args, **kwargs)
        return wrapped

    class SchedulerMixin:
        pass

    @dataclass
    class SchedulerOutput:
        prev_sample: torch.Tensor

    class KarrasDiffusionSchedulers:
        def __iter__(self):
            return iter(())
    KarrasDiffusionSchedulers = []  # iterable of enum-like members (empty)

    def deprecate(*a, **k):
        return None

    def randn_tensor(shape, generator=None, device=None, dtype=None):
        return torch.randn(shape, generator=generator, device=device, dtype=dtype)

    cu.ConfigMixin = ConfigMixin
    cu.register_to_config = register_to_config
    ut.deprecate = deprecate
    tu.randn_tensor = randn_tensor
    su.KarrasDiffusionSchedulers = KarrasDiffusionSchedulers
    su.SchedulerMixin = SchedulerMixin
    su.SchedulerOutput = SchedulerOutput
    d.configuration_utils, d.utils, d.schedulers = cu, ut, sc
    ut.torch_utils = tu
    sc.scheduling_utils = su
    for name, mod in [("diffusers", d), ("diffusers.configuration_utils", cu),
                      ("diffusers.utils", ut), ("diffusers.utils.torch_utils", tu),
                      ("diffusers.schedulers", sc),
                      ("diffusers.schedulers.scheduling_utils", su)]:
        sys.modules[name] = mod


def _patch_transformers():
    from transformers.models.auto import auto_factory
    orig = auto_factory._LazyAutoMapping.register

    def register(self, key, value, exist_ok=False):
        return orig(self, key, value, exist_ok=True)
    auto_factory._LazyAutoMapping.register = register

    import transformers.models.qwen2 as q2
    if "transformers.models.qwen2.tokenization_qwen2_fast" not in sys.modules:
        m = types.ModuleType("transformers.models.qwen2.tokenization_qwen2_fast")
        from transformers.models.qwen2.tokenization_qwen2 import Qwen2Tokenizer
        m.Qwen2TokenizerFast = Qwen2Tokenizer
        sys.modules[m.__name__] = m
        q2.tokenization_qwen2_fast = m


_loaded = {}


def load():
    """Import and return the reference modules needed for goldens."""
    if _loaded:
        return _loaded
    _install_diffusers_stub()
    _patch_transformers()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import vibevoice.schedule.dpm_solver as dpm
    import vibevoice.modular.configuration_vibevoice as cfg
    import vibevoice.modular.modular_vibevoice_diffusion_head as head
    import vibevoice.modular.modular_vibevoice_tokenizer as tok
    import vibevoice.modular.modeling_vibevoice as mv
    import vibevoice.modular.modeling_vibevoice_inference as mvi
    orig_tie = mvi.VibeVoiceForConditionalGenerationInference.tie_weights

    def tie_weights(self, *a, **k):
        return orig_tie(self)
    mvi.VibeVoiceForConditionalGenerationInference.tie_weights = tie_weights
    _loaded.update(dpm=dpm, cfg=cfg, head=head, tok=tok, mv=mv, mvi=mvi)
    return _loaded
