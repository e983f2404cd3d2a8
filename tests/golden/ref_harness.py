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
    # the repository ships its own `vibevoice/` import-path package (drop-in
    # names over vibevoice_amd): the reference's must win here
    if REF in sys.path:
        sys.path.remove(REF)
    sys.path.insert(0, REF)
    for name in [n for n in sys.modules if n == "vibevoice" or n.startswith("vibevoice.")]:
        if not (getattr(sys.modules[name], "__file__", "") or "").startswith(REF):
            del sys.modules[name]
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


def install_generate_shims(mvi, forced):
    """Let the reference's own generate() (modeling_vibevoice_inference.py:327-710)
    run under transformers 5.15 on CPU, for the G8 loop trace.

    Harness-side only.  The loop body (negative-stream reset / skip, diffusion,
    streaming codec, connectors) is the reference's code unchanged; the shims
    replace only the transformers-4.51.3 plumbing it calls, which 5.15 changed:
      * `_build_generate_config_model_kwargs` (:255-325): GenerationConfig with
        the tokenizer ids, max_length = L + max_new_tokens (4.51.3
        `_prepare_generated_length`), a fresh DynamicCache, cache_position =
        arange(L); the logits processors are the list returned to the loop,
        which here holds one `forced` schedule processor (the loop appends its
        own VibeVoiceTokenConstraintProcessor after it, :415-418);
      * GenerationMixin 4.51.3 `prepare_inputs_for_generation` /
        `_update_model_kwargs_for_generation` (position_ids =
        cumsum(mask) - 1 with masked -> 1, mask gets a column of ones,
        cache_position += 1);
      * `DynamicCache.key_cache / value_cache` (:572-576, 624-631): lists of the
        per-layer K/V tensors (5.15 keeps them in `layers[i].keys/values`);
    `forced[b][step]` (eos after the list ends) wins the argmax: its logit is
    raised to 1e30 before the reference's constraint processor runs; an empty
    `forced` leaves the scores alone (the do_sample fixture).
    """
    from transformers import GenerationConfig, LogitsProcessor, LogitsProcessorList
    from transformers.cache_utils import DynamicCache

    DynamicCache.key_cache = property(lambda self: [layer.keys for layer in self.layers])
    DynamicCache.value_cache = property(lambda self: [layer.values for layer in self.layers])

    class Forced(LogitsProcessor):
        def __init__(self, L0, eos):
            self.L0, self.eos = L0, eos

        def __call__(self, input_ids, scores):
            if not forced:          # an empty schedule list: the model's own choice (greedy or sampled)
                return scores
            step = input_ids.shape[1] - self.L0
            scores = scores.clone()
            for b in range(scores.shape[0]):
                tok = forced[b][step] if step < len(forced[b]) else self.eos
                scores[b, tok] = 1e30
            return scores

    def build(self, generation_config, inputs, tokenizer, return_processors=False, **kwargs):
        gc = GenerationConfig(**(generation_config or {}), bos_token_id=tokenizer.bos_token_id,
                              eos_token_id=tokenizer.eos_token_id, pad_token_id=tokenizer.pad_token_id)
        gc.speech_start_id = tokenizer.speech_start_id
        gc.speech_end_id = tokenizer.speech_end_id
        gc.speech_diffusion_id = tokenizer.speech_diffusion_id
        input_ids = kwargs["input_ids"]
        L = input_ids.shape[-1]
        gc.max_length = L + kwargs["max_new_tokens"]
        gc.use_cache = True
        model_kwargs = dict(attention_mask=kwargs["attention_mask"], use_cache=True,
                            past_key_values=DynamicCache(), cache_position=torch.arange(L, dtype=torch.long))
        if return_processors:
            return gc, model_kwargs, input_ids, LogitsProcessorList([Forced(L, gc.eos_token_id)]), None
        return gc, model_kwargs, input_ids

    def prepare_inputs_for_generation(self, input_ids, past_key_values=None, attention_mask=None,
                                      inputs_embeds=None, cache_position=None, use_cache=True, **kw):
        if inputs_embeds is not None or cache_position[-1] >= input_ids.shape[1]:
            input_ids = input_ids[:, -cache_position.shape[0]:]
        elif input_ids.shape[1] != cache_position.shape[0]:
            input_ids = input_ids[:, cache_position]
        pos = attention_mask.long().cumsum(-1) - 1
        pos.masked_fill_(attention_mask == 0, 1)
        return dict(input_ids=input_ids.clone(), inputs_embeds=None, cache_position=cache_position,
                    past_key_values=past_key_values, use_cache=use_cache, attention_mask=attention_mask,
                    position_ids=pos[:, -input_ids.shape[1]:].clone())

    def update_model_kwargs(self, outputs, model_kwargs, is_encoder_decoder=False, num_new_tokens=1):
        model_kwargs["past_key_values"] = outputs.past_key_values
        m = model_kwargs["attention_mask"]
        model_kwargs["attention_mask"] = torch.cat([m, m.new_ones((m.shape[0], 1))], dim=-1)
        model_kwargs["cache_position"] = model_kwargs["cache_position"][-1:] + num_new_tokens
        return model_kwargs

    cls = mvi.VibeVoiceForConditionalGenerationInference
    cls._build_generate_config_model_kwargs = build
    cls.prepare_inputs_for_generation = prepare_inputs_for_generation
    cls._update_model_kwargs_for_generation = update_model_kwargs
