"""VibeVoiceForConditionalGenerationInference — the drop-in generate() surface.

Keeps the reference's plugin API (vibevoice/modular/modeling_vibevoice_inference.py):
`from_pretrained(path, torch_dtype, device_map, attn_implementation)`,
`.eval()`, `.set_ddpm_inference_steps(n)` (:147-148) and
`.generate(**processor_outputs, cfg_scale, tokenizer, generation_config,
audio_streamer, stop_check_fn, refresh_negative, max_length_times, ...)`
(:327-710) returning `VibeVoiceGenerationOutput(sequences, speech_outputs,
reach_max_step_sample)` (:39-52).

The loop body's arithmetic runs in libvibevoice_hip.so (engine.py); this file
only does the reference's control flow (token choice among the valid ids,
finish / max-length bookkeeping, CFG negative-stream bookkeeping) on host
integers.  The negative stream is kept as a COMPACTED per-sample KV cache,
which is equivalent to the reference's mask/KV shuffling (:563-580, :609-639):
  * reset on speech_start (:563-580)   -> neg_len = 0
  * skip for non-diffusion samples in a diffusion step (:609-639)
                                       -> the step's entry is not committed
  * the negative pass consumes the same embedding the positive pass consumed
    this step (:594-596; [speech_start] at step 0, :378-385), so it is batched
    with the positive rows into one LM pass and committed afterwards.
"""
import math
import os
from dataclasses import dataclass
from typing import List, Optional

import torch

from . import _lib
from .config import VibeVoiceConfig
from .engine import Engine
from .weights import head_tp_default, synthetic_state_dict


@dataclass
class VibeVoiceGenerationOutput:
    sequences: torch.LongTensor = None
    speech_outputs: Optional[List[torch.Tensor]] = None
    reach_max_step_sample: Optional[torch.BoolTensor] = None


class _LMConfigView:
    def __init__(self, d, attn):
        self.__dict__.update(d)
        self._attn_implementation = attn


class _ModelView:
    """`model.model.*` attributes callers touch: the language model's config
    (inference_from_file.py:315-316), the noise scheduler (gradio_demo.py:114-118),
    the tokenizers / connectors / speech scaling of VibeVoiceModel
    (modeling_vibevoice.py:97-145) as views over the engine (tokenizer.py)."""

    def __init__(self, owner):
        from . import tokenizer as tk
        self._o = owner
        self.language_model = type("LM", (), {})()
        self.language_model.config = _LMConfigView(dict(owner.config.decoder_config), owner.attn_implementation)
        pool = tk._SlotPool(owner, max(8, owner.engine.max_batch))
        self.acoustic_tokenizer = tk.AcousticTokenizer(owner, pool, owner.config.acoustic_tokenizer_config)
        self.semantic_tokenizer = tk.SemanticTokenizer(owner, pool, owner.config.semantic_tokenizer_config)
        self.acoustic_connector = tk.Connector(owner, 0)
        self.semantic_connector = tk.Connector(owner, 1)

    @property
    def speech_scaling_factor(self):
        return self._o.engine.w["speech_scaling_factor"]

    @property
    def speech_bias_factor(self):
        return self._o.engine.w["speech_bias_factor"]

    @property
    def noise_scheduler(self):
        return self._o.engine.schedule

    @noise_scheduler.setter
    def noise_scheduler(self, sched):
        """gradio_demo.py:114-119 swaps in sde-dpmsolver++ via from_config, then calls
        set_ddpm_inference_steps; captured graphs of the old solver are dropped."""
        from .schedule import Schedule
        if not isinstance(sched, Schedule):
            raise TypeError("noise_scheduler must be built with noise_scheduler.from_config(...)")
        torch.cuda.synchronize(self._o.device)    # graphs may still be executing: drain before freeing them
        self._o.engine.set_schedule(sched)
        self._o._graph_cache.clear()
        self._o._graph_seen.clear()


def load_state_dict(path, cfg=None):
    """Safetensors shards of a HF checkpoint dir, loaded with the safe loader
    only.  With `model.safetensors.index.json` present exactly the shards its
    weight_map names are read (a HF loader's rule); otherwise every
    *.safetensors file.  lm_head follows the reference's tie rule
    (modeling_vibevoice_inference.py:120-129): tied to the embedding when the
    config's top-level tie_word_embeddings is set (or the checkpoint has none)."""
    import json
    from safetensors.torch import load_file
    index = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(index):
        with open(index) as f:
            wmap = json.load(f)["weight_map"]
        files = sorted(set(wmap.values()))
    else:
        files = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
    if not files:
        raise FileNotFoundError(f"no .safetensors files under {path}")
    sd = {}
    for f in files:
        sd.update(load_file(os.path.join(path, f)))
    emb = sd.get("model.language_model.embed_tokens.weight")
    tied = cfg.tie_word_embeddings if cfg is not None else "lm_head.weight" not in sd
    if emb is not None and (tied or "lm_head.weight" not in sd):
        sd["lm_head.weight"] = emb
    return sd


def resolve_device(device_map):
    """The one ROCm device a `device_map` (as HF / accelerate accept it) names.
    Accepted: "cuda", "cuda:N", torch.device("cuda", N), N, "auto" (the current
    device) and {"": <one of these>}.  Everything that asks for the CPU / MPS /
    disk, or splits the model over devices, raises: this engine has no CPU
    path, and tensor parallelism is requested with `tp_group=` instead."""
    d = device_map
    if isinstance(d, dict):
        vals = set(map(str, d.values()))
        if len(vals) != 1:
            raise ValueError(f"device_map {device_map!r} splits the model; the HIP engine keeps it on one GPU "
                             "(tensor parallelism: tp_group=)")
        d = next(iter(d.values()))
    if isinstance(d, int) and not isinstance(d, bool):
        d = torch.device("cuda", d)
    if d == "auto":
        d = torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
    if isinstance(d, str):
        try:
            d = torch.device(d)
        except RuntimeError:
            d = None
    if not isinstance(d, torch.device) or d.type != "cuda":
        raise ValueError(f"device_map={device_map!r}: the VibeVoice MI355X engine runs on a ROCm GPU only "
                         "(use device_map=\"cuda\"); there is no CPU/MPS path — the reference's CPU eager run "
                         "is the test oracle (oracle/), not part of this package")
    if d.index is None:
        d = torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
    return d


def resolve_dtype(torch_dtype):
    """bf16 is the compute type (the reference's GPU dtype,
    demo/inference_from_file.py:265); anything else raises."""
    if torch_dtype in (None, "auto", "bfloat16", torch.bfloat16):
        return torch.bfloat16
    raise ValueError(f"torch_dtype={torch_dtype!r}: the MI355X engine computes in bfloat16 "
                     "(torch_dtype=torch.bfloat16)")


class VibeVoiceTokenConstraintProcessor:
    """LogitsProcessor that keeps only the valid speech-control ids
    (modeling_vibevoice_inference.py:54-67).  generate() does not call it — the
    engine computes only those 4 logits (k_final_head) — it is exported for
    callers that apply it to their own scores."""

    def __init__(self, valid_token_ids, device=None):
        self.valid_token_ids = torch.tensor(valid_token_ids, dtype=torch.long, device=device)

    def __call__(self, input_ids, scores):
        mask = torch.full_like(scores, float("-inf"))
        mask[:, self.valid_token_ids] = 0
        return scores + mask


class VibeVoiceForConditionalGenerationInference:
    def __init__(self, config: VibeVoiceConfig, state_dict, device="cuda", attn_implementation="hip",
                 max_batch=8, max_ctx=8192, tp_group=None, tp_head=None, persistent=True):
        """tp_group: a torch.distributed process group whose ranks (one per GPU)
        tensor-parallel-shard the Qwen2 backbone over RCCL; every
        rank then runs generate() on the same inputs (SPMD) and gets the same
        result.  None: the whole model on this GPU.  tp_head: shard the
        diffusion head's FFN over the group too (None: when its per-step
        weights exceed the Infinity Cache, i.e. VibeVoice-Large).  persistent:
        False keeps the engine off the grid-waiting one-launch kernels
        (vv_set_persistent; for a GPU shared by several processes)."""
        self.config = config
        self.attn_implementation = attn_implementation
        self.device = torch.device(device)
        self.dtype = torch.bfloat16
        self._sd = state_dict
        tp_rank, tp_size, uid = 0, 1, None
        if tp_group is not None:
            import torch.distributed as dist
            tp_rank, tp_size = dist.get_rank(tp_group), dist.get_world_size(tp_group)
            if tp_size > 1:
                box = [Engine.tp_unique_id() if tp_rank == 0 else None]
                dist.broadcast_object_list(box, src=dist.get_global_rank(tp_group, 0), group=tp_group)
                uid = box[0]
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self.tp_head = head_tp_default(config, tp_size) if tp_head is None else bool(tp_head and tp_size > 1)
        self.engine = Engine(config, state_dict, self.device, max_batch=max_batch, tp_head=self.tp_head,
                             max_ctx=min(max_ctx, config.decoder_config.max_position_embeddings),
                             tp_rank=tp_rank, tp_size=tp_size, tp_unique_id=uid, persistent=persistent)
        self.ddpm_inference_steps = config.diffusion_head_config.ddpm_num_inference_steps
        self.model = _ModelView(self)
        self.use_graphs = True          # capture the steady-state loop body into hipGraphs
        self._bufs = {}
        self._graph_cache, self._graph_seen = {}, set()
        self._graph_epoch = None        # engine workspace epoch the cached graphs were captured at
        # this model's own capture stream: torch.cuda.graph() shares one side stream
        # process-wide and synchronizes the whole device, so two models generating
        # on two host threads would capture into each other's graphs
        self._capture_stream = None

    def _step_buffers(self, B):
        """Static device operands of the loop body for batch B (shared by every
        generate call of that batch size, so captured graphs stay valid)."""
        if B not in self._bufs:
            dev, eng, dt = self.device, self.engine, self.dtype
            H, D = eng.hidden, self.config.acoustic_vae_dim
            i32 = dict(device=dev, dtype=torch.int32)
            # host -> device control data travels in two copies per step:
            # [positions(2B) | next ids(B)] (int32) and [noise(B, D) bf16 | diffusion rows(B) int32]
            # (noise first: its rows stay 128-byte aligned)
            ctl_dev, ctl_pin = torch.zeros(3 * B, **i32), torch.zeros(3 * B, dtype=torch.int32, pin_memory=True)
            nb = B * D * torch.finfo(dt).bits // 8
            dn_dev = torch.zeros(nb + 4 * B, device=dev, dtype=torch.uint8)
            # two sets: the speculative diffusion of step k writes one while
            # step k-1's copy from the other may still be queued
            dn_pins = [torch.zeros(nb + 4 * B, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
            self._bufs[B] = dict(
                rows2=torch.arange(2 * B, **i32),
                x_in2=torch.zeros(2 * B, H, device=dev, dtype=dt),
                hid=torch.zeros(2 * B, H, device=dev, dtype=dt),
                logits=torch.zeros(2 * B, 4, device=dev, dtype=torch.float32),
                ctl_dev=ctl_dev, ctl_pin=ctl_pin,
                pos_dev=ctl_dev[:2 * B], ids_dev=ctl_dev[2 * B:], pos_pin=ctl_pin[:2 * B], ids_pin=ctl_pin[2 * B:],
                dn_dev=dn_dev, dn_pins=dn_pins,
                noise_dev=dn_dev[:nb].view(dt).view(B, D), didx_dev=dn_dev[nb:].view(torch.int32),
                noise_pins=[p[:nb].view(dt).view(B, D) for p in dn_pins],
                didx_pins=[p[nb:].view(torch.int32) for p in dn_pins],
                audio_dev=torch.zeros(B, eng.hop, device=dev, dtype=dt),
                logits_pin=torch.zeros(B, 4, dtype=torch.float32, pin_memory=True))
        return self._bufs[B]

    # ------------------------------------------------------------ loading
    config_class = VibeVoiceConfig          # AutoModelForCausalLM.register checks this name (vibevoice/ shim)

    @classmethod
    def from_pretrained(cls, path, torch_dtype=torch.bfloat16, device_map="cuda", attn_implementation="hip",
                        synthetic_seed=0, **kw):
        """`path`: a checkpoint dir (config.json + *.safetensors), or
        "synthetic:1.5B" / "synthetic:Large" for seeded random weights at the
        real shapes (no checkpoints are reachable offline).

        `device_map` / `torch_dtype` as the demos pass them
        (demo/inference_from_file.py:282-305): a CUDA (ROCm) device and bf16.
        The CPU / MPS / fp32 branches of the demo are refused with an explicit
        error — there is no CPU path behind this class."""
        resolve_dtype(torch_dtype)
        dev = resolve_device(device_map)
        if str(path).startswith("synthetic:"):
            cfg = VibeVoiceConfig.builtin(str(path).split(":", 1)[1])
            sd = synthetic_state_dict(cfg, seed=synthetic_seed, device=dev)
        else:
            cfg = VibeVoiceConfig.from_json_file(os.path.join(path, "config.json"))
            sd = load_state_dict(path, cfg)
        return cls(cfg, sd, dev, attn_implementation=attn_implementation, **kw)

    @classmethod
    def _from_config(cls, config, torch_dtype=None, device_map="cuda", attn_implementation="hip", seed=0, **kw):
        """AutoModelForCausalLM.from_config(config): random-init weights, as
        PreTrainedModel._from_config builds an untrained model (seeded here)."""
        resolve_dtype(torch_dtype)
        dev = resolve_device(device_map)
        return cls(config, synthetic_state_dict(config, seed=seed, device=dev), dev,
                   attn_implementation=attn_implementation, **kw)

    def eval(self):
        return self

    # modeling_vibevoice_inference.py:97-115
    acoustic_tokenizer = property(lambda self: self.model.acoustic_tokenizer)
    semantic_tokenizer = property(lambda self: self.model.semantic_tokenizer)
    acoustic_connector = property(lambda self: self.model.acoustic_connector)
    semantic_connector = property(lambda self: self.model.semantic_connector)
    speech_scaling_factor = property(lambda self: self.model.speech_scaling_factor)
    speech_bias_factor = property(lambda self: self.model.speech_bias_factor)

    def to(self, *args, **kwargs):
        """Moving the engine is not possible: accept only the device it lives on
        and bf16 (the reference's `.to("mps")` / fp32 branch raise here)."""
        for a in list(args) + list(kwargs.values()):
            if isinstance(a, torch.dtype):
                resolve_dtype(a)
            elif a is not None and not isinstance(a, bool):
                if resolve_device(a) != self.device:
                    raise ValueError(f"the engine lives on {self.device}; it cannot be moved to {a}")
        return self

    def set_ddpm_inference_steps(self, num_steps=None):
        self.ddpm_inference_steps = num_steps or self.config.diffusion_head_config.ddpm_num_inference_steps

    # ------------------------------------------------------------ prefill
    def _prompt_embeds(self, input_ids, attention_mask, speech_tensors, speech_masks, speech_input_mask):
        """Embeddings of the un-padded prompt tokens with voice latents spliced in
        (forward :217-225, _process_speech_inputs :150-164)."""
        dev, eng = self.device, self.engine
        keep = attention_mask.to(torch.bool)
        ids = input_ids[keep].to(device=dev, dtype=torch.int32)
        emb = eng.embed(ids)
        if speech_tensors is not None and speech_masks is not None and speech_input_mask is not None:
            audio = speech_tensors.to(device=dev, dtype=self.dtype)
            mean = eng.acoustic_encode(audio)                             # [Nv, F, D]
            fix_std = torch.tensor(self.config.acoustic_tokenizer_config.fix_std).to(self.dtype)
            value = (fix_std / 0.8).item()
            # the reference's gaussian sample draws, same order/dtypes (tokenizer :981-989)
            stdv = torch.randn(mean.shape[0], device=dev, dtype=mean.dtype) * value
            noise = torch.randn_like(mean)
            feats = eng.vae_features(mean, stdv, noise)
            sm = speech_masks.to(torch.bool).to(dev)
            if sm.shape[1] != mean.shape[1]:
                raise ValueError(f"speech_masks has {sm.shape[1]} frames, encoder produced {mean.shape[1]}")
            conn = eng.connector(0, feats[sm])                              # connector is row-wise
            # speech rows land at speech_input_mask positions, in row-major order (:225)
            sim = speech_input_mask.to(torch.bool).cpu()[attention_mask.to(torch.bool).cpu()]
            pos = torch.nonzero(sim).reshape(-1).to(device=dev, dtype=torch.int32)
            if pos.numel() != conn.shape[0]:
                raise ValueError(f"{pos.numel()} speech positions vs {conn.shape[0]} speech frames")
            eng.scatter_rows(conn, pos, emb)
        return emb

    # ------------------------------------------------------------ generate
    @torch.no_grad()
    def generate(self, inputs=None, generation_config=None, audio_streamer=None, speech_tensors=None,
                 speech_masks=None, speech_input_mask=None, return_speech=True, cfg_scale=1.0,
                 stop_check_fn=None, **kwargs):
        """The reference's generate() (modeling_vibevoice_inference.py:327-710), same
        arguments and return type.  Extra keywords: `forced_tokens` (bench /
        tests) = per-sample token schedule that replaces the constrained argmax
        (the argmax is still computed and read back every step); `generator` = a
        CPU torch.Generator for the per-step diffusion noise (default: the global
        RNG, as the reference's torch.randn at :716) — with one per call,
        generate() calls on several host threads draw independently of each
        other's interleaving (the Gradio demo serves from worker threads)."""
        verbose = kwargs.get("verbose", False)
        sess = self.generate_session(inputs, generation_config, audio_streamer, speech_tensors, speech_masks,
                                     speech_input_mask, cfg_scale, stop_check_fn, **kwargs)
        rng = range(sess.max_steps)
        if kwargs.get("show_progress_bar", True) and verbose:
            from tqdm import tqdm
            rng = tqdm(rng, desc="Generating", leave=True, ncols=100, mininterval=0.5)
        for _ in rng:
            if not sess.step():
                break
        return sess.result(return_speech)

    @torch.no_grad()
    def generate_session(self, inputs=None, generation_config=None, audio_streamer=None, speech_tensors=None,
                         speech_masks=None, speech_input_mask=None, cfg_scale=1.0, stop_check_fn=None, **kwargs):
        """generate() split into prefill (done here) + one `step()` per loop iteration."""
        return GenerateSession(self, inputs, generation_config, audio_streamer, speech_tensors, speech_masks,
                               speech_input_mask, cfg_scale, stop_check_fn, **kwargs)


class _Staging:
    """Pinned host ring -> device copies for the loop's small per-step operands
    (positions, slot lists, noise).  One async H2D each; the ring is drained
    (stream sync) only when it wraps."""

    def __init__(self, dev, dtype, n):
        self.host = torch.empty(n, dtype=dtype, pin_memory=True)
        self.dev = torch.empty(n, dtype=dtype, device=dev)
        self.n, self.off = n, 0

    def put(self, values):
        t = torch.as_tensor(values).reshape(-1).to(self.host.dtype)
        k = t.numel()
        if k > self.n:
            raise ValueError("staging ring too small")
        if self.off + k > self.n:
            torch.cuda.current_stream().synchronize()
            self.off = 0
        h = self.host[self.off:self.off + k]
        h.copy_(t)
        d = self.dev[self.off:self.off + k]
        d.copy_(h, non_blocking=True)
        self.off = (self.off + k + 63) // 64 * 64
        return d


class GenerateSession:
    """State of one generate() call (modeling_vibevoice_inference.py:327-710).

    Host side holds only the reference's control state (finished / reach_max /
    per-sample lengths / token ids); every tensor of the loop body lives on the
    device and every op on it is a libvibevoice_hip.so call.
    """

    def __init__(self, model, inputs, generation_config, audio_streamer, speech_tensors, speech_masks,
                 speech_input_mask, cfg_scale, stop_check_fn, **kwargs):
        tokenizer = kwargs.pop("tokenizer", None)
        kwargs.pop("parsed_scripts", None)
        kwargs.pop("all_speakers_list", None)
        self.m = model
        self.max_length_times = kwargs.pop("max_length_times", 2)
        self.refresh_negative = kwargs.get("refresh_negative", True)
        self.forced = kwargs.get("forced_tokens", None)
        self.gen = kwargs.get("generator", None)          # CPU generator of the diffusion noise (None: global RNG)
        self.cfg_scale = cfg_scale
        self.stop_check_fn = stop_check_fn
        self.audio_streamer = audio_streamer
        input_ids = kwargs["input_ids"] if inputs is None else inputs
        attention_mask = kwargs.get("attention_mask")
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        gen = dict(generation_config or {})
        self.do_sample = bool(gen.get("do_sample", False))

        dev, eng = model.device, model.engine
        self.dev, self.eng = dev, eng
        B, L = input_ids.shape
        self.B, self.L = B, L
        lmc = model.config.decoder_config
        max_new = kwargs.get("max_new_tokens")
        if max_new is None:
            max_new = lmc.max_position_embeddings - L                      # :371-372
        self.max_length = gen.get("max_length") or (L + max_new)
        Li = attention_mask.sum(-1).cpu().long()
        self.max_steps = min(self.max_length - L, int(self.max_length_times * L))        # :421
        self.per_sample_max = torch.minimum(self.max_length - Li, (self.max_length_times * Li).long())  # :422

        self.start_id, self.end_id = tokenizer.speech_start_id, tokenizer.speech_end_id
        self.diff_id, self.eos_id = tokenizer.speech_diffusion_id, tokenizer.eos_token_id
        self.valid = [self.start_id, self.end_id, self.diff_id, self.eos_id]                # :405-413
        bos = getattr(tokenizer, "bos_token_id", None)
        if bos is not None:
            raise NotImplementedError("a bos id in the constrained set (Qwen tokenizers have none)")
        self.order = sorted(range(4), key=lambda j: self.valid[j])         # argmax ties -> lowest id
        eng.set_valid_ids(self.valid)
        eng.set_steps(model.ddpm_inference_steps)
        need_ctx = int(Li.max()) + self.max_steps + 2
        if need_ctx > eng.max_ctx or B > eng.max_batch:
            raise RuntimeError(f"engine capacity (batch {eng.max_batch}, ctx {eng.max_ctx}) < request "
                               f"(batch {B}, ctx {need_ctx}); construct with larger max_batch/max_ctx")

        self.finished = torch.zeros(B, dtype=torch.bool)
        self.reach_max = torch.zeros(B, dtype=torch.bool)
        self.pos_len = Li.clone()
        self.neg_len = torch.zeros(B, dtype=torch.long)
        self.correct_cnt = torch.zeros(B, dtype=torch.long)                # :393
        self.neg_passes = 0                                                # negative cache length (all rows)
        self.audio_chunks = [[] for _ in range(B)]
        self.seq = [input_ids.cpu()]
        self.step_idx = 0
        self.done = False
        i32 = dict(device=dev, dtype=torch.int32)
        self.ints = _Staging(dev, torch.int32, 1 << 16)
        self.valid_t = torch.tensor(self.valid)
        self.order_t = torch.tensor(self.order)
        if self.do_sample:
            # torch.multinomial(softmax(scores), 1) (:502-505) over the full-vocabulary
            # constrained scores is ATen's one-sample path: argmax(p / q), q ~ Exp(1)
            # drawn for EVERY vocabulary entry on the logits' device generator.  The
            # same [B, vocab] draw is made here (same generator, same offsets), and only
            # its 4 legal columns are read back.
            self.vocab = int(model.config.decoder_config.vocab_size)
            self.q_cols = torch.tensor(self.valid, device=dev)
            self.q_pin = torch.zeros(B, 4, dtype=torch.float32, pin_memory=True)
        # static device operands of the loop body (graph-capturable): LM rows are
        # [positive B | negative B]; the negative rows consume the same input (:594-596)
        sb = model._step_buffers(B)
        for k, v in sb.items():
            setattr(self, k, v)
        self.use_graphs = kwargs.get("use_graphs", model.use_graphs)
        # sde-dpmsolver++ draws its per-step noise from the device generator
        # (dpm_solver.py:985-987), which a missed speculation could not rewind
        self.sde = eng.schedule.sde
        self.speculate = kwargs.get("speculate", True) and not self.sde
        if self.sde:
            self.sde_buf = torch.empty(eng.steps * 2 * B * model.config.acoustic_vae_dim, device=dev,
                                       dtype=torch.float32)
        self.spec_miss = 0
        self.pos_pushed = False
        self.logits_ready = torch.cuda.Event()
        # the engine's grid-wait error word, read back stream-ordered after every
        # diffusion step (vv_sync_error_async): a step's audio goes to the streamer
        # only once the word covering its diffusion has been read as clear
        self.err_pin = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.err_ready = torch.cuda.Event()
        self.err_queued = False      # a copy of the word is queued and err_pin not yet checked
        self.pending_put = None
        self.graphs = model._graph_cache
        self.seen = model._graph_seen

        # fresh streaming codec caches per call (VibeVoiceTokenizerStreamingCache() x2, :387-388)
        eng.codec_reset(torch.arange(B, **i32))
        # ---- step 0: positive prefill rows + speculative negative [speech_start] rows
        emb = model._prompt_embeds(input_ids.to(dev), attention_mask.to(dev), speech_tensors, speech_masks,
                                   speech_input_mask)
        neg_in = eng.embed(torch.full((B,), self.start_id, **i32))
        ntok = emb.shape[0]
        tok_slot = torch.cat([torch.repeat_interleave(torch.arange(B), Li), torch.arange(B, 2 * B)])
        tok_pos = torch.cat([torch.cat([torch.arange(int(n)) for n in Li]), torch.zeros(B, dtype=torch.long)])
        last = torch.cumsum(Li, 0) - 1
        out_idx = torch.cat([last, torch.arange(ntok, ntok + B)])
        step_in = torch.cat([emb, neg_in], 0)
        eng.lm_forward(step_in, tok_slot.to(**i32), tok_pos.to(**i32), out_idx.to(**i32), hidden_out=self.hid,
                       logits_out=self.logits, max_pos=int(tok_pos.max()))

    # ---------------------------------------------------------------- device phases
    def _replay(self, key, fn):
        """Run `fn` (device work only, on static buffers).  With graphs on, the
        second occurrence of `key` is captured into a hipGraph (the first runs
        eagerly so every kernel is loaded) and later ones replay it."""
        if not self.use_graphs:
            return fn()
        ep = _lib.lib().vv_ws_epoch()
        if ep != self.m._graph_epoch:    # a workspace moved (e.g. a longer prefill): captured pointers are stale
            torch.cuda.current_stream().synchronize()
            self.graphs.clear()
            self.seen.clear()
            self.m._graph_epoch = ep
        full = (self.B, self.m.engine.steps, float(self.cfg_scale), self.sde) + key
        g = self.graphs.get(full)
        if g is None:
            if full not in self.seen:
                self.seen.add(full)
                return fn()
            g = torch.cuda.CUDAGraph()
            cur = torch.cuda.current_stream()
            if self.m._capture_stream is None:
                self.m._capture_stream = torch.cuda.Stream(self.dev)
            cs = self.m._capture_stream
            cs.wait_stream(cur)
            with torch.cuda.stream(cs):
                # thread-local capture mode: another host thread's engine calls
                # (their own streams) stay legal while this one captures
                g.capture_begin(capture_error_mode="thread_local")
                try:
                    fn()
                finally:
                    g.capture_end()
            cur.wait_stream(cs)
            self.graphs[full] = g
        g.replay()

    def _lm_phase(self):
        """Positive + negative decode rows in one pass (:483-486, :598-600)."""
        B, eng = self.B, self.eng

        def body():
            eng.lm_forward(self.x_in2[:B], self.rows2, self.pos_dev, self.rows2, hidden_out=self.hid,
                           logits_out=self.logits, max_pos=eng.max_ctx - 1, ntok=2 * B)
        self._replay(("lm",), body)

    def _diff_phase(self, n):
        """CFG diffusion sampling for the n rows in didx_dev (:644, 712-725):
        noise_dev[:n] is replaced by the latents."""
        B, eng = self.B, self.eng

        def body():
            d = self.didx_dev[:n]
            if n == B:
                pos_h, neg_h = self.hid[:B], self.hid[B:]
            else:   # one gather keeps [pos | neg] adjacent (used in place by the engine)
                both = self.hid.index_select(0, torch.cat([d, d + B]))
                pos_h, neg_h = both[:n], both[n:]
            z = None
            if self.sde:   # one [2n, latent] fp32 draw per step, in step order (randn_tensor, :985-987)
                S, D = eng.steps, self.m.config.acoustic_vae_dim
                z = self.sde_buf[:S * 2 * n * D].view(S, 2 * n, D)
                for s in range(S):
                    torch.randn(2 * n, D, device=self.dev, dtype=torch.float32, out=z[s])
            eng.diffusion_sample(pos_h, neg_h, self.noise_dev[:n], self.cfg_scale, sde_noise=z)
        self._replay(("diff", n), body)

    def _post_phase(self, n):
        """next_embeds = embed(next tokens) (:584); for the n diffusion rows the
        streaming decode / encode and the connectors (:651-687), overwriting
        those rows' embeddings."""
        eng = self.eng

        def body():
            eng.embed(self.ids_dev, out=self.x_in2)
            if n:
                d = self.didx_dev[:n]
                eng.codec_step(d, self.noise_dev[:n], self.audio_dev[:n], embeds_out=self.x_in2, embed_rows=d)
        self._replay(("post", n), body)

    def _push_controls(self, nxt):
        """One H2D copy: this step's token ids (read by the post phase) and the
        next step's positive / negative positions (its LM phase), which are final
        once the bookkeeping of this step is done.  The previous copy from the
        same pinned buffer finished before this step's logits were read back."""
        B = self.B
        self.ids_pin.copy_(nxt)
        self.pos_pin[:B].copy_(self.pos_len)
        self.pos_pin[B:].copy_(self.neg_len)
        self.ctl_dev.copy_(self.ctl_pin, non_blocking=True)
        self.pos_pushed = True

    def _stage_diffusion(self, didx, buf):
        """Draw the diffusion noise from the CPU generator (:716) and queue the
        H2D copies of the row list and the noise (pinned set `buf`)."""
        n = didx.numel()
        dp, npin = self.didx_pins[buf], self.noise_pins[buf]
        dp[:n].copy_(didx)
        noise = torch.randn(2 * n, self.m.config.acoustic_vae_dim, generator=self.gen)
        npin[:n].copy_(noise[:n])
        self.dn_dev.copy_(self.dn_pins[buf], non_blocking=True)      # rows + noise in one copy

    def _speculate(self):
        """Queue the diffusion for the rows whose last token was speech_start or
        speech_diffusion BEFORE the token choice is read back, so the GPU runs it
        while the host reads the logits and does the bookkeeping.  The choice
        itself is unchanged: step() keeps the result only if exactly these rows
        chose speech_diffusion, else it restores the CPU generator and redoes the
        diffusion for the right rows.  Sampling (:505) draws on the device
        generator, the noise on the CPU one (:716), so both modes speculate;
        sde-dpmsolver++ (device-generator noise after the sampling draw) does not."""
        if not self.speculate:
            return None
        last = self.seq[-1][:, -1]
        rows = torch.nonzero(~self.finished & ((last == self.diff_id) | (last == self.start_id))).reshape(-1)
        if rows.numel() == 0:
            return None
        state = self.gen.get_state() if self.gen is not None else torch.get_rng_state()
        self._stage_diffusion(rows, self.step_idx & 1)
        self._diff_phase(rows.numel())
        return rows, state

    def _check_err(self):
        """Raise if the error word read back last (err_pin) is set: a one-launch
        kernel's in-launch grid wait gave up, the latents / audio of that step are
        invalid.  The wait counters that launch left part-advanced are reset
        first (vv_sync_reset), so the next generate() starts from a clean state."""
        self.err_queued = False
        if int(self.err_pin[0]):
            self.pending_put = None
            self.done = True
            self.err_pin.zero_()
            self.eng.sync_reset()
            raise RuntimeError("one-launch kernel: an in-launch grid wait gave up (workgroups not co-resident); "
                               "this step's latents and audio are invalid and were not streamed")

    def _drain_err(self):
        """Wait for the last queued error-word copy (if any) and check it: the
        loop's exits, where no later logits read-back covers it."""
        if self.err_queued:
            self.err_ready.synchronize()
            self._check_err()

    def _flush_audio(self, sync):
        """Put the previous diffusion step's audio into the streamer once the
        error word covering it has been read (sync=False: it already has, by the
        logits read-back that follows it on the stream)."""
        if self.pending_put is None:
            return
        if sync:
            self.err_ready.synchronize()
            self._check_err()
        audio, didx = self.pending_put
        self.pending_put = None
        self.audio_streamer.put(audio[:, None, :], didx)

    def _restore_rng(self, state):
        if self.gen is not None:
            self.gen.set_state(state)
        else:
            torch.set_rng_state(state)

    # ---------------------------------------------------------------- one iteration
    def step(self):
        """One iteration of the reference loop (:432-690).  Returns False (and
        does nothing) once the loop has ended."""
        if self.done or self.step_idx >= self.max_steps:
            self.done = True
            self._drain_err()
            return False
        B, eng, dev, step = self.B, self.eng, self.dev, self.step_idx
        st = self.audio_streamer
        if self.stop_check_fn is not None and self.stop_check_fn():       # :434-440
            if st is not None:
                self._flush_audio(sync=True)
                st.end()
            self.done = True
            self._drain_err()
            return False
        if st is not None and any(getattr(st, "finished_flags", [])):     # :443-447
            self.done = True
            self._drain_err()
            return False
        if bool(self.finished.all()):                                      # :449
            self.done = True
            self._drain_err()
            return False
        if self.L + step >= self.max_length:                               # :454-459
            self.reach_max[~self.finished] = True
            self.done = True
            self._drain_err()
            return False
        if step > 0:
            if not self.pos_pushed:   # normally sent with the previous step's ids (_push_controls)
                self.pos_pin[:B].copy_(self.pos_len)
                self.pos_pin[B:].copy_(self.neg_len)
                self.pos_dev.copy_(self.pos_pin, non_blocking=True)
            self.pos_pushed = False
            self._lm_phase()
            self.pos_len += 1
        # ---- token choice (:494-509); the argmax is always read back, as in the reference
        self.logits_pin.copy_(self.logits[:B], non_blocking=True)
        if self.do_sample:
            q = torch.empty(B, self.vocab, device=dev, dtype=torch.float32).exponential_(1)
            self.q_pin.copy_(q.index_select(1, self.q_cols), non_blocking=True)
        self.logits_ready.record()
        spec = self._speculate()
        self.logits_ready.synchronize()
        self._check_err()            # err_pin: copied behind the previous step's diffusion + codec
        if st is not None:
            self._flush_audio(sync=False)
        lg = self.logits_pin.clone()
        if self.do_sample:
            r = torch.softmax(lg, -1) / self.q_pin                            # ties -> lowest id, as over the vocab
            pick = self.order_t[r[:, self.order].argmax(-1)]
        else:
            pick = self.order_t[lg[:, self.order].argmax(-1)]
        nxt = self.valid_t[pick]
        if self.forced is not None:
            nxt = torch.tensor([f[step] if step < len(f) else self.eos_id for f in self.forced])
        finished = self.finished
        nxt[finished] = self.eos_id
        self.seq.append(nxt[:, None])
        # ---- negative stream when refresh_negative is False (:512-527): run and committed every step
        if not self.refresh_negative:
            self.neg_len += 1
            self.neg_passes += 1
        # ---- finish bookkeeping (:530-553)
        new_eos = (nxt == self.eos_id) & ~finished
        if new_eos.any():
            finished |= new_eos
            if st is not None:
                st.end(torch.nonzero(new_eos).reshape(-1))
        hit_max = (step >= self.per_sample_max) & ~finished
        if hit_max.any():
            finished |= hit_max
            self.reach_max |= hit_max
            if st is not None:
                st.end(torch.nonzero(hit_max).reshape(-1))
        ends = torch.nonzero(nxt == self.end_id).reshape(-1)              # :556-560
        if ends.numel():
            eng.codec_reset(self.ints.put(ends))
        starts = ~finished & (nxt == self.start_id)                         # :563-580
        if self.refresh_negative:
            self.neg_len[starts] = 0     # mask reset: empty context, next position 0
        diff = ~finished & (nxt == self.diff_id)                            # :588
        if diff.any():
            didx = torch.nonzero(diff).reshape(-1)
            n = didx.numel()
            if self.refresh_negative:                                       # negative pass :591-604
                self.neg_len += 1    # every row appends; rows reset above were computed speculatively
                self.neg_passes += 1  # and are always dropped again below (speech_start != diffusion)
            # non-diffusion correction (:609-639): drop the entry just appended.  Where the
            # reference's KV-shift test (:628) skips the shift while the mask shift (:618)
            # happens (correct_cnt == cache_len - 2), the new entry replaces the previous one.
            skip = torch.nonzero(~finished & ~diff).reshape(-1)
            quirk = [b for b in skip.tolist()
                     if int(self.correct_cnt[b]) == self.neg_passes - 2 and int(self.neg_len[b]) == 2]
            self.neg_len[skip] -= 1
            self.correct_cnt[skip] += 1
            if quirk:
                q = torch.tensor(quirk)
                eng.kv_copy(self.ints.put(q + B), self.ints.put(torch.ones_like(q)),
                            self.ints.put(torch.zeros_like(q)))
            self._push_controls(nxt)
            if spec is None or not torch.equal(spec[0], didx):
                if spec is not None:   # mispredicted: the speculative copies may still be queued
                    torch.cuda.current_stream().synchronize()
                    self._restore_rng(spec[1])
                    self.spec_miss += 1
                self._stage_diffusion(didx, self.step_idx & 1)
                self._diff_phase(n)
            self._post_phase(n)
            audio = self.audio_dev[:n].clone()
            self.eng.sync_error_async(self.err_pin)
            self.err_ready.record()
            self.err_queued = True
            for i, b in enumerate(didx.tolist()):
                self.audio_chunks[b].append(audio[i:i + 1])
            if st is not None:      # streamed once the next read-back shows the error word clear
                self.pending_put = (audio, didx)
        else:
            if spec is not None:
                self._restore_rng(spec[1])
                self.spec_miss += 1
            self._push_controls(nxt)
            self._post_phase(0)
        self.step_idx += 1
        return True

    def result(self, return_speech=True):
        if self.pending_put is not None:
            self._flush_audio(sync=True)
        self._drain_err()            # with or without a streamer: the last step's word
        self.eng.check_sync()
        if self.audio_streamer is not None:
            self.audio_streamer.end()
        outs = [torch.cat(c, dim=-1) if c else None for c in self.audio_chunks]
        return VibeVoiceGenerationOutput(sequences=torch.cat(self.seq, dim=1),
                                         speech_outputs=outs if return_speech else None,
                                         reach_max_step_sample=self.reach_max)
