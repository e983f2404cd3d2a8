"""Python handle on the native engine (libvibevoice_hip.so).

Thin: converts torch device tensors to pointers, keeps borrowed weights alive,
and forwards to the C ABI.  No arithmetic happens here.
"""
import ctypes

import torch

from . import _lib
from .config import VibeVoiceConfig
from .schedule import Schedule
from .weights import codec_channels, head_tp_check, pack

_VALID_IDS_DEFAULT = None


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def engine_config(cfg: VibeVoiceConfig, max_batch, max_ctx, tp_size=1, tp_head=False):
    """vv_config of one engine; with tensor parallelism the LM head and
    intermediate counts are this rank's local ones (and the head FFN width,
    with tp_head)."""
    lm = cfg.decoder_config
    hc = cfg.diffusion_head_config
    c = _lib.VVConfig()
    c.hidden = lm.hidden_size
    c.n_layers = lm.num_hidden_layers
    c.n_heads = lm.num_attention_heads // tp_size
    c.n_kv_heads = lm.num_key_value_heads // tp_size
    c.head_dim = lm.get("head_dim") or lm.hidden_size // lm.num_attention_heads
    c.intermediate = lm.intermediate_size // tp_size
    c.rms_eps = lm.rms_norm_eps
    c.rope_theta = lm.rope_theta
    c.head_layers = hc.head_layers
    c.head_ffn = int(hc.hidden_size * hc.head_ffn_ratio) // (tp_size if tp_head else 1)
    c.latent_dim = hc.latent_size
    c.head_eps = hc.rms_norm_eps
    c.n_stages = len(cfg.dec_depths)
    for i, r in enumerate(cfg.ratios):
        c.ratios[i] = r
    for i, v in enumerate(cfg.dec_depths):
        c.dec_depths[i] = v
    for i, v in enumerate(cfg.enc_depths):
        c.enc_depths[i] = v
    c.dec_n_filters = cfg.acoustic_tokenizer_config.decoder_n_filters
    c.sem_n_filters = cfg.semantic_tokenizer_config.encoder_n_filters
    c.ac_enc_n_filters = cfg.acoustic_tokenizer_config.encoder_n_filters
    c.semantic_dim = cfg.semantic_vae_dim
    c.codec_eps = cfg.acoustic_tokenizer_config.layernorm_eps
    c.max_batch = max_batch
    c.max_ctx = max_ctx
    return c


class Engine:
    """One device-resident VibeVoice model instance."""

    def __init__(self, cfg: VibeVoiceConfig, state_dict, device="cuda", max_batch=1, max_ctx=4096,
                 valid_ids=None, tp_rank=0, tp_size=1, tp_unique_id=None, packed=None, tp_head=False,
                 persistent=True):
        """tp_size > 1: rank tp_rank's shard of the LM; tp_unique_id (bytes of
        vv_tp_unique_id, shared by the group) creates its RCCL communicator, None
        leaves it for a single-process group (lm_forward_group).
        packed: another engine's packed weights (`Engine.w`) to bind instead of
        packing `state_dict` again — a second context over the same device
        weights (the standalone tokenizer API's own codec slots).
        tp_head: shard the diffusion head's FFN over the TP group as well
        (vv_tp_shard_head).
        persistent: False keeps this context off the grid-waiting one-launch
        kernels (vv_set_persistent 0); "follow" runs them while exactly one
        context of the device is registered, without registering itself (the
        standalone tokenizer API's codec context: it computes with its owner's
        kernels and never demotes it)."""
        L = _lib.lib()
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("the VibeVoice HIP engine runs on a ROCm GPU device only")
        self.max_batch = max_batch
        self.max_ctx = max_ctx
        self.hidden = cfg.decoder_config.hidden_size
        self.latent = cfg.diffusion_head_config.latent_size
        self.hop = cfg.hop
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self.tp_head = bool(tp_head and tp_size > 1)
        if self.tp_head:
            head_tp_check(cfg, tp_size)
        with torch.cuda.device(self.device):
            self.w = packed if packed is not None else pack(state_dict, cfg, self.device, tp_rank=tp_rank,
                                                            tp_size=tp_size, tp_head=self.tp_head)
            h = ctypes.c_void_p()
            self._ecfg = engine_config(cfg, max_batch, max_ctx, tp_size, self.tp_head)
            _lib.check(L.vv_create(ctypes.byref(self._ecfg), self.device.index or 0, ctypes.byref(h)), "create")
            self.h = h
            if tp_size > 1 or tp_unique_id is not None:
                uid = None if tp_unique_id is None else ctypes.create_string_buffer(bytes(tp_unique_id),
                                                                                   len(tp_unique_id))
                _lib.check(L.vv_tp_init(h, tp_rank, tp_size, uid), "tp_init")
                if self.tp_head:
                    _lib.check(L.vv_tp_shard_head(h, 1), "tp_shard_head")
            if persistent is not True:
                _lib.check(L.vv_set_persistent(h, 2 if persistent == "follow" else 0), "set_persistent")
            for name, t in self.w.items():
                shape = (ctypes.c_int64 * max(1, t.dim()))(*t.shape)
                _lib.check(L.vv_bind_weight(h, name.encode(), _ptr(t), shape, t.dim()), f"bind {name}")
            _lib.check(L.vv_finalize(h), "finalize")
            if valid_ids is not None:
                self.set_valid_ids(valid_ids)
        self.steps = None
        self.schedule = Schedule()

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().vv_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- setup
    def set_valid_ids(self, ids):
        self._valid = list(ids)
        arr = (ctypes.c_int * len(ids))(*ids)
        _lib.check(_lib.lib().vv_set_valid_ids(self.h, len(ids), arr), "set_valid_ids")
        self.n_valid = len(ids)

    def check_sync(self):
        """Raise if a grid-waiting kernel's in-launch wait gave up since the last
        check (its outputs are then invalid; vv_sync_error, which also resets the
        wait counters).  Synchronises."""
        r = _lib.lib().vv_sync_error(self.h)
        if r < 0:
            _lib.check(r, "sync_error")
        if r:
            raise RuntimeError("one-launch kernel: an in-launch grid wait gave up (workgroups not co-resident); "
                               "the outputs since the last check are invalid")

    def sync_reset(self):
        """Zero every grid-wait counter of this context (vv_sync_reset; after a
        wait gave up).  Synchronises the device."""
        _lib.check(_lib.lib().vv_sync_reset(self.h), "sync_reset")

    def persistent_active(self):
        return _lib.lib().vv_persistent_active(self.h) == 1

    def sync_error_async(self, dst, stream=None):
        """Queue on the stream a copy of the grid-wait error word into dst (a
        1-element int32 pinned host or device tensor) and its reset; dst is valid
        once work queued after this call has been waited for."""
        _lib.check(_lib.lib().vv_sync_error_async(self.h, _ptr(dst), _stream(stream)), "sync_error_async")

    def set_schedule(self, schedule):
        """Replace the solver (model.model.noise_scheduler = ...); coefficients are
        rebuilt at the next set_steps."""
        self.schedule = schedule
        self.steps = None

    def set_steps(self, steps, stream=None):
        if steps == self.steps:
            return
        _, coef = self.schedule.coefficients(steps)
        tf = self.schedule.timestep_features(steps).to(self.device)
        c = (ctypes.c_float * coef.size)(*coef.reshape(-1).tolist())
        _lib.check(_lib.lib().vv_set_schedule(self.h, steps, c, _ptr(tf), _stream(stream)), "set_schedule")
        torch.cuda.current_stream().synchronize() if stream is None else stream.synchronize()
        self.steps = steps

    # ---------------------------------------------------------------- hot path
    def lm_forward(self, embeds, slots, pos, out_idx, hidden_out=None, logits_out=None, max_pos=None, stream=None,
                   ntok=None):
        """embeds [rows, H] bf16 (token i reads row i % rows; ntok defaults to rows);
        slots/pos/out_idx int32 device tensors of ntok / nout entries."""
        rows = embeds.shape[0]
        ntok = rows if ntok is None else ntok
        nout = out_idx.shape[0]
        if hidden_out is None:
            hidden_out = torch.empty(nout, self.hidden, dtype=torch.bfloat16, device=self.device)
        if logits_out is None:
            logits_out = torch.empty(nout, self.n_valid, dtype=torch.float32, device=self.device)
        mp = int(max_pos if max_pos is not None else pos.max().item()) + 1
        _lib.check(_lib.lib().vv_lm_forward(self.h, ntok, _ptr(embeds), rows, _ptr(slots), _ptr(pos), mp, nout,
                                            _ptr(out_idx), _ptr(hidden_out), _ptr(logits_out), _stream(stream)),
                   "lm_forward")
        return hidden_out, logits_out

    def lm_forward_group(self, peers, embeds, slots, pos, out_idx, hidden_out=None, logits_out=None,
                         max_pos=None, stream=None, ntok=None):
        """Run the TP group [self] + peers (ranks 0..n-1, same device) layer by
        layer with an on-device all-reduce; outputs of rank 0 (= self)."""
        rows = embeds.shape[0]
        ntok = rows if ntok is None else ntok
        nout = out_idx.shape[0]
        if hidden_out is None:
            hidden_out = torch.empty(nout, self.hidden, dtype=torch.bfloat16, device=self.device)
        if logits_out is None:
            logits_out = torch.empty(nout, self.n_valid, dtype=torch.float32, device=self.device)
        if getattr(self, "_valid", None):
            for p in peers:      # only on change: the copy is synchronous (not allowed inside a graph capture)
                if getattr(p, "_valid", None) != self._valid:
                    p.set_valid_ids(self._valid)
        mp = int(max_pos if max_pos is not None else pos.max().item()) + 1
        ctxs = (ctypes.c_void_p * (1 + len(peers)))(self.h, *[p.h for p in peers])
        _lib.check(_lib.lib().vv_lm_forward_group(1 + len(peers), ctxs, ntok, _ptr(embeds), rows, _ptr(slots),
                                                  _ptr(pos), mp, nout, _ptr(out_idx), _ptr(hidden_out),
                                                  _ptr(logits_out), _stream(stream)), "lm_forward_group")
        return hidden_out, logits_out

    @staticmethod
    def tp_unique_id():
        buf = ctypes.create_string_buffer(256)
        n = _lib.lib().vv_tp_unique_id(buf, 256)
        if n <= 0:
            _lib.check(-1, "tp_unique_id")
        return buf.raw[:n]

    def kv_copy(self, slots, src, dst, stream=None):
        _lib.check(_lib.lib().vv_kv_copy(self.h, slots.shape[0], _ptr(slots), _ptr(src), _ptr(dst), _stream(stream)),
                   "kv_copy")

    def embed(self, ids, out=None, stream=None):
        if out is None:
            out = torch.empty(ids.shape[0], self.hidden, dtype=torch.bfloat16, device=self.device)
        _lib.check(_lib.lib().vv_embed(self.h, ids.shape[0], _ptr(ids), _ptr(out), _stream(stream)), "embed")
        return out

    def diffusion_sample(self, pos_h, neg_h, x_io, cfg_scale, sde_noise=None, stream=None):
        """sde_noise: [steps, 2n, latent] fp32 per-step draws (sde-dpmsolver++ only)."""
        if self.schedule.sde != (sde_noise is not None):
            raise ValueError("sde_noise must be given exactly when the schedule is sde-dpmsolver++")
        _lib.check(_lib.lib().vv_diffusion_sample(self.h, pos_h.shape[0], _ptr(pos_h), _ptr(neg_h), _ptr(x_io),
                                                  float(cfg_scale), _ptr(sde_noise), _stream(stream)),
                   "diffusion_sample")
        return x_io

    def diffusion_sample_group(self, peers, pos_h, neg_h, x_io, cfg_scale, sde_noise=None, stream=None):
        """The sharded diffusion head of the TP group [self] + peers (ranks
        0..n-1 with tp_head, same device), ranks interleaved layer by layer with
        an on-device sum as the all-reduce; x_io updated once."""
        if self.schedule.sde != (sde_noise is not None):
            raise ValueError("sde_noise must be given exactly when the schedule is sde-dpmsolver++")
        for p in peers:
            p.set_steps(self.steps)
        ctxs = (ctypes.c_void_p * (1 + len(peers)))(self.h, *[p.h for p in peers])
        _lib.check(_lib.lib().vv_diffusion_sample_group(1 + len(peers), ctxs, pos_h.shape[0], _ptr(pos_h), _ptr(neg_h),
                                                        _ptr(x_io), float(cfg_scale), _ptr(sde_noise),
                                                        _stream(stream)), "diffusion_sample_group")
        return x_io

    def codec_step(self, slots, latent, audio_out, sem_out=None, embeds_out=None, embed_rows=None, stream=None):
        _lib.check(_lib.lib().vv_codec_step(self.h, slots.shape[0], _ptr(slots), _ptr(latent), _ptr(audio_out),
                                            _ptr(sem_out), _ptr(embeds_out), _ptr(embed_rows), _stream(stream)),
                   "codec_step")

    def codec_reset(self, slots, stream=None):
        _lib.check(_lib.lib().vv_codec_reset(self.h, slots.shape[0], _ptr(slots), _stream(stream)), "codec_reset")

    def codec_decode(self, slots, z, audio_out, stream=None):
        """One streaming acoustic-decoder frame: z [n, latent] (decoder input) -> audio_out [n, hop]."""
        _lib.check(_lib.lib().vv_codec_decode(self.h, slots.shape[0], _ptr(slots), _ptr(z), _ptr(audio_out),
                                              _stream(stream)), "codec_decode")

    def codec_encode(self, slots, audio, sem_out, stream=None):
        """One streaming semantic-encoder frame: audio [n, hop] -> sem_out [n, semantic_dim]."""
        _lib.check(_lib.lib().vv_codec_encode(self.h, slots.shape[0], _ptr(slots), _ptr(audio), _ptr(sem_out),
                                              _stream(stream)), "codec_encode")

    def codec_reset_net(self, net, slots, stream=None):
        """set_to_zero of one net's streaming state: net 0 = acoustic decoder, 1 = semantic encoder."""
        _lib.check(_lib.lib().vv_codec_reset_net(self.h, int(net), slots.shape[0], _ptr(slots), _stream(stream)),
                   "codec_reset_net")

    # ---------------------------------------------------------------- prefill helpers
    def acoustic_encode(self, audio_bf16, stream=None):
        nv, L = audio_bf16.shape
        frames = -(-L // self.hop)
        mean = torch.empty(nv, frames, self.latent, dtype=torch.bfloat16, device=self.device)
        _lib.check(_lib.lib().vv_acoustic_encode(self.h, nv, L, _ptr(audio_bf16.contiguous()), _ptr(mean),
                                                 _stream(stream)), "acoustic_encode")
        return mean

    def semantic_encode(self, audio_bf16, stream=None):
        """Non-streaming semantic encode of nv clips [nv, L] (L need not be whole
        frames) -> [nv, ceil(L / hop), semantic_dim]."""
        nv, L = audio_bf16.shape
        frames = -(-L // self.hop)
        S = self.cfg.semantic_vae_dim
        mean = torch.empty(nv, frames, S, dtype=torch.bfloat16, device=self.device)
        _lib.check(_lib.lib().vv_semantic_encode(self.h, nv, L, _ptr(audio_bf16.contiguous()), _ptr(mean),
                                                 _stream(stream)), "semantic_encode")
        return mean

    def vae_features(self, mean, stdv, noise, stream=None):
        nv, frames, D = mean.shape
        out = torch.empty_like(mean)
        _lib.check(_lib.lib().vv_vae_features(self.h, nv, frames, _ptr(mean), _ptr(stdv), _ptr(noise), _ptr(out),
                                              _stream(stream)), "vae_features")
        return out

    def connector(self, which, x, stream=None):
        x = x.contiguous()
        out = torch.empty(x.shape[0], self.hidden, dtype=torch.bfloat16, device=self.device)
        _lib.check(_lib.lib().vv_connector(self.h, which, x.shape[0], _ptr(x), _ptr(out), _stream(stream)),
                   "connector")
        return out

    def scatter_rows(self, src, idx, dst, stream=None):
        _lib.check(_lib.lib().vv_scatter_rows(self.h, src.shape[0], src.shape[1], _ptr(src), src.stride(0),
                                              _ptr(idx), _ptr(dst), dst.stride(0), _stream(stream)), "scatter_rows")


def semantic_channels(cfg):
    return codec_channels(cfg, "encoder", "semantic")
