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

from .config import VibeVoiceConfig
from .engine import Engine
from .weights import synthetic_state_dict


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
    """`model.model.*` attributes callers touch (inference_from_file.py:315-316)."""

    def __init__(self, owner):
        self._o = owner
        self.language_model = type("LM", (), {})()
        self.language_model.config = _LMConfigView(dict(owner.config.decoder_config), owner.attn_implementation)

    @property
    def noise_scheduler(self):
        return self._o.engine.schedule


def load_state_dict(path):
    """Safetensors shards of a HF checkpoint dir (loaded with the safe loader only)."""
    from safetensors.torch import load_file
    files = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
    if not files:
        raise FileNotFoundError(f"no .safetensors files under {path}")
    sd = {}
    for f in files:
        sd.update(load_file(os.path.join(path, f)))
    if "lm_head.weight" not in sd and "model.language_model.embed_tokens.weight" in sd:
        sd["lm_head.weight"] = sd["model.language_model.embed_tokens.weight"]
    return sd


class VibeVoiceForConditionalGenerationInference:
    def __init__(self, config: VibeVoiceConfig, state_dict, device="cuda", attn_implementation="hip",
                 max_batch=8, max_ctx=8192):
        self.config = config
        self.attn_implementation = attn_implementation
        self.device = torch.device(device)
        self.dtype = torch.bfloat16
        self._sd = state_dict
        self.engine = Engine(config, state_dict, self.device, max_batch=max_batch,
                             max_ctx=min(max_ctx, config.decoder_config.max_position_embeddings))
        self.ddpm_inference_steps = config.diffusion_head_config.ddpm_num_inference_steps
        self.model = _ModelView(self)

    # ------------------------------------------------------------ loading
    @classmethod
    def from_pretrained(cls, path, torch_dtype=torch.bfloat16, device_map="cuda", attn_implementation="hip",
                        synthetic_seed=0, **kw):
        """`path`: a checkpoint dir (config.json + *.safetensors), or
        "synthetic:1.5B" / "synthetic:Large" for seeded random weights at the
        real shapes (no checkpoints are reachable offline)."""
        if torch_dtype not in (torch.bfloat16, None):
            raise ValueError("the MI355X engine computes in bfloat16 (torch_dtype=torch.bfloat16)")
        dev = device_map if isinstance(device_map, str) and device_map.startswith("cuda") else "cuda"
        if str(path).startswith("synthetic:"):
            cfg = VibeVoiceConfig.builtin(str(path).split(":", 1)[1])
            sd = synthetic_state_dict(cfg, seed=synthetic_seed, device=dev)
        else:
            cfg = VibeVoiceConfig.from_json_file(os.path.join(path, "config.json"))
            sd = load_state_dict(path)
        return cls(cfg, sd, dev, attn_implementation=attn_implementation, **kw)

    def eval(self):
        return self

    def to(self, *a, **k):
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
        tokenizer = kwargs.pop("tokenizer", None)
        kwargs.pop("parsed_scripts", None)
        kwargs.pop("all_speakers_list", None)
        max_length_times = kwargs.pop("max_length_times", 2)
        refresh_negative = kwargs.get("refresh_negative", True)
        verbose = kwargs.get("verbose", False)
        forced = kwargs.get("forced_tokens", None)      # bench / test hook: fixed token schedule
        input_ids = kwargs["input_ids"] if inputs is None else inputs
        attention_mask = kwargs.get("attention_mask")
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        gen = dict(generation_config or {})
        do_sample = bool(gen.get("do_sample", False))

        dev, eng = self.device, self.engine
        B, L = input_ids.shape
        lmc = self.config.decoder_config
        max_new = kwargs.get("max_new_tokens")
        if max_new is None:
            max_new = lmc.max_position_embeddings - L                      # :371-372
        max_length = gen.get("max_length") or (L + max_new)
        Li = attention_mask.sum(-1).cpu().long()
        max_steps = min(max_length - L, int(max_length_times * L))          # :421
        per_sample_max = torch.minimum(max_length - Li, (max_length_times * Li).long())  # :422

        start_id, end_id = tokenizer.speech_start_id, tokenizer.speech_end_id
        diff_id, eos_id = tokenizer.speech_diffusion_id, tokenizer.eos_token_id
        valid = [start_id, end_id, diff_id, eos_id]                          # :405-413
        bos = getattr(tokenizer, "bos_token_id", None)
        if bos is not None:
            raise NotImplementedError("a bos id in the constrained set (Qwen tokenizers have none)")
        order = sorted(range(4), key=lambda j: valid[j])                    # argmax ties -> lowest id
        eng.set_valid_ids(valid)
        eng.set_steps(self.ddpm_inference_steps)
        need_ctx = int(Li.max()) + max_steps + 2
        if need_ctx > eng.max_ctx or B > eng.max_batch:
            raise RuntimeError(f"engine capacity (batch {eng.max_batch}, ctx {eng.max_ctx}) < request "
                               f"(batch {B}, ctx {need_ctx}); construct with larger max_batch/max_ctx")

        finished = torch.zeros(B, dtype=torch.bool)
        reach_max = torch.zeros(B, dtype=torch.bool)
        pos_len = Li.clone()
        neg_len = torch.zeros(B, dtype=torch.long)
        correct_cnt = torch.zeros(B, dtype=torch.long)                     # :393
        neg_passes = 0                                                      # negative cache length (all rows)
        audio_chunks = [[] for _ in range(B)]
        seq = [input_ids.cpu()]
        H = eng.hidden
        i32 = dict(device=dev, dtype=torch.int32)

        # ---- step 0: positive prefill rows + speculative negative [speech_start] rows
        emb = self._prompt_embeds(input_ids.to(dev), attention_mask.to(dev), speech_tensors, speech_masks,
                                  speech_input_mask)
        neg_in = eng.embed(torch.full((B,), start_id, **i32))
        ntok = emb.shape[0]
        tok_slot = torch.cat([torch.repeat_interleave(torch.arange(B), Li), torch.arange(B, 2 * B)])
        tok_pos = torch.cat([torch.cat([torch.arange(int(n)) for n in Li]), torch.zeros(B, dtype=torch.long)])
        last = torch.cumsum(Li, 0) - 1
        out_idx = torch.cat([last, torch.arange(ntok, ntok + B)])
        step_in = torch.cat([emb, neg_in], 0)
        hid, logits = eng.lm_forward(step_in, tok_slot.to(**i32), tok_pos.to(**i32), out_idx.to(**i32),
                                     max_pos=int(tok_pos.max()))
        inputs_embeds = None
        rng = range(max_steps)
        if kwargs.get("show_progress_bar", True) and verbose:
            from tqdm import tqdm
            rng = tqdm(rng, desc="Generating", leave=True, ncols=100, mininterval=0.5)
        for step in rng:
            if stop_check_fn is not None and stop_check_fn():                # :434-440
                if audio_streamer is not None:
                    audio_streamer.end()
                break
            if audio_streamer is not None and any(getattr(audio_streamer, "finished_flags", [])):
                break
            if bool(finished.all()):
                break
            if L + step >= max_length:                                      # :454-459
                reach_max[~finished] = True
                break
            if step > 0:
                slots = torch.cat([torch.arange(B), torch.arange(B, 2 * B)])
                pos = torch.cat([pos_len, neg_len])
                in2 = torch.cat([inputs_embeds, inputs_embeds], 0)          # negative consumes the same input
                hid, logits = eng.lm_forward(in2, slots.to(**i32), pos.to(**i32), torch.arange(2 * B).to(**i32),
                                             max_pos=int(pos.max()))
                pos_len += 1
            # ---- token choice (:494-509)
            if forced is not None:
                nxt = torch.tensor([forced[b][step] if step < len(forced[b]) else eos_id for b in range(B)])
            else:
                lg = logits[:B].float().cpu()
                if do_sample:
                    pr = torch.softmax(lg, -1)
                    pick = torch.multinomial(pr, 1).squeeze(1)
                else:
                    lg_sorted = lg[:, order]
                    pick = torch.tensor(order)[lg_sorted.argmax(-1)]
                nxt = torch.tensor(valid)[pick]
            nxt[finished] = eos_id
            seq.append(nxt[:, None])
            # ---- negative stream when refresh_negative is False (:512-527): run and committed every step
            if not refresh_negative:
                neg_len += 1
                neg_passes += 1
            # ---- finish bookkeeping (:530-553)
            new_eos = (nxt == eos_id) & ~finished
            if new_eos.any():
                finished |= new_eos
                if audio_streamer is not None:
                    audio_streamer.end(torch.nonzero(new_eos).reshape(-1))
            hit_max = (step >= per_sample_max) & ~finished
            if hit_max.any():
                finished |= hit_max
                reach_max |= hit_max
                if audio_streamer is not None:
                    audio_streamer.end(torch.nonzero(hit_max).reshape(-1))
            ends = torch.nonzero(nxt == end_id).reshape(-1)                # :556-560
            if ends.numel():
                eng.codec_reset(ends.to(**i32))
            starts = ~finished & (nxt == start_id)                          # :563-580
            if refresh_negative:
                neg_len[starts] = 0     # mask reset: empty context, next position 0
            next_embeds = eng.embed(nxt.to(**i32))                          # :584
            diff = ~finished & (nxt == diff_id)                             # :588
            if diff.any():
                didx = torch.nonzero(diff).reshape(-1)
                n = didx.numel()
                if refresh_negative:                                        # negative pass :591-604
                    neg_len += 1        # every row appends; rows reset above were computed speculatively
                    neg_passes += 1     # and are always dropped again below (speech_start != diffusion)
                # non-diffusion correction (:609-639): drop the entry just appended.  Where the
                # reference's KV-shift test (:628) skips the shift while the mask shift (:618)
                # happens (correct_cnt == cache_len - 2), the new entry replaces the previous one.
                skip = torch.nonzero(~finished & ~diff).reshape(-1)
                quirk = [b for b in skip.tolist()
                         if int(correct_cnt[b]) == neg_passes - 2 and int(neg_len[b]) == 2]
                neg_len[skip] -= 1
                correct_cnt[skip] += 1
                if quirk:
                    q = torch.tensor(quirk)
                    eng.kv_copy((q + B).to(**i32), torch.ones_like(q).to(**i32), torch.zeros_like(q).to(**i32))
                pos_h = hid[didx.to(dev)]
                neg_h = hid[(didx + B).to(dev)]
                noise = torch.randn(2 * n, self.config.acoustic_vae_dim)    # CPU generator (:716)
                x = noise[:n].to(device=dev, dtype=self.dtype).contiguous()
                eng.diffusion_sample(pos_h.contiguous(), neg_h.contiguous(), x, cfg_scale)
                audio = torch.empty(n, eng.hop, dtype=self.dtype, device=dev)
                d32 = didx.to(**i32)
                eng.codec_step(d32, x, audio, embeds_out=next_embeds, embed_rows=d32)
                for i, b in enumerate(didx.tolist()):
                    audio_chunks[b].append(audio[i:i + 1])
                if audio_streamer is not None:
                    audio_streamer.put(audio[:, None, :], didx)
            inputs_embeds = next_embeds
        if audio_streamer is not None:
            audio_streamer.end()
        outs = [torch.cat(c, dim=-1) if c else None for c in audio_chunks]
        return VibeVoiceGenerationOutput(sequences=torch.cat(seq, dim=1), speech_outputs=outs if return_speech else None,
                                         reach_max_step_sample=reach_max)
