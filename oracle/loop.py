"""The generate loop (oracle), following the reference's control flow line by
line: vibevoice/modular/modeling_vibevoice_inference.py:327-710.

Unlike the product (vibevoice_amd/modeling_vibevoice_inference.py), the
negative CFG stream is kept exactly as the reference keeps it — a growing
cache plus an attention mask that is reset (:563-580) and shifted
(:609-639) in place, including the reference's KV-shift boundary condition
(:628 vs :618) — so a test comparing the two checks the product's compacted
bookkeeping against the reference's literal semantics.

Pinned by golden G8 (tests/golden/make_golden.py:g8_loop): the reference's
own generate() run end to end in fp32; tests/test_oracle_golden.py.

Supported: text prompts with or without voice prompts, refresh_negative True/False,
greedy choice among the valid ids, or a forced token schedule.
"""
import torch
import torch.nn.functional as F

from . import codec, head, lm


def _sub(sd, prefix):
    return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}


def connector(sd, p, x):
    """SpeechConnector (modeling_vibevoice.py:58-69)."""
    y = F.linear(x, sd[p + "fc1.weight"], sd[p + "fc1.bias"])
    y = lm.rms(y, sd[p + "norm.weight"], 1e-6)
    return F.linear(y, sd[p + "fc2.weight"], sd[p + "fc2.bias"])


def voice_embeds(sd, cfg, speech_tensors, speech_masks, dtype, voice_noise=None):
    """Voice-prompt prefill, `_process_speech_inputs(..., "audio")`
    (modeling_vibevoice_inference.py:150-163): non-streaming acoustic encode,
    sample(dist_type="gaussian") on the global RNG (modular_vibevoice_tokenizer.py:
    979-987: one randn per clip scaled by fix_std / 0.8, then randn_like(mean)),
    (z + bias) * scale, acoustic connector, rows of the valid frames.
    voice_noise = (per-clip draw [Nv], randn_like(mean)) replays the two draws
    of another generator (the GPU run draws them on the device, as the
    reference does there)."""
    asd = _sub(sd, "model.acoustic_tokenizer.")
    ed = codec.codec_dims(cfg.acoustic_tokenizer_config, "encoder")
    dev = sd["model.speech_scaling_factor"].device
    mean = codec.encode(asd, ed, speech_tensors.to(device=dev, dtype=dtype).unsqueeze(1), None, None, streaming=False)
    value = cfg.acoustic_tokenizer_config.fix_std / 0.8
    if voice_noise is None:
        std = torch.randn(mean.shape[0], dtype=mean.dtype).to(mean.device) * value
        eps = torch.randn_like(mean.cpu()).to(mean.device)              # randn_like keeps mean's (permuted) strides
    else:
        std = voice_noise[0].to(device=mean.device, dtype=mean.dtype) * value
        eps = voice_noise[1].to(device=mean.device, dtype=mean.dtype).reshape(mean.shape)
    z = mean + std[:, None, None] * eps
    feats = (z + sd["model.speech_bias_factor"]) * sd["model.speech_scaling_factor"]
    return connector(sd, "model.acoustic_connector.", feats)[speech_masks]


class _NegRow:
    """Cache + mask of one sample's negative stream (reference representation)."""

    def __init__(self, n_layers):
        self.kv = lm.RowKV(n_layers)
        self.mask = [1]            # attention_mask ones((B, 1)) (:380)


def generate(sd, cfg, input_ids, attention_mask, tokenizer_ids, ddpm_steps=10, cfg_scale=1.3,
             forced=None, refresh_negative=True, max_length_times=2, max_new_tokens=None, dtype=torch.bfloat16,
             record=None, speech_tensors=None, speech_masks=None, speech_input_mask=None, voice_noise=None,
             do_sample=False, sample_q=None, teacher=None):
    """Returns (sequences [B, L+steps], audio list per sample, reach_max [B]).

    sd: full state dict (reference names) in `dtype`.  cfg: VibeVoiceConfig.
    tokenizer_ids: dict(start, end, diffusion, eos).
    record: dict filled per loop step (the teacher-forcing trace the GPU
    parity tests replay): "prompt_embeds" (the un-padded prompt rows, voice
    spliced in, row-major over samples), per step "logits" [B, 4 valid],
    "hpos" [B, H], "hneg" [B, H] (None when no negative pass ran), "didx",
    "noise", "latents" [n, D], "audio" [n, 1, hop], "next_embeds" [B, H]
    (the next step's input).
    do_sample: `torch.multinomial(softmax(scores), 1)` over the constrained
    full-vocabulary fp32 scores (:496-505) on the global CPU generator, as the
    reference's CPU run draws it.  sample_q(step) -> [B, 4] replays another
    generator's Exp(1) draws at the 4 valid ids (sorted by id) instead: ATen's
    one-sample multinomial is argmax(p / q) over a [B, vocab] Exp(1) draw.
    teacher: another run's `record` — its prompt embeddings, per-step next
    inputs and latents replace this run's own (teacher forcing), so each step
    of this run sees exactly that run's inputs (per-step precision studies).
    """
    lmc = dict(cfg.decoder_config)
    lsd = _sub(sd, "model.language_model.")
    hsd = _sub(sd, "model.prediction_head.")
    asd = _sub(sd, "model.acoustic_tokenizer.")
    ssd = _sub(sd, "model.semantic_tokenizer.")
    nl = lmc["num_hidden_layers"]
    dd = codec.codec_dims(cfg.acoustic_tokenizer_config, "decoder")
    ed = codec.codec_dims(cfg.semantic_tokenizer_config, "encoder")
    start, end, diff, eos = (tokenizer_ids[k] for k in ("start", "end", "diffusion", "eos"))
    valid = sorted([start, end, diff, eos])
    emb_w = lsd["embed_tokens.weight"]
    dev = emb_w.device        # the oracle runs where its weights are (a GPU only as a test's checker)
    lm_head = sd.get("lm_head.weight", emb_w)
    scale, bias = sd["model.speech_scaling_factor"], sd["model.speech_bias_factor"]

    B, L = input_ids.shape
    Li = attention_mask.sum(-1).long()
    if max_new_tokens is None:
        max_new_tokens = lmc["max_position_embeddings"] - L           # :371-372
    max_length = L + max_new_tokens
    max_steps = min(max_length - L, int(max_length_times * L))       # :421
    per_max = torch.minimum(max_length - Li, (max_length_times * Li).long())
    finished = torch.zeros(B, dtype=torch.bool)
    reach = torch.zeros(B, dtype=torch.bool)
    correct_cnt = torch.zeros(B, dtype=torch.long)
    seqs = input_ids.clone()
    audio = [[] for _ in range(B)]
    a_state, s_state = codec.StreamState(B), codec.StreamState(B)
    pos_kv = [lm.RowKV(nl) for _ in range(B)]
    neg = [_NegRow(nl) for _ in range(B)]
    neg_started = False
    inputs_embeds = None
    dstep = 0                                                         # diffusion steps so far

    def logits_of(hrow):
        return (hrow @ lm_head.t()).float()                          # bf16 Linear then .float() (:494-498)

    for step in range(max_steps):
        if bool(finished.all()):
            break
        if seqs.shape[1] >= max_length:
            reach[~finished] = True
            break
        # ---- positive pass (:467-486)
        if step == 0:
            emb0 = emb_w[input_ids]
            if speech_tensors is not None and speech_masks is not None:       # forward :221-225
                emb0 = emb0.clone()
                v = voice_embeds(sd, cfg, speech_tensors, speech_masks, dtype, voice_noise)
                if speech_input_mask is not None:
                    emb0[speech_input_mask] = v.to(emb0.dtype)
            hs = []
            if teacher is not None:
                emb0 = emb0.clone()
                emb0[attention_mask.bool()] = teacher["prompt_embeds"].to(device=dev, dtype=emb0.dtype)
            if record is not None:
                record["prompt_embeds"] = emb0[attention_mask.bool()].clone()
            for b in range(B):
                keep = attention_mask[b].bool()
                x = emb0[b][keep][None]
                hs.append(lm.forward_rows(lsd, lmc, x, pos_kv[b:b + 1])[0, -1])
            hpos = torch.stack(hs)
        else:
            hpos = lm.forward_rows(lsd, lmc, inputs_embeds[:, None], pos_kv)[:, -1]
        lg = logits_of(hpos)
        if record is not None:
            record.setdefault("logits", []).append(lg[:, valid].clone())
            record.setdefault("hpos", []).append(hpos.clone())
        if forced is not None:
            nxt = torch.tensor([forced[b][step] if step < len(forced[b]) else eos for b in range(B)])
        elif do_sample:
            scores = torch.full_like(lg, float("-inf"))               # VibeVoiceTokenConstraintProcessor (:54-67)
            scores[:, valid] = lg[:, valid]
            if sample_q is None:
                nxt = torch.multinomial(F.softmax(scores, dim=-1), num_samples=1).squeeze(1)
            else:
                p = F.softmax(scores[:, valid], dim=-1)
                nxt = torch.tensor(valid)[(p / sample_q(step).to(p.device)).argmax(-1).cpu()]
        else:
            sub = lg[:, valid]
            nxt = torch.tensor(valid)[sub.argmax(-1).cpu()]
        nxt[finished] = eos                                           # :509
        seqs = torch.cat([seqs, nxt[:, None]], dim=1)

        def negative_pass():
            nonlocal neg_started
            x = inputs_embeds if inputs_embeds is not None else emb_w[torch.full((B,), start)]
            masks = [torch.tensor(neg[b].mask, dtype=torch.bool) for b in range(B)]
            hn = lm.forward_rows_masked(lsd, lmc, x[:, None], [neg[b].kv for b in range(B)], masks)[:, -1]
            for b in range(B):
                neg[b].mask.append(1)                                 # _update_model_kwargs_for_generation
            neg_started = True
            return hn

        hneg = None
        if not refresh_negative:                                      # :512-527
            hneg = negative_pass()
        new_eos = (nxt == eos) & ~finished                            # :530-541
        finished |= new_eos
        hit = (step >= per_max) & ~finished                           # :544-553
        finished |= hit
        reach |= hit
        ends = torch.nonzero(nxt == end).reshape(-1)                  # :556-560
        if ends.numel():
            a_state.zero(ends)
            s_state.zero(ends)
        starts = torch.arange(B)[~finished & (nxt == start)]          # :563-580
        if starts.numel() and refresh_negative:
            for b in starts.tolist():
                neg[b].mask = [0] * len(neg[b].mask)
                neg[b].mask[-1] = 1
        next_embeds = emb_w[nxt].clone()                              # :584
        didx = torch.arange(B)[~finished & (nxt == diff)]             # :588
        if didx.numel():
            if refresh_negative:
                hneg = negative_pass()                                # :591-604
            nd = torch.arange(B)[~finished & (nxt != diff)]           # :609-639
            for b in nd.tolist():
                c = int(correct_cnt[b])
                msk = neg[b].mask
                seq_len = len(msk)
                if c + 1 < seq_len - 1:
                    msk[c + 1:] = msk[c:-1]
                msk[c] = 0
                kvlen = neg[b].kv.length()
                if c + 1 < kvlen - 1:
                    for li in range(nl):
                        for t in (neg[b].kv.k, neg[b].kv.v):
                            t[li] = torch.cat([t[li][:, :c + 1], t[li][:, c:-1]], dim=1)
            correct_cnt[nd] += 1
            n = didx.numel()
            noise = torch.randn(2 * n, cfg.acoustic_vae_dim).to(device=dev, dtype=dtype)  # :716
            if record is not None:
                record.setdefault("noise", []).append(noise.clone())
            lat = head.sample_speech_tokens(hsd, hpos[didx], hneg[didx], noise, ddpm_steps, cfg_scale,
                                            cfg.diffusion_head_config.head_layers,
                                            cfg.diffusion_head_config.rms_norm_eps)
            own_lat = lat
            if teacher is not None:
                lat = teacher["latents"][dstep].to(device=dev, dtype=lat.dtype)
            dstep += 1
            z = (lat / scale - bias).unsqueeze(-1)                    # :651
            a = codec.decode(asd, dd, z, a_state, didx)
            for i, b in enumerate(didx.tolist()):
                audio[b].append(a[i])
            sem = codec.encode(ssd, ed, a, s_state, didx)[:, 0]
            next_embeds[didx] = connector(sd, "model.acoustic_connector.", lat) + \
                connector(sd, "model.semantic_connector.", sem)
            if record is not None:
                record.setdefault("latents", []).append(own_lat.clone())
                record.setdefault("audio", []).append(a.clone())
        if record is not None:
            record.setdefault("hneg", []).append(None if hneg is None else hneg.clone())
            record.setdefault("didx", []).append(didx.clone())
            record.setdefault("next_embeds", []).append(next_embeds.clone())
        if teacher is not None:
            next_embeds = teacher["next_embeds"][step].to(device=dev, dtype=next_embeds.dtype)
        inputs_embeds = next_embeds
    outs = [torch.cat(c, dim=-1) if c else None for c in audio]
    return seqs, outs, reach
