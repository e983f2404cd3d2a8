"""Synthetic processor outputs for offline benches and tests.

No Qwen tokenizer files or voice recordings are reachable offline, so this
module builds what `VibeVoiceProcessor.__call__` would return
(vibevoice/processor/vibevoice_processor.py:163-244) with the reference's
prompt layout (:246-304, voice prompt :420-450) and seeded random text ids:

  system prompt | " Voice input:\\n" | per speaker: " Speaker k:" speech_start
  diffusion x ceil(len/3200) speech_end "\\n" | " Text input:\\n" |
  per line " Speaker k: <text>\\n" | " Speech output:\\n" speech_start

Batches are left-padded with pad_id (:351-353).  Voice prompts are seeded white
noise normalised to -25 dBFS (vibevoice_tokenizer_processor.py:19-87).
"""
import math
import types

import torch

# Qwen2.5 vocabulary ids of the special tokens the loop uses
# (modular_vibevoice_text_tokenizer.py:163-183)
EOS, SPEECH_START, SPEECH_END, SPEECH_DIFFUSION, PAD = 151643, 151652, 151653, 151654, 151655

# token counts of the fixed prompt pieces under the Qwen2.5 BPE
SYSTEM_TOKENS = 25
SECTION_TOKENS = 4      # " Voice input:\n", " Text input:\n", " Speech output:\n"
SPEAKER_PREFIX = 4      # " Speaker k:"


def tokenizer_ids():
    """Stand-in for `processor.tokenizer`: only the ids the loop reads."""
    return types.SimpleNamespace(speech_start_id=SPEECH_START, speech_end_id=SPEECH_END,
                                 speech_diffusion_id=SPEECH_DIFFUSION, eos_token_id=EOS, bos_token_id=None,
                                 pad_token_id=PAD, pad_id=PAD)


def _text(g, n):
    return torch.randint(0, EOS, (n,), generator=g).tolist()


def _voice(g, seconds, sr=24000, dbfs=-25.0):
    wav = torch.randn(int(seconds * sr), generator=g)
    target = 10 ** (dbfs / 20)
    return wav * (target / wav.pow(2).mean().sqrt())


def synthetic_inputs(batch=1, speakers=1, voice_seconds=3.0, text_tokens=64, seed=0, hop=3200, text_jitter=0):
    """Processor-shaped dict: input_ids, attention_mask, speech_input_mask,
    speech_tensors, speech_masks (voice_seconds=0 -> no voice prompt).
    voice_seconds may be a list (cycled over the voices: ragged clips, zero-
    padded in speech_tensors as the processor pads them); text_jitter adds
    0..text_jitter random tokens per script line (ragged, left-padded rows)."""
    g = torch.Generator().manual_seed(seed)
    rows, masks, voices = [], [], []
    secs = list(voice_seconds) if isinstance(voice_seconds, (list, tuple)) else [voice_seconds]
    has_voice = any(v > 0 for v in secs)
    for _ in range(batch):
        ids = _text(g, SYSTEM_TOKENS)
        sim = [False] * len(ids)
        if has_voice:
            ids += _text(g, SECTION_TOKENS)
            sim += [False] * SECTION_TOKENS
            for _ in range(speakers):
                wav = _voice(g, secs[len(voices) % len(secs)])
                frames = math.ceil(wav.numel() / hop)
                piece = _text(g, SPEAKER_PREFIX) + [SPEECH_START] + [SPEECH_DIFFUSION] * frames + [SPEECH_END] + \
                    _text(g, 1)
                ids += piece
                sim += [False] * (SPEAKER_PREFIX + 1) + [True] * frames + [False, False]
                voices.append(wav)
        ids += _text(g, SECTION_TOKENS)
        sim += [False] * SECTION_TOKENS
        per = max(1, text_tokens // speakers)
        for _ in range(speakers):
            extra = int(torch.randint(0, text_jitter + 1, (1,), generator=g)) if text_jitter else 0
            line = _text(g, SPEAKER_PREFIX + per + extra + 1)
            ids += line
            sim += [False] * len(line)
        ids += _text(g, SECTION_TOKENS) + [SPEECH_START]
        sim += [False] * (SECTION_TOKENS + 1)
        rows.append(ids)
        masks.append(sim)
    L = max(len(r) for r in rows)
    input_ids = torch.full((batch, L), PAD, dtype=torch.long)
    attention_mask = torch.zeros(batch, L, dtype=torch.long)
    speech_input_mask = torch.zeros(batch, L, dtype=torch.bool)
    for b, (r, m) in enumerate(zip(rows, masks)):
        input_ids[b, L - len(r):] = torch.tensor(r)
        attention_mask[b, L - len(r):] = 1
        speech_input_mask[b, L - len(r):] = torch.tensor(m)
    out = dict(input_ids=input_ids, attention_mask=attention_mask, speech_input_mask=speech_input_mask)
    if voices:
        T = max(v.numel() for v in voices)
        frames = math.ceil(T / hop)
        st = torch.zeros(len(voices), T, dtype=torch.float32)
        sm = torch.zeros(len(voices), frames, dtype=torch.bool)
        for i, v in enumerate(voices):
            st[i, :v.numel()] = v
            sm[i, :math.ceil(v.numel() / hop)] = True
        out.update(speech_tensors=st, speech_masks=sm)
    else:
        out.update(speech_tensors=None, speech_masks=None)
    return out
