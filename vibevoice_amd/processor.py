"""Processor side of the drop-in surface (SURVEY.md §8b "Processor side", §8f
rank 3): script + voice prompts -> the BatchEncoding generate() consumes.

Same classes, arguments and outputs as the reference:
  * `VibeVoiceProcessor`          vibevoice/processor/vibevoice_processor.py:17-688
  * `VibeVoiceTokenizerProcessor` + `AudioNormalizer`
                                  vibevoice/processor/vibevoice_tokenizer_processor.py:19-480
  * `VibeVoiceTextTokenizerFast`  vibevoice/modular/modular_vibevoice_text_tokenizer.py:112-208

Host-side, offline-first re-implementation:
  * the text tokenizer is any local Qwen2-style byte-level BPE (`tokenizer.json`,
    read by the `tokenizers` backend through transformers); the reference's
    remote default "Qwen/Qwen2.5-1.5B" resolves only from a local path or the
    local HF cache (no network here);
  * audio I/O uses scipy (WAV read + polyphase resampling to 24 kHz, float32
    WAV write) instead of librosa / soundfile, which this image lacks;
  * `.pt` voice tensors load with `weights_only=True`.
Prompt layout (system prompt, voice section, text section, speech-output
section), left padding with `pad_id`, speech masks and the speaker-id
normalisation are the reference's; pinned by tests/golden/g9_processor.npz
(made by running the reference's processor, tests/golden/make_golden.py).
"""
from __future__ import annotations

import json
import math
import os
import re
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

SYSTEM_PROMPT = (" Transform the text provided by various speakers into speech output, utilizing the distinct voice "
                 "of each respective speaker.\n")
_SPEAKER_LINE = re.compile(r"^Speaker\s+(\d+)\s*:\s*(.*)$", re.IGNORECASE)


# ---------------------------------------------------------------------- audio
class AudioNormalizer:
    """RMS to target dBFS, then scale down if any sample would clip
    (vibevoice_tokenizer_processor.py:19-88)."""

    def __init__(self, target_dB_FS: float = -25, eps: float = 1e-6):
        self.target_dB_FS = target_dB_FS
        self.eps = eps

    def tailor_dB_FS(self, audio: np.ndarray):
        rms = np.sqrt(np.mean(audio ** 2))
        scalar = 10 ** (self.target_dB_FS / 20) / (rms + self.eps)
        return audio * scalar, rms, scalar

    def avoid_clipping(self, audio: np.ndarray, scalar: Optional[float] = None):
        if scalar is None:
            peak = np.max(np.abs(audio))
            scalar = peak + self.eps if peak > 1.0 else 1.0
        return audio / scalar, scalar

    def __call__(self, audio: np.ndarray) -> np.ndarray:
        audio, _, _ = self.tailor_dB_FS(audio)
        audio, _ = self.avoid_clipping(audio)
        return audio


def _read_wav(path: str, target_sr: int) -> np.ndarray:
    """Mono float32 at target_sr (the reference uses librosa.load(sr=, mono=True))."""
    from scipy.io import wavfile
    from scipy.signal import resample_poly
    sr, data = wavfile.read(path)
    if np.issubdtype(data.dtype, np.integer):
        info = np.iinfo(data.dtype)
        if info.min == 0:                                 # unsigned 8-bit PCM
            data = (data.astype(np.float32) - 128.0) / 128.0
        else:
            data = data.astype(np.float32) / float(-info.min)
    data = data.astype(np.float32)
    if data.ndim == 2:
        data = data.mean(axis=1)
    if sr != target_sr:
        g = math.gcd(int(sr), int(target_sr))
        data = resample_poly(data, target_sr // g, sr // g).astype(np.float32)
    return data


class VibeVoiceTokenizerProcessor:
    """Audio side of the processor: mono, optional dBFS normalisation, file I/O
    (vibevoice_tokenizer_processor.py:91-480)."""

    model_input_names = ["input_features"]

    def __init__(self, sampling_rate: int = 24000, normalize_audio: bool = True, target_dB_FS: float = -25,
                 eps: float = 1e-6, **kwargs):
        self.sampling_rate = sampling_rate
        self.normalize_audio = normalize_audio
        self.target_dB_FS = target_dB_FS
        self.eps = eps
        self.normalizer = AudioNormalizer(target_dB_FS, eps) if normalize_audio else None
        self.feature_extractor_dict = dict(sampling_rate=sampling_rate, normalize_audio=normalize_audio,
                                           target_dB_FS=target_dB_FS, eps=eps)

    def to_dict(self) -> Dict[str, Any]:
        return self.feature_extractor_dict

    @staticmethod
    def _ensure_mono(audio: np.ndarray) -> np.ndarray:
        if audio.ndim == 1:
            return audio
        if audio.ndim != 2:
            raise ValueError(f"Audio should be 1D or 2D, got shape: {audio.shape}")
        if audio.shape[0] == 2:
            return audio.mean(axis=0)
        if audio.shape[1] == 2:
            return audio.mean(axis=1)
        if 1 in audio.shape:
            return audio.reshape(-1)
        raise ValueError(f"Unexpected audio shape: {audio.shape}")

    def _process_single_audio(self, audio) -> np.ndarray:
        audio = self._ensure_mono(np.asarray(audio, dtype=np.float32))
        if self.normalize_audio and self.normalizer is not None:
            audio = self.normalizer(audio)
        return audio

    def _load_audio_from_path(self, audio_path: str) -> np.ndarray:
        ext = os.path.splitext(audio_path)[1].lower()
        if ext == ".wav":
            return _read_wav(audio_path, self.sampling_rate)
        if ext == ".npy":
            return np.load(audio_path).astype(np.float32)
        if ext == ".pt":
            t = torch.load(audio_path, map_location="cpu", weights_only=True)
            return (t.squeeze().numpy() if torch.is_tensor(t) else np.asarray(t)).astype(np.float32)
        if ext in (".mp3", ".flac", ".m4a", ".ogg"):
            raise ValueError(f"{ext} needs a decoder this image does not ship; convert to .wav (or .npy)")
        raise ValueError(f"Unsupported file format: {ext}. Supported formats: .wav, .pt, .npy")

    def __call__(self, audio=None, sampling_rate: Optional[int] = None, return_tensors: Optional[str] = None,
                 **kwargs):
        """{"audio": ...}: [B, 1, T] for return_tensors "pt" / "np", else the
        array or list (vibevoice_tokenizer_processor.py:188-269)."""
        if audio is None:
            raise ValueError("Audio input is required")
        if isinstance(audio, str):
            items = [self._load_audio_from_path(audio)]
        elif isinstance(audio, list):
            if not audio:
                raise ValueError("Empty audio list provided")
            if all(isinstance(a, str) for a in audio):
                items = [self._load_audio_from_path(p) for p in audio]
            elif isinstance(audio[0], (np.ndarray, list)):
                items = list(audio)
            else:
                items = [audio]
        else:
            items = [audio]
        out = [self._process_single_audio(a) for a in items]
        if return_tensors == "pt":
            feats = torch.stack([torch.from_numpy(a) for a in out]).unsqueeze(1)
        elif return_tensors == "np":
            feats = np.stack(out)[:, np.newaxis, :]
        else:
            feats = out[0] if len(out) == 1 else out
        return {"audio": feats}

    def preprocess_audio(self, audio_path_or_array, normalize: Optional[bool] = None) -> np.ndarray:
        a = (self._load_audio_from_path(audio_path_or_array) if isinstance(audio_path_or_array, str)
             else np.asarray(audio_path_or_array, dtype=np.float32))
        keep = self.normalize_audio
        if normalize is not None:
            self.normalize_audio = normalize
        try:
            return self._process_single_audio(a)
        finally:
            self.normalize_audio = keep

    @staticmethod
    def _prepare_audio_for_save(audio: np.ndarray, normalize: bool) -> np.ndarray:
        if audio.ndim > 1 and audio.shape[0] == 1:
            audio = audio[0]
        if normalize:
            peak = np.abs(audio).max()
            if peak > 0:
                audio = audio / peak
        return audio

    def save_audio(self, audio, output_path: str = "output.wav", sampling_rate: Optional[int] = None,
                   normalize: bool = False, batch_prefix: str = "audio_") -> List[str]:
        """float32 WAV file(s); a list or a batch > 1 is written as
        <output_path>/<batch_prefix><i>.wav (vibevoice_tokenizer_processor.py:352-457)."""
        from scipy.io import wavfile
        sr = sampling_rate or self.sampling_rate

        def host(a):
            return a.float().detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)

        def write(path, a):
            wavfile.write(path, sr, np.ascontiguousarray(self._prepare_audio_for_save(a, normalize),
                                                         dtype=np.float32))
            return path

        if isinstance(audio, list):
            os.makedirs(output_path, exist_ok=True)
            return [write(os.path.join(output_path, f"{batch_prefix}{i}.wav"), host(a)) for i, a in enumerate(audio)]
        if not (torch.is_tensor(audio) or isinstance(audio, np.ndarray)):
            raise ValueError(f"Unsupported audio type: {type(audio)}")
        a = host(audio)
        if a.ndim >= 3 and a.shape[0] > 1:
            os.makedirs(output_path, exist_ok=True)
            return [write(os.path.join(output_path, f"{batch_prefix}{i}.wav"), a[i]) for i in range(a.shape[0])]
        if a.ndim >= 3:
            a = a.squeeze()
        return [write(output_path, a)]


# ---------------------------------------------------------------------- text
class VibeVoiceTextTokenizerFast:
    """Qwen2 byte-level BPE plus the speech control tokens
    (modular_vibevoice_text_tokenizer.py:112-208): speech start / end / diffusion
    reuse <|vision_start|> / <|vision_end|> / <|vision_pad|>, padding uses
    <|image_pad|>, eos = <|endoftext|>; there is no bos."""

    model_input_names = ["input_ids", "attention_mask"]
    SPEECH_TOKENS = ("<|vision_start|>", "<|vision_end|>", "<|vision_pad|>")

    def __init__(self, backend):
        self._tok = backend
        self._tok.add_special_tokens({"additional_special_tokens": list(self.SPEECH_TOKENS)})
        ids = self._tok.convert_tokens_to_ids
        self._speech_start_id, self._speech_end_id, self._speech_diffusion_id = (ids(t) for t in self.SPEECH_TOKENS)
        self._eos_id = self._tok.eos_token_id
        self._pad_id = ids("<|image_pad|>")
        if self._eos_id is None or "<|image_pad|>" not in self._tok.get_vocab():
            raise ValueError("tokenizer lacks <|endoftext|> / <|image_pad|> (not a Qwen2-style vocabulary)")

    @classmethod
    def from_pretrained(cls, name_or_path, **kwargs):
        from transformers import AutoTokenizer
        kwargs.setdefault("eos_token", "<|endoftext|>")
        kwargs.setdefault("pad_token", "<|endoftext|>")
        kwargs.setdefault("unk_token", "<|endoftext|>")
        try:
            backend = AutoTokenizer.from_pretrained(name_or_path, local_files_only=True, **kwargs)
        except Exception as e:   # a hub name without a local copy: this deployment has no network
            raise OSError(f"text tokenizer {name_or_path!r} not found locally (a directory with tokenizer.json, "
                          f"or the local HF cache); point language_model_pretrained_name in "
                          f"preprocessor_config.json at a local path") from e
        return cls(backend)

    eos_id = property(lambda self: self._eos_id)
    eos_token_id = property(lambda self: self._eos_id)
    bos_token_id = property(lambda self: None)
    pad_token_id = property(lambda self: self._tok.pad_token_id)
    speech_start_id = property(lambda self: self._speech_start_id)
    speech_end_id = property(lambda self: self._speech_end_id)
    speech_diffusion_id = property(lambda self: self._speech_diffusion_id)
    pad_id = property(lambda self: self._pad_id)

    def encode(self, text, add_special_tokens: bool = True, **kw) -> List[int]:
        return self._tok.encode(text, add_special_tokens=add_special_tokens, **kw)

    def decode(self, *a, **kw):
        return self._tok.decode(*a, **kw)

    def batch_decode(self, *a, **kw):
        return self._tok.batch_decode(*a, **kw)

    def convert_tokens_to_ids(self, t):
        return self._tok.convert_tokens_to_ids(t)

    def __len__(self):
        return len(self._tok)

    def save_pretrained(self, path, **kw):
        return self._tok.save_pretrained(path, **kw)


# ---------------------------------------------------------------------- processor
class VibeVoiceProcessor:
    """Podcast script (+ one voice prompt per speaker) -> generate() inputs
    (vibevoice_processor.py:17-688)."""

    def __init__(self, tokenizer=None, audio_processor=None, speech_tok_compress_ratio: int = 3200,
                 db_normalize: bool = True, **kwargs):
        self.tokenizer = tokenizer
        self.audio_processor = audio_processor or VibeVoiceTokenizerProcessor()
        self.speech_tok_compress_ratio = speech_tok_compress_ratio
        self.db_normalize = db_normalize
        self.audio_normalizer = AudioNormalizer() if db_normalize else None
        self.system_prompt = SYSTEM_PROMPT

    # -------------------------------------------------------------- config I/O
    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, **kwargs):
        """Reads <path>/preprocessor_config.json (defaults when absent, as the
        reference falls back, :84-90) and the text tokenizer it names
        (`language_model_pretrained_name`, default "Qwen/Qwen2.5-1.5B"; a
        relative directory resolves against the model directory, and a
        tokenizer.json inside the model directory is used when the named one is
        not a local directory)."""
        path = str(pretrained_model_name_or_path)
        cfg_path = os.path.join(path, "preprocessor_config.json")
        config = {"speech_tok_compress_ratio": 3200, "db_normalize": True}
        if os.path.exists(cfg_path):
            with open(cfg_path) as f:
                config = json.load(f)
        name = config.get("language_model_pretrained_name") or kwargs.pop("language_model_pretrained_name",
                                                                          "Qwen/Qwen2.5-1.5B")
        if not os.path.isabs(name) and os.path.isdir(os.path.join(path, name)):
            name = os.path.join(path, name)
        elif not os.path.isdir(name) and os.path.exists(os.path.join(path, "tokenizer.json")):
            name = path
        if "qwen" not in name.lower() and not os.path.exists(os.path.join(name, "tokenizer.json")):
            raise ValueError(f"Unsupported tokenizer type for {name}. Supported types: Qwen.")
        tokenizer = VibeVoiceTextTokenizerFast.from_pretrained(name, **kwargs)
        ac = config.get("audio_processor", {})
        audio_processor = VibeVoiceTokenizerProcessor(sampling_rate=ac.get("sampling_rate", 24000),
                                                      normalize_audio=ac.get("normalize_audio", True),
                                                      target_dB_FS=ac.get("target_dB_FS", -25),
                                                      eps=ac.get("eps", 1e-6))
        return cls(tokenizer=tokenizer, audio_processor=audio_processor,
                   speech_tok_compress_ratio=config.get("speech_tok_compress_ratio", 3200),
                   db_normalize=config.get("db_normalize", True))

    def save_pretrained(self, save_directory, **kwargs):
        os.makedirs(save_directory, exist_ok=True)
        ap = self.audio_processor
        cfg = {
            "processor_class": "VibeVoiceProcessor",
            "speech_tok_compress_ratio": self.speech_tok_compress_ratio,
            "db_normalize": self.db_normalize,
            "audio_processor": {"feature_extractor_type": "VibeVoiceTokenizerProcessor",
                                "sampling_rate": getattr(ap, "sampling_rate", 24000),
                                "normalize_audio": getattr(ap, "normalize_audio", True),
                                "target_dB_FS": getattr(ap, "target_dB_FS", -25),
                                "eps": getattr(ap, "eps", 1e-6)},
        }
        with open(os.path.join(save_directory, "preprocessor_config.json"), "w") as f:
            json.dump(cfg, f, indent=2)

    # -------------------------------------------------------------- scripts
    @staticmethod
    def _convert_json_to_script(json_file: str) -> str:
        with open(json_file, encoding="utf-8") as f:
            data = json.load(f)
        if not isinstance(data, list):
            raise ValueError("JSON file must contain a list of speaker entries")
        lines = []
        for item in data:
            if not isinstance(item, dict) or item.get("speaker") is None or item.get("text") is None:
                continue
            try:
                sid = int(item["speaker"])
            except (TypeError, ValueError):
                continue
            text = item["text"].strip()
            if text:
                lines.append(f"Speaker {sid}: {text}")
        if not lines:
            raise ValueError("No valid entries found in JSON file")
        return "\n".join(lines)

    @staticmethod
    def _convert_text_to_script(text_file: str) -> str:
        with open(text_file, encoding="utf-8") as f:
            raw = f.readlines()
        lines = []
        for line in raw:
            line = line.strip()
            if not line:
                continue
            m = _SPEAKER_LINE.match(line)
            if m is None:
                lines.append(f"Speaker 1: {line}")        # plain text: the first speaker
            elif m.group(2).strip():
                lines.append(f"Speaker {int(m.group(1))}: {m.group(2).strip()}")
        if not lines:
            raise ValueError("No valid content found in text file")
        return "\n".join(lines)

    @staticmethod
    def _parse_script(script: str) -> List[Tuple[int, str]]:
        """[(speaker_id, " text")]; ids shift to start at 0 when all are >= 1."""
        parsed = []
        for line in script.strip().split("\n"):
            if not line.strip():
                continue
            m = _SPEAKER_LINE.match(line.strip())
            if m is not None:
                parsed.append((int(m.group(1)), " " + m.group(2).strip()))
        if not parsed:
            raise ValueError("No valid speaker lines found in script")
        if min(s for s, _ in parsed) > 0:
            parsed = [(s - 1, t) for s, t in parsed]
        return parsed

    def _enc(self, text: str) -> List[int]:
        return self.tokenizer.encode(text, add_special_tokens=False)

    def _create_voice_prompt(self, speaker_samples):
        """' Voice input:\\n', then per speaker ' Speaker i:' <start>
        <diffusion> x ceil(len / 3200) <end> '\\n' (the diffusion slots take the
        voice latents: speech mask True)."""
        tk = self.tokenizer
        tokens = self._enc(" Voice input:\n")
        mask = [False] * len(tokens)
        wavs = []
        for i, sample in enumerate(speaker_samples):
            prefix = self._enc(f" Speaker {i}:")
            wav = (self.audio_processor._load_audio_from_path(sample) if isinstance(sample, str)
                   else np.array(sample, dtype=np.float32))
            if self.db_normalize and self.audio_normalizer is not None:
                wav = self.audio_normalizer(wav)
            n = math.ceil(wav.shape[0] / self.speech_tok_compress_ratio)
            nl = self._enc("\n")
            tokens += prefix + [tk.speech_start_id] + [tk.speech_diffusion_id] * n + [tk.speech_end_id] + nl
            mask += [False] * (len(prefix) + 1) + [True] * n + [False] * (1 + len(nl))
            wavs.append(wav)
        return tokens, wavs, mask

    def _process_single(self, text, voice_samples=None) -> Dict[str, Any]:
        if not isinstance(text, str):
            raise ValueError(f"Could not process input text: {text}")
        if text.endswith(".json") and os.path.exists(text):
            script = self._convert_json_to_script(text)
        elif text.endswith(".txt") and os.path.exists(text):
            script = self._convert_text_to_script(text)
        else:
            script = text
        parsed = self._parse_script(script)
        speakers = list(set(s for s, _ in parsed))
        system = self.tokenizer.encode(self.system_prompt)
        if voice_samples:
            vt, vw, vm = self._create_voice_prompt(voice_samples[:len(speakers)])
        else:
            vt, vw, vm = [], [], []
        ids = system + vt
        mask = [False] * len(system) + vm
        body = self._enc(" Text input:\n")
        for sid, line in parsed:
            body += self._enc(f" Speaker {sid}:{line}\n")
        body += self._enc(" Speech output:\n")
        ids += body + [self.tokenizer.speech_start_id]
        mask += [False] * (len(body) + 1)
        return {"input_ids": ids, "speech_inputs": vw or None, "speech_input_mask": mask, "parsed_script": parsed,
                "all_speakers": speakers}

    def prepare_speech_inputs(self, speech_inputs: List[np.ndarray], return_tensors=None, device=None, dtype=None):
        """Zero-padded [N, T_max] waveforms + [N, ceil(T_max / 3200)] frame masks."""
        if not speech_inputs:
            return {"padded_speeches": None, "speech_masks": None}
        frames = [math.ceil(s.shape[0] / self.speech_tok_compress_ratio) for s in speech_inputs]
        tmax = max(s.shape[0] for s in speech_inputs)
        shape = (len(speech_inputs), tmax) + tuple(speech_inputs[0].shape[1:])
        padded = np.zeros(shape, dtype=np.float32)
        masks = np.zeros((len(speech_inputs), max(frames)), dtype=np.bool_)
        for i, (s, n) in enumerate(zip(speech_inputs, frames)):
            padded[i, :len(s)] = s
            masks[i, :n] = True
        if return_tensors == "pt":
            return {"padded_speeches": torch.tensor(padded, device=device, dtype=dtype or torch.float32),
                    "speech_masks": torch.tensor(masks, device=device, dtype=torch.bool)}
        return {"padded_speeches": padded, "speech_masks": masks}

    def _batch_encode(self, encodings, padding=True, truncation=False, max_length=None, return_tensors=None,
                      return_attention_mask=True):
        from transformers.tokenization_utils_base import BatchEncoding
        ids = [e["input_ids"] for e in encodings]
        smask = [e["speech_input_mask"] for e in encodings]
        if isinstance(padding, bool):
            strategy = "longest" if padding else "do_not_pad"
        else:
            strategy = str(getattr(padding, "value", padding))
        att = None
        if strategy != "do_not_pad":
            target = max_length if (strategy == "max_length" and max_length is not None) else max(map(len, ids))
            out_ids, att, out_sm = [], [], []
            for x, m in zip(ids, smask):
                if truncation and len(x) > target:
                    x, m = x[:target], m[:target]
                pad = target - len(x)                       # left padding
                out_ids.append([self.tokenizer.pad_id] * pad + x)
                att.append([0] * pad + [1] * len(x))
                out_sm.append([False] * pad + m)
            ids, smask = out_ids, out_sm
        elif return_attention_mask:
            att = [[1] * len(x) for x in ids]
        speech = [w for e in encodings if e["speech_inputs"] is not None for w in e["speech_inputs"]]
        be = BatchEncoding()
        if return_tensors is not None:
            be["input_ids"] = torch.tensor(ids, dtype=torch.long)
            if return_attention_mask and att is not None:
                be["attention_mask"] = torch.tensor(att, dtype=torch.long)
            be["speech_input_mask"] = torch.tensor(smask, dtype=torch.bool)
        else:
            be["input_ids"] = ids
            if return_attention_mask and att is not None:
                be["attention_mask"] = att
            be["speech_input_mask"] = smask
        if speech:
            sp = self.prepare_speech_inputs(speech, return_tensors=return_tensors)
            be["speech_tensors"], be["speech_masks"] = sp["padded_speeches"], sp["speech_masks"]
        else:
            be["speech_tensors"], be["speech_masks"] = None, None
        be["parsed_scripts"] = [e["parsed_script"] for e in encodings]
        be["all_speakers_list"] = [e["all_speakers"] for e in encodings]
        return be

    def __call__(self, text=None, voice_samples=None, padding=True, truncation=False, max_length=None,
                 return_tensors=None, return_attention_mask: bool = True, **kwargs):
        """BatchEncoding with input_ids, attention_mask, speech_input_mask,
        speech_tensors, speech_masks, parsed_scripts, all_speakers_list
        (vibevoice_processor.py:163-244)."""
        single = isinstance(text, str) or (isinstance(text, list) and len(text) > 0 and not isinstance(text[0], str))
        texts = [text] if single else text
        if voice_samples is None:
            voices = [None] * len(texts)
        elif single or isinstance(voice_samples[0], (str, np.ndarray)):
            voices = [voice_samples]
        else:
            voices = voice_samples
        encs = [self._process_single(t, v) for t, v in zip(texts, voices)]
        return self._batch_encode(encs, padding=padding, truncation=truncation, max_length=max_length,
                                  return_tensors=return_tensors, return_attention_mask=return_attention_mask)

    def batch_decode(self, *args, **kwargs):
        return self.tokenizer.batch_decode(*args, **kwargs)

    def decode(self, *args, **kwargs):
        return self.tokenizer.decode(*args, **kwargs)

    @property
    def model_input_names(self):
        names = list(self.tokenizer.model_input_names) + list(self.audio_processor.model_input_names)
        return list(dict.fromkeys(names + ["speech_inputs", "speech_input_mask"]))

    def save_audio(self, audio, output_path: str = "output.wav", sampling_rate: Optional[int] = None,
                   normalize: bool = False, batch_prefix: str = "audio_"):
        return self.audio_processor.save_audio(audio, output_path=output_path, sampling_rate=sampling_rate,
                                               normalize=normalize, batch_prefix=batch_prefix)


__all__ = ["VibeVoiceProcessor", "VibeVoiceTokenizerProcessor", "AudioNormalizer", "VibeVoiceTextTokenizerFast"]
