"""VibeVoiceProcessor parity (CPU) against golden G9, made by running the
reference's own processor and text tokenizer class over the same tiny
Qwen2-style vocabulary (tests/golden/make_golden.py g9_processor): prompt
layout, speech masks, dBFS voice normalisation (incl. the anti-clipping path),
left padding, ragged no-padding lists, speaker-id normalisation and the
.json / .txt script converters.  Plus from_pretrained / save_pretrained and the
WAV save/load round trip (scipy stands in for soundfile / librosa)."""
import json
import os

import numpy as np
import pytest
import torch

from golden_io import load
from vibevoice_amd.processor import (AudioNormalizer, VibeVoiceProcessor, VibeVoiceTextTokenizerFast,
                                     VibeVoiceTokenizerProcessor)

TOK_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tiny_qwen_tokenizer")


@pytest.fixture(scope="module")
def g9():
    return load("g9_processor.npz")


@pytest.fixture(scope="module")
def proc():
    return VibeVoiceProcessor(tokenizer=VibeVoiceTextTokenizerFast.from_pretrained(TOK_DIR),
                              audio_processor=VibeVoiceTokenizerProcessor())


def _voices(g):
    return [g[f"voice{i}"] for i in range(4)]


def _check(be, g, tag):
    for k in ("input_ids", "attention_mask", "speech_input_mask", "speech_tensors", "speech_masks"):
        key = f"{tag}_{k}"
        if key in g:
            got = be[k].numpy()
            if k == "speech_tensors":   # float32 normalisation arithmetic, same numpy ops
                np.testing.assert_allclose(got, g[key], rtol=1e-6, atol=1e-7)
            else:
                np.testing.assert_array_equal(got, g[key], err_msg=key)
        else:
            assert be.get(k) is None, key
    assert json.loads(json.dumps(be["parsed_scripts"])) == json.loads(str(g[f"{tag}_parsed"]))
    assert be["all_speakers_list"] == json.loads(str(g[f"{tag}_speakers"]))


def test_special_ids(g9, proc):
    t = proc.tokenizer
    assert [t.speech_start_id, t.speech_end_id, t.speech_diffusion_id, t.eos_token_id, t.pad_id] == g9["ids"].tolist()
    assert t.bos_token_id is None


def test_batch_with_ragged_voices(g9, proc):
    v = _voices(g9)
    scripts = [str(s) for s in g9["scripts"]]
    _check(proc(text=scripts, voice_samples=[[v[0], v[1]], [v[2]]], padding=True, return_tensors="pt"), g9, "a")


def test_single_script_extra_voices_dropped(g9, proc):
    v = _voices(g9)
    _check(proc(text=str(g9["scripts"][0]), voice_samples=[v[3], v[1], v[0]], return_tensors="pt"), g9, "b")


def test_no_voices(g9, proc):
    _check(proc(text=[str(s) for s in g9["scripts"]], padding=True, return_tensors="pt"), g9, "c")


def test_no_padding_lists(g9, proc):
    be = proc(text=[str(s) for s in g9["scripts"]], padding=False, return_tensors=None)
    assert [len(x) for x in be["input_ids"]] == g9["d_lengths"].tolist()
    np.testing.assert_array_equal(np.concatenate(be["input_ids"]), g9["d_input_ids"])
    np.testing.assert_array_equal(np.concatenate(be["attention_mask"]), g9["d_attention_mask"])


def test_script_files(g9, proc, tmp_path):
    pj, pt = tmp_path / "s.json", tmp_path / "s.txt"
    pj.write_text(str(g9["json_src"]))
    pt.write_text(str(g9["txt_src"]))
    assert proc._convert_json_to_script(str(pj)) == str(g9["json_script"])
    assert proc._convert_text_to_script(str(pt)) == str(g9["txt_script"])
    be = proc(text=[str(pj), str(pt)], padding=True, return_tensors="pt")
    np.testing.assert_array_equal(be["input_ids"].numpy(), g9["e_input_ids"])


def test_layout_feeds_generate(proc, g9):
    """speech_input_mask marks exactly ceil(len/3200) diffusion slots per voice,
    each between speech_start and speech_end (what _process_speech_inputs
    splices the voice latents into, modeling_vibevoice_inference.py:150-177)."""
    v = _voices(g9)
    be = proc(text=[str(s) for s in g9["scripts"]], voice_samples=[[v[0], v[1]], [v[2]]], return_tensors="pt")
    t = proc.tokenizer
    ids, sm = be["input_ids"], be["speech_input_mask"]
    assert torch.all(ids[sm] == t.speech_diffusion_id)
    assert int(sm.sum()) == int(be["speech_masks"].sum()) == 3 + 4 + 1
    assert torch.all(ids[:, -1] == t.speech_start_id)


def test_from_pretrained_and_save(tmp_path):
    VibeVoiceProcessor(tokenizer=None, audio_processor=VibeVoiceTokenizerProcessor(target_dB_FS=-20)) \
        .save_pretrained(str(tmp_path))
    cfg = json.loads((tmp_path / "preprocessor_config.json").read_text())
    assert cfg["audio_processor"]["target_dB_FS"] == -20 and cfg["speech_tok_compress_ratio"] == 3200
    cfg["language_model_pretrained_name"] = TOK_DIR
    (tmp_path / "preprocessor_config.json").write_text(json.dumps(cfg))
    p = VibeVoiceProcessor.from_pretrained(str(tmp_path))
    assert p.audio_processor.target_dB_FS == -20 and p.tokenizer.speech_diffusion_id is not None
    with pytest.raises(OSError):
        VibeVoiceTextTokenizerFast.from_pretrained(str(tmp_path / "missing-qwen"))


def test_audio_io_roundtrip(tmp_path):
    ap = VibeVoiceTokenizerProcessor()
    rng = np.random.default_rng(3)
    x = (0.2 * rng.standard_normal(4800)).astype(np.float32)
    path = ap.save_audio(torch.from_numpy(x)[None, None], str(tmp_path / "a.wav"))[0]
    np.testing.assert_array_equal(ap._load_audio_from_path(path), x)
    paths = ap.save_audio(torch.from_numpy(np.stack([x, x]))[:, None], str(tmp_path / "batch"))
    assert [os.path.basename(p) for p in paths] == ["audio_0.wav", "audio_1.wav"]
    # 16 kHz int16 input resampled to 24 kHz
    from scipy.io import wavfile
    wavfile.write(str(tmp_path / "b.wav"), 16000, (x[:3200] * 32767).astype(np.int16))
    y = ap._load_audio_from_path(str(tmp_path / "b.wav"))
    assert y.dtype == np.float32 and y.shape == (4800,)
    out = ap(audio=[x, x], return_tensors="pt")["audio"]
    assert out.shape == (2, 1, 4800)
    n = AudioNormalizer()(x)
    assert abs(20 * np.log10(np.sqrt(np.mean(n ** 2))) + 25) < 1e-3
