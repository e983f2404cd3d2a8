"""The standalone tokenizer API (vibevoice_amd/tokenizer.py) on the GPU:
`model.model.acoustic_tokenizer.decode(latents, cache=..., sample_indices=...,
use_cache=True)`, `model.model.semantic_tokenizer.encode(...)`,
`VibeVoiceTokenizerStreamingCache.set_to_zero / clear`, the connectors, as the
reference's generate() calls them (modeling_vibevoice_inference.py:651-687;
modular_vibevoice_tokenizer.py:193-256, 1081-1108).

* Streaming with a cache over several calls and sample subsets equals the
  oracle's streaming decode / encode with the same per-sample state; the
  non-cached decode of a T-frame sequence equals the oracle's non-streaming
  decode (rel L2 < 3e-2, cosine > 0.999: the codec tolerance of
  test_gpu_codec.py).
* The API frame for frame is bit-identical to the fused vv_codec_step that
  generate() runs (same kernels: the API's codec context follows its owner's
  one-launch kernels, vv_set_persistent 2; latent scaling done by the caller
  in bf16).
"""
import pytest
import torch

from gpu_util import cos, rel_err
from oracle import codec as ocodec
from tiny import tiny_config
from vibevoice.modular.modular_vibevoice_tokenizer import VibeVoiceTokenizerStreamingCache
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"


def _sub(sd, prefix):
    return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}


@pytest.fixture(scope="module")
def setup():
    cfg = tiny_config(hidden=256, layers=1, heads=2, kv_heads=1, inter=512, ratios=(8, 5, 5, 4, 2, 2),
                      depths="3-3-3-3-3-3-8", nf=32)
    sd = synthetic_state_dict(cfg, seed=41, device="cpu", mode="test", with_acoustic_encoder=False)
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=4, max_ctx=64)
    return cfg, sd, model


def test_streaming_decode_encode_with_cache(setup):
    cfg, sd, model = setup
    mm = model.model
    dd = ocodec.codec_dims(cfg.acoustic_tokenizer_config, "decoder")
    ed = ocodec.codec_dims(cfg.semantic_tokenizer_config, "encoder")
    sd_a, sd_s = _sub(sd, "model.acoustic_tokenizer."), _sub(sd, "model.semantic_tokenizer.")
    st_a, st_s = ocodec.StreamState(6), ocodec.StreamState(6)
    ac, sc = VibeVoiceTokenizerStreamingCache(), VibeVoiceTokenizerStreamingCache()
    g = torch.Generator().manual_seed(3)
    scale, bias = sd["model.speech_scaling_factor"], sd["model.speech_bias_factor"]
    for step, idx in enumerate([[0, 5], [0, 5], [5], [0, 3, 5], [3]]):
        n = len(idx)
        lat = torch.randn(n, 1, 64, generator=g).bfloat16()                  # speech_latent [n, 1, D]
        z = lat / scale - bias                                                # :651 (bf16, on the caller's side)
        sidx = torch.tensor(idx)
        audio = mm.acoustic_tokenizer.decode(z.to(dev), cache=ac, sample_indices=sidx.to(dev), use_cache=True)
        sem = mm.semantic_tokenizer.encode(audio, cache=sc, sample_indices=sidx, use_cache=True).mean
        a_ref = ocodec.decode(sd_a, dd, z.permute(0, 2, 1), st_a, sidx)
        s_ref = ocodec.encode(sd_s, ed, a_ref, st_s, sidx)
        assert audio.shape == a_ref.shape == (n, 1, cfg.hop) and sem.shape == s_ref.shape == (n, 1, 128)
        for name, got, ref in (("audio", audio, a_ref), ("sem", sem, s_ref)):
            e, c = rel_err(got, ref), cos(got, ref)
            print(f"step {step} {name}: rel {e:.3e} cos {c:.6f}")
            assert e < 3e-2 and c > 0.999
        if step == 1:                      # speech_end for sample 0 (:557-560)
            ac.set_to_zero(torch.tensor([0]))
            sc.set_to_zero(torch.tensor([0]))
            st_a.zero(torch.tensor([0]))
            st_s.zero(torch.tensor([0]))
    emb = mm.acoustic_connector(lat.to(dev)) + mm.semantic_connector(sem)
    assert emb.shape == (1, 1, cfg.decoder_config.hidden_size)
    ac.clear()
    sc.clear()
    assert not ac.cache and not sc.cache


def test_nonstreaming_decode_sequence(setup):
    """use_cache=False: a 4-frame latent sequence [n, D, T] decoded at once from
    zero state = the oracle's non-streaming TokenizerDecoder."""
    cfg, sd, model = setup
    dd = ocodec.codec_dims(cfg.acoustic_tokenizer_config, "decoder")
    z = torch.randn(2, 64, 4, generator=torch.Generator().manual_seed(4)).bfloat16()
    audio = model.model.acoustic_tokenizer.decode(z.to(dev))
    ref = ocodec.decode(_sub(sd, "model.acoustic_tokenizer."), dd, z, None, None, streaming=False)
    assert audio.shape == ref.shape == (2, 1, 4 * cfg.hop)
    e, c = rel_err(audio, ref), cos(audio, ref)
    print(f"non-streaming 4 frames: rel {e:.3e} cos {c:.6f}")
    assert e < 3e-2 and c > 0.999


def test_api_frames_bit_identical_to_codec_step(setup):
    """What generate() runs (fused vv_codec_step on its own slots) and the
    standalone API give the same bits, frame after frame."""
    cfg, sd, model = setup
    eng = model.engine
    slots = torch.arange(2, dtype=torch.int32, device=dev)
    eng.codec_reset(slots)
    ac, sc = VibeVoiceTokenizerStreamingCache(), VibeVoiceTokenizerStreamingCache()
    g = torch.Generator().manual_seed(5)
    scale, bias = model.model.speech_scaling_factor.cpu(), model.model.speech_bias_factor.cpu()
    for _ in range(3):
        lat = torch.randn(2, 64, generator=g).bfloat16()
        a1 = torch.empty(2, cfg.hop, dtype=torch.bfloat16, device=dev)
        s1 = torch.empty(2, 128, dtype=torch.bfloat16, device=dev)
        eng.codec_step(slots, lat.to(dev), a1, s1)
        z = (lat / scale - bias)[:, None]
        a2 = model.model.acoustic_tokenizer.decode(z.to(dev), cache=ac, sample_indices=torch.arange(2), use_cache=True)
        s2 = model.model.semantic_tokenizer.encode(a2, cache=sc, sample_indices=torch.arange(2), use_cache=True).mean
        torch.cuda.synchronize()
        assert torch.equal(a1, a2[:, 0]) and torch.equal(s1, s2[:, 0])


def test_tokenizer_views_on_a_tp_shard():
    """The tokenizer views of a tensor-parallel rank bind the rank's packed LM
    shards (the view engine used tp_size = 1 and failed the shape
    check on every TP model).  A TP = 2 rank-0 owner (single-process group, no
    communicator) decodes and encodes bit-identically to the TP = 1 model."""
    import types
    from vibevoice_amd import tokenizer as tk
    from vibevoice_amd.engine import Engine
    cfg = tiny_config(hidden=256, layers=1, heads=4, kv_heads=2, inter=512, ratios=(8, 5, 5, 4, 2, 2),
                      depths="3-3-3-3-3-3-8", nf=32)
    sd = synthetic_state_dict(cfg, seed=43, device="cpu", mode="test", with_acoustic_encoder=False)
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=4, max_ctx=64)
    shard = Engine(cfg, sd, dev, max_batch=4, max_ctx=64, tp_rank=0, tp_size=2)
    owner = types.SimpleNamespace(engine=shard, config=cfg, device=model.device, tp_rank=0, tp_size=2)
    pool = tk._SlotPool(owner, 4)
    ac = tk.AcousticTokenizer(owner, pool, cfg.acoustic_tokenizer_config)
    sc = tk.SemanticTokenizer(owner, pool, cfg.semantic_tokenizer_config)
    g = torch.Generator().manual_seed(9)
    z = torch.randn(2, 64, 3, generator=g).bfloat16().to(dev)
    a_tp = ac.decode(z)
    a_1 = model.model.acoustic_tokenizer.decode(z)
    assert torch.equal(a_tp, a_1)
    assert torch.equal(sc.encode(a_tp).mean, model.model.semantic_tokenizer.encode(a_1).mean)


@pytest.mark.parametrize("L", [1066, 8003, 9599, 9600])
def test_semantic_encode_partial_frame_nonstreaming(setup, L):
    """semantic_tokenizer.encode(audio) without a cache for clips ending in a
    partial frame (modular_vibevoice_tokenizer.py:127-133, 393-408: every
    strided conv right-pads its input to whole strides): ceil(L / hop) frames,
    vs the oracle's non-streaming encoder (pinned to the reference's
    VibeVoiceSemanticTokenizerModel by golden G5) at the real encoder shapes.
    L = 9600 (whole frames) streams from zero state and must match too."""
    cfg, sd, model = setup
    ed = ocodec.codec_dims(cfg.semantic_tokenizer_config, "encoder")
    sd_s = _sub(sd, "model.semantic_tokenizer.")
    g = torch.Generator().manual_seed(L)
    audio = (0.3 * torch.randn(2, 1, L, generator=g)).bfloat16()
    got = model.model.semantic_tokenizer.encode(audio.to(dev)).mean
    ref = ocodec.encode(sd_s, ed, audio, None, None, streaming=False)
    assert got.shape == ref.shape == (2, -(-L // cfg.hop), 128), (got.shape, ref.shape)
    for i in range(2):
        e, c = rel_err(got[i], ref[i]), cos(got[i], ref[i])
        print(f"semantic encode L={L} clip {i}: rel {e:.3e} cos {c:.6f}")
        assert e < 3e-2 and c > 0.999
    with pytest.raises(ValueError):
        from vibevoice.modular.modular_vibevoice_tokenizer import VibeVoiceTokenizerStreamingCache as Cache
        model.model.semantic_tokenizer.encode(audio[:, :, :L - 1 if L % cfg.hop == 0 else L].to(dev), cache=Cache(),
                                              sample_indices=torch.arange(2), use_cache=True)
