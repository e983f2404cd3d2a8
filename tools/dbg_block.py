import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from tiny import tiny_config
from vibevoice_amd import _lib
from vibevoice_amd.engine import Engine
from vibevoice_amd.weights import synthetic_state_dict
dev = "cuda"
for ratios, depths, nf in [((16,), "1-1", 128), ((32,), "1-1", 128), ((32,), "1-1", 64), ((64,), "1-1", 64),
                           ((64,), "1-1", 32), ((128,), "1-1", 32)]:
    try:
        cfg = tiny_config(ratios=ratios, depths=depths, nf=nf)
        sd = synthetic_state_dict(cfg, seed=3, device="cpu", mode="test", with_acoustic_encoder=False)
    except Exception as e:
        print(ratios, depths, "config error", e)
        continue
    eng = Engine(cfg, sd, dev, max_batch=1, max_ctx=64)
    H = cfg.decoder_config.hidden_size
    lat = torch.randn(1, 64, generator=torch.Generator().manual_seed(1)).bfloat16().to(dev)
    slots = torch.zeros(1, dtype=torch.int32, device=dev)
    outs = {}
    for mask in (0, 2):
        _lib.lib().vv_codec_mix_fusion(mask)
        eng.codec_reset(slots)
        audio = torch.empty(1, cfg.hop, dtype=torch.bfloat16, device=dev)
        sem = torch.empty(1, 128, dtype=torch.bfloat16, device=dev)
        emb = torch.zeros(1, H, dtype=torch.bfloat16, device=dev)
        eng.codec_step(slots, lat, audio, sem, emb, slots)
        torch.cuda.synchronize()
        outs[mask] = audio.clone()
    a, b = outs[0].float(), outs[2].float()
    print(ratios, depths, nf, "hop", cfg.hop, "equal", torch.equal(a, b), "maxdiff", (a - b).abs().max().item(),
          "ndiff", int((a != b).sum()), flush=True)
