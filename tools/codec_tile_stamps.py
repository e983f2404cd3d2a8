"""Where the tiled narrow codec stages' time goes (csrc/codec_tile.hip), measured
as the loop runs them: one sample's streaming codec step at the real 1.5B codec
shapes (seeded weights) captured into a hipGraph and replayed, with the six tile
launches writing per-workgroup s_memrealtime stamps (10 ns ticks): 0 start,
1 input rows in LDS, 2 transition conv done, per block j: 3+4j mixer norm,
4+4j conv + FFN norm, 5+4j fc1, 6+4j fc2; 15 end.  Prints, per launch, the
median over workgroups of each phase's time since the workgroup's start, and
the launch span (first start to last end).

usage: python tools/codec_tile_stamps.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.engine import Engine  # noqa: E402
from vibevoice_amd.weights import synthetic_state_dict  # noqa: E402
from tiny import tiny_config  # noqa: E402

NAMES = {0: "dec C=128 (3 blocks)", 1: "dec C=64 (convT + 3 blocks)", 2: "dec C=32 (convT + 3 blocks + head)",
         3: "enc C=32 (stem + 3 blocks)", 4: "enc C=64 (sconv + 3 blocks)", 5: "enc C=128 (sconv + 3 blocks)"}
TILES = {0: 50, 1: 100, 2: 200, 3: 200, 4: 100, 5: 50}


def main():
    L = _lib.lib()
    cfg = tiny_config(ratios=(8, 5, 5, 4, 2, 2), depths="3-3-3-3-3-3-8", nf=32)
    sd = synthetic_state_dict(cfg, seed=3, device="cpu", mode="test", with_acoustic_encoder=False)
    eng = Engine(cfg, sd, "cuda", max_batch=1, max_ctx=64)
    H = cfg.decoder_config.hidden_size
    slot = torch.zeros(1, dtype=torch.int32, device="cuda")
    lat = torch.randn(1, 64).bfloat16().cuda()
    audio = torch.empty(1, cfg.hop, dtype=torch.bfloat16, device="cuda")
    sem = torch.empty(1, 128, dtype=torch.bfloat16, device="cuda")
    emb = torch.zeros(1, H, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()

    def capture():
        eng.codec_step(slot, lat, audio, sem, emb, slot, stream=s)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            gr = torch.cuda.CUDAGraph()
            gr.capture_begin(capture_error_mode="thread_local")
            eng.codec_step(slot, lat, audio, sem, emb, slot, stream=s)
            gr.capture_end()
        return gr

    for mode in (0, 1, 0, 1):   # the narrow stages per Block1D / as tile launches (wide stages as built)
        L.vv_codec_tile(mode)
        gr = capture()
        best = 1e9
        for _ in range(20):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record(s)
                gr.replay()
                e1.record(s)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3)
        print(f"codec step, {'tile launches' if mode else 'k_block per Block1D'}: best of 20 graph replays "
              f"{best:.1f} us", flush=True)
    st = torch.zeros(6 * 4096, dtype=torch.int64, device="cuda")
    L.vv_codec_tile_stamps(st.data_ptr())
    gr = capture()
    for _ in range(3):
        with torch.cuda.stream(s):
            gr.replay()
        torch.cuda.synchronize()
    L.vv_codec_tile_stamps(None)
    eng.check_sync()
    wst = torch.zeros(4 * 8192, dtype=torch.int64, device="cuda")
    if L.vv_codec_wide_active(eng.h, 1):
        L.vv_codec_wide_stamps(wst.data_ptr())
        gr = capture()
        for _ in range(3):
            with torch.cuda.stream(s):
                gr.replay()
            torch.cuda.synchronize()
        L.vv_codec_wide_stamps(None)
        eng.check_sync()
    all_t = st.view(6, 256, 16).cpu().double() * 10e-3   # us
    for li in range(6):
        t = all_t[li, :TILES[li]]
        used = [k for k in range(16) if bool((t[:, k] != 0).all())]
        rel = t[:, used] - t[:, :1]
        med = rel.median(0).values
        span = (t[:, 15] - t[:, 0].min()).max() if 15 in used else float("nan")
        print(f"{NAMES[li]}: span {span:.2f} us; start skew {float((t[:, 0] - t[:, 0].min()).max()):.2f} us; "
              "median per phase since start: " + ", ".join(f"{k}:{float(m):.2f}" for k, m in zip(used, med)))
    if wst.any():
        wide_report(wst)




def wide_report(wst):
    """codec_wide.hip stamps: 0 start, 1 input rows in LDS, per block j: 2+4j mixer
    done, 3+4j fc2 partial stored, 4+4j reduce wait released, 5+4j gather wait
    released; 15 end."""
    names = {0: "dec C=256 (13 tiles x 8)", 1: "dec C=512 (3 tiles x 16)", 2: "enc C=256", 3: "enc C=512"}
    wgs = {0: 104, 1: 48, 2: 104, 3: 48}
    for li in range(4):
        t = wst[li * 8192:(li * 8192) + wgs[li] * 16].view(wgs[li], 16).cpu().double() * 10e-3
        used = [k for k in range(16) if bool((t[:, k] != 0).all())]
        rel = t[:, used] - t[:, :1]
        med = rel.median(0).values
        span = (t[:, 15] - t[:, 0].min()).max() if 15 in used else float("nan")
        print(f"{names[li]}: span {span:.2f} us; median per phase since start: "
              + ", ".join(f"{k}:{float(m):.2f}" for k, m in zip(used, med)))


if __name__ == "__main__":
    main()
