"""Where the persistent codec stage's time goes (csrc/codec_stage.hip), measured
as the decode loop runs it: one sample's streaming codec step at the real 1.5B
codec shapes (seeded weights), captured into a hipGraph and replayed.
  * the whole codec step (decoder + semantic encoder + connectors), best of 20
    graph replays, with the stage launch and with the launch-per-GEMV path;
  * per-workgroup s_memrealtime stamps (10 ns ticks) of the acoustic decoder's
    stage launch, per block j: 8j + 0 front half begins, 1 fc1 input in LDS,
    2 fc1 slice landed (compute wave 0), 3 fc1 partials in LDS, 4 hidden-row
    wait released, 5 hidden row in LDS, 6 fc2 partials in LDS, 7 next-input
    wait released; median / max over the 256 workgroups relative to the first
    stamp, and the phase-to-phase medians.

usage: python tools/codec_stage_stamps.py [stage] [modes]   (the decoder's stage: 0 = C 2,048 T 1, 1 = C 1,024 T 8;
modes: comma-separated vv_codec_stage values, e.g. 1,3,1,3: bits 1..3 pick the weight-stream issue, engine.cpp)"""
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


def main():
    stage = int(sys.argv[1]) if len(sys.argv) > 1 else 0
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
        eng.codec_step(slot, lat, audio, sem, emb, slot, stream=s)   # eager first (plans, workspaces)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            gr = torch.cuda.CUDAGraph()
            gr.capture_begin(capture_error_mode="thread_local")
            eng.codec_step(slot, lat, audio, sem, emb, slot, stream=s)
            gr.capture_end()
        return gr

    modes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 0, 1]
    for mode in modes:   # vv_codec_stage values; stamps taken with the last
        L.vv_codec_stage(mode)
        assert L.vv_codec_stage_active(eng.h) == (mode & 1)
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
        print(f"codec step, vv_codec_stage({mode}): best of 20 graph replays {best:.1f} us",
              flush=True)
    st = torch.zeros(256 * 64, dtype=torch.int64, device="cuda")
    L.vv_codec_stage_stamps(st.data_ptr(), stage)
    gr = capture()   # the stamp pointer is a launch argument
    for _ in range(3):
        with torch.cuda.stream(s):
            gr.replay()
        torch.cuda.synchronize()
    L.vv_codec_stage_stamps(None, 0)
    eng.check_sync()
    t = st.view(256, 64).cpu().double() * 10e-3   # us
    used = [k for k in range(64) if bool((st.view(256, 64)[:, k] != 0).all())]
    t0 = t[:, 0].min()
    rel = t - t0
    names = ["front half begins", "fc1 input in LDS", "fc1 slice landed (wave 0)", "fc1 partials in LDS",
             "hidden-row wait released", "hidden row in LDS", "fc2 partials in LDS", "next-input wait released"]
    # k_codec_stage_s (C = 1,024) also stamps its front half at 40 + 4j + k
    front = ["(front) input rows landed", "(front) mixer-norm inverses", "(front) conv + residual done",
             "(front) FFN-norm inverses"]

    def label(k):
        return f"block {k // 8} {names[k % 8]}" if k < 40 else f"block {(k - 40) // 4} {front[(k - 40) % 4]}"
    print(f"acoustic decoder stage {stage}, us from the first workgroup's first stamp (median / max over workgroups):")
    prev = None
    used = [k for k in used if k < 40] + [k for k in used if k >= 40]   # block phases, then the front-half detail
    for k in used:
        col = rel[:, k]
        d = "" if prev is None else f"   +{(col - rel[:, prev]).median():.2f} from the previous (median)"
        print(f"  {k:2d} {label(k):38s} {col.median():8.2f} {col.max():8.2f}{d}")
        prev = k


if __name__ == "__main__":
    main()
