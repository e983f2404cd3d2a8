"""Where the B = 8 head layer's time goes (csrc/head_m16.hip), measured as the
loop runs it: the 1.5B head (seeded weights, real shapes) sampled for n = 8
samples (16 rows) inside a graph replay, the LAST k_head_m16 launch writing
per-workgroup s_memrealtime stamps (10 ns ticks):
  0 entry          1 A side landed (compute wave 0)   2 row norms
  3 transform      4 gate|up partials in LDS          5 SiLU * up
  6 hand-off released (after the grid wait)           7 act rows in LDS
  8 down partials in LDS                              9 end (owners)
Layers l >= 1 build the A side distributed (vv_head_m16_pre, default): 1, 10,
12, 13 are then not written, 2 = that form's first grid wait released, 3 = the
transformed rows in LDS.
Prints per phase the median / max over the 256 workgroups relative to the
first entry, and the phase-to-phase medians.

  10 A side landed (wave 7)  11 gate / x columns landed (control wave)
  12 / 13 wave 0's norm / transform loop done (before the barrier)  14 wave 0 past the barrier before the norm
The stamped run uses the variant given (vv_head_m16's value: 1 default, + 2 =
every A-side DMA issued before any weight load (default at > 8 rows), + 8 =
never, + 4 = the down weights issued
right after the gate|up products instead of after SiLU * up).

usage: python tools/head_m16_stamps.py [n] [variant]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.engine import Engine  # noqa: E402
from vibevoice_amd.weights import synthetic_state_dict  # noqa: E402
from test_gpu_head import real_head_sd  # noqa: E402
from tiny import tiny_config  # noqa: E402


def capture(eng, pos, neg, x, s):
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        gr.capture_begin(capture_error_mode="thread_local")
        eng.diffusion_sample(pos, neg, x, 1.3, stream=s)
        gr.capture_end()
    return gr


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    variant = int(sys.argv[2]) if len(sys.argv) > 2 else 1   # vv_head_m16's value: 2 = A side first, 8 = not first (default: first at > 8 rows)
    g = torch.Generator().manual_seed(5)
    sdh, hc, H = real_head_sd(g)
    cfg = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    sd = synthetic_state_dict(cfg, seed=0, device="cpu", mode="test", with_acoustic_encoder=False)
    for k, v in sdh.items():
        sd["model.prediction_head." + k] = v
    eng = Engine(cfg, sd, "cuda", max_batch=8, max_ctx=64)   # the GEMV layout
    eng.set_steps(10)
    pos = torch.randn(n, H, generator=g).bfloat16().cuda()
    neg = torch.randn(n, H, generator=g).bfloat16().cuda()
    x0 = torch.randn(n, 64, generator=g).bfloat16().cuda()
    x = x0.clone()
    L = _lib.lib()
    s = torch.cuda.Stream()
    for mode, pre in ((0, 1), (5, 0), (1, 0), (5, 1), (3, 1), (9, 1), (1, 1), (variant, 1)):
        L.vv_head_m16(mode)
        L.vv_head_m16_pre(pre)
        assert L.vv_head_m16_active(eng.h, n) == (1 if mode else 0)
        eng.diffusion_sample(pos, neg, x, 1.3)
        gr = capture(eng, pos, neg, x, s)
        best = 1e9
        for rep in range(8):
            x.copy_(x0)
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                ev0.record(s)
                gr.replay()
                ev1.record(s)
            torch.cuda.synchronize()
            best = min(best, ev0.elapsed_time(ev1) * 1e3)
        print(f"{'k_head_m16' if mode else 'GEMV pair'}{' A side first' if mode & 2 else ' A side not first' if mode & 8 else ''}"
              f"{' down issued after gate|up' if mode & 4 else ''}"
              f"{' (distributed A side)' if mode and pre else ''}: whole head sample (cond + adaLN + "
              f"{eng.steps} steps x {hc.head_layers} layers), best of 8 graph replays: {best:.1f} us")
    st = torch.zeros(256 * 16, dtype=torch.int64, device="cuda")
    L.vv_head_m16_stamps(st.data_ptr())
    gr = capture(eng, pos, neg, x, s)   # the stamp pointer is a launch argument
    for _ in range(3):
        x.copy_(x0)
        with torch.cuda.stream(s):
            gr.replay()
        torch.cuda.synchronize()
    L.vv_head_m16_stamps(None)
    eng.check_sync()
    t = st.view(256, 16).cpu().double() * 10e-3   # us
    t0 = t[:, 0].min()
    rel = t - t0
    names = ["entry", "A side landed", "row norms", "transform", "gate|up partials", "SiLU * up",
             "hand-off released", "act rows in LDS", "down partials", "end (owners)",
             "A side landed (w7)", "gate / x cols (ctl)", "norm loop done (w0)", "transform loop done (w0)", "barrier passed (w0)"]
    print("last launch's phases, us from the first workgroup's entry (median / max over workgroups):")
    prev = None
    for k in (0, 11, 1, 10, 14, 12, 2, 13, 3, 4, 5, 6, 7, 8, 9):   # in phase order
        name = names[k]
        col = rel[:, k]
        ok = t[:, k] >= t[:, 0]   # (a stamp the last launch's form does not write holds an earlier launch's)
        col = col[ok]
        if col.numel() == 0:
            continue
        d = "" if prev is None else f"   +{(rel[ok, k] - rel[ok, prev]).median():.2f} from the previous (median)"
        print(f"  {k} {name:20s} {col.median():8.2f} {col.max():8.2f}  ({int(ok.sum())} wg){d}")
        prev = k
    L.vv_head_m16(1)


if __name__ == "__main__":
    main()
