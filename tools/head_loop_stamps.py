"""Where the persistent diffusion head's time goes (csrc/head_loop.hip),
measured as the loop runs it: the 1.5B head (seeded weights, real shapes)
sampled for n samples inside a graph replay, the launch writing per-workgroup
s_memrealtime stamps (10 ns ticks) of its LAST diffusion step's phases:
  40 / 41 noisy projection stored / its wait released
  8l + 0  layer l: operands in LDS (the control wave's DMA landed)
  8l + 1  transform in LDS        8l + 2  gate|up dots done (next slice issued)
  8l + 3  down rows in registers  8l + 4  partial in LDS
  8l + 5  slab stores issued      8l + 6  slabs in LDS (after the wait)
  8l + 7  state slice stored (before the second wait)
  63      end of the launch
plus stamp 62 (launch entry).  Prints per phase the median / max over the 256
workgroups relative to the first entry, and the phase-to-phase medians.

usage: python tools/head_loop_stamps.py [n] [mode]   (mode: vv_head_loop's value for the persistent
launch, 2 = plain launch with shard-polled waits (default), 3 = generation-word waits, 1 = cooperative)"""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    mode = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    g = torch.Generator().manual_seed(5)
    sdh, hc, H = real_head_sd(g)
    cfg = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    sd = synthetic_state_dict(cfg, seed=0, device="cpu", mode="test", with_acoustic_encoder=False)
    for k, v in sdh.items():
        sd["model.prediction_head." + k] = v
    eng = Engine(cfg, sd, "cuda", max_batch=2, max_ctx=64, head_layout="both")
    eng.set_steps(10)
    pos = torch.randn(n, H, generator=g).bfloat16().cuda()
    neg = torch.randn(n, H, generator=g).bfloat16().cuda()
    x0 = torch.randn(n, 64, generator=g).bfloat16().cuda()
    x = x0.clone()
    L = _lib.lib()
    s = torch.cuda.Stream()
    for loop in (0, mode):   # the per-layer launches, then the persistent launch
        L.vv_head_loop(loop)
        assert L.vv_head_loop_active(eng.h, n) == (1 if loop else 0)
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
        print(f"{'persistent launch' if loop else 'per-layer launches'}: whole head sample (cond + adaLN + "
              f"{eng.steps} steps), best of 8 graph replays: {best:.1f} us")
    st = torch.zeros(256 * 64, dtype=torch.int64, device="cuda")
    L.vv_head_loop_stamps(st.data_ptr())
    gr = capture(eng, pos, neg, x, s)   # the stamp pointer is a launch argument
    for _ in range(3):
        x.copy_(x0)
        with torch.cuda.stream(s):
            gr.replay()
        torch.cuda.synchronize()
    L.vv_head_loop_stamps(None)
    eng.check_sync()
    t = st.view(256, 64).cpu().double() * 10e-3   # us
    t0 = t[:, 62].min()
    rel = t - t0
    names = ["operands in LDS", "transform", "gate|up dots", "down rows in regs", "partial in LDS",
             "slab stores issued", "slabs in LDS", "slice stored"]
    phases = [(40, "noisy stored"), (41, "noisy wait released")]
    for li in range(hc.head_layers):
        phases += [(8 * li + k, f"L{li} {nm}") for k, nm in enumerate(names)]
    phases.append((63, "end"))
    print("last step's phases, us from the first workgroup's entry (median / max over workgroups):")
    prev = None
    for k, name in phases:
        col = rel[:, k]
        d = "" if prev is None else f"   +{(col - rel[:, prev]).median():.2f} from the previous phase (median)"
        print(f"  {k:2d} {name:26s} {col.median():9.2f} {col.max():9.2f}{d}")
        prev = k


if __name__ == "__main__":
    main()
