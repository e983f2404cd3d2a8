"""Where a fused head FFN layer's time goes (csrc/head_ffn.hip), measured the
way the loop runs it: the 1.5B head (seeded weights, real shapes) sampled for
n = 1 inside a graph replay, every layer launch writing per-workgroup
s_memrealtime stamps (10 ns ticks) of its last launch: entry, transformed A
rows ready, gate|up done, slab written + arrival, grid wait released + slabs loaded, end.

usage: python tools/head_ffn_stamps.py [n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.engine import Engine  # noqa: E402
from vibevoice_amd.weights import synthetic_state_dict  # noqa: E402
from test_gpu_head import real_head_sd  # noqa: E402
from tiny import tiny_config  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    g = torch.Generator().manual_seed(5)
    sdh, hc, H = real_head_sd(g)
    cfg = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    sd = synthetic_state_dict(cfg, seed=0, device="cpu", mode="test", with_acoustic_encoder=False)
    for k, v in sdh.items():
        sd["model.prediction_head." + k] = v
    eng = Engine(cfg, sd, "cuda", max_batch=4, max_ctx=64)
    eng.set_steps(10)
    pos = torch.randn(n, H, generator=g).bfloat16().cuda()
    neg = torch.randn(n, H, generator=g).bfloat16().cuda()
    x0 = torch.randn(n, 64, generator=g).bfloat16().cuda()
    x = x0.clone()
    eng.diffusion_sample(pos, neg, x, 1.3)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        gr.capture_begin(capture_error_mode="thread_local")
        eng.diffusion_sample(pos, neg, x, 1.3, stream=s)
        gr.capture_end()
    st = torch.zeros(256 * 8, dtype=torch.int64, device="cuda")
    L = _lib.lib()
    for rep in range(6):
        L.vv_head_ffn_stamps(st.data_ptr() if rep == 5 else None)
        # the stamp pointer is a launch argument: re-capture for the stamped replay
        if rep == 5:
            with torch.cuda.stream(s):
                gr = torch.cuda.CUDAGraph()
                gr.capture_begin(capture_error_mode="thread_local")
                eng.diffusion_sample(pos, neg, x, 1.3, stream=s)
                gr.capture_end()
        x.copy_(x0)
        gr.replay()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(s)
        with torch.cuda.stream(s):
            gr.replay()
        ev1.record(s)
        torch.cuda.synchronize()
        print(f"replay {rep}: whole head sample {ev0.elapsed_time(ev1) * 1e3:.1f} us")
    L.vv_head_ffn_stamps(None)
    eng.check_sync()
    raw = st.view(256, 8).cpu()
    h = raw[:, 6]
    key = (((h >> 32) & 0xF) << 8) | (((h >> 13) & 0x7) << 5) | (((h >> 12) & 1) << 4) | ((h >> 8) & 0xF)
    u, inv, c = torch.unique(key, return_inverse=True, return_counts=True)
    shared = c[inv] > 1
    print(f"placement: 256 workgroups on {len(u)} distinct CUs (max {int(c.max())} per CU); per XCC "
          f"{torch.bincount(((h >> 32) & 0xF).long(), minlength=8).tolist()}")
    t = raw.double() * 10e-3   # us
    if shared.any():
        print(f"  arrival of workgroups sharing a CU: median {(t[shared, 3] - t[:, 0].min()).median():.2f} us, "
              f"alone: {(t[~shared, 3] - t[:, 0].min()).median():.2f} us")
    t0 = t[:, 0].min()
    rel = t - t0
    names = ["entry", "A ready", "gate|up done", "arrived", "slabs in", "end"]
    print("stamps of the last layer launch (us from the first workgroup's entry):")
    for k, nm in enumerate(names):
        c = rel[:, k]
        print(f"  {nm:14s} min {c.min():6.2f}  median {c.median():6.2f}  max {c.max():6.2f}")
    print(f"  per workgroup: A staging {(t[:, 1] - t[:, 0]).median():.2f}, gate|up {(t[:, 2] - t[:, 1]).median():.2f}, "
          f"down + slab {(t[:, 3] - t[:, 2]).median():.2f}, wait + slab loads {(t[:, 4] - t[:, 3]).median():.2f}, "
          f"reduce {(t[:, 5] - t[:, 4]).median():.2f}")
    print(f"  last arrival -> first slabs in {rel[:, 4].min() - rel[:, 3].max():.2f}; span {rel[:, 5].max():.2f}")


if __name__ == "__main__":
    main()
