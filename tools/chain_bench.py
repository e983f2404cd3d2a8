"""Time the diffusion head (vv_diffusion_sample, S steps) per-op vs persistent
chain (chain.hip), graph-replayed, at the real 1.5B head shapes.
usage: python tools/chain_bench.py [n ...]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_gpu_head import real_head_sd  # noqa: E402
from tiny import tiny_config  # noqa: E402
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.engine import Engine  # noqa: E402
from vibevoice_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    # --lib <so>: another build (tools/build_variant.sh); --timeline: the per-op stamps
    # of one launch (needs the default one-workgroup-per-CU grid: the stamp buffer is sized by CUs)
    args = sys.argv[1:]
    if "--lib" in args:
        i = args.index("--lib")
        _lib.LIB_PATH = os.path.abspath(args[i + 1])
        del args[i:i + 2]
    timeline = "--timeline" in args
    args = [a for a in args if a != "--timeline"]
    ns = [int(a) for a in args] or [1, 4, 8]
    g = torch.Generator().manual_seed(21)
    sd_head, hc, H = real_head_sd(g)
    cfg = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    sd = synthetic_state_dict(cfg, seed=0, device="cpu", mode="test", with_acoustic_encoder=False)
    for k, v in sd_head.items():
        sd["model.prediction_head." + k] = v
    eng = Engine(cfg, sd, "cuda", max_batch=8, max_ctx=64)
    eng.set_steps(10)
    L = _lib.lib()
    for n in ns:
        pos = torch.randn(n, H, generator=g).bfloat16().cuda()
        neg = torch.randn(n, H, generator=g).bfloat16().cuda()
        x = torch.randn(n, 64, generator=g).bfloat16().cuda()
        for mode, u in ((0, 8), (1, 4), (1, 8), (2, 8)):
            L.vv_chain_tune(mode)
            L.vv_chain_tune_u(u)
            eng.diffusion_sample(pos, neg, x, 1.3)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                eng.diffusion_sample(pos, neg, x, 1.3)
            for _ in range(3):
                gr.replay()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    gr.replay()
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
            err = L.vv_chain_error(eng.h)
            print(f"n={n} mode={mode} u={u}: {best:8.1f} us per diffusion_sample (S=10)  err={err}", flush=True)
    if not timeline:
        return
    # per-op timeline of one chain launch (n = first n): last signal of op j-1 ->
    # first workgroup past its wait for op j (hand-off latency), and op spans
    n = ns[0]
    nops = 10 * (2 + 2 * hc.head_layers)
    G = torch.cuda.get_device_properties(0).multi_processor_count
    pos = torch.randn(n, H, generator=g).bfloat16().cuda()
    neg = torch.randn(n, H, generator=g).bfloat16().cuda()
    x = torch.randn(n, 64, generator=g).bfloat16().cuda()
    for mode in (1, 2):
        L.vv_chain_tune(mode)
        L.vv_chain_tune_u(8)
        st = torch.zeros(G * nops * 4, dtype=torch.int64, device="cuda")
        eng.diffusion_sample(pos, neg, x, 1.3)
        torch.cuda.synchronize()
        L.vv_chain_stamps(ctypes.c_void_p(st.data_ptr()))
        eng.diffusion_sample(pos, neg, x, 1.3)
        torch.cuda.synchronize()
        L.vv_chain_stamps(None)
        s = st.view(G, nops, 4).cpu().double() * 10.0   # 100 MHz -> ns
        t0 = s[:, 0, 0][s[:, 0, 0] > 0].min()
        print(f"mode {mode}: op  ready_first  end_last  (us from launch start)  handoff  span")
        prev_end = None
        for j in range(nops):
            rdy = s[:, j, 1]
            end = s[:, j, 2]
            rdy = rdy[rdy > 0]
            end = end[end > 0]
            if rdy.numel() == 0 or end.numel() == 0:
                continue
            r0, e1 = (rdy.min() - t0) / 1e3, (end.max() - t0) / 1e3
            ho = (r0 - prev_end) if prev_end is not None else 0.0
            if j < 12 or j >= nops - 2:
                print(f"  {j:3d}  {r0:9.2f}  {e1:9.2f}   handoff {ho:6.2f}  span {e1 - r0:6.2f}")
            prev_end = e1
    L.vv_chain_tune(0)
    L.vv_chain_tune_u(8)


if __name__ == "__main__":
    main()
