"""Per-rank cost of the TP-sharded VibeVoice-Large diffusion head (configs[3]),
measured on ONE MI355X: the head (H 3,584, FFN 10,752, 4 layers, S = 10, CFG
1.3, seeded weights at real shapes) sampled for n diffusing rows
  * at TP = 1 (one engine, Engine.diffusion_sample), and
  * as a TP group of `tp` engines on the same GPU (vv_diffusion_sample_group:
    the ranks' shards interleaved layer by layer, an on-device row sum standing
    in for the per-layer all-reduce),
each captured into a hipGraph and replayed (best of 20).  The group's replay
runs every rank's kernels back to back, so per-rank head time = (group time -
the sums) / tp; run it under `rocprofv3 --kernel-trace --stats` for the sums'
share (k_sum_rows).  The RCCL all-reduce of [2n, 3,584] bf16 per layer (14-57
KB) replaces the sum on a real TP group.

usage: python tools/tp_head_time.py [tp] [n ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from vibevoice_amd.engine import Engine  # noqa: E402
from vibevoice_amd.weights import synthetic_state_dict  # noqa: E402
from tiny import tiny_config  # noqa: E402

LARGE = dict(hidden=3584, heads=28, kv_heads=4, inter=18944, vocab=152064)


def best_replay(fn, reps=20):
    s = torch.cuda.Stream()
    fn(s)   # eager warm-up (builds plans outside the capture)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        gr.capture_begin(capture_error_mode="thread_local")
        fn(s)
        gr.capture_end()
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            gr.replay()
            e1.record(s)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3)
    return best


def main():
    tp = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ns = [int(v) for v in sys.argv[2:]] or [1, 4]
    cfg = tiny_config(layers=1, **LARGE)
    sd = synthetic_state_dict(cfg, seed=22, device="cpu", mode="test", with_acoustic_encoder=False)
    mb = max(ns)
    full = Engine(cfg, sd, "cuda", max_batch=mb, max_ctx=64)
    group = [Engine(cfg, sd, "cuda", max_batch=mb, max_ctx=64, tp_rank=r, tp_size=tp, tp_head=True) for r in range(tp)]
    full.set_steps(10)
    group[0].set_steps(10)
    g = torch.Generator().manual_seed(3)
    for n in ns:
        pos = torch.randn(n, 3584, generator=g).bfloat16().cuda()
        neg = torch.randn(n, 3584, generator=g).bfloat16().cuda()
        x = torch.randn(n, 64, generator=g).bfloat16().cuda()
        t1 = best_replay(lambda s: full.diffusion_sample(pos, neg, x, 1.3, stream=s))
        tg = best_replay(lambda s: group[0].diffusion_sample_group(group[1:], pos, neg, x, 1.3, stream=s))
        print(f"Large head n={n} (rows {2 * n}), S=10: TP=1 {t1:.1f} us per token; TP={tp} group on one GPU "
              f"{tg:.1f} us = {tg / tp:.1f} us per rank incl. the sums (x {tp} ranks back to back)", flush=True)
    full.check_sync()


if __name__ == "__main__":
    main()
