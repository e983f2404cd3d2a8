"""Where a long-context decode attention launch's time goes, in the LM pass as
the loop runs it (graph-replayed vv_lm_forward, 1.5B layer shapes, 2 layers):
row 0 attends `ctx` keys (synthetic K/V), row 1 (the negative stream) a short
context.  Per-workgroup s_memrealtime stamps (10 ns ticks) of the last layer's
attention launch: start -> this workgroup's K/V/Q landed -> its waves done ->
(group / split merge) stored.

usage: python tools/attn_long_stamps.py [--group N] [ctx ...]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from gpu_util import kv_synthetic  # noqa: E402
from tiny import tiny_config  # noqa: E402
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.engine import Engine  # noqa: E402
from vibevoice_amd.weights import synthetic_state_dict  # noqa: E402

I32 = dict(dtype=torch.int32, device="cuda")


def main():
    args = sys.argv[1:]
    group = None
    if "--group" in args:   # vv_attn_group cap (diagnostic): at most this many splits per (row, kv head)
        i = args.index("--group")
        group = int(args[i + 1])
        args = args[:i] + args[i + 2:]
    ctxs = [int(x) for x in args] or [65000, 32000, 16000]
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    cfg.decoder_config["max_position_embeddings"] = 65536
    sd = synthetic_state_dict(cfg, seed=3, device="cpu", mode="test", with_acoustic_encoder=False)
    eng = Engine(cfg, sd, "cuda", max_batch=1, max_ctx=65040, valid_ids=[1, 2, 3, 4])
    L = _lib.lib()
    if group is not None:
        L.vv_attn_group(group)
    x = torch.randn(2, 1536, device="cuda").bfloat16()
    slots = torch.tensor([0, 1], **I32)
    oi = torch.zeros(1, **I32)
    hid = torch.empty(1, 1536, dtype=torch.bfloat16, device="cuda")
    lg = torch.empty(1, 4, dtype=torch.float32, device="cuda")
    st = torch.zeros(2048, 4, dtype=torch.int64, device="cuda")
    for ctx in ctxs:
        kv_synthetic(eng, torch.tensor([0], **I32), 0, ctx, seed=1)
        kv_synthetic(eng, torch.tensor([1], **I32), 0, 200, seed=2)
        pos = torch.tensor([ctx, 200], **I32)
        s = torch.cuda.Stream()
        L.vv_attn_stamps(ctypes.c_void_p(st.data_ptr()))
        eng.lm_forward(x, slots, pos, oi, hid, lg, max_pos=65039)
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            g.capture_begin(capture_error_mode="thread_local")
            eng.lm_forward(x, slots, pos, oi, hid, lg, max_pos=65039, stream=s)
            g.capture_end()
        L.vv_attn_stamps(None)
        for _ in range(3):
            st.zero_()
            g.replay()
            torch.cuda.synchronize()
        raw = st.cpu()
        t = raw.double() * 10e-3
        act = t[:, 1] > 0
        # placement (slot 3 at entry: bit 62 | XCC_ID << 32 | HW_ID), keyed workgroups
        hw = raw[act.nonzero().flatten(), 3]
        marked = (hw >> 62) & 1 == 1
        if marked.any():
            h = hw[marked]
            key = (((h >> 32) & 0xF) << 8) | (((h >> 13) & 0x7) << 5) | (((h >> 12) & 1) << 4) | ((h >> 8) & 0xF)
            u, c = torch.unique(key, return_counts=True)
            print(f"   placement: {int(marked.sum())} keyed workgroups on {len(u)} distinct CUs "
                  f"(max {int(c.max())} per CU, {int((c > 1).sum())} CUs with more than one); per XCC: "
                  f"{torch.bincount(((h >> 32) & 0xF).long(), minlength=8).tolist()}")
            t[act.nonzero().flatten()[marked], 3] = 0
        a = t[act]
        t0 = t[t[:, 0] > 0, 0].min()
        end = torch.where(a[:, 3] > 0, a[:, 3], a[:, 2])
        mer = a[:, 3] > 0
        print(f"ctx {ctx}: {int((t[:, 0] > 0).sum())} workgroups started, {int(act.sum())} with keys, "
              f"{int(mer.sum())} merging | start spread {(a[:, 0] - t0).max():.2f} us | loads landed "
              f"med {(a[:, 1] - a[:, 0]).median():.2f} max {(a[:, 1] - a[:, 0]).max():.2f} | waves done after "
              f"landing med {(a[:, 2] - a[:, 1]).median():.2f} max {(a[:, 2] - a[:, 1]).max():.2f} | "
              f"merge {(a[mer, 3] - a[mer, 2]).median() if mer.any() else 0:.2f} | "
              f"last workgroup done {(end - t0).max():.2f} us after the first start", flush=True)
        q = torch.quantile(end - t0, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
        print(f"   done-time quantiles 10/50/90 %: {q[0]:.2f} {q[1]:.2f} {q[2]:.2f} us; "
              f"start quantiles: {torch.quantile(a[:, 0] - t0, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64)).tolist()}")


if __name__ == "__main__":
    main()
