"""Where a decode attention launch's time goes: 28 graph-replayed launches over
28 separate KV caches (one per layer, as in the loop), per-workgroup
s_memrealtime stamps (10 ns): start -> K/V/Q landed -> keys done -> output
stored, plus the gap to the next launch.  usage: python tools/attn_stamps.py"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from tests_engine import tiny_engine  # noqa: E402
from vibevoice_amd import _lib  # noqa: E402


def main():
    eng = tiny_engine()
    L = _lib.lib()
    for ctx, stride in ((250, 256), (1000, 1024), (16000, 16000)):   # strides: whole 32-position V blocks
        nq, nh, nkv, NL = 2, 12, 2, 28
        Ks = [torch.randn(nq, nkv, stride, 128, device="cuda").bfloat16() for _ in range(NL)]
        Vs = [torch.randn_like(k) for k in Ks]
        q = torch.randn(nq, nh * 128, device="cuda").bfloat16()
        out = torch.empty_like(q)
        slots = torch.arange(nq, device="cuda", dtype=torch.int32)
        pos = torch.full((nq,), ctx - 1, device="cuda", dtype=torch.int32)
        st = torch.zeros(NL, 1024, 4, dtype=torch.int64, device="cuda")   # >= workgroups per launch

        def run(i):
            L.vv_attn_stamps(ctypes.c_void_p(st[i].data_ptr()))
            _lib.check(L.vv_attention_bf16(nq, nh, nkv, ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(Ks[i].data_ptr()),
                                           ctypes.c_void_p(Vs[i].data_ptr()), nkv * stride * 128, stride * 128,
                                           ctypes.c_void_p(slots.data_ptr()), ctypes.c_void_p(pos.data_ptr()), ctx,
                                           ctypes.c_void_p(out.data_ptr()), eng.h,
                                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
            L.vv_attn_stamps(None)
        run(0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(NL):
                run(i)
        g.replay()
        torch.cuda.synchronize()
        s = st.cpu().double() * 10e-3
        nwg = int((s[0, :, 0] > 0).sum())
        s = s[:, :nwg]
        first = s[:, :, 0].min(1).values
        done = s[:, :, 3] > 0                       # workgroups that stored output (others hand off partials)
        s3 = torch.where(done, s[:, :, 3], s[:, :, 2])
        last = s3.max(1).values
        print(f"ctx {ctx} stride {stride}: {nwg} workgroups/launch | span {(last - first)[1:].mean():.2f} us, gap to next "
              f"{(first[1:] - last[:-1]).mean():.2f} us | per WG: loads {(s[:, :, 1] - s[:, :, 0]).mean():.2f} "
              f"all waves done {(s[:, :, 2] - s[:, :, 1]).mean():.2f} merge+store "
              f"{(s[:, :, 3] - s[:, :, 2])[done].mean():.2f} ({int(done[0].sum())} storing WGs) | "
              f"start spread {(s[:, :, 0].max(1).values - first).mean():.2f}", flush=True)


if __name__ == "__main__":
    main()
