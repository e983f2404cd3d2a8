"""Graph-replayed timing of the decode attention kernel alone (vv_attention_bf16)
at the loop's shapes: 2B query rows (positive + negative), 12 q / 2 kv heads."""
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
    for B, ctx in [(1, 170), (1, 1000), (1, 4000), (1, 16000), (1, 65536), (8, 170), (8, 1000)]:
        nq, nh, nkv = 2 * B, 12, 2
        K = torch.randn(nq, nkv, ctx, 128, device="cuda").bfloat16()
        V = torch.randn_like(K)
        q = torch.randn(nq, nh * 128, device="cuda").bfloat16()
        out = torch.empty_like(q)
        slots = torch.arange(nq, device="cuda", dtype=torch.int32)
        pos = torch.full((nq,), ctx - 1, device="cuda", dtype=torch.int32)

        def run():
            _lib.check(L.vv_attention_bf16(nq, nh, nkv, ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(K.data_ptr()),
                                           ctypes.c_void_p(V.data_ptr()), nkv * ctx * 128, ctx * 128,
                                           ctypes.c_void_p(slots.data_ptr()), ctypes.c_void_p(pos.data_ptr()), ctx,
                                           ctypes.c_void_p(out.data_ptr()), eng.h,
                                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
        run()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(50):
                run()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        kv_bytes = 2 * nq * nkv * ctx * 128 * 2
        print(f"B={B} rows={nq} ctx={ctx:6d}: {us:7.2f} us  KV {kv_bytes / 1e6:7.2f} MB -> "
              f"{kv_bytes / us / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
