"""Causal prefill attention alone (k_attn_pf via vv_attention_bf16, prefill
kernel forced): one slot, nq query rows at positions 0..nq-1, 1.5B layout
(12 q / 2 kv heads).  usage: python tools/attn_pf_bench.py [nq] [--lib other.so]
(ablation builds: results not checked)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from vibevoice_amd import _lib  # noqa: E402


def main():
    nq = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 16384
    if "--lib" in sys.argv:
        _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
        probe = ctypes.CDLL(_lib.LIB_PATH)
        _lib.EXPORTS = [e for e in _lib.EXPORTS if hasattr(probe, e[0])]
    from tests_engine import tiny_engine
    eng = tiny_engine()
    L = _lib.lib()
    nh, nkv = 12, 2
    ctx = (nq + 63) // 64 * 64
    g = torch.Generator(device="cuda").manual_seed(1)
    K = torch.randn(1, nkv, ctx, 128, device="cuda", generator=g).bfloat16()
    VB = torch.randn(1, nkv, ctx // 32, 128, 32, device="cuda", generator=g).bfloat16()
    q = torch.randn(nq, nh * 128, device="cuda", generator=g).bfloat16()
    out = torch.empty_like(q)
    slots = torch.zeros(nq, device="cuda", dtype=torch.int32)
    pos = torch.arange(nq, device="cuda", dtype=torch.int32)
    L.vv_attn_prefill(1)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        _lib.check(L.vv_attention_bf16(nq, nh, nkv, ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(K.data_ptr()),
                                       ctypes.c_void_p(VB.data_ptr()), nkv * ctx * 128, ctx * 128,
                                       ctypes.c_void_p(slots.data_ptr()), ctypes.c_void_p(pos.data_ptr()), ctx,
                                       ctypes.c_void_p(out.data_ptr()), eng.h, st), "attn")
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        run()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 5
    flop = 4.0 * (nq * (nq + 1) / 2) * 128 * nh
    print(f"nq={nq}: {ms:.3f} ms  {flop / ms / 1e9:.1f} TF/s  {flop / ms / 1e9 / 2500:.3f} of peak", flush=True)
    L.vv_attn_prefill(-1)


if __name__ == "__main__":
    main()
