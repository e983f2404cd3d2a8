"""Prefill-shaped GEMM throughput (vv_gemm_bf16, EPI_STORE): the 256 x 256 tile
(k_gemm_xl, A rows plain or MFMA-fragment packed) vs the 128 x 128 tile
(k_gemm_big<2>).  usage: python tools/gemm_bench.py [M] [--only xl]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.weights import mfma_pack  # noqa: E402

PEAK = 2500.0


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 16384
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    check = True
    if "--lib" in sys.argv:   # another build (ablation variants: results not checked)
        import ctypes as ct
        _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
        probe = ct.CDLL(_lib.LIB_PATH)
        _lib.EXPORTS = [e for e in _lib.EXPORTS if hasattr(probe, e[0])]
        check = False
    L = _lib.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for N, K, name in ((17920, 1536, "gate|up"), (1536, 8960, "down"), (2048, 1536, "q|k|v"), (1536, 1536, "o")):
        A = torch.randn(M, K, device="cuda").bfloat16()
        Ap = mfma_pack(A)
        W = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
        Wp = mfma_pack(W)
        Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = None
        for label, mode, apack in (("xl", 3, 0), ("xl+apack", 3, 1), ("big2", 2, 0)):
            if only and label != only:
                continue
            L.vv_gemm_tune_big(mode)
            L.vv_gemm_tune_apack(apack)
            src = Ap if apack else A

            def run():
                _lib.check(L.vv_gemm_bf16(M, N, K, ctypes.c_void_p(src.data_ptr()), K, ctypes.c_void_p(Wp.data_ptr()),
                                          None, 0, ctypes.c_void_p(Y.data_ptr()), N, None, None, None, st), "gemm")
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = Y.clone()
            elif check:
                assert torch.equal(Y, ref), f"{label} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) / 10 * 1e3
            tf = 2.0 * M * N * K / us / 1e6
            print(f"{name:8s} M={M} N={N} K={K} {label:9s} {us:9.1f} us  {tf:7.1f} TF/s  {tf / PEAK:.3f} of peak", flush=True)
    L.vv_gemm_tune_big(-1)
    L.vv_gemm_tune_apack(0)


if __name__ == "__main__":
    main()
