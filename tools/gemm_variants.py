"""Interleaved same-process A/B of library builds on the prefill GEMMs
(k_gemm_xl, the 256 x 256 tile) at the 1.5B projection shapes.

usage: python tools/gemm_variants.py name=path.so [name=path.so ...] [--m 16384] [--rounds R]

Each build is loaded with its own ctypes handle.  Per round, every build runs
every shape (random operands: cdna_hip_programming.md §5.4 rule 25; A rows
MFMA-fragment packed as the engine's RMSNorm producer writes them for q|k|v and
gate|up); the median / min over rounds and TFLOP/s against the 2.5 PF dense
bf16 peak are printed, with each build's rel L2 vs torch fp32.
"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.weights import mfma_pack  # noqa: E402

PEAK = 2500.0
SHAPES = [("gate|up", 17920, 1536, "silu_mul", 1), ("down", 1536, 8960, "store", 0),
          ("q|k|v", 2048, 1536, "store", 1), ("o", 1536, 1536, "store", 0)]


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, res, args in _lib.EXPORTS:
        if hasattr(L, name):
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
    return L


def main():
    specs = [a.split("=", 1) for a in sys.argv[1:] if "=" in a and not a.startswith("--")]
    M = int(sys.argv[sys.argv.index("--m") + 1]) if "--m" in sys.argv else 16384
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 5
    libs = [(n, load(p)) for n, p in specs]
    P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
    torch.manual_seed(0)
    for name, N, K, epi, apack in SHAPES:
        A = torch.randn(M, K, device="cuda").bfloat16()
        W = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
        Wp, Ap = mfma_pack(W), (mfma_pack(A) if apack else A)
        ref = A.float() @ W.float().t()
        outN = N
        if epi == "silu_mul":
            a_ = ref.view(M, N // 16, 2, 8)
            ref = torch.nn.functional.silu(a_[:, :, 0].reshape(M, -1).bfloat16().float()) * \
                a_[:, :, 1].reshape(M, -1).bfloat16().float()
            outN = N // 2
        Ys = [torch.empty(M, outN, device="cuda", dtype=torch.bfloat16) for _ in libs]

        def run(L, Y):
            L.vv_gemm_tune_apack(apack)
            rc = L.vv_gemm_bf16(M, N, K, P(Ap), K, P(Wp), None, _lib.EPI[epi], P(Y), outN, None, None, None,
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            if rc:
                raise RuntimeError(L.vv_last_error().decode())
        errs = []
        for (_, L), Y in zip(libs, Ys):
            run(L, Y)
            torch.cuda.synchronize()
            errs.append(((Y.float() - ref).norm() / ref.norm()).item())
        times = [[] for _ in libs]
        for _ in range(rounds):
            for i, ((_, L), Y) in enumerate(zip(libs, Ys)):
                run(L, Y)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run(L, Y)
                e1.record()
                e1.synchronize()
                times[i].append(e0.elapsed_time(e1) * 1e3 / 5)
        fl = 2.0 * M * N * K
        line = f"{name:8s} M={M} N={N:5d} K={K:5d} |"
        for (ln, _), t, e in zip(libs, times, errs):
            med = statistics.median(t)
            line += (f" {ln}: med {med:7.1f} us min {min(t):7.1f} = {fl / med / 1e6:6.0f} TF/s "
                     f"({fl / med / 1e6 / PEAK:.3f}) rel {e:.1e} |")
        print(line, flush=True)


if __name__ == "__main__":
    main()
