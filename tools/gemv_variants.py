"""Interleaved same-process A/B of library builds on the decode GEMV shapes.

usage: python tools/gemv_variants.py name=path.so [name=path.so ...] [--rounds R]

Each build is loaded with its own ctypes handle (distinct file paths, so their
kernels register separately); every round times every build on every shape
(graph-replayed back-to-back launches over weight copies that overflow the
Infinity Cache, as tools/gemv_sweep.py), and the per-shape median and min over
rounds are printed (cdna_hip_programming.md §5.4 rule 24).  Each build's output
is checked against the first build's (bitwise) and a torch fp32 reference.
"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.weights import mfma_pack  # noqa: E402

SHAPES = [  # name, M, N, K, epi, norm
    ("lm.gu+norm", 2, 17920, 1536, "silu_mul", True), ("lm.gu.b8+norm", 16, 17920, 1536, "silu_mul", True),
    ("lm.qkv+norm", 2, 2048, 1536, "store", True), ("lm.qkv.b8+norm", 16, 2048, 1536, "store", True),
    ("head.gu+norm", 2, 9216, 1536, "silu_mul", True), ("head.gu.b8+norm", 16, 9216, 1536, "silu_mul", True),
    ("lm.down", 2, 1536, 8960, "res", False), ("lm.down.b8", 16, 1536, 8960, "res", False),
    ("lm.o", 2, 1536, 1536, "res", False), ("head.down", 2, 1536, 4608, "res", False),
    ("codec.fc1+norm", 1, 8192, 2048, "gelu", True), ("codec.fc2", 1, 2048, 8192, "res", False),
]


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, res, args in _lib.EXPORTS:
        if hasattr(L, name):
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
    return L


def main():
    specs = [a.split("=", 1) for a in sys.argv[1:] if "=" in a]
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 5
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    libs = [(n, load(p)) for n, p in specs]
    dev = "cuda"
    torch.manual_seed(0)
    for name, M, N, K, epi, norm in SHAPES:
        if only and name not in only:
            continue
        ncopy = max(2, (512 << 20) // (N * K * 2) + 1)
        Ws = [mfma_pack((torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()) for _ in range(ncopy)]
        A = torch.randn(M, K, device=dev).bfloat16()
        outN = N // 2 if epi == "silu_mul" else N
        R = torch.randn(M, outN, device=dev).bfloat16() if epi == "res" else None
        nw_ = (1 + 0.1 * torch.randn(K, device=dev)).bfloat16() if norm else None
        Ys = [torch.empty(M, outN, device=dev, dtype=torch.bfloat16) for _ in libs]

        def run(L, W, Y):
            sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            if norm:
                rc = L.vv_gemm_bf16_norm(M, N, K, P(A), K, P(nw_), 1e-6, P(W), _lib.EPI[epi], P(Y), outN, None, sp)
            else:
                rc = L.vv_gemm_bf16(M, N, K, P(A), K, P(W), None, _lib.EPI[epi], P(Y), outN, P(R), None, None, sp)
            if rc:
                raise RuntimeError(L.vv_last_error().decode())

        graphs = []
        reps = max(16, 2 * len(Ws))
        for (ln, L), Y in zip(libs, Ys):
            run(L, Ws[0], Y)
            run(L, Ws[1], Y)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(reps):
                    run(L, Ws[i % len(Ws)], Y)
            graphs.append(g)
        for (ln, L), Y in zip(libs, Ys):
            run(L, Ws[0], Y)
        torch.cuda.synchronize()
        same = [torch.equal(Y, Ys[0]) for Y in Ys]
        times = [[] for _ in libs]
        for _ in range(rounds):
            for i, g in enumerate(graphs):
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                times[i].append(e0.elapsed_time(e1) * 1e3 / reps)
        line = f"{name:16s} M={M:3d} N={N:6d} K={K:5d} |"
        for (ln, _), t, sm in zip(libs, times, same):
            line += f" {ln}: med {statistics.median(t):6.2f} min {min(t):6.2f} us{'' if sm else ' (DIFFERS)'} |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
