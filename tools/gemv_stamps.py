"""Where a decode GEMV's time goes, measured the way the generate loop runs it:
graph-replayed back-to-back launches over weight copies that overflow the
Infinity Cache, each launch writing per-workgroup s_memrealtime stamps (10 ns
ticks): dispatch spread, A staging, weight stream, epilogue, and the gap
between the last workgroup of one launch and the first of the next.

usage: python tools/gemv_stamps.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.weights import mfma_pack  # noqa: E402

SHAPES = [("lm.gu", 2, 17920, 1536, "silu_mul"), ("head.gu", 2, 9216, 1536, "silu_mul"),
          ("lm.down", 2, 1536, 8960, "res"), ("lm.o", 2, 1536, 1536, "res"), ("lm.qkv", 2, 2048, 1536, "store"),
          ("codec.fc1", 1, 8192, 2048, "gelu"), ("codec.fc2", 1, 2048, 8192, "res"),
          ("lm.gu+norm", 2, 17920, 1536, "silu_mul"), ("lm.gu.b8", 16, 17920, 1536, "silu_mul"),
          ("lm.gu.b8+norm", 16, 17920, 1536, "silu_mul"), ("head.gu.b8+norm", 16, 9216, 1536, "silu_mul")]


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def main():
    if "--lib" in sys.argv:   # another build of the library (tools/build_variant.sh)
        _lib.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
    L = _lib.lib()
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    # --tune nw,u,tpw[;nw,u,tpw...]: GEMV plans to stamp (vv_gemv_tune / vv_gemv_tune_tpw), built-in first
    tunes = [None] + ([tuple(int(x) for x in t.split(",")) for t in sys.argv[sys.argv.index("--tune") + 1].split(";")]
                      if "--tune" in sys.argv else [])
    if len(tunes) > 1:
        tunes.append(None)    # the built-in plan again, last (the first configuration of a shape can read slow)
    for (name, M, N, K, epi), tune in [(sh, t) for sh in SHAPES for t in tunes]:
        if only and name not in only:
            continue
        if tune is None:
            L.vv_gemv_tune(0, 0, -1, 0, 0)
            L.vv_gemv_tune_tpw(0)
        else:
            L.vv_gemv_tune(tune[0], 1, 1, 0, tune[1])
            L.vv_gemv_tune_tpw(tune[2])
        norm = name.endswith("+norm")
        if tune is not None:
            name = f"{name}[nw{tune[0]} u{tune[1]} tpw{tune[2]}]"
        ncopy = max(2, (512 << 20) // (N * K * 2) + 1)
        Ws = [mfma_pack((torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()) for _ in range(ncopy)]
        A = torch.randn(M, K, device="cuda").bfloat16()
        outN = N // 2 if epi == "silu_mul" else N
        Y = torch.empty(M, outN, device="cuda", dtype=torch.bfloat16)
        R = torch.randn(M, outN, device="cuda").bfloat16() if epi == "res" else None
        reps = max(16, 2 * ncopy)
        G = N // 16
        st = torch.zeros(reps, G, 4, dtype=torch.int64, device="cuda")

        nw_ = (1 + 0.1 * torch.randn(K, device="cuda")).bfloat16()

        def run(i):
            L.vv_gemv_stamps(ctypes.c_void_p(st[i].data_ptr()))
            sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            if norm:
                _lib.check(L.vv_gemm_bf16_norm(M, N, K, P(A), K, P(nw_), 1e-6, P(Ws[i % ncopy]), _lib.EPI[epi],
                                               P(Y), outN, None, sp))
            else:
                _lib.check(L.vv_gemm_bf16(M, N, K, P(A), K, P(Ws[i % ncopy]), None, _lib.EPI[epi], P(Y), outN,
                                          P(R), None, None, sp))
            L.vv_gemv_stamps(None)
        run(0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(reps):
                run(i)
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        s = st.cpu().double() * 10e-3                                 # us
        G = int((s[0, :, 0] > 0).sum())                               # launched workgroups (tiles per group, K splits)
        s = s[reps // 4:, :G]                                         # steady state
        first = s[:, :, 0].min(1).values
        last_end = s[:, :, 3].max(1).values
        span = (last_end - first).mean().item()
        gap = (first[1:] - last_end[:-1]).mean().item()
        spread = (s[:, :, 0].max(1).values - first).mean().item()
        stg = (s[:, :, 1] - s[:, :, 0]).mean().item()
        stm = (s[:, :, 2] - s[:, :, 1]).mean().item()
        epi_ = (s[:, :, 3] - s[:, :, 2]).mean().item()
        wg = (s[:, :, 3] - s[:, :, 0]).mean().item()
        # time from first start until 90% of workgroups have finished (tail effect)
        ends = (s[:, :, 3] - first[:, None]).sort(1).values
        p90 = ends[:, int(0.9 * G) - 1].mean().item()
        mb = N * K * 2 / 1e6
        print(f"{name:9s} WGs {G:5d} {mb:5.1f} MB: span {span:5.2f} us (gap {gap:4.2f}) | start spread {spread:4.2f} "
              f"| per WG: staging {stg:4.2f} stream {stm:4.2f} epilogue {epi_:4.2f} total {wg:5.2f} "
              f"| 90% done {p90:5.2f} | {mb / (span + gap) * 1e-3:4.2f} TB/s", flush=True)
        del Ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
