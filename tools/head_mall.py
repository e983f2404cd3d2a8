"""Does the diffusion head's per-step weight set (adaLN 66 MB + 4 x gate|up 28 MB
+ 4 x down 14 MB = 236 MB at 1.5B) stay in the 256 MiB Infinity Cache across
the S diffusion steps?  Replays the head's GEMV sequence (same shapes, random
weights) S times in one graph and reports us per diffusion step.  Run it with
two builds of the library (nt / default-policy weight loads) to compare:
  python tools/head_mall.py [path/to/libvibevoice_hip.so]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.weights import mfma_pack  # noqa: E402

ARGS = [a for a in sys.argv[1:] if not a.startswith("--")]
if ARGS:
    _lib.LIB_PATH = os.path.abspath(ARGS[0])
WITH_ADA = "--no-ada" not in sys.argv   # the loop now computes all steps' adaLN rows once per token


def main():
    L = _lib.lib()
    H, I, NLY, S = 1536, 4608, 4, 10
    M = 2
    dev = "cuda"

    def W(n, k):
        return mfma_pack((torch.randn(n, k, device=dev) / k ** 0.5).bfloat16())
    ada = W((3 * NLY + 2) * H, H)
    gus = [W(2 * I, H) for _ in range(NLY)]
    downs = [W(H, I) for _ in range(NLY)]
    x = torch.randn(M, H, device=dev).bfloat16()
    vec = torch.randn(H, device=dev).bfloat16()
    mod = torch.empty(M, (3 * NLY + 2) * H, device=dev, dtype=torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(H, device=dev)).bfloat16()
    hbuf = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
    res = torch.randn(M, H, device=dev).bfloat16()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def step():
        sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        if WITH_ADA:
            _lib.check(L.vv_gemm_bf16(M, ada.shape[0], H, P(x), H, P(ada), None, _lib.EPI["store"], P(mod),
                                      mod.shape[1], None, None, None, sp))
        for l in range(NLY):
            _lib.check(L.vv_gemm_bf16_norm(M, 2 * I, H, P(x), H, P(nw), 1e-5, P(gus[l]), _lib.EPI["silu_mul"], P(hbuf),
                                           I, None, sp))
            _lib.check(L.vv_gemm_bf16(M, H, I, P(hbuf), I, P(downs[l]), None, _lib.EPI["res"], P(x), H, P(res), None,
                                      None, sp))
    step()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(S):
            step()
    junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    for rep in range(3):
        junk.fill_(rep)                    # flush the Infinity Cache between token-level replays
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        print(f"{os.path.basename(_lib.LIB_PATH)}: {e0.elapsed_time(e1) * 1e3 / S:8.2f} us per diffusion step "
              f"({'9 launches, 236' if WITH_ADA else '8 launches, 170'} MB of weights)", flush=True)


if __name__ == "__main__":
    main()
