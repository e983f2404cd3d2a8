"""MFMA utilisation of the diffusion head's GEMMs vs batch (north-star target:
>= 40 % bf16 MFMA utilisation on the diffusion-head GEMM, BASELINE.json).

One configuration per process (so a rocprofv3 --pmc pass attributes every
dispatch to it):
  python tools/head_mfma.py --n N        whole vv_diffusion_sample for N diffusing
                                         rows (M = 2N GEMV rows), real 1.5B head
  python tools/head_mfma.py --lmffn       the LM MLP block at B = 1 (k_lm_ffn, 5 x 28 launches)
  python tools/head_mfma.py --m M        the head's gate|up (N 9216, K 1536) and
                                         down (N 1536, K 4608) shapes at M rows
                                         through vv_gemm_bf16 (the dispatch the
                                         engine makes at that M: k_gemv* / k_gemm /
                                         k_gemm_big)
Each runs 5 times.  Summarise with tools/pmc_mfma.py (see profiles/r02_head_mfma.txt)."""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from vibevoice_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--m", type=int, default=0)
    ap.add_argument("--lmffn", action="store_true", help="the LM MLP block at B = 1 as the loop runs it (k_lm_ffn)")
    args = ap.parse_args()
    L = _lib.lib()
    if args.lmffn:
        from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
        model = VibeVoiceForConditionalGenerationInference.from_pretrained("synthetic:1.5B", device_map="cuda",
                                                                            synthetic_seed=0, max_batch=1, max_ctx=256)
        assert L.vv_lm_ffn_active(model.engine.h, 2) == 1
        x = (torch.randn(2, 1536, device="cuda") * 0.5).bfloat16()
        act = torch.empty(2, 8960, device="cuda", dtype=torch.bfloat16)
        sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(L.vv_lm_mlp_replay(model.engine.h, 2, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(act.data_ptr()),
                                      5, sp), "lm_mlp_replay")
        torch.cuda.synchronize()
        print("lmffn: M=2 rows, 5 passes over the 28 layers' MLP blocks")
        return
    if args.n:
        from test_gpu_head import real_head_sd
        from tiny import tiny_config
        from vibevoice_amd.engine import Engine
        from vibevoice_amd.weights import synthetic_state_dict
        g = torch.Generator().manual_seed(3)
        sd_head, hc, H = real_head_sd(g)
        cfg = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
        sd = synthetic_state_dict(cfg, seed=0, device="cpu", mode="test", with_acoustic_encoder=False)
        for k, v in sd_head.items():
            sd["model.prediction_head." + k] = v
        eng = Engine(cfg, sd, "cuda", max_batch=max(args.n, 1), max_ctx=64)
        eng.set_steps(10)
        n = args.n
        pos = torch.randn(n, H, generator=g).bfloat16().cuda()
        neg = torch.randn(n, H, generator=g).bfloat16().cuda()
        x = torch.randn(n, 64, generator=g).bfloat16().cuda()
        for _ in range(5):
            eng.diffusion_sample(pos, neg, x, 1.3)
        torch.cuda.synchronize()
        print(f"head n={n}: M={2 * n} rows, 5 x vv_diffusion_sample(S=10)")
        return
    M = args.m
    for N, K in ((9216, 1536), (1536, 4608)):
        A = torch.randn(M, K, device="cuda").bfloat16()
        W = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
        from vibevoice_amd.weights import mfma_pack
        Wp = mfma_pack(W)
        Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(5):
            _lib.check(L.vv_gemm_bf16(M, N, K, ctypes.c_void_p(A.data_ptr()), K, ctypes.c_void_p(Wp.data_ptr()), None,
                                      _lib.EPI["store"], ctypes.c_void_p(Y.data_ptr()), N, None, None, None, st), "gemm")
        torch.cuda.synchronize()
        ref = A.float() @ W.float().t()
        err = ((Y.float() - ref).norm() / ref.norm()).item()
        print(f"M={M} N={N} K={K}: rel err {err:.2e}")
        assert err < 1e-2


if __name__ == "__main__":
    main()
