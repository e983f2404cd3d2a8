"""GEMM / GEMV kernel family (csrc/gemm.hip) vs a plain PyTorch fp32 reference.

Tolerance: the kernels accumulate in fp32 and round once to bf16, so the
result must match fp32(A)·fp32(W)^T rounded to bf16 within 1 bf16 ulp-ish
(rel L2 < 4e-3).
"""
import ctypes

import pytest
import torch

from gpu_util import max_rel, rel_err
from vibevoice_amd import _lib
from vibevoice_amd.weights import mfma_pack

pytestmark = pytest.mark.gpu
dev = "cuda"


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def run(M, N, K, epi, bias=True, res=False, gamma=False, ws_ctx=None):
    g = torch.Generator(device=dev).manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, device=dev, generator=g).bfloat16()
    W = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
    b = (0.1 * torch.randn(N, device=dev, generator=g)).bfloat16() if bias else None
    outN = N // 2 if epi == "silu_mul" else N
    Y = torch.empty(M, outN, device=dev, dtype=torch.float32 if epi == "f32" else torch.bfloat16)
    R = torch.randn(M, outN, device=dev, generator=g).bfloat16() if res else None
    G = torch.randn(outN, device=dev, generator=g).bfloat16() if gamma else None
    Wp = mfma_pack(W) if N % 16 == 0 and K % 32 == 0 else W
    rc = _lib.lib().vv_gemm_bf16(M, N, K, P(A), K, P(Wp), P(b), _lib.EPI[epi], P(Y), outN, P(R), P(G), ws_ctx,
                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    _lib.check(rc, "gemm")
    torch.cuda.synchronize()
    acc = A.float() @ W.float().t()
    if b is not None:
        acc = acc + b.float()
    if epi == "store":
        ref = acc.bfloat16()
    elif epi == "f32":
        ref = acc
    elif epi == "gelu":
        ref = torch.nn.functional.gelu(acc.bfloat16().float()).bfloat16()
    elif epi == "silu_mul":
        a = acc.view(M, N // 16, 2, 8)
        gate, up = a[:, :, 0].reshape(M, N // 2), a[:, :, 1].reshape(M, N // 2)
        ref = (torch.nn.functional.silu(gate.bfloat16().float()).bfloat16().float() * up.bfloat16().float()).bfloat16()
    else:
        y = acc.bfloat16().float()
        if G is not None:
            y = (y * G.float()).bfloat16().float()
        ref = (R.float() + y).bfloat16()
    return Y, ref


@pytest.mark.parametrize("M", [1, 2, 5, 16, 17, 33, 64])
@pytest.mark.parametrize("N,K", [(1536, 1536), (2048, 1536), (1536, 8960), (64, 1536), (1536, 64), (128, 448)])
def test_gemv_store(M, N, K):
    Y, ref = run(M, N, K, "store")
    assert rel_err(Y, ref) < 4e-3 and max_rel(Y, ref) < 2e-2


@pytest.mark.parametrize("M", [65, 200, 3200])
@pytest.mark.parametrize("N,K", [(128, 32), (32, 128), (512, 128), (64, 256), (2048, 1536)])
def test_tiled_store(M, N, K):
    Y, ref = run(M, N, K, "store")
    assert rel_err(Y, ref) < 4e-3


@pytest.mark.parametrize("M", [2, 16, 300])
@pytest.mark.parametrize("epi", ["gelu", "silu_mul", "f32", "res"])
def test_epilogues(M, epi):
    Y, ref = run(M, 1024, 512, epi, bias=epi != "silu_mul", res=epi == "res", gamma=epi == "res")
    assert rel_err(Y, ref) < 5e-3


def test_shape_rejected():
    with pytest.raises(RuntimeError):
        run(4, 100, 64, "store")


@pytest.mark.parametrize("M,N,K,weighted", [(2, 17920, 1536, True), (16, 1024, 2048, True), (5, 64, 1536, False),
                                            (40, 256, 512, True), (96, 256, 256, True)])
def test_fused_rmsnorm_producer(M, N, K, weighted):
    """XF_NORM A transform (input_layernorm / ConvRMSNorm / adaLN-free final norm)
    vs torch: y = bf16(bf16(x * rsqrt(mean(x^2) + eps)) * w), then the GEMM."""
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    A = (3 * torch.randn(M, K, device=dev, generator=g)).bfloat16()
    W = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
    nw = (1 + 0.2 * torch.randn(K, device=dev, generator=g)).bfloat16() if weighted else None
    eps = 1e-6
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    rc = _lib.lib().vv_gemm_bf16_norm(M, N, K, P(A), K, P(nw), eps, P(mfma_pack(W)), _lib.EPI["store"], P(Y), N,
                                      None, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    _lib.check(rc, "gemm_norm")
    torch.cuda.synchronize()
    xf = A.float()
    a = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).bfloat16()
    if nw is not None:
        a = (a.float() * nw.float()).bfloat16()
    ref = (a.float() @ W.float().t()).bfloat16()
    e = rel_err(Y, ref)
    print(M, N, K, e)
    assert e < 4e-3


@pytest.mark.parametrize("tpw", [0, 1, 2, 4, 8])
@pytest.mark.parametrize("M,N,epi", [(16, 8208, "store"), (8, 8192, "res"), (12, 17920, "silu_mul"),
                                     (2, 2064, "store")])
def test_gemv_tiles_per_workgroup(tpw, M, N, epi):
    """k_gemv1 with several 16-row weight tiles per workgroup sharing one A
    staging (vv_gemv_tune_tpw; 0 = built-in plan), incl. a ragged last group
    (N = 8208: 513 tiles) and waves that own no tile."""
    L = _lib.lib()
    L.vv_gemv_tune(8, 0, -1, 0, 0)
    L.vv_gemv_tune_tpw(tpw)
    try:
        Y, ref = run(M, N, 1536, epi, bias=epi == "store", res=epi == "res")
    finally:
        L.vv_gemv_tune(0, 0, -1, 0, 0)
        L.vv_gemv_tune_tpw(0)
    assert rel_err(Y, ref) < 5e-3 and max_rel(Y, ref) < 3e-2


@pytest.mark.parametrize("wide", [1, 0])
@pytest.mark.parametrize("M,N,K,epi", [(17, 4096, 1024, "gelu"), (33, 9216, 1536, "silu_mul"),
                                       (64, 17920, 1536, "silu_mul"), (48, 8192, 4608, "res"),
                                       (40, 21504, 1536, "store"), (64, 16400, 1024, "store")])
def test_gemv_wide_rows(wide, M, N, K, epi):
    """16 < M <= 64 with >= 256 weight tiles: k_gemvw (A per K slice held in
    registers across 1-4 tiles, slices reduced in LDS) and, for comparison,
    k_gemv; K blocks that end inside a wave's slice (K = 1024, 4608) and a
    ragged last tile group (N = 16400: 1025 tiles in groups of 4)."""
    L = _lib.lib()
    L.vv_gemv_tune_wide(wide)
    try:
        Y, ref = run(M, N, K, epi, bias=epi != "silu_mul", res=epi == "res")
    finally:
        L.vv_gemv_tune_wide(1)
    assert rel_err(Y, ref) < 5e-3 and max_rel(Y, ref) < 3e-2


@pytest.mark.parametrize("lds", [0, 151552])
@pytest.mark.parametrize("M,N,K,epi", [(16, 1536, 8960, "res"), (16, 1536, 4608, "res"), (8, 2048, 8192, "res"),
                                       (12, 1536, 8960, "store"), (16, 1024, 16384, "gelu")])
def test_gemv_large_lds_staging(lds, M, N, K, epi):
    """M <= 16 long-row GEMVs (B = 8 down projections, split over two
    workgroups): the A slice staged in > 64 KB of LDS (per-kernel opt-in,
    tuning hook) vs the built-in per-wave fragment form; K = 16384 still
    exceeds the LDS limit and takes the fragment form either way."""
    L = _lib.lib()
    L.vv_gemv_tune_lds(lds)
    try:
        Y, ref = run(M, N, K, epi, bias=True, res=epi == "res")
    finally:
        L.vv_gemv_tune_lds(0)
    assert rel_err(Y, ref) < 5e-3 and max_rel(Y, ref) < 3e-2


@pytest.mark.parametrize("M,N,K,epi", [(256, 2048, 1536, "store"), (257, 1536, 1536, "res"), (1000, 1536, 8960, "res"),
                                       (1000, 17920, 1536, "silu_mul"), (4100, 2048, 1536, "store"),
                                       (300, 1024, 512, "gelu"), (640, 512, 128, "f32")])
def test_gemm_big_tile(M, N, K, epi):
    """Prefill-sized GEMMs on the LDS-staged 256 x 256 tile (k_gemm_xl, 4-stage
    ring), the 128 x 128 tile (k_gemm_big, two stages; and its single-stage
    form) vs torch fp32, and vs k_gemm (same K order of MFMA accumulation:
    bit-identical) -- ragged last row tile, every epilogue kind the prefill uses."""
    L = _lib.lib()
    outs = {}
    try:
        for mode in (7, 6, 5, 0):   # k_gemm_xl / k_gemm_big 2 / 1 stages at any tile count; k_gemm
            L.vv_gemm_tune_big(mode)
            outs[mode], ref = run(M, N, K, epi, bias=epi != "silu_mul", res=epi == "res")
    finally:
        L.vv_gemm_tune_big(-1)
    assert rel_err(outs[7], ref) < 5e-3 and rel_err(outs[6], ref) < 5e-3
    assert torch.equal(outs[7], outs[0]) and torch.equal(outs[6], outs[0]) and torch.equal(outs[5], outs[0])


@pytest.mark.parametrize("handoff", [0, 1])
@pytest.mark.parametrize("M", [1, 2, 5])
@pytest.mark.parametrize("epi", ["res", "store", "silu_mul"])
def test_gemv_small_m_splitk(handoff, M, epi):
    """The M < 8 split-K plan (LM down projection: 96 tiles x K 8,960, two
    workgroups per tile) with the residual epilogue and under both hand-off forms
    (0: plain stores + agent release/acquire fences, 1: sc1 write-through), vs
    torch fp32; the split-K result must equal the unsplit one bit for bit."""
    L = _lib.lib()
    N, K = (3072, 8960) if epi == "silu_mul" else (1536, 8960)
    try:
        L.vv_gemv_tune(0, 2, handoff, 0, 0)          # 2 K splits
        Y2, ref = run(M, N, K, epi, bias=epi != "silu_mul", res=epi == "res")
        L.vv_gemv_tune(0, 1, -1, 0, 0)               # one workgroup per tile
        Y1, _ = run(M, N, K, epi, bias=epi != "silu_mul", res=epi == "res")
    finally:
        L.vv_gemv_tune(0, 0, -1, 0, 0)
    assert rel_err(Y2, ref) < 4e-3 and max_rel(Y2, ref) < 3e-2
    assert rel_err(Y1, ref) < 4e-3

