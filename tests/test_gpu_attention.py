"""Decode / prefill attention kernel (k_attn via vv_attention_bf16) vs a plain
PyTorch fp32 reference (softmax(q k^T / sqrt(128)) v, GQA), at the 1.5B head
layout (12 q / 2 kv heads) and the Large layout (28 / 4), cache in the engine's
layout (K [slot][kv_head][ctx][128], V [slot][kv_head][ctx/32][128][32]): single-workgroup
contexts, the in-launch split merge (<= 8 splits of 64 keys), the k_attn_merge pass
(longer), splits of 128 and 192 keys (4 and 8 waves), ragged rows sharing a
launch, and length-1 rows.  Tolerance: rel L2 < 1e-2 (bf16 output)."""
import ctypes

import pytest
import torch

from gpu_util import rel_err
from tests_engine import tiny_engine
from vibevoice_amd import _lib

pytestmark = pytest.mark.gpu
dev = "cuda"


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def run_attention(eng, q, K, V, slots, pos, max_pos_p1):
    nq, nh = q.shape[0], q.shape[1] // 128
    nslot, nkv, ctx, _ = K.shape
    out = torch.empty_like(q)
    # engine layout: V in blocks of 32 positions, each [128 dims][32 positions]
    VB = V.view(nslot, nkv, ctx // 32, 32, 128).transpose(3, 4).contiguous()
    rc = _lib.lib().vv_attention_bf16(nq, nh, nkv, P(q), P(K), P(VB), nkv * ctx * 128, ctx * 128, P(slots), P(pos),
                                      max_pos_p1, P(out), eng.h,
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    _lib.check(rc, "attention")
    return out


def reference(q, K, V, slots, pos):
    nq, nh = q.shape[0], q.shape[1] // 128
    nkv = K.shape[1]
    G = nh // nkv
    out = torch.empty(nq, nh * 128)
    for i in range(nq):
        s, L = int(slots[i]), int(pos[i]) + 1
        qi = q[i].float().view(nh, 128)
        k = K[s, :, :L].float().repeat_interleave(G, 0)       # [nh, L, 128]
        v = V[s, :, :L].float().repeat_interleave(G, 0)
        p = torch.softmax((k @ qi[:, :, None])[..., 0] / 128 ** 0.5, -1)
        out[i] = (p[:, None, :] @ v)[:, 0].reshape(-1)
    return out


@pytest.mark.parametrize("nh,nkv,lens", [(12, 2, [1, 37, 170, 1024]), (12, 2, [1025, 3000, 64]),
                                         (28, 4, [300, 5000]), (12, 2, [65536 // 8]),
                                         (12, 2, [1, 63, 65, 200, 512]),      # <= 8 splits: in-kernel merge
                                         (12, 2, [20000, 5]),                 # 128-key splits, 4 waves
                                         (12, 2, [40000, 700]),               # 192-key splits, 8 waves
                                         (12, 2, [65000, 3]),                 # configs[4]: 64K context
                                         (28, 4, [32768, 17])])               # Large at its 32K limit
def test_attention_vs_torch(nh, nkv, lens):
    eng = tiny_engine()
    g = torch.Generator(device=dev).manual_seed(sum(lens) + nh)
    nslot = len(lens)
    ctx = (max(lens) + 31) // 32 * 32                  # cache capacity: whole 32-position V blocks
    K = torch.randn(nslot, nkv, ctx, 128, device=dev, generator=g).bfloat16()
    V = torch.randn(nslot, nkv, ctx, 128, device=dev, generator=g).bfloat16()
    q = torch.randn(len(lens), nh * 128, device=dev, generator=g).bfloat16()
    slots = torch.arange(nslot, device=dev, dtype=torch.int32)
    pos = torch.tensor([n - 1 for n in lens], device=dev, dtype=torch.int32)
    out = run_attention(eng, q, K, V, slots, pos, ctx)
    torch.cuda.synchronize()
    ref = reference(q.cpu(), K.cpu(), V.cpu(), slots.cpu(), pos.cpu())
    e = rel_err(out, ref)
    print(lens, e)
    assert e < 1e-2


@pytest.mark.parametrize("chunk,merge_in", [(64, 8), (64, 0), (128, 8), (128, 0), (1024, 8)])
def test_attention_plan_variants(chunk, merge_in):
    """Every split plan the tuning hook can select (keys per split -> 2 / 4 / 8
    waves; in-kernel ticket merge or the separate merge pass) gives the same
    attention within bf16 tolerance."""
    eng = tiny_engine()
    L = _lib.lib()
    lens = [1, 40, 300, 700]
    g = torch.Generator(device=dev).manual_seed(chunk + merge_in)
    K = torch.randn(4, 2, 704, 128, device=dev, generator=g).bfloat16()
    V = torch.randn(4, 2, 704, 128, device=dev, generator=g).bfloat16()
    q = torch.randn(4, 12 * 128, device=dev, generator=g).bfloat16()
    slots = torch.arange(4, device=dev, dtype=torch.int32)
    pos = torch.tensor([n - 1 for n in lens], device=dev, dtype=torch.int32)
    _lib.check(L.vv_attn_tune(chunk, merge_in), "attn_tune")
    try:
        out = run_attention(eng, q, K, V, slots, pos, 700)
        torch.cuda.synchronize()
    finally:
        L.vv_attn_tune(0, -1)
    ref = reference(q.cpu(), K.cpu(), V.cpu(), slots.cpu(), pos.cpu())
    assert rel_err(out, ref) < 1e-2


def _prefill_case(nh, nkv, runs, g):
    """runs: [(slot, first_pos, count)] -> query rows in that order (consecutive
    positions per run), cache filled for every slot up to its last position."""
    nslot = max(s for s, _, _ in runs) + 1
    ctx = (max(p + n for _, p, n in runs) + 63) // 64 * 64
    K = torch.randn(nslot, nkv, ctx, 128, device=dev, generator=g).bfloat16()
    V = torch.randn(nslot, nkv, ctx, 128, device=dev, generator=g).bfloat16()
    slots = torch.tensor([s for s, p, n in runs for _ in range(n)], device=dev, dtype=torch.int32)
    pos = torch.tensor([p + i for s, p, n in runs for i in range(n)], device=dev, dtype=torch.int32)
    q = torch.randn(slots.numel(), nh * 128, device=dev, generator=g).bfloat16()
    return q, K, V, slots, pos, ctx


@pytest.mark.parametrize("nh,nkv,runs", [
    (12, 2, [(0, 0, 700)]),                               # one prompt's causal prefill
    (12, 2, [(0, 0, 137), (1, 0, 300), (2, 0, 45)]),      # B = 3 ragged prompts in one launch (tiles span slots)
    (12, 2, [(1, 500, 70), (0, 0, 33)]),                  # a continuation chunk (keys before the first row)
    (28, 4, [(0, 0, 260), (1, 0, 5)]),                    # Large head layout (G = 7)
    (8, 8, [(0, 0, 100)]),                                # G = 1
])
def test_prefill_attention_vs_torch(nh, nkv, runs):
    """k_attn_pf (32-row tiles x the G heads of a kv head, transposed MFMA
    softmax) vs the fp32 torch reference, causal per row, rows of several
    slots in one launch.  Tolerance as above (bf16 P and output)."""
    g = torch.Generator(device=dev).manual_seed(len(runs) * 1000 + nh)
    q, K, V, slots, pos, ctx = _prefill_case(nh, nkv, runs, g)
    eng = tiny_engine()
    L = _lib.lib()
    L.vv_attn_prefill(1)
    try:
        out = run_attention(eng, q, K, V, slots, pos, ctx)
        torch.cuda.synchronize()
    finally:
        L.vv_attn_prefill(-1)
    ref = reference(q.cpu(), K.cpu(), V.cpu(), slots.cpu(), pos.cpu())
    assert torch.isfinite(out).all()
    assert rel_err(out, ref) < 1e-2


def test_prefill_attention_scattered_rows():
    """Rows in arbitrary (slot, position) order -- every tile needs several
    slot passes; the prefill kernel and the per-row decode kernel agree."""
    g = torch.Generator(device=dev).manual_seed(77)
    nslot, ctx, n = 5, 512, 150
    K = torch.randn(nslot, 2, ctx, 128, device=dev, generator=g).bfloat16()
    V = torch.randn(nslot, 2, ctx, 128, device=dev, generator=g).bfloat16()
    slots = torch.randint(0, nslot, (n,), device=dev, generator=g, dtype=torch.int32)
    pos = torch.randint(0, ctx, (n,), device=dev, generator=g, dtype=torch.int32)
    q = torch.randn(n, 12 * 128, device=dev, generator=g).bfloat16()
    eng = tiny_engine()
    L = _lib.lib()
    outs = []
    for mode in (1, 0):
        L.vv_attn_prefill(mode)
        try:
            outs.append(run_attention(eng, q, K, V, slots, pos, ctx))
            torch.cuda.synchronize()
        finally:
            L.vv_attn_prefill(-1)
    ref = reference(q.cpu(), K.cpu(), V.cpu(), slots.cpu(), pos.cpu())
    assert rel_err(outs[0], ref) < 1e-2 and rel_err(outs[1], ref) < 1e-2
    assert rel_err(outs[0], outs[1]) < 1e-2
