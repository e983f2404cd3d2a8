"""Tensor-parallel Qwen2 backbone on the GPU.

* A TP group of 2 / 4 engines (Megatron shards from weights.pack) driven on ONE
  MI355X by vv_lm_forward_group (layer-by-layer interleave, on-device sum as
  the all-reduce) reproduces the TP=1 engine: prefill of ragged rows + decode
  steps, hidden state and valid-id logits.  Tolerance rel L2 < 2e-2, cosine
  > 0.999 (bf16: partial sums are rounded before the reduction).
* The RCCL path (ncclAllReduce after o_proj / down_proj) runs with a
  single-rank communicator — RCCL rejects two ranks on one GPU — and must equal
  the communicator-free engine bit for bit, eagerly and under hipGraph capture.
"""
import pytest
import torch

from gpu_util import cos, rel_err
from tiny import tiny_config
from vibevoice_amd.engine import Engine
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"
I32 = dict(dtype=torch.int32, device=dev)
VALID = [151643, 151652, 151653, 151654]


def _inputs(seed, lens, H):
    g = torch.Generator().manual_seed(seed)
    x = torch.cat([torch.randn(n, H, generator=g) for n in lens]).bfloat16().to(dev)
    slots = torch.cat([torch.full((n,), r) for r, n in enumerate(lens)]).to(**I32)
    pos = torch.cat([torch.arange(n) for n in lens]).to(**I32)
    out_idx = torch.tensor([sum(lens[:r + 1]) - 1 for r in range(len(lens))]).to(**I32)
    return g, x, slots, pos, out_idx


@pytest.mark.parametrize("tp,H,heads,kv,inter", [(2, 1536, 12, 2, 8960), (4, 1024, 8, 4, 2048)])
def test_tp_group_matches_single_engine(tp, H, heads, kv, inter):
    cfg = tiny_config(hidden=H, layers=2, heads=heads, kv_heads=kv, inter=inter)
    sd = synthetic_state_dict(cfg, seed=11, device="cpu", mode="test", with_acoustic_encoder=False)
    full = Engine(cfg, sd, dev, max_batch=2, max_ctx=512, valid_ids=VALID)
    group = [Engine(cfg, sd, dev, max_batch=2, max_ctx=512, valid_ids=VALID, tp_rank=r, tp_size=tp)
             for r in range(tp)]
    lens = [40, 14]
    g, x, slots, pos, out_idx = _inputs(tp, lens, H)
    h1, l1 = full.lm_forward(x, slots, pos, out_idx)
    hg, lg = group[0].lm_forward_group(group[1:], x, slots, pos, out_idx)
    torch.cuda.synchronize()
    print("prefill", rel_err(hg, h1), cos(hg, h1))
    assert rel_err(hg, h1) < 2e-2 and cos(hg, h1) > 0.999
    assert torch.allclose(lg, l1, rtol=2e-2, atol=2e-2 * l1.abs().max().item())
    L = torch.tensor(lens)
    for s in range(3):
        step = torch.randn(2, H, generator=g).bfloat16().to(dev)
        rows = torch.arange(2).to(**I32)
        h1, _ = full.lm_forward(step, rows, L.to(**I32), rows)
        hg, _ = group[0].lm_forward_group(group[1:], step, rows, L.to(**I32), rows)
        L += 1
        torch.cuda.synchronize()
        print("step", s, rel_err(hg, h1), cos(hg, h1))
        assert rel_err(hg, h1) < 2e-2 and cos(hg, h1) > 0.999


def test_rccl_allreduce_path_single_rank():
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=12, device="cpu", mode="test", with_acoustic_encoder=False)
    plain = Engine(cfg, sd, dev, max_batch=2, max_ctx=128, valid_ids=VALID)
    rccl = Engine(cfg, sd, dev, max_batch=2, max_ctx=128, valid_ids=VALID, tp_rank=0, tp_size=1,
                  tp_unique_id=Engine.tp_unique_id())
    _, x, slots, pos, out_idx = _inputs(5, [20, 9], 256)
    ha, la = plain.lm_forward(x, slots, pos, out_idx)
    hb, lb = rccl.lm_forward(x, slots, pos, out_idx)
    torch.cuda.synchronize()
    assert torch.equal(ha, hb) and torch.equal(la, lb)
    # decode step captured into a hipGraph with the RCCL call inside
    step = torch.randn(2, 256, device=dev).bfloat16()
    rows = torch.arange(2).to(**I32)
    p2 = torch.tensor([20, 9]).to(**I32)
    hc = torch.empty(2, 256, device=dev, dtype=torch.bfloat16)
    lc = torch.empty(2, 4, device=dev, dtype=torch.float32)
    plain.lm_forward(step, rows, p2, rows, hidden_out=hc, logits_out=lc, max_pos=127)
    gph = torch.cuda.CUDAGraph()
    hd = torch.empty_like(hc)
    ld = torch.empty_like(lc)
    rccl.lm_forward(step, rows, p2, rows, hidden_out=hd, logits_out=ld, max_pos=127)   # warm
    with torch.cuda.graph(gph):
        rccl.lm_forward(step, rows, p2, rows, hidden_out=hd, logits_out=ld, max_pos=127)
    gph.replay()
    torch.cuda.synchronize()
    assert torch.equal(hc, hd) and torch.equal(lc, ld)


def test_rccl_head_allreduce_path_single_rank():
    """The sharded diffusion head's RCCL path (one all-reduce of [2n, H] per
    head layer) with a single-rank communicator: bit-exact against the
    communicator-free engine, eagerly and inside a captured hipGraph."""
    from vibevoice_amd import _lib
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=13, device="cpu", mode="test", with_acoustic_encoder=False)
    plain = Engine(cfg, sd, dev, max_batch=2, max_ctx=128, valid_ids=VALID)
    rccl = Engine(cfg, sd, dev, max_batch=2, max_ctx=128, valid_ids=VALID, tp_rank=0, tp_size=1,
                  tp_unique_id=Engine.tp_unique_id())
    _lib.check(_lib.lib().vv_tp_shard_head(rccl.h, 1), "tp_shard_head")
    for e in (plain, rccl):
        e.set_steps(10)
    g = torch.Generator().manual_seed(4)
    pos = torch.randn(2, 256, generator=g).bfloat16().to(dev)
    neg = torch.randn(2, 256, generator=g).bfloat16().to(dev)
    x0 = torch.randn(2, 64, generator=g).bfloat16().to(dev)
    xa, xb = x0.clone(), x0.clone()
    plain.diffusion_sample(pos, neg, xa, 1.3)
    rccl.diffusion_sample(pos, neg, xb, 1.3)
    torch.cuda.synchronize()
    assert torch.equal(xa, xb)
    xc = x0.clone()
    rccl.diffusion_sample(pos, neg, xc, 1.3)   # warm
    xc.copy_(x0)
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        rccl.diffusion_sample(pos, neg, xc, 1.3)
    xc.copy_(x0)
    gph.replay()
    torch.cuda.synchronize()
    assert torch.equal(xa, xc)
