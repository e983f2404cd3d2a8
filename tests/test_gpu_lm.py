"""Qwen2 decoder rows on the GPU (vv_lm_forward): compacted per-row KV cache,
RoPE, GQA attention (single and split-K), SwiGLU, final norm, restricted lm_head.

Pinned against the reference's Qwen2 golden (g7: left-padded prefill + 3 decode
steps, bf16) and against the CPU oracle at the 1.5B layer shapes (12 q / 2 kv
heads, H 1536, I 8960) with contexts up to 2500 keys (several attention splits of
<= 1024 keys merged in-launch).
Tolerance: rel L2 < 2e-2, cosine > 0.999 (bf16 model).
"""
import pytest
import torch

from golden_io import load, t, weights
from gpu_util import cos, kv_synthetic, rel_err
from oracle import lm as olm
from tiny import tiny_config
from vibevoice_amd.engine import Engine
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"
I32 = dict(dtype=torch.int32, device=dev)


@pytest.fixture(autouse=True)
def _collect_engines():
    """Engines of earlier tests / modules that are garbage but not yet collected
    count as registered contexts (engine.cpp hl_register): collected mid-test,
    they would switch the one-launch kernels on between two runs a test compares
    bitwise."""
    import gc
    gc.collect()
    yield


def make_engine(cfg, lm_sd=None, seed=0, max_batch=2, max_ctx=1024):
    sd = synthetic_state_dict(cfg, seed=seed, device="cpu", mode="test", with_acoustic_encoder=False)
    if lm_sd is not None:
        for k, v in lm_sd.items():
            sd["model.language_model." + k] = v
        sd["lm_head.weight"] = sd["model.language_model.embed_tokens.weight"]
    eng = Engine(cfg, sd, dev, max_batch=max_batch, max_ctx=max_ctx, valid_ids=[151643, 151652, 151653, 151654])
    return eng, sd


def test_lm_vs_reference_golden():
    z = load("g7_qwen2.npz")
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    lm_sd = weights(z, dtype=torch.bfloat16)
    lm_sd.pop("embed_tokens.weight")
    eng, _ = make_engine(cfg, lm_sd)
    emb = t(z, "emb_bf16", torch.bfloat16)
    steps = t(z, "steps_bf16", torch.bfloat16)
    mask = torch.from_numpy(z["mask0"]).bool()
    ref = t(z, "hidden_bf16")
    keep = [emb[r][mask[r]] for r in range(2)]
    lens = [k.shape[0] for k in keep]
    x = torch.cat(keep).to(dev)
    slots = torch.cat([torch.full((n,), r) for r, n in enumerate(lens)]).to(**I32)
    pos = torch.cat([torch.arange(n) for n in lens]).to(**I32)
    out_idx = torch.tensor([lens[0] - 1, lens[0] + lens[1] - 1]).to(**I32)
    h, _ = eng.lm_forward(x, slots, pos, out_idx)
    torch.cuda.synchronize()
    print("prefill", rel_err(h, ref[0]), cos(h, ref[0]))
    assert rel_err(h, ref[0]) < 2e-2 and cos(h, ref[0]) > 0.999
    L = torch.tensor(lens)
    for s in range(3):
        h, _ = eng.lm_forward(steps[s, :, 0].contiguous().to(dev), torch.arange(2).to(**I32), L.to(**I32),
                              torch.arange(2).to(**I32))
        L += 1
        torch.cuda.synchronize()
        print("step", s, rel_err(h, ref[s + 1]), cos(h, ref[s + 1]))
        assert rel_err(h, ref[s + 1]) < 2e-2 and cos(h, ref[s + 1]) > 0.999


def oracle_sd(sd):
    return {k[len("model.language_model."):]: v for k, v in sd.items() if k.startswith("model.language_model.")}


@pytest.mark.parametrize("ctx,pf", [(40, -1), (600, -1), (2500, -1), (600, 0)])
def test_lm_real_shapes_vs_oracle(ctx, pf):
    """pf = -1: the engine's own attention choice (the 801- and 3,334-row
    prefills take the 32-row-tile prefill kernel); 0: the per-row decode
    kernel forced for the prefill too."""
    from vibevoice_amd import _lib
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    eng, sd = make_engine(cfg, seed=1, max_batch=2, max_ctx=4096)
    _lib.lib().vv_attn_prefill(pf)
    try:
        _lm_real_shapes(eng, sd, cfg, ctx)
    finally:
        _lib.lib().vv_attn_prefill(-1)


def _lm_real_shapes(eng, sd, cfg, ctx):
    lcfg = dict(cfg.decoder_config)
    osd = oracle_sd(sd)
    g = torch.Generator().manual_seed(ctx)
    lens = [ctx, ctx // 3 + 1]
    xs = [torch.randn(n, 1536, generator=g).bfloat16() for n in lens]
    kvs = [olm.RowKV(2) for _ in lens]
    ref = torch.stack([olm.forward_rows(osd, lcfg, xs[r][None], kvs[r:r + 1])[0, -1] for r in range(2)])
    x = torch.cat(xs).to(dev)
    slots = torch.cat([torch.full((n,), r) for r, n in enumerate(lens)]).to(**I32)
    pos = torch.cat([torch.arange(n) for n in lens]).to(**I32)
    out_idx = torch.tensor([lens[0] - 1, sum(lens) - 1]).to(**I32)
    h, logits = eng.lm_forward(x, slots, pos, out_idx)
    torch.cuda.synchronize()
    print("prefill", rel_err(h, ref), cos(h, ref))
    assert rel_err(h, ref) < 2e-2 and cos(h, ref) > 0.999
    # restricted lm_head: bf16(h . W[id]) for the 4 valid ids
    W = sd["lm_head.weight"]
    lref = (h.float().cpu() @ W[[151643, 151652, 151653, 151654]].float().t()).bfloat16().float()
    assert torch.allclose(logits.cpu(), lref, rtol=1e-2, atol=1e-2 * lref.abs().max().item())
    # decode steps: both rows, positions continue after their prompts
    L = torch.tensor(lens)
    for s in range(3):
        step_x = torch.randn(2, 1536, generator=g).bfloat16()
        ref = olm.forward_rows(osd, lcfg, step_x[:, None], kvs)[:, -1]
        h, _ = eng.lm_forward(step_x.to(dev), torch.arange(2).to(**I32), L.to(**I32), torch.arange(2).to(**I32))
        L += 1
        torch.cuda.synchronize()
        print("step", s, rel_err(h, ref), cos(h, ref))
        assert rel_err(h, ref) < 2e-2 and cos(h, ref) > 0.999


def test_rope_table_bit_identical():
    """The q|k|v epilogue's per-position cos / sin table (k_rope_table) vs the
    inline cosf / sinf: identical hidden states, logits and KV caches after a
    3,000-row prefill (the 256^2-tile GEMM path) and two decode steps."""
    from vibevoice_amd import _lib
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    outs = []
    for tab in (1, 0):
        _lib.lib().vv_rope_table(tab)
        try:
            eng, sd = make_engine(cfg, seed=3, max_batch=1, max_ctx=4096)
            g = torch.Generator().manual_seed(5)
            x = torch.randn(3000, 1536, generator=g).bfloat16().to(dev)
            h0, l0 = eng.lm_forward(x, torch.zeros(3000, **I32), torch.arange(3000).to(**I32),
                                    torch.tensor([2999]).to(**I32))
            hs = [h0.clone(), l0.clone()]
            for s in range(2):
                xs = torch.randn(1, 1536, generator=g).bfloat16().to(dev)
                h, lg = eng.lm_forward(xs, torch.zeros(1, **I32), torch.tensor([3000 + s]).to(**I32),
                                       torch.zeros(1, **I32))
                hs += [h.clone(), lg.clone()]
            torch.cuda.synchronize()
            outs.append(hs)
        finally:
            _lib.lib().vv_rope_table(1)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("nrows,chunk,maxpos", [(2, 256, 1790), (12, 256, 1790), (4, 128, 3000)])
def test_attn_defer_bit_identical(nrows, chunk, maxpos):
    """Deferred split merge (vv_attn_defer: k_attn leaves every split's partial,
    o_proj's XF_ATTN_MERGE staging merges them) vs the same splits merged inside
    k_attn (vv_attn_tune with the chunk the engine picks: `chunk`, or 8 splits
    of ceil(max / 8) rounded to 32 keys past 8 chunks): identical hidden states
    and logits; and close to the default 1,024-key plan.  Rows at contexts from
    1 key to 8 splits (nact 1 rows take the merge's trivial case)."""
    from vibevoice_amd import _lib
    L = _lib.lib()
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    eng, _ = make_engine(cfg, seed=4, max_batch=nrows, max_ctx=4096)
    slots = torch.arange(nrows).to(**I32)
    kv_synthetic(eng, slots, 0, 4096, seed=11)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(nrows, 1536, generator=g).bfloat16().to(dev)
    pos = torch.tensor([(97 + 263 * i) % maxpos for i in range(nrows)], dtype=torch.int32).to(dev)
    pos[0] = maxpos - 1
    if nrows > 2:
        pos[1] = 3                                 # one split
    ns = -(-maxpos // chunk)
    eff = chunk if ns <= 8 else (-(-maxpos // 8) + 31) // 32 * 32
    outs = {}
    L.vv_lm_attn(0)   # the three-launch attention half (the one-launch form has no split plans)
    try:
        for name, defer, tune in (("defer", 1, 0), ("inkernel", 0, eff), ("default", 0, 0)):
            _lib.check(L.vv_attn_defer(16 if defer else 0, chunk), "attn_defer")   # <= 16 rows defer
            _lib.check(L.vv_attn_tune(tune, -1), "attn_tune")
            h, lg = eng.lm_forward(x, slots, pos, torch.arange(nrows).to(**I32))
            torch.cuda.synchronize()
            outs[name] = (h.clone(), lg.clone())
    finally:
        L.vv_attn_defer(1, 128)
        L.vv_attn_tune(0, -1)
        L.vv_lm_attn(1)
    assert torch.equal(outs["defer"][0], outs["inkernel"][0])
    assert torch.equal(outs["defer"][1], outs["inkernel"][1])
    h, ref = outs["defer"][0].float(), outs["default"][0].float()
    print("vs 1,024-key plan", rel_err(h, ref), cos(h, ref))
    assert rel_err(h, ref) < 1e-2 and cos(h, ref) > 0.9999


def test_norm_pack_bit_identical():
    """The prefill's producers writing MFMA-fragment-packed A rows for the
    256 x 256-tile GEMMs (vv_norm_pack: RMSNorm rows for q|k|v and gate|up,
    gate|up's SiLU*up rows for down) vs row-major rows, and the 256 x 256 tile's
    row-contiguous epilogues (q|k|v RoPE + K / V cache append, SiLU*up,
    residual) vs the 128 x 128 tile's per-lane ones: identical hidden states and
    logits after a ragged 8,200-row prefill (last row tile partial) and one
    decode step that reads the prefill's K / V cache."""
    from vibevoice_amd import _lib
    L = _lib.lib()
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    outs = []
    try:
        # packed / row-major A rows on the 256^2 tile (its row-contiguous RoPE + KV
        # epilogue), then the 128^2 tile with epi_tile's per-lane epilogue
        for pack, big in ((1, -1), (0, -1), (0, 2)):
            L.vv_norm_pack(pack)
            L.vv_gemm_tune_big(big)
            eng, _ = make_engine(cfg, seed=6, max_batch=1, max_ctx=8448)
            g = torch.Generator().manual_seed(8)
            x = torch.randn(8200, 1536, generator=g).bfloat16().to(dev)
            h0, l0 = eng.lm_forward(x, torch.zeros(8200, **I32), torch.arange(8200).to(**I32),
                                    torch.tensor([0, 5170, 8199]).to(**I32))
            xs = torch.randn(1, 1536, generator=g).bfloat16().to(dev)
            h1, l1 = eng.lm_forward(xs, torch.zeros(1, **I32), torch.tensor([8200]).to(**I32), torch.zeros(1, **I32))
            torch.cuda.synchronize()
            outs.append([h0.clone(), l0.clone(), h1.clone(), l1.clone()])
    finally:
        L.vv_norm_pack(1)
        L.vv_gemm_tune_big(-1)
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


def test_lm_ffn_one_launch_vs_oracle_and_gemv_pair():
    """The LM MLP block at decode as ONE launch (lm_ffn.hip: MFMA gate|up over
    4-5 tiles per workgroup, one grid-wide hand-off of the SiLU*up rows, MFMA
    down over half a tile per owner) on the 1.5B layer shapes (H 1536, I 8960),
    2 rows: each decode step vs the oracle (rel < 2e-2, cosine > 0.999) and vs
    the gate|up + down GEMV pair on the same KV state (within bf16: the GEMM
    sums run in another order), repeated runs bitwise equal."""
    import gc
    from vibevoice_amd import _lib
    gc.collect()   # the one-launch block runs only for the device's sole registered context
    L_ = _lib.lib()
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    eng, sd = make_engine(cfg, seed=3, max_batch=1, max_ctx=512)
    assert L_.vv_lm_ffn_active(eng.h, 2) == 1
    lcfg = dict(cfg.decoder_config)
    osd = oracle_sd(sd)
    g = torch.Generator().manual_seed(7)
    lens = [40, 17]
    xs = [torch.randn(n, 1536, generator=g).bfloat16() for n in lens]
    kvs = [olm.RowKV(2) for _ in lens]
    for r in range(2):
        olm.forward_rows(osd, lcfg, xs[r][None], kvs[r:r + 1])
    x = torch.cat(xs).to(dev)
    slots = torch.cat([torch.full((n,), r) for r, n in enumerate(lens)]).to(**I32)
    pos = torch.cat([torch.arange(n) for n in lens]).to(**I32)
    eng.lm_forward(x, slots, pos, torch.tensor([lens[0] - 1, sum(lens) - 1]).to(**I32))
    L = torch.tensor(lens)
    try:
        for s in range(3):
            step_x = torch.randn(2, 1536, generator=g).bfloat16()
            ref = olm.forward_rows(osd, lcfg, step_x[:, None], kvs)[:, -1]
            outs = {}
            for on in (0, 1, 1):
                L_.vv_lm_ffn(on)
                h, _ = eng.lm_forward(step_x.to(dev), torch.arange(2).to(**I32), L.to(**I32),
                                      torch.arange(2).to(**I32))
                torch.cuda.synchronize()
                outs.setdefault(on, []).append(h.clone())
            L += 1
            one, pair = outs[1][0], outs[0][0]
            print(f"step {s}: one launch rel {rel_err(one, ref):.3e} vs oracle (GEMV pair {rel_err(pair, ref):.3e}), "
                  f"{rel_err(one, pair):.3e} vs the GEMV pair")
            assert torch.equal(one, outs[1][1])
            assert rel_err(one, ref) < 2e-2 and cos(one, ref) > 0.999
            assert rel_err(one, pair) < 2e-2 and cos(one, pair) > 0.999
    finally:
        L_.vv_lm_ffn(1)
    eng.check_sync()


@pytest.mark.parametrize("n", [8, 3])
def test_lm_ffn16_one_launch_vs_oracle_and_gemv_pair(n):
    """configs[2]'s LM MLP block (B = 8: 16 rows; n = 3: 6 rows) as ONE launch
    (lm_ffn.hip k_lm_ffn16: MFMA gate|up over 4-5 tiles per workgroup, one grid
    wait, down split by column group x hidden range with the 4 fp32 partials of
    a group summed in range order by its last arrival) on the 1.5B layer shapes:
    each decode step vs the oracle (rel < 2e-2, cosine > 0.999) and vs the
    gate|up + down GEMV pair on the same KV state (within bf16), repeated runs
    bitwise equal."""
    import gc
    from vibevoice_amd import _lib
    gc.collect()
    L_ = _lib.lib()
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    eng, sd = make_engine(cfg, seed=5, max_batch=8, max_ctx=256)
    R = 2 * n
    assert L_.vv_lm_ffn_active(eng.h, R) == 1
    lcfg = dict(cfg.decoder_config)
    osd = oracle_sd(sd)
    g = torch.Generator().manual_seed(11 + n)
    lens = [5 + 3 * r for r in range(R)]
    xs = [torch.randn(m, 1536, generator=g).bfloat16() for m in lens]
    kvs = [olm.RowKV(2) for _ in lens]
    for r in range(R):
        olm.forward_rows(osd, lcfg, xs[r][None], kvs[r:r + 1])
    x = torch.cat(xs).to(dev)
    slots = torch.cat([torch.full((m,), r) for r, m in enumerate(lens)]).to(**I32)
    pos = torch.cat([torch.arange(m) for m in lens]).to(**I32)
    last = torch.cumsum(torch.tensor(lens), 0) - 1
    eng.lm_forward(x, slots, pos, last.to(**I32))
    Lt = torch.tensor(lens)
    try:
        for s in range(3):
            step_x = torch.randn(R, 1536, generator=g).bfloat16()
            ref = olm.forward_rows(osd, lcfg, step_x[:, None], kvs)[:, -1]
            outs = {}
            for on in (3, 1, 1):   # 3: the GEMV pair at > 2 rows, 1: k_lm_ffn16
                L_.vv_lm_ffn(on)
                h, _ = eng.lm_forward(step_x.to(dev), torch.arange(R).to(**I32), Lt.to(**I32),
                                      torch.arange(R).to(**I32))
                torch.cuda.synchronize()
                outs.setdefault(on, []).append(h.clone())
            Lt += 1
            one, pair = outs[1][0], outs[3][0]
            print(f"n={n} step {s}: one launch rel {rel_err(one, ref):.3e} vs oracle (GEMV pair "
                  f"{rel_err(pair, ref):.3e}), {rel_err(one, pair):.3e} vs the GEMV pair")
            assert torch.equal(one, outs[1][1])
            assert rel_err(one, ref) < 2e-2 and cos(one, ref) > 0.999
            assert rel_err(one, pair) < 2e-2 and cos(one, pair) > 0.999
    finally:
        L_.vv_lm_ffn(1)
    eng.check_sync()


@pytest.mark.parametrize("n,lens", [(1, [600, 33]), (3, [1, 31, 32, 64, 200, 97]),
                                    (8, [5 + 61 * r for r in range(16)])])
def test_lm_attn_one_launch_vs_oracle_and_three_launches(n, lens):
    """The LM attention half at decode as ONE launch (lm_attn.hip k_lm_attn:
    q|k|v tiles + RoPE + cache append, one grid wait, attention in 32-key units
    over all 256 workgroups, one wait, per-head merge of the units, one wait,
    o_proj from resident weights + residual) on the 1.5B layer shapes at 2 n
    rows: each decode step vs the oracle (rel < 2e-2, cosine > 0.999) and vs the
    q|k|v + k_attn + o_proj launches on the same KV state (within bf16: the
    projections sum in another order, the keys merge in 32-key units), repeated
    runs and the issue-order variants bitwise equal.  Contexts from 2 keys to
    ~1,000, across unit edges."""
    import gc
    from vibevoice_amd import _lib
    gc.collect()
    L_ = _lib.lib()
    R = 2 * n
    assert len(lens) == R
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    eng, sd = make_engine(cfg, seed=13 + n, max_batch=max(n, 1), max_ctx=1024)
    assert L_.vv_lm_attn_active(eng.h, R, max(lens) + 3) == 1
    lcfg = dict(cfg.decoder_config)
    osd = oracle_sd(sd)
    g = torch.Generator().manual_seed(21 + n)
    xs = [torch.randn(m, 1536, generator=g).bfloat16() for m in lens]
    kvs = [olm.RowKV(2) for _ in lens]
    for r in range(R):
        olm.forward_rows(osd, lcfg, xs[r][None], kvs[r:r + 1])
    x = torch.cat(xs).to(dev)
    slots = torch.cat([torch.full((m,), r) for r, m in enumerate(lens)]).to(**I32)
    pos = torch.cat([torch.arange(m) for m in lens]).to(**I32)
    last = torch.cumsum(torch.tensor(lens), 0) - 1
    eng.lm_forward(x, slots, pos, last.to(**I32))
    Lt = torch.tensor(lens)
    try:
        for s in range(3):
            step_x = torch.randn(R, 1536, generator=g).bfloat16()
            ref = olm.forward_rows(osd, lcfg, step_x[:, None], kvs)[:, -1]
            outs = {}
            for on in (0, 1, 1, 15):   # 15: the round-6 first form (16 A rows, o_proj weights at entry)
                L_.vv_lm_attn(on)
                h, _ = eng.lm_forward(step_x.to(dev), torch.arange(R).to(**I32), Lt.to(**I32),
                                      torch.arange(R).to(**I32))
                torch.cuda.synchronize()
                outs.setdefault(on, []).append(h.clone())
            Lt += 1
            one, three = outs[1][0], outs[0][0]
            print(f"n={n} step {s}: one launch rel {rel_err(one, ref):.3e} vs oracle (three launches "
                  f"{rel_err(three, ref):.3e}), {rel_err(one, three):.3e} vs the three launches")
            assert torch.equal(one, outs[1][1]) and torch.equal(one, outs[15][0])   # same sums
            assert rel_err(one, ref) < 2e-2 and cos(one, ref) > 0.999
            assert rel_err(one, three) < 2e-2 and cos(one, three) > 0.999
    finally:
        L_.vv_lm_attn(1)
    eng.check_sync()


def test_lm_attn_one_launch_limits():
    """Where the one-launch attention half does not apply: more than 16 rows,
    contexts past 4,096 keys (the split plans of k_attn take them), the switch
    off."""
    import gc
    from vibevoice_amd import _lib
    gc.collect()
    L_ = _lib.lib()
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    eng, _ = make_engine(cfg, seed=2, max_batch=8, max_ctx=8192)
    assert L_.vv_lm_attn_active(eng.h, 16, 4096) == 1
    assert L_.vv_lm_attn_active(eng.h, 16, 4097) == 0
    assert L_.vv_lm_attn_active(eng.h, 17, 100) == 0
    L_.vv_lm_attn(0)
    try:
        assert L_.vv_lm_attn_active(eng.h, 2, 100) == 0
    finally:
        L_.vv_lm_attn(1)
    assert L_.vv_lm_attn_active(eng.h, 2, 100) == 1
