"""VibeVoice-Large shapes, tensor parallelism at real shapes, and the 64K
context (BASELINE.json configs[3] and configs[4]) on the MI355X.

* Large Qwen2 layers (qwen2.5_7b_32k.json: H 3584, I 18944, 28 q / 4 kv heads,
  vocab 152,064) vs oracle/lm.py: ragged prefill + decode steps, and the
  restricted lm_head (the 4 legal rows of the Large vocabulary).
* The Large diffusion head (H 3584, FFN 10,752, 4 layers), S = 10, CFG 1.3,
  vs oracle/head.py, for 1 and 4 diffusing rows (configs[3]: 4 speakers).
* TP = 4 (and 2) of the Large layers — the Megatron split of
  configuration_vibevoice.py:175-183, driven by vv_lm_forward_group (the
  ranks' shards interleaved layer by layer on one GPU, on-device sum as the
  all-reduce) — vs the TP = 1 engine.
* configs[4]: a 65,000-token 1.5B-shape prefill followed by decode steps vs
  oracle/lm.py run as the checker on the GPU (chunked causal prefill); the
  decode step captured into a hipGraph (the loop's max_ctx plan) and replayed
  at 65K keys, bitwise equal to eager launches; TP = 2 at a 65,000-token
  context vs the TP = 1 engine, and its graph-replayed decode vs its eager one.
Tolerance: rel L2 < 2e-2 and cosine > 0.999 (bf16), as test_gpu_lm.py.
"""
import pytest
import torch

from gpu_util import cos, rel_err
from oracle import head as ohead
from oracle import lm as olm
from tiny import tiny_config
from vibevoice_amd.config import VibeVoiceConfig
from vibevoice_amd.engine import Engine
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"
I32 = dict(dtype=torch.int32, device=dev)
VALID = [151643, 151652, 151653, 151654]
LARGE = dict(hidden=3584, heads=28, kv_heads=4, inter=18944, vocab=152064)


def large_cfg(layers=2):
    return tiny_config(layers=layers, **LARGE)


def oracle_sd(sd, device="cpu"):
    p = "model.language_model."
    return {k[len(p):]: v.to(device) for k, v in sd.items() if k.startswith(p)}


def _rows(g, lens, H):
    x = [torch.randn(n, H, generator=g).bfloat16() for n in lens]
    slots = torch.cat([torch.full((n,), r) for r, n in enumerate(lens)]).to(**I32)
    pos = torch.cat([torch.arange(n) for n in lens]).to(**I32)
    out_idx = torch.tensor([sum(lens[:r + 1]) - 1 for r in range(len(lens))]).to(**I32)
    return x, slots, pos, out_idx


@pytest.mark.parametrize("ctx", [40, 700])
def test_large_lm_layers_vs_oracle(ctx):
    cfg = large_cfg()
    sd = synthetic_state_dict(cfg, seed=21, device="cpu", mode="test", with_acoustic_encoder=False)
    assert sd["lm_head.weight"].shape == (152064, 3584)
    eng = Engine(cfg, sd, dev, max_batch=2, max_ctx=1024, valid_ids=VALID)
    osd, lcfg = oracle_sd(sd), dict(cfg.decoder_config)
    g = torch.Generator().manual_seed(ctx)
    lens = [ctx, ctx // 3 + 1]
    xs, slots, pos, out_idx = _rows(g, lens, 3584)
    kvs = [olm.RowKV(2) for _ in lens]
    ref = torch.stack([olm.forward_rows(osd, lcfg, xs[r][None], kvs[r:r + 1])[0, -1] for r in range(2)])
    h, logits = eng.lm_forward(torch.cat(xs).to(dev), slots, pos, out_idx)
    torch.cuda.synchronize()
    print(f"Large prefill ctx {ctx}: rel {rel_err(h, ref):.3e} cos {cos(h, ref):.6f}")
    assert rel_err(h, ref) < 2e-2 and cos(h, ref) > 0.999
    # the final head: bf16(h . W[id]) over the 4 legal rows of the Large lm_head
    lref = (h.float().cpu() @ sd["lm_head.weight"][VALID].float().t()).bfloat16().float()
    assert torch.allclose(logits.cpu(), lref, rtol=1e-2, atol=1e-2 * lref.abs().max().item())
    L = torch.tensor(lens)
    for s in range(3):
        step_x = torch.randn(2, 3584, generator=g).bfloat16()
        ref = olm.forward_rows(osd, lcfg, step_x[:, None], kvs)[:, -1]
        h, _ = eng.lm_forward(step_x.to(dev), torch.arange(2).to(**I32), L.to(**I32), torch.arange(2).to(**I32))
        L += 1
        torch.cuda.synchronize()
        print(f"Large step {s}: rel {rel_err(h, ref):.3e} cos {cos(h, ref):.6f}")
        assert rel_err(h, ref) < 2e-2 and cos(h, ref) > 0.999


@pytest.mark.parametrize("n", [1, 4])
def test_large_head_vs_oracle(n):
    """modular_vibevoice_diffusion_head.py:254-280 + the CFG DPM-Solver++ loop
    (modeling_vibevoice_inference.py:712-725) at H = 3584."""
    cfg = VibeVoiceConfig.builtin("Large")
    hc = cfg.diffusion_head_config
    lm_cfg = tiny_config(layers=1, **LARGE)
    sd = synthetic_state_dict(lm_cfg, seed=22, device="cpu", mode="test", with_acoustic_encoder=False)
    hsd = {k[len("model.prediction_head."):]: v for k, v in sd.items() if k.startswith("model.prediction_head.")}
    assert hsd["layers.0.ffn.gate_proj.weight"].shape == (int(3584 * hc.head_ffn_ratio), 3584)
    eng = Engine(lm_cfg, sd, dev, max_batch=4, max_ctx=64)
    S = 10
    eng.set_steps(S)
    g = torch.Generator().manual_seed(n)
    pos = torch.randn(n, 3584, generator=g).bfloat16()
    neg = torch.randn(n, 3584, generator=g).bfloat16()
    noise = torch.randn(2 * n, 64, generator=g).bfloat16()
    x = noise[:n].to(dev).contiguous()
    eng.diffusion_sample(pos.to(dev), neg.to(dev), x, 1.3)
    torch.cuda.synchronize()
    ref = ohead.sample_speech_tokens(hsd, pos, neg, noise, S, 1.3, hc.head_layers)
    ref32 = ohead.sample_speech_tokens({k: v.float() for k, v in hsd.items()}, pos.float(), neg.float(),
                                       noise.float(), S, 1.3, hc.head_layers)
    e, c, sdev = rel_err(x, ref), cos(x, ref), rel_err(ref32, ref)
    print(f"Large head n={n}: rel {e:.3e} cos {c:.6f} (bf16 reference vs fp32 {sdev:.3e})")
    assert e < max(2e-2, 2 * sdev) and c > 0.999


@pytest.mark.parametrize("tp", [2, 4])
def test_large_tp_group_matches_single_engine(tp):
    """configs[3]: the Large backbone split over `tp` ranks (whole KV heads per
    rank: 4 kv heads -> TP <= 4)."""
    cfg = large_cfg()
    sd = synthetic_state_dict(cfg, seed=23, device="cpu", mode="test", with_acoustic_encoder=False)
    full = Engine(cfg, sd, dev, max_batch=2, max_ctx=512, valid_ids=VALID)
    group = [Engine(cfg, sd, dev, max_batch=2, max_ctx=512, valid_ids=VALID, tp_rank=r, tp_size=tp)
             for r in range(tp)]
    g = torch.Generator().manual_seed(tp)
    lens = [60, 23]
    xs, slots, pos, out_idx = _rows(g, lens, 3584)
    x = torch.cat(xs).to(dev)
    h1, l1 = full.lm_forward(x, slots, pos, out_idx)
    hg, lg = group[0].lm_forward_group(group[1:], x, slots, pos, out_idx)
    torch.cuda.synchronize()
    print(f"Large TP={tp} prefill: rel {rel_err(hg, h1):.3e} cos {cos(hg, h1):.6f}")
    assert rel_err(hg, h1) < 2e-2 and cos(hg, h1) > 0.999
    assert torch.allclose(lg, l1, rtol=2e-2, atol=2e-2 * l1.abs().max().item())
    L = torch.tensor(lens)
    rows = torch.arange(2).to(**I32)
    for s in range(3):
        step = torch.randn(2, 3584, generator=g).bfloat16().to(dev)
        h1, _ = full.lm_forward(step, rows, L.to(**I32), rows)
        hg, _ = group[0].lm_forward_group(group[1:], step, rows, L.to(**I32), rows)
        L += 1
        torch.cuda.synchronize()
        print(f"Large TP={tp} step {s}: rel {rel_err(hg, h1):.3e} cos {cos(hg, h1):.6f}")
        assert rel_err(hg, h1) < 2e-2 and cos(hg, h1) > 0.999


def _oracle_prefill_gpu(osd, lcfg, x, kv, chunk=4096):
    """oracle/lm.py on the GPU, causal prefill in chunks of `chunk` rows (the
    [rows x keys] fp32 scores of one chunk fit; the whole 65K x 65K would not)."""
    h = None
    for i in range(0, x.shape[0], chunk):
        h = olm.forward_rows(osd, lcfg, x[None, i:i + chunk], [kv])
    return h[0, -1]


def test_64k_context_prefill_and_decode_vs_oracle():
    """configs[4]: a 65,000-position context (the 1.5B LM allows 65,536) built
    by a real prefill (k_attn_pf + k_gemm_big), then 3 decode steps attending
    all of it (k_attn splits + merge), 1.5B layer shapes, 2 layers."""
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    cfg.decoder_config["max_position_embeddings"] = 65536
    sd = synthetic_state_dict(cfg, seed=24, device="cpu", mode="test", with_acoustic_encoder=False)
    N = 65000
    eng = Engine(cfg, sd, dev, max_batch=1, max_ctx=N + 8, valid_ids=VALID)
    osd, lcfg = oracle_sd(sd, dev), dict(cfg.decoder_config)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(N, 1536, device=dev, generator=g).bfloat16()
    zero = torch.zeros(N, **I32)
    h, _ = eng.lm_forward(x, zero, torch.arange(N).to(**I32), torch.tensor([N - 1]).to(**I32))
    kv = olm.RowKV(2)
    with torch.no_grad():
        ref = _oracle_prefill_gpu(osd, lcfg, x, kv)
    torch.cuda.synchronize()
    print(f"64K prefill: rel {rel_err(h, ref):.3e} cos {cos(h, ref):.6f}")
    assert rel_err(h, ref) < 2e-2 and cos(h, ref) > 0.999
    for s in range(3):
        step = torch.randn(1, 1536, device=dev, generator=g).bfloat16()
        h, _ = eng.lm_forward(step, torch.zeros(1, **I32), torch.tensor([N + s]).to(**I32),
                              torch.zeros(1, **I32))
        with torch.no_grad():
            ref = olm.forward_rows(osd, lcfg, step[None], [kv])[0, -1]
        torch.cuda.synchronize()
        print(f"64K decode step {s} (attends {N + s + 1} keys): rel {rel_err(h, ref):.3e} cos {cos(h, ref):.6f}")
        assert rel_err(h, ref) < 2e-2 and cos(h, ref) > 0.999


def _graph_vs_eager(run, set_step, n_steps):
    """Eager decode steps, then the same call captured into a hipGraph and
    replayed on the same static buffers: bitwise equal outputs.  Re-running a
    step at its position rewrites that position's K/V with the same values and
    attends keys [0, pos], so the replays see exactly the eager state."""
    eager = []
    for s in range(n_steps):
        set_step(s)
        eager.append(run())
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    replayed = []
    for s in range(n_steps):
        set_step(s)
        g.replay()
        replayed.append(run.out())
    torch.cuda.synchronize()
    return eager, replayed


class _Dec:
    """Static-buffer decode call (one row) for graph capture."""

    def __init__(self, eng, peers=None):
        self.eng, self.peers = eng, peers
        self.x = torch.zeros(1, eng.hidden, dtype=torch.bfloat16, device=dev)
        self.pos = torch.zeros(1, **I32)
        self.rows = torch.zeros(1, **I32)
        self.h = torch.zeros(1, eng.hidden, dtype=torch.bfloat16, device=dev)
        self.lg = torch.zeros(1, 4, dtype=torch.float32, device=dev)

    def __call__(self):
        a = (self.x, self.rows, self.pos, self.rows)
        kw = dict(hidden_out=self.h, logits_out=self.lg, max_pos=self.eng.max_ctx - 1)   # the loop's graph plan
        if self.peers is None:
            self.eng.lm_forward(*a, **kw)
        else:
            self.eng.lm_forward_group(self.peers, *a, **kw)
        return self.out()

    def out(self):
        return self.h.clone(), self.lg.clone()


def test_64k_graph_decode_matches_eager():
    """configs[4]'s decode step as the loop runs it — captured into a hipGraph
    with the max_ctx split plan and replayed — at a real 65,000-token context
    (prefilled by k_attn_pf / k_gemm_xl, 1.5B layer shapes, 2 layers): bitwise
    equal to eager launches, and the first replayed step vs oracle/lm.py."""
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    cfg.decoder_config["max_position_embeddings"] = 65536
    sd = synthetic_state_dict(cfg, seed=26, device="cpu", mode="test", with_acoustic_encoder=False)
    N = 65000
    eng = Engine(cfg, sd, dev, max_batch=1, max_ctx=N + 40, valid_ids=VALID)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(N, 1536, device=dev, generator=g).bfloat16()
    eng.lm_forward(x, torch.zeros(N, **I32), torch.arange(N).to(**I32), torch.tensor([N - 1]).to(**I32))
    steps = torch.randn(4, 1536, device=dev, generator=g).bfloat16()
    dec = _Dec(eng)

    def set_step(s):
        dec.x.copy_(steps[s:s + 1])
        dec.pos.fill_(N + s)
    eager, replayed = _graph_vs_eager(dec, set_step, 4)
    for s, ((he, le), (hg, lg)) in enumerate(zip(eager, replayed)):
        print(f"64K graph step {s} (attends {N + s + 1} keys): bitwise {torch.equal(he, hg) and torch.equal(le, lg)}")
        assert torch.equal(he, hg) and torch.equal(le, lg)
    osd, lcfg = oracle_sd(sd, dev), dict(cfg.decoder_config)
    kv = olm.RowKV(2)
    with torch.no_grad():
        _oracle_prefill_gpu(osd, lcfg, x, kv)
        ref = olm.forward_rows(osd, lcfg, steps[None, :1], [kv])[0, -1]
    print(f"64K graph step 0 vs oracle: rel {rel_err(replayed[0][0], ref):.3e} cos {cos(replayed[0][0], ref):.6f}")
    assert rel_err(replayed[0][0], ref) < 2e-2 and cos(replayed[0][0], ref) > 0.999


def test_tp2_long_context_matches_single_engine():
    """configs[4] under TP = 2 (1.5B: 2 kv heads -> one per rank): a
    65,000-token prefill and decode steps, group vs the TP = 1 engine; then the
    group's decode captured into a hipGraph and replayed, bitwise equal to the
    group's eager launches."""
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    cfg.decoder_config["max_position_embeddings"] = 65536
    sd = synthetic_state_dict(cfg, seed=25, device="cpu", mode="test", with_acoustic_encoder=False)
    N = 65000
    full = Engine(cfg, sd, dev, max_batch=1, max_ctx=N + 40, valid_ids=VALID)
    group = [Engine(cfg, sd, dev, max_batch=1, max_ctx=N + 40, valid_ids=VALID, tp_rank=r, tp_size=2)
             for r in range(2)]
    g = torch.Generator(device=dev).manual_seed(6)
    x = torch.randn(N, 1536, device=dev, generator=g).bfloat16()
    args = (x, torch.zeros(N, **I32), torch.arange(N).to(**I32), torch.tensor([N - 1]).to(**I32))
    h1, l1 = full.lm_forward(*args)
    hg, lg = group[0].lm_forward_group(group[1:], *args)
    torch.cuda.synchronize()
    print(f"TP=2 65K prefill: rel {rel_err(hg, h1):.3e} cos {cos(hg, h1):.6f}")
    assert rel_err(hg, h1) < 2e-2 and cos(hg, h1) > 0.999
    steps = torch.randn(3, 1536, device=dev, generator=g).bfloat16()
    for s in range(3):
        a = (steps[s:s + 1], torch.zeros(1, **I32), torch.tensor([N + s]).to(**I32), torch.zeros(1, **I32))
        h1, _ = full.lm_forward(*a)
        hg, _ = group[0].lm_forward_group(group[1:], *a)
        torch.cuda.synchronize()
        print(f"TP=2 65K step {s}: rel {rel_err(hg, h1):.3e} cos {cos(hg, h1):.6f}")
        assert rel_err(hg, h1) < 2e-2 and cos(hg, h1) > 0.999
    dec = _Dec(group[0], group[1:])

    def set_step(s):
        dec.x.copy_(steps[s:s + 1])
        dec.pos.fill_(N + s)
    eager, replayed = _graph_vs_eager(dec, set_step, 3)
    for s, ((he, le), (hr, lr)) in enumerate(zip(eager, replayed)):
        print(f"TP=2 65K graph step {s}: bitwise {torch.equal(he, hr) and torch.equal(le, lr)}")
        assert torch.equal(he, hr) and torch.equal(le, lr)


def test_28_layer_32k_prefill_graph_decode_vs_oracle():
    """configs[4]'s long-context path at FULL depth: VibeVoice-1.5B's 28 Qwen2
    layers (H 1536, 12 q / 2 kv heads, I 8960), a 32,768-token causal prefill
    through the product path (k_attn_pf + k_gemm_xl), then 3 decode steps
    captured into ONE hipGraph with the loop's max_ctx split plan and replayed
    (k_attn splits + merge over 32K keys) — bitwise equal to the eager
    launches, and every replayed step's final-norm hidden state within rel L2
    3e-2 of oracle/lm.py (the full-size hidden bound, tests/teacher.py) run as
    the checker on the GPU."""
    cfg = tiny_config(hidden=1536, layers=28, heads=12, kv_heads=2, inter=8960)
    cfg.decoder_config["max_position_embeddings"] = 65536
    sd = synthetic_state_dict(cfg, seed=27, device=dev, mode="test", with_acoustic_encoder=False)
    N = 32768
    eng = Engine(cfg, sd, dev, max_batch=1, max_ctx=N + 40, valid_ids=VALID)
    g = torch.Generator(device=dev).manual_seed(8)
    x = torch.randn(N, 1536, device=dev, generator=g).bfloat16()
    hp, _ = eng.lm_forward(x, torch.zeros(N, **I32), torch.arange(N).to(**I32), torch.tensor([N - 1]).to(**I32))
    steps = torch.randn(3, 1536, device=dev, generator=g).bfloat16()
    dec = _Dec(eng)

    def set_step(s):
        dec.x.copy_(steps[s:s + 1])
        dec.pos.fill_(N + s)
    eager, replayed = _graph_vs_eager(dec, set_step, 3)
    osd, lcfg = oracle_sd(sd, dev), dict(cfg.decoder_config)
    kv = olm.RowKV(28)
    with torch.no_grad():
        ref_p = _oracle_prefill_gpu(osd, lcfg, x, kv)
    e = rel_err(hp, ref_p)
    print(f"28-layer 32K prefill: rel {e:.3e} cos {cos(hp, ref_p):.6f}")
    assert e < 3e-2 and cos(hp, ref_p) > 0.999
    for s, ((he, le), (hr, lr)) in enumerate(zip(eager, replayed)):
        with torch.no_grad():
            ref = olm.forward_rows(osd, lcfg, steps[None, s:s + 1], [kv])[0, -1]
        torch.cuda.synchronize()
        e = rel_err(hr, ref)
        same = torch.equal(he, hr) and torch.equal(le, lr)
        print(f"28-layer 32K graph step {s} (attends {N + s + 1} keys): bitwise-eager {same} "
              f"rel {e:.3e} cos {cos(hr, ref):.6f}")
        assert same
        assert e < 3e-2 and cos(hr, ref) > 0.999


def test_long_context_grouped_split_merge_ragged_rows():
    """Decode over contexts past 8,192 keys with rows of very different lengths
    (20,000 / 9,001 / 300 keys, max_ctx 32K): up to 128 splits of >= 256 keys,
    each group of consecutive splits merged by its last-arriving workgroup and
    the groups merged by o_proj (XF_ATTN_MERGE) — vs oracle/lm.py, and vs the
    1,024-key plan with k_attn_merge (vv_attn_group(0)) within bf16."""
    from vibevoice_amd import _lib
    cfg = tiny_config(hidden=1536, layers=2, heads=12, kv_heads=2, inter=8960)
    cfg.decoder_config["max_position_embeddings"] = 65536
    sd = synthetic_state_dict(cfg, seed=28, device="cpu", mode="test", with_acoustic_encoder=False)
    eng = Engine(cfg, sd, dev, max_batch=3, max_ctx=32768, valid_ids=VALID)
    osd, lcfg = oracle_sd(sd, dev), dict(cfg.decoder_config)
    g = torch.Generator(device=dev).manual_seed(9)
    lens = [20000, 9001, 300]
    kvs = []
    for r, n in enumerate(lens):   # one slot at a time (k_attn_pf prefill of each row)
        x = torch.randn(n, 1536, device=dev, generator=g).bfloat16()
        eng.lm_forward(x, torch.full((n,), r, **I32), torch.arange(n).to(**I32), torch.tensor([n - 1]).to(**I32))
        kv = olm.RowKV(2)
        with torch.no_grad():
            _oracle_prefill_gpu(osd, lcfg, x, kv)
        kvs.append(kv)
    L = torch.tensor(lens)
    rows = torch.arange(3).to(**I32)
    for s in range(2):
        step = torch.randn(3, 1536, device=dev, generator=g).bfloat16()
        outs = {}
        for mode in (1, 0):
            _lib.lib().vv_attn_group(mode)
            try:
                outs[mode], _ = eng.lm_forward(step, rows, (L + s).to(**I32), rows, max_pos=32767)
            finally:
                _lib.lib().vv_attn_group(1)
        with torch.no_grad():
            ref = olm.forward_rows(osd, lcfg, step[:, None], kvs)[:, -1]
        torch.cuda.synchronize()
        for r in range(3):
            e, e0 = rel_err(outs[1][r], ref[r]), rel_err(outs[1][r], outs[0][r])
            print(f"grouped merge step {s} row {r} ({lens[r] + s + 1} keys): rel {e:.3e} vs oracle, "
                  f"{e0:.3e} vs the k_attn_merge plan")
            assert e < 2e-2 and cos(outs[1][r], ref[r]) > 0.999
            assert e0 < 1e-2


@pytest.mark.parametrize("tp,n", [(4, 1), (4, 4), (2, 4)])
def test_large_head_tp_group_matches_single_engine(tp, n):
    """configs[3]: the VibeVoice-Large diffusion head (H 3,584, FFN 10,752,
    4 layers, S = 10, CFG 1.3) sharded over `tp` ranks (gate|up
    column-parallel, down row-parallel, one all-reduce of [2n, H] per head
    layer; adaLN / noisy / final / DPM replicated) — the ranks' shards
    interleaved on one GPU with an on-device sum as the all-reduce
    (vv_diffusion_sample_group) — vs the TP = 1 engine and vs oracle/head.py,
    within bf16."""
    cfg = VibeVoiceConfig.builtin("Large")
    hc = cfg.diffusion_head_config
    lm_cfg = tiny_config(layers=1, **LARGE)
    sd = synthetic_state_dict(lm_cfg, seed=22, device="cpu", mode="test", with_acoustic_encoder=False)
    hsd = {k[len("model.prediction_head."):]: v for k, v in sd.items() if k.startswith("model.prediction_head.")}
    full = Engine(lm_cfg, sd, dev, max_batch=4, max_ctx=64)
    group = [Engine(lm_cfg, sd, dev, max_batch=4, max_ctx=64, tp_rank=r, tp_size=tp, tp_head=True) for r in range(tp)]
    assert group[1].w["head.0.down_w"].shape == (3584, 10752 // tp)
    S = 10
    full.set_steps(S)
    group[0].set_steps(S)
    g = torch.Generator().manual_seed(10 + n)
    pos = torch.randn(n, 3584, generator=g).bfloat16()
    neg = torch.randn(n, 3584, generator=g).bfloat16()
    noise = torch.randn(2 * n, 64, generator=g).bfloat16()
    x1 = noise[:n].to(dev).contiguous()
    xg = x1.clone()
    full.diffusion_sample(pos.to(dev), neg.to(dev), x1, 1.3)
    group[0].diffusion_sample_group(group[1:], pos.to(dev), neg.to(dev), xg, 1.3)
    torch.cuda.synchronize()
    ref = ohead.sample_speech_tokens(hsd, pos, neg, noise, S, 1.3, hc.head_layers)
    e1, eg = rel_err(xg, x1), rel_err(xg, ref)
    print(f"Large head TP={tp} n={n}: rel {e1:.3e} vs TP=1, {eg:.3e} vs oracle (TP=1 vs oracle {rel_err(x1, ref):.3e})")
    assert e1 < 2e-2 and cos(xg, x1) > 0.999
    assert eg < 2e-2 and cos(xg, ref) > 0.999
    # a sharded engine refuses the single-engine call without a communicator
    with pytest.raises(RuntimeError):
        group[1].diffusion_sample(pos.to(dev), neg.to(dev), xg.clone(), 1.3)
