"""Throughput of VibeVoice's next-token-diffusion generate loop on MI355X.

One bench "step" = one iteration of the reference's generate loop
(vibevoice/modular/modeling_vibevoice_inference.py:432-690) for every sample
of the batch, through the product path (GenerateSession.step -> the C-ABI of
libvibevoice_hip.so): positive + negative Qwen2 decode (batched rows), the
constrained argmax read back to the host, S-step CFG DPM-Solver++ diffusion
head, streaming acoustic decode + semantic encode, connectors.  The token
schedule is forced to `speech_diffusion` (random weights emit arbitrary control
tokens), so every step emits one 3200-sample audio frame per sample.

Default workload = BASELINE.json configs[1]: VibeVoice-1.5B bf16, 1 speaker
(3 s voice prompt + 1-sentence script), 10 diffusion steps, TP=1, one MI355X.
`--batch 8 --speakers 2` is configs[2].  With `--gpus N` every rank (one
process per GPU) runs its own independent dialogues: DP replicas, no
collective on the data path (DESIGN.md "Multi-GPU").  `--tp T` groups T
consecutive ranks into one tensor-parallel replica (RCCL all-reduce).
`--gpus N` outside a torchrun environment starts the N ranks itself (a child
`torch.distributed.run` on 127.0.0.1, before this process touches a GPU) and
exits with its status; inside one, WORLD_SIZE must equal N.

Prints ONE JSON line on rank 0 (metric contract: BASELINE.json / SURVEY.md §8d).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SR, HOP = 24000, 3200
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
IC_MEASURED_GBS = 8600.0       # Infinity-Cache-resident reads, measured (MI355X_MICROARCH.md "Indexed rows")
METRIC = "audio-sec/wall-sec (RTF) + acoustic tokens/sec, VibeVoice-1.5B at 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=750, help="timed steps (SURVEY.md §8d C2: K = 750, 100 s of audio)")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1, help="dialogues per GPU")
    ap.add_argument("--speakers", type=int, default=1)
    ap.add_argument("--ddpm-steps", type=int, default=10)
    ap.add_argument("--model", default="1.5B", choices=["1.5B", "Large"])
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel ranks per model replica (RCCL)")
    ap.add_argument("--context", type=int, default=0,
                    help="prompt length in tokens: a long script prefilled through the product path "
                         "(k_attn_pf + k_gemm_xl) before timing decode at that context "
                         "(SURVEY.md §8d config 5: 64K-position decode)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-tokens", type=int, default=8, help="timed tokens of the CPU oracle sample")
    ap.add_argument("--plumbing", action="store_true",
                    help="tests only: run the launch / barrier / max-over-ranks / JSON path with an empty step "
                         "(no engine; works on a CPU host over gloo)")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def maybe_launch(args, argv=None):
    """`--gpus N` (N > 1) without a torchrun environment: run this script under
    `torch.distributed.run` with N ranks on 127.0.0.1 as a CHILD process and
    return its exit status (None: nothing launched, run in-process).  Called
    before any GPU call, so this process never initialises the GPU."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess
    argv = sys.argv[1:] if argv is None else argv
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def tp_groups(world, rank, T):
    """Consecutive ranks form one TP group of T; the groups are DP replicas.
    Every rank creates every group (torch.distributed.new_group is collective).
    Returns (this rank's group or None for T == 1, replica index, replicas)."""
    if world % T:
        raise SystemExit(f"--tp {T} must divide the {world} ranks")
    group = None
    if T > 1:
        groups = [torch.distributed.new_group(list(range(g * T, (g + 1) * T))) for g in range(world // T)]
        group = groups[rank // T]
    return group, rank // T, world // T


# ------------------------------------------------------------------ algorithmic bytes
HEAD_SC = 16   # engine.cpp: the adaLN modulations of up to 16 diffusion steps come from ONE batched GEMM


def weight_bytes(w, B=1, S=10):
    """Bytes of the packed device weights the loop reads, by role (SURVEY.md §8d
    conventions).  head_step: read by EVERY diffusion step (noisy / final
    projections, the per-layer norms and FFN weights in the layout the loop
    reads); head_token: read once per token (cond_proj, and the
    stacked adaLN matrix once per HEAD_SC steps -- its GEMM covers the steps'
    modulations at once)."""
    def sz(pred):
        return sum(t.numel() * t.element_size() for k, t in w.items() if pred(k))
    H = w["lm.norm"].numel()
    ffn = (".gu_w", ".down_w")

    def per_step(k):
        if k in ("head.noisy_w", "head.final_w"):
            return True
        parts = k.split(".")
        return len(parts) == 3 and parts[1].isdigit() and (parts[2] == "norm" or k.endswith(ffn))
    return dict(
        lm=sz(lambda k: k.startswith("lm.") and k.split(".")[1].isdigit()) + sz(lambda k: k == "lm.norm"),
        lm_head4=4 * H * 2,
        head_step=sz(lambda k: k.startswith("head.") and per_step(k)),
        head_token=sz(lambda k: k == "head.cond_w") + -(-S // HEAD_SC) * sz(lambda k: k == "head.ada_w"),
        codec=sz(lambda k: k.startswith("dec.") or k.startswith("sem.")),
        conn=sz(lambda k: k.startswith("conn.")),
        head_layout="GEMV layout (gu_w / down_w)",
    )


def bytes_per_token(wb, cfg, B, S, ctx_pos, ctx_neg):
    lmc = cfg.decoder_config
    d = lmc.get("head_dim") or lmc.hidden_size // lmc.num_attention_heads
    kv_pos = lmc.num_hidden_layers * 2 * lmc.num_key_value_heads * d * 2      # 28,672 B at 1.5B
    shared = wb["lm"] + wb["lm_head4"] + S * wb["head_step"] + wb["head_token"] + wb["codec"] + wb["conn"]
    return shared / B + kv_pos * (ctx_pos + ctx_neg + 2)


def roof(kernel, shape, alg_bytes, seconds, traffic=None, **extra):
    """A roofline object against the 8 TB/s HBM peak.  A fraction above 1 is a
    measurement error (e.g. events on an idle stream), never a result: it is
    reported as an `error` field with no `frac`."""
    ach = alg_bytes / seconds / 1e9 if seconds > 0 else float("inf")
    d = dict(kernel=kernel, shape=shape, bound="hbm", peak=HBM_PEAK_GBS, unit="GB/s", avg_us=round(seconds * 1e6, 2),
             alg_bytes_per_launch=int(alg_bytes), traffic=traffic,
             traffic_unit="HBM bytes per launch (rocprofv3 PMC)" if traffic else None)
    if not (ach / HBM_PEAK_GBS <= 1.0):
        d.update(achieved=None, frac=None,
                 error=f"implausible: {alg_bytes} B in {seconds * 1e6:.2f} us = {ach:.0f} GB/s exceeds the peak")
    else:
        d.update(achieved=round(ach, 1), frac=round(ach / HBM_PEAK_GBS, 4))
    d.update(extra)
    return d


# ------------------------------------------------------------------ dominant kernel, live
# U = 4 chunks in flight, XF_NORM, non-temporal weights, tiles per workgroup (gemm.hip gemv_resolve: 1 at
# M < 8; at 8 <= M <= 16 the balanced form, 4-5 of the 1,120 tiles on each of the 256 CUs: TPW = 5),
# row-per-wave norm prologue (RW = 1); HBM traffic per launch from tools/pmc_traffic.py (rocprofv3 PMC,
# committed per M)
def roof_kernel(M):
    return f"k_gemv1<4, 1, false, {5 if M >= 8 else 1}, 1>"


def pmc_file(M):
    for r in ("r05", "r04", "r03"):
        p = os.path.join(ROOT, "profiles", f"{r}_pmc_traffic_m{M}.json")
        if os.path.exists(p):
            return p
    return os.path.join(ROOT, "profiles", f"r04_pmc_traffic_m{M}.json")


def measure_gemv(model, B, iters=6):
    """The LM MLP gate|up weight-streaming GEMV (k_gemv1, XF_NORM prologue,
    EPI_SILU_MUL): the largest single launch of the loop (2I x H bf16 = 55 MB at
    1.5B, 28 per LM pass).  vv_gemm_bf16_norm with the engine handle goes
    through the engine's own GEMM dispatch, so at M = 2B > 16 this times what
    the loop launches there (k_rmsnorm once + the GEMV on normalised rows).  The 28 layers' launches are captured into a hipGraph
    (as the loop runs them) and replayed; HIP events on the replay stream time
    `iters` replays.  Rotating over the 28 layers' weights (1.5 GB) keeps the
    Infinity Cache from serving them.  `traffic`: HBM bytes per launch from the
    rocprofv3 PMC passes of tools/pmc_traffic.py (FETCH_SIZE x 2 on gfx950 +
    WRITE_SIZE, MI355X_MICROARCH.md "HBM"), committed in profiles/."""
    from vibevoice_amd import _lib
    eng = model.engine
    lmc = model.config.decoder_config
    H, I, nl = lmc.hidden_size, lmc.intermediate_size, lmc.num_hidden_layers
    M = 2 * B
    A = torch.randn(M, H, device=model.device).bfloat16()
    norm_w = [eng.w[f"lm.{l}.post_norm"] for l in range(nl)]
    Y = torch.empty(M, I, device=model.device, dtype=torch.bfloat16)
    L = _lib.lib()
    Ws = [eng.w[f"lm.{l}.gu_w"] for l in range(nl)]

    def run():
        sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for Wt, nw_ in zip(Ws, norm_w):   # the in-loop variant: post_attention_layernorm fused on load
            _lib.check(L.vv_gemm_bf16_norm(M, 2 * I, H, ctypes.c_void_p(A.data_ptr()), H,
                                           ctypes.c_void_p(nw_.data_ptr()), float(lmc.rms_norm_eps),
                                           ctypes.c_void_p(Wt.data_ptr()), _lib.EPI["silu_mul"],
                                           ctypes.c_void_p(Y.data_ptr()), I, eng.h, sp), "gemv")
    run()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    g.replay()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        g.replay()
    e1.record(stream)
    e1.synchronize()
    avg_s = e0.elapsed_time(e1) / 1e3 / (iters * nl)
    alg = 2 * I * H * 2 + M * H * 2 + M * I * 2
    shape = f"M={M} N={2 * I} K={H}"
    traffic = None
    if os.path.exists(pmc_file(M)):
        with open(pmc_file(M)) as f:
            pmc = json.load(f)
        if pmc.get("kernel") == roof_kernel(M) and pmc.get("shape") == shape:
            traffic = pmc["hbm_bytes_per_launch"]
    kernel = (f"{roof_kernel(M)} (LM post-norm + gate|up + SiLU*up, graph-replayed)" if M <= 16 else
              "k_rmsnorm + k_gemv/k_gemvw (the engine's M > 16 dispatch: post-norm once, then gate|up + SiLU*up; "
              "graph-replayed, both launches timed)")
    return roof(kernel, shape, alg, avg_s, traffic, launches_per_token=nl)


def measure_lm_ffn(model, B, reps=2, iters=4):
    """The LM MLP block as the B = 1 loop runs it: ONE k_lm_ffn launch per layer
    (lm_ffn.hip: post-norm + gate|up + SiLU*up + down + residual, one grid-wide
    hand-off; decode with 2B <= 2 rows).  vv_lm_mlp_replay runs 1 or 1 + reps
    passes over the 28 layers' blocks inside two captured graphs (rotating over
    2.3 GB of weights: no cache reuse); the difference of their replay times
    (HIP events on the replay stream) over reps x layers is the time per block.
    Algorithmic bytes per block: gate|up + down weights + the rows in / out."""
    from vibevoice_amd import _lib
    eng = model.engine
    lmc = model.config.decoder_config
    H, I, nl = lmc.hidden_size, lmc.intermediate_size, lmc.num_hidden_layers
    M = 2 * B
    lib = _lib.lib()
    if lib.vv_lm_ffn_active(eng.h, M) != 1:
        return None
    x = (torch.randn(M, H, device=model.device) * 0.5).bfloat16()
    act = torch.empty(M, I, device=model.device, dtype=torch.bfloat16)
    stream = torch.cuda.Stream(model.device)

    def call(n):
        return lib.vv_lm_mlp_replay(eng.h, M, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(act.data_ptr()), n,
                                    ctypes.c_void_p(stream.cuda_stream))
    with torch.cuda.stream(stream):
        _lib.check(call(1), "lm_mlp_replay")
    stream.synchronize()

    def graph(n):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            g.capture_begin(capture_error_mode="thread_local")
            try:
                rc = call(n)
            finally:
                g.capture_end()
        _lib.check(rc, "lm_mlp_replay")
        return g
    g1, gn = graph(1), graph(1 + reps)
    times = []
    with torch.cuda.stream(stream):
        for g in (g1, gn):
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                g.replay()
            e1.record(stream)
            e1.synchronize()
            times.append(e0.elapsed_time(e1) / 1e3 / iters)
    eng.check_sync()
    per = (times[1] - times[0]) / (reps * nl)
    alg = 3 * I * H * 2 + M * H * 2 * 2
    shape = f"rows={M} H={H} I={I}"
    traffic = None
    for pf in (os.path.join(ROOT, "profiles", f"r06_pmc_lm_ffn_r{M}.json"),
               os.path.join(ROOT, "profiles", f"r05_pmc_lm_ffn_r{M}.json")):
        if traffic is None and os.path.exists(pf):
            with open(pf) as f:
                pmc = json.load(f)
            if pmc.get("kernel") == ("k_lm_ffn" if M <= 2 else "k_lm_ffn16") and pmc.get("shape") == shape:
                traffic = pmc["hbm_bytes_per_launch"]
    kname = "k_lm_ffn" if M <= 2 else "k_lm_ffn16"
    return roof(f"{kname} (LM post-norm + gate|up + SiLU*up + down + residual in one launch, one grid-wide "
                "hand-off; graph-replayed)", shape, alg, per, traffic, launches_per_token=nl,
                note="graph-replayed MLP blocks of the 28 layers (vv_lm_mlp_replay), HIP events on the replay "
                     "stream; weights read once per pass (2.3 GB rotation), non-temporal")


def measure_lm_attn(model, B, ctx, reps=2, iters=4):
    """The LM attention half as the loop runs it at this batch: ONE k_lm_attn
    launch per layer (lm_attn.hip: input_layernorm + q|k|v + RoPE + KV append,
    attention, o_proj + residual; decode with 2B <= 16 rows and <= 4,096 keys).
    vv_lm_attn_replay runs 1 or 1 + reps passes over the 28 layers' attention
    halves, 2B rows at position ~ctx (the loop's average context; after the timed
    loop, so the cache rows it overwrites are no longer read), inside two captured
    graphs; the difference of their replay times (HIP events on the replay
    stream) over reps x layers is the time per half.  Algorithmic bytes: q|k|v
    (+bias) and o_proj weights, the norm weight, the rows in / out, the K / V
    rows read (ctx + 1 keys per row) and appended."""
    from vibevoice_amd import _lib
    eng = model.engine
    lmc = model.config.decoder_config
    H, nl = lmc.hidden_size, lmc.num_hidden_layers
    nh, nkv = lmc.num_attention_heads, lmc.num_key_value_heads
    d = H // nh
    M = 2 * B
    lib = _lib.lib()
    keys = int(ctx) + 1
    if lib.vv_lm_attn_active(eng.h, M, keys) != 1:
        return None
    dev = model.device
    x = (torch.randn(M, H, device=dev) * 0.5).bfloat16()
    slots = torch.arange(M, device=dev, dtype=torch.int32)
    pos = torch.full((M,), keys - 1, device=dev, dtype=torch.int32)
    stream = torch.cuda.Stream(dev)

    def call(n):
        return lib.vv_lm_attn_replay(eng.h, M, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(slots.data_ptr()),
                                     ctypes.c_void_p(pos.data_ptr()), keys, n, ctypes.c_void_p(stream.cuda_stream))
    with torch.cuda.stream(stream):
        _lib.check(call(1), "lm_attn_replay")
    stream.synchronize()

    def graph(n):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            g.capture_begin(capture_error_mode="thread_local")
            try:
                rc = call(n)
            finally:
                g.capture_end()
        _lib.check(rc, "lm_attn_replay")
        return g
    g1, gn = graph(1), graph(1 + reps)
    times = []
    with torch.cuda.stream(stream):
        for g in (g1, gn):
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                g.replay()
            e1.record(stream)
            e1.synchronize()
            times.append(e0.elapsed_time(e1) / 1e3 / iters)
    eng.check_sync()
    per = (times[1] - times[0]) / (reps * nl)
    nq = (nh + 2 * nkv) * d
    alg = (nq * H + nq + H * H + H) * 2 + M * H * 2 * 2 + M * keys * nkv * d * 2 * 2 + M * nkv * d * 2 * 2
    return roof("k_lm_attn (LM attention half in one launch: input_layernorm + q|k|v + RoPE + KV append, "
                "attention over 32-key units, merge, o_proj + residual; three grid waits; graph-replayed)",
                f"rows={M} H={H} keys={keys}", alg, per, None, launches_per_token=nl,
                note="graph-replayed attention halves of the 28 layers (vv_lm_attn_replay), HIP events on the "
                     "replay stream; latency-bound (11 MB of weights + the KV rows per launch)")


def measure_head_layers(model, B, reps=10, iters=4):
    """The diffusion head's FFN layers as the loop runs them at this batch
    (vv_head_layers_replay: k_head_m16, one launch per layer at 2 <= 2n <= 16
    rows; else the gate|up + down GEMVs), S x head_layers of them per token.  Two graphs (1 and
    1 + reps passes over the layers, each after the same condition / adaLN set-up)
    are replayed on one stream between HIP events; their difference over reps x
    head_layers is the time per layer.  Algorithmic bytes per layer: the layer's
    gate|up and down weights + its rows."""
    from vibevoice_amd import _lib
    eng = model.engine
    hc = model.config.diffusion_head_config
    H, L = hc.hidden_size, hc.head_layers
    F = int(H * hc.head_ffn_ratio) // (eng.tp_size if eng.tp_head else 1)
    if eng.tp_head:
        return None
    R = 2 * B
    cond = torch.randn(R, H, device=model.device).bfloat16()
    lib = _lib.lib()
    stream = torch.cuda.Stream(model.device)

    def graph(passes):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            g.capture_begin(capture_error_mode="thread_local")
            try:
                rc = lib.vv_head_layers_replay(eng.h, B, ctypes.c_void_p(cond.data_ptr()),
                                               ctypes.c_void_p(cond[B:].data_ptr()), passes,
                                               ctypes.c_void_p(stream.cuda_stream))
            finally:
                g.capture_end()
        _lib.check(rc, "head_layers_replay")
        return g

    with torch.cuda.stream(stream):   # eager warm-up (plans, workspaces)
        _lib.check(lib.vv_head_layers_replay(eng.h, B, ctypes.c_void_p(cond.data_ptr()),
                                             ctypes.c_void_p(cond[B:].data_ptr()), 1,
                                             ctypes.c_void_p(stream.cuda_stream)), "head_layers_replay")
    stream.synchronize()
    g1, gn = graph(1), graph(1 + reps)
    times = []
    # graph replays launch on the CURRENT stream: replay and record the events on
    # the same one (round 4 recorded them on an idle stream: frac 29.4)
    with torch.cuda.stream(stream):
        for g in (g1, gn):
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                g.replay()
            e1.record(stream)
            e1.synchronize()
            times.append(e0.elapsed_time(e1) / 1e3 / iters)
    eng.check_sync()
    per_layer = (times[1] - times[0]) / (reps * L)
    alg = 3 * F * H * 2 + R * H * 2 * 2
    m16 = lib.vv_head_m16_active(eng.h, B) == 1
    kernel = ("k_head_m16 (one head FFN layer at 2n <= 16 rows in one launch: MFMA gate|up + SiLU*up, one "
              "grid-wide hand-off, MFMA down + gated residual; above 4 rows the A side built distributed)" if m16 else
              "k_gemv1 gate|up + k_gemv/k_gemv1 down (one head FFN layer = two GEMV launches, timed together)")
    traffic = None
    for pf in (os.path.join(ROOT, "profiles", f"r06_pmc_head_r{R}.json"),
               os.path.join(ROOT, "profiles", f"r05_pmc_head_r{R}.json")):
        if traffic is None and os.path.exists(pf):
            with open(pf) as f:
                pmc = json.load(f)
            if pmc.get("kernel") == kernel.split(" (")[0] and pmc.get("shape") == f"rows={R} H={H} F={F}":
                traffic = pmc["hbm_bytes_per_launch"]
    return roof(kernel, f"rows={R} H={H} F={F}", alg, per_layer, traffic,
                launches_per_token=int(model.ddpm_inference_steps * L),
                note="graph-replayed head FFN layers (vv_head_layers_replay), HIP events on the replay stream; "
                     "the head's 170 MB are re-read by each of the S steps and served from the 256 MB Infinity "
                     "Cache (default cache policy), so the bound is the Infinity-Cache read rate, not HBM",
                ic_roof=dict(peak=IC_MEASURED_GBS, unit="GB/s",
                             frac=round(alg / per_layer / 1e9 / IC_MEASURED_GBS, 4) if per_layer > 0 else None,
                             source="MI355X_MICROARCH.md 'Indexed rows: gather into LDS': a 38 MB "
                                    "Infinity-Cache-resident table read at 8.6 TB/s chip-wide (a measured "
                                    "rate; the guide states no spec peak for the Infinity Cache)"))


def us_per_step(r):
    """A roofline candidate's time per loop step: from the committed step profile
    of the loop when it holds the kernel (the loop's own clock: the isolated
    replays of the three candidates differ from it by up to ~5 %), else the
    replay average x launches per step."""
    if not r or "error" in r or not r.get("avg_us"):
        return -1.0
    if r.get("in_loop"):
        return r["in_loop"]["us_per_step"]
    return r["avg_us"] * r.get("launches_per_token", 1)


def pick_roofline(*cands):
    """(roofline, roofline_2): the candidates ordered by time per step, largest
    first -- the dominant kernel of the step is the line's `roofline`."""
    c = sorted([r for r in cands if r is not None], key=us_per_step, reverse=True)
    return (c[0] if c else None), (c[1] if len(c) > 1 else None)


# the committed step profile of this round per batch (tools/prof_step.sh: rocprofv3 --kernel-trace over
# bench.py's timed loop, profiles/summarize.py over its last 20 steps): the per-kernel averages in the loop
STEP_PROFILE = {1: "r06_step_kernels_b1.json", 8: "r06_step_kernels_b8.json"}


def in_loop_average(r, B):
    """Beside the isolated replay: the kernel's average duration inside the loop
    itself, from the committed step profile for this batch (if one exists), and
    the roofline fraction at that average."""
    name = STEP_PROFILE.get(B)
    path = os.path.join(ROOT, "profiles", name) if name else None
    if not path or not os.path.exists(path):
        return
    with open(path) as f:
        prof = json.load(f)["kernels"]
    k = prof.get(r["kernel"].split(" (")[0])
    if k:
        r["in_loop"] = dict(avg_us=k["avg_us"], us_per_step=k["us_per_step"], source=f"profiles/{name}",
                            frac=round(r["alg_bytes_per_launch"] / (k["avg_us"] * 1e-6) / 1e9 / r["peak"], 4))


# ------------------------------------------------------------------ TP collective share
def measure_tp_collective(make_pass, n_layers, world, dev, iters=20, reps=3):
    """Time of one LM pass with its 2 x n_layers RCCL all-reduces and with
    them skipped (vv_tp_null_collective: the outputs are then wrong, so this
    runs after the timed loop), max over ranks; their difference is the
    collectives' share of the pass.  make_pass(null) returns a callable that
    runs one pass (a hipGraph replay of the loop's LM phase, captured with the
    switch set as given).  Each figure is the best of `reps` interleaved
    blocks of `iters` passes (a block's time is the slowest rank's), so a
    noisy block on a shared host does not invert the two."""
    runs = {null: make_pass(null) for null in (False, True)}

    def timed(run):
        run()
        barrier(world)
        t0 = time.perf_counter()
        for _ in range(iters):
            run()
        barrier(world)
        return max_over_ranks(time.perf_counter() - t0, world, dev) / iters
    best = {False: float("inf"), True: float("inf")}
    for _ in range(reps):
        for null in (False, True):
            best[null] = min(best[null], timed(runs[null]))
    on, off = best[False], best[True]
    return dict(lm_pass_us=round(on * 1e6, 2), lm_pass_us_null_collective=round(off * 1e6, 2),
                allreduce_us_per_pass=round(max(0.0, on - off) * 1e6, 2), allreduce_calls_per_pass=2 * n_layers,
                allreduce_share=round(max(0.0, on - off) / on, 4) if on > 0 else None,
                note="RCCL all-reduce (sum, bf16, in place) of the [2B, H] residual after o_proj and down_proj; "
                     "max over ranks of graph-replayed LM passes with / without the collectives")


def head_pass_maker(model, sess):
    """make_pass for the sharded diffusion head (tp_head): one diffusion call of
    the loop (all B rows, S steps) with its S x head_layers all-reduces."""
    from vibevoice_amd import _lib
    eng, B = model.engine, sess.B
    L = _lib.lib()
    pos, neg = sess.hid[:B], sess.hid[B:]
    x = sess.noise_dev[:B]

    def make(null):
        L.vv_tp_null_collective(1 if null else 0)
        try:
            eng.diffusion_sample(pos, neg, x, 1.3)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                eng.diffusion_sample(pos, neg, x, 1.3)
        finally:
            L.vv_tp_null_collective(0)
        return g.replay
    return make


def lm_pass_maker(model, sess):
    """make_pass for measure_tp_collective: the loop's LM phase body on the
    session's static buffers, captured into a hipGraph per switch setting."""
    from vibevoice_amd import _lib
    eng, B = model.engine, sess.B
    L = _lib.lib()

    def body():
        eng.lm_forward(sess.x_in2[:B], sess.rows2, sess.pos_dev, sess.rows2, hidden_out=sess.hid,
                       logits_out=sess.logits, max_pos=eng.max_ctx - 1, ntok=2 * B)

    def make(null):
        L.vv_tp_null_collective(1 if null else 0)
        try:
            body()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                body()
        finally:
            L.vv_tp_null_collective(0)
        return g.replay
    return make


# ------------------------------------------------------------------ CPU baseline (oracle)
def cpu_baseline(cfg, tokens, S, model_name="1.5B"):
    """The oracle's fp32 eager restatement of the reference loop (the
    reference's own CPU path runs fp32 + eager/sdpa attention,
    demo/inference_from_file.py:268) on the host cores: text prompt, forced
    diffusion tokens.  Per-token time = (T(1 + k tokens) - T(1 token)) / k."""
    from oracle import loop as oloop
    from vibevoice_amd.weights import synthetic_state_dict
    from vibevoice_amd.synthetic import synthetic_inputs, tokenizer_ids
    torch.manual_seed(0)
    sd = synthetic_state_dict(cfg, seed=0, device="cpu", dtype=torch.float32, with_acoustic_encoder=False)
    inp = synthetic_inputs(batch=1, speakers=1, voice_seconds=0, text_tokens=16, seed=1)
    tk = tokenizer_ids()
    ids = dict(eos=tk.eos_token_id, start=tk.speech_start_id, end=tk.speech_end_id, diffusion=tk.speech_diffusion_id)

    # per-stage clocks: the oracle functions the loop calls for
    # each stage, wrapped for the duration of the CPU leg
    stages = dict(lm_positive=(oloop.lm, "forward_rows"), lm_negative=(oloop.lm, "forward_rows_masked"),
                  diffusion=(oloop.head, "sample_speech_tokens"), acoustic_decode=(oloop.codec, "decode"),
                  semantic_encode=(oloop.codec, "encode"))
    clock = {k: 0.0 for k in stages}

    def timed(name, fn):
        def w(*a, **kw):
            t0 = time.perf_counter()
            try:
                return fn(*a, **kw)
            finally:
                clock[name] += time.perf_counter() - t0
        return w

    def run(k):
        forced = [[tk.speech_diffusion_id] * k + [tk.eos_token_id]]
        for n in clock:
            clock[n] = 0.0
        t0 = time.perf_counter()
        with torch.no_grad():
            oloop.generate(sd, cfg, inp["input_ids"], inp["attention_mask"], ids, ddpm_steps=S, cfg_scale=1.3,
                           forced=forced, dtype=torch.float32)
        return time.perf_counter() - t0, dict(clock)
    saved = {n: getattr(mod, attr) for n, (mod, attr) in stages.items()}
    for n, (mod, attr) in stages.items():
        setattr(mod, attr, timed(n, saved[n]))
    try:
        run(1)                                   # warm-up (allocator, thread pool)
        t1, c1 = run(1)
        tk_, ck = run(1 + tokens)
    finally:
        for n, (mod, attr) in stages.items():
            setattr(mod, attr, saved[n])
    per = (tk_ - t1) / tokens
    tps = 1.0 / per
    stage_ms = {n: round((ck[n] - c1[n]) / tokens * 1e3, 2) for n in stages}
    stage_ms["other"] = round(per * 1e3 - sum(stage_ms.values()), 2)
    return dict(value=round(tps * HOP / SR, 4), unit="audio-sec/wall-sec", tokens_per_s=round(tps, 3),
                cores=torch.get_num_threads(), kind="port", stage_ms_per_token=stage_ms,
                sample=f"oracle/loop.py fp32 eager on CPU, VibeVoice-{model_name} shapes (seeded random weights), "
                       f"B=1, S={S}, {tokens} timed diffusion tokens after a 1-token run (difference of two runs)")


# ------------------------------------------------------------------ multi-rank plumbing
def dist_setup():
    """One process per GPU (torchrun env).  Returns (world, rank, local, device).
    Backend: RCCL ("nccl") on the GPUs; gloo when no GPU is visible (CPU tests)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    # VV_BENCH_BACKEND=gloo rehearses the multi-rank path with every rank on
    # the visible GPU(s) (RCCL needs one GPU per rank)
    backend = os.environ.get("VV_BENCH_BACKEND", "nccl" if gpu else "gloo")
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count())) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return world, rank, local, dev


def barrier(world):
    if world > 1:
        torch.distributed.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def max_over_ranks(x, world, dev):
    """The job's time is the slowest rank's (contract: max over ranks)."""
    if world == 1:
        return float(x)
    gloo = torch.distributed.get_backend() == "gloo"
    t = torch.tensor([float(x)], device="cpu" if gloo else dev, dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def throughput(dt, batch, steps, world):
    """Whole-job acoustic tokens/s and audio-sec/wall-sec (weak scaling: every
    rank serves `batch` dialogues, one frame per dialogue per step)."""
    tps = batch * steps * world / dt
    return tps, tps * HOP / SR


# ------------------------------------------------------------------ main
def main():
    args = parse()
    rc = maybe_launch(args)
    if rc is not None:
        sys.exit(rc)
    world, rank, local, dev = dist_setup()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with --nproc-per-node {args.gpus}")
    if args.plumbing:
        return plumbing(args, world, rank, dev)

    from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
    from vibevoice_amd.synthetic import synthetic_inputs, tokenizer_ids

    B, S, K, W = args.batch, args.ddpm_steps, args.steps, args.warmup
    T = args.tp
    tp_group, replica, replicas = tp_groups(world, rank, T)
    total = W + K + 4
    text_tokens = 64
    if args.context:   # a long script: the timed steps end at most at max_position_embeddings (65,536 at 1.5B)
        from vibevoice_amd.config import VibeVoiceConfig
        mpe = VibeVoiceConfig.builtin(args.model).decoder_config.max_position_embeddings
        args.context = min(args.context, mpe - total - 8)
        base = synthetic_inputs(batch=1, speakers=args.speakers, voice_seconds=3.0, text_tokens=0, seed=0)
        text_tokens = max(64, args.context - base["input_ids"].shape[1])
    inp = synthetic_inputs(batch=B, speakers=args.speakers, voice_seconds=3.0, text_tokens=text_tokens,
                           seed=100 + replica)
    L = inp["input_ids"].shape[1]
    model = VibeVoiceForConditionalGenerationInference.from_pretrained(
        f"synthetic:{args.model}", device_map=str(dev), synthetic_seed=0, max_batch=B,
        max_ctx=L + total + 8, tp_group=tp_group)
    model.set_ddpm_inference_steps(S)
    tk = tokenizer_ids()
    forced = [[tk.speech_diffusion_id] * total for _ in range(B)]
    torch.manual_seed(1234)
    torch.cuda.synchronize()
    t_pf = time.perf_counter()
    sess = model.generate_session(**inp, tokenizer=tk, cfg_scale=1.3, generation_config={"do_sample": False},
                                  forced_tokens=forced, max_length_times=total / L + 1, max_new_tokens=total + 2)
    torch.cuda.synchronize()
    prefill_ms = (time.perf_counter() - t_pf) * 1e3
    for _ in range(W):
        assert sess.step()
    ctx0 = int(sess.pos_len.float().mean())

    barrier(world)
    t0 = time.perf_counter()
    for _ in range(K):
        assert sess.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    barrier(world)
    dt = max_over_ranks(dt, world, dev)
    ctx1 = int(sess.pos_len.float().mean())
    tps, audio_per_s = throughput(dt, B, K, replicas)
    wb = weight_bytes(model.engine.w, B, S)
    ctx_avg = (ctx0 + ctx1) / 2
    bpt = bytes_per_token(wb, model.config, B, S, ctx_avg, (ctx0 + ctx1) / 2 - L)
    # `roofline` = whichever of the two candidates (the LM MLP block, the head FFN
    # layer) takes more time per step (avg x launches per step), i.e. the top row
    # of the step profile (profiles/r06_steps_b1.txt); the other is `roofline_2`
    try:   # the LM MLP block in one launch (B = 1), else the LM gate|up GEMV
        roof_lm = measure_lm_ffn(model, B)
    except Exception as e:   # noqa: BLE001
        print(f"bench: LM MLP block roofline not measured: {e}", file=sys.stderr, flush=True)
        roof_lm = None
    roof_lm = roof_lm or measure_gemv(model, B)
    roof_head = None
    if world == 1 or T == 1:
        try:
            roof_head = measure_head_layers(model, B)
        except Exception as e:   # noqa: BLE001
            print(f"bench: head roofline not measured: {e}", file=sys.stderr, flush=True)
            roof_head = {"error": str(e)[:200]}
    roof_attn = None
    try:
        roof_attn = measure_lm_attn(model, B, ctx_avg)
    except Exception as e:   # noqa: BLE001
        print(f"bench: LM attention half roofline not measured: {e}", file=sys.stderr, flush=True)
    for r in (roof_lm, roof_head, roof_attn):
        if r and "error" not in r:
            in_loop_average(r, B)
    roofline, roofline_2 = pick_roofline(roof_lm, roof_head, roof_attn)
    tp_coll = None
    if T > 1:   # after the timed loop: the null-collective passes corrupt the session's state
        tp_coll = measure_tp_collective(lm_pass_maker(model, sess), model.config.decoder_config.num_hidden_layers,
                                        world, dev)
        if model.tp_head:   # the sharded diffusion head's S x head_layers all-reduces per token
            hl = model.config.diffusion_head_config.head_layers
            hc = measure_tp_collective(head_pass_maker(model, sess), hl * S / 2, world, dev)
            tp_coll["head"] = dict(diffusion_call_us=hc["lm_pass_us"],
                                   diffusion_call_us_null_collective=hc["lm_pass_us_null_collective"],
                                   allreduce_us_per_call=hc["allreduce_us_per_pass"],
                                   allreduce_calls_per_call=int(hl * S), allreduce_share=hc["allreduce_share"],
                                   note="RCCL all-reduce of the [2B, H] head state after each head layer's "
                                        "row-parallel down_proj (sharded head, tp_head)")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:   # bounded CPU sample, N=1 only
        cpu = cpu_baseline(model.config, args.cpu_tokens, S, args.model)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(audio_per_s, 3),
            "unit": "audio-sec/wall-sec",
            "acoustic_tokens_per_sec": round(tps, 2),
            "rtf_wall_per_audio": round(1.0 / audio_per_s, 5),
            "n_gpus": world, "steps": K, "warmup": W,
            "ms_per_step": round(dt / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic: seeded random-init VibeVoice weights at real shapes, seeded -25 dBFS noise voice "
                    "prompt (3 s/speaker), random script ids in the processor's prompt layout, forced "
                    "speech_diffusion schedule (constrained argmax still computed and read back each step)",
            "config": {"workload": f"VibeVoice-{args.model} bf16, {B} dialogue(s)/replica x {args.speakers} "
                                   f"speaker(s), {S} diffusion steps, TP={T}, prompt {L} tokens"
                                   + (f", long-form context: a {L}-token script prefilled through the product "
                                      f"path ({prefill_ms:.0f} ms incl. the voice encoder), decode timed from there"
                                      if args.context else ""),
                       "model": f"VibeVoice-{args.model}", "global_batch": B * replicas, "seq_len": L,
                       "diffusion_steps": S, "parallelism": f"dp{replicas} (independent replicas), tp{T}",
                       "context_start": ctx0, "context_end": ctx1},
            "roofline": roofline,
            "roofline_2": roofline_2,
            "step_roofline": dict(roof("whole loop iteration", f"B={B} S={S}", bpt * B, dt / K),
                                  alg_bytes_per_token=int(bpt), head_layout=wb["head_layout"],
                                  note="SURVEY.md §8d bytes, each weight role counted once in the layout the loop "
                                       "reads (bench.py weight_bytes); avg_us = ms_per_step"),
            "cpu_baseline": cpu,
        }
        if tp_coll is not None:
            line["tp_collective"] = tp_coll
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def plumbing(args, world, rank, dev):
    """--plumbing: the multi-rank harness of main() (groups, barrier + sync on
    both sides, max over ranks, whole-job value, one JSON line on rank 0)
    around an empty step of known length (rank r sleeps 1 ms x (r + 1))."""
    _, _, replicas = tp_groups(world, rank, args.tp)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(1e-3 * (rank + 1))
    barrier(world)
    dt = max_over_ranks(time.perf_counter() - t0, world, dev)
    tps, audio_per_s = throughput(dt, args.batch, args.steps, replicas)
    tp_coll = None
    if args.tp > 1:   # the field's plumbing: a "pass" of 1 ms, 0.25 ms of it the collective
        tp_coll = measure_tp_collective(lambda null: (lambda: time.sleep(0.75e-3 if null else 1e-3)), 2, world,
                                        dev, iters=10)
    if rank == 0:
        line = {"metric": METRIC, "value": round(audio_per_s, 3), "unit": "audio-sec/wall-sec",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(dt / args.steps * 1e3, 4), "scaling": "weak",
                "data": "plumbing (empty step)", "config": {"parallelism": f"dp{replicas}, tp{args.tp}"},
                "backend": torch.distributed.get_backend() if world > 1 else None}
        if tp_coll is not None:
            line["tp_collective"] = tp_coll
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
