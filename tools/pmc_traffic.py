"""HBM traffic of bench.py's roofline kernel (the LM gate|up GEMV, k_gemv1<4, 1, false, tpw, 1>,
M=2 N=17920 K=1536 at 1.5B, B=1) from rocprofv3 PMC counters, collected the way
MI355X_MICROARCH.md "HBM" / "rocprofv3 PMC slots" prescribe: FETCH_SIZE and
WRITE_SIZE in separate passes (they do not fit one TCC pass), FETCH_SIZE
doubled on gfx950 (it tallies 128-B streaming requests at 64 B), per dispatch.

usage (GPU box):
  python tools/pmc_traffic.py run [M]         # the workload alone (what rocprofv3 wraps)
  python tools/pmc_traffic.py collect [M]     # both rocprofv3 passes + summary ->
                                              # profiles/r05_pmc_traffic_m<M>.json
  python tools/pmc_traffic.py collect-head [R]  # the same for the diffusion head's FFN layer kernel
                                              # (k_head_m16 at R = 2n rows)
                                              # -> profiles/r06_pmc_head_r<R>.json
  python tools/pmc_traffic.py collect-lmffn 2  # the LM MLP block in one launch (k_lm_ffn, B = 1;
                                              # 16: k_lm_ffn16, B = 8) -> profiles/r06_pmc_lm_ffn_r<M>.json
M = 2 (B = 1, one tile per workgroup) or 16 (B = 8: the balanced form, 4-5 tiles per workgroup).
"""
import csv
import ctypes
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
M = int(sys.argv[2]) if len(sys.argv) > 2 else 2
N, K, NL = 17920, 1536, 28
KERNEL = f"k_gemv1<4, 1, false, {5 if M >= 8 else 1}, 1>"  # U, XF_NORM, non-temporal, tiles per workgroup, RW form


def run():
    import torch
    from vibevoice_amd import _lib
    from vibevoice_amd.weights import mfma_pack
    L = _lib.lib()
    torch.manual_seed(0)
    Ws = [mfma_pack((torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()) for _ in range(NL)]
    nws = [(1 + 0.1 * torch.randn(K, device="cuda")).bfloat16() for _ in range(NL)]
    A = torch.randn(M, K, device="cuda").bfloat16()
    Y = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(4):
        for W, nw in zip(Ws, nws):
            _lib.check(L.vv_gemm_bf16_norm(M, N, K, ctypes.c_void_p(A.data_ptr()), K, ctypes.c_void_p(nw.data_ptr()),
                                           1e-6, ctypes.c_void_p(W.data_ptr()), _lib.EPI["silu_mul"],
                                           ctypes.c_void_p(Y.data_ptr()), N // 2, None, sp), "gemv")
    torch.cuda.synchronize()


def run_head():
    """The diffusion head's FFN layers as the loop runs them (k_head_m16 in the
    default GEMV layout, 40 launches per token at S = 10): vv_head_layers_replay
    on the real 1.5B head, a warm-up pass then 24 more layers."""
    import torch
    from vibevoice_amd import _lib
    from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
    n = M // 2
    model = VibeVoiceForConditionalGenerationInference.from_pretrained("synthetic:1.5B", device_map="cuda",
                                                                        synthetic_seed=0, max_batch=n, max_ctx=256)
    model.set_ddpm_inference_steps(10)
    model.engine.set_steps(10)
    cond = torch.randn(2 * n, 1536, device="cuda").bfloat16()
    L = _lib.lib()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for reps in (1, 6):
        _lib.check(L.vv_head_layers_replay(model.engine.h, n, ctypes.c_void_p(cond.data_ptr()),
                                           ctypes.c_void_p(cond[n:].data_ptr()), reps, sp), "head_layers_replay")
    torch.cuda.synchronize()
    model.engine.check_sync()


def run_lm_ffn():
    """The LM MLP blocks as the B = 1 loop runs them (k_lm_ffn, 28 launches per LM
    pass): vv_lm_mlp_replay on the 1.5B LM shapes, a warm-up pass then 3 more."""
    import torch
    from vibevoice_amd import _lib
    from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
    n = M // 2
    model = VibeVoiceForConditionalGenerationInference.from_pretrained("synthetic:1.5B", device_map="cuda",
                                                                        synthetic_seed=0, max_batch=n, max_ctx=256)
    L = _lib.lib()
    assert L.vv_lm_ffn_active(model.engine.h, M) == 1
    x = (torch.randn(M, 1536, device="cuda") * 0.5).bfloat16()
    act = torch.empty(M, 8960, device="cuda", dtype=torch.bfloat16)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for reps in (1, 3):
        _lib.check(L.vv_lm_mlp_replay(model.engine.h, M, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(act.data_ptr()),
                                      reps, sp), "lm_mlp_replay")
    torch.cuda.synchronize()
    model.engine.check_sync()


HEAD = len(sys.argv) > 1 and sys.argv[1].endswith("head")
LMF = len(sys.argv) > 1 and sys.argv[1].endswith("lmffn")
if LMF:   # k_lm_ffn at <= 2 rows, k_lm_ffn16 at 3..16
    KERNEL, NL = ("k_lm_ffn" if M <= 2 else "k_lm_ffn16"), 28
    N, K = 8960, 1536                     # I, H
if HEAD:   # the one-launch layer of head_m16.hip (the default GEMV head layout, 2n <= 16 rows)
    KERNEL, NL = "k_head_m16", 4
    N, K = 4608, 1536                     # F, H


def per_dispatch(path, counter):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if KERNEL + "(" in name:
                if row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return vals


def collect():
    out = os.path.join(ROOT, "gpurun_out", f"pmc_{'head_r' if HEAD else 'lmffn_r' if LMF else 'm'}{M}")
    res = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out, counter.lower())
        cmd = ["rocprofv3", "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__),
               "run-head" if HEAD else "run-lmffn" if LMF else "run",
               str(M)]
        subprocess.run(cmd, check=True, timeout=120)
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        with open(files[0]) as f:
            print(counter, "header:", f.readline().strip()[:300])
        vals = per_dispatch(files[0], counter)
        print(counter, "dispatches", len(vals), "first values", vals[:3])
        vals = vals[NL:]                      # drop the first sweep (cold code / TLB)
        res[counter] = sum(vals) / len(vals)
        res[counter + "_dispatches"] = len(vals)
    # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB
    fetch = res["FETCH_SIZE"] * 1024 * 2       # gfx950: 128-B requests tallied at 64 B
    write = res["WRITE_SIZE"] * 1024
    if HEAD:   # the layer's gate|up + down weights + its rows in / out
        alg, shape = 3 * N * K * 2 + M * K * 2 * 2, f"rows={M} H={K} F={N}"
    elif LMF:  # the block's gate|up + down weights + its rows in / out
        alg, shape = 3 * N * K * 2 + M * K * 2 * 2, f"rows={M} H={K} I={N}"
    else:
        alg, shape = N * K * 2 + M * K * 2 + M * (N // 2) * 2, f"M={M} N={N} K={K}"
    summary = dict(kernel=KERNEL, shape=shape, fetch_size_kib_raw=round(res["FETCH_SIZE"], 1),
                   write_size_kib=round(res["WRITE_SIZE"], 1), dispatches=res["FETCH_SIZE_dispatches"],
                   hbm_read_bytes=int(fetch), hbm_write_bytes=int(write), hbm_bytes_per_launch=int(fetch + write),
                   alg_bytes_per_launch=alg, traffic_over_alg=round((fetch + write) / alg, 4),
                   method="rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, tools/pmc_traffic.py run; "
                          "FETCH_SIZE x 2 (gfx950), KiB -> bytes")
    name = (f"r06_pmc_head_r{M}.json" if HEAD else f"r06_pmc_lm_ffn_r{M}.json" if LMF else
            f"r05_pmc_traffic_m{M}.json")
    for path in (os.path.join(ROOT, "profiles", name), os.path.join(out, "pmc_traffic.json")):
        with open(path, "w") as f:
            json.dump(summary, f, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    {"run": run, "collect": collect, "run-head": run_head, "collect-head": collect, "run-lmffn": run_lm_ffn,
     "collect-lmffn": collect}[sys.argv[1]]()
