"""Where k_lm_ffn16's (B = 8, 16 rows) or k_lm_ffn's (B = 1, 2 rows) time goes: graph-replayed
vv_lm_mlp_replay passes over the 28 layers of the 1.5B LM with per-workgroup
s_memrealtime stamps (10 ns ticks) of the last launch: 0 start, 1 A side in LDS,
2 normalised, 3 gate|up products, 4 SiLU * up, 5 hand-off released, 6 act rows
+ down weights landed, 7 down products, 8 partial published, 9 end.  Prints the
median per phase since each workgroup's start (owners / all) and the launch span.
(k_lm_ffn stamps 0-6 and 9.)
usage: python tools/lm_ffn16_stamps.py [rows: 16 | 2] [vv_lm_ffn modes, e.g. 1,3]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference  # noqa: E402


def main():
    L = _lib.lib()
    model = VibeVoiceForConditionalGenerationInference.from_pretrained("synthetic:1.5B", device_map="cuda",
                                                                        synthetic_seed=0, max_batch=8, max_ctx=256)
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    modes = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1]
    assert L.vv_lm_ffn_active(model.engine.h, M) == 1
    x = (torch.randn(M, 1536, device="cuda") * 0.5).bfloat16()
    act = torch.empty(M, 8960, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.Stream()

    def call(n):
        return L.vv_lm_mlp_replay(model.engine.h, M, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(act.data_ptr()),
                                  n, ctypes.c_void_p(s.cuda_stream))
    with torch.cuda.stream(s):
        _lib.check(call(1), "replay")
    torch.cuda.synchronize()
    for mode in modes:   # stamps taken with the last
        L.vv_lm_ffn(mode)
        times = []
        for n in (1, 3):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                g.capture_begin(capture_error_mode="thread_local")
                call(n)
                g.capture_end()
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(4):
                    g.replay()
                e1.record(s)
            e1.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / 4)
        print(f"M={M} vv_lm_ffn({mode}): {(times[1] - times[0]) / (2 * 28):.2f} us per block "
              f"(graph replays, 28 layers)", flush=True)
    st = torch.zeros(256 * 16, dtype=torch.int64, device="cuda")
    L.vv_lm_ffn_stamps(st.data_ptr())
    with torch.cuda.stream(s):
        _lib.check(call(1), "replay")
    torch.cuda.synchronize()
    L.vv_lm_ffn_stamps(None)
    model.engine.check_sync()
    t = st.view(256, 16).cpu().double() * 10e-3
    own = torch.tensor([((w >> 3) & 3) != 3 for w in range(256)])
    for name, rows in (("owners", t[own]), ("non-owners", t[~own])):
        used = [k for k in range(10) if bool((rows[:, k] != 0).all())]
        rel = rows[:, used] - rows[:, :1]
        med = rel.median(0).values
        print(f"{name}: " + ", ".join(f"{k}:{float(m):.2f}" for k, m in zip(used, med)))
    print(f"launch span {float(t[own][:, 9].max() - t[:, 0].min()):.2f} us, start skew {float(t[:, 0].max() - t[:, 0].min()):.2f}")
    # who holds the hand-off back: SiLU * up done (stamp 4) since the launch's first start
    a4 = t[:, 4] - t[:, 0].min()
    q = torch.quantile(a4, torch.tensor([0.5, 0.9, 0.99, 1.0], dtype=a4.dtype))
    print("stamp 4 since launch: p50 %.2f p90 %.2f p99 %.2f max %.2f" % tuple(float(v) for v in q))
    print("latest 12:", ", ".join(f"wg{int(i)}(xcd{int(i) % 8},{'o' if own[i] else 'n'}):{float(a4[i]):.2f}"
                                   for i in a4.argsort(descending=True)[:12]))
    print("per-XCD max:", ", ".join(f"{x}:{float(a4[x::8].max()):.2f}" for x in range(8)))
    print("stamp 0 since launch, max per XCD:", ", ".join(f"{x}:{float((t[x::8, 0] - t[:, 0].min()).max()):.2f}"
                                                          for x in range(8)))


if __name__ == "__main__":
    main()
