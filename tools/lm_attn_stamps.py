"""Where the LM attention half's time goes (k_lm_attn, lm_attn.hip): graph-replayed
decode passes of the 1.5B LM (28 layers) at 2 B rows over ~`ctx` cached keys,
the one-launch attention half against the three launches (q|k|v, k_attn, o_proj),
then per-workgroup s_memrealtime stamps (10 ns ticks) of the last k_lm_attn
launch: 0 start, 1 A side / weights issued, 2 q|k|v stored, 3 wait 1 released,
4 attention units done, 5 wait 2 released, 6 merge done, 7 wait 3 released,
8 o_proj stored.  Prints the median per phase since each workgroup's start.
usage: python tools/lm_attn_stamps.py [B] [ctx] [vv_lm_attn modes, e.g. 1,3,5,7]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vibevoice_amd import _lib  # noqa: E402
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 900
    L = _lib.lib()
    model = VibeVoiceForConditionalGenerationInference.from_pretrained("synthetic:1.5B", device_map="cuda",
                                                                        synthetic_seed=0, max_batch=B,
                                                                        max_ctx=ctx + 64)
    eng = model.engine
    if not hasattr(eng, "n_valid"):
        eng.set_valid_ids([151643, 151652, 151653, 151654])
    R = 2 * B
    I32 = dict(dtype=torch.int32, device="cuda")
    slots = torch.arange(R, **I32)
    _lib.check(L.vv_kv_synthetic(eng.h, R, ctypes.c_void_p(slots.data_ptr()), 0, ctx + 8, 7,
                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "kv_synthetic")
    pos = torch.tensor([ctx - 97 * (r % 2) - 3 * r for r in range(R)], **I32)   # positive / shorter negative rows
    mp = int(pos.max()) + 1
    print(f"B={B}: rows {R}, keys {int(pos.min()) + 1}..{mp}; one launch active: {L.vv_lm_attn_active(eng.h, R, mp)}")
    x = (torch.randn(R, 1536, device="cuda") * 0.5).bfloat16()
    idx = torch.arange(R, **I32)
    h = torch.empty(R, 1536, device="cuda", dtype=torch.bfloat16)
    lg = torch.empty(R, eng.n_valid, device="cuda", dtype=torch.float32)
    s = torch.cuda.Stream()

    def timed(on):
        L.vv_lm_attn(on)
        with torch.cuda.stream(s):
            eng.lm_forward(x, slots, pos, idx, hidden_out=h, logits_out=lg, max_pos=mp - 1, stream=s)
            g = torch.cuda.CUDAGraph()
            g.capture_begin(capture_error_mode="thread_local")
            eng.lm_forward(x, slots, pos, idx, hidden_out=h, logits_out=lg, max_pos=mp - 1, stream=s)
            g.capture_end()
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                g.replay()
            e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / 20
    t3, t1 = timed(0), timed(1)
    print(f"LM pass: three launches {t3:.1f} us, one launch {t1:.1f} us -> {(t3 - t1) / 28:.2f} us per layer saved")
    modes = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else []
    for mode in modes:   # vv_lm_attn values (bits 1..: LmAttnArgs::variant); stamps taken with the last
        print(f"LM pass, vv_lm_attn({mode}): {timed(mode):.1f} us", flush=True)
    st = torch.zeros(256 * 16, dtype=torch.int64, device="cuda")
    L.vv_lm_attn_stamps(st.data_ptr())
    with torch.cuda.stream(s):
        eng.lm_forward(x, slots, pos, idx, hidden_out=h, logits_out=lg, max_pos=mp - 1, stream=s)
    torch.cuda.synchronize()
    L.vv_lm_attn_stamps(None)
    eng.check_sync()
    t = st.view(256, 16).cpu().double() * 10e-3
    t0 = t[:, 0].min()
    for name, rows in (("q|k|v", t[:128]), ("o_proj", t[128:224]), ("rest", t[224:])):
        used = [k for k in range(9) if bool((rows[:, k] != 0).all())]
        med = (rows[:, used] - t0).median(0).values
        mx = (rows[:, used] - t0).max(0).values
        print(f"{name}: " + ", ".join(f"{k}:{float(m):.2f}/{float(x_):.2f}" for k, m, x_ in zip(used, med, mx)))
    print(f"launch span {float(t[128:224, 8].max() - t0):.2f} us (median / max since the launch's first start)")


if __name__ == "__main__":
    main()
