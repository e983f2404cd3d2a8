"""CPU-side checks of the C ABI library: it builds, loads and exports every
entry point declared in include/vibevoice_hip.h (the product interface) and
include/vibevoice_hip_diag.h (kernel entry points, tuning hooks, stamps), and
the product header declares none of the diagnostics (no GPU compute here)."""
import ctypes
import os
import re

from vibevoice_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(headers=("vibevoice_hip.h", "vibevoice_hip_diag.h")):
    names = set()
    for h in headers:
        src = open(os.path.join(ROOT, "include", h)).read()
        names |= set(re.findall(r"^\s*(?:const char\*|int|void)\s+(vv_\w+)\(", src, re.M))
    return sorted(names)


def test_header_declares_entry_points():
    names = declared_symbols()
    assert "vv_lm_forward" in names and "vv_diffusion_sample" in names and "vv_codec_step" in names
    assert set(names) == {n for n, _, _ in _lib.EXPORTS}


def test_product_header_has_no_diagnostics():
    """Tuning hooks, stamps, kernel entry points and benchmark-only switches
    (process-wide state) live in the diag header only."""
    product = set(declared_symbols(("vibevoice_hip.h",)))
    diag = set(declared_symbols(("vibevoice_hip_diag.h",)))
    assert not product & diag
    for n in product:
        assert not re.search(r"tune|stamps|null_collective|synthetic|_bf16$|plan|chain|pack|rope_table|defer|"
                             r"mix_fusion|attn_prefill", n), n
    assert {"vv_tp_null_collective", "vv_kv_synthetic", "vv_gemv_tune", "vv_gemm_bf16"} <= diag
    # nothing in the product package calls a diagnostic entry point
    pkg = os.path.join(ROOT, "vibevoice_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py") and f != "_lib.py":
            src = open(os.path.join(pkg, f)).read()
            for n in diag:
                assert n + "(" not in src, (f, n)


def test_library_loads_and_exports_all_symbols():
    L = _lib.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name


def test_config_struct_matches_header():
    # vv_config: 6 ints, 2 floats, 3 ints, 1 float, 1 int, 3 x int[8], 4 ints, 1 float, 2 ints
    assert ctypes.sizeof(_lib.VVConfig) == 4 * (6 + 2 + 3 + 1 + 1 + 24 + 4 + 1 + 2)


def test_create_rejects_bad_config():
    L = _lib.lib()
    c = _lib.VVConfig()
    c.head_dim = 64
    h = ctypes.c_void_p()
    assert L.vv_create(ctypes.byref(c), 0, ctypes.byref(h)) != 0
    assert b"head_dim" in L.vv_last_error()


def _plan(M, N, K, xf=0, w=False, mod=False):
    out = (ctypes.c_int * 7)()
    assert _lib.lib().vv_gemv_plan(M, N, K, xf, int(w), int(mod), out) == 0
    return dict(zip(("kernel", "waves", "ksplit", "u", "tpw", "rw", "lds"), list(out)))


def test_gemv_plan_rules():
    """The decode-GEMV launch plans DESIGN.md §3 documents (host logic only)."""
    NORM = 1
    # B = 1 (M = 2): LM gate|up, 2-wave one-tile workgroups, row-per-wave norm
    p = _plan(2, 17920, 1536, NORM, w=True)
    assert (p["kernel"], p["waves"], p["ksplit"], p["u"], p["tpw"], p["rw"]) == (0, 2, 1, 4, 1, 1)
    # B = 8 (M = 16): 8 tiles per 8-wave workgroup, two rows per wave
    p = _plan(16, 17920, 1536, NORM, w=True)
    assert (p["waves"], p["tpw"], p["rw"]) == (8, 8, 1)
    # B = 8 LM down: K split until the A slice fits 64 KB of LDS (5 ways), staged once
    p = _plan(16, 1536, 8960)
    assert (p["kernel"], p["ksplit"], p["waves"]) == (0, 5, 8) and p["lds"] <= 65536
    # codec fc1 at C = 2,048 (512 tiles), B = 8: two tiles per workgroup (256 workgroups)
    p = _plan(8, 8192, 2048)
    assert (p["kernel"], p["tpw"], p["waves"]) == (0, 2, 8)
    # codec fc2 at C = 2,048 keeps its 2-way split on k_gemv (the split-to-fit rule cost 20 us there)
    p = _plan(16, 2048, 8192)
    assert (p["kernel"], p["ksplit"], p["waves"]) == (1, 2, 8)
    # VibeVoice-Large LM down at M = 2: split until the 76 KB of A rows fit
    p = _plan(2, 3584, 18944)
    assert (p["kernel"], p["ksplit"], p["waves"]) == (0, 2, 8)
    # Large head layers (K 3,584, norm weight + adaLN): the LDS-DMA row form; no adaLN: registers
    assert _plan(2, 21504, 3584, NORM, w=True, mod=True)["rw"] == 2
    assert _plan(2, 37888, 3584, NORM, w=True)["rw"] == 1
    # the RW form is an XF_NORM-only, unsplit-K form
    assert _plan(2, 1536, 8960)["rw"] == 0
    assert _plan(16, 64, 1536, NORM, mod=True)["ksplit"] == 8 and _plan(16, 64, 1536, NORM, mod=True)["rw"] == 0
    # the diagnostic switch turns it off and back on
    L = _lib.lib()
    L.vv_gemv_tune_rw(99)
    try:
        assert _plan(2, 17920, 1536, NORM, w=True)["rw"] == 0
    finally:
        L.vv_gemv_tune_rw(0)
    assert _plan(2, 17920, 1536, NORM, w=True)["rw"] == 1


def _attn(ntok, max_pos_p1, lm_slots=2):
    out = (ctypes.c_int * 6)()
    assert _lib.lib().vv_attn_pass_plan(ntok, lm_slots, 128, 2, max_pos_p1, out) == 0
    return dict(zip(("prefill", "nsplit", "chunk", "defer", "group", "ngroups"), list(out)))


def test_attention_pass_plan_rules():
    """The decode attention plans DESIGN.md §3 documents (host logic only)."""
    L = _lib.lib()
    # B = 1 short context: 2..8 deferred splits of >= 128 keys, merged by o_proj
    p = _attn(2, 900)
    assert (p["prefill"], p["defer"], p["nsplit"], p["chunk"], p["group"]) == (0, 1, 8, 128, 0)
    # B = 8 (16 rows) does not defer: one 1,024-key split per (row, kv head) at this length
    p = _attn(16, 900, lm_slots=16)
    assert (p["defer"], p["nsplit"], p["group"]) == (0, 1, 0)
    # 64K: at most 120 splits of >= 256 keys in <= 8 groups of <= 16 (one CU per keyed workgroup)
    p = _attn(2, 65040)
    assert (p["nsplit"], p["chunk"], p["group"], p["ngroups"]) == (120, 544, 15, 8)
    p = _attn(2, 20000)
    assert (p["nsplit"], p["chunk"], p["group"], p["ngroups"]) == (79, 256, 10, 8)
    # the switch: 0 = 1,024-key splits merged by k_attn_merge; n = at most n splits
    L.vv_attn_group(0)
    try:
        p = _attn(2, 65040)
        assert (p["nsplit"], p["chunk"], p["group"]) == (64, 1024, 0)
        L.vv_attn_group(128)
        assert _attn(2, 65040)["nsplit"] == 128
    finally:
        L.vv_attn_group(1)
    assert _attn(2, 65040)["nsplit"] == 120
    # the kernels' limits, over every context the group plan takes: k_attn's group
    # merge holds <= 16 split partials, o_proj's XF_ATTN_MERGE <= 8 group partials
    for max_len in range(8193, 65537, 997):
        p = _attn(2, max_len)
        if p["group"]:
            assert p["group"] <= 16 and p["ngroups"] <= 8 and p["nsplit"] <= 128
            assert p["ngroups"] * p["group"] * p["chunk"] >= max_len
    # grouped merge, ragged rows in one pass (the plan is sized by the longest row):
    # the producer's active groups for a row of n keys, ceil(ceil(n / chunk) / group),
    # equal the consumer's ceil(n / (group * chunk)) and never exceed ngroups
    for max_len in (8193, 20000, 32768, 65040, 65536):
        p = _attn(2, max_len)
        ch, gs, ng = p["chunk"], p["group"], p["ngroups"]
        assert gs > 0 and ng * gs * ch >= max_len
        for n in (1, 200, ch - 1, ch, ch + 1, gs * ch, gs * ch + 1, max_len // 3, max_len - 1, max_len):
            prod = -(-(-(-n // ch)) // gs)
            cons = min(-(-n // (gs * ch)), ng)
            assert prod == cons <= ng, (max_len, n, prod, cons)
    # a prompt: the prefill kernel (>= 256 rows and >= 32 rows per slot), no splits
    p = _attn(512, 512)
    assert (p["prefill"], p["nsplit"]) == (1, 1)


def test_persist_decision_rule():
    """The rule every grid-waiting launch applies before it is issued (VERDICT
    r5 item 8; host logic only): the whole one-per-CU grid resident by the
    occupancy query, no scratch, the kernels enabled for the context, and the
    context the device's only registered one -- else the GEMV launches run."""
    d = _lib.lib().vv_persist_decision
    assert d(1, 256, 0, 256, 1, 1) == 1
    assert d(2, 256, 0, 256, 1, 1) == 1          # more room than needed
    assert d(1, 240, 0, 256, 1, 1) == 0          # fewer CUs (e.g. a CU mask) than workgroups
    assert d(0, 256, 0, 256, 1, 1) == 0          # the build does not fit a CU
    assert d(1, 256, 64, 256, 1, 1) == 0         # scratch: waves may wait for slots
    assert d(1, 256, 0, 256, 2, 1) == 0          # a second registered context on the device
    assert d(1, 256, 0, 256, 1, 0) == 0          # switched off (VIBEVOICE_PERSISTENT=0 / vv_set_persistent)
