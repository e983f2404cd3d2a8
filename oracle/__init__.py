"""CPU ORACLE — test infrastructure only.

A plain-PyTorch (CPU, eager) restatement of the reference's generate-loop
arithmetic (lzhgus/VibeVoice, `vibevoice/modular/*`, `vibevoice/schedule/
dpm_solver.py`).  Every function cites the reference file:line it follows.

Rules:
  * Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline`
    leg may import this package, and only as the CHECKER / CPU baseline.
    The product (`vibevoice_amd/`) never imports it and has no CPU fallback.
  * The oracle is pinned against golden vectors produced by running the
    reference's own modules (tests/golden/make_golden.py, fixtures in
    tests/golden/*.npz).  The Qwen2 arithmetic is pinned at transformers
    5.15.0 (the reference pins 4.51.3, absent offline): decode math is the
    same in both, but 4.51.3 bit-level parity is "parity unpinned at the
    version level" (SURVEY.md §8c).
  * Tensors may be float32 or bfloat16.  Run with bf16 weights and bf16
    activations it reproduces the reference's GPU rounding points (every
    torch op rounds its result to the tensor dtype); with float32 it is the
    "reference CPU eager path" (demo/inference_from_file.py:268 loads fp32
    on CPU).
"""
