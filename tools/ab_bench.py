"""A/B a library switch on one box: python tools/ab_bench.py <switch> <value> [bench args]
(switch: codec_mix_fusion; or "lib" <path> to load another build of the
library, e.g. an older commit's build kept under tools/lib_*.so).  Runs
bench.py's main with it set first."""
import os
import sys

import torch  # noqa: F401  (torch first: the library binds to its HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vibevoice_amd import _lib  # noqa: E402

name, val = sys.argv[1], sys.argv[2]
if name == "lib":
    import ctypes
    _lib.LIB_PATH = os.path.abspath(val)
    probe = ctypes.CDLL(_lib.LIB_PATH)     # an older build may lack newer (diagnostic) exports
    _lib.EXPORTS = [e for e in _lib.EXPORTS if hasattr(probe, e[0])]
    _lib.lib()
else:   # e.g. attn_tune 128,8; gemv_tune_shape 2048,8192,1,8,2,4,1 (several: separated by ';')
    for v in val.split(";"):
        getattr(_lib.lib(), "vv_" + name)(*[int(x) for x in v.split(",")])
if len(sys.argv) > 3 and sys.argv[3] == "--prefill":   # tools/prefill_bench.py instead of bench.py
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.argv = ["prefill_bench.py"] + sys.argv[4:]
    import prefill_bench  # noqa: E402
    prefill_bench.main()
    sys.exit(0)
sys.argv = ["bench.py"] + sys.argv[3:]
import bench  # noqa: E402

bench.main()
