"""Kernel-boundary floor on the MI355X: graph-replayed back-to-back launches."""
import ctypes
import os
import subprocess
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "libfloor.so")
if not os.path.exists(so):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                    os.path.join(HERE, "floor.hip"), "-o", so], check=True)
L = ctypes.CDLL(so)
x = torch.randn(1 << 22, device="cuda")
y = torch.empty_like(x)
for kind, blocks, threads, n in [(0, 1, 64, 0), (0, 256, 256, 0), (0, 1024, 256, 0), (1, 256, 256, 0),
                                 (2, 1, 64, 64), (2, 256, 256, 65536), (2, 4096, 256, 1 << 20),
                                 (2, 16384, 256, 1 << 22)]:
    def run():
        L.fl_launch(kind, blocks, threads, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), n,
                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    run()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(200):
            run()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    e1.synchronize()
    print(f"kind {kind} blocks {blocks:6d} threads {threads}: {e0.elapsed_time(e1) * 1e3 / 1000:.2f} us per launch")
