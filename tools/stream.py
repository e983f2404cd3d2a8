"""Calibrate a pure HBM read stream on MI355X: GB/s vs workgroups, waves, loads in flight."""
import ctypes
import os
import subprocess
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "libfloor.so")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                os.path.join(HERE, "floor.hip"), "-o", so], check=True)
L = ctypes.CDLL(so)
L.fl_stream.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p]
out = torch.zeros(4, dtype=torch.int32, device="cuda")
for MB in (27.5, 55):
    nbytes = int(MB * 1e6) // (1 << 16) * (1 << 16)
    bufs = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(max(2, 600 // int(MB)))]
    for b in bufs:
        b.random_(0, 255)
    for G in (96, 192, 256, 512, 1024, 2048):
        for W in (1, 2, 4, 8):
            for U in (4, 8, 16):
                if nbytes // (G * W) < 1024 * U:
                    continue
                def run(i):
                    L.fl_stream(G, W, U, ctypes.c_void_p(bufs[i % len(bufs)].data_ptr()), nbytes,
                                ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                run(0)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for i in range(len(bufs)):
                        run(i)
                g.replay(); torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); g.replay(); e1.record(); e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / len(bufs)
                print(f"{MB:5.1f} MB G={G:5d} W={W} U={U:2d}: {us:7.2f} us {nbytes / us / 1e3:7.0f} GB/s", flush=True)
    del bufs
    torch.cuda.empty_cache()
