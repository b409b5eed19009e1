"""Throughput of the general path's product kernel (ggnn_dbg_gemm) on square
problems; run under rocprofv3 (--kernel-trace --stats, or --pmc passes)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from ggnn_amd import _lib  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda", 0)
    a = torch.randn(n, n, device=dev)
    b = torch.randn(n, n, device=dev)
    d = torch.empty(n, n, device=dev)
    dims = _lib.dims(1, 1, 64, 1, 1, True, prec)
    lib = _lib.load()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (ctypes.byref(dims), n, n, n, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
            ctypes.c_void_p(d.data_ptr()), s)
    _lib.check(lib.ggnn_dbg_gemm(*args), "gemm")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        lib.ggnn_dbg_gemm(*args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    f = 2.0 * n ** 3
    issued = f * (3 if prec == "fp32" else 1)
    print("n=%d %s: %.3f ms, %.1f TFLOP/s algorithmic, %.1f issued" % (n, prec, ms, f / ms / 1e9, issued / ms / 1e9))
