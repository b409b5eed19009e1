"""Throughput of the general path's product kernel (ggnn_dbg_gemm): M N K
[precision] [reps]; GGNN_GEMM_TILE = 11 | 21 | 22 forces a block-tile variant.
Run under rocprofv3 for per-kernel times / counters."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from ggnn_amd import _lib  # noqa: E402


def run(M, N, K, prec="fp32", reps=10):
    dev = torch.device("cuda", 0)
    a = torch.randn(M, K, device=dev)
    b = torch.randn(K, N, device=dev)
    d = torch.empty(M, N, device=dev)
    dims = _lib.dims(1, 1, 64, 1, 1, True, prec)
    lib = _lib.load()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (ctypes.byref(dims), M, N, K, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
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
    f = 2.0 * M * N * K
    return ms, f / ms / 1e9


if __name__ == "__main__":
    shapes = [(4096, 4096, 4096), (32768, 150, 512), (32768, 512, 150), (32768, 512, 256), (128, 256, 256)]
    for M, N, K in shapes:
        ms, tf = run(M, N, K)
        print("tile=%s M=%d N=%d K=%d: %.4f ms, %.1f TFLOP/s algorithmic (fp32 split)" % (
            os.environ.get("GGNN_GEMM_TILE", "auto"), M, N, K, ms, tf))
