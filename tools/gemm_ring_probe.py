"""k_gemm vs k_gemm_ring (ggnn_dbg_gemm_ex) on the general path's product
shapes: M N K a_layout b_layout per line; prints ms and algorithmic TFLOP/s."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from ggnn_amd import _lib  # noqa: E402

SHAPES = [  # (M, N, K, a_layout, b_layout)
    (4096, 4096, 4096, 0, 0),
    (32768, 800, 400, 0, 0),    # gates at hidden 400, b*v = 32768
    (32768, 400, 400, 0, 1),    # dzc Wc^T
    (400, 800, 32768, 1, 0),    # weight gradient (split-K shape without the split)
    (128, 400, 400, 0, 0),      # one (graph, channel) message transform
    (32768, 256, 512, 0, 0),
    (32768, 152, 512, 0, 0),    # a head's logits (o padded to 152)
]


def run(M, N, K, al, bl, prec, kernel, reps=10):
    dev = torch.device("cuda", 0)
    a = torch.randn(M * K, device=dev)
    b = torch.randn(K * N, device=dev)
    d = torch.empty(M, N, device=dev)
    dims = _lib.dims(1, 1, 64, 1, 1, True, prec)
    lib = _lib.load()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (ctypes.byref(dims), M, N, K, ctypes.c_void_p(a.data_ptr()), al, ctypes.c_void_p(b.data_ptr()), bl,
            ctypes.c_void_p(d.data_ptr()), kernel, s)
    _lib.check(lib.ggnn_dbg_gemm_ex(*args), "gemm_ex")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        lib.ggnn_dbg_gemm_ex(*args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return ms, 2.0 * M * N * K / ms / 1e9


if __name__ == "__main__":
    if len(sys.argv) > 1:  # one shape: M N K a_layout b_layout prec kernel [reps]
        M, N, K, al, bl = (int(x) for x in sys.argv[1:6])
        ms, tf = run(M, N, K, al, bl, sys.argv[6], int(sys.argv[7]), int(sys.argv[8]) if len(sys.argv) > 8 else 10)
        print("M=%d N=%d K=%d: %.4f ms %.1f TF" % (M, N, K, ms, tf))
        sys.exit(0)
    for prec in ("fp32", "bf16"):
        for M, N, K, al, bl in SHAPES:
            r = [run(M, N, K, al, bl, prec, k) for k in (1, 2)]
            print("%s M=%d N=%d K=%d layout=%d%d: k_gemm %.4f ms %.1f TF | ring %.4f ms %.1f TF | x%.2f" % (
                prec, M, N, K, al, bl, r[0][0], r[0][1], r[1][0], r[1][1], r[0][0] / r[1][0]), flush=True)
