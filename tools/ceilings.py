"""Measured MFMA and HBM ceilings of the box ("confirm on the box
with a hipBLASLt bf16 GEMM ceiling and a copy kernel").

  python tools/ceilings.py [out.json]      (GPU box; ~20 s)

* GEMM: torch.matmul (hipBLASLt / rocBLAS) on 8192^3 bf16 and f16 operands,
  median of 20 timed calls after warm-up -> dense TFLOP/s.
* Copy: device-to-device copy of a 2 GiB fp32 buffer, median of 20 -> GB/s of
  read + write traffic.
These are library ceilings measured with the same clocks bench.py runs at; they
sit below the spec peaks (2.5 PF dense bf16/f16, 8 TB/s) and are reported beside
them in bench.py's roofline (``frac_of_measured``).
"""
import json
import sys

import torch


def _time(fn, n=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2] * 1e-3


def main():
    dev = torch.device("cuda", 0)
    out = {"device": torch.cuda.get_device_name(0)}
    n = 8192
    for name, dt in (("bf16", torch.bfloat16), ("f16", torch.float16)):
        x = torch.randn(n, n, device=dev, dtype=dt)
        y = torch.randn(n, n, device=dev, dtype=dt)
        z = torch.empty(n, n, device=dev, dtype=dt)
        s = _time(lambda: torch.matmul(x, y, out=z))
        out["gemm_%s_tflops" % name] = 2 * n ** 3 / s / 1e12
        del x, y, z
    nbytes = 2 << 30
    src = torch.empty(nbytes // 4, device=dev, dtype=torch.float32).fill_(1.0)
    dst = torch.empty_like(src)
    s = _time(lambda: dst.copy_(src))
    out["copy_gbs"] = 2 * nbytes / s / 1e9
    out["method"] = ("torch.matmul 8192^3 (hipBLASLt/rocBLAS), median of 20; device copy of 2 GiB fp32, "
                     "median of 20, read + write bytes")
    print(json.dumps(out))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
