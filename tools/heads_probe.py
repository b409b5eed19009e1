"""Kernel-level probe of the btb callers (embedding front-end + output heads)
at the bench's b=256, v=128, h=256: run under rocprofv3 --kernel-trace --stats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    print(bench.callers_side(dev, 256, 128, 256, reps=int(sys.argv[1]) if len(sys.argv) > 1 else 10))
