"""The real-density side line of bench.py (b=256 dependency trees, v=30,
hidden 256, C=92, T=5, fwd+bwd) alone, for rocprofv3 --kernel-trace --stats."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.real_density_side(torch.device("cuda", 0))))
