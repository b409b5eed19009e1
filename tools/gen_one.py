"""One general-path shape under the profiler: b v h C T [trees] [generic]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from generic_probe import run  # noqa: E402

if __name__ == "__main__":
    b, v, h, C, T = (int(x) for x in sys.argv[1:6])
    flags = sys.argv[6:]
    print(json.dumps(run(b, v, h, C, T, "generic" in flags, trees="trees" in flags, steps=10)))
