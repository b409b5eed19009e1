"""One general-path shape under the profiler: b v h C T [trees]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from generic_probe import run  # noqa: E402

if __name__ == "__main__":
    b, v, h, C, T = (int(x) for x in sys.argv[1:6])
    print(json.dumps(run(b, v, h, C, T, False, trees=len(sys.argv) > 6 and sys.argv[6] == "trees")))
