"""Build tools/libggnn_memset.so: libggnn with the round-2 form of its fill /
copy helpers (hipMemsetAsync / hipMemcpyAsync, i.e. memset and memcpy nodes
under stream capture) for tools/capture_probe.py (DESIGN §6, round 4's
captured-memset question).  The product source is not changed: a copy of
ggnn_amd/csrc in a temporary directory gets the two early returns.

    python tools/build_memset_probe_lib.py
    GGNN_LIB=tools/libggnn_memset.so python tools/capture_probe.py
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from ggnn_amd.build import hipcc
    out = os.path.join(ROOT, "tools", "libggnn_memset.so")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "ggnn_amd", "csrc")
        shutil.copytree(os.path.join(ROOT, "ggnn_amd", "csrc"), src)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
        api = os.path.join(src, "ggnn_api.hip")
        s = open(api).read()
        a = "void fill_async(void* p, unsigned char byte, size_t nbytes, hipStream_t s) {\n  if (!nbytes) return;\n"
        b = "void copy_async(float* dst, const float* src, long n, hipStream_t s) {\n  if (n <= 0) return;\n"
        assert a in s and b in s, "fill_async / copy_async changed: update this script"
        s = s.replace(a, a + "  (void)hipMemsetAsync(p, byte, nbytes, s);\n  return;\n")
        s = s.replace(b, b + "  (void)hipMemcpyAsync(dst, src, (size_t)n * 4, hipMemcpyDeviceToDevice, s);\n  return;\n")
        open(api, "w").write(s)
        subprocess.check_call([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                               "-o", out, api])
    print(out)


if __name__ == "__main__":
    main()
