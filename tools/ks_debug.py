"""Element-mapping probe of k_gemm_ks (ggnn_dbg_gemm_ex kernel 3): one-hot A
or B operands make every output a single operand element, so a wrong LDS
mapping or a stale limb shows as the exact (m, n) it hits.  Found the missing
VALU -> MFMA wait states after the inline-asm limb split (ggnn_common.h pk_lo)."""
import sys, os, ctypes
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from ggnn_amd import _lib
dev = torch.device("cuda", 0)
def run(A, B, bl, kern, M, N, K):
    a = torch.from_numpy(np.ascontiguousarray(A)).to(dev); b = torch.from_numpy(np.ascontiguousarray(B)).to(dev)
    d = torch.full((M, N), float("nan"), device=dev)
    dims = _lib.dims(1, 1, 64, 1, 1, True, "fp32")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.load().ggnn_dbg_gemm_ex(ctypes.byref(dims), M, N, K, ctypes.c_void_p(a.data_ptr()), 0,
               ctypes.c_void_p(b.data_ptr()), bl, ctypes.c_void_p(d.data_ptr()), kern, s), "x")
    return d.cpu().numpy()
M, N, K = 64, 64, 32
A = np.zeros((M, K), np.float32)
for m in range(M): A[m, m % 32] = 1
B = (np.arange(K)[:, None] * 1000 + np.arange(N)[None, :]).astype(np.float32)  # value = k*1000 + n
for bl in (0, 1):
    Bop = B if bl == 0 else B.T
    D = run(A, Bop, bl, 3, M, N, K)
    bad = 0
    for m in range(M):
        for n in range(N):
            want = (m % 32) * 1000 + n
            if D[m, n] != want:
                if bad < 20: print("bl", bl, "m", m, "n", n, "got", D[m, n], "want", want)
                bad += 1
    print("bl", bl, "bad", bad)
# B = identity-ish: D = A[:, n % 32]
A2 = (np.arange(M)[:, None] * 1000 + np.arange(K)[None, :]).astype(np.float32)
B2 = np.zeros((K, N), np.float32)
for n in range(N): B2[n % 32, n] = 1
for bl in (0, 1):
    Bop = B2 if bl == 0 else B2.T
    D = run(A2, Bop, bl, 3, M, N, K)
    bad = 0
    for m in range(M):
        for n in range(N):
            want = m * 1000 + n % 32
            if D[m, n] != want:
                if bad < 20: print("A-test bl", bl, "m", m, "n", n, "got", D[m, n], "want", want)
                bad += 1
    print("A-test bl", bl, "bad", bad)
