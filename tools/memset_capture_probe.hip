// What does stream capture make of hipMemsetAsync on this ROCm?  (VERDICT r3
// item 7 / ADVICE r3: the pre-6e755f9 library issued hipMemsetAsync calls in
// its captured step -- adjacency tiles to 0, the pair-row index table to 0xFF
// (= -1 sentinels), pair degrees and dW accumulators to 0 -- and replays of
// that graph gave wrong edge-weight gradients and once a garbage pair index
// and a fault.  Kernel-only graphs replay exactly.)
//
// For a set of (value, byte count, byte offset) cases that cover the
// library's calls, this program captures  k_poison -> memset -> k_readback
// on one stream, dumps every node of the graph (type, memset node params,
// dependency edges), replays it, and checks
//   (1) the bytes the memset node wrote (value, extent, guard bytes), and
//   (2) that k_readback saw the memset's bytes, i.e. the edges order it.
// Build: hipcc --offload-arch=gfx950 -O2 tools/memset_capture_probe.hip -o tools/memset_capture_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHK(x)                                                                                  \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::printf("HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, __LINE__, #x); \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

// writes 0x5A into [p, p+n): what the memset must overwrite
__global__ void k_poison(unsigned char* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = 0x5A;
}

// copies [p, p+n) to out: what the consumer of the memset reads
__global__ void k_readback(const unsigned char* p, unsigned char* out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = p[i];
}

// part 2 kernels: X[i] = ctr + 1 (this launch's stamp); count Y[i] != want;
// then advance ctr (one vector atomic, its own node: ordered after k_check)
__global__ void k_stamp(unsigned* X, size_t n, const unsigned* ctr) {
  const unsigned v = *ctr + 1;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) X[i] = v;
}
__global__ void k_check(const unsigned* Y, size_t n, const unsigned* ctr, int copy, unsigned* err) {
  const unsigned want = copy ? *ctr + 1 : 0u;
  unsigned bad = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    bad += Y[i] != want;
  if (bad) atomicAdd(err, bad);
}
__global__ void k_bump(unsigned* ctr) {
  if (threadIdx.x == 0) atomicAdd(ctr, 1u);
}

static const char* type_name(hipGraphNodeType t) {
  switch (t) {
    case hipGraphNodeTypeKernel: return "kernel";
    case hipGraphNodeTypeMemcpy: return "memcpy";
    case hipGraphNodeTypeMemset: return "memset";
    case hipGraphNodeTypeEmpty: return "empty";
    default: return "other";
  }
}

struct Case {
  int value;
  size_t bytes;
  size_t offset;
  const char* what;
};

int main() {
  const size_t guard = 256, cap = (64u << 20) + 2 * guard;
  unsigned char *buf, *out;
  CHK(hipMalloc(&buf, cap));
  CHK(hipMalloc(&out, cap));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<Case> cases = {
      {0xFF, 4 * 1024, 0, "pair-row index table to 0xFF (-1), 1024 ints"},
      {0xFF, 4 * 5000, 0, "pair-row index table to 0xFF (-1), 5000 ints"},
      {0x00, 4 * 5000, 0, "pair degrees to 0"},
      {0x00, 20 * 92, 0, "tile occupancy bytes b*C = 20*92"},
      {0x00, 17 * 92 + 1, 0, "byte count not a multiple of 4"},
      {0x00, 4093, 2, "unaligned base, odd count"},
      {0xFF, 4095, 1, "0xFF, unaligned base, odd count"},
      {0x00, (size_t)92 * 400 * 400 * 4, 0, "dW accumulator C*H*H fp32 (58.9 MB)"},
      {0x00, (size_t)20 * 92 * 120 * 120 * 2, 0, "adjacency tiles b*C*v*vp u16 (52.9 MB)"},
  };
  std::vector<unsigned char> host(cap), host_out(cap);
  int bad_cases = 0;
  for (size_t ci = 0; ci < cases.size(); ++ci) {
    const Case& c = cases[ci];
    unsigned char* p = buf + guard + c.offset;
    // guards and region to 0xAB, eagerly
    CHK(hipMemsetAsync(buf, 0xAB, cap, s));
    CHK(hipMemsetAsync(out, 0x00, cap, s));
    CHK(hipStreamSynchronize(s));
    hipGraph_t g;
    CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(k_poison, dim3(1024), dim3(256), 0, s, p, c.bytes);
    CHK(hipMemsetAsync(p, c.value, c.bytes, s));
    hipLaunchKernelGGL(k_readback, dim3(1024), dim3(256), 0, s, p, out + guard + c.offset, c.bytes);
    CHK(hipStreamEndCapture(s, &g));
    size_t nn = 0;
    CHK(hipGraphGetNodes(g, nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn);
    CHK(hipGraphGetNodes(g, nodes.data(), &nn));
    std::printf("case %zu: value 0x%02X, %zu bytes at +%zu (%s): %zu nodes\n", ci, c.value, c.bytes, c.offset, c.what, nn);
    for (size_t i = 0; i < nn; ++i) {
      hipGraphNodeType t;
      CHK(hipGraphNodeGetType(nodes[i], &t));
      size_t nd = 0;
      CHK(hipGraphNodeGetDependencies(nodes[i], nullptr, &nd));
      std::vector<hipGraphNode_t> deps(nd);
      if (nd) CHK(hipGraphNodeGetDependencies(nodes[i], deps.data(), &nd));
      std::printf("  node %zu %-6s deps [", i, type_name(t));
      for (size_t j = 0; j < nd; ++j)
        for (size_t k = 0; k < nn; ++k)
          if (nodes[k] == deps[j]) std::printf("%s%zu", j ? "," : "", k);
      std::printf("]");
      if (t == hipGraphNodeTypeMemset) {
        hipMemsetParams mp;
        std::memset(&mp, 0, sizeof(mp));
        CHK(hipGraphMemsetNodeGetParams(nodes[i], &mp));
        std::printf("  dst %+lld elementSize %u width %zu height %zu pitch %zu value 0x%08X",
                    (long long)((unsigned char*)mp.dst - p), mp.elementSize, mp.width, mp.height, mp.pitch, mp.value);
      }
      std::printf("\n");
    }
    hipGraphExec_t ge;
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    int bad_fill = 0, bad_guard = 0, bad_read = 0;
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
      CHK(hipGraphLaunch(ge, s));
      CHK(hipStreamSynchronize(s));
      CHK(hipMemcpy(host.data(), buf, cap, hipMemcpyDeviceToHost));
      CHK(hipMemcpy(host_out.data(), out, cap, hipMemcpyDeviceToHost));
      const size_t lo = guard + c.offset, hi = lo + c.bytes;
      for (size_t i = lo; i < hi; ++i) {
        bad_fill += host[i] != (unsigned char)c.value;
        bad_read += host_out[i] != (unsigned char)c.value;
      }
      for (size_t i = 0; i < guard; ++i) bad_guard += host[lo - guard + i] != 0xAB && i < guard - c.offset;
      for (size_t i = hi; i < hi + guard && i < cap; ++i) bad_guard += host[i] != 0xAB;
    }
    std::printf("  %d replays: wrong bytes in the region %d, guard bytes changed %d, consumer saw wrong bytes %d  -> %s\n",
                reps, bad_fill, bad_guard, bad_read, (bad_fill || bad_guard || bad_read) ? "BAD" : "ok");
    bad_cases += (bad_fill || bad_guard || bad_read) ? 1 : 0;
    CHK(hipGraphExecDestroy(ge));
    CHK(hipGraphDestroy(g));
  }
  std::printf("memset_capture_probe: %d of %zu cases wrong\n", bad_cases, cases.size());

  // Part 2: back-to-back replays without a host sync, as run_epoch issues them.
  //   k_stamp: ctr += 1; X[i] = ctr          (every element)
  //   memset(Y, 0) / memcpy(Y <- X)          (the node under test, 64 MiB)
  //   k_check: counts i with Y[i] != expected (0, or ctr + 1 for the copy); k_bump: ctr += 1
  // 200 launches of each graph in a row; any node overlapping its predecessor
  // (inside one launch or across launches) shows up as mismatches.
  {
    const size_t n = (64u << 20) / 4;
    unsigned *X, *Y, *ctr, *err;
    CHK(hipMalloc(&X, n * 4));
    CHK(hipMalloc(&Y, n * 4));
    CHK(hipMalloc(&ctr, 4));
    CHK(hipMalloc(&err, 4));
    for (int kind = 0; kind < 2; ++kind) {
      CHK(hipMemsetAsync(ctr, 0, 4, s));
      CHK(hipMemsetAsync(err, 0, 4, s));
      CHK(hipStreamSynchronize(s));
      hipGraph_t g;
      CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      hipLaunchKernelGGL(k_stamp, dim3(2048), dim3(256), 0, s, X, n, ctr);
      if (kind == 0) CHK(hipMemsetAsync(Y, 0, n * 4, s));
      else CHK(hipMemcpyAsync(Y, X, n * 4, hipMemcpyDeviceToDevice, s));
      hipLaunchKernelGGL(k_check, dim3(2048), dim3(256), 0, s, Y, n, ctr, kind, err);
      hipLaunchKernelGGL(k_bump, dim3(1), dim3(64), 0, s, ctr);
      CHK(hipStreamEndCapture(s, &g));
      hipGraphExec_t ge;
      CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      const int reps = 200;
      for (int r = 0; r < reps; ++r) CHK(hipGraphLaunch(ge, s));
      CHK(hipStreamSynchronize(s));
      unsigned herr = 0, hctr = 0;
      CHK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      CHK(hipMemcpy(&hctr, ctr, 4, hipMemcpyDeviceToHost));
      std::printf("back-to-back %s node, 64 MiB, %d launches: counter %u, mismatching elements %u -> %s\n",
                  kind ? "memcpy D2D" : "memset", reps, hctr, herr, (herr || hctr != (unsigned)reps) ? "BAD" : "ok");
      CHK(hipGraphExecDestroy(ge));
      CHK(hipGraphDestroy(g));
    }
    CHK(hipFree(X));
    CHK(hipFree(Y));
    CHK(hipFree(ctr));
    CHK(hipFree(err));
  }
  CHK(hipFree(buf));
  CHK(hipFree(out));
  CHK(hipStreamDestroy(s));
  return 0;
}
