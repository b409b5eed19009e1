// k_optim.h -- the reference's optimizer step for the path's variables, fused:
//   g' = s * g                      (s = 1/N: data-parallel mean of per-rank sums)
//   g'' = tf.clip_by_norm(g', c)  = g' * c / max(||g'||_2, c)   per tensor
//   TF1 AdamOptimizer (chem_tensorflow.py:494-503; tf.compat.v1.train.AdamOptimizer):
//     m = b1 m + (1-b1) g'' ;  v = b2 v + (1-b2) g''^2
//     p -= lr * sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps)
// Two launches: per-tensor sums of squares (one partial per block, summed in
// block order), then the elementwise update.  HBM-bound: 4 reads + 3 writes of
// fp32 per element, as 16-byte pieces.  Blocks of OPT_THREADS = 1024: a launch
// has GGNN_ADAM_SCRATCH_PER_TENSOR (256) blocks per tensor, so the largest
// tensor (the edge weights, the word table) sets its duration, and with
// 256-thread blocks that tensor's share of the chip was one block, 4 waves, per
// CU -- too few loads in flight for HBM (2.3-3.5 TB/s measured)
#pragma once
#include "ggnn_common.h"

#define GGNN_OPT_MAXT 16
#define OPT_THREADS 1024
struct OptTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  long n;
  const float* sqo;  // squared-norm override (IndexedSlices norm), or nullptr
};
struct OptArgs {
  OptTensor t[GGNN_OPT_MAXT];
  long begin[GGNN_OPT_MAXT + 1];  // prefix offsets over the concatenated elements
  int count;
  float gscale, clip, lr_t, b1, b2, eps;
  // ggnn_adam_step_dev: the step count is read from device memory and lr_t
  // derived from it in-kernel (lr = the undecayed rate)
  const int64_t* step;
  double lr;
};

// per-tensor sum of (gscale * g)^2 into sq[tensor]; blockIdx.y = tensor,
// blockIdx.x strides over its elements (one atomic per block)
__global__ void __launch_bounds__(OPT_THREADS) k_opt_sqnorm(OptArgs a, float* __restrict__ sq) {
  __shared__ float red[OPT_THREADS / 64];
  const OptTensor& T = a.t[blockIdx.y];
  float acc = 0.f;
  if (!T.sqo) {
    const long st = (long)gridDim.x * blockDim.x;
    long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if ((((unsigned long)T.g) & 15) == 0) {  // 16-byte pieces, then the tail
      for (; 4 * e + 3 < T.n; e += st) {
        const float4 q = *(const float4*)(T.g + 4 * e);
        const float x = a.gscale * q.x, y = a.gscale * q.y, z = a.gscale * q.z, w = a.gscale * q.w;
        acc += (x * x + y * y) + (z * z + w * w);
      }
      e = (T.n & ~3L) + (long)blockIdx.x * blockDim.x + threadIdx.x;
    }
    for (; e < T.n; e += st) {
      const float g = a.gscale * T.g[e];
      acc += g * g;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  // per-block partial (no atomics, no zeroing): sq[tensor * gridDim.x + block]
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < OPT_THREADS / 64; ++w) t += red[w];
    sq[blockIdx.y * gridDim.x + blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(OPT_THREADS) k_opt_adam(OptArgs a, const float* __restrict__ sq) {
  const OptTensor& T = a.t[blockIdx.y];
  __shared__ float tot, lr_t;
  if (threadIdx.x == 64) {
    if (a.step) {  // TF1 Adam folds both bias corrections into the step size
      const double t = (double)*a.step;
      lr_t = (float)(a.lr * sqrt(1.0 - pow((double)a.b2, t)) / (1.0 - pow((double)a.b1, t)));
    } else {
      lr_t = a.lr_t;
    }
  }
  if (threadIdx.x < 64) {  // this tensor's squared norm from the sqnorm launch's partials
    float x = 0.f;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += 64) x += sq[blockIdx.y * gridDim.x + i];
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    if (threadIdx.x == 0) tot = T.sqo ? a.gscale * a.gscale * *T.sqo : x;
  }
  __syncthreads();
  // tf.clip_by_norm: t * clip / max(l2norm, clip)
  const float scale = a.gscale * a.clip / fmaxf(sqrtf(tot), a.clip);
  auto upd = [&](float gg, float& m, float& v, float& p) {
    const float g = gg * scale;
    m = a.b1 * m + (1.0f - a.b1) * g;
    v = a.b2 * v + (1.0f - a.b2) * g * g;
    p -= lr_t * m / (sqrtf(v) + a.eps);
  };
  const long st = (long)gridDim.x * blockDim.x;
  long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  // 16-byte pieces when all four arrays allow it (the same per-element
  // arithmetic), then the tail
  if (((((unsigned long)T.p) | ((unsigned long)T.g) | ((unsigned long)T.m) | ((unsigned long)T.v)) & 15) == 0) {
    for (; 4 * e + 3 < T.n; e += st) {
      const float4 g = *(const float4*)(T.g + 4 * e);
      float4 m = *(const float4*)(T.m + 4 * e), v = *(const float4*)(T.v + 4 * e), p = *(const float4*)(T.p + 4 * e);
      upd(g.x, m.x, v.x, p.x);
      upd(g.y, m.y, v.y, p.y);
      upd(g.z, m.z, v.z, p.z);
      upd(g.w, m.w, v.w, p.w);
      *(float4*)(T.m + 4 * e) = m;
      *(float4*)(T.v + 4 * e) = v;
      *(float4*)(T.p + 4 * e) = p;
    }
    e = (T.n & ~3L) + (long)blockIdx.x * blockDim.x + threadIdx.x;
  }
  for (; e < T.n; e += st) {
    float m = T.m[e], v = T.v[e], p = T.p[e];
    upd(T.g[e], m, v, p);
    T.m[e] = m;
    T.v[e] = v;
    T.p[e] = p;
  }
}
