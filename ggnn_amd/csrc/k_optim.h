// k_optim.h -- the reference's optimizer step for the path's variables, fused:
//   g' = s * g                      (s = 1/N: data-parallel mean of per-rank sums)
//   g'' = tf.clip_by_norm(g', c)  = g' * c / max(||g'||_2, c)   per tensor
//   TF1 AdamOptimizer (chem_tensorflow.py:494-503; tf.compat.v1.train.AdamOptimizer):
//     m = b1 m + (1-b1) g'' ;  v = b2 v + (1-b2) g''^2
//     p -= lr * sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps)
// Two launches: per-tensor sums of squares (fp32 atomics into `sq`), then the
// elementwise update.  HBM-bound: 4 reads + 3 writes of fp32 per element.
#pragma once
#include "ggnn_common.h"

#define GGNN_OPT_MAXT 16
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
};

// per-tensor sum of (gscale * g)^2 into sq[tensor]; blockIdx.y = tensor,
// blockIdx.x strides over its elements (one atomic per block)
__global__ void __launch_bounds__(256) k_opt_sqnorm(OptArgs a, float* __restrict__ sq) {
  __shared__ float red[4];
  const OptTensor& T = a.t[blockIdx.y];
  float acc = 0.f;
  if (!T.sqo) {
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < T.n; e += (long)gridDim.x * blockDim.x) {
      const float g = a.gscale * T.g[e];
      acc += g * g;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  // per-block partial (no atomics, no zeroing): sq[tensor * gridDim.x + block]
  if (threadIdx.x == 0) sq[blockIdx.y * gridDim.x + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) k_opt_adam(OptArgs a, const float* __restrict__ sq) {
  const OptTensor& T = a.t[blockIdx.y];
  __shared__ float tot;
  if (threadIdx.x < 64) {  // this tensor's squared norm from the sqnorm launch's partials
    float x = 0.f;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += 64) x += sq[blockIdx.y * gridDim.x + i];
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    if (threadIdx.x == 0) tot = T.sqo ? a.gscale * a.gscale * *T.sqo : x;
  }
  __syncthreads();
  // tf.clip_by_norm: t * clip / max(l2norm, clip)
  const float scale = a.gscale * a.clip / fmaxf(sqrtf(tot), a.clip);
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < T.n; e += (long)gridDim.x * blockDim.x) {
    const float g = T.g[e] * scale;
    const float m = a.b1 * T.m[e] + (1.0f - a.b1) * g;
    const float v = a.b2 * T.v[e] + (1.0f - a.b2) * g * g;
    T.m[e] = m;
    T.v[e] = v;
    T.p[e] -= a.lr_t * m / (sqrtf(v) + a.eps);
  }
}
