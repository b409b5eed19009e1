// k_head.h -- the callers either side of the propagation path (SURVEY §8f
// rank 1), btb task:
//   front-end  get_initial_node_representation, chem_tensorflow_dense.py:264-306:
//              h0[g,i,:] = [dropout(E_s[word_inputs[g,i,col_s]]) for s] ++ zero pad to h
//   heads      gated_regression, chem_tensorflow_dense.py:439-516, with the
//              MLP(2h, o, []) of utils.py:40-84 and the btb loss of
//              chem_tensorflow.py:349-403:
//                z = [h_T | h0] @ dropout(W) + b ;  p = softmax(z) over o
//                loss = sum_rows -sum_o y log p / task_target_num
// Small next to the propagation (b*v*2h*o MACs per head), so plain fp32 FMA
// tiles (fp32 parity by construction) rather than MFMA limb products.
#pragma once
#include "ggnn_common.h"

// ---------------------------------------------------------------------------
// embedding front-end
// ---------------------------------------------------------------------------
#define EMB_MAXSEG 8
struct EmbSeg {
  const float* table;
  long rows;
  int width, column, offset;  // columns [offset, offset + width) of h0
};
struct EmbArgs {
  EmbSeg s[EMB_MAXSEG];
  int nseg, ncols, H;
  long rows;  // b * v node rows
  Drop dr;    // emb_dropout_keep_prob
};
// embedding dropout mask of element (row r, column k): counter (r>>2, k, 0, 0xC0000000), word r&3
DEV uint4 emb_words(const Drop& d, long r, int k) {
  return philox4x32_10(make_uint4((uint32_t)(r >> 2), (uint32_t)k, 0u, 0xC0000000u), d.k0, d.k1);
}
DEV int emb_find(const EmbArgs& a, int k) {
  int s = -1;
#pragma unroll
  for (int i = 0; i < EMB_MAXSEG; ++i)
    if (i < a.nseg && k >= a.s[i].offset && k < a.s[i].offset + a.s[i].width) s = i;
  return s;
}

// h0 [rows][H]: one thread per element (tiny: b*v*H)
__global__ void __launch_bounds__(256) k_embed_fwd(EmbArgs a, const int* __restrict__ wi, float* __restrict__ h0) {
  const long total = a.rows * a.H;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long r = e / a.H;
    const int k = (int)(e % a.H);
    const int s = emb_find(a, k);
    float x = 0.f;
    if (s >= 0) {
      const EmbSeg& S = a.s[s];
      const int id = wi[r * a.ncols + S.column];
      if (id >= 0 && id < S.rows) x = S.table[(long)id * S.width + (k - S.offset)];
      if (a.dr.thr) x = drop_apply(a.dr, u4_get(emb_words(a.dr, r, k), (int)(r & 3)), x);
    }
    h0[e] = x;
  }
}

// d_table[id] += dropout'(dh0 (+ dh0_add)) per lookup (fp32 atomics, tables
// zeroed by the host), and the sum of squares of the per-lookup gradient rows
// per segment: the norm tf.clip_by_norm takes of an embedding's IndexedSlices
// gradient (its values, duplicates not merged) -- chem_tensorflow.py:498-503.
struct EmbGrad {
  float* dtable[EMB_MAXSEG];
};
__global__ void __launch_bounds__(256) k_embed_bwd(EmbArgs a, EmbGrad gd, const int* __restrict__ wi,
                                                   const float* __restrict__ dh0, const float* __restrict__ dh0_add,
                                                   float* __restrict__ sq) {
  float acc[EMB_MAXSEG];
#pragma unroll
  for (int i = 0; i < EMB_MAXSEG; ++i) acc[i] = 0.f;
  const long total = a.rows * a.H;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long r = e / a.H;
    const int k = (int)(e % a.H);
    const int s = emb_find(a, k);
    if (s < 0) continue;
    const EmbSeg& S = a.s[s];
    float g = dh0[e] + (dh0_add ? dh0_add[e] : 0.f);
    if (a.dr.thr) g = drop_apply(a.dr, u4_get(emb_words(a.dr, r, k), (int)(r & 3)), g);
    const int id = wi[r * a.ncols + S.column];
    if (id < 0 || id >= S.rows) continue;
    atomicAdd(gd.dtable[s] + (long)id * S.width + (k - S.offset), g);
#pragma unroll
    for (int i = 0; i < EMB_MAXSEG; ++i)
      if (i == s) acc[i] += g * g;
  }
  __shared__ float red[4][EMB_MAXSEG];
#pragma unroll
  for (int i = 0; i < EMB_MAXSEG; ++i) {
    float x = acc[i];
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][i] = x;
  }
  __syncthreads();
  if (threadIdx.x < a.nseg) {
    const int i = threadIdx.x;
    atomicAdd(sq + i, red[0][i] + red[1][i] + red[2][i] + red[3][i]);
  }
}

// ---------------------------------------------------------------------------
// output heads
// ---------------------------------------------------------------------------
// out-layer weight dropout mask of W[i][j] of head hd: counter (i>>2, j, hd, 0xA0000000), word i&3
DEV uint4 head_words(const Drop& d, int hd, int i, int j) {
  return philox4x32_10(make_uint4((uint32_t)i >> 2, (uint32_t)j, (uint32_t)hd, 0xA0000000u), d.k0, d.k1);
}
// Wd = W * mask / keep and S = mask / keep ([K][o], K = 2H), once per step
__global__ void k_head_wdrop(const float* __restrict__ W, int K, int o, int hd, Drop dr, float* __restrict__ Wd,
                             float* __restrict__ S) {
  const long total = (long)K * o;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int i = (int)(e / o), j = (int)(e % o);
    const float s = dr.thr ? drop_apply(dr, u4_get(head_words(dr, hd, i, j), i & 3), 1.0f) : 1.0f;
    S[e] = s;
    Wd[e] = W[e] * s;
  }
}

// fp32 tile GEMM C[M][N] = sum_k A(m,k) B(k,n) over a K range (split-K over
// blockIdx.z); 64x64 tiles, 256 threads, 4x4 outputs per thread.  The problem
// type P supplies the operand reads (with the coalesced index fastest) and the
// epilogue.
template <class P>
__global__ void __launch_bounds__(256) k_sgemm(P p) {
  constexpr int BM = 64, BN = 64, BK = 16;
  __shared__ float As[BK][BM + 4], Bs[BK][BN + 4];
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const long kper = (p.K + gridDim.z - 1) / gridDim.z;
  const long kb = (long)blockIdx.z * kper, ke = min((long)p.K, kb + kper);
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  float acc[4][4] = {};
  for (long k0 = kb; k0 < ke; k0 += BK) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      int m, kk;
      if (P::kAmFast) { m = e % BM; kk = e / BM; } else { kk = e % BK; m = e / BK; }
      const long k = k0 + kk;
      As[kk][m] = (m0 + m < p.M && k < ke) ? p.a(m0 + m, k) : 0.f;
      int n, kk2;
      if (P::kBnFast) { n = e % BN; kk2 = e / BN; } else { kk2 = e % BK; n = e / BK; }
      const long k2 = k0 + kk2;
      Bs[kk2][n] = (n0 + n < p.N && k2 < ke) ? p.b(k2, n0 + n) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + ty + 16 * i, n = n0 + tx + 16 * j;
      if (m < p.M && n < p.N) p.store(m, n, acc[i][j]);
    }
}

// z[r][j] = [hT | h0][r] . Wd[:, j] + b[j]
struct HeadLogitsP {
  static constexpr bool kAmFast = false, kBnFast = true;
  const float *hT, *h0, *Wd, *bias;
  float* z;
  int M, N, K, H;
  DEV float a(int m, long k) const { return k < H ? hT[(long)m * H + k] : h0[(long)m * H + (k - H)]; }
  DEV float b(long k, int n) const { return Wd[k * N + n]; }
  DEV void store(int m, int n, float v) const { z[(long)m * N + n] = v + bias[n]; }
};
// [dhT | dh0][r][c] (+)= sum_j dZ[r][j] Wd[c][j]
struct HeadDxP {
  static constexpr bool kAmFast = false, kBnFast = false;
  const float *dZ, *Wd;
  float *dhT, *dh0;
  int M, N, K, H, accumulate;
  DEV float a(int m, long k) const { return dZ[(long)m * K + k]; }
  DEV float b(long k, int n) const { return Wd[(long)n * K + k]; }
  DEV void store(int m, int n, float v) const {
    float* d = n < H ? dhT + (long)m * H + n : dh0 + (long)m * H + (n - H);
    *d = accumulate ? *d + v : v;
  }
};
// dW[c][j] += S[c][j] * sum_r [hT | h0][r][c] dZ[r][j]   (split over rows: atomics)
struct HeadDwP {
  static constexpr bool kAmFast = true, kBnFast = true;
  const float *hT, *h0, *dZ, *S;
  float* dW;
  int M, N, H;
  long K;
  DEV float a(int m, long k) const { return m < H ? hT[k * H + m] : h0[k * H + (m - H)]; }
  DEV float b(long k, int n) const { return dZ[k * N + n]; }
  DEV void store(int m, int n, float v) const { atomicAdd(dW + (long)m * N + n, v * S[(long)m * N + n]); }
};

// in place z -> p = softmax(z) per row (one wave per row, rows grid-strided
// over a few hundred blocks), loss += -sum y log p / num (one atomic per block:
// one per 4 rows serialised 8192 same-address atomics at b*v = 32768)
__global__ void __launch_bounds__(256) k_head_softmax(float* __restrict__ zp, const float* __restrict__ y, long rows,
                                                      int o, float inv_num, float* __restrict__ loss) {
  const int lane = threadIdx.x & 63;
  float term = 0.f;
  for (long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (long)gridDim.x * 4) {
    float* z = zp + r * o;
    float mx = -INFINITY;
    for (int j = lane; j < o; j += 64) mx = fmaxf(mx, z[j]);
    for (int s = 32; s >= 1; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s));
    float se = 0.f;
    for (int j = lane; j < o; j += 64) se += expf(z[j] - mx);
    for (int s = 32; s >= 1; s >>= 1) se += __shfl_xor(se, s);
    const float lse = mx + logf(se);
    for (int j = lane; j < o; j += 64) {
      const float zj = z[j];
      // log p computed as z - logsumexp (the reference takes log(softmax): the
      // same value wherever softmax does not underflow to 0)
      if (y) term -= y[r * o + j] * (zj - lse);
      z[j] = expf(zj - lse);
    }
  }
  if (y) {
    for (int s = 32; s >= 1; s >>= 1) term += __shfl_xor(term, s);
    __shared__ float red[4];
    if (lane == 0) red[threadIdx.x >> 6] = term;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(loss, (red[0] + red[1] + red[2] + red[3]) * inv_num);
  }
}

// dZ = g * (p * sum(y) - y) / num per row (d/dz of -sum y log softmax(z)), and
// the bias gradient db[j] += sum_r dZ[r][j]: column partials in registers
// (lane l owns columns l + 64i, o <= HEAD_MAXO), summed over the block's waves
// in LDS, one global atomic per column per block
#define HEAD_MAXO 1024
__global__ void __launch_bounds__(256) k_head_dz(const float* __restrict__ p, const float* __restrict__ y, long rows,
                                                 int o, float inv_num, const float* __restrict__ dloss,
                                                 float* __restrict__ dZ, float* __restrict__ db) {
  constexpr int NI = HEAD_MAXO / 64;
  __shared__ float cs[4][HEAD_MAXO];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float g = (dloss ? *dloss : 1.0f) * inv_num;
  float part[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) part[i] = 0.f;
  for (long r = (long)blockIdx.x * 4 + w; r < rows; r += (long)gridDim.x * 4) {
    float sy = 0.f;
    for (int j = lane; j < o; j += 64) sy += y[r * o + j];
    for (int s = 32; s >= 1; s >>= 1) sy += __shfl_xor(sy, s);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = lane + 64 * i;
      if (j < o) {
        const float d = g * (p[r * o + j] * sy - y[r * o + j]);
        dZ[r * o + j] = d;
        part[i] += d;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i)
    if (lane + 64 * i < o) cs[w][lane + 64 * i] = part[i];
  __syncthreads();
  for (int j = threadIdx.x; j < o; j += 256) atomicAdd(db + j, cs[0][j] + cs[1][j] + cs[2][j] + cs[3][j]);
}

// db[j] = sum_r dZ[r][j] (2D grid: blockIdx.y strides the rows; atomics)
__global__ void k_colsum(const float* __restrict__ dZ, long rows, int o, float* __restrict__ db) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= o) return;
  float s = 0.f;
  for (long r = blockIdx.y; r < rows; r += gridDim.y) s += dZ[r * o + j];
  atomicAdd(db + j, s);
}
