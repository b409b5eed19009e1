// k_head.h -- the callers either side of the propagation path (SURVEY §8f
// rank 1), btb task:
//   front-end  get_initial_node_representation, chem_tensorflow_dense.py:264-306:
//              h0[g,i,:] = [dropout(E_s[word_inputs[g,i,col_s]]) for s] ++ zero pad to h
//   heads      gated_regression, chem_tensorflow_dense.py:439-516, with the
//              MLP(2h, o, []) of utils.py:40-84 and the btb loss of
//              chem_tensorflow.py:349-403:
//                z = [h_T | h0] @ dropout(W) + b ;  p = softmax(z) over o
//                loss = sum_rows -sum_o y log p / task_target_num
// The three products of a head (logits, d[hT | h0], dW) run on the general
// path's MFMA GEMM (k_gemm_ring / k_gemm, split f16 limbs in the fp32 mode);
// this file holds the element-wise parts.  Wd and dZ rows are padded to a
// multiple of 4 columns (zeros) so their 16-byte chunks stay whole.
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
  return philox4x32_10(make_uint4((uint32_t)(r >> 2), (uint32_t)k, 0u, 0xC0000000u), dkey0(d), dkey1(d));
}
DEV int emb_find(const EmbArgs& a, int k) {
  int s = -1;
#pragma unroll
  for (int i = 0; i < EMB_MAXSEG; ++i)
    if (i < a.nseg && k >= a.s[i].offset && k < a.s[i].offset + a.s[i].width) s = i;
  return s;
}

// h0 [rows][H]: one thread per (row quad, column): one Philox block serves
// the quad's 4 rows (its 4 words are the 4 rows' masks)
__global__ void __launch_bounds__(256) k_embed_fwd(EmbArgs a, const int* __restrict__ wi, float* __restrict__ h0) {
  const Drop dr = drop_resolve(a.dr);  // (a device-resident key: loaded once)
  const long nq = (a.rows + 3) >> 2, total = nq * a.H;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long q = e / a.H;
    const int k = (int)(e % a.H);
    const int s = emb_find(a, k);
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (s >= 0 && dr.thr) w = emb_words(dr, q * 4, k);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long r = q * 4 + i;
      if (r >= a.rows) break;
      float x = 0.f;
      if (s >= 0) {
        const EmbSeg& S = a.s[s];
        const int id = wi[r * a.ncols + S.column];
        if (id >= 0 && id < S.rows) x = S.table[(long)id * S.width + (k - S.offset)];
        if (dr.thr) x = drop_apply(dr, u4_get(w, i), x);
      }
      h0[r * a.H + k] = x;
    }
  }
}

// d_table[id] += dropout'(dh0 (+ dh0_add)) per lookup (fp32 atomics, tables
// zeroed by the host), and the sum of squares of the per-lookup gradient rows
// per segment: the norm tf.clip_by_norm takes of an embedding's IndexedSlices
// gradient (its values, duplicates not merged) -- chem_tensorflow.py:498-503.
// One thread per (row quad, column), as k_embed_fwd.
struct EmbGrad {
  float* dtable[EMB_MAXSEG];
  int sqslot[EMB_MAXSEG];  // lookup_sqnorm slot of each segment: the first segment with the same d_table
};
__global__ void __launch_bounds__(256) k_embed_bwd(EmbArgs a, EmbGrad gd, const int* __restrict__ wi,
                                                   const float* __restrict__ dh0, const float* __restrict__ dh0_add,
                                                   float* __restrict__ sq) {
  const Drop dr = drop_resolve(a.dr);  // (a device-resident key: loaded once)
  float acc[EMB_MAXSEG];
#pragma unroll
  for (int i = 0; i < EMB_MAXSEG; ++i) acc[i] = 0.f;
  const long nq = (a.rows + 3) >> 2, total = nq * a.H;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long q = e / a.H;
    const int k = (int)(e % a.H);
    const int s = emb_find(a, k);
    if (s < 0) continue;
    const EmbSeg& S = a.s[s];
    const uint4 w = dr.thr ? emb_words(dr, q * 4, k) : make_uint4(0u, 0u, 0u, 0u);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long r = q * 4 + i;
      if (r >= a.rows) break;
      float g = dh0[r * a.H + k] + (dh0_add ? dh0_add[r * a.H + k] : 0.f);
      if (dr.thr) g = drop_apply(dr, u4_get(w, i), g);
      const int id = wi[r * a.ncols + S.column];
      if (id < 0 || id >= S.rows) continue;
      atomicAdd(gd.dtable[s] + (long)id * S.width + (k - S.offset), g);
      ss += g * g;
    }
#pragma unroll
    for (int i = 0; i < EMB_MAXSEG; ++i)
      if (i == s) acc[i] += ss;
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
    atomicAdd(sq + gd.sqslot[i], red[0][i] + red[1][i] + red[2][i] + red[3][i]);
  }
}

// ---- the deterministic form (ggnn_embed_backward_ws, round 5).  The lookups
// add into a 64-bit fixed-point copy of each table (EMB_FX fractional bits):
// integer addition does not depend on the order the atomics land in, so the
// table gradient is the same bits run to run (and for any split of the
// lookups).  Each looked-up row also records its owner, the first lookup row
// of that id (atomicMax of rows - r); k_embed_fin then has the owner's wave
// convert the row to fp32, clear it and release the owner slot, so the
// workspace is all zeros again after every call (the caller zero-fills it
// once).  Per-lookup squared norms: one partial per (block, segment), summed
// in a fixed order by k_embed_fin's last block.  Range: |table gradient
// element| < 2^23; resolution 2^-40.
#define EMB_FX 40
#define EMB_SQ_BLOCKS 4096  // k_embed_bwd_det blocks at most (one squared-norm partial row each)
struct EmbAcc {
  long long* acc[EMB_MAXSEG];  // [rows][width] fixed-point accumulator of segment s's table (shared per table)
  int* own[EMB_MAXSEG];        // [rows] owner slots (emb_owner of the first lookup), 0 = none
};
// owner code of lookup (row r, segment s): the largest code is the smallest
// row, then the smallest segment (segments sharing a table share the slots)
DEV int emb_owner(long rows, long r, int s) { return (int)(((rows - r) << 3) | (EMB_MAXSEG - 1 - s)); }
__global__ void __launch_bounds__(256) k_embed_bwd_det(EmbArgs a, EmbAcc ea, const int* __restrict__ wi,
                                                       const float* __restrict__ dh0,
                                                       const float* __restrict__ dh0_add, float* __restrict__ sqp) {
  const Drop dr = drop_resolve(a.dr);
  float acc[EMB_MAXSEG];
#pragma unroll
  for (int i = 0; i < EMB_MAXSEG; ++i) acc[i] = 0.f;
  const long nq = (a.rows + 3) >> 2, total = nq * a.H;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long q = e / a.H;
    const int k = (int)(e % a.H);
    const int s = emb_find(a, k);
    if (s < 0 || !ea.acc[s]) continue;  // (no accumulator: a segment without a gradient here)
    const EmbSeg& S = a.s[s];
    const uint4 w = dr.thr ? emb_words(dr, q * 4, k) : make_uint4(0u, 0u, 0u, 0u);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long r = q * 4 + i;
      if (r >= a.rows) break;
      float g = dh0[r * a.H + k] + (dh0_add ? dh0_add[r * a.H + k] : 0.f);
      if (dr.thr) g = drop_apply(dr, u4_get(w, i), g);
      const int id = wi[r * a.ncols + S.column];
      if (id < 0 || id >= S.rows) continue;
      const long long fx = __double2ll_rn((double)g * (double)(1LL << EMB_FX));
      atomicAdd((unsigned long long*)(ea.acc[s] + (long)id * S.width + (k - S.offset)), (unsigned long long)fx);
      if (k == S.offset) atomicMax(ea.own[s] + id, emb_owner(a.rows, r, s));
      ss += g * g;
    }
#pragma unroll
    for (int i = 0; i < EMB_MAXSEG; ++i)
      if (i == s) acc[i] += ss;
  }
  __shared__ float red[4][EMB_MAXSEG];
#pragma unroll
  for (int i = 0; i < EMB_MAXSEG; ++i) {
    float x = acc[i];
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][i] = x;
  }
  __syncthreads();
  if (threadIdx.x < EMB_MAXSEG)
    sqp[(long)blockIdx.x * EMB_MAXSEG + threadIdx.x] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}
// one wave per (lookup row, segment): the owner converts its id's row into
// d_table (zeroed before), clears the accumulator row and releases the slot;
// the last block sums the squared-norm partials (nblk rows) per slot:
// 256 threads over contiguous block ranges, then a fixed-order LDS tree
__global__ void __launch_bounds__(256) k_embed_fin(EmbArgs a, EmbAcc ea, EmbGrad gd, const int* __restrict__ wi,
                                                   float* __restrict__ sqp, int nblk, float* __restrict__ sq) {
  if (blockIdx.x == gridDim.x - 1) {
    __shared__ float t[256][EMB_MAXSEG + 1];
    const int per = (nblk + 255) / 256, b0 = threadIdx.x * per, b1 = min(nblk, b0 + per);
    float v[EMB_MAXSEG];
#pragma unroll
    for (int i = 0; i < EMB_MAXSEG; ++i) v[i] = 0.f;
    for (int b = b0; b < b1; ++b)
#pragma unroll
      for (int i = 0; i < EMB_MAXSEG; ++i) v[i] += sqp[(long)b * EMB_MAXSEG + i];
#pragma unroll
    for (int i = 0; i < EMB_MAXSEG; ++i) t[threadIdx.x][i] = v[i];
    // (the partials are cleared too: the whole workspace is zero after a call)
    for (int b = b0; b < b1; ++b)
#pragma unroll
      for (int i = 0; i < EMB_MAXSEG; ++i) sqp[(long)b * EMB_MAXSEG + i] = 0.f;
    __syncthreads();
    for (int h = 128; h >= 1; h >>= 1) {
      if (threadIdx.x < h)
#pragma unroll
        for (int i = 0; i < EMB_MAXSEG; ++i) t[threadIdx.x][i] += t[threadIdx.x + h][i];
      __syncthreads();
    }
    if (threadIdx.x < a.nseg) {
      const int slot = threadIdx.x;
      float x = 0.f;
      for (int i = 0; i < a.nseg; ++i)
        if (gd.sqslot[i] == slot) x += t[0][i];
      sq[slot] = x;
    }
    return;
  }
  const long wv = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wv >= a.rows * a.nseg) return;
  const long r = wv / a.nseg;
  const int s = (int)(wv % a.nseg);
  const EmbSeg& S = a.s[s];
  if (!ea.acc[s]) return;
  const int id = wi[r * a.ncols + S.column];
  if (id < 0 || id >= S.rows || ea.own[s][id] != emb_owner(a.rows, r, s)) return;
  long long* ar = ea.acc[s] + (long)id * S.width;
  float* dt = gd.dtable[s] + (long)id * S.width;
  for (int k = lane; k < S.width; k += 64) {
    dt[k] = (float)((double)ar[k] * (1.0 / (double)(1LL << EMB_FX)));
    ar[k] = 0;
  }
  if (lane == 0) ea.own[s][id] = 0;
}

// One segment's per-lookup gradient rows, as the reference's IndexedSlices
// holds them (values, indices; chem_tensorflow.py:496-500): rows[r][j] =
// dropout'(dh0 + dh0_add)[r][offset + j], ids[r] = the looked-up row (-1 out of
// range); rows r in [rows, cap) are zero with id -1.  The data-parallel step
// all-gathers them and accumulates the union (ggnn_embed_backward_ws, exact
// in fixed point) instead of all-reducing the dense table.
__global__ void __launch_bounds__(256) k_embed_rows(EmbArgs a, int s, const int* __restrict__ wi,
                                                    const float* __restrict__ dh0, const float* __restrict__ dh0_add,
                                                    float* __restrict__ rows, int* __restrict__ ids, long cap) {
  const Drop dr = drop_resolve(a.dr);
  const EmbSeg& S = a.s[s];
  const long total = cap * S.width;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long r = e / S.width;
    const int j = (int)(e % S.width), k = S.offset + j;
    float g = 0.f;
    int id = -1;
    if (r < a.rows) {
      g = dh0[r * a.H + k] + (dh0_add ? dh0_add[r * a.H + k] : 0.f);
      if (dr.thr) g = drop_apply(dr, u4_get(emb_words(dr, (r >> 2) * 4, k), (int)(r & 3)), g);
      id = wi[r * a.ncols + S.column];
      if (id < 0 || id >= S.rows) id = -1;
    }
    rows[e] = g;
    if (j == 0) ids[r] = id;
  }
}

// ---------------------------------------------------------------------------
// output heads
// ---------------------------------------------------------------------------
// out-layer weight dropout mask of W[i][j] of head hd: counter (i>>2, j, hd, 0xA0000000), word i&3
DEV uint4 head_words(const Drop& d, int hd, int i, int j) {
  return philox4x32_10(make_uint4((uint32_t)i >> 2, (uint32_t)j, (uint32_t)hd, 0xA0000000u), dkey0(d), dkey1(d));
}
// head hd's columns [off, off + op) of the concatenated W * mask / keep and
// mask / keep ([K][Ot], K = 2H; op = o rounded up to 4, padding zeros) and of
// the concatenated bias, once per step
__global__ void k_head_wdrop(const float* __restrict__ W, const float* __restrict__ bias, int K, int o, int op, int Ot,
                             int off, int hd, Drop dr, float* __restrict__ Wd, float* __restrict__ S,
                             float* __restrict__ ball) {
  dr = drop_resolve(dr);  // (a device-resident key: loaded once)
  const long total = (long)K * op;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int i = (int)(e / op), j = (int)(e % op);
    const long d = (long)i * Ot + off + j;
    if (i == 0) ball[off + j] = j < o ? bias[j] : 0.f;
    if (j >= o) {
      Wd[d] = 0.f;
      S[d] = 0.f;
      continue;
    }
    const float s = dr.thr ? drop_apply(dr, u4_get(head_words(dr, hd, i, j), i & 3), 1.0f) : 1.0f;
    S[d] = s;
    Wd[d] = W[(long)i * o + j] * s;
  }
}
// d_weight [K][o] = head's columns of the concatenated dW [K][Ot]
__global__ void k_head_dw_out(const float* __restrict__ dWall, int Ot, int K, int o, float* __restrict__ dW) {
  const long total = (long)K * o;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x)
    dW[e] = dWall[(e / o) * Ot + e % o];
}
// loss = sum of the softmax blocks' partials (one block)
__global__ void __launch_bounds__(256) k_head_loss(const float* __restrict__ lp, int n, float* __restrict__ loss) {
  float x = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) x += lp[i];
  for (int s = 32; s >= 1; s >>= 1) x += __shfl_xor(x, s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) *loss = red[0] + red[1] + red[2] + red[3];
}

// p = softmax(z) per row (z: a head's columns of the concatenated logits, row
// stride zs), and the block's share of -sum y log p / num (lpart[block],
// summed by k_head_loss: same-address atomics from every block serialise).
// One wave per row, two rows per iteration, rows held in registers (lane l:
// columns l + 64 i, o <= HEAD_MAXO): one load round trip per row pair.
#define HEAD_MAXO 1024
template <int NI>
__global__ void __launch_bounds__(256) k_head_softmax(const float* __restrict__ zin, int zs, float* __restrict__ pout,
                                                      const float* __restrict__ y, long rows, int o, float inv_num,
                                                      const float* __restrict__ num_dev, float* __restrict__ lpart) {
  const int lane = threadIdx.x & 63;
  if (num_dev) inv_num = 1.0f / *num_dev;  // (ggnn_heads_forward_dev: target_num in device memory)
  const long stride = (long)gridDim.x * 4;
  float term = 0.f;
  // two rows per wave and iteration: both rows' loads in flight together
  for (long r0 = (long)blockIdx.x * 4 + (threadIdx.x >> 6); r0 < rows; r0 += 2 * stride) {
    float x[2][NI], yy[2][NI];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long r = r0 + u * stride;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int j = lane + 64 * i;
        const bool ok = r < rows && j < o;
        x[u][i] = ok ? zin[r * zs + j] : -INFINITY;
        yy[u][i] = (y && ok) ? y[r * o + j] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long r = r0 + u * stride;
      if (r >= rows) break;
      float mx = x[u][0];
#pragma unroll
      for (int i = 1; i < NI; ++i) mx = fmaxf(mx, x[u][i]);
      for (int s = 32; s >= 1; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s));
      float se = 0.f;
#pragma unroll
      for (int i = 0; i < NI; ++i) se += lane + 64 * i < o ? expf(x[u][i] - mx) : 0.f;
      for (int s = 32; s >= 1; s >>= 1) se += __shfl_xor(se, s);
      const float lse = mx + logf(se);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int j = lane + 64 * i;
        if (j < o) {
          // log p computed as z - logsumexp (the reference takes log(softmax): the
          // same value wherever softmax does not underflow to 0)
          term -= yy[u][i] * (x[u][i] - lse);
          pout[r * o + j] = expf(x[u][i] - lse);
        }
      }
    }
  }
  if (y) {
    for (int s = 32; s >= 1; s >>= 1) term += __shfl_xor(term, s);
    __shared__ float red[4];
    if (lane == 0) red[threadIdx.x >> 6] = term;
    __syncthreads();
    if (threadIdx.x == 0) lpart[blockIdx.x] = (red[0] + red[1] + red[2] + red[3]) * inv_num;
  }
}

// dZ = g * (p * sum(y) - y) / num per row (d/dz of -sum y log softmax(z)), and
// the bias gradient's block partials dbp[block * ldp + j] = sum over the
// block's rows of dZ[r][j]: column partials in registers (lane l owns columns
// l + 64i, o <= HEAD_MAXO), summed over the block's waves in LDS in wave order
// (the blocks' rows are summed in block order afterwards: k_sum_rows)
// (dZ: the head's columns of the concatenated [rows][ldz] array, padded to op
// with zeros; the row's p and y held in registers)
template <int NI>
__global__ void __launch_bounds__(256) k_head_dz(const float* __restrict__ p, const float* __restrict__ y, long rows,
                                                 int o, int op, float inv_num, const float* __restrict__ num_dev,
                                                 const float* __restrict__ dloss, float* __restrict__ dZ, int ldz,
                                                 float* __restrict__ dbp, int ldp) {
  __shared__ float cs[4][NI * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (num_dev) inv_num = 1.0f / *num_dev;
  const float g = (dloss ? *dloss : 1.0f) * inv_num;
  float part[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) part[i] = 0.f;
  const long stride = (long)gridDim.x * 4;
  constexpr int RP = 4;  // rows per wave and iteration, loads in flight together
  for (long r0 = (long)blockIdx.x * 4 + w; r0 < rows; r0 += RP * stride) {
    float pv[RP][NI], yv[RP][NI];
#pragma unroll
    for (int u = 0; u < RP; ++u) {
      const long r = r0 + u * stride;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int j = lane + 64 * i;
        const bool ok = r < rows && j < o;
        pv[u][i] = ok ? p[r * o + j] : 0.f;
        yv[u][i] = ok ? y[r * o + j] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < RP; ++u) {
      const long r = r0 + u * stride;
      if (r >= rows) break;
      float sy = 0.f;
#pragma unroll
      for (int i = 0; i < NI; ++i) sy += yv[u][i];
      for (int s = 32; s >= 1; s >>= 1) sy += __shfl_xor(sy, s);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int j = lane + 64 * i;
        if (j < o) {
          const float d = g * (pv[u][i] * sy - yv[u][i]);
          dZ[r * ldz + j] = d;
          part[i] += d;
        } else if (j < op) {
          dZ[r * ldz + j] = 0.f;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i)
    if (lane + 64 * i < o) cs[w][lane + 64 * i] = part[i];
  __syncthreads();
  for (int j = threadIdx.x; j < o; j += 256) dbp[(long)blockIdx.x * ldp + j] = ((cs[0][j] + cs[1][j]) + cs[2][j]) + cs[3][j];
}
