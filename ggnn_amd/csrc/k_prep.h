// k_prep.h -- boundary conversion kernels (HBM-bound, small next to the hot
// kernels): weight packing, adjacency staging, state padding / transposes.
#pragma once
#include "ggnn_common.h"

// Pack B operand Bmat[K][N] (Bmat = S or S^T, S row-major fp32, leading dim
// ldS) into MFMA fragment order [N/32][K/16][64][8] of 16-bit limbs (bf16, or
// f16 for the split mode), hi part at `out`, lo part (x - limb(x)) at
// `out + lo_off`.  blockIdx.y selects a matrix of a batch (strides sS / sO).
// With dr.thr != 0 the source is W[c] (c = blockIdx.y) under the edge-weight
// dropout mask of timestep t (chem_tensorflow_dense.py:397-403), applied in
// the reference's element coordinates (i = input row, j = output column) so
// that the forward pack (Bmat = W_c) and the backward pack (Bmat = W_c^T)
// see the same mask.
template <bool F16>
__global__ void k_pack_B(const float* __restrict__ S, int ldS, long sS, int K, int N, int trans,
                         u16* __restrict__ out, long sO, long lo_off, Drop dr, int t) {
  dr = drop_resolve(dr);  // (a device-resident key: loaded once)
  const int total = (N / 32) * (K / 16) * 64;
  const float* Sb = S + sS * blockIdx.y;
  u16* ob = out + sO * blockIdx.y;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < total; q += gridDim.x * blockDim.x) {
    const int lane = q & 63, fi = q >> 6;  // fragment index
    const int nks = K / 16;
    const int ks = fi % nks, strip = fi / nks;
    const int n = strip * 32 + (lane & 31), k0 = ks * 16 + 8 * (lane >> 5);
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = trans ? Sb[(long)n * ldS + k0 + j] : Sb[(long)(k0 + j) * ldS + n];
    if (dr.thr) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int wi = trans ? n : k0 + j, wj = trans ? k0 + j : n;
        x[j] = drop_apply(dr, u4_get(edge_words(dr, blockIdx.y, wi, wj, t), wi & 3), x[j]);
      }
    }
    *(uint4*)(ob + (size_t)q * 8) = pk8<F16>(x);
    *(uint4*)(ob + lo_off + (size_t)q * 8) = pk8_lo<F16>(x);
  }
}

__global__ void k_copy_f32(const float* __restrict__ s, float* __restrict__ d, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    d[i] = s ? s[i] : 0.0f;
}

// Adjacency [b][C][vin][vin] fp32 -> per (g,c) tile:
//   Ab  [V][V] bf16, columns permuted inside every 16-column group (8-byte
//       chunks 1 and 2 swapped) = the k order of an accumulator-as-B operand
//       (k_prop_fwd's AGG);
//   AbT [V][V] bf16 = A^T, natural order (B operand of k_prop_bwd);
//   deg [V] 16-bit limbs = row sums (in-degree per channel, <= 128: exact),
//       the B operand of k_prop_bwd's dL/dbeta product.
template <int V, bool F16>
__global__ void __launch_bounds__(256) k_prep_adj(const float* __restrict__ A, int vin,
                                                  u16* __restrict__ Ab, u16* __restrict__ AbT,
                                                  u16* __restrict__ deg) {
  constexpr int P = V + 8;           // row pitch (u16): 16-B aligned rows, odd dword pitch / 4
  __shared__ __attribute__((aligned(16))) u16 tt[V][P];  // A[j][i] (transposed)
  const long tile = blockIdx.x;  // g*C + c
  const float* src = A + tile * (long)vin * vin;
  u16* ab = Ab + tile * V * V;
  u16* at = AbT + tile * V * V;
  if (vin == V) {
    // unpadded: one unit = 4 rows x the 8 columns of one Ab output chunk
    // (columns c0..c0+3 and c0+8..c0+11, c0 = g16 + 4 h), all loads of a
    // thread issued before any use; Ab straight from registers, A^T through
    // LDS as 4-row uint2 pieces, deg as a row sum over the V/8 lanes of a row
    // group (exact for the reference's 0/1 adjacency)
    constexpr int SL = V / 8;                  // units (lanes) per 4-row group
    constexpr int U = V * V / 32;              // units per tile
    constexpr int UPT = (U + 255) / 256;       // units per thread
    float4 x[UPT][4][2];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int u = threadIdx.x + k * 256;
      if (U % 256 == 0 || u < U) {
        const int i = (u / SL) * 4, sl = u % SL, c0 = (sl >> 1) * 16 + (sl & 1) * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[k][r][0] = *(const float4*)(src + (i + r) * V + c0);
          x[k][r][1] = *(const float4*)(src + (i + r) * V + c0 + 8);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) x[k][r][0] = x[k][r][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int u = threadIdx.x + k * 256;
      const bool act = U % 256 == 0 || u < U;
      const int i = (u / SL) * 4, sl = u % SL, c0 = (sl >> 1) * 16 + (sl & 1) * 4;
      u16 a[4][8];
      float rs[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v8[8] = {x[k][r][0].x, x[k][r][0].y, x[k][r][0].z, x[k][r][0].w,
                             x[k][r][1].x, x[k][r][1].y, x[k][r][1].z, x[k][r][1].w};
        rs[r] = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a[r][e] = to_limb<F16>(v8[e]);
          rs[r] += from_limb<F16>(a[r][e]);
        }
      }
      if (act) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *(uint4*)(ab + (i + r) * V + (sl >> 1) * 16 + (sl & 1) * 8) =
              make_uint4(a[r][0] | ((uint32_t)a[r][1] << 16), a[r][2] | ((uint32_t)a[r][3] << 16),
                         a[r][4] | ((uint32_t)a[r][5] << 16), a[r][6] | ((uint32_t)a[r][7] << 16));
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int j = c0 + (e & 3) + (e >> 2) * 8;
          *(uint2*)&tt[j][i] = make_uint2(a[0][e] | ((uint32_t)a[1][e] << 16), a[2][e] | ((uint32_t)a[3][e] << 16));
        }
      }
      // row sums over the SL lanes of this row group (contiguous, SL | 64)
#pragma unroll
      for (int o = 1; o < SL; o <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) rs[r] += __shfl_xor(rs[r], o);
      if (act && sl == 0)
#pragma unroll
        for (int r = 0; r < 4; ++r) deg[tile * V + i + r] = to_limb<F16>(rs[r]);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < V * V / 8; q += 256) {
      const int i = q / (V / 8), p = (q % (V / 8)) * 8;
      *(uint4*)(at + i * V + p) = *(const uint4*)&tt[i][p];
    }
    return;
  }
  // padded graphs (vin < V): element-wise, Ab's permuted column order
  // (inside every 16-column group the 8-byte chunks 1 and 2 swapped) applied
  // on the store
  for (int q = threadIdx.x; q < V * V; q += 256) {
    const int i = q / V, j = q % V;
    const u16 a = to_limb<F16>((i < vin && j < vin) ? src[i * vin + j] : 0.0f);
    const int jj = (j & ~15) | (((j >> 2) & 3) == 1 ? (j & 3) + 8 : ((j >> 2) & 3) == 2 ? (j & 3) + 4 : (j & 15));
    ab[i * V + jj] = a;
    tt[j][i] = a;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < V * V / 8; q += 256) {
    const int i = q / (V / 8), p = (q % (V / 8)) * 8;
    *(uint4*)(at + i * V + p) = *(const uint4*)&tt[i][p];
  }
  if (threadIdx.x < V) {
    float s = 0.f;
    for (int j = 0; j < V; ++j) s += from_limb<F16>(tt[j][threadIdx.x]);
    deg[tile * V + threadIdx.x] = to_limb<F16>(s);
  }
}

// h0 [b][vin][H] fp32 -> hf [N][H] fp32 (pad rows zero) and optional hb in
// the limb format (bf16, or f16 when f16 != 0).  With dr.thr != 0 the state
// dropout mask of timestep t is applied (backward: dL/dh_T -> dL/dh'_{T-1}).
__global__ void k_pad_state(const float* __restrict__ h0, int vin, int V, int H, float* __restrict__ hf,
                            u16* __restrict__ hb, long N, int f16, Drop dr, int t, const uint32_t* gmax) {
  dr = drop_resolve(dr);  // (a device-resident key: loaded once)
  // one thread per (4-row quad, column): V is a multiple of 4, so a quad lies
  // inside one graph and its 4 state-dropout masks are one Philox block
  const long total = N / 4 * H;
  const float sc = gscale(gmax);  // backward staging of dL/dh_T: the gradient scale (ggnn_common.h)
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const long rq = q / H;
    const int col = (int)(q - rq * H);
    const long row0 = rq * 4, g = row0 / V;
    const int i0 = (int)(row0 - g * V);
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (dr.thr) w = state_words(dr, (int)g, i0, col, t);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u;
      const long e = (row0 + u) * H + col;
      float x = (i < vin) ? h0[(g * vin + i) * H + col] * sc : 0.0f;
      if (dr.thr) x = drop_apply(dr, u4_get(w, u), x);
      if (hf) hf[e] = x;
      if (hb) hb[e] = f16 ? to_limb<true>(x) : to_limb<false>(x);
    }
  }
}

// hf [N][H] fp32 -> out [b][vin][H]
__global__ void k_unpad_state(const float* __restrict__ hf, int vin, int V, int H, float* __restrict__ out, long b,
                              const uint32_t* gmax) {
  const long total = b * vin * (long)H;
  const float sc = gunscale(gmax);  // backward: undo the gradient scale
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const long r = q / H;
    const int col = q % H;
    const long g = r / vin;
    const int i = r % vin;
    out[q] = hf[(g * V + i) * H + col] * sc;
  }
}

// [N][H] fp32 -> [H][N] of element type TO (fp32, or 16-bit limbs: f16 if F16
// else bf16), 64x64 tiles through LDS
template <typename TI, typename TO, bool F16>
__global__ void __launch_bounds__(256) k_transpose(const TI* __restrict__ in, TO* __restrict__ out, long N, int H) {
  __shared__ float t[64][65];
  const long r0 = (long)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  for (int q = threadIdx.x; q < 64 * 64; q += 256) {
    const int i = q / 64, j = q % 64;
    float x = 0.f;
    if (r0 + i < N) {
      if constexpr (std::is_same<TI, float>::value) x = in[(r0 + i) * H + c0 + j];
      else x = from_limb<F16>(in[(r0 + i) * H + c0 + j]);
    }
    t[i][j] = x;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < 64 * 64; q += 256) {
    const int j = q / 64, i = q % 64;
    if (r0 + i < N) {
      if constexpr (std::is_same<TO, float>::value) out[(long)(c0 + j) * N + r0 + i] = t[i][j];
      else out[(long)(c0 + j) * N + r0 + i] = to_limb<F16>(t[i][j]);
    }
  }
}

// d edge_weights under edge dropout: dW[c][i][j] = sum_t mask_t(c,i,j)/keep *
// G[t][c][i][j], G = the per-timestep h_t^T dM_{c,t} from k_wgrad.  One thread
// per 4 consecutive rows i (one Philox draw per timestep).
__global__ void k_edge_mask_reduce(const float* __restrict__ G, float* __restrict__ dW, int C, int H, int T, Drop dr) {
  dr = drop_resolve(dr);  // (a device-resident key: loaded once)
  const long total = (long)C * (H / 4) * H;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int j = q % H;
    const int i0 = (int)((q / H) % (H / 4)) * 4;
    const int c = (int)(q / ((long)H * (H / 4)));
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < T; ++t) {
      const uint4 w = edge_words(dr, c, i0, j, t);
      const float* g = G + (((long)t * C + c) * H + i0) * H + j;
#pragma unroll
      for (int e = 0; e < 4; ++e) s[e] += drop_apply(dr, u4_get(w, e), g[(long)e * H]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) dW[((long)c * H + i0 + e) * H + j] = s[e];
  }
}

// verification: the keep-mask the kernels apply (kind 0: edge [C][H][H] of
// timestep t; kind 1: state [b][vin][H] of timestep t), 1 = kept
__global__ void k_dropout_mask(int kind, int C, int H, int b, int vin, int t, Drop dr, uint8_t* __restrict__ m) {
  dr = drop_resolve(dr);  // (a device-resident key: loaded once)
  const long total = kind == 0 ? (long)C * H * H : (long)b * vin * H;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int k = q % H;
    const long r = q / H;
    uint32_t w;
    if (kind == 0) {
      const int i = r % H, c = (int)(r / H);
      w = u4_get(edge_words(dr, c, i, k, t), i & 3);
    } else {
      const int i = r % vin, g = (int)(r / vin);
      w = u4_get(state_words(dr, g, i, k, t), i & 3);
    }
    m[q] = (dr.thr == 0 || w < dr.thr) ? 1 : 0;
  }
}

// Column sums of row partials in a fixed order (deterministic: no atomics).
// Element e in [0, E) = (ec, ek) = (e / Nc, e % Nc); row (t, w), t < T, w < nw,
// holds it at part[t * sT + w * sW + ec * sC + ek]; a row is skipped where
// mask && !mask[t * mT + ec * mC].  out = (add ? out : 0) + the sum over the
// rows in (t, w) order, columns e < split to out0[e], the others to
// out1[e - split].  Uses: dL/dbeta from k_prop_bwd's per-(timestep, graph)
// partials, dL/dbg and dL/dbc from k_gru_bwd's per-(timestep, workgroup) rows,
// the general path's bias partials, the heads' bias columns.  Two launches:
// k_sum_rows sums row chunk rc of 64 columns per block (4 waves on
// interleaved rows, combined in wave order) into scratch[rc][E];
// k_sum_rows_fin adds the chunks in chunk order.
#define SUMJ_MAX 4
struct SumJob {
  const float* part;
  float* out0;
  float* out1;
  float* scratch;  // [rcs][E]
  const unsigned char* mask;
  const uint32_t* ugmax;  // if set: the sums are multiplied by the gradient unscale (gunscale)
  long sT, sW, sC, mT, mC, E, Nc, split;
  int T, nw, rcs, add;  // rcs: row chunks
};
struct SumJobs {
  SumJob j[SUMJ_MAX];
  int bx[SUMJ_MAX + 1];  // first block of each job (k_sum_rows: colgroups * rcs blocks)
  int fx[SUMJ_MAX + 1];  // first block of each job (k_sum_rows_fin: E / 256 blocks)
  int count;
};
__global__ void __launch_bounds__(256) k_sum_rows(SumJobs js) {
  int ji = 0;
  while (ji + 1 < js.count && js.bx[ji + 1] <= (int)blockIdx.x) ++ji;
  const SumJob& J = js.j[ji];
  const int lb = blockIdx.x - js.bx[ji], cg = lb / J.rcs, rc = lb % J.rcs;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long e = (long)cg * 64 + lane;
  const long rows = (long)J.T * J.nw, per = (rows + J.rcs - 1) / J.rcs;
  const long r0 = rc * per, r1 = min(rows, r0 + per);
  __shared__ float red[4][64];
  float s = 0.f;
  if (e < J.E && r0 + w < r1) {
    const long ec = e / J.Nc, eo = ec * J.sC + e % J.Nc;
    // row r = t * nw + ww walked incrementally (a 64-bit division per row
    // bounded the kernel: 16 us for 26 MB at config 3, round 5)
    int t = (int)((r0 + w) / J.nw), ww = (int)((r0 + w) % J.nw);
#pragma unroll 4
    for (long r = r0 + w; r < r1; r += 4) {
      if (!J.mask || J.mask[t * J.mT + ec * J.mC]) s += J.part[t * J.sT + ww * J.sW + eo];
      ww += 4;
      while (ww >= J.nw) {
        ww -= J.nw;
        ++t;
      }
    }
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && e < J.E) J.scratch[(long)rc * J.E + e] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}
__global__ void __launch_bounds__(256) k_sum_rows_fin(SumJobs js) {
  int ji = 0;
  while (ji + 1 < js.count && js.fx[ji + 1] <= (int)blockIdx.x) ++ji;
  const SumJob& J = js.j[ji];
  const long e = (long)(blockIdx.x - js.fx[ji]) * 256 + threadIdx.x;
  if (e >= J.E) return;
  float s = J.scratch[e];
#pragma unroll 8
  for (int rc = 1; rc < J.rcs; ++rc) s += J.scratch[(long)rc * J.E + e];
  s *= gunscale(J.ugmax);
  float* o = e < J.split ? J.out0 + e : J.out1 + (e - J.split);
  *o = J.add ? *o + s : s;
}

// Training-forward staging of h0 in one pass: h0 [b][vin][H] fp32 -> hf [N][H]
// fp32 (pad rows zero), optional hb (16-bit limbs), and hT [H][N] (16-bit,
// wg_off layout;
// limbs, the weight-gradient operand of timestep 0).  64x64 tiles via LDS.
template <bool F16>
__global__ void __launch_bounds__(256) k_stage_h0(const float* __restrict__ h0, int vin, int V, float* __restrict__ hf,
                                                  u16* __restrict__ hb, u16* __restrict__ hT, long N, int H) {
  __shared__ float t[64][65];
  const long r0 = (long)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  for (int q = threadIdx.x; q < 64 * 16; q += 256) {
    const int i = q / 16, j4 = (q % 16) * 4;
    const long row = r0 + i;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < N) {
      const long g = row / V;
      const int iv = (int)(row % V);
      if (iv < vin) x = *(const float4*)(h0 + (g * vin + iv) * H + c0 + j4);
      *(float4*)(hf + row * H + c0 + j4) = x;
      if (hb) *(uint2*)(hb + row * H + c0 + j4) = make_uint2(pk<F16>(x.x, x.y), pk<F16>(x.z, x.w));
    }
    t[i][j4] = x.x; t[i][j4 + 1] = x.y; t[i][j4 + 2] = x.z; t[i][j4 + 3] = x.w;
  }
  __syncthreads();
  // hT: 8 consecutive node rows of one hidden column are 16 contiguous bytes
  // of the wg_off layout (N % 32 == 0, so a piece is all in or all out)
  for (int q = threadIdx.x; q < 64 * 8; q += 256) {
    const int j = q / 8, i = (q % 8) * 8;
    if (r0 + i < N) {
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = pk<F16>(t[i + 2 * e][j], t[i + 2 * e + 1][j]);
      *(uint4*)(hT + wg_off(c0 + j, r0 + i, H)) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// ---- compact adjacency producer (upload edge lists instead of the
// dense [b][2E][v][v] float64 feed).  Restates graph_to_adj_mat_bd,
// chem_tensorflow_dense.py:65-83, straight into the staged layouts: for every
// edge (src, e, dest) of graph g
//   A[e-1][dest][src] = A[e-1+E][src][dest] = A[E-1][dest][dest-1]
//   = A[2E-1][dest-1][dest] = 1,
// dest-1 = -1 wrapping to v-1 as numpy's negative index does.  Ab / AbT must be
// zeroed first; a cell set twice stays 1.  Edges outside the graph (label not
// in 1..E, node not in 0..v-1) are skipped (the Python layer rejects them).
template <int V, bool F16>
__global__ void k_adj_from_edges(const int* __restrict__ edges, const int* __restrict__ offs, int b, int vin, int E,
                                 u16* __restrict__ Ab, u16* __restrict__ AbT) {
  const u16 one = to_limb<F16>(1.0f);
  const int C = 2 * E;
  const long total = offs[b];
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    // graph of edge q: binary search in the offsets
    int lo = 0, hi = b;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (offs[mid] <= q) lo = mid; else hi = mid;
    }
    const int g = lo;
    const int src = edges[3 * q], e = edges[3 * q + 1], dst = edges[3 * q + 2];
    if (e < 1 || e > E || src < 0 || src >= vin || dst < 0 || dst >= vin) continue;
    const int prev = dst >= 1 ? dst - 1 : vin - 1;
    const int ch[4] = {e - 1, e - 1 + E, E - 1, 2 * E - 1};
    const int ro[4] = {dst, src, dst, prev};
    const int co[4] = {src, dst, prev, dst};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long tile = (long)g * C + ch[k];
      const int i = ro[k], j = co[k];
      const int w = j & 15, p = (j & ~15) + ((w < 4 || w >= 12) ? w : (w < 8) ? w + 4 : w - 4);
      Ab[(tile * V + i) * V + p] = one;   // columns permuted as k_prep_adj writes them
      AbT[(tile * V + j) * V + i] = one;
    }
  }
}

// deg[tile][i] = row sums of the staged adjacency (after k_adj_from_edges)
template <int V, bool F16>
__global__ void __launch_bounds__(V) k_adj_deg(const u16* __restrict__ Ab, u16* __restrict__ deg) {
  const long tile = blockIdx.x;
  const u16* row = Ab + (tile * V + threadIdx.x) * V;
  float s = 0.f;
  for (int j = 0; j < V; j += 8) {
    const uint4 x = *(const uint4*)(row + j);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) s += from_limb<F16>((u16)(w[k] & 0xFFFF)) + from_limb<F16>((u16)(w[k] >> 16));
  }
  deg[tile * V + threadIdx.x] = to_limb<F16>(s);
}

// ---- per-graph list of non-empty channels (about 60 % of
// the 92 real-data channels are empty per graph).  chl[g*(C+1)] = count n,
// chl[g*(C+1) + 1 + i] = i-th channel with an edge, ascending.  A channel is
// empty iff every in-degree is zero (deg holds exact row sums).
#define CHL_MAXC 4096
// Block 0 also writes the identity list [C, 0, 1, .., C-1] at chl_all (the
// dense channel loop, GGNN_DENSE_CHANNELS: read with graph stride 0).
template <int V>
__global__ void __launch_bounds__(256) k_chan_list(const u16* __restrict__ deg, int C, int* __restrict__ chl,
                                                   int* __restrict__ chl_all, unsigned char* __restrict__ occ) {
  __shared__ unsigned char fl[CHL_MAXC];
  const int g = blockIdx.x;
  if (g == 0) {
    for (int c = threadIdx.x; c < C; c += 256) chl_all[1 + c] = c;
    if (threadIdx.x == 0) chl_all[0] = C;
  }
  for (int c = threadIdx.x; c < C; c += 256) {
    const uint4* d = (const uint4*)(deg + ((long)g * C + c) * V);
    uint32_t any = 0;
#pragma unroll
    for (int k = 0; k < V / 8; ++k) {
      const uint4 x = d[k];
      any |= x.x | x.y | x.z | x.w;
    }
    fl[c] = any != 0;
    occ[(long)g * C + c] = any != 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int* out = chl + (long)g * (C + 1);
    int n = 0;
    for (int c = 0; c < C; ++c)
      if (fl[c]) out[1 + n++] = c;
    out[0] = n;
  }
}

// per-channel graph lists cgl[c] = [count, graphs with an edge in channel c
// (ascending)] from the (graph, channel) occupancy k_chan_list writes: the
// weight-gradient kernel sums dW_c over those graphs' rows only.  One wave per
// channel, 64 graphs per ballot.
__global__ void __launch_bounds__(64) k_chan_graphs(const unsigned char* __restrict__ occ, int b, int C,
                                                    int* __restrict__ cgl) {
  const int c = blockIdx.x, lane = threadIdx.x;
  const unsigned long long below = (1ull << lane) - 1;
  int* o = cgl + (long)c * (b + 1);
  int n = 0;
  for (int g0 = 0; g0 < b; g0 += 64) {
    const int g = g0 + lane;
    const bool f = g < b && occ[(long)g * C + c];
    const unsigned long long m = __ballot(f);
    if (f) o[1 + n + __popcll(m & below)] = g;
    n += __popcll(m);
  }
  if (lane == 0) o[0] = n;
}

// ---- all weight packs of one ggnn_pack_weights call in ONE launch: a job
// table of k_pack_B problems (and fp32 copies for the biases); block b runs
// job j with blk_begin[j] <= b < blk_begin[j+1]
#define PACK_MAXJ 24
struct PackJob {
  const float* S;
  u16* out;      // copy jobs: float* destination
  // masked W copies (copy 2 with drop): the timestep's keep bits as well, in
  // the layout of the pair dW product's GemmArgs::mbits (word
  // (c * H + j) * W32 + i / 32, bit i % 32 = keep of W[c][i][j]); nullptr: none
  uint32_t* bits;
  long sS, sO, lo_off, total;  // total: fragment-lanes (pack) or elements (copy)
  int ldS, K, N, trans, t, drop, copy;
  // f8 = 1: the lo part holds the fp8 correction fragments of mfma_f8corr (ggnn_common.h)
  // instead of f16 lo limbs: [strip][32-k block][64 lanes][32 bytes], lane half 0
  // e4m3(b_lo 2^(F8_Q+F8_M)), half 1 e4m3(b_hi 2^F8_Q) (the same bytes as the limbs;
  // k_prop_bwd).  f8 = 2: [strip][64-k block][64 lanes][32 bytes] of e4m3(b_lo
  // 2^(F8_Q+F8_M)), byte j of lane half hh = k 64 kb + 32 hh + j (half the bytes;
  // k_gru_bwd)
  int f8;
};
struct PackJobs {
  PackJob j[PACK_MAXJ];
  int blk_begin[PACK_MAXJ + 1];
  int count;
  Drop dr;
  // ggnn_pack_weights_batch: per-channel occupancy of the staged batch; the
  // masked fp32 copies (general path, edge dropout) skip channels nobody uses
  const unsigned char* chocc;
};

// chocc[c] = 1 iff some graph of the staged batch has an edge in channel c
// (occ: the general path's [b][C] tile occupancy)
__global__ void __launch_bounds__(256) k_chan_any(const unsigned char* __restrict__ occ, int b, int C,
                                                  unsigned char* __restrict__ chocc) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  unsigned char f = 0;
  for (int g = 0; g < b && !f; ++g) f = occ[(long)g * C + c];
  chocc[c] = f;
}
template <bool F16>
__global__ void __launch_bounds__(256) k_pack_multi(PackJobs a) {
  const Drop dr = drop_resolve(a.dr);  // (a device-resident key: loaded once)
  int ji = 0;
  while (ji + 1 < a.count && a.blk_begin[ji + 1] <= (int)blockIdx.x) ++ji;
  const PackJob& J = a.j[ji];
  const long q = (long)(blockIdx.x - a.blk_begin[ji]) * 256 + threadIdx.x;
  if (q >= J.total) return;
  if (J.copy == 1) {  // fp32 copy (zeros when S is null)
    ((float*)J.out)[q] = J.S ? J.S[q] : 0.0f;
    return;
  }
  if (J.copy == 2) {  // fp32 copy of W [C][H][H] (H = J.K), edge-dropout mask of timestep J.t when J.drop
    if (J.trans) {
      // 16-byte pieces (the host sets trans when H % 4 == 0 and both ends are
      // 16-byte aligned): unmasked, J.total = C*H*H/4 float4s; masked, one
      // thread per 32-row block of 4 columns (J.total = C*W32*(H/4)), walking
      // its 8 row quads with the same Philox block per (c, row quad, column)
      // as the scalar form, and storing the block's keep bits (4 words)
      if (!J.drop) {
        ((float4*)J.out)[q] = ((const float4*)J.S)[q];
        return;
      }
      const int H = J.K, h4 = H >> 2, W32 = (H + 31) >> 5;
      const int j4 = (int)(q % h4), w = (int)((q / h4) % W32), c = (int)(q / ((long)h4 * W32));
      if (a.chocc && !a.chocc[c]) return;  // a channel the staged batch does not use
      uint32_t wb[4] = {0u, 0u, 0u, 0u};
      for (int iq = 8 * w; iq < min(8 * w + 8, h4); ++iq) {
        const long e0 = ((long)c * H + 4 * iq) * H + 4 * j4;
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *(const float4*)(J.S + e0 + (long)u * H);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint4 x = edge_words(dr, c, 4 * iq, 4 * j4 + k, J.t);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            float* y = (float*)&v[u] + k;
            *y = drop_apply(dr, u4_get(x, u), *y);
            wb[k] |= (uint32_t)(u4_get(x, u) < dr.thr) << (4 * (iq - 8 * w) + u);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) *(float4*)((float*)J.out + e0 + (long)u * H) = v[u];
      }
      if (J.bits)
#pragma unroll
        for (int k = 0; k < 4; ++k) J.bits[((long)c * H + 4 * j4 + k) * W32 + w] = wb[k];
      return;
    }
    if (!J.drop) {
      ((float*)J.out)[q] = J.S[q];
      return;
    }
    // masked: one thread per 32-row block of one column (J.total = C*W32*H),
    // its row quads' 4 masks the 4 words of one Philox block each (the last
    // quad of a W_c is partial when H % 4 != 0)
    const int H = J.K, hq = (H + 3) >> 2, W32 = (H + 31) >> 5;
    const int wj = (int)(q % H), w = (int)((q / H) % W32), c = (int)(q / ((long)H * W32));
    if (a.chocc && !a.chocc[c]) return;
    uint32_t wb = 0u;
    for (int iq = 8 * w; iq < min(8 * w + 8, hq); ++iq) {
      const uint4 x = edge_words(dr, c, 4 * iq, wj, J.t);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (4 * iq + u >= H) break;
        const long e = ((long)c * H + 4 * iq + u) * H + wj;
        ((float*)J.out)[e] = drop_apply(dr, u4_get(x, u), J.S[e]);
        wb |= (uint32_t)(u4_get(x, u) < dr.thr) << (4 * (iq - 8 * w) + u);
      }
    }
    if (J.bits) J.bits[((long)c * H + wj) * W32 + w] = wb;
    return;
  }
  const int per = (J.N / 32) * (J.K / 16) * 64;  // fragment-lanes per matrix
  const int mat = (int)(q / per), r = (int)(q % per);
  const float* Sb = J.S + J.sS * mat;
  u16* ob = J.out + J.sO * mat;
  const int lane = r & 63, fi = r >> 6;
  const int nks = J.K / 16;
  const int ks = fi % nks, strip = fi / nks;
  const int n = strip * 32 + (lane & 31), k0 = ks * 16 + 8 * (lane >> 5);
  float x[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = J.trans ? Sb[(long)n * J.ldS + k0 + e] : Sb[(long)(k0 + e) * J.ldS + n];
  if (J.drop) {
    if (!J.trans) {  // rows k0 .. k0 + 7 of column n: two quads, two Philox blocks
      const uint4 w0 = edge_words(dr, mat, k0, n, J.t), w1 = edge_words(dr, mat, k0 + 4, n, J.t);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = drop_apply(dr, u4_get(e < 4 ? w0 : w1, e & 3), x[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        x[e] = drop_apply(dr, u4_get(edge_words(dr, mat, n, k0 + e, J.t), n & 3), x[e]);
    }
  }
  *(uint4*)(ob + (size_t)r * 8) = pk8<F16>(x);
  if (J.f8 == 2) {
    // k_gru_bwd's fp8 lo fragments: e4m3(b_lo 2^(F8_Q+F8_M)); this thread's 8 k's
    // (k0 .. k0 + 7) are bytes (k0 & 31) .. + 7 of lane (col) + 32 ((k0 & 63) >> 5)
    // of 64-k block k0 >> 6
    float lo[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float h = (float)(_Float16)x[e];
      lo[e] = fminf(fmaxf((x[e] - h) * (float)(1 << (F8_Q + F8_M)), -448.0f), 448.0f);
    }
    char* f8 = (char*)(ob + J.lo_off) +
               ((size_t)(strip * (nks / 4) + (k0 >> 6)) * 64 + (lane & 31) + 32 * ((k0 & 63) >> 5)) * 32 + (k0 & 31);
    *(uint2*)f8 = make_uint2(pk4_fp8(lo[0], lo[1], lo[2], lo[3]), pk4_fp8(lo[4], lo[5], lo[6], lo[7]));
    return;
  }
  if (J.f8) {
    // this thread's 8 k's (k0 .. k0 + 7 = 32 kb + 16 (ks & 1) + 8 (lane >> 5) + e)
    // go to bytes 16 (ks & 1) + 8 (lane >> 5) + e of lane (col) [lo] and lane
    // (col) + 32 [hi] of block kb's fragment
    float lo[8], hi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float h = (float)(_Float16)x[e];
      const float cl = 448.0f;
      lo[e] = fminf(fmaxf((x[e] - h) * (float)(1 << (F8_Q + F8_M)), -cl), cl);
      hi[e] = fminf(fmaxf(h * (float)(1 << F8_Q), -cl), cl);
    }
    const int kb = ks >> 1, byte = 16 * (ks & 1) + 8 * (lane >> 5);
    char* f8 = (char*)(ob + J.lo_off) + ((size_t)(strip * (nks / 2) + kb) * 64 + (lane & 31)) * 32 + byte;
    *(uint2*)f8 = make_uint2(pk4_fp8(lo[0], lo[1], lo[2], lo[3]), pk4_fp8(lo[4], lo[5], lo[6], lo[7]));
    *(uint2*)(f8 + 32 * 32) = make_uint2(pk4_fp8(hi[0], hi[1], hi[2], hi[3]), pk4_fp8(hi[4], hi[5], hi[6], hi[7]));
    return;
  }
  *(uint4*)(ob + J.lo_off + (size_t)r * 8) = pk8_lo<F16>(x);
}

// ---- zero the backward's gradient accumulators in one launch (they are
// accumulated by atomics / per-step adds), instead of one hipMemsetAsync per
// buffer (each a separate ~5 us fill dispatch).  blockIdx.y = buffer.
// byte fill / fp32 copy as kernels rather than hipMemsetAsync / hipMemcpyAsync:
// a step captured into a hipGraph then holds kernel nodes only (memset nodes
// captured from a stream were seen to race with their neighbouring kernels on
// replay).  k_fill: n bytes of `byte` at p (any alignment; 16-byte pieces over
// the aligned middle, single bytes at the ends)
__device__ __forceinline__ void fill_bytes(unsigned char* __restrict__ p, size_t n, unsigned byte) {
  const size_t mis = (size_t)((16 - ((uintptr_t)p & 15)) & 15);
  const size_t head = mis < n ? mis : n;
  const size_t body = (n - head) & ~(size_t)15;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
  const unsigned w = byte * 0x01010101u;
  const uint4 v = make_uint4(w, w, w, w);
  uint4* q = (uint4*)(p + head);
  for (size_t i = tid; i < body / 16; i += st) q[i] = v;
  if (tid < head) p[tid] = (unsigned char)byte;
  const size_t t0 = head + body;
  if (tid < n - t0) p[t0 + tid] = (unsigned char)byte;
}
__global__ void __launch_bounds__(256) k_fill(unsigned char* __restrict__ p, size_t n, unsigned byte) {
  fill_bytes(p, n, byte);
}
// several fills in one launch (blockIdx.y = fill): the staging of one batch
// clears up to five buffers, each a ~5 us launch on its own
#define FILL_MAXJ 8
struct FillJobs {
  unsigned char* p[FILL_MAXJ];
  size_t n[FILL_MAXJ];
  unsigned byte[FILL_MAXJ];
};
__global__ void __launch_bounds__(256) k_fill_multi(FillJobs f) {
  fill_bytes(f.p[blockIdx.y], f.n[blockIdx.y], f.byte[blockIdx.y]);
}
// dst[0, n) = src[0, n), fp32 (16-byte pieces when both are 16-byte aligned)
__global__ void __launch_bounds__(256) k_copy32(float* __restrict__ dst, const float* __restrict__ src, long n) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x, st = (long)gridDim.x * blockDim.x;
  long i = tid;
  if (((((uintptr_t)dst) | ((uintptr_t)src)) & 15) == 0) {
    for (; 4 * i + 3 < n; i += st) *(float4*)(dst + 4 * i) = *(const float4*)(src + 4 * i);
    i = (n & ~3L) + tid;
  }
  for (; i < n; i += st) dst[i] = src[i];
}

#define ZERO_MAXJ 16
struct ZeroJobs {
  float* p[ZERO_MAXJ];
  long n[ZERO_MAXJ];  // floats
};
__global__ void __launch_bounds__(256) k_zero_multi(ZeroJobs a) {
  float* p = a.p[blockIdx.y];
  const long n = a.n[blockIdx.y];
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  if ((((unsigned long)p) & 15) == 0) {
    for (; 4 * i + 3 < n; i += stride) *(float4*)(p + 4 * i) = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long k = (n & ~3L) + (long)blockIdx.x * 256 + threadIdx.x; k < n; k += stride) p[k] = 0.f;
  } else {
    for (; i < n; i += stride) p[i] = 0.f;
  }
}

// ---- max |x| over n floats into *gmax (as bits): the backward's gradient
// scale (gscale, ggnn_common.h).  Two launches, no atomics: ABSMAX_BLOCKS
// blocks store their maxima, one block takes the max of those.  (One
// same-address atomicMax per block -- device-scope atomics on one line are
// serialised past the XCDs' L2s -- plus the zeroing of *gmax took 21.5 + 4.2
// us per config-3 backward for 33 MB, round 5.)
#define ABSMAX_BLOCKS 256
#define ABSMAX_THREADS 1024
__global__ void __launch_bounds__(ABSMAX_THREADS) k_absmax(const float* __restrict__ x, long n, float* __restrict__ part) {
  float m = 0.0f;
  const long stride = (long)gridDim.x * ABSMAX_THREADS;
  long i = (long)blockIdx.x * ABSMAX_THREADS + threadIdx.x;
  if ((((unsigned long)x) & 15) == 0) {
    // four independent 16-byte loads in flight per thread, then the rest
    for (; 4 * (i + 3 * stride) + 3 < n; i += 4 * stride) {
      float4 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = *(const float4*)(x + 4 * (i + u * stride));
#pragma unroll
      for (int u = 0; u < 4; ++u)
        m = fmaxf(m, fmaxf(fmaxf(fabsf(a[u].x), fabsf(a[u].y)), fmaxf(fabsf(a[u].z), fabsf(a[u].w))));
    }
    for (; 4 * i + 3 < n; i += stride) {
      const float4 a = *(const float4*)(x + 4 * i);
      m = fmaxf(m, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
    }
    for (long k = (n & ~3L) + (long)blockIdx.x * ABSMAX_THREADS + threadIdx.x; k < n; k += stride) m = fmaxf(m, fabsf(x[k]));
  } else {
    for (; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  }
  // (fmaxf drops NaN; an inf stays inf and disables the scaling)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float wm[ABSMAX_THREADS / 64];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < ABSMAX_THREADS / 64; ++w) m = fmaxf(m, wm[w]);
    part[blockIdx.x] = m;
  }
}
__global__ void __launch_bounds__(64) k_absmax_fin(const float* __restrict__ part, int nb, uint32_t* __restrict__ gmax) {
  float m = 0.0f;
  for (int i = threadIdx.x; i < nb; i += 64) m = fmaxf(m, part[i]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (threadIdx.x == 0) *gmax = __float_as_uint(m);
}

