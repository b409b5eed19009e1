// k_generic.h -- the element-wise and staging kernels of the general path
// (any hidden size, any vertex count; k_gemm.h does the products).  fp32
// activations, rows = b*v unpadded (row g*v + i = node i of graph g).
//
// Reference (chem_tensorflow_dense.py): the T-loop :312-340, the fast step
// :391-437, the TF1 GRUCell (reset before the matmul, [x, h] concat, r then u)
// + DropoutWrapper state dropout :237-241, :333; adjacency :65-83.
#pragma once
#include "ggnn_common.h"

// ---- adjacency staging: A [b][C][v][v] fp32 (0/1) -> Ag [b][C][v][vp] 16-bit
// limbs (natural order, row pitch vp = v rounded up to 8, zero padding), its
// transpose AgT (same layout: the k-contiguous A operand of dM = A^T dX) and
// the per-tile occupancy occ[b*C] (1 = the tile holds an edge).  One block
// per tile.
template <bool F16>
__global__ void __launch_bounds__(256) k_gen_adj(const float* __restrict__ A, int v, int vp, u16* __restrict__ Ag,
                                                 u16* __restrict__ AgT, unsigned char* __restrict__ occ) {
  const long tile = blockIdx.x;
  const float* src = A + tile * (long)v * v;
  u16* dst = Ag + tile * (long)v * vp;
  u16* dsT = AgT + tile * (long)v * vp;
  int any = 0;
  for (long q = threadIdx.x; q < (long)v * vp; q += 256) {
    const int i = (int)(q / vp), j = (int)(q % vp);
    const float x = j < v ? src[(long)i * v + j] : 0.f;
    any |= x != 0.f;
    dst[q] = to_limb<F16>(x);
    if (j < v) dsT[(long)j * vp + i] = to_limb<F16>(x);
    else dsT[q] = 0;  // (row i of AgT, padding column j)
  }
  any = __syncthreads_or(any);
  if (threadIdx.x == 0) occ[tile] = (unsigned char)(any != 0);
}

// the same from the reference's edge lists (graph_to_adj_mat_bd semantics,
// k_prep.h k_adj_from_edges): after a memset of Ag, AgT and occ
__global__ void __launch_bounds__(256) k_gen_adj_edges(const int* __restrict__ edges, const int* __restrict__ goff,
                                                       int b, int v, int vp, int E, int f16, u16* __restrict__ Ag,
                                                       u16* __restrict__ AgT, unsigned char* __restrict__ occ) {
  const int C = 2 * E;
  const u16 one = f16 ? (u16)0x3C00 : (u16)0x3F80;
  for (int g = blockIdx.x; g < b; g += gridDim.x) {
    for (int e = goff[g] + threadIdx.x; e < goff[g + 1]; e += 256) {
      const int src = edges[3 * e], lab = edges[3 * e + 1], dst = edges[3 * e + 2];
      if (lab < 1 || lab > E || src < 0 || src >= v || dst < 0 || dst >= v) continue;
      const int prv = dst - 1 < 0 ? v - 1 : dst - 1;  // numpy's wrap of index -1
      const int ch[4] = {lab - 1, lab - 1 + E, E - 1, 2 * E - 1};
      const int ro[4] = {dst, src, dst, prv};
      const int co[4] = {src, dst, prv, dst};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const long tile = (long)g * C + ch[k];
        Ag[(tile * v + ro[k]) * vp + co[k]] = one;
        AgT[(tile * v + co[k]) * vp + ro[k]] = one;
        occ[tile] = 1;
      }
    }
  }
}

// per-graph channel lists chl[g*(C+1)] = (count, channels...) and per-channel
// graph lists cgl[c*(b+1)] = (count, graphs...) from occ (and cut into chunks, cgc); with dense != 0
// every tile counts as occupied (GGNN_DENSE_CHANNELS).  One wave per list,
// compacted 64 entries at a time by ballots (ascending order)
__global__ void __launch_bounds__(256) k_gen_lists(const unsigned char* __restrict__ occ, int b, int C, int dense,
                                                   int* __restrict__ chl, int* __restrict__ cgl, int* __restrict__ cgc,
                                                   int nch, int gch) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const unsigned long long below = (1ull << lane) - 1ull;
  if (t < b) {
    int* o = chl + (long)t * (C + 1);
    int n = 0;
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + lane;
      const bool f = c < C && (dense || occ[(long)t * C + c]);
      const unsigned long long m = __ballot(f);
      if (f) o[1 + n + __popcll(m & below)] = c;
      n += __popcll(m);
    }
    if (lane == 0) o[0] = n;
  } else if (t < b + C) {
    const int c = t - b;
    int* o = cgl + (long)c * (b + 1);
    int* q = cgc + (long)c * nch * (gch + 1);
    int n = 0;
    for (int g0 = 0; g0 < b; g0 += 64) {
      const int g = g0 + lane;
      const bool f = g < b && (dense || occ[(long)g * C + c]);
      const unsigned long long m = __ballot(f);
      if (f) {
        const int idx = n + __popcll(m & below);
        o[1 + idx] = g;
        // the same list in nch chunks of <= gch graphs: cgc[(c*nch + j)*(gch+1)] = (count, graphs...)
        q[(long)(idx / gch) * (gch + 1) + 1 + idx % gch] = g;
      }
      n += __popcll(m);
    }
    if (lane == 0) o[0] = n;
    for (int j = lane; j < nch; j += 64) q[(long)j * (gch + 1)] = max(0, min(n - j * gch, gch));
  }
}

// ---- edge-weight dropout (the fast path's Philox counter: (i>>2, j, c, t),
// word i&3): one thread per (channel, row quad, column), the quad's 4 masks
// being the words of one Philox block.
// dW[c][i][j] += mask_t / keep * G[c][i][j]   (edge dropout backward, one timestep)
__global__ void k_gen_wmask_acc(const float* __restrict__ G, float* __restrict__ dW, int C, int H, int t, Drop dr) {
  dr = drop_resolve(dr);  // (a device-resident key: loaded once)
  const int HQ = (H + 3) / 4;
  const long total = (long)C * HQ * H;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int j = (int)(e % H), i0 = 4 * (int)((e / H) % HQ), c = (int)(e / ((long)HQ * H));
    const uint4 w = edge_words(dr, c, i0, j, t);
    for (int q = 0; q < 4 && i0 + q < H; ++q) {
      const long o = ((long)c * H + i0 + q) * H + j;
      dW[o] += drop_apply(dr, u4_get(w, q), G[o]);
    }
  }
}

// ---- forward element-wise steps (G = sigmoid gates [N][2H] = (r | u))
// rh = r * h
__global__ void k_gen_rh(const float* __restrict__ G, const float* __restrict__ h, float* __restrict__ rh, long N,
                         int H) {
  const long total = N * H;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long row = e / H;
    const int k = (int)(e % H);
    rh[e] = G[row * 2 * H + k] * h[e];
  }
}
// State-dropout element-wise kernels: one thread per (graph, row quad,
// column) -- rows unpadded (v = vin), so a graph's last quad may be partial --
// drawing the quad's 4 masks as one Philox block (counter (i >> 2, k, g, t),
// word i & 3), with one division pair per 4 elements.
struct QuadIdx {
  long row0;  // first row of the quad
  int g, i0, k, nr;  // graph, first node, column, rows in the quad
};
DEV bool quad_idx(long q, int H, int v, long b, QuadIdx& x) {
  const int vq = (v + 3) >> 2;
  if (q >= b * vq * H) return false;
  const long r = q / H;
  x.k = (int)(q - r * H);
  x.g = (int)(r / vq);
  x.i0 = (int)(r - (long)x.g * vq) * 4;
  x.nr = min(4, v - x.i0);
  x.row0 = (long)x.g * v + x.i0;
  return true;
}
// h' = u h + (1 - u) c, then the DropoutWrapper state dropout of timestep t
__global__ void k_gen_blend(const float* __restrict__ G, const float* __restrict__ h, const float* __restrict__ cc,
                            float* __restrict__ hout, long N, int H, int v, Drop sd, int t) {
  sd = drop_resolve(sd);  // (a device-resident key: loaded once)
  const long b = N / v, total = b * ((v + 3) >> 2) * H;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    QuadIdx x;
    quad_idx(q, H, v, b, x);
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (sd.thr) w = state_words(sd, x.g, x.i0, x.k, t);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u >= x.nr) break;
      const long row = x.row0 + u, e = row * H + x.k;
      const float ug = G[row * 2 * H + H + x.k];
      float y = gru_blend(ug, h[e], cc[e]);
      if (sd.thr) y = drop_apply(sd, u4_get(w, u), y);
      hout[e] = y;
    }
  }
}

// ---- backward element-wise steps, timestep t (Appendix A of SURVEY.md):
// e1: dc = d(1-u); du = d(h-c); dzc = dc(1-c^2); dzg_u = du u(1-u);
//     dh (second half of the [N][2H] buffer DXH) = d u
// with the step's delta d formed on the fly (round 5: no k_gen_delta /
// k_gen_delta0 launch in front of it): d = din[row * ldin + k] * gscale(gmax)
// through the state dropout of timestep tm (tm < 0: none) -- din = dL/dh_T
// (ldin H, the gradient scale) at the last timestep, else the second half of
// DXH (ldin 2H, the dh the step after left there, read before this thread
// overwrites it)
__global__ void __launch_bounds__(256) k_gen_bwd1(const float* din, long ldin, const uint32_t* __restrict__ gmax,
                                                  Drop sd, int tm, int v, const float* __restrict__ G,
                                                  const float* __restrict__ h, const float* __restrict__ cc,
                                                  float* __restrict__ dzc, float* __restrict__ dzg,
                                                  float* DXH, long N, int H, float* __restrict__ bpart) {
  // grid (column blocks, row slices): column k per thread, the slice's rows in
  // turn; the bias gradients' slice partials sum dzg_u, sum dzc go to the
  // slice's row of bpart ([slices][dbg_r | dbg_u | dbc], summed in a fixed
  // order after the backward: k_sum_rows)
  sd = drop_resolve(sd);  // (a device-resident key: loaded once)
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H) return;
  const long per = (N + gridDim.y - 1) / gridDim.y, r0 = blockIdx.y * per, r1 = min(N, r0 + per);
  const float dsc = gscale(gmax);
  const bool drop = sd.thr && tm >= 0;
  float sc = 0.f, su = 0.f;
  uint4 w = make_uint4(0u, 0u, 0u, 0u);
  int gi = (int)(r0 / v), ii = (int)(r0 - (long)gi * v);  // graph and node of the current row
  if (drop && r0 < r1) w = state_words(sd, gi, ii & ~3, k, tm);
  for (long row = r0; row < r1; ++row) {
    if (drop && (ii & 3) == 0 && row != r0) w = state_words(sd, gi, ii, k, tm);  // a new row quad
    const long e = row * H + k, g2 = row * 2 * H + H + k;
    float dl = din[row * ldin + k] * dsc;
    if (drop) dl = drop_apply(sd, u4_get(w, ii & 3), dl);
    if (++ii == v) { ii = 0; ++gi; }
    const float u = G[g2], c = cc[e];
    const float zc = dl * (1.0f - u) * (1.0f - c * c), zu = dl * (h[e] - c) * u * (1.0f - u);
    dzc[e] = zc;
    dzg[g2] = zu;
    DXH[g2] = dl * u;
    sc += zc;
    su += zu;
  }
  bpart[(long)blockIdx.y * 3 * H + H + k] = su;
  bpart[(long)blockIdx.y * 3 * H + 2 * H + k] = sc;
}
// e2: d(rh) -> dr = d(rh) h, dzg_r = dr r(1-r); dh += d(rh) r; dbg[:H] += sum dzg_r
__global__ void __launch_bounds__(256) k_gen_bwd2(const float* __restrict__ drh, const float* __restrict__ G,
                                                  const float* __restrict__ h, float* __restrict__ dzg,
                                                  float* __restrict__ DXH, long N, int H, float* __restrict__ bpart) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H) return;
  const long per = (N + gridDim.y - 1) / gridDim.y, r0 = blockIdx.y * per, r1 = min(N, r0 + per);
  float sr = 0.f;
#pragma unroll 4
  for (long row = r0; row < r1; ++row) {
    const long e = row * H + k;
    const float r = G[row * 2 * H + k], x = drh[e];
    const float zr = gru_dzg_r(x, h[e], r);
    dzg[row * 2 * H + k] = zr;
    DXH[row * 2 * H + H + k] = __builtin_fmaf(x, r, DXH[row * 2 * H + H + k]);
    sr += zr;
  }
  bpart[(long)blockIdx.y * 3 * H + k] = sr;
}
// dL/dh_t (second half of DXH) -> the next (earlier) step's delta: the state
// dropout backward of timestep tm = t-1 (tm < 0: none), times osc (the
// gradient unscale on the last step, else 1)
__global__ void k_gen_delta(const float* __restrict__ DXH, float* __restrict__ out, long N, int H, int v, Drop sd,
                            int tm, const uint32_t* __restrict__ gmax, int unscale) {
  sd = drop_resolve(sd);  // (a device-resident key: loaded once)
  const long b = N / v, total = b * ((v + 3) >> 2) * H;
  const float osc = unscale ? gunscale(gmax) : 1.0f;
  const bool drop = sd.thr && tm >= 0;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    QuadIdx x;
    quad_idx(q, H, v, b, x);
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (drop) w = state_words(sd, x.g, x.i0, x.k, tm);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u >= x.nr) break;
      const long row = x.row0 + u;
      float y = DXH[row * 2 * H + H + x.k] * osc;
      if (drop) y = drop_apply(sd, u4_get(w, u), y);
      out[row * H + x.k] = y;
    }
  }
}
// dL/dh_T staging: delta = S * dL/dh_T (gradient scale), state dropout of T-1
__global__ void k_gen_delta0(const float* __restrict__ dhT, float* __restrict__ out, long N, int H, int v, Drop sd,
                             int tm, const uint32_t* __restrict__ gmax) {
  sd = drop_resolve(sd);  // (a device-resident key: loaded once)
  const long b = N / v, total = b * ((v + 3) >> 2) * H;
  const float sc = gscale(gmax);
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    QuadIdx x;
    quad_idx(q, H, v, b, x);
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (sd.thr) w = state_words(sd, x.g, x.i0, x.k, tm);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u >= x.nr) break;
      const long e = (x.row0 + u) * H + x.k;
      float y = dhT[e] * sc;
      if (sd.thr) y = drop_apply(sd, u4_get(w, u), y);
      out[e] = y;
    }
  }
}
