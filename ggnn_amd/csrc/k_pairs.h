// k_pairs.h -- the general path's sparse message passing ("pair mode",
// GGNN_SPARSE_PAIRS) for adjacency with few edges per node, e.g. the
// reference's dependency trees (C = 92 channels, ~0.1 % density, ~4
// (node, channel) pairs with an incoming edge per node).
//
// The reference contracts X[g,i] = sum_c sum_j A[g,c,i,j] (h[g,j] W_c + beta_c)
// (chem_tensorflow_dense.py:391-437).  The dense tile path computes
// M[g,c] = h[g] W_c for EVERY row of every non-empty (graph, channel) tile
// (~26 tiles x v rows per sentence graph), then the adjacency product.  Pair
// mode re-associates the same sum as
//   X[g,i] = sum over pairs p = (g,i,c) with deg_p = sum_j A[g,c,i,j] > 0 of
//            Y_p W_c + deg_p beta_c,          Y_p = sum_j A[g,c,i,j] h[g,j]
// so the message transform runs over the ~4 pair rows per node instead of
// ~26 tile rows, and W_c streams once per 32 pair rows of channel c.
//
// Pair rows are grouped by channel, each channel's range padded to a multiple
// of PAIR_TILE rows, so a 32-row product tile has ONE channel: the products
// are ordinary k_gemm_ring launches whose z = tile carries its channel as a
// one-entry term list (ptile).  Built once per staged batch on the device
// (k_pair_degree / _scan / _layout / _fill); every sum is in a fixed order, so
// the results are deterministic.  Backward (same
// decomposition): dXg_p = dX[row_p]; dY = dXg W_c^T; dh[g,j] += sum over pairs
// with A[g,c,i,j] = 1 of dY_p; dW_c += Y_c^T dXg_c (split-K over chunks of
// pair_chunk() tiles, the edge-dropout mask applied in the product's epilogue);
// dbeta_c += sum_p deg_p dXg_p.
#pragma once
#include "ggnn_common.h"

#define PAIR_TILE 32   // rows per product tile (the ring kernel's 32-row variant)
// tiles per split-K term list of the dW product: 4 (128 rows) at small
// batches, 16 (512 rows) at large ones (pair_chunk).  16 was the atomic-era
// choice everywhere; with slab partials a shorter list caps the longest
// workgroup's walk at the 20-sentence batch (its busiest channel: 64 -> 16
// slices; with the ring's lean epilogue the product went 159 -> 105 us,
// tools/ts_probe_generic.py), while at b = 256 the 4x more slab partials cost
// more than the walk saves (wgrad 0.958 vs 1.038 ms per step, round 5)
HDI int pair_chunk(int cap_tiles) { return cap_tiles <= 512 ? 4 : 16; }

// S1: in-degree per (channel, node row) from the staged 16-bit rows (0/1
// limbs: nonzero bits <=> 1); one block per (graph, channel) tile, a wave per row
__global__ void __launch_bounds__(256) k_pair_degree(const u16* __restrict__ Ag, const unsigned char* __restrict__ occ,
                                                     int b, int C, int v, int vp, u16* __restrict__ degc) {
  const int tile = blockIdx.x, g = tile / C, c = tile - g * C;
  const long N = (long)b * v;
  u16* out = degc + (long)c * N + (long)g * v;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  if (!occ[tile]) {
    for (int i = tid; i < v; i += 256) out[i] = 0;
    return;
  }
  for (int i = w; i < v; i += 4) {
    const u16* row = Ag + ((long)tile * v + i) * vp;
    int cnt = 0;
    for (int j = lane; j < vp; j += 64) cnt += row[j] != 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (lane == 0) out[i] = (u16)cnt;
  }
}

// S2: per channel (one block), the position of every node row with an
// incoming edge among the channel's pair rows (ascending node order), -1
// elsewhere; pcnt[c] = the channel's pair count
__global__ void __launch_bounds__(1024) k_pair_scan(const u16* __restrict__ degc, long N, int* __restrict__ pidx,
                                                    int* __restrict__ pcnt) {
  const int c = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const u16* d = degc + (long)c * N;
  int* o = pidx + (long)c * N;
  __shared__ int wsum[16];
  int base = 0;
  for (long r0 = 0; r0 < N; r0 += 1024) {
    const long r = r0 + tid;
    const int f = r < N && d[r] != 0;
    const unsigned long long m = __ballot(f);
    const int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int woff = 0, tot = 0;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      woff += u < w ? wsum[u] : 0;
      tot += wsum[u];
    }
    if (r < N) o[r] = f ? base + woff + pre : -1;
    base += tot;
    __syncthreads();  // wsum is rewritten by the next chunk
  }
  if (tid == 0) pcnt[c] = base;
}

// S3: channel offsets (padded to PAIR_TILE), the per-tile term lists of the
// products (ptile[2z] = 1 live / 0 dead, ptile[2z+1] = channel; pmask), and the
// dW product's split-K chunks (wtl[z*(1+chunk)] = tile count, then the
// tile indices; wmap[z] = channel; wmask: 1 live, 2 live and its channel's
// only chunk, whose dW tiles are then stored instead of added atomically:
// fp32 atomics bound the dW product at small batches, ~65 G adds/s).  One block.
__global__ void __launch_bounds__(1024) k_pair_layout(const int* __restrict__ pcnt, int C, int cap_tiles, int zw_cap,
                                                      int chunk,
                                                      int* __restrict__ poff, int* __restrict__ ptile,
                                                      unsigned char* __restrict__ pmask, int* __restrict__ wtl,
                                                      int* __restrict__ wmap, unsigned char* __restrict__ wmask,
                                                      int* __restrict__ wst) {
  __shared__ int soff[CHL_MAXC + 1], cst[CHL_MAXC + 1];
  const int tid = threadIdx.x;
  if (tid == 0) {
    int off = 0, ch = 0;
    for (int c = 0; c < C; ++c) {
      soff[c] = off;
      cst[c] = ch;
      const int t = (pcnt[c] + PAIR_TILE - 1) / PAIR_TILE;
      off += t * PAIR_TILE;
      ch += (t + chunk - 1) / chunk;
    }
    soff[C] = off;
    cst[C] = ch;
  }
  __syncthreads();
  for (int c = tid; c <= C; c += blockDim.x) {
    poff[c] = soff[c];
    wst[c] = cst[c];  // channel c's dW chunks: [wst[c], wst[c+1]) (k_slab_reduce)
  }
  const int live_tiles = soff[C] / PAIR_TILE;
  // the channel of a tile / chunk: the last c with start <= x (binary search)
  auto find = [&](const int* st, int x) {
    int lo = 0, hi = C - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (st[mid] <= x) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  for (int z = tid; z < cap_tiles; z += blockDim.x) {
    const bool live = z < live_tiles;
    ptile[2 * z] = live ? 1 : 0;
    ptile[2 * z + 1] = live ? find(soff, z * PAIR_TILE) : 0;
    pmask[z] = live ? 1 : 0;
  }
  for (int z = tid; z < zw_cap; z += blockDim.x) {
    int* q = wtl + (long)z * (1 + chunk);
    if (z < cst[C]) {
      const int c = find(cst, z), j = z - cst[c];
      const int t0 = soff[c] / PAIR_TILE, nt = (soff[c + 1] - soff[c]) / PAIR_TILE;
      const int cnt = min(chunk, nt - j * chunk);
      q[0] = cnt;
      for (int e = 0; e < cnt; ++e) q[1 + e] = t0 + j * chunk + e;
      wmap[z] = c;
      wmask[z] = cst[c + 1] - cst[c] == 1 ? 2 : 1;  // 2: the channel's only chunk (k_gemm_ring stores)
    } else {
      q[0] = 0;
      wmap[z] = 0;
      wmask[z] = 0;
    }
  }
}

// S4: pair rows: prow[p] = node row, pdeg[p] = in-degree; pidx[c][r] becomes
// the global pair row of (r, c) (or -1).  prow / pdeg were set to -1 / 0.
__global__ void k_pair_fill(const u16* __restrict__ degc, int* __restrict__ pidx, const int* __restrict__ poff, long N,
                            long total, int cap, int* __restrict__ prow, float* __restrict__ pdeg) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int pos = pidx[e];
    if (pos < 0) continue;
    const int c = (int)(e / N);
    const long r = e - (long)c * N;
    const int p = poff[c] + pos;
    if (p < cap) {
      prow[p] = (int)r;
      pdeg[p] = (float)degc[e];
    }
    pidx[e] = p < cap ? p : -1;
  }
}


// B5: the dW product's term lists over all T timesteps: chunk z's tiles
// (wtl[z*(1+chunk)]) repeated per timestep as q = t * cap_tiles + tile,
// t ascending (groups of equal size: GemmArgs::tgroups)
__global__ void k_pair_wtl_expand(const int* __restrict__ wtl, int zw, int T, int cap_tiles, int chunk,
                                  int* __restrict__ out) {
  const int z = blockIdx.x * blockDim.x + threadIdx.x;
  if (z >= zw) return;
  const int* q = wtl + (long)z * (1 + chunk);
  int* o = out + (long)z * (1 + (long)T * chunk);
  const int n = q[0];
  o[0] = n * T;
  for (int t = 0; t < T; ++t)
    for (int e = 0; e < n; ++e) o[1 + t * n + e] = t * cap_tiles + q[1 + e];
}

// S5: the backward's reverse gather lists: for every node row r = (g, j) the
// pair rows p = (g, i, c) with A[g,c,i,j] = 1, in (ascending channel among the
// graph's occupied ones, ascending i) -- the order k_pair_scatter_dh sums them
// in.  FILL = false: counts rcnt[r]; FILL = true: rlist[roff[r] ...] after the
// scan.  A wave per row, its sources by ballots over the staged transpose row.
// (<= 4 nonzeros per edge, so the lists fit the pair-row capacity.)
template <bool FILL>
__global__ void __launch_bounds__(256) k_pair_rev(const u16* __restrict__ AgT, const unsigned char* __restrict__ occ,
                                                  const int* __restrict__ pidx, int b, int v, int vp, int C,
                                                  int* __restrict__ rcnt, const int* __restrict__ roff,
                                                  int* __restrict__ rlist, int cap) {
  const int lane = threadIdx.x & 63;
  const long N = (long)b * v;
  for (long r = blockIdx.x * 4 + (threadIdx.x >> 6); r < N; r += (long)gridDim.x * 4) {
    const int g = (int)(r / v), j = (int)(r - (long)g * v);
    long pos = FILL ? roff[r] : 0;
    int cnt = 0;
    const unsigned char* og = occ + (long)g * C;
    for (int cb = 0; cb < C; cb += 64) {
      // the graph's occupied channels of this block of 64, ascending
      unsigned long long mc = __ballot(cb + lane < C && og[cb + lane] != 0);
      while (mc) {
        const int c = cb + __ffsll((long long)mc) - 1;
        mc &= mc - 1ull;
        const u16* arow = AgT + (((long)g * C + c) * v + j) * vp;
        const int* pc = pidx + (long)c * N + (long)g * v;
        for (int ib = 0; ib < v; ib += 64) {
          const int i = ib + lane;
          const bool nz = i < v && arow[i] != 0;
          const unsigned long long m = __ballot(nz);
          if (FILL && nz) {
            const long q = pos + __popcll(m & ((1ull << lane) - 1ull));
            if (q < cap) rlist[q] = pc[i];
          }
          pos += __popcll(m);
          cnt += __popcll(m);
        }
      }
    }
    if (!FILL && lane == 0) rcnt[r] = cnt;
  }
}
// exclusive scan of rcnt[0, N) into roff[0, N] (one block)
__global__ void __launch_bounds__(1024) k_pair_rev_scan(const int* __restrict__ rcnt, long N, int* __restrict__ roff) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  __shared__ int wsum[16];
  int base = 0;
  for (long r0 = 0; r0 < N; r0 += 1024) {
    const long r = r0 + tid;
    const int x = r < N ? rcnt[r] : 0;
    int incl = x;  // inclusive scan within the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int woff = 0, tot = 0;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      woff += u < w ? wsum[u] : 0;
      tot += wsum[u];
    }
    if (r < N) roff[r] = base + woff + incl - x;
    base += tot;
    __syncthreads();
  }
  if (tid == 0) roff[N] = base;
}

// F1 (and its recomputation in the backward): Y[p][k] = sum_j A[g,c,i,j] h[g*v+j][k]
// for every pair row p = (g*v+i, c) of a live tile; padding rows of a live
// tile get zeros (the products read whole tiles).  One wave per pair row,
// 4 columns per lane (H % 4 == 0), the row's sources found by ballots over the
// staged adjacency row.
__global__ void __launch_bounds__(256) k_pair_gather_y(const u16* __restrict__ Ag, const int* __restrict__ prow,
                                                       const int* __restrict__ ptile,
                                                       const unsigned char* __restrict__ pmask,
                                                       const float* __restrict__ h, float* __restrict__ Y, int C,
                                                       int v, int vp, int H, int rows) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  for (int p = blockIdx.x * 4 + (threadIdx.x >> 6); p < rows; p += nw) {
    if (!pmask[p / PAIR_TILE]) continue;
    const int r = prow[p];
    float* y = Y + (long)p * H;
    if (r < 0) {
      for (int k = 4 * lane; k < H; k += 256) *(float4*)(y + k) = make_float4(0.f, 0.f, 0.f, 0.f);
      continue;
    }
    const int c = ptile[2 * (p / PAIR_TILE) + 1];
    const int g = r / v, i = r - g * v;
    const u16* arow = Ag + (((long)g * C + c) * v + i) * vp;
    const float* hg = h + (long)g * v * H;
    for (int k0 = 0; k0 < H; k0 += 256) {
      const int k = k0 + 4 * lane;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int jb = 0; jb < v; jb += 64) {
        const int j = jb + lane;
        unsigned long long m = __ballot(j < v && arow[j] != 0);
        while (m) {
          const int jj = jb + __ffsll((long long)m) - 1;
          m &= m - 1ull;
          if (k < H) {
            const float4 x = *(const float4*)(hg + (long)jj * H + k);
            acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
          }
        }
      }
      if (k < H) *(float4*)(y + k) = acc;
    }
  }
}

// F3: X[r][k] = sum over the channels c of r's graph (ascending) with a pair
// (r, c) of Z[p][k] + deg_p beta[c][k]; one thread per (row, column quad)
__global__ void k_pair_reduce_x(const int* __restrict__ pidx, const float* __restrict__ pdeg,
                                const int* __restrict__ chl, const float* __restrict__ Z,
                                const float* __restrict__ beta, float* __restrict__ X, long N, int v, int C, int H) {
  const int hq = H >> 2;
  const long total = N * hq;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long r = e / hq;
    const int k = 4 * (int)(e - r * hq);
    const int g = (int)(r / v);
    const int* cl = chl + (long)g * (C + 1);
    const int n = cl[0];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    // 8 channels per step: their pair lookups, then their Z / deg / beta loads,
    // all issued before the first add (a sentence graph has ~27 channels and
    // ~3 pairs per row: one dependent lookup-then-load per channel was the
    // kernel's latency); the adds stay in ascending channel order
    for (int u0 = 0; u0 < n; u0 += 8) {
      int cc[8], pp[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) cc[j] = u0 + j < n ? cl[1 + u0 + j] : 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) pp[j] = u0 + j < n ? pidx[(long)cc[j] * N + r] : -1;
      float4 z[8];
      float d[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const long q = pp[j] < 0 ? 0 : pp[j];
        z[j] = *(const float4*)(Z + q * H + k);
        d[j] = beta ? pdeg[q] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (pp[j] < 0) continue;
        acc.x += z[j].x; acc.y += z[j].y; acc.z += z[j].z; acc.w += z[j].w;
        if (beta) {
          const float4 bb = *(const float4*)(beta + (long)cc[j] * H + k);
          acc.x += d[j] * bb.x; acc.y += d[j] * bb.y; acc.z += d[j] * bb.z; acc.w += d[j] * bb.w;
        }
      }
    }
    *(float4*)(X + r * H + k) = acc;
  }
}

// B1: dXg[p] = dX[prow[p]] (dX = the first half of the [N][2H] DXH rows); 0 on
// the padding rows of live tiles
__global__ void k_pair_gather_dx(const int* __restrict__ prow, const unsigned char* __restrict__ pmask,
                                 const float* __restrict__ DXH, float* __restrict__ dXg, int rows, int H) {
  const int hq = H >> 2;
  const long total = (long)rows * hq;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int p = (int)(e / hq), k = 4 * (int)(e - (long)p * hq);
    if (!pmask[p / PAIR_TILE]) continue;
    const int r = prow[p];
    const float4 x = r >= 0 ? *(const float4*)(DXH + (long)r * 2 * H + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    *(float4*)(dXg + (long)p * H + k) = x;
  }
}

// k_pair_gather_dx and the dL/dbeta tile partials of k_pair_dbeta in one
// pass (round 5): block = one live pair tile, thread = one 4-column quad of
// every row of the tile (H / 4 <= 256): dXg[p] = dX of p's node row, and
// part[tile][k..k+3] = sum over the tile's rows in row order of deg_p dXg[p]
__global__ void __launch_bounds__(256) k_pair_gather_dx_dbeta(const int* __restrict__ prow,
                                                              const unsigned char* __restrict__ pmask,
                                                              const float* __restrict__ pdeg,
                                                              const float* __restrict__ DXH, float* __restrict__ dXg,
                                                              float* __restrict__ part, int H) {
  const int tile = blockIdx.x, k = 4 * threadIdx.x;
  if (k >= H || !pmask[tile]) return;
  const long p0 = (long)tile * PAIR_TILE;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int i = 0; i < PAIR_TILE; ++i) {
    const long p = p0 + i;
    const int r = prow[p];
    const float4 x = r >= 0 ? *(const float4*)(DXH + (long)r * 2 * H + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    *(float4*)(dXg + p * H + k) = x;
    const float dg = pdeg[p];
    s.x += dg * x.x; s.y += dg * x.y; s.z += dg * x.z; s.w += dg * x.w;
  }
  if (part) *(float4*)(part + (long)tile * H + k) = s;
}

// dL/dbeta partials: part[tile][k] = sum over the pair tile's rows (one
// channel's, padding rows of degree 0) of deg_p dXg[p][k]; grid (column
// blocks, pair tiles).  The channels' sums over their tiles (and the
// timesteps) follow in a fixed order (k_slab_reduce): no atomics.
__global__ void __launch_bounds__(256) k_pair_dbeta(const unsigned char* __restrict__ pmask,
                                                    const float* __restrict__ pdeg, const float* __restrict__ dXg,
                                                    float* __restrict__ part, int H) {
  const int k = blockIdx.x * 256 + threadIdx.x, tile = blockIdx.y;
  if (k >= H || !pmask[tile]) return;
  const long p0 = (long)tile * PAIR_TILE;
  float s = 0.f;
#pragma unroll 4
  for (int i = 0; i < PAIR_TILE; ++i) s += pdeg[p0 + i] * dXg[(p0 + i) * H + k];
  part[(long)tile * H + k] = s;
}

// B3: DXH[g*v+j][H + k] += sum over the channels c of g (ascending) and the
// receivers i of j on c (A[g,c,i,j] = 1, ascending) of dY[pair(g*v+i, c)][k];
// one wave per source row walking its reverse list (S5: built once per staged
// batch, not per timestep)
__global__ void __launch_bounds__(256) k_pair_scatter_dh(const int* __restrict__ roff, const int* __restrict__ rlist,
                                                         const float* __restrict__ dY, float* __restrict__ DXH, long N,
                                                         int H) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  for (long r = blockIdx.x * 4 + (threadIdx.x >> 6); r < N; r += nw) {
    const int e0 = roff[r], e1 = roff[r + 1];
    for (int k0 = 0; k0 < H; k0 += 256) {
      const int k = k0 + 4 * lane;
      if (k >= H) continue;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int e = e0; e < e1; ++e) {
        const int p = rlist[e];
        if (p >= 0) {
          const float4 x = *(const float4*)(dY + (long)p * H + k);
          acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
        }
      }
      float4* d = (float4*)(DXH + r * 2 * H + H + k);
      float4 o = *d;
      o.x += acc.x; o.y += acc.y; o.z += acc.z; o.w += acc.w;
      *d = o;
    }
  }
}
