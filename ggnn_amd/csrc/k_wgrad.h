// k_wgrad.h -- weight gradients as one grouped split-K "NT" GEMM launch:
//   out[m][n] = sum_{t < T} sum_{chunks} sum_{k in chunk} P_t[m][k] * Q_t[n][k]
// (stored once by k_wgrad_reduce, not accumulated onto out)
// P_t / Q_t are the transposed activations saved per timestep ([M][K] and
// [N][K], K = the b*V node rows), each a stack of [H][K] arrays in the
// K-blocked wg_off layout (ggnn_common.h).  Problems (reference autodiff,
// chem_tensorflow.py:496):
//   d gates_kernel     = [X | h]^T  dzg        d candidate_kernel = [X | r*h]^T dzc
//   d edge_weights[c]  = h^T dM_c
// Each workgroup sums its K chunk over all T steps.  Deterministic reduction
// over the K chunks (WgArgs::part, round 5): the workgroup stores its partial
// tile in the accumulator's own register order (16-byte stores, one
// [TS][TS] block per (tile, chunk)), and k_wgrad_reduce sums the chunks of a
// tile in chunk order and writes the output once (times the backward's
// gradient unscale, WgArgs::gmax) -- the same bits whatever order the
// workgroups ran in (with part == nullptr: one fp32 atomicAdd per
// output element and chunk, order-dependent).
// Edge dropout (round 6): the dW problem's chunks are timestep-aligned
// (WgProb::cpt chunks of KCt rows inside ONE timestep each, chunk k at
// timestep k / cpt), and k_wgrad_reduce forms
//   dW_c[i][j] = sum_t mask_t(c,i,j)/keep * (sum of timestep t's chunks)
// with the pack's Philox draws (edge_words: counter (i>>2, j, c, t)).
#pragma once
#include "ggnn_common.h"

struct WgProb {
  const void* P;
  const void* Q;
  float* out;
  long ldP, ldQ, stepP, stepQ;  // elements
  long sQb, sOb;                // batch strides of Q and out (batched problem, e.g. one per channel)
  long sPb;                     // batch stride of P, applied to (batch index / pdiv)
  int pdiv, T;                  // T: timesteps summed by this problem
  int ldO, M, N, tiles_n, tiles_b, tile_begin;
  // k_wgrad256 only: K runs over the rows of listed graphs instead of every row
  // (dW_c over the graphs with an edge in channel c: the others' dM_c rows are
  // zero and are not written).  List of batch index bi at gl + (bi % glmod) *
  // gls: [count, graph, ...]; a graph is V32 slices of 32 rows.  nullptr: all rows.
  const int* gl;
  int gls, glmod, V32;
  // workgroups of this problem: tiles x nch chunks, from workgroup wg_begin
  // (its partial tiles at part + (wg_begin + tile_local * nch + chunk) * TS^2).
  // cpt > 0: timestep-aligned chunks (cpt per timestep, KCt rows each)
  int nch, cpt, KCt, wg_begin;
};
#define WG_LIST_MAX 256  // graphs of one K chunk held in registers (4 VGPRs)
#define WG_MAXP 8
struct WgArgs {
  WgProb p[WG_MAXP];
  int nprob, nchunks, KC;
  int H;  // rows of one operand array (wg_off layout); ldP / ldQ hold its N
  float* part;  // partial tiles (deterministic reduction, one per workgroup), or nullptr: atomics
  const uint32_t* gmax;  // if set: k_wgrad_reduce stores the sums times the gradient unscale (gunscale)
  Drop edrop;            // edge dropout of the timestep-aligned problem (thr 0: off)
};

// (problem, tile of the launch, chunk) of workgroup `wg`
struct WgWork {
  int pi, tile, chunk;
};
DEV WgWork wg_work(const WgArgs& args, int wg) {
  int pi = 0;
  while (pi + 1 < args.nprob && args.p[pi + 1].wg_begin <= wg) ++pi;
  const WgProb& pr = args.p[pi];
  const int local = wg - pr.wg_begin;
  return WgWork{pi, pr.tile_begin + local / pr.nch, local % pr.nch};
}
// K range of a workgroup: rows [kbase, kbase + kits * BK) of timesteps
// [t0, t0 + nt) (T-summed problems: chunk * KC, all T; timestep-aligned:
// timestep chunk / cpt, rows (chunk % cpt) * KCt)
struct WgK {
  long kbase;
  int kits, t0, nt;
};
template <int BK>
DEV WgK wg_k(const WgArgs& args, const WgProb& pr, int chunk) {
  if (pr.cpt) return WgK{(long)(chunk % pr.cpt) * pr.KCt, pr.KCt / BK, chunk / pr.cpt, 1};
  return WgK{(long)chunk * args.KC, args.KC / BK, 0, pr.T};
}

// (problem, batch index, tile origin) of tile `tile` (TS x TS tiles)
struct WgTile {
  int pi, bi, m0, n0;
};
template <int TS>
DEV WgTile wg_tile(const WgArgs& args, int tile) {
  int pi = 0;
  while (pi + 1 < args.nprob && args.p[pi + 1].tile_begin <= tile) ++pi;
  const WgProb& pr = args.p[pi];
  const int lt0 = tile - pr.tile_begin;
  const int lt = lt0 % pr.tiles_b;
  return WgTile{pi, lt0 / pr.tiles_b, (lt / pr.tiles_n) * TS, (lt % pr.tiles_n) * TS};
}

// A workgroup's partial tile in accumulator order: float4 index
// f = ((((wave * NI + i) * NJ + j) * 4 + quad) * 64 + lane) holds rows
// acc_row(4 quad + e, lane >> 5) of the (wave, i, j) 32 x 32 block, column lane & 31
template <int NI, int NJ>
DEV void wg_store_part(float* pp, const f32x16 (&acc)[NI][NJ], int wv, int lane) {
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *(float4*)(pp + ((((wv * NI + i) * NJ + j) * 4 + q) * 64 + lane) * 4) =
            make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]);
}

// out = sum over the K chunks of the partial tiles, in chunk order.  TS = 256:
// k_wgrad256's 8 waves as 2 (m) x 4 (n) of 128 x 64 (NI = 4, NJ = 2); TS = 128:
// k_wgrad's 4 waves as 2 x 2 of 64 x 64 (NI = NJ = 2).  One thread per float4
// of a tile; grid = tiles * TS * TS / 1024 blocks of 256.
template <int TS>
__global__ void __launch_bounds__(256) k_wgrad_reduce(WgArgs args) {
  constexpr int NI = TS == 256 ? 4 : 2, NJ = 2, WN = TS == 256 ? 4 : 2, WMR = NI * 32, WNC = NJ * 32;
  constexpr int BPT = TS * TS / 1024;  // blocks per tile
  const int tile = blockIdx.x / BPT;
  const int f = (blockIdx.x % BPT) * 256 + threadIdx.x;
  const WgTile wt = wg_tile<TS>(args, tile);
  const WgProb& pr = args.p[wt.pi];
  const int lane = f & 63, q = (f >> 6) & 3, j = (f >> 8) % NJ, i = (f >> 8) / NJ % NI, wv = (f >> 8) / (NJ * NI);
  const int m = wt.m0 + (wv / WN) * WMR + i * 32 + acc_row(4 * q, lane >> 5);
  const int nn = wt.n0 + (wv % WN) * WNC + j * 32 + (lane & 31);
  const float* src = args.part + (long)(pr.wg_begin + (tile - pr.tile_begin) * pr.nch) * (TS * TS) + f * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (pr.cpt && args.edrop.thr) {
    // edge dropout: timestep t's chunks summed in order, times mask_t / keep
    // (rows m..m+3 = one Philox block's 4 words: m is a multiple of 4), then
    // the timesteps in order
    const Drop dr = drop_resolve(args.edrop);
    for (int t = 0; t < pr.T; ++t) {
      float4 st = *(const float4*)(src + (long)t * pr.cpt * (TS * TS));
      for (int c = 1; c < pr.cpt; ++c) {
        const float4 x = *(const float4*)(src + (long)(t * pr.cpt + c) * (TS * TS));
        st.x += x.x; st.y += x.y; st.z += x.z; st.w += x.w;
      }
      const uint4 w = edge_words(dr, wt.bi, m, nn, t);
      s.x += drop_apply(dr, w.x, st.x);
      s.y += drop_apply(dr, w.y, st.y);
      s.z += drop_apply(dr, w.z, st.z);
      s.w += drop_apply(dr, w.w, st.w);
    }
  } else {
    s = *(const float4*)src;
    for (int c = 1; c < pr.nch; ++c) {
      const float4 x = *(const float4*)(src + (long)c * (TS * TS));
      s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
    }
  }
  float* o = pr.out + (long)wt.bi * pr.sOb + (long)m * pr.ldO + nn;
  const float us = gunscale(args.gmax);
  o[0] = s.x * us;
  o[pr.ldO] = s.y * us;
  o[2L * pr.ldO] = s.z * us;
  o[3L * pr.ldO] = s.w * us;
}

template <int BK, int PREC>
__global__ void __launch_bounds__(256) k_wgrad(WgArgs args) {
  constexpr bool SPLIT = Prec<PREC>::split, F16 = Prec<PREC>::f16;
  using Act = ActT<PREC>;
  constexpr int CH = BK / 8;                 // 16-B chunks per LDS tile row
  constexpr int TB = 128 * BK * 2;           // bytes of one bf16 operand image
  constexpr int NIMG = SPLIT ? 2 : 1;
  constexpr int BUF = 2 * NIMG * TB;         // P and Q images of one stage
  constexpr int PT = 128 * CH / 256;         // 8-element chunks per thread per operand
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const WgWork wk = wg_work(args, blockIdx.x);
  const WgProb pr = args.p[wk.pi];
  const int lt0 = wk.tile - pr.tile_begin;
  const int bi = lt0 / pr.tiles_b, lt = lt0 % pr.tiles_b;
  const int m0 = (lt / pr.tiles_n) * 128, n0 = (lt % pr.tiles_n) * 128;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int wm = wv >> 1, wn = wv & 1;
  constexpr int RPB = 256 / (BK * 2);        // tile rows per 256-B LDS bank row
  auto soff = [&](int row, int ch) { return row * BK * 2 + ((ch ^ ((row / RPB) & (CH - 1))) << 4); };

  const WgK K = wg_k<BK>(args, pr, wk.chunk);
  const int kits = K.kits, nit = kits * K.nt, H = args.H;
  const long kbase = K.kbase;
  const Act* Pb = (const Act*)pr.P + (long)(bi / pr.pdiv) * pr.sPb + (long)K.t0 * pr.stepP;
  const Act* Qb = (const Act*)pr.Q + (long)bi * pr.sQb + (long)K.t0 * pr.stepQ;
  float* const outp = pr.out + (long)bi * pr.sOb;
  // staging registers: one 8-element chunk = 16 B (bf16) or 32 B (fp32)
  typedef typename std::conditional<SPLIT, float4, uint4>::type V4;
  constexpr int PER = SPLIT ? 2 : 1;
  V4 rp[PT][PER], rq[PT][PER];
  auto gload = [&](int it) {
    const int t = it / kits;
    const long k0 = kbase + (long)(it % kits) * BK;
    const Act* P = Pb + (long)t * pr.stepP;
    const Act* Q = Qb + (long)t * pr.stepQ;
#pragma unroll
    for (int p = 0; p < PT; ++p) {
      const int q = tid + p * 256, row = q / CH, ch = q % CH;
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const int mr = m0 + row, nr = n0 + row;
        rp[p][e] = *(const V4*)(P + (long)(mr / H) * H * pr.ldP + wg_off(mr % H, k0 + ch * 8 + 4 * e, H));
        rq[p][e] = *(const V4*)(Q + (long)(nr / H) * H * pr.ldQ + wg_off(nr % H, k0 + ch * 8 + 4 * e, H));
      }
    }
  };
  auto put = [&](char* hi, char* lo, int off, const V4* v) {
    if constexpr (SPLIT) {
      const float x[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
      st16(hi + off, pk8<true>(x));
      st16(lo + off, pk8_lo<true>(x));
    } else {
      st16(hi + off, v[0]);
    }
  };
  auto sstore = [&](int buf) {
    char* b = smem + buf * BUF;
    char* ph = b;
    char* pl = b + (SPLIT ? TB : 0);
    char* qh = b + NIMG * TB;
    char* ql = qh + (SPLIT ? TB : 0);
#pragma unroll
    for (int p = 0; p < PT; ++p) {
      const int q = tid + p * 256, row = q / CH, ch = q % CH;
      put(ph, pl, soff(row, ch), rp[p]);
      put(qh, ql, soff(row, ch), rq[p]);
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = splat(0.f);

  gload(0);
  sstore(0);
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const bool pre = it + 1 < nit;
    if (pre) gload(it + 1);
    const char* b = smem + (it & 1) * BUF;
    const char* ph = b;
    const char* pl = b + (SPLIT ? TB : 0);
    const char* qh = b + NIMG * TB;
    const char* ql = qh + (SPLIT ? TB : 0);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      frag ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int off = soff(wm * 64 + i * 32 + l32, 2 * s + hh);
        ah[i] = lds_frag(ph, off);
        al[i] = SPLIT ? lds_frag(pl, off) : ah[i];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int off = soff(wn * 64 + j * 32 + l32, 2 * s + hh);
        bh[j] = lds_frag(qh, off);
        bl[j] = SPLIT ? lds_frag(ql, off) : bh[j];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mma<PREC>(acc[i][j], ah[i], al[i], bh[j], bl[j]);
    }
    if (pre) sstore((it + 1) & 1);
    __syncthreads();
  }
  if (args.part) {
    wg_store_part<2, 2>(args.part + (long)blockIdx.x * (128 * 128), acc, wv, lane);
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + acc_row(r, hh);
        const int nn = n0 + wn * 64 + j * 32 + l32;
        atomicAdd(outp + (long)m * pr.ldO + nn, acc[i][j][r]);
      }
}

// ===========================================================================
// k_wgrad256: the same grouped NT problem set with 256x256 output tiles (all
// problems have M = 256 and N a multiple of 256 at hidden = 256), so every
// operand slice is read by one workgroup only (dW: P and Q once; dWg: P
// twice).  8 waves as 2 (m) x 4 (n), 128x64 outputs each.  K slices of 32
// rows arrive by LDS-DMA into a 4-deep ring: two slices stay in flight while
// one is consumed (counted vmcnt + raw s_barrier; a __syncthreads would drain
// the DMAs every step).  16-bit operands only (the split mode's weight-gradient
// operands are single f16 limbs).
// ===========================================================================
template <int PREC>
__global__ void __launch_bounds__(512) k_wgrad256(WgArgs args) {
  constexpr bool F16 = Prec<PREC>::f16;
  static_assert(!Prec<PREC>::split, "16-bit operands only");
  constexpr int BK = 32, CH = BK / 8;        // 4 chunks of 16 B per image row
  constexpr int TB = 256 * BK * 2;           // 16 KiB per operand image
  constexpr int NBUF = 4;
  constexpr int GPW = 256 * CH / 64 / 8;     // glds per wave per operand per slice (= 2)
  // one __shared__ object per ring slot, each addressed with a compile-time
  // slot index: the waitcnt pass can then tell a ds_read of slot u from the
  // DMAs still landing in the other slots (with one array and a runtime slot
  // it waits vmcnt(0) before every read)
  __shared__ __attribute__((aligned(16))) char sp0[TB], sp1[TB], sp2[TB], sp3[TB];  // P images
  __shared__ __attribute__((aligned(16))) char sq0[TB], sq1[TB], sq2[TB], sq3[TB];  // Q images
  auto pslot = [&](int u) -> char* { return u == 0 ? sp0 : u == 1 ? sp1 : u == 2 ? sp2 : sp3; };
  auto qslot = [&](int u) -> char* { return u == 0 ? sq0 : u == 1 ? sq1 : u == 2 ? sq2 : sq3; };
  TSCLK(0, 0);
  const WgWork wk = wg_work(args, blockIdx.x);
  const WgProb pr = args.p[wk.pi];
  const int lt0 = wk.tile - pr.tile_begin;
  const int bi = lt0 / pr.tiles_b, lt = lt0 % pr.tiles_b;
  const int m0 = (lt / pr.tiles_n) * 256, n0 = (lt % pr.tiles_n) * 256;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int wm = wv >> 2, wn = wv & 3;
  // image: row r = 64 B, chunk slot pc holds logical chunk pc ^ ((r >> 2) & 3)
  auto soff = [](int row, int ch) { return row * BK * 2 + ((ch ^ ((row >> 2) & 3)) << 4); };

  const WgK K = wg_k<BK>(args, pr, wk.chunk);
  const u16* Pb = (const u16*)pr.P + (long)(bi / pr.pdiv) * pr.sPb + (long)K.t0 * pr.stepP;
  const u16* Qb = (const u16*)pr.Q + (long)bi * pr.sQb + (long)K.t0 * pr.stepQ;
  float* const outp = pr.out + (long)bi * pr.sOb;
  // K slices: the chunk's rows (kits slices) x its timesteps, or, with a graph
  // list, the chunk's share of the listed graphs' slices (any count: nit may
  // be 0 -- nothing to add -- and need not be a multiple of NBUF)
  int kits = K.kits;
  long kbase = K.kbase;
  int glr[4] = {0, 0, 0, 0};  // the chunk's graphs, lane-distributed (read back by readlane)
  bool listed = false;        // K walks the list (else the contiguous rows from kbase)
  if (pr.gl) {
    const int* list = pr.gl + (long)(bi % pr.glmod) * pr.gls;
    // a timestep-aligned problem splits the list over its cpt chunks of a timestep
    const int nsplit = pr.cpt ? pr.cpt : args.nchunks, ci = pr.cpt ? wk.chunk % pr.cpt : wk.chunk;
    const int cnt = list[0], per = (cnt + nsplit - 1) / nsplit;
    const int gb = min(cnt, ci * per), ge = min(cnt, gb + per);
    kits = (ge - gb) * pr.V32;
    if (ge > gb) {
      const int g0 = list[1 + gb], g1 = list[ge];
      if (g1 - g0 == ge - gb - 1) {
        kbase = (long)g0 * pr.V32 * 32;  // consecutive graphs: their rows are contiguous
      } else {
        listed = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) glr[j] = (gb + j * 64 + lane < ge) ? list[1 + gb + j * 64 + lane] : 0;
      }
    }
  }
  const int nit = kits * K.nt;
  if (nit == 0 && !args.part) return;  // (partials: a zero tile still has to be stored)
  // row of slice `it`'s first K element: graph glr[i] (i = slice / V32) row (slice % V32) * 32
  auto krow = [&](int sl) -> long {
    if (!listed) return kbase + (long)sl * BK;
    const int i = sl / pr.V32;
    const int v = i < 64 ? glr[0] : i < 128 ? glr[1] : i < 192 ? glr[2] : glr[3];
    return (long)__builtin_amdgcn_readlane(v, i & 63) * (pr.V32 * 32) + (long)(sl % pr.V32) * 32;
  };

  auto stage = [&](int it, char* bp, char* bq) {
    const int t = it / kits;
    const long k0 = krow(it % kits);
    // wg_off layout at H = 256: the slice is one contiguous [256][32] block of
    // the (m0 / 256)-th [H][N] array
    const u16* P = Pb + (long)t * pr.stepP + (long)(m0 >> 8) * 256 * pr.ldP + (k0 >> 5) * 8192;
    const u16* Q = Qb + (long)t * pr.stepQ + (long)(n0 >> 8) * 256 * pr.ldQ + (k0 >> 5) * 8192;
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const int qb = (g * 8 + wv) * 64;  // first 16-B slot of this wave-instruction
      const int q = qb + lane, row = q / CH, pc = q % CH, lc = pc ^ ((row >> 2) & 3);
      glds16_asm(P + row * 32 + lc * 8, bp + qb * 16);
      glds16_asm(Q + row * 32 + lc * 8, bq + qb * 16);
    }
  };
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = splat(0.f);

  // prologue: slices 0, 1, 2 in flight
#pragma unroll
  for (int u = 0; u < NBUF - 1; ++u)
    if (u < nit) stage(u, pslot(u), qslot(u));
  // slice `it` from ring slot u = it % NBUF
  auto slice = [&](int it, int u) {
    // slice `it` landed (this wave's DMAs: the two younger slices may stay in flight)
    if (it + 2 < nit) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * GPW) : "memory");
    else if (it + 1 < nit) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMAs of slice `it` landed; slice it-1 fully read
    if (it + NBUF - 1 < nit) stage(it + NBUF - 1, pslot((u + NBUF - 1) % NBUF), qslot((u + NBUF - 1) % NBUF));
    const char* bp = pslot(u);
    const char* bq = qslot(u);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      frag a[4], bb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = lds_frag(bp, soff(wm * 128 + i * 32 + l32, 2 * s + hh));
#pragma unroll
      for (int j = 0; j < 2; ++j) bb[j] = lds_frag(bq, soff(wn * 64 + j * 32 + l32, 2 * s + hh));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma<F16>(a[i], bb[j], acc[i][j]);
    }
  };
  // whole groups of NBUF slices with no exit test inside the unrolled group
  // (a per-slice break there cost the dense config-3 product ~5 %), then the
  // tail a graph list may leave
  const int nfull = nit - nit % NBUF;
  for (int it0 = 0; it0 < nfull; it0 += NBUF) {
#pragma unroll
    for (int u = 0; u < NBUF; ++u) slice(it0 + u, u);
  }
  for (int u = 0; u < nit - nfull; ++u) slice(nfull + u, u);
  if (args.part) {
    wg_store_part<4, 2>(args.part + (long)blockIdx.x * (256 * 256), acc, wv, lane);
    TSCLK(0, 1);
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + i * 32 + acc_row(r, hh);
        const int nn = n0 + wn * 64 + j * 32 + l32;
        atomicAdd(outp + (long)m * pr.ldO + nn, acc[i][j][r]);
      }
}
