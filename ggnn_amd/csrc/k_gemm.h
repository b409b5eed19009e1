// k_gemm.h -- generic MFMA GEMM over term lists: the engine's general path
// (hidden sizes and vertex counts outside the fused kernels' envelope, e.g.
// the reference's default hidden_size 400, chem_tensorflow.py:95, and its
// 198-node buckets, chem_tensorflow_dense.py:584-585) and the output heads.
//
// For every z in [0, Z) and every term e of z (term = a pair (p, q)):
//   D_z[m][n] (op)= epi( alpha * sum_e sum_k A_pq[m][k] B_pq[k][n] + bias_z[n] )
// with every operand addressed by strides, so one kernel covers
//   * batched products (z = graph, or z = (graph, channel) pairs),
//   * reductions over channel lists (terms of z = the channels of graph z),
//   * concatenated operands ([x, h] @ W: two terms whose A bases differ by a
//     constant distance inside one workspace),
//   * split-K over long row ranges (z = row chunk, atomic accumulation).
// Operands are read as fp32 (or exact 16-bit limbs for the 0/1 adjacency) and
// converted to the precision policy's limbs while staged into LDS
// (ggnn_common.h: split = f16 hi/lo, 3 MFMAs per product).
//
// Tile 64 x 64 per workgroup (4 waves, 32 x 32 each: one
// v_mfma_f32_32x32x16 accumulator), K in slices of 32, double-buffered LDS with
// the next slice's global loads in flight during the current slice's MFMAs.
#pragma once
#include "ggnn_common.h"

#define GG_EPI_NONE 0
#define GG_EPI_SIGMOID 1
#define GG_EPI_TANH 2
#define GG_STORE 0
#define GG_ADD 1     // D += result (one writer per element)
#define GG_ATOMIC 2  // atomicAdd (split-K: several z per output element)

struct GemmArgs {
  const void* A;        // fp32, or 16-bit exact limbs (A16)
  const void* A2;       // if set: the A base of the terms with q == 1 (two separate operands, e.g. [hT | h0])
  const float* B;
  float* D;
  const float* bias;    // [N] at zp*sbp + zq*sbq, or null
  const float* E;       // if set: D's element-wise multiplier (same offsets as D), e.g. a dropout scale
  float scA, scB;       // exact power-of-two operand scales applied before the limb split (small
                        // operands stay in the f16 normal range); alpha undoes them
  long sAp, sAq, sAm, sAk;
  long sBp, sBq, sBk, sBn;
  long sDz, sDp, sDq, sDm, sDn;
  long sbp, sbq;
  // z -> (zp, zq) = (z / zdiv, z % zdiv); z is skipped when zmask && !zmask[z]
  int zdiv;
  const unsigned char* zmask;
  // terms of z: tl == null: nterm terms (zp, zq + e) (nterm 0 = 1); else
  // nt = tl[z*ts] terms (zp, tl[z*ts + 1 + e]) (a count-prefixed list, e.g. a
  // graph's channels)
  const int* tl;
  long ts;
  int nterm;
  int Z, M, N, K;       // per-term K; term k range [p*sKp, p*sKp + K) clipped to Ktot
  long Ktot, sKp;
  float alpha;
  int epi, mode;
  // row / column splits of one product over two buffers (Msplit, Nsplit
  // multiples of 64; 0 = none): A rows m >= Msplit come from Am2 (row
  // m - Msplit), outputs n >= Nsplit go to D2 (column n - Nsplit; row
  // stride sD2m, or sDm when 0)
  const void* Am2;
  int Msplit;
  float* D2;
  int Nsplit;
  long sD2m;
  // if set: csum[zp*scp + zq*scq + n] += sum over m of the stored values of
  // column n (e.g. the edge-bias gradient from dM), one atomic per column per
  // wave pair
  float* csum;
  long scp, scq;
  // if set: zp = zmap[z], zq = 0 (z -> an arbitrary operand group, e.g. the
  // pair-mode dW chunks of channel zmap[z], k_pairs.h)
  const int* zmap;
  // if dr.thr: every stored value (m, n) of z is multiplied by the edge-dropout
  // mask of (channel zp, row m, column n, timestep drop_t) / keep -- the
  // masked weight gradient dW_c += mask_t * (Y^T dX) accumulated straight into
  // dW (Philox counter (m>>2, n, zp, t), word m&3: one block per row quad)
  Drop dr;
  int drop_t;
  // if set: the scales come from a device float t (the heads' target_num,
  // ggnn_heads_backward_dev): S = tnum_scale(*snum) replaces scA (sdev bit 0)
  // and / or scB (bit 1), and alpha = 1 / S
  const float* snum;
  int sdev;
  // tgroups > 1 (k_gemm_ring only): z's terms form tgroups equal groups, group
  // k being timestep k: the accumulator is multiplied by the dropout mask dr of
  // timestep k (not drop_t) at each group's end and banked, so one launch sums
  // mask_t-weighted products over t (the pair-mode dW over all timesteps)
  int tgroups;
  // TGRP with dropout: the keep masks as bits (written by the pack beside its
  // masked W copies, PackJob::bits; required, the
  // kernel draws no Philox words): word ((t*C + zp)*N + n)*mbw + m/32, bit m%32
  // (mbC = C)
  const uint32_t* mbits;
  int mbw, mbC;
  // GG_ATOMIC with a slab (deterministic split-K, round 5): z stores its
  // partial product at slab[z * sSlab + m * N + n] instead of adding into D;
  // k_slab_reduce then sums each output's z's in z order.  (The pair dW chunk
  // that is its channel's only one, zmask 2, still stores straight into D.)
  float* slab;
  long sSlab;
  // with csum: the column sums as deterministic partials instead of atomics,
  // cpart[(z * cslots + m / 32) * N + n] = the sum over one 32-row slice's
  // stored values (cslots = ceil(M / 32); a wave covering several slices puts
  // its sum in the first and zeros in the others), summed in (z, slice) order
  // afterwards (k_sum_rows)
  float* cpart;
  int cslots;
  // if set: alpha also carries the backward's gradient unscale 1 / S
  // (gunscale, ggnn_common.h), so a weight-gradient product stores final
  // values (S a power of two: the same bits as unscaling afterwards)
  const uint32_t* ugmax;
  // if set (GG_EPI_SIGMOID, the GRU gates [r | u] of width 2 auxN): the
  // reset-gated state aux[m * auxN + n] = r * auxin[m * auxN + n] for the
  // columns n < auxN, stored next to the gates (k_gemm_ks's epilogue; after
  // a ring launch gg_launch runs k_gen_rh instead)
  float* aux;
  const float* auxin;
  int auxN;
  // if set (GG_EPI_TANH, the GRU candidate c of width N): the blended state
  // bout[m * N + n] = u h + (1 - u) c, u = bu[m * 2N + N + n], h = bh[m * N + n],
  // then the state dropout bsd of timestep bt (graphs of bv rows), as
  // k_gen_blend computes it (k_gemm_ks's epilogue; else k_gen_blend after)
  float* bout;
  const float* bh;
  const float* bu;
  int bv, bt;
  Drop bsd;
  // if set (the product [dX1 | d(rh)] = dzc Wc^T, Nsplit = H): k_gen_bwd2 on
  // the d(rh) columns n >= H (k = n - H), x = d(rh), r = b2r[m * 2H + k],
  // h = b2h[m * H + k]: b2dzg[m * 2H + k] = x h r (1 - r), b2dxh[m * 2H + H + k]
  // += x r, and the dbg_r partial of each wave's rows in b2part[(32-row tile *
  // WK + wk) * H + k] (k_gemm_ks only)
  const float* b2r;
  const float* b2h;
  float* b2dzg;
  float* b2dxh;
  float* b2part;
  // -DGGNN_TS experiment builds: k + 1 = record this launch's per-workgroup
  // phase stamps in g_ts[k] (tools/ts_probe_generic.py); 0 = none
  int tsprobe;
};
// column-sum partial of the wave whose rows start at row mw and cover nsl
// 32-row slices (GemmArgs::cpart)
DEV void csum_part(const GemmArgs& a, int z, int mw, int nsl, int n, float cs) {
  const int s0 = mw >> 5;
  for (int i = 0; i < nsl; ++i)
    if (s0 + i < a.cslots) a.cpart[((long)z * a.cslots + s0 + i) * a.N + n] = i ? 0.f : cs;
}

// exact power of two S <= t carrying the heads' dZ ~ 1/t into the f16 normal
// range (frexp exponent e: S = 2^(e-1), clamped to 2^+-100); host and device
HDI float tnum_scale(float t) {
  int ex = 0;
  frexpf(t, &ex);
  const int e = ex - 1 < -100 ? -100 : ex - 1 > 100 ? 100 : ex - 1;
  return ldexpf(1.0f, e);
}
// the operand scales and alpha of one launch (device-resolved under snum)
struct GemmScales {
  float sa, sb, alpha;
};
DEV GemmScales gemm_scales(const GemmArgs& a) {
  GemmScales g{a.scA, a.scB, a.alpha};
  if (a.snum) {
    const float S = tnum_scale(*a.snum);
    if (a.sdev & 1) g.sa = S;
    if (a.sdev & 2) g.sb = S;
    g.alpha = 1.0f / S;
  }
  if (a.ugmax) g.alpha *= gunscale(a.ugmax);
  return g;
}

namespace gg {
constexpr int BM = 64, BN = 64, BK = 32, NT = 256;
constexpr int PITCH = 80;                  // bytes per LDS row: 32 limbs + 16 B pad
constexpr int TILE = 64 * PITCH;           // one [64][32] limb image
}  // namespace gg

// One operand's share of a [64 rows][32 k] stage per thread (8 values), rows
// = m (A) or n (B), element (row, k) at base + row*sR + k*sK:
//   KC (k contiguous): row tid>>2, k (tid&3)*8 .. +7    -> 16-byte loads
//   else (rows contiguous): rows 2(tid&31) and +1, k (tid>>5)*4 .. +3
//                           -> 8-byte loads per k (lanes cover 64 rows: 256 B)
// with a scalar, bounds-checked fallback on edge tiles / unaligned operands.
template <bool KC, bool U16, bool F16L>
DEV void gg_load(float* x, const void* P, long base, long sR, long sK, int r0, int R, int kk0, int K, long kg0,
                 long Ktot, float sc, int tid) {
  auto val = [&](long off) -> float {
    if constexpr (U16) return from_limb<F16L>(((const u16*)P)[off]);
    else return ((const float*)P)[off] * sc;
  };
  if constexpr (KC) {
    const int row = r0 + (tid >> 2), kq = (tid & 3) * 8;
    const long off = base + (long)row * sR + (long)(kk0 + kq) * sK;
    const bool full = row < R && kk0 + kq + 7 < K && kg0 + kq + 7 < Ktot && sK == 1;
    if constexpr (U16) {
      const u16* p = (const u16*)P + off;
      if (full && ((uintptr_t)p & 15) == 0) {
        const uint4 w = *(const uint4*)p;
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x[2 * j] = from_limb<F16L>((u16)(ws[j] & 0xFFFF));
          x[2 * j + 1] = from_limb<F16L>((u16)(ws[j] >> 16));
        }
        return;
      }
    } else {
      const float* p = (const float*)P + off;
      if (full && ((uintptr_t)p & 15) == 0) {
        const float4 a0 = *(const float4*)p, a1 = *(const float4*)(p + 4);
        x[0] = a0.x * sc; x[1] = a0.y * sc; x[2] = a0.z * sc; x[3] = a0.w * sc;
        x[4] = a1.x * sc; x[5] = a1.y * sc; x[6] = a1.z * sc; x[7] = a1.w * sc;
        return;
      }
      if (full && ((uintptr_t)p & 7) == 0) {  // rows of an odd number of float pairs (e.g. o = 150)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float2 w = *(const float2*)(p + 2 * j);
          x[2 * j] = w.x * sc;
          x[2 * j + 1] = w.y * sc;
        }
        return;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = row < R && kk0 + kq + j < K && kg0 + kq + j < Ktot;
      x[j] = ok ? val(base + (long)row * sR + (long)(kk0 + kq + j) * sK) : 0.f;
    }
  } else {
    const int row = r0 + 2 * (tid & 31), kq = (tid >> 5) * 4;
    const bool full = row + 1 < R && kk0 + kq + 3 < K && kg0 + kq + 3 < Ktot && sR == 1;
    const long off = base + (long)row + (long)(kk0 + kq) * sK;
    if constexpr (U16) {
      const u16* p = (const u16*)P + off;
      if (full && ((uintptr_t)p & 3) == 0 && (sK & 1) == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t w = *(const uint32_t*)(p + j * sK);
          x[j] = from_limb<F16L>((u16)(w & 0xFFFF));
          x[4 + j] = from_limb<F16L>((u16)(w >> 16));
        }
        return;
      }
    } else {
      const float* p = (const float*)P + off;
      if (full && ((uintptr_t)p & 7) == 0 && (sK & 1) == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float2 w = *(const float2*)(p + j * sK);
          x[j] = w.x * sc;
          x[4 + j] = w.y * sc;
        }
        return;
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = row + r < R && kk0 + kq + j < K && kg0 + kq + j < Ktot;
        x[4 * r + j] = ok ? val(base + (long)(row + r) * sR + (long)(kk0 + kq + j) * sK) : 0.f;
      }
  }
}
// the same share into the [row][k] limb image(s) (hi; lo when LO)
template <bool KC, bool F16, bool LO>
DEV void gg_store(char* hi, char* lo, const float* x, int tid) {
  using namespace gg;
  if constexpr (KC) {
    const int o = (tid >> 2) * PITCH + (tid & 3) * 16;
    st16(hi + o, pk8<F16>(x));
    if constexpr (LO) st16(lo + o, pk8_lo<true>(x));
  } else {
    const int row = 2 * (tid & 31), kq = (tid >> 5) * 4;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int o = (row + r) * PITCH + kq * 2;
      const float* y = x + 4 * r;
      *(uint2*)(hi + o) = make_uint2(pk<F16>(y[0], y[1]), pk<F16>(y[2], y[3]));
      if constexpr (LO) *(uint2*)(lo + o) = make_uint2(pk_lo<true>(y[0], y[1]), pk_lo<true>(y[2], y[3]));
    }
  }
}

// WM x WN accumulators per wave: block tile (64 WM) x (64 WN), 4 waves in 2 x 2
template <int PREC, bool A16, bool AKC, bool BKC, int WM, int WN>
__global__ void __launch_bounds__(256) k_gemm(GemmArgs a) {
  const Drop dr = drop_resolve(a.dr);  // (a device-resident key: loaded once)
  using namespace gg;
  constexpr bool SPLIT = Prec<PREC>::split, F16 = Prec<PREC>::f16;
  constexpr int BMt = 64 * WM, BNt = 64 * WN;
  constexpr int AT = BMt * PITCH, BT = BNt * PITCH, BUF = 2 * AT + 2 * BT;
  // [buf][A hi, A lo, B hi, B lo]
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int wm = w & 1, wn = w >> 1;
  const int n0 = blockIdx.x * BNt, m0 = blockIdx.y * BMt;
  const int kc = (a.K + BK - 1) / BK;
  const GemmScales gs = gemm_scales(a);

  for (int z = blockIdx.z; z < a.Z; z += gridDim.z) {
    if (a.zmask && !a.zmask[z]) continue;
    const int zp = a.zmap ? a.zmap[z] : z / a.zdiv, zq = a.zmap ? 0 : z % a.zdiv;
    const int nt = a.tl ? a.tl[(long)z * a.ts] : max(a.nterm, 1);
    const int nst = nt * kc;
    auto term = [&](int e, int& p, int& q) {
      p = zp;
      q = a.tl ? a.tl[(long)z * a.ts + 1 + e] : zq + e;
    };

    // ---- global -> registers: 8 values per 64-row share of each operand
    float ra[8 * WM], rb[8 * WN];
    auto load = [&](int st) {
      int p, q;
      term(st / kc, p, q);
      const int kk0 = (st % kc) * BK;
      const long kg0 = (long)p * a.sKp + kk0;  // global k of the slice's first column
      const bool second = a.A2 && q == 1;
      const bool lowm = a.Msplit && m0 >= a.Msplit;  // block-uniform row split
      const void* Ab = lowm ? a.Am2 : second ? a.A2 : a.A;
      const int am0 = lowm ? m0 - a.Msplit : m0;
      const int aM = lowm ? a.M - a.Msplit : a.Msplit ? a.Msplit : a.M;
      const long abase = p * a.sAp + (second ? 0 : q * a.sAq);
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        if constexpr (A16)
          gg_load<AKC, true, F16>(ra + 8 * i, Ab, abase, a.sAm, a.sAk, am0 + 64 * i, aM, kk0, a.K, kg0, a.Ktot, 1.0f,
                                  tid);
        else
          gg_load<AKC, false, F16>(ra + 8 * i, Ab, abase, a.sAm, a.sAk, am0 + 64 * i, aM, kk0, a.K, kg0, a.Ktot, gs.sa,
                                   tid);
      }
#pragma unroll
      for (int j = 0; j < WN; ++j)
        gg_load<BKC, false, F16>(rb + 8 * j, a.B, p * a.sBp + q * a.sBq, a.sBn, a.sBk, n0 + 64 * j, a.N, kk0, a.K, kg0,
                                 a.Ktot, gs.sb, tid);
    };
    // ---- registers -> LDS limb images ([row][k], k contiguous)
    auto store = [&](int buf) {
      char* ah = smem + buf * BUF;
#pragma unroll
      for (int i = 0; i < WM; ++i) gg_store<AKC, F16, SPLIT && !A16>(ah + 64 * i * PITCH, ah + AT + 64 * i * PITCH, ra + 8 * i, tid);
#pragma unroll
      for (int j = 0; j < WN; ++j)
        gg_store<BKC, F16, SPLIT>(ah + 2 * AT + 64 * j * PITCH, ah + 2 * AT + BT + 64 * j * PITCH, rb + 8 * j, tid);
    };

    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[i][j] = splat(0.f);
    if (nst > 0) {
      load(0);
      store(0);
    }
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
      const bool more = st + 1 < nst;
      if (more) load(st + 1);
      const char* ah = smem + (st & 1) * BUF;
      const char* al = ah + AT;
      const char* bh = ah + 2 * AT;
      const char* bl = bh + BT;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        frag fah[WM], fal[WM], fbh[WN], fbl[WN];
#pragma unroll
        for (int i = 0; i < WM; ++i) {
          const int oa = (wm * 32 * WM + 32 * i + l32) * PITCH + (2 * s + hh) * 16;
          fah[i] = lds_frag(ah, oa);
          fal[i] = (SPLIT && !A16) ? lds_frag(al, oa) : fah[i];
        }
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          const int ob = (wn * 32 * WN + 32 * j + l32) * PITCH + (2 * s + hh) * 16;
          fbh[j] = lds_frag(bh, ob);
          fbl[j] = SPLIT ? lds_frag(bl, ob) : fbh[j];
        }
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            if constexpr (A16) mma_xa<PREC>(acc[i][j], fah[i], fbh[j], fbl[j]);
            else mma<PREC>(acc[i][j], fah[i], fal[i], fbh[j], fbl[j]);
          }
      }
      if (more) store((st + 1) & 1);
      __syncthreads();
    }

    // ---- epilogue
    const long dbase = (long)z * a.sDz + (long)zp * a.sDp + (long)zq * a.sDq;
    const float* bias = a.bias ? a.bias + (long)zp * a.sbp + (long)zq * a.sbq : nullptr;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int n = n0 + wn * 32 * WN + 32 * j + l32;
      float cs = 0.f;
      if (n < a.N) {
        const float bn = bias ? bias[n] : 0.f;
        const bool hi_n = a.Nsplit && n >= a.Nsplit;
        uint4 dq = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * 32 * WM + 32 * i + acc_row(r, hh);
            if (dr.thr && (r & 3) == 0) dq = edge_words(dr, zp, m, n, a.drop_t);  // rows m .. m + 3
            if (m >= a.M) continue;
            float x = gs.alpha * acc[i][j][r] + bn;
            if (a.epi == GG_EPI_SIGMOID) x = sigm(x);
            else if (a.epi == GG_EPI_TANH) x = tanh_f(x);
            if (dr.thr) x = drop_apply(dr, u4_get(dq, r & 3), x);
            const long doff = dbase + (long)m * (hi_n && a.sD2m ? a.sD2m : a.sDm) + (long)(hi_n ? n - a.Nsplit : n) * a.sDn;
            if (a.E) x *= a.E[doff];
            cs += x;
            float* d = (hi_n ? a.D2 : a.D) + doff;
            if (a.mode == GG_ATOMIC) {
              if (a.slab) a.slab[(long)z * a.sSlab + (long)m * a.N + n] = x;
              else atomicAdd(d, x);
            } else if (a.mode == GG_ADD) *d += x;
            else *d = x;
          }
      }
      if (a.csum) {
        cs += __shfl_xor(cs, 32);
        if (hh == 0 && n < a.N) {
          if (a.cpart) csum_part(a, z, m0 + wm * 32 * WM, WM, n, cs);
          else atomicAdd(a.csum + (long)zp * a.scp + (long)zq * a.scq + n, cs);
        }
      }
    }
    __syncthreads();  // the next z's prologue rewrites buffer 0
  }
}

// ---- deterministic split-K reduction of slab partials (GemmArgs::slab):
// group g's output (m, n) at D + g * sDg + m * sDm + n = (add ? D : 0) + the sum
// of the partials of g's z's in (t, z) order, t < nt (slab z of t at
// t * zT + z; nt = 1 for a product's own slab): z in [zs[g] / zsdiv,
// zs[g+1] / zsdiv) (zs set) or [g * zper, (g + 1) * zper); z skipped where
// zmask[z] == 0; sole: a group of one z stored its outputs itself (pair dW,
// zmask 2) and is left alone; a group with no z writes nothing when adding,
// zeros otherwise.
struct SlabRed {
  const float* slab;
  long sSlab, zT;
  float* D;
  long sDg, sDm;
  int M, N, G, zper, zsdiv, nt;
  const int* zs;
  const unsigned char* zmask;
  int sole, add;
  const uint32_t* ugmax;  // if set: the sums are multiplied by gunscale (ggnn_common.h)
};
// Segment sums (slab_reduce_t: group g's z in [zs[g] / zsdiv, zs[g+1] / zsdiv)
// over nt timestep slab sets): one wave per output piece of V columns, its
// 64 lanes taking the group's (timestep, z) items lane-strided, each in order,
// then a fixed butterfly across the lanes -- deterministic.  k_slab_reduce's
// one thread per piece walked a whole segment serially: the pair dbeta of a
// b = 256 batch, up to ~400 items per channel, took ~0.1 ms (round 5).
template <int V>
__global__ void __launch_bounds__(256) k_seg_reduce(SlabRed r) {
  const int lane = threadIdx.x & 63;
  const long e = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * V;
  const int g = blockIdx.y;
  if (e >= (long)r.M * r.N) return;  // (a whole wave)
  const int z0 = r.zs[g] / r.zsdiv, nz = r.zs[g + 1] / r.zsdiv - z0, items = r.nt * nz;
  float s[V];
#pragma unroll
  for (int v = 0; v < V; ++v) s[v] = 0.f;
  for (int it = lane; it < items; it += 64) {
    const int t = it / nz, z = z0 + (it - t * nz);
    const float* src = r.slab + ((long)t * r.zT + z) * r.sSlab + e;
    if constexpr (V == 4) {
      const float4 q = *(const float4*)src;
      s[0] += q.x; s[1] += q.y; s[2] += q.z; s[3] += q.w;
    } else {
      s[0] += *src;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
    for (int v = 0; v < V; ++v) s[v] += __shfl_xor(s[v], o);
  if (lane) return;
  const float us = gunscale(r.ugmax);
  const int m = (int)(e / r.N), n = (int)(e % r.N);
  float* d = r.D + (long)g * r.sDg + (long)m * r.sDm + n;
#pragma unroll
  for (int v = 0; v < V; ++v) d[v] = r.add ? d[v] + s[v] * us : s[v] * us;
}

// V = 4: four consecutive outputs per thread (N, sDm and sSlab multiples of 4),
// 16-byte loads; the z's are fetched four at a time (their loads issue
// together) and added one by one in z order: the same sums as V = 1
template <int V>
__global__ void __launch_bounds__(256) k_slab_reduce(SlabRed r) {
  const long e = ((long)blockIdx.x * 256 + threadIdx.x) * V;
  const int g = blockIdx.y;
  if (e >= (long)r.M * r.N) return;
  const int z0 = r.zs ? r.zs[g] / r.zsdiv : g * r.zper, z1 = r.zs ? r.zs[g + 1] / r.zsdiv : (g + 1) * r.zper;
  if (r.sole && z1 - z0 == 1) return;
  float s[V];
#pragma unroll
  for (int v = 0; v < V; ++v) s[v] = 0.f;
  bool any = false;
  for (int t = 0; t < r.nt; ++t)
    for (int z = z0; z < z1; z += 4) {
      float x[4][V];
      bool ok[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int zz = z + u;
        ok[u] = zz < z1 && (!r.zmask || r.zmask[zz]);
        const float* src = r.slab + ((long)t * r.zT + (ok[u] ? zz : z0)) * r.sSlab + e;
        if constexpr (V == 4) {
          const float4 q = ok[u] ? *(const float4*)src : make_float4(0.f, 0.f, 0.f, 0.f);
          x[u][0] = q.x; x[u][1] = q.y; x[u][2] = q.z; x[u][3] = q.w;
        } else {
          x[u][0] = ok[u] ? *src : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (ok[u]) {
#pragma unroll
          for (int v = 0; v < V; ++v) s[v] = any ? s[v] + x[u][v] : x[u][v];
          any = true;
        }
    }
  if (!any && r.add) return;
  const float us = gunscale(r.ugmax);
  const int m = (int)(e / r.N), n = (int)(e % r.N);  // (V = 4: the four share row m)
  float* d = r.D + (long)g * r.sDg + (long)m * r.sDm + n;
#pragma unroll
  for (int v = 0; v < V; ++v) d[v] = r.add ? d[v] + s[v] * us : s[v] * us;
}
