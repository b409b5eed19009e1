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
  const float* B;
  float* D;
  const float* bias;    // [N] at zp*sbp + zq*sbq, or null
  long sAp, sAq, sAm, sAk;
  long sBp, sBq, sBk, sBn;
  long sDz, sDp, sDq, sDm, sDn;
  long sbp, sbq;
  // z -> (zp, zq) = (z / zdiv, z % zdiv); z is skipped when zmask && !zmask[z]
  int zdiv;
  const unsigned char* zmask;
  // terms of z: tl == null: one term (zp, zq); else nt = tl[z*ts] terms
  // (zp, tl[z*ts + 1 + e]) (a count-prefixed list, e.g. a graph's channels)
  const int* tl;
  long ts;
  int Z, M, N, K;       // per-term K; term k range [p*sKp, p*sKp + K) clipped to Ktot
  long Ktot, sKp;
  float alpha;
  int epi, mode;
};

namespace gg {
constexpr int BM = 64, BN = 64, BK = 32, NT = 256;
constexpr int PITCH = 80;                  // bytes per LDS row: 32 limbs + 16 B pad
constexpr int TILE = 64 * PITCH;           // one [64][32] limb image
}  // namespace gg

template <int PREC, bool A16, bool AKC, bool BKC>
__global__ void __launch_bounds__(256) k_gemm(GemmArgs a) {
  using namespace gg;
  constexpr bool SPLIT = Prec<PREC>::split, F16 = Prec<PREC>::f16;
  // [buf][A hi, A lo, B hi, B lo]
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int wm = w & 1, wn = w >> 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int kc = (a.K + BK - 1) / BK;

  for (int z = blockIdx.z; z < a.Z; z += gridDim.z) {
    if (a.zmask && !a.zmask[z]) continue;
    const int zp = z / a.zdiv, zq = z % a.zdiv;
    const int nt = a.tl ? a.tl[(long)z * a.ts] : 1;
    const int nst = nt * kc;
    auto term = [&](int e, int& p, int& q) {
      p = zp;
      q = a.tl ? a.tl[(long)z * a.ts + 1 + e] : zq;
    };

    // ---- global -> registers: this thread's 8 A values and 8 B values of a stage
    float ra[8], rb[8];
    auto load = [&](int st) {
      int p, q;
      term(st / kc, p, q);
      const int kk0 = (st % kc) * BK;
      const long kg0 = (long)p * a.sKp + kk0;  // global k of the slice's first column
      // A: AKC -> (row m = tid>>2, 8 k at (tid&3)*8); else (k = tid>>3, 8 m at (tid&7)*8)
      {
        const int mi = AKC ? (tid >> 2) : (tid & 7) * 8;
        const int ki = AKC ? (tid & 3) * 8 : (tid >> 3);
        const long base = p * a.sAp + q * a.sAq;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int m = m0 + mi + (AKC ? 0 : j), kk = kk0 + ki + (AKC ? j : 0);
          const long kg = kg0 + ki + (AKC ? j : 0);
          float x = 0.f;
          if (m < a.M && kk < a.K && kg < a.Ktot) {
            const long off = base + m * a.sAm + kk * a.sAk;
            if constexpr (A16) x = from_limb<F16>(((const u16*)a.A)[off]);
            else x = ((const float*)a.A)[off];
          }
          ra[j] = x;
        }
      }
      // B: BKC -> (col n = tid>>2, 8 k at (tid&3)*8); else (k = tid>>3, 8 n at (tid&7)*8)
      {
        const int ni = BKC ? (tid >> 2) : (tid & 7) * 8;
        const int ki = BKC ? (tid & 3) * 8 : (tid >> 3);
        const long base = p * a.sBp + q * a.sBq;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int n = n0 + ni + (BKC ? 0 : j), kk = kk0 + ki + (BKC ? j : 0);
          const long kg = kg0 + ki + (BKC ? j : 0);
          float x = 0.f;
          if (n < a.N && kk < a.K && kg < a.Ktot) x = a.B[base + n * a.sBn + kk * a.sBk];
          rb[j] = x;
        }
      }
    };
    // ---- registers -> LDS limb images ([row][k], k contiguous)
    auto store = [&](int buf) {
      char* ah = smem + buf * 4 * TILE;
      char* al = ah + TILE;
      char* bh = ah + 2 * TILE;
      char* bl = ah + 3 * TILE;
      if constexpr (AKC) {
        const int o = (tid >> 2) * PITCH + (tid & 3) * 16;
        st16(ah + o, pk8<F16>(ra));
        if constexpr (SPLIT && !A16) st16(al + o, pk8_lo<true>(ra));
      } else {
        const int k = tid >> 3, mb = (tid & 7) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int o = (mb + j) * PITCH + k * 2;
          *(u16*)(ah + o) = to_limb<F16>(ra[j]);
          if constexpr (SPLIT && !A16) *(u16*)(al + o) = to_limb<true>(lo_part<true>(ra[j]));
        }
      }
      if constexpr (BKC) {
        const int o = (tid >> 2) * PITCH + (tid & 3) * 16;
        st16(bh + o, pk8<F16>(rb));
        if constexpr (SPLIT) st16(bl + o, pk8_lo<true>(rb));
      } else {
        const int k = tid >> 3, nb = (tid & 7) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int o = (nb + j) * PITCH + k * 2;
          *(u16*)(bh + o) = to_limb<F16>(rb[j]);
          if constexpr (SPLIT) *(u16*)(bl + o) = to_limb<true>(lo_part<true>(rb[j]));
        }
      }
    };

    f32x16 acc = splat(0.f);
    if (nst > 0) {
      load(0);
      store(0);
    }
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
      const bool more = st + 1 < nst;
      if (more) load(st + 1);
      const char* ah = smem + (st & 1) * 4 * TILE;
      const char* al = ah + TILE;
      const char* bh = ah + 2 * TILE;
      const char* bl = ah + 3 * TILE;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        const int oa = (wm * 32 + l32) * PITCH + (2 * s + hh) * 16;
        const int ob = (wn * 32 + l32) * PITCH + (2 * s + hh) * 16;
        const frag fah = lds_frag(ah, oa), fbh = lds_frag(bh, ob);
        const frag fbl = SPLIT ? lds_frag(bl, ob) : fbh;
        if constexpr (A16) {
          mma_xa<PREC>(acc, fah, fbh, fbl);
        } else {
          const frag fal = SPLIT ? lds_frag(al, oa) : fah;
          mma<PREC>(acc, fah, fal, fbh, fbl);
        }
      }
      if (more) store((st + 1) & 1);
      __syncthreads();
    }

    // ---- epilogue
    const long dbase = (long)z * a.sDz + (long)zp * a.sDp + (long)zq * a.sDq;
    const float* bias = a.bias ? a.bias + (long)zp * a.sbp + (long)zq * a.sbq : nullptr;
    const int n = n0 + wn * 32 + l32;
    if (n < a.N) {
      const float bn = bias ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 + acc_row(r, hh);
        if (m >= a.M) continue;
        float x = a.alpha * acc[r] + bn;
        if (a.epi == GG_EPI_SIGMOID) x = sigm(x);
        else if (a.epi == GG_EPI_TANH) x = tanh_f(x);
        float* d = a.D + dbase + (long)m * a.sDm + (long)n * a.sDn;
        if (a.mode == GG_ATOMIC) atomicAdd(d, x);
        else if (a.mode == GG_ADD) *d += x;
        else *d = x;
      }
    }
    __syncthreads();  // the next z's prologue rewrites buffer 0
  }
}
