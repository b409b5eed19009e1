// k_gemm_ring.h -- the general path's product kernel for aligned operands
// (same GemmArgs contract as k_gemm, k_gemm.h).
//
// k_gemm stages every 64 x 32 operand slice through VGPRs with one slice in
// flight per workgroup; at 4096^3 it reached 115 TFLOP/s in the split mode
// and 107 in bf16 (tools/gemm_probe.py): latency-bound on its operand reads,
// not on the MFMAs.  This kernel instead:
//   * takes 128 x 128 block tiles (4 waves in 2 x 2, 64 x 64 outputs each:
//     four v_mfma_f32_32x32x16 accumulators), half the operand bytes per flop;
//   * DMAs raw operand K-slices (fp32, or the exact 16-bit adjacency) straight
//     into an LDS ring with global_load_lds_dwordx4 -- no VGPR staging,
//     completion counted by hand (vmcnt + s_barrier).  Two slots (64 KiB, two
//     workgroups per CU) measured 1.4-2x faster than four slots (three slices
//     in flight, one workgroup per CU);
//   * converts on the LDS -> register path: each wave reads its fragments'
//     8 fp32 values and forms the precision policy's limbs (split: f16 hi/lo)
//     right before the MFMAs, so there is no second LDS image and one barrier
//     per slice.
// Out-of-range rows / k cost no branches in the MFMA loop: row addresses are
// clamped into the operand (their outputs are discarded), and a chunk whose k
// lies past the term's K is DMA'd from a zero block instead, so both operands
// carry zeros there.  K is a multiple of the chunk (4 fp32) for fp32
// k-contiguous operands; a 16-bit operand's columns between K and the next
// multiple of 8 must hold zeros (the staged adjacency's padding does).
//
// Slice images (one ring slot = A image, then B image):
//   k-contiguous fp32  [128 rows][32 k]: 128 B rows, 16-B chunk c of row r at
//                      slot c ^ ((r >> 1) & 7) -- 16 consecutive rows of one
//                      fragment read hit 16 distinct 4-bank groups;
//   k-contiguous u16   [128 rows][32 k]: 64 B rows, chunk c at c ^ ((r >> 2) & 3);
//   row-contiguous fp32 [32 k][128 rows]: 512 B k-rows, chunk c (4 rows) at
//                      c ^ (8 * ((k >> 3) & 1)) -- the two lane halves of a
//                      fragment (k and k + 8) read opposite bank halves.
#pragma once
#include "k_gemm.h"

__device__ __attribute__((aligned(16))) const float g_ring_zero[4] = {0.f, 0.f, 0.f, 0.f};

namespace gr {
constexpr int BM = 128, BN = 128, BK = 32, NT = 256;

DEV int kc32_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
DEV int kc16_off(int r, int c) { return r * 64 + ((c ^ ((r >> 2) & 3)) << 4); }
DEV int rc32_off(int kr, int r) { return kr * 512 + (((r >> 2) ^ (((kr >> 3) & 1) << 3)) << 4) + ((r & 3) << 2); }

// 8 fp32 of image row r at k0 .. k0 + 7 (k0 a multiple of 8)
template <bool KC>
DEV void rd8(const char* img, int r, int k0, float* x) {
  if constexpr (KC) {
    const int c = k0 >> 2;
    const float4 p = *(const float4*)(img + kc32_off(r, c));
    const float4 q = *(const float4*)(img + kc32_off(r, c + 1));
    x[0] = p.x; x[1] = p.y; x[2] = p.z; x[3] = p.w;
    x[4] = q.x; x[5] = q.y; x[6] = q.z; x[7] = q.w;
  } else {
    const char* b = img + rc32_off(k0, r);  // (k0 >> 3) & 1 is the same for k0 .. k0 + 7
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = *(const float*)(b + j * 512);
  }
}
}  // namespace gr

// blockIdx.x -> (z, m tile, n tile): consecutive dispatch ids go round-robin
// over the 8 XCDs (private L2 each), so ids are first remapped bijectively
// (guide T1) to give every XCD a contiguous run of the logical order, and the
// logical order walks groups of GM m-tiles with n fastest inside a group: the
// ~32 tiles an XCD holds at once share a few A row-panels and B column-panels.
DEV void ring_tile(int nwg, int tm, int tn, int& z, int& mt, int& nt) {
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per = tm * tn;
  z = lin / per;
  const int t = lin - z * per;
  constexpr int GM = 4;
  const int g = t / (GM * tn), m0 = g * GM, gs = min(tm - m0, GM);
  const int u = t - g * GM * tn;
  mt = m0 + u % gs;
  nt = u / gs;
}

// BMT: block rows, 128 (4 waves in 2 x 2, 64 x 64 each) or 32 (4 waves in
// 1 x 4, 32 x 32 each: products whose M is one small graph's node count, e.g.
// v = 30 sentence graphs, where a 128-row tile would spend 3/4 of its MFMAs and
// A bytes on padding rows; k-contiguous A only)
// TGRP: per-timestep term groups (GemmArgs::tgroups): the accumulator is masked
// and banked at each group's end, the epilogue stores the bank.  It asks for 2
// waves per EU (two workgroups per CU: 238 VGPRs, no AGPRs; at 1 it held 249 +
// 64 AGPRs, one workgroup per CU, 1.37 vs 0.95 ms) and banks from ONE call site
// (the unrolled slot loop inlined it twice).
// LEAN: the host guarantees plain stores (GG_STORE, or GG_ATOMIC into a slab /
// a sole chunk) with no activation, dropout or column split (an E factor and a
// bias are taken): only the lean epilogue is compiled, and the kernel asks for
// 2 waves per EU
template <int PREC, bool A16, bool AKC, bool BKC, bool SCALE, int NBUF, int BMT, bool TGRP = false, bool LEAN = false>
__global__ void __launch_bounds__(256, TGRP || LEAN ? 2 : 1) k_gemm_ring(GemmArgs a, int tm, int tn) {
  const Drop dr = drop_resolve(a.dr);  // (a device-resident key: loaded once)
  using namespace gr;
  constexpr bool SPLIT = Prec<PREC>::split, F16 = Prec<PREC>::f16;
  static_assert(!A16 || AKC, "16-bit A operands are k-contiguous");
  static_assert(BMT == 128 || (BMT == 32 && AKC), "32-row tiles: k-contiguous A only");
  const GemmScales gs = gemm_scales(a);
  constexpr int BM = BMT;
  constexpr int WMW = BMT == 128 ? 2 : 1, WNW = 4 / WMW;  // wave grid
  constexpr int AM = BMT / (32 * WMW), AN = BN / (32 * WNW);  // accumulators per wave
  constexpr int ES = A16 ? 2 : 4;                       // A element bytes
  constexpr int AB = BM * BK * ES;                      // A slice image bytes
  constexpr int BB = BN * BK * 4;
  constexpr int NA = AB / 1024;                         // A wave-instructions per slice
  constexpr int GA = (NA + 3) / 4, GB = BB / 1024 / 4;  // DMA instructions per wave per slice
  constexpr bool AJUNK = GA * 4 > NA;                   // waves past the A image DMA a dummy chunk
  constexpr int SB = AB + BB + (AJUNK ? 1024 : 0);
  constexpr int GPW = GA + GB;
  // one __shared__ object per ring slot, addressed with compile-time indices
  // (NBUF = 4: three slices in flight, one workgroup per CU; NBUF = 2: one
  // slice in flight, 64 KiB, two workgroups per CU)
  static_assert(NBUF == 2 || NBUF == 4, "ring depth");
  __shared__ __attribute__((aligned(16))) char s0[SB], s1[SB], s2[NBUF > 2 ? SB : 16], s3[NBUF > 2 ? SB : 16];
  auto slot = [&](int u) -> char* { return u == 0 ? s0 : u == 1 ? s1 : u == 2 ? s2 : s3; };
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int wm = w % WMW, wn = w / WMW;
  int z, mt, ntile;
  if constexpr (TGRP) {
    // term groups (the pair dW: z = a chunk of one channel's tiles, chunks of
    // very different lengths in channel order): whole z's round-robin over
    // the 8 XCDs (z % 8 = the XCD), a z's output tiles together on its XCD
    // (they share its operand rows).  ring_tile's contiguous runs of z per
    // XCD piled the heavy channels' chunks onto one or two XCDs.  The host
    // rounds the grid up to a multiple of 8 z's.
    const int bid = blockIdx.x, per = tm * tn, q8 = bid >> 3;
    z = (bid & 7) + 8 * (q8 / per);
    const int t = q8 - (q8 / per) * per;
    mt = t / tn;
    ntile = t - mt * tn;
  } else {
    ring_tile(gridDim.x, tm, tn, z, mt, ntile);
  }
  const int tsk = a.tsprobe - 1;
  if (tsk >= 0) TSMARK(tsk, 0);
  if (z >= a.Z) return;
  // zmask[z]: 0 skip z, 1 live, 2 live and the only z writing its outputs
  // (GG_ATOMIC then stores: the pair dW chunk that is its channel's only one)
  const unsigned zm = a.zmask ? a.zmask[z] : 1u;
  if (!zm) return;
  const bool sole = zm == 2;
  const int n0 = ntile * BN, m0 = mt * BM;
  // a wave whose whole row or column slice lies past M / N (the last tile of
  // N = 400: 16 of its 128 columns valid) still moves its share of every slice
  // and meets every barrier, but reads no fragments and issues no MFMAs
  const bool live = __builtin_amdgcn_readfirstlane((int)(n0 + wn * AN * 32 < a.N && m0 + wm * AM * 32 < a.M));
  const int kc = (a.K + BK - 1) / BK;
  const int zp = a.zmap ? a.zmap[z] : z / a.zdiv, zq = a.zmap ? 0 : z % a.zdiv;
  const int nterms = a.tl ? a.tl[(long)z * a.ts] : max(a.nterm, 1);
  const int nit = nterms * kc;
  // z's first 128 terms in two VGPRs (lane l: terms l and 64 + l), fetched
  // by v_readlane: a global or LDS read of the list inside the ring would come
  // with a vmcnt(0) wait that drains the DMAs in flight
  int tl0 = 0, tl1 = 0;
  if (a.tl) {
    const int* tz = a.tl + (long)z * a.ts + 1;
    if (lane < nterms) tl0 = tz[lane];
    if (64 + lane < nterms) tl1 = tz[64 + lane];
  }
  asm volatile("" : "+v"(tl0), "+v"(tl1));  // the loads' wait goes here, before the ring
  const int keff = (int)min((long)a.K, a.Ktot - (long)zp * a.sKp);  // valid k of every term of z

  // ---- per-lane DMA source of every chunk this wave moves, at the term's
  // k = 0 (rebuilt when a new term starts); a slice adds kk0 * kstep
  const char* pa[GA];
  const char* pb[GB];
  int ka[GA], kb[GB];  // chunk k offset inside the slice (KC) or k-row (row-contiguous)
  auto term_bases = [&](int e) {
    const int q = !a.tl ? zq + e
                  : e < 64 ? __builtin_amdgcn_readlane(tl0, e)
                  : e < 128 ? __builtin_amdgcn_readlane(tl1, e - 64)
                            : a.tl[(long)z * a.ts + 1 + e];
    const bool second = a.A2 && q == 1;
    const long abase = (long)zp * a.sAp + (second ? 0 : (long)q * a.sAq);
    const char* A1 = (const char*)(second ? a.A2 : a.A);
#pragma unroll
    for (int g = 0; g < GA; ++g) {
      const int qs = (g * 4 + w) * 64 + lane;
      int row;
      if constexpr (A16) {
        row = qs >> 2;
        ka[g] = ((qs & 3) ^ ((row >> 2) & 3)) << 3;
      } else if constexpr (AKC) {
        row = qs >> 3;
        ka[g] = ((qs & 7) ^ ((row >> 1) & 7)) << 2;
      } else {
        ka[g] = qs >> 5;
        row = ((qs & 31) ^ (((ka[g] >> 3) & 1) << 3)) << 2;
      }
      int mg = m0 + row;
      const char* P = A1;
      int lim = a.Msplit ? a.Msplit : a.M;
      if (a.Msplit && mg >= a.Msplit) {
        P = (const char*)a.Am2;
        mg -= a.Msplit;
        lim = a.M - a.Msplit;
      }
      mg = AKC ? min(mg, lim - 1) : min(mg, (lim - 1) & ~3);
      pa[g] = P + (abase + (long)mg * a.sAm) * ES;
    }
    const long bbase = (long)zp * a.sBp + (long)q * a.sBq;
#pragma unroll
    for (int g = 0; g < GB; ++g) {
      const int qs = (g * 4 + w) * 64 + lane;
      int row;
      if constexpr (BKC) {
        row = qs >> 3;
        kb[g] = ((qs & 7) ^ ((row >> 1) & 7)) << 2;
        row = min(n0 + row, a.N - 1);
      } else {
        kb[g] = qs >> 5;
        row = min(n0 + (((qs & 31) ^ (((kb[g] >> 3) & 1) << 3)) << 2), (a.N - 1) & ~3);
      }
      pb[g] = (const char*)a.B + (bbase + (long)row * a.sBn) * 4;
    }
  };

  // ---- DMA of slice `it` (term it / kc, k offset (it % kc) * BK) into ring slot `buf`
  auto stage = [&](int it, char* buf) {
    const int j = it % kc, kk0 = j * BK;
    if (j == 0) term_bases(it / kc);
    const char* zero = (const char*)g_ring_zero;
#pragma unroll
    for (int g = 0; g < GA; ++g) {
      const int k = kk0 + ka[g];
      const char* src = AKC ? pa[g] + (long)k * ES : pa[g] + (long)k * a.sAk * 4;
      const int qi = g * 4 + w;  // A wave-instruction index (>= NA: dummy into the junk chunk)
      glds16_asm(k < keff ? src : zero, buf + (AJUNK && qi >= NA ? AB + BB : qi * 1024));
    }
#pragma unroll
    for (int g = 0; g < GB; ++g) {
      const int k = kk0 + kb[g];
      const char* src = BKC ? pb[g] + (long)k * 4 : pb[g] + (long)k * a.sBk * 4;
      glds16_asm(k < keff ? src : zero, buf + AB + (g * 4 + w) * 1024);
    }
  };

  f32x16 acc[AM][AN];
#pragma unroll
  for (int i = 0; i < AM; ++i)
#pragma unroll
    for (int j = 0; j < AN; ++j) acc[i][j] = splat(0.f);
  // TGRP: the masked sum of the finished groups
  f32x16 bank[TGRP ? AM : 1][TGRP ? AN : 1];
  if constexpr (TGRP) {
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
      for (int j = 0; j < AN; ++j) bank[i][j] = splat(0.f);
  }

  // ---- MFMAs of the slice in ring slot `buf` (straight-line: the LDS reads
  // of both k-steps issue together)
  auto compute = [&](const char* buf) {
    const char* ia = buf;
    const char* ib = buf + AB;
    const float sa = gs.sa, sb = gs.sb;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int k0 = 16 * s + 8 * hh;
      frag ah[AM], al[AM], bh[AN], bl[AN];
#pragma unroll
      for (int i = 0; i < AM; ++i) {
        const int r = wm * AM * 32 + i * 32 + l32;
        if constexpr (A16) {
          ah[i] = *(const frag*)(ia + kc16_off(r, k0 >> 3));
          al[i] = ah[i];
        } else {
          float x[8];
          rd8<AKC>(ia, r, k0, x);
          if constexpr (SCALE)
#pragma unroll
            for (int t = 0; t < 8; ++t) x[t] *= sa;
          ah[i] = pk8<F16>(x);
          al[i] = SPLIT ? pk8_lo<true>(x) : ah[i];
        }
      }
#pragma unroll
      for (int j = 0; j < AN; ++j) {
        const int r = wn * AN * 32 + j * 32 + l32;
        float x[8];
        rd8<BKC>(ib, r, k0, x);
        if constexpr (SCALE)
#pragma unroll
          for (int t = 0; t < 8; ++t) x[t] *= sb;
        bh[j] = pk8<F16>(x);
        bl[j] = SPLIT ? pk8_lo<true>(x) : bh[j];
      }
#pragma unroll
      for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j) {
          if constexpr (A16) mma_xa<PREC>(acc[i][j], ah[i], bh[j], bl[j]);
          else mma<PREC>(acc[i][j], ah[i], al[i], bh[j], bl[j]);
        }
    }
  };

  // ---- TGRP: group tg (timestep tg) done: bank += mask_tg * acc, acc = 0.
  // The group's mask words (GemmArgs::mbits, the pack's keep bits) are loaded
  // at its first slice (mw: this lane's 32-row word per accumulator tile);
  // drawing Philox words here, per 128 x 128 tile and timestep, was most of the
  // kernel's issue at small batches and spilled at 2 waves per EU
  const int gsz = TGRP ? nit / max(a.tgroups, 1) : 0;
  uint32_t mw[TGRP ? AM : 1][TGRP ? AN : 1];
  auto load_masks = [&](int tg) {
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
      for (int j = 0; j < AN; ++j) {
        const int n = n0 + wn * AN * 32 + 32 * j + l32, mb = m0 + wm * AM * 32 + 32 * i;
        mw[i][j] = (n < a.N && mb < a.M) ? a.mbits[(((long)tg * a.mbC + zp) * a.N + n) * a.mbw + (mb >> 5)] : 0u;
      }
  };
  auto bank_group = [&]() {
#pragma unroll
    for (int j = 0; j < AN; ++j)
#pragma unroll
      for (int i = 0; i < AM; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float x = acc[i][j][r];
          bank[i][j][r] += !a.mbits ? x : ((mw[i][j] >> (acc_row(r, hh) & 31)) & 1u) ? x * dr.scale : 0.0f;
        }
        acc[i][j] = splat(0.f);
      }
  };

  // ---- the ring: slices it+1, it+2 stay in flight while slice it is consumed
  if (tsk >= 0) {
    TSMARK(tsk, 1);
    TSVAL(tsk, 5, nit);
    TSVAL(tsk, 6, z);
  }
#pragma unroll
  for (int u = 0; u < NBUF - 1; ++u)
    if (u < nit) stage(u, slot(u));
  if constexpr (TGRP && NBUF == 2) {
    // one call site of the masked banking (the unrolled slot loop inlined it
    // twice): the slot is picked at run time
    for (int it = 0; it < nit; ++it) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's DMAs of slice it landed; slice it-1 fully read
      // (issued ahead of the slice's DMAs: the compiler's wait before their
      // use at the group's end is a vmcnt(0) that also covers those)
      if constexpr (TGRP)
        if (a.mbits && live && gsz > 0 && it % gsz == 0) load_masks(it / gsz);
      if (it + 1 < nit) stage(it + 1, (it & 1) ? s0 : s1);
      if (live) {
        compute((it & 1) ? s1 : s0);
        if constexpr (TGRP)
          if (gsz > 0 && (it + 1) % gsz == 0) bank_group();
      }
    }
  } else
  for (int it0 = 0; it0 < nit; it0 += NBUF) {
#pragma unroll
    for (int u = 0; u < NBUF; ++u) {
      const int it = it0 + u;
      if (it < nit) {
        if (NBUF > 2 && it + 2 < nit) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory");
        else if (NBUF > 2 && it + 1 < nit) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's DMAs of slice it landed; slice it-1 fully read
        if constexpr (TGRP)
          if (a.mbits && live && gsz > 0 && it % gsz == 0) load_masks(it / gsz);
        if (it + NBUF - 1 < nit) stage(it + NBUF - 1, slot((u + NBUF - 1) % NBUF));
        if (live) {
          compute(slot(u));
          if constexpr (TGRP)
            if (gsz > 0 && (it + 1) % gsz == 0) bank_group();
        }
      }
    }
  }
  if (tsk >= 0) TSMARK(tsk, 2);
  const long dbase = (long)z * a.sDz + (long)zp * a.sDp + (long)zq * a.sDq;
  const float* bias = a.bias ? a.bias + (long)zp * a.sbp + (long)zq * a.sbq : nullptr;
  // Plain stores (GG_STORE, a sole chunk, a split-K slab) with no activation,
  // dropout, E factor or column split take a lean epilogue: the general one
  // below unrolls every option's code for each of the 64 accumulator elements
  // (~11k instructions with the Philox draws), and walking it cost 14-16 us per
  // workgroup -- more than the K loop at the 20-sentence batch's split-K and
  // pair products (round 5, tools/ts_probe_generic.py).  Row-major outputs
  // (unit column stride, 16-byte aligned rows) go through LDS: each wave
  // parks its tile row-major (XOR-swizzled 16-byte chunks) and stores whole
  // 16-byte row pieces, a quarter of the store instructions -- a workgroup's
  // scalar stores of a 128 x 128 tile took ~8 us, one outstanding-store
  // window after another.  Same arithmetic, same bits.
  const bool to_slab = a.mode == GG_ATOMIC && !sole;
  // (LEAN instances, chosen by the host, and the term-group products; the
  // other instances keep only the general epilogue: the lean one's registers
  // on top cost them their second workgroup per CU -- 256 VGPRs + 85 AGPRs
  // against round 4's 188 + 64, +30-50 % at b = 256, round 5)
  const bool lean = LEAN || (TGRP && !a.E && a.epi == GG_EPI_NONE && !a.Nsplit &&
                             (a.mode == GG_STORE || sole || (to_slab && a.slab)));
  if constexpr (LEAN || TGRP) if (lean) {
    float* const Db = to_slab ? a.slab + (long)z * a.sSlab : a.D + dbase;
    const long sm = to_slab ? (long)a.N : a.sDm, sn = to_slab ? 1 : a.sDn;
    constexpr int WR = AM * 32, WC = AN * 32, C4 = WC / 4;  // a wave's tile, its 16-byte chunks per row
    // (the parked tiles take both ring slots at 128-row tiles, one at 32)
    constexpr bool PARK_OK = BMT == 128 ? SB >= 2 * WR * WC * 4 : SB >= 4 * WR * WC * 4;
    const bool vec = PARK_OK && sn == 1 && a.N % 4 == 0 && sm % 4 == 0 && ((uintptr_t)Db & 15) == 0;
    if (vec) __syncthreads();  // every wave is done with the ring: its slots take the tiles
    if (!live) return;
    float* const park = BMT == 128 ? (float*)(w < 2 ? s0 : s1) + (w & 1) * WR * WC : (float*)s0 + w * WR * WC;
    auto pk_off = [&](int row, int col) { return row * WC + ((((col >> 2) ^ row) & (C4 - 1)) << 2) + (col & 3); };
#pragma unroll
    for (int j = 0; j < AN; ++j) {
      const int n = n0 + wn * AN * 32 + 32 * j + l32;
      float cs = 0.f;
      if (n < a.N) {
        const float bn = bias ? bias[n] : 0.f;
        float* const Dc = Db + (long)n * sn;
        // E factors (the heads' dropout-scaled weight gradient) at D's
        // coordinates, loaded up front (the stores below may alias them)
        float ef[LEAN ? AM : 1][16];
        if constexpr (LEAN)
          if (a.E) {
            const float* Ec = a.E + dbase + (long)n * a.sDn;
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
              for (int r = 0; r < 16; ++r)
                ef[i][r] = Ec[(long)min(m0 + wm * AM * 32 + 32 * i + acc_row(r, hh), a.M - 1) * a.sDm];
          }
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rl = 32 * i + acc_row(r, hh), m = m0 + wm * AM * 32 + rl;
            float x = gs.alpha * (TGRP ? bank[i][j][r] : acc[i][j][r]) + bn;
            if constexpr (LEAN)
              if (a.E) x *= ef[i][r];
            if (m < a.M) cs += x;
            if (vec) park[pk_off(rl, 32 * j + l32)] = x;
            else if (m < a.M) Dc[(long)m * sm] = x;
          }
      }
      if (a.csum) {
        cs += __shfl_xor(cs, 32);
        if (hh == 0 && n < a.N) {
          if (a.cpart) csum_part(a, z, m0 + wm * AM * 32, AM, n, cs);
          else atomicAdd(a.csum + (long)zp * a.scp + (long)zq * a.scq + n, cs);
        }
      }
    }
    if (vec) {
      __builtin_amdgcn_wave_barrier();  // (the wave's own LDS writes, in order)
      const int mw0 = m0 + wm * AM * 32, nw0 = n0 + wn * AN * 32;
#pragma unroll
      for (int q = 0; q < WR * C4 / 64; ++q) {
        const int idx = q * 64 + lane, rl = idx / C4, c4 = idx % C4;
        const int m = mw0 + rl, n = nw0 + 4 * c4;
        if (m < a.M && n < a.N)
          *(float4*)(Db + (long)m * sm + n) = *(const float4*)(park + rl * WC + (((c4 ^ rl) & (C4 - 1)) << 2));
      }
    }
    if (tsk >= 0) TSMARK(tsk, 3);
    return;
  }
  if constexpr (LEAN) return;  // (the lean epilogue above took every case)
  if (!live) return;  // nothing of this wave's to store (no barrier follows)

  // ---- epilogue (as k_gemm)
  constexpr bool EPI_PRE = !TGRP && !A16;  // (masked dW products: atomics only; adjacency products: kept at 3 workgroups per CU)
#pragma unroll
  for (int j = 0; j < AN; ++j) {
    const int n = n0 + wn * AN * 32 + 32 * j + l32;
    float cs = 0.f;
    if (n < a.N) {
      const float bn = bias ? bias[n] : 0.f;
      const bool hi_n = a.Nsplit && n >= a.Nsplit;
      float* const Dn = hi_n ? a.D2 : a.D;
      const long sm = hi_n && a.sD2m ? a.sD2m : a.sDm, dn = dbase + (long)(hi_n ? n - a.Nsplit : n) * a.sDn;
      // the column's E factors / old D values (GG_ADD) loaded up front: read
      // one at a time between the stores, each waited for its own round trip
      // (the compiler cannot move a load past a store that may alias it), 64
      // serialised latencies per lane at 128 rows (E and GG_ADD never meet:
      // gg_launch refuses the pair)
      float pre[EPI_PRE ? AM : 1][16];
      const bool ld = a.E || a.mode == GG_ADD;
      if (EPI_PRE && ld) {
        const float* src = a.E ? a.E : Dn;
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = min(m0 + wm * AM * 32 + 32 * i + acc_row(r, hh), a.M - 1);
            pre[i][r] = src[dn + (long)m * sm];
          }
      }
      uint4 dq = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * AM * 32 + 32 * i + acc_row(r, hh);
          if (!TGRP && dr.thr && (r & 3) == 0) dq = edge_words(dr, zp, m, n, a.drop_t);  // rows m .. m + 3
          if (m >= a.M) continue;
          float x = gs.alpha * (TGRP ? bank[i][j][r] : acc[i][j][r]) + bn;
          if (a.epi == GG_EPI_SIGMOID) x = sigm(x);
          else if (a.epi == GG_EPI_TANH) x = tanh_f(x);
          if (!TGRP && dr.thr) x = drop_apply(dr, u4_get(dq, r & 3), x);
          const long doff = dn + (long)m * sm;
          if (a.E) x *= EPI_PRE ? pre[EPI_PRE ? i : 0][r] : a.E[doff];
          cs += x;
          float* d = Dn + doff;
          if (a.mode == GG_ATOMIC && !sole) {
            // (128-row tiles of fp32 operands: slab products always take the
            // lean epilogue -- gg_launch sends them to the LEAN instances --
            // and this one keeps round 4's registers: 188 VGPRs + 64 AGPRs,
            // two workgroups per CU)
            if (A16 || BMT != 128) {
              if (a.slab) a.slab[(long)z * a.sSlab + (long)m * a.N + n] = x;
              else atomicAdd(d, x);
            } else {
              atomicAdd(d, x);
            }
          }
          else if (a.mode == GG_ADD) *d = (EPI_PRE ? pre[EPI_PRE ? i : 0][r] : *d) + x;
          else *d = x;
        }
    }
    // column sums (GemmArgs::csum): lanes l and l + 32 hold the same column
    if (a.csum) {
      cs += __shfl_xor(cs, 32);
      if (hh == 0 && n < a.N) {
        if (a.cpart) csum_part(a, z, m0 + wm * AM * 32, AM, n, cs);
        else atomicAdd(a.csum + (long)zp * a.scp + (long)zq * a.scq + n, cs);
      }
    }
  }
  if (tsk >= 0) TSMARK(tsk, 3);
}

// ---- k_gemm_ks: 32-row tiles whose K slices are split over the waves (same
// GemmArgs contract; fp32 k-contiguous A).  For products whose 32-row ring
// grid leaves most CUs idle (the GRU and pair products of a 20-sentence batch:
// 100-400 workgroups), where a launch takes one workgroup's time and that is
// a serial walk over K: ~7 us + 0.6 us per 32-deep slice, the slice's cost
// being one wave's LDS-read -> limb-convert -> dependent-MFMA chain, not its
// DMA (a 4-slot ring walked at the same rate; profiles/r04l_small_gemm_trace.txt).
// The 4 waves form WN (columns, 32 each) x WK = 4 / WN (K) groups: wave
// (wn, wk) walks slices wk, wk + WK, ... of columns n0 + 32 wn through a
// private 2-slot LDS ring (8 KiB a slot; its own vmcnt plus one barrier a
// round); the WK partial accumulators of a column block are summed in LDS in
// a fixed order (deterministic), each of the WK waves storing 16 / WK of
// every lane's 16 rows.  WN = 1 (32 x 32 tiles) has the shortest walk and
// re-reads A most; WN = 4 is the ring's 32 x 128 tile without the split.
//   A image [32 m][32 k]: kc32_off;  B k-contiguous [32 n][32 k]: kc32_off;
//   B row-contiguous [32 k][32 n]: k-row k at row (k & 7) * 4 + (k >> 3), so the
//   two lane halves of a fragment read (k and k + 8) sit in opposite bank halves.
namespace gks {
DEV int rcs_row(int k) { return (k & 7) * 4 + (k >> 3); }
}  // namespace gks

template <int PREC, bool BKC, bool SCALE, int WN>
__global__ void __launch_bounds__(256, 2) k_gemm_ks(GemmArgs a, int tm, int tn) {
  const Drop dr = drop_resolve(a.dr);
  using namespace gr;
  constexpr bool SPLIT = Prec<PREC>::split, F16 = Prec<PREC>::f16;
  constexpr int WK = 4 / WN, SLOT = 8192, HALF = 4096;  // one slot: A image, then B image
  static_assert(WN == 1 || WN == 2 || WN == 4, "wave split");
  __shared__ __attribute__((aligned(16))) char ring[4 * 2 * SLOT];
  const GemmScales gs = gemm_scales(a);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int wn = w % WN, wk = w / WN;
  int z, mt, ntile;
  ring_tile(gridDim.x, tm, tn, z, mt, ntile);
  const int tsk = a.tsprobe - 1;
  if (tsk >= 0) TSMARK(tsk, 0);
  if (z >= a.Z) return;
  if (a.zmask && !a.zmask[z]) return;
  const int n0 = ntile * 32 * WN + 32 * wn, m0 = mt * 32;  // n0: this wave's column block
  const int kc = (a.K + BK - 1) / BK;
  const int zp = a.zmap ? a.zmap[z] : z / a.zdiv, zq = a.zmap ? 0 : z % a.zdiv;
  const int nterms = a.tl ? a.tl[(long)z * a.ts] : max(a.nterm, 1);
  const int nit = nterms * kc;
  int tl0 = 0, tl1 = 0;
  if (a.tl) {
    const int* tz = a.tl + (long)z * a.ts + 1;
    if (lane < nterms) tl0 = tz[lane];
    if (64 + lane < nterms) tl1 = tz[64 + lane];
  }
  asm volatile("" : "+v"(tl0), "+v"(tl1));
  const int keff = (int)min((long)a.K, a.Ktot - (long)zp * a.sKp);
  char* const my = ring + w * 2 * SLOT;

  // this wave's DMA sources (4 A + 4 B chunks a lane) at the term's k = 0
  const char* pa[4];
  const char* pb[4];
  int ka[4], kb[4];
  int cur = -1;
  auto term_bases = [&](int e) {
    const int q = !a.tl ? zq + e
                  : e < 64 ? __builtin_amdgcn_readlane(tl0, e)
                  : e < 128 ? __builtin_amdgcn_readlane(tl1, e - 64)
                            : a.tl[(long)z * a.ts + 1 + e];
    const bool second = a.A2 && q == 1;
    const long abase = (long)zp * a.sAp + (second ? 0 : (long)q * a.sAq);
    const char* A1 = (const char*)(second ? a.A2 : a.A);
    const long bbase = (long)zp * a.sBp + (long)q * a.sBq;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int qs = g * 64 + lane, row = qs >> 3;
      ka[g] = ((qs & 7) ^ ((row >> 1) & 7)) << 2;
      int mg = m0 + row;
      const char* P = A1;
      int lim = a.Msplit ? a.Msplit : a.M;
      if (a.Msplit && mg >= a.Msplit) {
        P = (const char*)a.Am2;
        mg -= a.Msplit;
        lim = a.M - a.Msplit;
      }
      pa[g] = P + (abase + (long)min(mg, lim - 1) * a.sAm) * 4;
      if constexpr (BKC) {
        kb[g] = ka[g];
        pb[g] = (const char*)a.B + (bbase + (long)min(n0 + row, a.N - 1) * a.sBn) * 4;
      } else {
        kb[g] = (row & 3) * 8 + (row >> 2);  // the k-row this LDS row holds
        pb[g] = (const char*)a.B + (bbase + (long)min(n0 + 4 * (qs & 7), (a.N - 1) & ~3)) * 4;
      }
    }
  };
  auto stage = [&](int it, char* buf) {
    const int e = it / kc, kk0 = (it - e * kc) * BK;
    if (e != cur) {
      term_bases(e);
      cur = e;
    }
    const char* zero = (const char*)g_ring_zero;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int k = kk0 + ka[g];
      glds16_asm(k < keff ? pa[g] + (long)k * 4 : zero, buf + g * 1024);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int k = kk0 + kb[g];
      const char* src = BKC ? pb[g] + (long)k * 4 : pb[g] + (long)k * a.sBk * 4;
      glds16_asm(k < keff ? src : zero, buf + HALF + g * 1024);
    }
  };
  auto compute = [&](const char* buf, f32x16& acc) {
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int k0 = 16 * s + 8 * hh;
      float x[8];
      rd8<true>(buf, l32, k0, x);
      if constexpr (SCALE)
#pragma unroll
        for (int t = 0; t < 8; ++t) x[t] *= gs.sa;
      const frag ah = pk8<F16>(x), al = SPLIT ? pk8_lo<true>(x) : ah;
      if constexpr (BKC) {
        rd8<true>(buf + HALF, l32, k0, x);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = *(const float*)(buf + HALF + gks::rcs_row(k0 + j) * 128 + l32 * 4);
      }
      if constexpr (SCALE)
#pragma unroll
        for (int t = 0; t < 8; ++t) x[t] *= gs.sb;
      const frag bh = pk8<F16>(x), bl = SPLIT ? pk8_lo<true>(x) : bh;
      mma<PREC>(acc, ah, al, bh, bl);
    }
  };

  f32x16 acc = splat(0.f);
  const int mine = nit > wk ? (nit - wk + WK - 1) / WK : 0;  // slices wk, wk + WK, ...
  const int rounds = (nit + WK - 1) / WK;                     // (wk = 0's count: every wave meets each barrier)
  if (mine > 0) stage(wk, my);
  for (int u = 0; u < rounds; ++u) {
    // slice u of this wave landed: its vmcnt, then a barrier before the reads
    // (a DMA's LDS write is ordered for ds_read only by the wait AND a barrier
    // passed after it, cdna_hip_programming.md "Read a staged buffer ...")
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (u + 1 < mine) stage(wk + WK * (u + 1), my + ((u + 1) & 1) * SLOT);
    if (u < mine) compute(my + (u & 1) * SLOT, acc);
  }
  if constexpr (WK > 1) {
    // partials -> this wave's slot 0 (its DMAs are done, its reads consumed)
    float* red = (float*)my;
#pragma unroll
    for (int r = 0; r < 16; ++r) red[r * 64 + lane] = acc[r];
    __syncthreads();
  }

  // ---- epilogue: wave (wn, wk) stores accumulator entries r of quads
  // wk * 4 / WK .. (wk + 1) * 4 / WK - 1 (rows acc_row(r, hh)) of column block wn
  const int n = n0 + l32;
  if (n >= a.N) return;
  const long dbase = (long)z * a.sDz + (long)zp * a.sDp + (long)zq * a.sDq;
  const float* bias = a.bias ? a.bias + (long)zp * a.sbp + (long)zq * a.sbq : nullptr;
  const float bn = bias ? bias[n] : 0.f;
  const bool hi_n = a.Nsplit && n >= a.Nsplit;
  float* const Dn = hi_n ? a.D2 : a.D;
  const long sm = hi_n && a.sD2m ? a.sD2m : a.sDm, dn = dbase + (long)(hi_n ? n - a.Nsplit : n) * a.sDn;
  // E factors / old D values (GG_ADD) loaded up front (as k_gemm_ring)
  // (or the state h of the fused r * h output, GemmArgs::aux)
  float pre[16 / WK], pre2[16 / WK];
  const bool rhn = a.aux && n < a.auxN, bln = a.bout != nullptr;
  if (a.E || a.mode == GG_ADD) {
    const float* src = a.E ? a.E : Dn;
#pragma unroll
    for (int e = 0; e < 16 / WK; ++e)
      pre[e] = src[dn + (long)min(m0 + acc_row(4 * (wk * (4 / WK) + (e >> 2)), hh) + (e & 3), a.M - 1) * sm];
  } else if (rhn) {
#pragma unroll
    for (int e = 0; e < 16 / WK; ++e)
      pre[e] = a.auxin[(long)min(m0 + acc_row(4 * (wk * (4 / WK) + (e >> 2)), hh) + (e & 3), a.M - 1) * a.auxN + n];
  } else if (bln) {
#pragma unroll
    for (int e = 0; e < 16 / WK; ++e) {
      const long row = min(m0 + acc_row(4 * (wk * (4 / WK) + (e >> 2)), hh) + (e & 3), a.M - 1);
      pre[e] = a.bh[row * a.N + n];
      pre2[e] = a.bu[row * 2 * a.N + a.N + n];
    }
  }
  // the fused k_gen_bwd2 (GemmArgs::b2dzg) on the d(rh) columns: r, h and
  // the dh half of DXH loaded up front
  const bool b2n = a.b2dzg && hi_n;
  const int k2 = n - a.Nsplit;
  const long H2 = 2L * a.Nsplit;
  float pr[16 / WK], ph[16 / WK], pd[16 / WK];
  if (b2n) {
#pragma unroll
    for (int e = 0; e < 16 / WK; ++e) {
      const long row = min(m0 + acc_row(4 * (wk * (4 / WK) + (e >> 2)), hh) + (e & 3), a.M - 1);
      pr[e] = a.b2r[row * H2 + k2];
      ph[e] = a.b2h[row * a.Nsplit + k2];
      pd[e] = a.b2dxh[row * H2 + a.Nsplit + k2];
    }
  }
  float s2 = 0.f;
  const Drop sd = bln ? drop_resolve(a.bsd) : Drop{};
  long wkey = -1;  // the first row of the state-dropout quad whose words w holds
  uint4 sw = make_uint4(0u, 0u, 0u, 0u);
  float cs = 0.f;
#pragma unroll
  for (int qq = 0; qq < 4 / WK; ++qq) {
    const int quad = wk * (4 / WK) + qq;
    const int mq = m0 + acc_row(4 * quad, hh);  // rows mq .. mq + 3
    uint4 dq = make_uint4(0u, 0u, 0u, 0u);
    if (dr.thr) dq = edge_words(dr, zp, mq, n, a.drop_t);
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const int r = 4 * quad + r4, m = mq + r4;
      if (m >= a.M) continue;
      float v;
      if constexpr (WK == 1) {
        v = acc[r];
      } else {
        const float* rp = (const float*)ring + wn * (2 * SLOT / 4) + r * 64 + lane;  // wave (wn, 0)
        constexpr int ST = WN * 2 * SLOT / 4;                                          // next wk
        if constexpr (WK == 2) v = rp[0] + rp[ST];
        else v = (rp[0] + rp[ST]) + (rp[2 * ST] + rp[3 * ST]);
      }
      float x = gs.alpha * v + bn;
      if (a.epi == GG_EPI_SIGMOID) x = sigm(x);
      else if (a.epi == GG_EPI_TANH) x = tanh_f(x);
      if (rhn) a.aux[(long)m * a.auxN + n] = x * pre[4 * qq + r4];
      if (bln) {
        const float ug = pre2[4 * qq + r4];
        float y = gru_blend(ug, pre[4 * qq + r4], x);
        if (sd.thr) {
          const int g = m / a.bv, i = m - g * a.bv;
          if ((long)m - (i & 3) != wkey) {
            wkey = (long)m - (i & 3);
            sw = state_words(sd, g, i, n, a.bt);
          }
          y = drop_apply(sd, u4_get(sw, i & 3), y);
        }
        a.bout[(long)m * a.N + n] = y;
      }
      if (b2n) {
        const float r = pr[4 * qq + r4], zr = gru_dzg_r(x, ph[4 * qq + r4], r);
        a.b2dzg[(long)m * H2 + k2] = zr;
        a.b2dxh[(long)m * H2 + a.Nsplit + k2] = __builtin_fmaf(x, r, pd[4 * qq + r4]);
        s2 += zr;
      }
      if (dr.thr) x = drop_apply(dr, u4_get(dq, r4), x);
      const long doff = dn + (long)m * sm;
      if (a.E) x *= pre[4 * qq + r4];
      cs += x;
      float* d = Dn + doff;
      if (a.mode == GG_ATOMIC) {
        if (a.slab) a.slab[(long)z * a.sSlab + (long)m * a.N + n] = x;
        else atomicAdd(d, x);
      } else if (a.mode == GG_ADD) *d = pre[4 * qq + r4] + x;
      else *d = x;
    }
  }
  if (a.csum) {
    cs += __shfl_xor(cs, 32);
    if (hh == 0) atomicAdd(a.csum + (long)zp * a.scp + (long)zq * a.scq + n, cs);  // (k_gemm_ks: no cpart callers)
  }
  if (b2n) {
    s2 += __shfl_xor(s2, 32);
    if (hh == 0) a.b2part[((long)mt * WK + wk) * a.Nsplit + k2] = s2;
  }
}
