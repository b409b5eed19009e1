// k_gru2.h -- GRUCell forward for hidden = 256 in the split (fp32-parity)
// mode, 128-row tiles with K-streamed activations.
//
// Same math as k_gru_fwd (k_gru.h; reference: TF1 GRUCell built at
// chem_tensorflow_dense.py:237-241, applied at :333):
//   [r | u] = sigmoid([x, h] @ Wg + bg);  c = tanh([x, r*h] @ Wc + bc)
//   h' = u*h + (1-u)*c   (then DropoutWrapper state dropout, :239-240)
//
// Why a second kernel: with 64-row tiles the whole [x | h] tile sits in LDS
// as f16 hi/lo limbs (128 KiB), one workgroup fits a CU, and every 64 rows
// stream the full Wg + Wc fragment set (1.5 MiB) from L2.  That ran the MFMA
// phases at the L2 rate for CU-shared data (~65 GB/s per CU, measured by
// in-kernel stamps) with the HBM phases serialized between them.  Here a
// workgroup owns 128 rows (half the weight bytes per row) and the activations
// arrive in 32-column chunks, loaded into registers two chunks ahead of use,
// so the HBM reads overlap the MFMAs:
//   pass A  k over [x | h] (32 k-steps): x chunks through a 2-slot LDS ring;
//           h chunks straight into the full h image (reused for r*h)
//   r*h     in place over the h image (each lane owns its elements)
//   pass B  k over [r*h | x]: r*h from the image, x streamed again (L2/MALL)
//   blend   h' from the fp32 state (reloaded), stores
// LDS: h / r*h image 2 x 64 KiB + ring 2 slots x (hi + lo) 8 KiB = 160 KiB.
#pragma once
#include "ggnn_common.h"

namespace gru2 {
constexpr int H = 256, R = 128, RT = 4, NS = 8, NT = 512;
constexpr int KS = H / 16, KSG = 2 * KS;  // k-steps over H and over 2H
constexpr int NCHK = H / 32;              // 32-column activation chunks per operand
constexpr int IMG = R * H * 2;            // one limb image, bytes
constexpr int SLOT = R * 32 * 2;          // one limb of a ring slot, bytes
constexpr int CB = R * 16;                // bytes of one 16-B column chunk over all rows
// LDS images are chunk-major: 16-B chunk ch (8 consecutive k) of row `row`
// sits at ch * CB + row * 16.  The 16 lanes of a ds_read_b128 group read 16
// rows of one chunk: 256 contiguous bytes, conflict-free; and the k offset
// of every fragment read is an immediate (one address VGPR per image).
DEV int koff(int row, int ch) { return ch * CB + row * 16; }

typedef __attribute__((ext_vector_type(4))) unsigned int v4u32;
DEV uint4 bld16(rsrc_t r, int vo, int so) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
}
// one 32-column chunk of a row-major fp32 [R][H] tile: thread tid holds row
// crow(tid), columns 8*cq(tid) .. +8 of the chunk (vo = chunk_vo(tid)).  Eight
// consecutive lanes take eight consecutive rows of one 16-B column piece, so
// their ds_write_b128 into the chunk-major image is one contiguous 128 B
// (conflict-free); a wave still covers 16 whole 128-B rows of the chunk.
struct Chunk { uint4 a, b; };
DEV int crow_of(int tid) { return (tid & 7) + 8 * (tid >> 5); }
DEV int cq_of(int tid) { return (tid >> 3) & 3; }
DEV int chunk_vo(int tid) { return (crow_of(tid) * H + cq_of(tid) * 8) * 4; }
DEV Chunk chunk_ld(rsrc_t r, int vo, int ck) { return Chunk{bld16(r, vo, ck * 128), bld16(r, vo, ck * 128 + 16)}; }
DEV void chunk_put(char* hi, char* lo, int off, const Chunk& v) {
  const float x[8] = {__uint_as_float(v.a.x), __uint_as_float(v.a.y), __uint_as_float(v.a.z), __uint_as_float(v.a.w),
                      __uint_as_float(v.b.x), __uint_as_float(v.b.y), __uint_as_float(v.b.z), __uint_as_float(v.b.w)};
  st16(hi + off, pk8<true>(x));
  st16(lo + off, pk8_lo<true>(x));
}
// B fragment of k-step ks of the packed strip whose lane offset is vo
DEV frag wld(rsrc_t r, int vo, int ks) { return bld16(r, vo, ks * 1024); }
}  // namespace gru2

__global__ void __launch_bounds__(512)
k_gru_fwd2(const float* __restrict__ Xa, const float* __restrict__ hf, const u16* __restrict__ Wgp,
           const float* __restrict__ bg, const u16* __restrict__ Wcp, const float* __restrict__ bc, long wlo_g,
           long wlo_c, float* __restrict__ hf_out, u16* __restrict__ hT_out, float* __restrict__ r_out,
           float* __restrict__ u_out, float* __restrict__ c_out, u16* __restrict__ rhT_out, long N, Drop dr, int t,
           int vsh) {
  dr = drop_resolve(dr);  // (a device-resident key: loaded once)
  using namespace gru2;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG + 4 * SLOT];
  char* img_hi = smem;
  char* img_lo = smem + IMG;
  auto slot_hi = [&](int u) { return smem + 2 * IMG + u * 2 * SLOT; };
  auto slot_lo = [&](int u) { return smem + 2 * IMG + u * 2 * SLOT + SLOT; };

  const int tid = threadIdx.x, lane = tid & 63, ns = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int n = ns * 32 + l32;
  const long row0 = (long)blockIdx.x * R;
  const rsrc_t rx = mkrsrc(Xa + row0 * H, R * H * 4), rhs = mkrsrc(hf + row0 * H, R * H * 4);
  const int cvo = chunk_vo(tid);
  // this thread's 16-B slot in a chunk write (chunk cq of row crow)
  const int crow = crow_of(tid), cq = cq_of(tid);
  const int cso = koff(crow, cq);
  TSMARK(0, 0);

  // ======================= pass A: [x | h] @ Wg -> r, u =======================
  f32x16 ar[RT], au[RT];
  {
    const float br = bg[n], bu = bg[H + n];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) { ar[rt] = splat(br); au[rt] = splat(bu); }
  }
  const rsrc_t wgh = mkrsrc(Wgp, 4 * H * H * 2), wgl = mkrsrc(Wgp + wlo_g, 4 * H * H * 2);
  const int vr = ((ns * KSG) * 64 + lane) * 16, vu = (((NS + ns) * KSG) * 64 + lane) * 16;
  auto ldg = [&](int k) { return F4{wld(wgh, vr, k), wld(wgl, vr, k), wld(wgh, vu, k), wld(wgl, vu, k)}; };
  // chunk c of pass A: c < 8 -> x columns [32c, +32), else h columns [32(c-8), +32)
  auto ld_a = [&](int c) { return c < NCHK ? chunk_ld(rx, cvo, c) : chunk_ld(rhs, cvo, c - NCHK); };
  auto put_a = [&](int c, const Chunk& v) {
    if (c < NCHK) chunk_put(slot_hi(c & 1), slot_lo(c & 1), cso, v);
    else chunk_put(img_hi, img_lo, cso + (c - NCHK) * 4 * CB, v);
  };
  Chunk st0 = ld_a(0), st1 = ld_a(1);
  F4 w0 = ldg(0), w1 = ldg(1);
  put_a(0, st0);
  st0 = ld_a(2);
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 2 * NCHK; ++c) {
    // chunk c+1 -> its slot (read last by chunk c-1, fenced by the barrier
    // that closed iteration c-1); chunk c+3 -> registers
    if (c + 1 < 2 * NCHK) {
      put_a(c + 1, (c & 1) ? st0 : st1);
      if (c + 3 < 2 * NCHK) {
        if (c & 1) st0 = ld_a(c + 3);
        else st1 = ld_a(c + 3);
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ks = 2 * c + s;
      const F4 w = s ? w1 : w0;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int row = rt * 32 + l32;
        const char* ih = c < NCHK ? slot_hi(c & 1) : img_hi;
        const char* il = c < NCHK ? slot_lo(c & 1) : img_lo;
        const int off = c < NCHK ? koff(row, 2 * s + hh) : koff(row, (c - NCHK) * 4 + 2 * s + hh);
        const frag ah = lds_frag(ih, off), al = lds_frag(il, off);
        mma<PREC_SPLIT>(ar[rt], ah, al, w.a, w.b);
        mma<PREC_SPLIT>(au[rt], ah, al, w.c, w.d);
      }
      if (s) w1 = ldg(min(ks + 2, KSG - 1));
      else w0 = ldg(min(ks + 2, KSG - 1));
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
  }
  TSMARK(0, 1);
  // pass B's first x chunks: in flight during the r*h phase
  st0 = chunk_ld(rx, cvo, 0);
  st1 = chunk_ld(rx, cvo, 1);

  // ========== r*h in place over the h image; r and (r*h)^T to HBM ==========
  const int vo = (4 * hh * H + n) * 4;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float rh[16], rv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      au[rt][r] = sigm(au[rt][r]);
      const float rr = sigm(ar[rt][r]);
      rv[r] = rr;
      const int row = rt * 32 + acc_row(r, hh);
      const int eo = koff(row, n >> 3) + (n & 7) * 2;
      const float hx = from_limb<true>(*(const u16*)(img_hi + eo)) + from_limb<true>(*(const u16*)(img_lo + eo));
      rh[r] = rr * hx;
      *(u16*)(img_hi + eo) = to_limb<true>(rh[r]);
      *(u16*)(img_lo + eo) = to_limb<true>(lo_part<true>(rh[r]));
    }
    if (r_out) {  // row-quad-major save
#pragma unroll
      for (int q = 0; q < 4; ++q)
        gst4(r_out + row0 * H, qm_vo(hh, n, H), qm_so(rt, q, H), make_float4(rv[4 * q], rv[4 * q + 1], rv[4 * q + 2], rv[4 * q + 3]));
    }
    if (rhT_out) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st_col4w<PREC_SPLIT>(rhT_out + wg_off(n, row0 + rt * 32 + 4 * hh, H) + 8 * q, rh[4 * q], rh[4 * q + 1],
                             rh[4 * q + 2], rh[4 * q + 3]);
    }
  }
  chunk_put(slot_hi(0), slot_lo(0), cso, st0);
  st0 = chunk_ld(rx, cvo, 2);
  __syncthreads();
  TSMARK(0, 2);

  // ============ pass B: [r*h | x] @ [Wc_h ; Wc_x] -> candidate ============
  f32x16 ac[RT];
  {
    const float b0 = bc[n];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) ac[rt] = splat(b0);
  }
  const rsrc_t wch = mkrsrc(Wcp, 2 * H * H * 2), wcl = mkrsrc(Wcp + wlo_c, 2 * H * H * 2);
  auto ldc = [&](int k) { return F2{wld(wch, vr, k), wld(wcl, vr, k)}; };
  // r*h rows of Wc (k-steps KS..2KS-1) first: no loads to wait for
  {
    F2 v0 = ldc(KS), v1 = ldc(KS + 1);
#pragma unroll
    for (int ks = 0; ks < KS; ks += 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const F2 w = s ? v1 : v0;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int off = koff(rt * 32 + l32, 2 * (ks + s) + hh);
          mma<PREC_SPLIT>(ac[rt], lds_frag(img_hi, off), lds_frag(img_lo, off), w.a, w.b);
        }
        // ring runs on into the x rows (k-steps 0, 1) for the loop below
        const int nk = ks + s + 2;
        const F2 nw = ldc(nk < KS ? KS + nk : nk - KS);
        if (s) v1 = nw;
        else v0 = nw;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    w0 = F4{v0.a, v0.b, frag{}, frag{}};
    w1 = F4{v1.a, v1.b, frag{}, frag{}};
  }
#pragma unroll
  for (int c = 0; c < NCHK; ++c) {
    if (c + 1 < NCHK) {
      chunk_put(slot_hi((c + 1) & 1), slot_lo((c + 1) & 1), cso, (c & 1) ? st0 : st1);
      if (c + 3 < NCHK) {
        if (c & 1) st0 = chunk_ld(rx, cvo, c + 3);
        else st1 = chunk_ld(rx, cvo, c + 3);
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ks = 2 * c + s;
      const F4 w = s ? w1 : w0;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int off = koff(rt * 32 + l32, 2 * s + hh);
        mma<PREC_SPLIT>(ac[rt], lds_frag(slot_hi(c & 1), off), lds_frag(slot_lo(c & 1), off), w.a, w.b);
      }
      const F2 nw = ldc(min(ks + 2, KS - 1));
      if (s) w1 = F4{nw.a, nw.b, frag{}, frag{}};
      else w0 = F4{nw.a, nw.b, frag{}, frag{}};
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c + 1 < NCHK) __syncthreads();
  }

  TSMARK(0, 3);
  // ================================ blend ================================
  const rsrc_t ho = mkrsrc(hf_out + row0 * H, R * H * 4);
  uint4 dw = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float hn[16], uv[16], cv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int so = (rt * 32 + acc_row0(r)) * H * 4;
      const float cc = tanh_f(ac[rt][r]);
      uv[r] = au[rt][r];
      cv[r] = cc;
      const float u = au[rt][r];
      const float hprev = bld(rhs, vo, so);
      float x = u * hprev + (1.0f - u) * cc;
      if (dr.thr) {  // DropoutWrapper state dropout of the new state (chem_tensorflow_dense.py:239-240)
        if ((r & 3) == 0) {
          const long grow = row0 + rt * 32 + acc_row0(r) + 4 * hh;
          dw = state_words(dr, (int)(grow >> vsh), (int)(grow & ((1 << vsh) - 1)), n, t);
        }
        x = drop_apply(dr, u4_get(dw, r & 3), x);
      }
      hn[r] = x;
      bst(ho, x, vo, so);
    }
    if (u_out) {  // row-quad-major saves
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        gst4(u_out + row0 * H, qm_vo(hh, n, H), qm_so(rt, q, H), make_float4(uv[4 * q], uv[4 * q + 1], uv[4 * q + 2], uv[4 * q + 3]));
        gst4(c_out + row0 * H, qm_vo(hh, n, H), qm_so(rt, q, H), make_float4(cv[4 * q], cv[4 * q + 1], cv[4 * q + 2], cv[4 * q + 3]));
      }
    }
    if (hT_out) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st_col4w<PREC_SPLIT>(hT_out + wg_off(n, row0 + rt * 32 + 4 * hh, H) + 8 * q, hn[4 * q], hn[4 * q + 1],
                             hn[4 * q + 2], hn[4 * q + 3]);
    }
  }
  TSMARK(0, 4);
}
