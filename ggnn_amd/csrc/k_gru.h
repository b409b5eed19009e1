// k_gru.h -- TF1 GRUCell (reset-before-matmul) forward and backward, fused.
//
// Reference: tf.compat.v1.nn.rnn_cell.GRUCell built at
// chem_tensorflow_dense.py:237-241, applied at :333 (external TF op):
//   [r | u] = sigmoid([x, h] @ Wg + bg)        Wg [2H][2H], rows [x ; h]
//   c       = tanh([x, r*h] @ Wc + bc)         Wc [2H][H],  rows [x ; r*h]
//   h'      = u*h + (1-u)*c
// A workgroup owns 32*RT consecutive node rows; wave w owns hidden columns
// [32w, 32w+32) of r, u and c, so r*h for ALL columns is shared through LDS
// before the candidate product.
#pragma once
#include "ggnn_common.h"

// cache policy of k_gru_bwd's saved-activation loads (r, u, c, delta: read
// once): nontemporal, so they do not evict the Wc^T / Wg^T fragments the
// products stream from L2 (measured -2.8 % on k_gru_bwd, A/B on one box); the
// state h is read in both phases and keeps the default policy
constexpr int kGbAux = kNT;

// weight-fragment ring loops: outer loop unrolled by 2 (measured against 1 and
// full unrolling, which spills at H = 256)
constexpr int GF_UNROLL = 2, GB_UNROLL = 2;
// k_gru_bwd's weight-fragment ring depth (k-steps in flight)
constexpr int GB_DEPTH = 2;

// gru_bwd elementwise phases: loads of GB_GROUP row quads (x 4 arrays) in flight
// between scheduling barriers (measured: 4 > 2 > 1; VGPRs stay within budget)
constexpr int GB_GROUP = 4;

// ===========================================================================
// k_gru_fwd
//   pass A: [X | h] @ Wg            -> r, u      (K = 2H)
//   r*h -> LDS (over the h image), r*h^T -> HBM (training)
//   pass B: X @ Wc[0:H] + (r*h) @ Wc[H:2H] -> c  (K = 2H)
//   h' = u*h + (1-u)*tanh(c + bc)
// ===========================================================================
template <int H, int RT, int PREC>
__global__ void __launch_bounds__(2 * H)
k_gru_fwd(const ActT<PREC>* __restrict__ Xa, const u16* __restrict__ hb16, const float* __restrict__ hf,
          const u16* __restrict__ Wgp, const float* __restrict__ bg, const u16* __restrict__ Wcp,
          const float* __restrict__ bc, long wlo_g, long wlo_c, float* __restrict__ hf_out, u16* __restrict__ hb_out,
          u16* __restrict__ hT_out, float* __restrict__ r_out, float* __restrict__ u_out,
          float* __restrict__ c_out, u16* __restrict__ rhT_out, long N, Drop dr, int t, int vsh) {
  dr = drop_resolve(dr);  // (a device-resident key: loaded once)
  constexpr bool SPLIT = Prec<PREC>::split, F16 = Prec<PREC>::f16;
  constexpr int NS = H / 32, NT = 64 * NS, KS = H / 16, R = 32 * RT, HCH = H / 8, KSG = 2 * KS;
  typedef Swz<HCH> SH;
  constexpr int NIMG = SPLIT ? 2 : 1;
  constexpr int IMG = R * H * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * NIMG * IMG];
  char* x_hi = smem;
  char* x_lo = smem + (SPLIT ? IMG : 0);
  char* h_hi = smem + NIMG * IMG;
  char* h_lo = h_hi + (SPLIT ? IMG : 0);

  const int tid = threadIdx.x, lane = tid & 63, ns = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int n = ns * 32 + l32;
  const long row0 = (long)blockIdx.x * R;
  TSMARK(0, 0);
  stage_rows<PREC, R, H, NT>(x_hi, x_lo, Xa + row0 * H, H, tid);
  if constexpr (SPLIT) stage_rows<PREC_SPLIT, R, H, NT>(h_hi, h_lo, hf + row0 * H, H, tid);
  else stage_rows<PREC, R, H, NT>(h_hi, h_lo, hb16 + row0 * H, H, tid);
  __syncthreads();
  TSMARK(0, 1);

  f32x16 ar[RT], au[RT];
  {
    const float br = bg[n], bu = bg[H + n];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) { ar[rt] = splat(br); au[rt] = splat(bu); }
  }
  // ---- pass A over k in [0, 2H): x rows then h rows of Wg
  auto ldg = [&](int k) {
    return F4{frag_ld(Wgp, ns, k, KSG, lane), SPLIT ? frag_ld(Wgp + wlo_g, ns, k, KSG, lane) : frag{},
              frag_ld(Wgp, NS + ns, k, KSG, lane), SPLIT ? frag_ld(Wgp + wlo_g, NS + ns, k, KSG, lane) : frag{}};
  };
  b_pipeline<KSG, 2, GF_UNROLL>(ldg, [&](int k, const F4& w) {
    const char* ih = (k < KS) ? x_hi : h_hi;
    const char* il = (k < KS) ? x_lo : h_lo;
    const int kk = (k < KS) ? k : k - KS;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int off = SH::off(rt * 32 + l32, 2 * kk + hh);
      const frag ah = lds_frag(ih, off), al = SPLIT ? lds_frag(il, off) : ah;
      mma<PREC>(ar[rt], ah, al, w.a, w.b);
      mma<PREC>(au[rt], ah, al, w.c, w.d);
    }
  });
  TSMARK(0, 2);
  const rsrc_t rh_in = mkrsrc(hf + row0 * H, R * H * 4);
  const int vo = (4 * hh * H + n) * 4;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      ar[rt][r] = sigm(ar[rt][r]);
      au[rt][r] = sigm(au[rt][r]);
    }
  __syncthreads();  // every wave is done reading the h image
  // ---- r*h -> h image(s).  The r and (r*h)^T stores wait for the epilogue:
  // vmcnt is in order, so a store issued here would make every weight-fragment
  // wait of pass B cover it.
  // (At RT = 4 keeping r live through pass B spills: store early there.)
  constexpr bool DEFER = RT <= 2;
  // h (fp32) of this lane's elements, kept in registers for the blend (the h
  // image is overwritten by r*h); at RT = 4 the blend re-reads it instead
  float hv[DEFER ? RT : 1][16];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float rh[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float hx = bld(rh_in, vo, (rt * 32 + acc_row0(r)) * H * 4);
      if constexpr (DEFER) hv[rt][r] = hx;
      rh[r] = ar[rt][r] * hx;
      img_put<PREC, HCH>(h_hi, h_lo, rt * 32 + acc_row(r, hh), n, rh[r]);
    }
    if constexpr (!DEFER) {
      if (rhT_out) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          st_col4w<PREC>(rhT_out + wg_off(n, row0 + rt * 32 + 4 * hh, H) + 8 * q, rh[4 * q], rh[4 * q + 1],
                         rh[4 * q + 2], rh[4 * q + 3]);
      }
      if (r_out) {  // row-quad-major save
#pragma unroll
        for (int q = 0; q < 4; ++q)
          gst4(r_out + row0 * H, qm_vo(hh, n, H), qm_so(rt, q, H),
               make_float4(ar[rt][4 * q], ar[rt][4 * q + 1], ar[rt][4 * q + 2], ar[rt][4 * q + 3]));
      }
    }
  }
  __syncthreads();
  TSMARK(0, 3);
  // ---- pass B: candidate
  f32x16 ac[RT];
  {
    const float b0 = bc[n];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) ac[rt] = splat(b0);
  }
  auto ldc = [&](int ks) {
    return F4{frag_ld(Wcp, ns, ks, KSG, lane), SPLIT ? frag_ld(Wcp + wlo_c, ns, ks, KSG, lane) : frag{},
              frag_ld(Wcp, ns, KS + ks, KSG, lane), SPLIT ? frag_ld(Wcp + wlo_c, ns, KS + ks, KSG, lane) : frag{}};
  };
  b_pipeline<KS, 2, GF_UNROLL>(ldc, [&](int ks, const F4& w) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int off = SH::off(rt * 32 + l32, 2 * ks + hh);
      const frag xh = lds_frag(x_hi, off), xl = SPLIT ? lds_frag(x_lo, off) : xh;
      const frag qh = lds_frag(h_hi, off), ql = SPLIT ? lds_frag(h_lo, off) : qh;
      mma<PREC>(ac[rt], xh, xl, w.a, w.b);
      mma<PREC>(ac[rt], qh, ql, w.c, w.d);
    }
  });
  TSMARK(0, 4);
  // ---- blend + outputs
  const rsrc_t ho = mkrsrc(hf_out + row0 * H, R * H * 4);
  uint4 dw = make_uint4(0, 0, 0, 0);
  if constexpr (!SPLIT) __syncthreads();  // the h image is reused to stage h' (bf16) below
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float u4[4], c4[4], r4[4];  // one accumulator quad of u, c, r (row-quad-major saves)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int so = (rt * 32 + acc_row0(r)) * H * 4;
      const float cc = tanh_f(ac[rt][r]);
      const float u = au[rt][r];
      float hprev;
      if constexpr (DEFER) hprev = hv[rt][r];
      else hprev = bld(rh_in, vo, so);
      float hn = u * hprev + (1.0f - u) * cc;
      if (dr.thr) {  // DropoutWrapper state dropout of the new state (chem_tensorflow_dense.py:239-240)
        if ((r & 3) == 0) {
          const long grow = row0 + rt * 32 + acc_row0(r) + 4 * hh;
          dw = state_words(dr, (int)(grow >> vsh), (int)(grow & ((1 << vsh) - 1)), n, t);
        }
        hn = drop_apply(dr, u4_get(dw, r & 3), hn);
      }
      bst(ho, hn, vo, so);
      if (u_out) {
        u4[r & 3] = u;
        c4[r & 3] = cc;
        r4[r & 3] = ar[rt][r];
        if ((r & 3) == 3) {
          const int qo = qm_so(rt, r >> 2, H), qv = qm_vo(hh, n, H);
          gst4(u_out + row0 * H, qv, qo, make_float4(u4[0], u4[1], u4[2], u4[3]));
          gst4(c_out + row0 * H, qv, qo, make_float4(c4[0], c4[1], c4[2], c4[3]));
          if constexpr (DEFER) gst4(r_out + row0 * H, qv, qo, make_float4(r4[0], r4[1], r4[2], r4[3]));
        }
      }
      if (DEFER && rhT_out) au[rt][r] = ar[rt][r] * hprev;  // r*h (u is dead from here)
      ac[rt][r] = hn;
      if constexpr (!SPLIT) *(u16*)(h_hi + SH::eoff(rt * 32 + acc_row(r, hh), n)) = to_limb<F16>(hn);
    }
    if (DEFER && rhT_out) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st_col4w<PREC>(rhT_out + wg_off(n, row0 + rt * 32 + 4 * hh, H) + 8 * q, au[rt][4 * q], au[rt][4 * q + 1],
                       au[rt][4 * q + 2], au[rt][4 * q + 3]);
    }
    if (hT_out) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st_col4w<PREC>(hT_out + wg_off(n, row0 + rt * 32 + 4 * hh, H) + 8 * q, ac[rt][4 * q], ac[rt][4 * q + 1],
                       ac[rt][4 * q + 2], ac[rt][4 * q + 3]);
    }
  }
  if constexpr (!SPLIT) {
    __syncthreads();
    for (int q = tid; q < R * HCH; q += NT) {
      const int row = q / HCH, ch = q % HCH;
      st16(hb_out + (row0 + row) * H + ch * 8, ld16(h_hi + SH::off(row, ch)));
    }
  }
  TSMARK(0, 5);
}

// ===========================================================================
// k_gru_bwd: backward of the GRUCell, delta = dL/dh'
//   dzc = delta (1-u) (1-c^2)                      -> LDS, dzc^T, dbc
//   [dX1 | d(rh)] = dzc @ Wc^T                     (K = H)
//   dh  = delta u + d(rh) r
//   dzg = [d(rh) h r(1-r) | delta (h-c) u(1-u)]    -> LDS, dzg^T, dbg
//   [dX2 | dh2] = dzg @ Wg^T                       (K = 2H)
//   out: dX^T = (dX1 + dX2)^T, dh + dh2 (fp32)
// ===========================================================================
// The 16-bit modes' products: dz @ W^T on one MFMA per k-step and tile (the
// split mode's fp8-corrected form is gb_f8_product in the kernel)
template <int PREC>
DEV void gb_mma(f32x16& a1, f32x16& a2, frag ah, frag al, const F2& w) {
  mma_xb<PREC>(a1, ah, al, w.a);
  mma_xb<PREC>(a2, ah, al, w.b);
}

template <int H, int RT, int PREC>
__global__ void __launch_bounds__(2 * H, RT == 1 ? 2 : 1)
k_gru_bwd(const float* __restrict__ delta, const float* __restrict__ hf, const float* __restrict__ rin,
          const float* __restrict__ uin, const float* __restrict__ cin, const u16* __restrict__ WcTp,
          const u16* __restrict__ WgTp, long wlo_c, long wlo_g, ActT<PREC>* __restrict__ dXT,
          float* __restrict__ dh_out, u16* __restrict__ dzcT, u16* __restrict__ dzgT,
          float* __restrict__ dbc, float* __restrict__ dbg, long N, const uint32_t* __restrict__ gmax,
          float* __restrict__ bpart, const uint2* __restrict__ sbits, float sscale) {
  // bpart: this timestep's [workgroup][dbg (2H) | dbc (H)] rows of bias partials
  // (summed in a fixed order by k_sum_rows: deterministic), or nullptr: atomics.
  // sbits (first backward step, dL/dh_T read in place under state dropout):
  // the forward's keep bits of the last timestep's state mask (k_fwd_fused,
  // 128-row graphs: word (graph, thread), bit (jt & 1) * 16 + r of word jt >> 1
  // for row tile jt of the graph), applied to delta with scale sscale = 1/keep
  constexpr bool SPLIT = Prec<PREC>::split, F16 = Prec<PREC>::f16;
  constexpr int NS = H / 32, KS = H / 16, R = 32 * RT, ZCH = 2 * H / 8;
  constexpr int GBD = GB_DEPTH;
  const float ds = gscale(gmax);  // gradient scale of dL/dh_T read in place (ggnn_common.h), else 1
  TSCLK(1, 0);
  typedef Swz<ZCH> SZ;
  // split mode: the f16 image of dz and its e5m2 image (the fp8 MFMA's A operand,
  // 1 byte per element, 16-byte chunks swizzled like the f16 image)
  typedef Swz<2 * H / 16> SZ8;
  constexpr int IMG = R * 2 * H * 2;
  __shared__ __attribute__((aligned(16))) char smem[SPLIT ? IMG + IMG / 2 : IMG];
  char* z_hi = smem;
  char* z8 = smem + IMG;
  // one dz element into the f16 image; the split mode's e5m2 image is filled
  // from it by z8_fill after each phase (a chunk-wise pass: per-element byte
  // stores in the phases cost registers the products need)
  auto zput = [&](int row, int e, float v) { *(u16*)(z_hi + SZ::eoff(row, e)) = to_limb<F16>(v); };
  auto z8_fill = [&](int c0, int nch) {  // 16-column chunks [c0, c0 + nch) of every row
    for (int q = (int)threadIdx.x; q < R * nch; q += 2 * H) {
      const int row = q / nch, c = c0 + q % nch;
      const uint4 u[2] = {ld16(z_hi + SZ::off(row, 2 * c)), ld16(z_hi + SZ::off(row, 2 * c + 1))};
      uint32_t o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint4 x = u[i >> 1];
        const uint32_t w0 = (i & 1) ? x.z : x.x, w1 = (i & 1) ? x.w : x.y;
        const _Float16 h0 = __builtin_bit_cast(_Float16, (u16)(w0 & 0xffff)), h1 = __builtin_bit_cast(_Float16, (u16)(w0 >> 16));
        const _Float16 h2 = __builtin_bit_cast(_Float16, (u16)(w1 & 0xffff)), h3 = __builtin_bit_cast(_Float16, (u16)(w1 >> 16));
        o[i] = pk4_bf8((float)h0, (float)h1, (float)h2, (float)h3);
      }
      st16(z8 + SZ8::off(row, c), make_uint4(o[0], o[1], o[2], o[3]));
    }
  };

  const int tid = threadIdx.x, lane = tid & 63, ns = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int n = ns * 32 + l32;
  const long row0 = (long)blockIdx.x * R;
  const uint32_t tbytes = R * H * 4;
  const long tb0 = row0 * H;
  const rsrc_t pd = mkrsrc(delta + tb0, tbytes), ph = mkrsrc(hf + tb0, tbytes), pr = mkrsrc(rin + tb0, tbytes),
               pu = mkrsrc(uin + tb0, tbytes), pc = mkrsrc(cin + tb0, tbytes);
  const int vo = (4 * hh * H + n) * 4;
  const long twg = wg_off(n, row0 + 4 * hh, H);  // dX^T, dzc^T, dzg^T: K-blocked [H][N] arrays
  TSMARK(1, 0);

  // ---- phase 1: dzc, and the u half of dzg (needs no product): one read of
  // delta, u, c, h and r; delta*u and r stay in registers for phase 2 (round
  // 6: phase 2 loaded r from HBM after product 1, a lockstep memory phase;
  // now it re-reads only h, which phase 1 left in L2)
  float csum = 0.f, usum = 0.f;
  float du[RT][16], rk[RT][16];
  uint2 kb = make_uint2(0u, 0u);
  const int jt0 = (int)((row0 & 127) >> 5);  // first 32-row tile of this workgroup in its graph
  if (sbits) kb = sbits[(row0 >> 7) * (2 * H) + tid];
  const rsrc_t pdo = mkrsrc(dh_out + tb0, tbytes);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float dz[4], zu[4];
      const float4 u4 = bld4_p<kGbAux>(pu, qm_vo(hh, n, H), qm_so(rt, q, H)), c4 = bld4_p<kGbAux>(pc, qm_vo(hh, n, H), qm_so(rt, q, H));
      const float4 r4 = bld4_p<kGbAux>(pr, qm_vo(hh, n, H), qm_so(rt, q, H));
      const float uq[4] = {u4.x, u4.y, u4.z, u4.w}, cq[4] = {c4.x, c4.y, c4.z, c4.w};
      rk[rt][4 * q] = r4.x; rk[rt][4 * q + 1] = r4.y; rk[rt][4 * q + 2] = r4.z; rk[rt][4 * q + 3] = r4.w;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ro = rt * 32 + acc_row0(4 * q + i);
        const int so = ro * H * 4;
        float d = bld_p<kGbAux>(pd, vo, so) * ds;
        if (sbits) {
          const int jt = jt0 + rt;
          d = (((jt >> 1 ? kb.y : kb.x) >> ((jt & 1) * 16 + 4 * q + i)) & 1u) ? d * sscale : 0.0f;
        }
        const float u = uq[i], c = cq[i], h = bld_p<0>(ph, vo, so);
        dz[i] = d * (1.0f - u) * (1.0f - c * c);
        zu[i] = d * (h - c) * u * (1.0f - u);
        du[rt][4 * q + i] = d * u;
        csum += dz[i];
        usum += zu[i];
        zput(ro + 4 * hh, n, dz[i]);
        zput(ro + 4 * hh, H + n, zu[i]);  // K >= H: not read by product 1
      }
      st_col4w<PREC>(dzcT + twg + rt * 32 * H + 8 * q, dz[0], dz[1], dz[2], dz[3]);
      st_col4w<PREC>(dzgT + twg + (long)H * N + rt * 32 * H + 8 * q, zu[0], zu[1], zu[2], zu[3]);
      if ((q & (GB_GROUP - 1)) == GB_GROUP - 1) __builtin_amdgcn_sched_barrier(0);  // bound the loads in flight (VGPR budget)
    }
  }
  csum += __shfl_xor(csum, 32);
  usum += __shfl_xor(usum, 32);
  if (hh == 0) {
    if (bpart) {
      bpart[(long)blockIdx.x * 3 * H + H + n] = usum;
      bpart[(long)blockIdx.x * 3 * H + 2 * H + n] = csum;
    } else {
      atomicAdd(dbc + n, csum);
      atomicAdd(dbg + H + n, usum);
    }
  }
  __syncthreads();
  if constexpr (SPLIT) {
    z8_fill(0, 2 * H / 16);  // dzc and dzg_u
    __syncthreads();
  }
  TSMARK(1, 1);

  // ---- product 1: [dX1 | d(rh)] = dzc @ Wc^T
  f32x16 a1[RT], a2[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) { a1[rt] = splat(0.f); a2[rt] = splat(0.f); }
  // Split mode (round 6): dz @ W^T ~= f16(dz) f16(W)^T  [f16 MFMAs, 1 per 16 k and tile]
  //                                 + e5m2(dz) e4m3(W_lo 2^18)^T 2^-18  [one fp8 32x32x64
  //                                   MFMA per 64 k and tile, mfma_f8corr's scales]
  // 6 cycle units per 64 k and tile instead of 8 for round 5's dz hi/lo x W hi,
  // with W's lo limb back in: the seven gradients' error 5.5-10.1e-4 -> 3.1-5.4e-4
  // (oracle backward_operand_policy, gru_wt "f8lo", b = 8, T = 5 / 8, three seeds).
  // The fragment ring alternates 6 units per 64 k in two slots of 8 VGPRs: the f16
  // fragments of 4 k-steps (both tiles), then the 32-byte fp8 fragment of each
  // tile (k_pack_multi f8 = 2: [strip][64-k block][64 lanes][32 B], byte j of lane
  // half hh = k 64 kb + 32 hh + j); 4 cycle units of MFMA per unit at RT = 2.
  auto gb_f8_product = [&](auto nks_c, const u16* WT, const char* W8) {
    constexpr int NKS = decltype(nks_c)::value, NKB = NKS / 4;
    auto ldh = [&](int ks) { return F2{frag_ld(WT, ns, ks, NKS, lane), frag_ld(WT, NS + ns, ks, NKS, lane)}; };
    auto ldf = [&](int strip, int kb) {
      const uint4* f = (const uint4*)(W8 + ((size_t)(strip * NKB + kb) * 64 + lane) * 32);
      return F2{f[0], f[1]};
    };
    auto hi = [&](int ks, const F2& w) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const frag ah = lds_frag(z_hi, SZ::off(rt * 32 + l32, 2 * ks + hh));
        a1[rt] = mfma<true>(ah, w.a, a1[rt]);
        a2[rt] = mfma<true>(ah, w.b, a2[rt]);
      }
    };
    auto f8 = [&](int kb, const F2& w, auto second) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int row = rt * 32 + l32;
        const uint4 p0 = ld16(z8 + SZ8::off(row, 4 * kb + 2 * hh)), p1 = ld16(z8 + SZ8::off(row, 4 * kb + 2 * hh + 1));
        if constexpr (decltype(second)::value) a2[rt] = mfma_f8corr(p0, p1, w.a, w.b, a2[rt]);
        else a1[rt] = mfma_f8corr(p0, p1, w.a, w.b, a1[rt]);
      }
    };
    F2 r0 = ldh(0), r1 = ldh(1);
#pragma unroll 1
    for (int kb = 0; kb < NKB; ++kb) {
      const int kn = min(kb + 1, NKB - 1);
      hi(4 * kb, r0);
      r0 = ldh(4 * kb + 2);
      __builtin_amdgcn_sched_barrier(0);
      hi(4 * kb + 1, r1);
      r1 = ldh(4 * kb + 3);
      __builtin_amdgcn_sched_barrier(0);
      hi(4 * kb + 2, r0);
      r0 = ldf(ns, kb);
      __builtin_amdgcn_sched_barrier(0);
      hi(4 * kb + 3, r1);
      r1 = ldf(NS + ns, kb);
      __builtin_amdgcn_sched_barrier(0);
      f8(kb, r0, std::false_type{});
      r0 = ldh(4 * kn);
      __builtin_amdgcn_sched_barrier(0);
      f8(kb, r1, std::true_type{});
      r1 = ldh(4 * kn + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  if constexpr (SPLIT) {
    gb_f8_product(std::integral_constant<int, H / 16>{}, WcTp, (const char*)(WcTp + wlo_c));
  } else {
    auto ld1 = [&](int ks) { return F2{frag_ld(WcTp, ns, ks, KS, lane), frag_ld(WcTp, NS + ns, ks, KS, lane)}; };
    b_pipeline<KS, GBD, GB_UNROLL>(ld1, [&](int ks, const auto& w) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const frag ah = lds_frag(z_hi, SZ::off(rt * 32 + l32, 2 * ks + hh));
        gb_mma<PREC>(a1[rt], a2[rt], ah, ah, w);
      }
    });
  }
  __syncthreads();  // dzc reads done
  TSMARK(1, 2);

  // ---- phase 2: dh (into a2), the r half of dzg
  float rsum = 0.f;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float zr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * q + i;
        const int ro = rt * 32 + acc_row0(r);
        const float h = bld_p<0>(ph, vo, ro * H * 4), rr = rk[rt][r];
        const float drh = a2[rt][r];
        a2[rt][r] = du[rt][r] + drh * rr;
        zr[i] = drh * h * rr * (1.0f - rr);
        rsum += zr[i];
        zput(ro + 4 * hh, n, zr[i]);
      }
      st_col4w<PREC>(dzgT + twg + rt * 32 * H + 8 * q, zr[0], zr[1], zr[2], zr[3]);
    }
  }
  rsum += __shfl_xor(rsum, 32);
  if (hh == 0) {
    if (bpart) bpart[(long)blockIdx.x * 3 * H + n] = rsum;
    else atomicAdd(dbg + n, rsum);
  }
  __syncthreads();
  if constexpr (SPLIT) {
    z8_fill(0, H / 16);  // dzg_r
    __syncthreads();
  }
  TSMARK(1, 3);

  // ---- product 2: [dX2 | dh2] = dzg @ Wg^T
  if constexpr (SPLIT) {
    gb_f8_product(std::integral_constant<int, H / 8>{}, WgTp, (const char*)(WgTp + wlo_g));
  } else {
    auto ld2 = [&](int ks) { return F2{frag_ld(WgTp, ns, ks, 2 * KS, lane), frag_ld(WgTp, NS + ns, ks, 2 * KS, lane)}; };
    b_pipeline<2 * KS, GBD, GB_UNROLL>(ld2, [&](int ks, const auto& w) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const frag ah = lds_frag(z_hi, SZ::off(rt * 32 + l32, 2 * ks + hh));
        gb_mma<PREC>(a1[rt], a2[rt], ah, ah, w);
      }
    });
  }
  TSMARK(1, 4);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      st_col4<PREC>(dXT + twg + rt * 32 * H + 8 * q, a1[rt][4 * q], a1[rt][4 * q + 1], a1[rt][4 * q + 2],
                     a1[rt][4 * q + 3]);
#pragma unroll
    for (int r = 0; r < 16; ++r) bst(pdo, a2[rt][r], vo, (rt * 32 + acc_row0(r)) * H * 4);
  }
  TSMARK(1, 5);
  TSCLK(1, 1);
}
