// ggnn_common.h -- device helpers shared by the GGNN kernels (gfx950 / CDNA4).
//
// MFMA fragment maps of v_mfma_f32_32x32x16_bf16 (the only matrix instruction
// used):
//   A[32x16]: lane l holds A[l&31][8*(l>>5) + j], j = 0..7
//   B[16x32]: lane l holds B[8*(l>>5) + j][l&31]
//   C/D     : lane l, reg r holds D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]
// An accumulator tile is reused as the next product's B operand when the next
// product contracts over its ROW index: k-step s takes regs 8s..8s+7, and
// element j of lane-half hh is row 16s + 8(j>>2) + 4hh + (j&3).
//
// Precision policy (template parameter PREC):
//   PREC = 0  "bf16": operands rounded to bf16, fp32 accumulation;
//             activations between kernels stored as bf16.
//   PREC = 1  "fp16": the same with f16 operands (3 more mantissa bits, same
//             MFMA rate; the path's operands are range-bounded, |x| << 65504).
//   PREC = 2  "fp32-class" (SPLIT): every non-exact operand x is carried as two
//                  fp16 limbs x_hi = f16(x), x_lo = f16(x - x_hi) (~22-bit
//                  mantissa); a product is a_hi*b_hi + a_hi*b_lo + a_lo*b_hi
//                  on v_mfma_f32_32x32x16_f16 (3 MFMAs, 2 when one side is
//                  exact, e.g. the 0/1 adjacency); activations between kernels
//                  stored as fp32.  The f16 range (|x| < 65504) covers every
//                  operand of the path (|h| < 1, |W| < 1, |X|, |M|, |dz| << 1e4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

typedef uint16_t u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
// an MFMA A/B operand fragment: 8 x 16-bit (bf16 or f16 limbs)
typedef uint4 frag;
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));

#define DEV __device__ __forceinline__
#define HDI __host__ __device__ inline
#ifdef GGNN_TS
__device__ unsigned long long g_ts[4][2048 * 8];
#define TSMARK(k, i) do { if (threadIdx.x == 0) g_ts[k][blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define TSVAL(k, i, v) do { if (threadIdx.x == 0) g_ts[k][blockIdx.x * 8 + (i)] = (unsigned long long)(v); } while (0)
// in-kernel clock (MI355X_MICROARCH.md "DVFS give-back" item 6): shader-clock
// ticks (s_memtime) and 100 MHz ticks (s_memrealtime) at a workgroup's start
// and end; clock = d(memtime) / d(memrealtime) x 100 MHz.  Diagnostic build
// only: the stamps go to g_clk, which nothing in the kernels reads.
__device__ unsigned long long g_clk[4][2048 * 4];
#define TSCLK(k, e) do { if (threadIdx.x == 0) { \
    g_clk[k][blockIdx.x * 4 + 2 * (e)] = __builtin_amdgcn_s_memrealtime(); \
    g_clk[k][blockIdx.x * 4 + 2 * (e) + 1] = __builtin_amdgcn_s_memtime(); } } while (0)
#else
#define TSCLK(k, e) do {} while (0)
#define TSMARK(k, i) do {} while (0)
#define TSVAL(k, i, v) do {} while (0)
#endif

enum { PREC_BF16 = 0, PREC_F16 = 1, PREC_SPLIT = 2 };
template <int PREC> struct Prec {
  static constexpr bool split = PREC == PREC_SPLIT;  // two f16 limbs per operand
  static constexpr bool f16 = PREC != PREC_BF16;     // limb format
};
// storage type of activations passed between kernels: limbs, or fp32 (split)
template <int PREC>
using ActT = typename std::conditional<Prec<PREC>::split, float, u16>::type;

DEV u16 f2bf(float x) { return __builtin_bit_cast(u16, (__bf16)x); }
DEV float bf2f(u16 x) { return __uint_as_float(((uint32_t)x) << 16); }
DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

// ---- 16-bit operand limbs: bf16 (F16 = false) or f16 (F16 = true)
template <bool F16> DEV u16 to_limb(float x) {
  if constexpr (F16) return __builtin_bit_cast(u16, (_Float16)x);
  else return f2bf(x);
}
template <bool F16> DEV float from_limb(u16 x) {
  if constexpr (F16) return (float)__builtin_bit_cast(_Float16, x);
  else return bf2f(x);
}
// residual of the limb rounding of x
template <bool F16> DEV float lo_part(float x) { return x - from_limb<F16>(to_limb<F16>(x)); }
// pairs through the packed converts (v_cvt_pk_f16_f32 / v_cvt_pk_bf16_f32:
// one instruction per pair, round to nearest even like the scalar casts)
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
template <bool F16> DEV uint32_t pk(float a, float b) {
  const f32x2v v = {a, b};
  if constexpr (F16) return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2v));
  else return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}
#ifndef GGNN_LIMB_MIX
#define GGNN_LIMB_MIX 1
#endif
template <bool F16, bool MIX = GGNN_LIMB_MIX> DEV uint32_t pk_lo(float a, float b) {
  if constexpr (F16 && MIX) {
    // f16 residuals by v_fma_mix{lo,hi}_f16: f16(x - f32(hi)) in one
    // instruction per element (x - hi is exact in fp32, then one RNE rounding:
    // the same bits as the convert / subtract / convert sequence, 3 instead of
    // 5 instructions per pair; tools/limb_mix_test.hip checks it on the GPU).
    // MIX = false keeps the convert sequence: k_fwd_fused measured ~1.4 %
    // slower with the asm pair in its blend (fewer scheduling choices there),
    // while the ring GEMM and k_prop_bwd gained 1-5 %
    const uint32_t hi = pk<true>(a, b);
    uint32_t lo;
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(lo) : "v"(a), "v"(hi));
    // (the result is an MFMA A/B operand: the VALU write -> MFMA read wait
    // states go INSIDE the string, hipcc pads only one state after an asm
    // statement; with that one, k_gemm_ks read stale limbs in fp32 mode)
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\ts_nop 1" : "+v"(lo) : "v"(b), "v"(hi));
    return lo;
  }
  const f32x2v v = {a, b};
  f32x2v back;
  if constexpr (F16) back = __builtin_convertvector(__builtin_convertvector(v, f16x2v), f32x2v);
  else back = __builtin_convertvector(__builtin_convertvector(v, bf16x2v), f32x2v);
  const f32x2v lo = v - back;
  return pk<F16>(lo.x, lo.y);
}
template <bool F16> DEV frag pk8(const float* x) {
  return make_uint4(pk<F16>(x[0], x[1]), pk<F16>(x[2], x[3]), pk<F16>(x[4], x[5]), pk<F16>(x[6], x[7]));
}
// one element's f16 residual limb (v_fma_mixlo_f16 under GGNN_LIMB_MIX)
DEV u16 lo_limb16(float v) {
  if constexpr (GGNN_LIMB_MIX) {
    const uint32_t hi = __builtin_bit_cast(u16, (_Float16)v);
    uint32_t lo;
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(lo) : "v"(v), "v"(hi));
    return (u16)lo;
  }
  return to_limb<true>(lo_part<true>(v));
}
template <bool F16, bool MIX = GGNN_LIMB_MIX> DEV frag pk8_lo(const float* x) {
  return make_uint4(pk_lo<F16, MIX>(x[0], x[1]), pk_lo<F16, MIX>(x[2], x[3]), pk_lo<F16, MIX>(x[4], x[5]),
                    pk_lo<F16, MIX>(x[6], x[7]));
}
template <bool F16> DEV float limb_elem(frag f, int j) {
  const uint32_t w = (j < 2) ? f.x : (j < 4) ? f.y : (j < 6) ? f.z : f.w;
  return from_limb<F16>((u16)((j & 1) ? (w >> 16) : (w & 0xffff)));
}

template <bool F16> DEV f32x16 mfma(frag a, frag b, f32x16 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
DEV f32x16 splat(float x) {
  f32x16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = x;
  return r;
}
DEV float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }
DEV float tanh_f(float x) { return 1.0f - 2.0f / (__expf(2.0f * x) + 1.0f); }
DEV constexpr int acc_row0(int r) { return (r & 3) + 8 * (r >> 2); }
DEV int acc_row(int r, int hh) { return acc_row0(r) + 4 * hh; }

// operand fragment(s) of k-step s taken from an accumulator tile
template <bool F16> DEV frag acc_hi(const f32x16& a, int s) {
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = a[8 * s + j];
  return pk8<F16>(x);
}
template <bool F16, bool MIX = GGNN_LIMB_MIX> DEV frag acc_lo(const f32x16& a, int s) {
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = a[8 * s + j];
  return pk8_lo<F16, MIX>(x);
}

// D += A*B with the precision policy (split: f16 limbs, 3 products)
template <int PREC>
DEV void mma(f32x16& acc, frag ah, frag al, frag bh, frag bl) {
  if constexpr (Prec<PREC>::split) {
    acc = mfma<true>(al, bh, acc);
    acc = mfma<true>(ah, bl, acc);
  }
  acc = mfma<Prec<PREC>::f16>(ah, bh, acc);
}
// D += A*B where A is exact in the limb format (0/1 adjacency)
template <int PREC>
DEV void mma_xa(f32x16& acc, frag a, frag bh, frag bl) {
  if constexpr (Prec<PREC>::split) acc = mfma<true>(a, bl, acc);
  acc = mfma<Prec<PREC>::f16>(a, bh, acc);
}
// D += A*B where B is exact in the limb format
template <int PREC>
DEV void mma_xb(f32x16& acc, frag ah, frag al, frag b) {
  if constexpr (Prec<PREC>::split) acc = mfma<true>(al, b, acc);
  acc = mfma<Prec<PREC>::f16>(ah, b, acc);
}

// ---- limb corrections on the block-scaled fp8 MFMA (fp32-parity mode, k_prop_bwd's
// dh += dM W_c^T).  The split product a.b = a_hi b_hi + a_hi b_lo + a_lo b_hi takes
// its main term on v_mfma_f32_32x32x16_f16 (2 per 32 k) and BOTH correction terms
// of 32 k's on one v_mfma_scale_f32_32x32x64_f8f6f4 (K = 64, twice the cycles of
// one 16-bit 32x32x16 form): 4 instead of 6 cycle units per 32 k.  Operand layout
// (measured, tools/mx_hybrid_probe.hip, profiles/r06n_mx_layout.json): lane l holds
// 32 bytes; A byte j of lane l meets B byte j of lane l' iff l >> 5 == l' >> 5
// (row = A lane & 31, column = B lane & 31); bytes 0-15 of both lane halves take
// the scale of lane (l & 31), bytes 16-31 that of lane (l & 31) + 32.  Here:
//   A lane half 0: e5m2(a)            A lane half 1: e5m2(a_lo 2^F8_M)
//   B lane half 0: e4m3(b_lo 2^(F8_Q + F8_M))   B lane half 1: e4m3(b_hi 2^F8_Q)
// each byte j = k offset j inside the 32-k block; both halves carry 2^(F8_Q+F8_M),
// which B's E8M0 scale (127 - F8_Q - F8_M) removes.  The activation side is
// e5m2 (range 2^-16 .. 57344, no per-block scale needed); the weight side e4m3
// with a fixed 2^F8_Q: |W| up to 448 / 2^F8_Q = 3.5 is represented, larger
// weights saturate (k_pack_multi clamps), which costs only correction-term
// accuracy.  Error budget (oracle emulation, tools/precision_policies.py
// --hybrid): the seven gradients' max |err| / max |ref| unchanged (5.3-6.6e-4
// against 5.3-6.6e-4 for the 3-product form, b = 8, T = 5 and 8).
constexpr int F8_Q = 7, F8_M = 11;
typedef int i32x8 __attribute__((ext_vector_type(8)));
// 4 floats -> 4 packed bytes (byte i = value i), OCP e5m2 / e4m3, RNE
DEV uint32_t pk4_bf8(float a, float b, float c, float d) {
  uint32_t w = (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(c, d, (int)w, true);
}
DEV uint32_t pk4_fp8(float a, float b, float c, float d) {
  uint32_t w = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c, d, (int)w, true);
}
// D += (A8 . B8) 2^-(F8_Q + F8_M): A e5m2, B e4m3, one 32x32x64 MFMA
DEV f32x16 mfma_f8corr(uint4 a0, uint4 a1, uint4 b0, uint4 b1, f32x16 c) {
  const i32x8 fa = {(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
  const i32x8 fb = {(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa, fb, c, 1, 0, 0, 127, 0, 127 - F8_Q - F8_M);
}

// XOR swizzle of 16-byte chunks inside rows of NCH chunks so that the 32
// distinct rows of one MFMA operand read land on distinct LDS bank slots.
template <int NCH>
struct Swz {
  static constexpr int M = (NCH % 16 == 0) ? 15 : (NCH % 8 == 0) ? 7 : (NCH % 4 == 0) ? 3 : 0;
  static DEV int off(int row, int ch) { return row * NCH * 16 + ((ch ^ (row & M)) << 4); }
  static DEV int eoff(int row, int e) { return off(row, e >> 3) + ((e & 7) << 1); }
};

DEV uint4 ld16(const void* p) { return *(const uint4*)p; }
DEV void st16(void* p, uint4 v) { *(uint4*)p = v; }
DEV frag lds_frag(const char* img, int off) { return ld16(img + off); }

// LDS-DMA staging of a [R][NCH] tile of 16-byte chunks (row-major in global)
// into a Swz<NCH> LDS image.  The DMA destination is lane-linear (wave base +
// 16*lane), so the swizzle goes on the SOURCE address: LDS slot (row, pc)
// receives logical chunk pc ^ (row & M), the same involution Swz::off reads
// with.  No VGPR staging; completion is on vmcnt (a __syncthreads drains it).
template <int NCH, int R, int NT, int AUX = 0>
DEV void glds_tile(char* lds, const u16* src, int tid) {
  typedef Swz<NCH> S;
  constexpr int TOT = R * NCH;
  const int lane = tid & 63;
#pragma unroll
  for (int p = 0; p < (TOT + NT - 1) / NT; ++p) {
    const int qb = p * NT + (tid & ~63);  // wave-uniform first slot
    if (qb < TOT) {
      const int q = qb + lane, row = q / NCH, pc = q % NCH;
      __builtin_amdgcn_global_load_lds((const void*)(src + (row * NCH + (pc ^ (row & S::M))) * 8),
                                       (__attribute__((address_space(3))) void*)(lds + qb * 16), 16, 0, AUX);
    }
  }
}

// LDS-DMA of 16 B per lane in inline asm: invisible to hipcc's waitcnt pass,
// which would otherwise wait vmcnt(0) before every ds_read of the ring (it
// cannot tell the ring slots apart); completion is counted by hand below.
DEV void glds16_asm(const void* gsrc, const char* lds_dst) {
  unsigned keep;
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_dst);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}

// B-operand fragment of a packed matrix: [strip][kstep][64 lanes][8] limbs
DEV frag frag_ld(const u16* base, int strip, int ks, int nks, int lane) {
  return ld16(base + ((size_t)(strip * nks + ks) * 64 + lane) * 8);
}

// ---- software pipeline for B-operand fragments streamed from packed weights
// (L2-resident): the fragments of k-step ks+D are loaded while k-step ks runs
// its MFMAs, so each load has D k-steps of MFMA work to hide its L2 latency.
// The ring is indexed statically (inner loop unrolled by D); the outer loop is
// kept rolled so the scheduler cannot hoist a whole K sweep of LDS reads into
// registers.
struct F2 { frag a, b; };
struct F4 { frag a, b, c, d; };
// UNROLL: 0 = fully unrolled k loop (exact vmcnt counts everywhere), else the
// outer loop is unrolled by that factor (smaller code and register live ranges;
// the waitcnt pass is conservative at the loop head).
template <int KS, int D, int UNROLL = 0, typename LD, typename BODY>
DEV void b_pipeline(LD&& ld, BODY&& body) {
  static_assert(KS % D == 0, "k-steps must be a multiple of the pipeline depth");
  using FB = decltype(ld(0));
  FB ring[D];
#pragma unroll
  for (int p = 0; p < D; ++p) ring[p] = ld(p);
#pragma unroll (UNROLL == 0 ? KS / D : UNROLL)
  for (int k0 = 0; k0 < KS; k0 += D) {
#pragma unroll
    for (int p = 0; p < D; ++p) {
      // consume slot p, then refill it: the refill is issued after the MFMAs
      // that read the slot, so the slot keeps its registers (no copies, whose
      // moves would force a vmcnt(0) on the younger loads)
      // (unconditional, clamped: a branch here makes the waitcnt pass assume
      // the worst case and emit vmcnt(0) at the loop head)
      body(k0 + p, ring[p]);
      ring[p] = ld(min(k0 + p + D, KS - 1));
      __builtin_amdgcn_sched_barrier(0);  // keep the refill here (not sunk to the loop end)
    }
  }
}

// The same k loop without the explicit ring (fragments loaded at their k-step;
// the compiler schedules them): better where the ring's registers would spill
// or the fully unrolled loop already hides the latency.
template <int KS, int U, typename LD, typename BODY>
DEV void b_direct(LD&& ld, BODY&& body) {
#pragma unroll U
  for (int ks = 0; ks < KS; ++ks) body(ks, ld(ks));
}

// Raw buffer access with an SRD built from wave-uniform values: one 32-bit
// voffset VGPR per lane, per-element constants in the SGPR soffset.
// 4x4 transpose of 16-bit values inside each lane quad.  Lane L (= lane & 3)
// holds column L of a 4-row block: P0 = rows (0,1), P1 = rows (2,3), low half
// first.  Returns row L's 4 columns (column 0 in the low half of .x): an
// accumulator quad (registers 4q..4q+3 = 4 consecutive rows, column = lane)
// becomes one 8-byte row-contiguous store per lane.  Two DPP exchanges.
DEV v2u32 quad_transpose4(uint32_t P0, uint32_t P1, int L) {
  const bool up = L & 2, odd = L & 1;
  const uint32_t Y = __builtin_amdgcn_update_dpp(0u, up ? P0 : P1, 0x4E, 0xF, 0xF, false);  // lane ^ 2
  const uint32_t Q0 = up ? Y : P0, Q1 = up ? P1 : Y;  // rows 2(L>>1)+{0,1} of columns L&1, (L&1)+2
  const uint32_t S = odd ? ((Q0 & 0xFFFFu) | (Q1 << 16)) : ((Q0 >> 16) | (Q1 & 0xFFFF0000u));
  const uint32_t R = __builtin_amdgcn_update_dpp(0u, S, 0xB1, 0xF, 0xF, false);            // lane ^ 1
  v2u32 w;
  if (!odd) {
    w.x = (Q0 & 0xFFFFu) | (R << 16);
    w.y = (Q1 & 0xFFFFu) | (R & 0xFFFF0000u);
  } else {
    w.x = (R & 0xFFFFu) | (Q0 & 0xFFFF0000u);
    w.y = (R >> 16) | (Q1 & 0xFFFF0000u);
  }
  return w;
}

// ---- dropout: Philox4x32-10 (Salmon et al., SC'11; Random123 constants)
// keyed by the 64-bit step seed.  A counter names a group of 4 consecutive
// rows at one column, and the 4 output words are the 4 rows' draws, which
// matches the MFMA accumulator layout (4 consecutive rows per register quad):
//   edge-weight mask, timestep t, W[c][i][j]:  ctr = (i>>2, j, c, t)
//   state mask,       timestep t, h[g][i][k]:  ctr = (i>>2, k, g, 0x80000000|t)
// element kept iff word[i&3] < thr, thr = floor(keep * 2^32); kept elements
// are scaled by 1/keep (tf.nn.dropout: x * (1/keep) * mask).
struct Drop {
  uint32_t k0, k1;  // key = seed
  uint32_t thr;     // 0 = dropout off
  float scale;      // 1 / keep
  // GGNN_SEED_DEVICE: the key is read from device memory at run time
  // (kp[0] = low, kp[1] = high word of the uint64 seed), so a captured
  // hipGraph replays with each step's fresh seed
  const uint32_t* kp;
};
DEV uint32_t dkey0(const Drop& d) { return d.kp ? d.kp[0] : d.k0; }
DEV uint32_t dkey1(const Drop& d) { return d.kp ? d.kp[1] : d.k1; }
// the Drop a kernel works with: a device-resident key loaded once at kernel
// entry; the copy's kp is a known null, so dkey* fold to k0 / k1 in its loops
DEV Drop drop_resolve(Drop d) {
  if (d.kp) {
    d.k0 = d.kp[0];
    d.k1 = d.kp[1];
  }
  d.kp = nullptr;
  return d;
}
DEV uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t lo0 = c.x * 0xD2511F53u, hi0 = __umulhi(c.x, 0xD2511F53u);
    const uint32_t lo1 = c.z * 0xCD9E8D57u, hi1 = __umulhi(c.z, 0xCD9E8D57u);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
DEV uint32_t u4_get(const uint4& w, int j) { return j == 0 ? w.x : j == 1 ? w.y : j == 2 ? w.z : w.w; }
DEV uint4 state_words(const Drop& d, int g, int i, int k, int t) {
  return philox4x32_10(make_uint4((uint32_t)i >> 2, (uint32_t)k, (uint32_t)g, 0x80000000u | (uint32_t)t), dkey0(d), dkey1(d));
}
DEV uint4 edge_words(const Drop& d, int c, int i, int j, int t) {
  return philox4x32_10(make_uint4((uint32_t)i >> 2, (uint32_t)j, (uint32_t)c, (uint32_t)t), dkey0(d), dkey1(d));
}
DEV float drop_apply(const Drop& d, uint32_t w, float x) { return w < d.thr ? x * d.scale : 0.0f; }
// the GRU state update h' = u h + (1 - u) c with one rounding order wherever
// it is formed (k_gen_blend, k_gemm_ks's fused epilogue)
DEV float gru_blend(float u, float h, float c) { return __builtin_fmaf(u, h, (1.0f - u) * c); }
// dzg_r = d(rh) h r (1 - r) (k_gen_bwd2, k_gemm_ks's fused epilogue)
DEV float gru_dzg_r(float x, float h, float r) { return x * h * r * (1.0f - r); }

// ---- backward gradient scaling.  The btb loss is divided by the number of
// targets (chem_tensorflow.py:360,399-403), so dL/dh_T arrives at ~1/b per
// element; as f16 limbs such values sit at or below the f16 normal range
// (2^-14) and lose their low bits.  The backward therefore runs on
// S * dL/dh_T with S = 2^-floor(log2 max|dL/dh_T|) (exact: a power of two,
// so S*x and x/S are the same fp32 mantissas) and divides every output by S.
// gmax holds the bit pattern of max|dL/dh_T| (non-negative floats order like
// their bits, so an atomicMax on the bits is a max on the values).
DEV int gscale_exp(uint32_t gmax_bits) {
  const float m = __uint_as_float(gmax_bits);
  if (!(m > 0.0f) || !(m < 3.0e38f)) return 0;  // zero / non-finite: no scaling
  int e = ((int)(gmax_bits >> 23) & 0xff) - 127;  // floor(log2 m) for normal m
  if (e == -127) e = -126;                         // subnormal maxima: scale by 2^126 at most
  return -max(-126, min(126, e));
}
DEV float gscale(const uint32_t* gmax) { return gmax ? __builtin_ldexpf(1.0f, gscale_exp(*gmax)) : 1.0f; }
DEV float gunscale(const uint32_t* gmax) { return gmax ? __builtin_ldexpf(1.0f, -gscale_exp(*gmax)) : 1.0f; }

typedef __amdgpu_buffer_rsrc_t rsrc_t;
// cache-policy operand of the raw buffer builtins: nontemporal (gfx950 NT bit),
// for write-once streams that are read back only by a later kernel (measured:
// -5 % on k_prop_bwd's dM^T stream, and less L2 pollution for the next kernel)
constexpr int kNT = 2;
DEV rsrc_t mkrsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}
DEV float bld(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
DEV void bst(rsrc_t r, float v, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, soff, 0);
}

// ---- block-cooperative staging of a row-major [R][K] activation tile into
// swizzled LDS image(s): bf16 -> one image; fp32 -> hi and lo images.
template <int PREC, int R, int K, int NT>
DEV void stage_rows(char* hi, char* lo, const ActT<PREC>* src, long ld, int tid) {
  constexpr int KCH = K / 8;
  typedef Swz<KCH> S;
  for (int q = tid; q < R * KCH; q += NT) {
    const int row = q / KCH, ch = q % KCH;
    if constexpr (Prec<PREC>::split) {
      const float4 a = *(const float4*)(src + row * ld + ch * 8);
      const float4 b = *(const float4*)(src + row * ld + ch * 8 + 4);
      const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      st16(hi + S::off(row, ch), pk8<true>(x));
      st16(lo + S::off(row, ch), pk8_lo<true>(x));
    } else {
      st16(hi + S::off(row, ch), ld16(src + row * ld + ch * 8));
    }
  }
}

// ---- chunk-major LDS image of R rows: 16-byte chunk ch (8 consecutive k) of
// row r at ch * (R * 16) + r * 16.  A fragment read (16 lanes = 16 rows of one
// chunk) is 256 contiguous bytes, and its k offset is an immediate.
template <int R> DEV int kimg(int row, int ch) { return ch * (R * 16) + row * 16; }
// block-cooperative staging into chunk-major image(s); consecutive lanes take
// consecutive rows of one chunk (conflict-free 16-byte LDS writes)
template <int PREC, int R, int K, int NT>
DEV void stage_rows_k(char* hi, char* lo, const ActT<PREC>* src, long ld, int tid) {
  for (int q = tid; q < R * (K / 8); q += NT) {
    const int row = q % R, ch = q / R;
    if constexpr (Prec<PREC>::split) {
      const float4 a = *(const float4*)(src + row * ld + ch * 8);
      const float4 b = *(const float4*)(src + row * ld + ch * 8 + 4);
      const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      st16(hi + kimg<R>(row, ch), pk8<true>(x));
      st16(lo + kimg<R>(row, ch), pk8_lo<true>(x));
    } else {
      st16(hi + kimg<R>(row, ch), ld16(src + row * ld + ch * 8));
    }
  }
}

// Saved GRU activations r, u, c (fp32, written by the GRU forward kernels and
// read only by k_gru_bwd) are stored row-quad-major: element (row, n) sits at
// float ((row >> 2) * H + n) * 4 + (row & 3).  The 4 consecutive rows an MFMA
// accumulator quad holds (registers 4q..4q+3) are 16 contiguous bytes: one
// dwordx4 per quad, no cross-lane shuffle.  Offsets are relative to the row
// tile's base pointer (first row a multiple of 4).
DEV int qm_vo(int hh, int n, int H) { return (hh * H + n) * 16; }
DEV int qm_so(int rt, int q, int H) { return (8 * rt + 2 * q) * H * 16; }
// 16-byte global store, saddr form (wave-uniform base + soff, 32-bit lane
// offset).  Not buffer_store_dwordx4: that store read its data VGPRs after a
// following instruction had rewritten them (DESIGN.md §4 lessons).
DEV void gst4(void* base, int voff, int soff, float4 v) {
  *(float4*)((char*)base + soff + (unsigned long)(unsigned)voff) = v;
}
DEV float4 bld4(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
// the same with a cache-policy operand (kNT: nontemporal)
template <int AUX> DEV float bld_p(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX));
}
template <int AUX> DEV float4 bld4_p(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, AUX));
}
// 16-byte nontemporal global store (saddr form as gst4)
DEV void gst4_nt(void* base, int voff, int soff, float4 v) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, (f4v*)((char*)base + soff + (unsigned long)(unsigned)voff));
}

// ---- store 4 consecutive rows (acc regs 4q..4q+3) of one column into a
// transposed [col][row] activation array (rows contiguous)
template <int PREC>
DEV void st_col4(ActT<PREC>* dst, float a, float b, float c, float d) {
  if constexpr (Prec<PREC>::split) *(float4*)dst = make_float4(a, b, c, d);
  else *(uint2*)dst = make_uint2(pk<Prec<PREC>::f16>(a, b), pk<Prec<PREC>::f16>(c, d));
}

// Weight-gradient operand layout.  An operand is an [H][N] array (hidden
// index n, node row k) stored in K-blocks of 32 rows: block k>>5 holds
// [H][32], so element (n, k) sits at wg_off(n, k, H).  A weight-gradient K
// slice (all H rows x 32 node rows) is then one contiguous 16 KiB span
// instead of H 64-byte pieces 2N bytes apart, which all fell into the same
// L2 sets (k_wgrad256: 0.42 -> 0.32 ms/step at config 3), and a 4-row store
// of 8 lanes fills one 64-byte row.  Needs N % 32 == 0 (V is 32, 64 or 128).
DEV long wg_off(int n, long k, int H) { return ((k >> 5) * H + n) * 32 + (k & 31); }

// Weight-gradient operands (X^T, h^T, (r*h)^T, dzc^T, dzg^T, dM^T) are only
// summed into the weight gradients, where rounding errors do not compound over
// timesteps: they are stored as ONE 16-bit limb in every mode (f16 unless the
// mode is bf16), i.e. the split mode runs k_wgrad with single f16 operands.
template <int PREC>
DEV void st_col4w(u16* dst, float a, float b, float c, float d) {
  // (a nontemporal store here measured 10 % slower end to end: these 8-byte
  // stores are 2N bytes apart across lanes and rely on L2 write combining)
  *(uint2*)dst = make_uint2(pk<Prec<PREC>::f16>(a, b), pk<Prec<PREC>::f16>(c, d));
}
template <int PREC> struct WgradPrec { static constexpr int value = Prec<PREC>::split ? PREC_F16 : PREC; };

// ---- write one accumulator element (value v at row, column e) into image(s)
template <int PREC, int NCH>
DEV void img_put(char* hi, char* lo, int row, int e, float v) {
  *(u16*)(hi + Swz<NCH>::eoff(row, e)) = to_limb<Prec<PREC>::f16>(v);
  if constexpr (Prec<PREC>::split) *(u16*)(lo + Swz<NCH>::eoff(row, e)) = lo_limb16(v);
}
