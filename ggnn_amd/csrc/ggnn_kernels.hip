// ggnn_kernels.hip -- MI355X (gfx950, CDNA4) kernels + C ABI of the GGNN
// propagation engine.  See include/ggnn.h for the boundary and DESIGN.md for
// the data layout / roofline of every kernel.
//
// Reference semantics (crismolav/ggnn):
//   message + aggregation  chem_tensorflow_dense.py:391-437 (compute_timestep_fast)
//     X[g,i,:] = sum_c sum_j A[g,c,i,j] * (h[g,j,:] @ W[c] + beta[c])
//   TF1 GRUCell            chem_tensorflow_dense.py:237-241,333
//     s = sigmoid([X,h] @ Wg + bg); r,u = split(s); c = tanh([X, r*h] @ Wc + bc)
//     h' = u*h + (1-u)*c
//   T-step loop            chem_tensorflow_dense.py:312-340
//   backward = TF autodiff chem_tensorflow.py:496 (explicit here)
//
// Every hot kernel runs on v_mfma_f32_32x32x16_bf16 (bf16 operands, fp32
// accumulation).  MFMA fragment maps (gfx950):
//   A[32x16]: lane l holds A[l&31][8*(l>>5) + j], j = 0..7
//   B[16x32]: lane l holds B[8*(l>>5) + j][l&31]
//   C/D     : lane l, reg r holds D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]
// An accumulator tile is reused as the next product's B operand when the next
// product contracts over its ROW index (k-step s takes regs 8s..8s+7; element
// j of lane-half hh is row 16s + 8(j>>2) + 4hh + (j&3)).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <string>
#include <algorithm>
#include <vector>

#include "../../include/ggnn.h"

typedef uint16_t u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define DEV __device__ __forceinline__

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
DEV f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
DEV bf16x8 as_frag(uint4 v) { return __builtin_bit_cast(bf16x8, v); }
DEV u16 f2bf(float x) { return __builtin_bit_cast(u16, (__bf16)x); }
DEV float bf2f(u16 x) { return __uint_as_float(((uint32_t)x) << 16); }
DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
DEV f32x16 splat(float x) {
  f32x16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = x;
  return r;
}
DEV float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }
DEV float tanh_f(float x) { return 1.0f - 2.0f / (__expf(2.0f * x) + 1.0f); }
// row of accumulator register r for lane-half hh (within a 32x32 tile)
DEV int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }
// row of register r without the lane-half term (compile-time for unrolled r)
DEV constexpr int acc_row0(int r) { return (r & 3) + 8 * (r >> 2); }
// bf16 fragment for k-step s from an accumulator tile (see header comment)
DEV bf16x8 acc_to_frag(const f32x16& a, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)a[8 * s + j];
  return f;
}

// XOR swizzle of 16-byte chunks inside a row of NCH chunks: keeps the 32
// distinct rows of one MFMA operand read on distinct LDS bank slots.
template <int NCH>
struct Swz {
  static constexpr int M = (NCH % 16 == 0) ? 15 : (NCH % 8 == 0) ? 7 : (NCH % 4 == 0) ? 3 : 0;
  static DEV int off(int row, int ch) { return row * NCH * 16 + ((ch ^ (row & M)) << 4); }
  // byte offset of element e (bf16) in the row
  static DEV int eoff(int row, int e) { return off(row, e >> 3) + ((e & 7) << 1); }
};

DEV uint4 ld16(const void* p) { return *(const uint4*)p; }

// Raw buffer access (SRD built from wave-uniform values): one 32-bit voffset
// VGPR per lane, the per-element constant goes to the SGPR soffset.  Used for
// the accumulator-layout element-wise phases, where flat addressing would
// need one 64-bit address per element.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
DEV rsrc_t mkrsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}
DEV float bld(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
DEV void bst(rsrc_t r, float v, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, soff, 0);
}
DEV void st16(void* p, uint4 v) { *(uint4*)p = v; }
// B-operand fragment of a packed matrix: [strip][kstep][64 lanes][8]
DEV bf16x8 frag_ld(const u16* base, int strip, int ks, int nks, int lane) {
  return as_frag(ld16(base + ((size_t)(strip * nks + ks) * 64 + lane) * 8));
}

// ---------------------------------------------------------------------------
// error handling
// ---------------------------------------------------------------------------
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) { g_err = msg; return code; }
#define HIPCHK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) return fail(GGNN_ELAUNCH, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define LAUNCHCHK()                                                               \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) return fail(GGNN_ELAUNCH, std::string("launch: ") + hipGetErrorString(e_)); \
  } while (0)

// ===========================================================================
// Prep kernels
// ===========================================================================
// Pack B operand Bmat[K][N] (Bmat = S or S^T, S row-major fp32 with leading
// dim ldS) into MFMA fragment order [N/32][K/16][64][8] bf16.  blockIdx.y
// selects a matrix in a batch (strides sS / sO).
__global__ void k_pack_B(const float* __restrict__ S, int ldS, long sS, int K, int N, int trans,
                         u16* __restrict__ out, long sO) {
  const int total = (N / 32) * (K / 16) * 64;
  const float* Sb = S + sS * blockIdx.y;
  u16* ob = out + sO * blockIdx.y;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < total; q += gridDim.x * blockDim.x) {
    const int lane = q & 63, t = q >> 6;
    const int nks = K / 16;
    const int ks = t % nks, strip = t / nks;
    const int n = strip * 32 + (lane & 31), k0 = ks * 16 + 8 * (lane >> 5);
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int ka = k0 + 2 * j, kb = ka + 1;
      float a = trans ? Sb[(long)n * ldS + ka] : Sb[(long)ka * ldS + n];
      float b = trans ? Sb[(long)n * ldS + kb] : Sb[(long)kb * ldS + n];
      w[j] = pack2(a, b);
    }
    *(uint4*)(ob + (size_t)q * 8) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

__global__ void k_copy_f32(const float* __restrict__ s, float* __restrict__ d, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    d[i] = s ? s[i] : 0.0f;
}

// Adjacency [b][C][vin][vin] fp32 -> per (g,c) tile:
//   Ab  [V][V] bf16, columns permuted inside every 16-column group
//       (8-byte chunks 1 and 2 swapped) to match the accumulator-as-B-operand
//       k order of k_prop_fwd;
//   AbT [V][V] bf16 = A^T, natural order;  deg [V] fp32 = row sums.
template <int V>
__global__ void __launch_bounds__(256) k_prep_adj(const float* __restrict__ A, int vin,
                                                  u16* __restrict__ Ab, u16* __restrict__ AbT,
                                                  float* __restrict__ deg) {
  __shared__ u16 t[V][V + 2];
  const long tile = blockIdx.x;  // g*C + c
  const float* src = A + tile * (long)vin * vin;
  for (int q = threadIdx.x; q < V * V; q += 256) {
    int i = q / V, j = q % V;
    float x = (i < vin && j < vin) ? src[i * vin + j] : 0.0f;
    t[i][j] = f2bf(x);
  }
  __syncthreads();
  u16* ab = Ab + tile * V * V;
  u16* at = AbT + tile * V * V;
  for (int q = threadIdx.x; q < V * V; q += 256) {
    int i = q / V, p = q % V;
    // destination position p in the permuted row holds source column j
    int grp = p & ~15, w = p & 15;
    int j = grp + ((w < 4) ? w : (w < 8) ? w + 4 : (w < 12) ? w - 4 : w);
    ab[q] = t[i][j];
    at[q] = t[p][i];  // AbT[i][p] = A[p][i]
  }
  if (threadIdx.x < V) {
    float s = 0.f;
    for (int j = 0; j < V; ++j) s += bf2f(t[threadIdx.x][j]);
    deg[tile * V + threadIdx.x] = s;
  }
}

// h0 [b][vin][H] fp32 -> hf [N][H] fp32 (pad rows zero) and hb [N][H] bf16
__global__ void k_pad_state(const float* __restrict__ h0, int vin, int V, int H,
                            float* __restrict__ hf, u16* __restrict__ hb, long N) {
  long total = N * H;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    long row = q / H; int col = q % H;
    long g = row / V; int i = row % V;
    float x = (i < vin) ? h0[(g * vin + i) * H + col] : 0.0f;
    if (hf) hf[q] = x;
    if (hb) hb[q] = f2bf(x);
  }
}

// hf [N][H] fp32 -> out [b][vin][H]
__global__ void k_unpad_state(const float* __restrict__ hf, int vin, int V, int H,
                              float* __restrict__ out, long b) {
  long total = b * vin * (long)H;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    long r = q / H; int col = q % H;
    long g = r / vin; int i = r % vin;
    out[q] = hf[(g * V + i) * H + col];
  }
}

// [N][H] bf16 -> [H][N] bf16 (64x64 tiles through LDS; N may be a multiple of 32)
__global__ void __launch_bounds__(256) k_transpose_bf16(const u16* __restrict__ in, u16* __restrict__ out,
                                                        long N, int H) {
  __shared__ u16 t[64][66];
  long r0 = (long)blockIdx.x * 64; int c0 = blockIdx.y * 64;
  for (int q = threadIdx.x; q < 64 * 64; q += 256) {
    int i = q / 64, j = q % 64;
    t[i][j] = (r0 + i < N) ? in[(r0 + i) * H + c0 + j] : (u16)0;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < 64 * 64; q += 256) {
    int j = q / 64, i = q % 64;
    if (r0 + i < N) out[(long)(c0 + j) * N + r0 + i] = t[i][j];
  }
}

// ===========================================================================
// k_prop_fwd: fused message transform + adjacency aggregation, one graph per
// workgroup, wave w owns output columns [32w, 32w+32).
//   per channel c:  M_c = h W_c + beta_c          (MT, K = H)
//                   X  += A_c M_c                 (AGG, K = V; M_c stays in
//                                                  registers as the B operand)
// LDS: h[g] (V x H bf16) + double-buffered A_c (V x V bf16).
// ===========================================================================
template <int V, int H>
__global__ void __launch_bounds__(2 * H)
k_prop_fwd(const u16* __restrict__ hb, const u16* __restrict__ Ab, const u16* __restrict__ Wp,
           const float* __restrict__ beta, u16* __restrict__ Xb, u16* __restrict__ XT, int C, long N) {
  constexpr int NS = H / 32, NT = 64 * NS, VT = V / 32, KS = H / 16;
  constexpr int HCH = H / 8, ACH = V / 8;
  typedef Swz<HCH> SH;
  typedef Swz<ACH> SA;
  constexpr int HS_BYTES = V * H * 2, A_BYTES = V * V * 2;
  constexpr int R2 = (2 * A_BYTES > V * H * 2) ? 2 * A_BYTES : V * H * 2;
  constexpr int APT = (V * ACH + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) char smem[HS_BYTES + R2];
  char* hs = smem;
  char* as0 = smem + HS_BYTES;

  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, ns = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int n = ns * 32 + l32;

  const u16* hg = hb + (long)g * V * H;
  for (int q = tid; q < V * HCH; q += NT) {
    int row = q / HCH, ch = q % HCH;
    st16(hs + SH::off(row, ch), ld16(hg + row * H + ch * 8));
  }
  const u16* ag = Ab + (long)g * C * V * V;
  uint4 areg[APT];
#pragma unroll
  for (int p = 0; p < APT; ++p) {
    int q = tid + p * NT;
    if (q < V * ACH) areg[p] = ld16(ag + q * 8);
  }
#pragma unroll
  for (int p = 0; p < APT; ++p) {
    int q = tid + p * NT;
    if (q < V * ACH) st16(as0 + SA::off(q / ACH, q % ACH), areg[p]);
  }
  __syncthreads();

  f32x16 accx[VT];
#pragma unroll
  for (int it = 0; it < VT; ++it) accx[it] = splat(0.f);

  for (int c = 0; c < C; ++c) {
    char* asc = as0 + (c & 1) * A_BYTES;
    const bool pre = (c + 1 < C);
    if (pre) {
      const u16* an = ag + (long)(c + 1) * V * V;
#pragma unroll
      for (int p = 0; p < APT; ++p) {
        int q = tid + p * NT;
        if (q < V * ACH) areg[p] = ld16(an + q * 8);
      }
    }
    // ---- MT: M_c[j][n] = sum_k h[j][k] W_c[k][n] + beta_c[n]
    const float bb = beta ? beta[c * H + n] : 0.0f;
    f32x16 accm[VT];
#pragma unroll
    for (int rt = 0; rt < VT; ++rt) accm[rt] = splat(bb);
    const u16* wp = Wp + (size_t)c * H * H;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 bw = frag_ld(wp, ns, ks, KS, lane);
#pragma unroll
      for (int rt = 0; rt < VT; ++rt) {
        bf16x8 a = as_frag(ld16(hs + SH::off(rt * 32 + l32, 2 * ks + hh)));
        accm[rt] = mfma(a, bw, accm[rt]);
      }
    }
    // ---- AGG: X[i][n] += sum_j A_c[i][j] M_c[j][n]
    bf16x8 bm[VT][2];
#pragma unroll
    for (int rt = 0; rt < VT; ++rt) {
      bm[rt][0] = acc_to_frag(accm[rt], 0);
      bm[rt][1] = acc_to_frag(accm[rt], 1);
    }
#pragma unroll
    for (int it = 0; it < VT; ++it) {
#pragma unroll
      for (int rt = 0; rt < VT; ++rt) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 a = as_frag(ld16(asc + SA::off(it * 32 + l32, 4 * rt + 2 * s + hh)));
          accx[it] = mfma(a, bm[rt][s], accx[it]);
        }
      }
    }
    if (pre) {
      char* asn = as0 + ((c + 1) & 1) * A_BYTES;
#pragma unroll
      for (int p = 0; p < APT; ++p) {
        int q = tid + p * NT;
        if (q < V * ACH) st16(asn + SA::off(q / ACH, q % ACH), areg[p]);
      }
    }
    __syncthreads();
  }

  // ---- epilogue: X^T (transposed, for the weight-gradient GEMMs)
  const long rowg = (long)g * V;
  if (XT) {
#pragma unroll
    for (int it = 0; it < VT; ++it)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint2 w = make_uint2(pack2(accx[it][4 * q], accx[it][4 * q + 1]),
                             pack2(accx[it][4 * q + 2], accx[it][4 * q + 3]));
        *(uint2*)(XT + (long)n * N + rowg + it * 32 + 8 * q + 4 * hh) = w;
      }
  }
  // ---- X row-major via LDS (A buffers are free after the last barrier)
  char* xs = as0;
#pragma unroll
  for (int it = 0; it < VT; ++it)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int row = it * 32 + acc_row(r, hh);
      *(u16*)(xs + SH::eoff(row, n)) = f2bf(accx[it][r]);
    }
  __syncthreads();
  u16* xg = Xb + rowg * H;
  for (int q = tid; q < V * HCH; q += NT) {
    int row = q / HCH, ch = q % HCH;
    st16(xg + row * H + ch * 8, ld16(xs + SH::off(row, ch)));
  }
}

// ===========================================================================
// k_gru_fwd: fused TF1 GRUCell over 32*RT rows; wave w owns hidden columns
// [32w, 32w+32) of r, u and the candidate.
//   pass 1: [X | h] @ Wg -> r,u   and X @ Wc[0:H] -> cand (partial)
//   r*h -> LDS (over X),  pass 2: cand += (r*h) @ Wc[H:2H]
//   h' = u*h + (1-u)*tanh(cand + bc)
// ===========================================================================
template <int H, int RT>
__global__ void __launch_bounds__(2 * H)
k_gru_fwd(const u16* __restrict__ Xb, const u16* __restrict__ hb, const float* __restrict__ hf,
          const u16* __restrict__ Wgp, const float* __restrict__ bg, const u16* __restrict__ Wcp,
          const float* __restrict__ bc, float* __restrict__ hf_out, u16* __restrict__ hb_out,
          u16* __restrict__ hT_out, float* __restrict__ r_out, float* __restrict__ u_out,
          float* __restrict__ c_out, u16* __restrict__ rhT_out, long N) {
  constexpr int NS = H / 32, NT = 64 * NS, KS = H / 16, R = 32 * RT, HCH = H / 8;
  constexpr int KSG = 2 * KS;  // k-steps of the [2H x *] gate / candidate kernels
  typedef Swz<HCH> SH;
  __shared__ __attribute__((aligned(16))) char smem[2 * R * H * 2];
  char* xs = smem;
  char* hs = smem + R * H * 2;

  const int tid = threadIdx.x, lane = tid & 63, ns = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int n = ns * 32 + l32;
  const long row0 = (long)blockIdx.x * R;

  for (int q = tid; q < R * HCH; q += NT) {
    int row = q / HCH, ch = q % HCH;
    st16(xs + SH::off(row, ch), ld16(Xb + (row0 + row) * H + ch * 8));
    st16(hs + SH::off(row, ch), ld16(hb + (row0 + row) * H + ch * 8));
  }
  __syncthreads();

  f32x16 ar[RT], au[RT], ac[RT];
  {
    const float br = bg[n], bu = bg[H + n], bcc = bc[n];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) { ar[rt] = splat(br); au[rt] = splat(bu); ac[rt] = splat(bcc); }
  }
#pragma unroll 2
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 wr = frag_ld(Wgp, ns, ks, KSG, lane);
    bf16x8 wu = frag_ld(Wgp, NS + ns, ks, KSG, lane);
    bf16x8 wc = frag_ld(Wcp, ns, ks, KSG, lane);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      bf16x8 a = as_frag(ld16(xs + SH::off(rt * 32 + l32, 2 * ks + hh)));
      ar[rt] = mfma(a, wr, ar[rt]);
      au[rt] = mfma(a, wu, au[rt]);
      ac[rt] = mfma(a, wc, ac[rt]);
    }
  }
#pragma unroll 2
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 wr = frag_ld(Wgp, ns, KS + ks, KSG, lane);
    bf16x8 wu = frag_ld(Wgp, NS + ns, KS + ks, KSG, lane);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      bf16x8 a = as_frag(ld16(hs + SH::off(rt * 32 + l32, 2 * ks + hh)));
      ar[rt] = mfma(a, wr, ar[rt]);
      au[rt] = mfma(a, wu, au[rt]);
    }
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      ar[rt][r] = sigm(ar[rt][r]);
      au[rt][r] = sigm(au[rt][r]);
    }
  __syncthreads();  // all waves done reading xs (X)
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float rh[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      rh[r] = ar[rt][r] * hf[(row0 + 4 * hh) * H + n + (rt * 32 + acc_row0(r)) * H];
      *(u16*)(xs + SH::eoff(rt * 32 + acc_row(r, hh), n)) = f2bf(rh[r]);
    }
    if (rhT_out) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint2 w = make_uint2(pack2(rh[4 * q], rh[4 * q + 1]), pack2(rh[4 * q + 2], rh[4 * q + 3]));
        *(uint2*)(rhT_out + (long)n * N + row0 + rt * 32 + 8 * q + 4 * hh) = w;
      }
    }
  }
  __syncthreads();
#pragma unroll 2
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 wc = frag_ld(Wcp, ns, KS + ks, KSG, lane);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      bf16x8 a = as_frag(ld16(xs + SH::off(rt * 32 + l32, 2 * ks + hh)));
      ac[rt] = mfma(a, wc, ac[rt]);
    }
  }
  // blend + outputs
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long idx = (row0 + 4 * hh) * H + n + (rt * 32 + acc_row0(r)) * H;
      const float cc = tanh_f(ac[rt][r]);
      const float u = au[rt][r];
      const float hn = u * hf[idx] + (1.0f - u) * cc;
      hf_out[idx] = hn;
      if (r_out) { r_out[idx] = ar[rt][r]; u_out[idx] = u; c_out[idx] = cc; }
      ac[rt][r] = hn;
      *(u16*)(hs + SH::eoff(rt * 32 + acc_row(r, hh), n)) = f2bf(hn);
    }
    if (hT_out) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint2 w = make_uint2(pack2(ac[rt][4 * q], ac[rt][4 * q + 1]), pack2(ac[rt][4 * q + 2], ac[rt][4 * q + 3]));
        *(uint2*)(hT_out + (long)n * N + row0 + rt * 32 + 8 * q + 4 * hh) = w;
      }
    }
  }
  __syncthreads();
  for (int q = tid; q < R * HCH; q += NT) {
    int row = q / HCH, ch = q % HCH;
    st16(hb_out + (row0 + row) * H + ch * 8, ld16(hs + SH::off(row, ch)));
  }
}

// ===========================================================================
// k_gru_bwd: backward of the GRUCell over 32*RT rows.
//   in : delta = dL/dh' , saved h, r, u, c (fp32)
//   out: dX^T (bf16, for k_prop_bwd), dh_gru (fp32), dzc^T, dzg^T (bf16, for
//        the weight-gradient GEMMs), dbc / dbg (fp32 atomics)
// ===========================================================================
template <int H, int RT>
__global__ void __launch_bounds__(2 * H)
k_gru_bwd(const float* __restrict__ delta, const float* __restrict__ hf, const float* __restrict__ rin,
          const float* __restrict__ uin, const float* __restrict__ cin, const u16* __restrict__ WcTp,
          const u16* __restrict__ WgTp, u16* __restrict__ dXT, float* __restrict__ dh_out,
          u16* __restrict__ dzcT, u16* __restrict__ dzgT, float* __restrict__ dbc,
          float* __restrict__ dbg, long N) {
  constexpr int NS = H / 32, KS = H / 16, R = 32 * RT, ZCH = 2 * H / 8;
  typedef Swz<ZCH> SZ;
  __shared__ __attribute__((aligned(16))) char zs[R * 2 * H * 2];

  const int tid = threadIdx.x, lane = tid & 63, ns = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int n = ns * 32 + l32;
  const long row0 = (long)blockIdx.x * R;

  // phase 1: dzc = delta (1-u) (1-c^2)  -> LDS, dzc^T, dbc
  // buffer views of this tile; element (rt, r) sits at lane offset vo plus
  // the constant (rt*32 + acc_row0(r)) * H * 4
  const uint32_t tbytes = R * H * 4;
  const long tb0 = row0 * H;
  const rsrc_t pd = mkrsrc(delta + tb0, tbytes), ph = mkrsrc(hf + tb0, tbytes), pr = mkrsrc(rin + tb0, tbytes),
               pu = mkrsrc(uin + tb0, tbytes), pc = mkrsrc(cin + tb0, tbytes);
  const int vo = (4 * hh * H + n) * 4;
  const long tb = (long)n * N + row0 + 4 * hh;
  float csum = 0.f;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float dz[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ro = rt * 32 + acc_row0(4 * q + i);
        const float d = bld(pd, vo, ro * H * 4), u = bld(pu, vo, ro * H * 4), c = bld(pc, vo, ro * H * 4);
        dz[i] = d * (1.0f - u) * (1.0f - c * c);
        csum += dz[i];
        *(u16*)(zs + SZ::eoff(ro + 4 * hh, n)) = f2bf(dz[i]);
      }
      *(uint2*)(dzcT + tb + rt * 32 + 8 * q) = make_uint2(pack2(dz[0], dz[1]), pack2(dz[2], dz[3]));
      __builtin_amdgcn_sched_barrier(0);  // bound the loads in flight (VGPR budget)
    }
  }
  csum += __shfl_xor(csum, 32);
  if (hh == 0) atomicAdd(dbc + n, csum);
  __syncthreads();

  // product 1: [dX1 | d(rh)] = dzc @ Wc^T   (K = H, N = 2H)
  f32x16 a1[RT], a2[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) { a1[rt] = splat(0.f); a2[rt] = splat(0.f); }
#pragma unroll 2
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 b1 = frag_ld(WcTp, ns, ks, KS, lane);
    bf16x8 b2 = frag_ld(WcTp, NS + ns, ks, KS, lane);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      bf16x8 a = as_frag(ld16(zs + SZ::off(rt * 32 + l32, 2 * ks + hh)));
      a1[rt] = mfma(a, b1, a1[rt]);
      a2[rt] = mfma(a, b2, a2[rt]);
    }
  }
  __syncthreads();  // done reading dzc

  // phase 2: dh = delta u + d(rh) r ; dzg = [d(rh) h r(1-r) | delta (h-c) u(1-u)]
  float rsum = 0.f, usum = 0.f;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float zr[4], zu[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * q + i;
        const int ro = rt * 32 + acc_row0(r);
        const int so = ro * H * 4;
        const float d = bld(pd, vo, so), h = bld(ph, vo, so), rr = bld(pr, vo, so), u = bld(pu, vo, so),
                    c = bld(pc, vo, so);
        const float drh = a2[rt][r];
        a2[rt][r] = d * u + drh * rr;  // a2 now holds dh (GRU part, before dh2)
        zr[i] = drh * h * rr * (1.0f - rr);
        zu[i] = d * (h - c) * u * (1.0f - u);
        rsum += zr[i];
        usum += zu[i];
        *(u16*)(zs + SZ::eoff(ro + 4 * hh, n)) = f2bf(zr[i]);
        *(u16*)(zs + SZ::eoff(ro + 4 * hh, H + n)) = f2bf(zu[i]);
      }
      *(uint2*)(dzgT + tb + rt * 32 + 8 * q) = make_uint2(pack2(zr[0], zr[1]), pack2(zr[2], zr[3]));
      *(uint2*)(dzgT + tb + (long)H * N + rt * 32 + 8 * q) = make_uint2(pack2(zu[0], zu[1]), pack2(zu[2], zu[3]));
      __builtin_amdgcn_sched_barrier(0);  // bound the loads in flight (VGPR budget)
    }
  }
  rsum += __shfl_xor(rsum, 32);
  usum += __shfl_xor(usum, 32);
  if (hh == 0) { atomicAdd(dbg + n, rsum); atomicAdd(dbg + H + n, usum); }
  __syncthreads();

  // product 2: [dX2 | dh2] = dzg @ Wg^T   (K = 2H, N = 2H)
#pragma unroll 1
  for (int ks = 0; ks < 2 * KS; ++ks) {
    bf16x8 b1 = frag_ld(WgTp, ns, ks, 2 * KS, lane);
    bf16x8 b2 = frag_ld(WgTp, NS + ns, ks, 2 * KS, lane);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      bf16x8 a = as_frag(ld16(zs + SZ::off(rt * 32 + l32, 2 * ks + hh)));
      a1[rt] = mfma(a, b1, a1[rt]);
      a2[rt] = mfma(a, b2, a2[rt]);
    }
  }
  const rsrc_t pdo = mkrsrc(dh_out + tb0, tbytes);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint2 w = make_uint2(pack2(a1[rt][4 * q], a1[rt][4 * q + 1]), pack2(a1[rt][4 * q + 2], a1[rt][4 * q + 3]));
      *(uint2*)(dXT + tb + rt * 32 + 8 * q) = w;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) bst(pdo, a2[rt][r], vo, (rt * 32 + acc_row0(r)) * H * 4);
  }
}

// ===========================================================================
// k_prop_bwd: backward of message+aggregation, one graph per workgroup.
//   per channel c:
//     dM_c^T[n][j] = sum_i dX^T[n][i] A_c[i][j]     (K = V; A operand dX^T
//                                                   kept in registers)
//     dM_c -> LDS [j][n] bf16, dM_c^T -> HBM (weight-gradient operand)
//     dh[j][k]   += sum_n dM_c[j][n] W_c[k][n]      (K = H)
//     dbeta_c[n] += sum_i deg_c[i] dX[i][n]          (= sum_j dM_c[j][n])
// ===========================================================================
template <int V, int H>
__global__ void __launch_bounds__(2 * H)
k_prop_bwd(const u16* __restrict__ dXT, const u16* __restrict__ AbT, const float* __restrict__ deg,
           const u16* __restrict__ WTp, const float* __restrict__ dh_in, float* __restrict__ dh_out,
           u16* __restrict__ dMT, float* __restrict__ dbeta, int C, long N) {
  constexpr int NS = H / 32, NT = 64 * NS, VT = V / 32, KV = V / 16, KS = H / 16;
  constexpr int HCH = H / 8, ACH = V / 8;
  typedef Swz<HCH> SH;
  typedef Swz<ACH> SA;
  constexpr int A_BYTES = V * V * 2, M_BYTES = V * H * 2;
  constexpr int APT = (V * ACH + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) char smem[A_BYTES + M_BYTES];
  char* as = smem;
  char* ms = smem + A_BYTES;

  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, ns = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int n = ns * 32 + l32;
  const long rowg = (long)g * V;

  // dX^T fragments for this wave's 32 columns (A operand of the dM^T product)
  bf16x8 dxf[KV];
#pragma unroll
  for (int s = 0; s < KV; ++s) dxf[s] = as_frag(ld16(dXT + (long)n * N + rowg + 16 * s + 8 * hh));

  const u16* ag = AbT + (long)g * C * V * V;
  uint4 areg[APT];
#pragma unroll
  for (int p = 0; p < APT; ++p) {
    int q = tid + p * NT;
    if (q < V * ACH) st16(as + SA::off(q / ACH, q % ACH), ld16(ag + q * 8));
  }
  f32x16 adh[VT];
#pragma unroll
  for (int jt = 0; jt < VT; ++jt)
#pragma unroll
    for (int r = 0; r < 16; ++r) adh[jt][r] = dh_in[(rowg + 4 * hh) * H + n + (jt * 32 + acc_row0(r)) * H];
  __syncthreads();

  for (int c = 0; c < C; ++c) {
    const bool pre = (c + 1 < C);
    if (pre) {
      const u16* an = ag + (long)(c + 1) * V * V;
#pragma unroll
      for (int p = 0; p < APT; ++p) {
        int q = tid + p * NT;
        if (q < V * ACH) areg[p] = ld16(an + q * 8);
      }
    }
    if (dbeta) {
      const float* dg = deg + ((long)g * C + c) * V;
      float s = 0.f;
#pragma unroll
      for (int ss = 0; ss < KV; ++ss) {
        const float4 d0 = *(const float4*)(dg + 16 * ss + 8 * hh);
        const float4 d1 = *(const float4*)(dg + 16 * ss + 8 * hh + 4);
        s += d0.x * (float)dxf[ss][0] + d0.y * (float)dxf[ss][1] + d0.z * (float)dxf[ss][2] + d0.w * (float)dxf[ss][3];
        s += d1.x * (float)dxf[ss][4] + d1.y * (float)dxf[ss][5] + d1.z * (float)dxf[ss][6] + d1.w * (float)dxf[ss][7];
        asm volatile("" ::: "memory");
      }
      s += __shfl_xor(s, 32);
      if (hh == 0) atomicAdd(dbeta + c * H + n, s);
    }
    // phase a: dM_c^T tile rows n (this wave), cols j -- one 32-column tile
    // at a time, written to LDS ([j][n], 8-byte writes) and to dM^T in HBM
#pragma unroll
    for (int jt = 0; jt < VT; ++jt) {
      f32x16 am = splat(0.f);
#pragma unroll
      for (int s = 0; s < KV; ++s) {
        bf16x8 bA = as_frag(ld16(as + SA::off(jt * 32 + l32, 2 * s + hh)));
        am = mfma(dxf[s], bA, am);
      }
      const int j = jt * 32 + l32;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = ns * 32 + 8 * q + 4 * hh;
        uint2 w = make_uint2(pack2(am[4 * q], am[4 * q + 1]), pack2(am[4 * q + 2], am[4 * q + 3]));
        *(uint2*)(ms + SH::eoff(j, n0)) = w;
      }
      if (dMT) {
        u16* dst = dMT + (long)c * H * N + rowg + j + (long)(ns * 32 + 4 * hh) * N;
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(long)acc_row0(r) * N] = f2bf(am[r]);
      }
    }
    __syncthreads();  // ms complete, as reads done
    if (pre) {
#pragma unroll
      for (int p = 0; p < APT; ++p) {
        int q = tid + p * NT;
        if (q < V * ACH) st16(as + SA::off(q / ACH, q % ACH), areg[p]);
      }
    }
    // phase b: dh[j][k] += sum_n dM_c[j][n] W_c^T[n][k]
    const u16* wt = WTp + (size_t)c * H * H;
#pragma unroll 2
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 bw = frag_ld(wt, ns, ks, KS, lane);
#pragma unroll
      for (int jt = 0; jt < VT; ++jt) {
        bf16x8 a = as_frag(ld16(ms + SH::off(jt * 32 + l32, 2 * ks + hh)));
        adh[jt] = mfma(a, bw, adh[jt]);
      }
    }
    __syncthreads();  // ms reads done, next A staged
  }
#pragma unroll
  for (int jt = 0; jt < VT; ++jt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dh_out[(rowg + 4 * hh) * H + n + (jt * 32 + acc_row0(r)) * H] = adh[jt][r];
}

// ===========================================================================
// k_wgrad: grouped split-K "NT" GEMM for the weight gradients,
//   out[m][n] += sum_{t, k} P_t[m][k] * Q_t[n][k]
// P, Q bf16 with K (= graph-node rows) contiguous; K split into chunks of KC
// rows, every chunk summed over all T steps inside the workgroup, then one
// fp32 atomicAdd per output element per workgroup.  128x128 tile, 4 waves.
// ===========================================================================
struct WgProb {
  const u16* P; const u16* Q; float* out;
  long ldP, ldQ, stepP, stepQ;
  int ldO, M, N, tiles_n, tile_begin;
};
#define WG_MAXP 24
struct WgArgs {
  WgProb p[WG_MAXP];
  int nprob, nchunks, KC, T;
};

template <int BK>
__global__ void __launch_bounds__(256) k_wgrad(WgArgs args) {
  constexpr int CH = BK / 8;                 // 16-B chunks per tile row
  constexpr int TB = 128 * BK * 2;           // bytes per operand tile
  constexpr int PT = 128 * CH / 256;         // chunks per thread per operand
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];
  const int tile = blockIdx.x / args.nchunks, chunk = blockIdx.x % args.nchunks;
  int pi = 0;
  while (pi + 1 < args.nprob && args.p[pi + 1].tile_begin <= tile) ++pi;
  const WgProb pr = args.p[pi];
  const int lt = tile - pr.tile_begin;
  const int m0 = (lt / pr.tiles_n) * 128, n0 = (lt % pr.tiles_n) * 128;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int wm = wv >> 1, wn = wv & 1;
  // swizzle: rows of BK*2 bytes, RPB rows per 256-B bank row
  constexpr int RPB = 256 / (BK * 2);
  auto soff = [&](int row, int ch) { return row * BK * 2 + ((ch ^ ((row / RPB) & (CH - 1))) << 4); };

  const int kits = args.KC / BK, nit = kits * args.T;
  const long kbase = (long)chunk * args.KC;
  uint4 rp[PT], rq[PT];
  auto gload = [&](int it) {
    const int t = it / kits;
    const long k0 = kbase + (long)(it % kits) * BK;
    const u16* P = pr.P + (long)t * pr.stepP;
    const u16* Q = pr.Q + (long)t * pr.stepQ;
#pragma unroll
    for (int p = 0; p < PT; ++p) {
      int q = tid + p * 256, row = q / CH, ch = q % CH;
      rp[p] = ld16(P + (long)(m0 + row) * pr.ldP + k0 + ch * 8);
      rq[p] = ld16(Q + (long)(n0 + row) * pr.ldQ + k0 + ch * 8);
    }
  };
  auto sstore = [&](int buf) {
    char* ps = smem + buf * 2 * TB;
    char* qs = ps + TB;
#pragma unroll
    for (int p = 0; p < PT; ++p) {
      int q = tid + p * 256, row = q / CH, ch = q % CH;
      st16(ps + soff(row, ch), rp[p]);
      st16(qs + soff(row, ch), rq[p]);
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
    const char* ps = smem + (it & 1) * 2 * TB;
    const char* qs = ps + TB;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = as_frag(ld16(ps + soff(wm * 64 + i * 32 + l32, 2 * s + hh)));
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = as_frag(ld16(qs + soff(wn * 64 + j * 32 + l32, 2 * s + hh)));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    }
    if (pre) sstore((it + 1) & 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + acc_row(r, hh);
        const int nn = n0 + wn * 64 + j * 32 + l32;
        atomicAdd(pr.out + (long)m * pr.ldO + nn, acc[i][j][r]);
      }
}

// ===========================================================================
// Host side: layouts, dispatch, C ABI
// ===========================================================================
namespace {

// ---- optional per-kernel-kind timing with HIP events (bench.py roofline)
const char* const kKindNames[GGNN_NUM_KERNEL_KINDS] = {
    "pack_weights", "prep_adjacency", "state_io", "prop_fwd", "gru_fwd", "gru_bwd", "prop_bwd", "wgrad"};
struct ProfState {
  bool on = false;
  int cap = 0, used = 0;
  std::vector<hipEvent_t> ev;   // 2 per record
  std::vector<int> kind;
};
ProfState g_prof;
struct Prof {
  int idx = -1;
  hipStream_t s;
  Prof(int k, hipStream_t st) : s(st) {
    if (g_prof.on && g_prof.used < g_prof.cap) {
      idx = g_prof.used++;
      g_prof.kind[idx] = k;
      hipEventRecord(g_prof.ev[2 * idx], s);
    }
  }
  ~Prof() {
    if (idx >= 0) hipEventRecord(g_prof.ev[2 * idx + 1], s);
  }
};

struct Cfg {
  int b, vin, V, H, C, T, flags;
  long N;
};

int pad_v(int v) { return v <= 32 ? 32 : v <= 64 ? 64 : v <= 128 ? 128 : -1; }

int make_cfg(const ggnn_dims* d, Cfg* c) {
  if (!d) return fail(GGNN_EINVAL, "dims is NULL");
  if (d->b < 1 || d->v < 1 || d->C < 1 || d->T < 1)
    return fail(GGNN_EINVAL, "dims: b, v, C, T must be >= 1");
  if (!(d->h == 64 || d->h == 128 || d->h == 256))
    return fail(GGNN_EUNSUP, "hidden size must be 64, 128 or 256 (got " + std::to_string(d->h) + ")");
  int V = pad_v(d->v);
  if (V < 0) return fail(GGNN_EUNSUP, "v must be <= 128 (got " + std::to_string(d->v) + ")");
  c->b = d->b; c->vin = d->v; c->V = V; c->H = d->h; c->C = d->C; c->T = d->T; c->flags = d->flags;
  c->N = (long)d->b * V;
  return GGNN_OK;
}

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// ---- weight pack layout
struct PackL {
  size_t Wf, WT, beta, Wg, WgT, Wc, WcT, bg, bc, total;
};
PackL pack_layout(const Cfg& c) {
  PackL L; size_t o = 0; const size_t H = c.H;
  L.Wf = o;  o += al(c.C * H * H * 2);
  L.WT = o;  o += al(c.C * H * H * 2);
  L.beta = o; o += al(c.C * H * 4);
  L.Wg = o;  o += al(4 * H * H * 2);
  L.WgT = o; o += al(4 * H * H * 2);
  L.Wc = o;  o += al(2 * H * H * 2);
  L.WcT = o; o += al(2 * H * H * 2);
  L.bg = o;  o += al(2 * H * 4);
  L.bc = o;  o += al(H * 4);
  L.total = o;
  return L;
}

// ---- workspace layout
struct AdjL {
  size_t Ab, AbT, deg, total;
};
AdjL adj_layout(const Cfg& c) {
  AdjL L; size_t o = 0;
  L.Ab = o;  o += al((size_t)c.b * c.C * c.V * c.V * 2);
  L.AbT = o; o += al((size_t)c.b * c.C * c.V * c.V * 2);
  L.deg = o; o += al((size_t)c.b * c.C * c.V * 4);
  L.total = o;
  return L;
}
struct WsL {
  size_t hf[2], hb[2];           // inference ping-pong
  size_t hfT, hbuf;              // training: hf[t] t=0..T (fp32), hb ping-pong
  size_t Xb;
  size_t hT, XT, rhT, r, u, c;   // training, per step
  size_t dA, dB, dXT, dzcT, dzgT, dMT;
  size_t total;
};
WsL ws_layout(const Cfg& c, bool training) {
  WsL L; memset(&L, 0, sizeof(L)); size_t o = 0;
  const size_t N = c.N, H = c.H, T = c.T, C = c.C;
  const size_t nh4 = al(N * H * 4), nh2 = al(N * H * 2);
  L.hb[0] = o; o += nh2;
  L.hb[1] = o; o += nh2;
  L.Xb = o; o += nh2;
  if (!training) {
    L.hf[0] = o; o += nh4;
    L.hf[1] = o; o += nh4;
  } else {
    L.hfT = o; o += nh4 * (T + 1);
    L.hT = o;  o += nh2 * T;
    L.XT = o;  o += nh2 * T;
    L.rhT = o; o += nh2 * T;
    L.r = o;   o += nh4 * T;
    L.u = o;   o += nh4 * T;
    L.c = o;   o += nh4 * T;
    L.dA = o;  o += nh4;
    L.dB = o;  o += nh4;
    L.dXT = o; o += nh2;
    L.dzcT = o; o += nh2 * T;
    L.dzgT = o; o += 2 * nh2 * T;
    L.dMT = o; o += C * nh2 * T;
  }
  L.total = o;
  return L;
}

template <typename T> T* P(void* base, size_t off) { return (T*)((char*)base + off); }
template <typename T> const T* P(const void* base, size_t off) { return (const T*)((const char*)base + off); }

int grid1d(long n, int bs = 256) { long g = (n + bs - 1) / bs; return (int)std::min<long>(g, 8192); }

// ---- kernel dispatch on (V, H)
template <int V, int H>
void launch_prop_fwd(const Cfg& c, const u16* hb, const u16* Ab, const u16* Wp, const float* beta,
                     u16* Xb, u16* XT, hipStream_t s) {
  Prof p(3, s);
  hipLaunchKernelGGL((k_prop_fwd<V, H>), dim3(c.b), dim3(2 * H), 0, s, hb, Ab, Wp, beta, Xb, XT, c.C, c.N);
}
template <int V, int H>
void launch_prop_bwd(const Cfg& c, const u16* dXT, const u16* AbT, const float* deg, const u16* WTp,
                     const float* dh_in, float* dh_out, u16* dMT, float* dbeta, hipStream_t s) {
  Prof p(6, s);
  hipLaunchKernelGGL((k_prop_bwd<V, H>), dim3(c.b), dim3(2 * H), 0, s, dXT, AbT, deg, WTp, dh_in, dh_out,
                     dMT, dbeta, c.C, c.N);
}

#define DISPATCH_VH(c, FN, ...)                                               \
  do {                                                                        \
    switch ((c).H) {                                                          \
      case 64:                                                                \
        if ((c).V == 32) FN<32, 64>(__VA_ARGS__);                             \
        else if ((c).V == 64) FN<64, 64>(__VA_ARGS__);                        \
        else FN<128, 64>(__VA_ARGS__);                                        \
        break;                                                                \
      case 128:                                                               \
        if ((c).V == 32) FN<32, 128>(__VA_ARGS__);                            \
        else if ((c).V == 64) FN<64, 128>(__VA_ARGS__);                       \
        else FN<128, 128>(__VA_ARGS__);                                       \
        break;                                                                \
      default:                                                                \
        if ((c).V == 32) FN<32, 256>(__VA_ARGS__);                            \
        else if ((c).V == 64) FN<64, 256>(__VA_ARGS__);                       \
        else FN<128, 256>(__VA_ARGS__);                                       \
        break;                                                                \
    }                                                                         \
  } while (0)

template <int H, int RT>
void launch_gru_fwd_t(const Cfg& c, const u16* Xb, const u16* hb, const float* hf, const PackL& PL,
                      const void* pk, float* hf_out, u16* hb_out, u16* hT_out, float* r, float* u,
                      float* cc, u16* rhT, hipStream_t s) {
  Prof p(4, s);
  hipLaunchKernelGGL((k_gru_fwd<H, RT>), dim3(c.N / (32 * RT)), dim3(2 * H), 0, s, Xb, hb, hf,
                     P<u16>(pk, PL.Wg), P<float>(pk, PL.bg), P<u16>(pk, PL.Wc), P<float>(pk, PL.bc),
                     hf_out, hb_out, hT_out, r, u, cc, rhT, c.N);
}
template <int H, int RT>
void launch_gru_bwd_t(const Cfg& c, const float* delta, const float* hf, const float* r, const float* u,
                      const float* cc, const PackL& PL, const void* pk, u16* dXT, float* dh_out, u16* dzcT,
                      u16* dzgT, float* dbc, float* dbg, hipStream_t s) {
  Prof p(5, s);
  hipLaunchKernelGGL((k_gru_bwd<H, RT>), dim3(c.N / (32 * RT)), dim3(2 * H), 0, s, delta, hf, r, u, cc,
                     P<u16>(pk, PL.WcT), P<u16>(pk, PL.WgT), dXT, dh_out, dzcT, dzgT, dbc, dbg, c.N);
}
#define DISPATCH_H_RT(c, FN, ...)                                             \
  do {                                                                        \
    const bool rt2 = ((c).N % 64) == 0;                                       \
    switch ((c).H) {                                                          \
      case 64: if (rt2) FN<64, 2>(__VA_ARGS__); else FN<64, 1>(__VA_ARGS__); break;    \
      case 128: if (rt2) FN<128, 2>(__VA_ARGS__); else FN<128, 1>(__VA_ARGS__); break; \
      default: if (rt2) FN<256, 2>(__VA_ARGS__); else FN<256, 1>(__VA_ARGS__); break;  \
    }                                                                         \
  } while (0)

void launch_pack(const float* S, int ldS, long sS, int K, int N, int trans, u16* out, long sO, int batch,
                 hipStream_t s) {
  int total = (N / 32) * (K / 16) * 64;
  Prof p(0, s);
  hipLaunchKernelGGL(k_pack_B, dim3((total + 255) / 256, batch), dim3(256), 0, s, S, ldS, sS, K, N, trans, out, sO);
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int ggnn_version(void) { return 1; }

const char* ggnn_kernel_kind_name(int kind) {
  return (kind >= 0 && kind < GGNN_NUM_KERNEL_KINDS) ? kKindNames[kind] : "";
}

int ggnn_profile_begin(int max_launches) {
  if (max_launches < 1) return fail(GGNN_EINVAL, "profile_begin: max_launches < 1");
  for (hipEvent_t e : g_prof.ev) hipEventDestroy(e);
  g_prof.ev.assign(2 * (size_t)max_launches, nullptr);
  g_prof.kind.assign(max_launches, 0);
  for (auto& e : g_prof.ev) HIPCHK(hipEventCreate(&e));
  g_prof.cap = max_launches;
  g_prof.used = 0;
  g_prof.on = true;
  return GGNN_OK;
}

int ggnn_profile_end(double* total_ms, int* launches) {
  if (!g_prof.on) return fail(GGNN_EINVAL, "profile_end without profile_begin");
  g_prof.on = false;
  for (int k = 0; k < GGNN_NUM_KERNEL_KINDS; ++k) {
    if (total_ms) total_ms[k] = 0.0;
    if (launches) launches[k] = 0;
  }
  for (int i = 0; i < g_prof.used; ++i) {
    HIPCHK(hipEventSynchronize(g_prof.ev[2 * i + 1]));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]));
    if (total_ms) total_ms[g_prof.kind[i]] += ms;
    if (launches) launches[g_prof.kind[i]] += 1;
  }
  const int overflow = g_prof.used >= g_prof.cap;
  g_prof.used = 0;
  return overflow ? fail(GGNN_EINVAL, "profile buffer full: raise max_launches") : GGNN_OK;
}
const char* ggnn_last_error(void) { return g_err.c_str(); }

int ggnn_check_dims(const ggnn_dims* d) {
  Cfg c;
  return make_cfg(d, &c);
}

int ggnn_workspace_bytes(const ggnn_dims* d, int training, size_t* bytes) {
  Cfg c; int e = make_cfg(d, &c); if (e) return e;
  if (!bytes) return fail(GGNN_EINVAL, "bytes is NULL");
  *bytes = ws_layout(c, training != 0).total;
  return GGNN_OK;
}

int ggnn_weight_pack_bytes(const ggnn_dims* d, size_t* bytes) {
  Cfg c; int e = make_cfg(d, &c); if (e) return e;
  if (!bytes) return fail(GGNN_EINVAL, "bytes is NULL");
  *bytes = pack_layout(c).total;
  return GGNN_OK;
}

int ggnn_pack_weights(const ggnn_dims* d, void* pack, const float* W, const float* beta, const float* Wg,
                      const float* bg, const float* Wc, const float* bc, ggnn_stream_t stream) {
  Cfg c; int e = make_cfg(d, &c); if (e) return e;
  if (!pack || !W || !Wg || !bg || !Wc || !bc) return fail(GGNN_EINVAL, "pack_weights: NULL pointer");
  if ((c.flags & GGNN_USE_EDGE_BIAS) && !beta) return fail(GGNN_EINVAL, "pack_weights: edge_biases NULL with USE_EDGE_BIAS");
  hipStream_t s = (hipStream_t)stream;
  const PackL L = pack_layout(c);
  const int H = c.H;
  // W_c (MT, Bmat = W_c) and W_c^T (dh product of the backward)
  launch_pack(W, H, (long)H * H, H, H, 0, P<u16>(pack, L.Wf), (long)H * H, c.C, s);
  launch_pack(W, H, (long)H * H, H, H, 1, P<u16>(pack, L.WT), (long)H * H, c.C, s);
  launch_pack(Wg, 2 * H, 0, 2 * H, 2 * H, 0, P<u16>(pack, L.Wg), 0, 1, s);
  launch_pack(Wg, 2 * H, 0, 2 * H, 2 * H, 1, P<u16>(pack, L.WgT), 0, 1, s);
  launch_pack(Wc, H, 0, 2 * H, H, 0, P<u16>(pack, L.Wc), 0, 1, s);        // Bmat = Wc [2H][H]
  launch_pack(Wc, H, 0, H, 2 * H, 1, P<u16>(pack, L.WcT), 0, 1, s);       // Bmat = Wc^T [H][2H]
  const float* bsrc = (c.flags & GGNN_USE_EDGE_BIAS) ? beta : nullptr;
  { Prof p_(0, s); hipLaunchKernelGGL(k_copy_f32, dim3(grid1d((long)c.C * H)), dim3(256), 0, s, bsrc, P<float>(pack, L.beta), (long)c.C * H); }
  { Prof p_(0, s); hipLaunchKernelGGL(k_copy_f32, dim3(grid1d(2 * H)), dim3(256), 0, s, bg, P<float>(pack, L.bg), (long)2 * H); }
  { Prof p_(0, s); hipLaunchKernelGGL(k_copy_f32, dim3(grid1d(H)), dim3(256), 0, s, bc, P<float>(pack, L.bc), (long)H); }
  LAUNCHCHK();
  return GGNN_OK;
}

int ggnn_adjacency_bytes(const ggnn_dims* d, size_t* bytes) {
  Cfg c; int e = make_cfg(d, &c); if (e) return e;
  if (!bytes) return fail(GGNN_EINVAL, "bytes is NULL");
  *bytes = adj_layout(c).total;
  return GGNN_OK;
}

int ggnn_set_adjacency(const ggnn_dims* d, void* ws, const float* A, ggnn_stream_t stream) {
  Cfg c; int e = make_cfg(d, &c); if (e) return e;
  if (!ws || !A) return fail(GGNN_EINVAL, "set_adjacency: NULL pointer");
  hipStream_t s = (hipStream_t)stream;
  const AdjL L = adj_layout(c);
  dim3 grid((unsigned)(c.b * c.C));
  Prof p(1, s);
  if (c.V == 32) hipLaunchKernelGGL(k_prep_adj<32>, grid, dim3(256), 0, s, A, c.vin, P<u16>(ws, L.Ab), P<u16>(ws, L.AbT), P<float>(ws, L.deg));
  else if (c.V == 64) hipLaunchKernelGGL(k_prep_adj<64>, grid, dim3(256), 0, s, A, c.vin, P<u16>(ws, L.Ab), P<u16>(ws, L.AbT), P<float>(ws, L.deg));
  else hipLaunchKernelGGL(k_prep_adj<128>, grid, dim3(256), 0, s, A, c.vin, P<u16>(ws, L.Ab), P<u16>(ws, L.AbT), P<float>(ws, L.deg));
  LAUNCHCHK();
  return GGNN_OK;
}

int ggnn_forward(const ggnn_dims* d, const void* pack, const void* adj, void* ws, int training, const float* h0,
                 float* hT, ggnn_stream_t stream) {
  Cfg c; int e = make_cfg(d, &c); if (e) return e;
  if (!pack || !adj || !ws || !h0 || !hT) return fail(GGNN_EINVAL, "forward: NULL pointer");
  const AdjL AL = adj_layout(c);
  hipStream_t s = (hipStream_t)stream;
  const bool tr = training != 0;
  const WsL L = ws_layout(c, tr);
  const PackL PL = pack_layout(c);
  const long N = c.N, H = c.H;
  const size_t nh4 = al(N * H * 4), nh2 = al(N * H * 2);
  const float* beta = P<float>(pack, PL.beta);

  float* hf0 = tr ? P<float>(ws, L.hfT) : P<float>(ws, L.hf[0]);
  { Prof p_(2, s); hipLaunchKernelGGL(k_pad_state, dim3(grid1d(N * H)), dim3(256), 0, s, h0, c.vin, c.V, c.H, hf0,
                     P<u16>(ws, L.hb[0]), N); }
  if (tr) {
    { Prof p_(2, s); hipLaunchKernelGGL(k_transpose_bf16, dim3((N + 63) / 64, H / 64), dim3(256), 0, s, P<u16>(ws, L.hb[0]),
                       P<u16>(ws, L.hT), N, c.H); }
  }
  for (int t = 0; t < c.T; ++t) {
    const u16* hb_in = P<u16>(ws, L.hb[t & 1]);
    u16* hb_out = P<u16>(ws, L.hb[(t + 1) & 1]);
    const float* hf_in = tr ? P<float>(ws, L.hfT + nh4 * t) : P<float>(ws, L.hf[t & 1]);
    float* hf_out = tr ? P<float>(ws, L.hfT + nh4 * (t + 1)) : P<float>(ws, L.hf[(t + 1) & 1]);
    u16* XT = tr ? P<u16>(ws, L.XT + nh2 * t) : nullptr;
    DISPATCH_VH(c, launch_prop_fwd, c, hb_in, P<u16>(adj, AL.Ab), P<u16>(pack, PL.Wf), beta, P<u16>(ws, L.Xb), XT, s);
    u16* hTo = (tr && t + 1 < c.T) ? P<u16>(ws, L.hT + nh2 * (t + 1)) : nullptr;
    float* ro = tr ? P<float>(ws, L.r + nh4 * t) : nullptr;
    float* uo = tr ? P<float>(ws, L.u + nh4 * t) : nullptr;
    float* co = tr ? P<float>(ws, L.c + nh4 * t) : nullptr;
    u16* rhT = tr ? P<u16>(ws, L.rhT + nh2 * t) : nullptr;
    DISPATCH_H_RT(c, launch_gru_fwd_t, c, P<u16>(ws, L.Xb), hb_in, hf_in, PL, pack, hf_out, hb_out, hTo, ro, uo, co, rhT, s);
  }
  const float* hfin = tr ? P<float>(ws, L.hfT + nh4 * c.T) : P<float>(ws, L.hf[c.T & 1]);
  { Prof p_(2, s); hipLaunchKernelGGL(k_unpad_state, dim3(grid1d((long)c.b * c.vin * H)), dim3(256), 0, s, hfin, c.vin, c.V, c.H, hT, (long)c.b); }
  LAUNCHCHK();
  return GGNN_OK;
}

int ggnn_backward(const ggnn_dims* d, const void* pack, const void* adj, void* ws, const float* dhT, float* dh0,
                  float* dW, float* dbeta, float* dWg, float* dbg, float* dWc, float* dbc, ggnn_stream_t stream) {
  Cfg c; int e = make_cfg(d, &c); if (e) return e;
  const AdjL AL = adj_layout(c);
  if (!pack || !adj || !ws || !dhT || !dh0 || !dW || !dWg || !dbg || !dWc || !dbc)
    return fail(GGNN_EINVAL, "backward: NULL pointer");
  const bool use_bias = (c.flags & GGNN_USE_EDGE_BIAS) != 0;
  if (use_bias && !dbeta) return fail(GGNN_EINVAL, "backward: d_edge_biases NULL with USE_EDGE_BIAS");
  hipStream_t s = (hipStream_t)stream;
  const WsL L = ws_layout(c, true);
  const PackL PL = pack_layout(c);
  const long N = c.N, H = c.H;
  const size_t nh4 = al(N * H * 4), nh2 = al(N * H * 2);

  HIPCHK(hipMemsetAsync(dW, 0, (size_t)c.C * H * H * 4, s));
  if (use_bias) HIPCHK(hipMemsetAsync(dbeta, 0, (size_t)c.C * H * 4, s));
  HIPCHK(hipMemsetAsync(dWg, 0, (size_t)4 * H * H * 4, s));
  HIPCHK(hipMemsetAsync(dbg, 0, (size_t)2 * H * 4, s));
  HIPCHK(hipMemsetAsync(dWc, 0, (size_t)2 * H * H * 4, s));
  HIPCHK(hipMemsetAsync(dbc, 0, (size_t)H * 4, s));

  float* dA = P<float>(ws, L.dA);
  float* dB = P<float>(ws, L.dB);
  { Prof p_(2, s); hipLaunchKernelGGL(k_pad_state, dim3(grid1d(N * H)), dim3(256), 0, s, dhT, c.vin, c.V, c.H, dA, (u16*)nullptr, N); }
  for (int t = c.T - 1; t >= 0; --t) {
    DISPATCH_H_RT(c, launch_gru_bwd_t, c, dA, P<float>(ws, L.hfT + nh4 * t), P<float>(ws, L.r + nh4 * t),
                  P<float>(ws, L.u + nh4 * t), P<float>(ws, L.c + nh4 * t), PL, pack, P<u16>(ws, L.dXT), dB,
                  P<u16>(ws, L.dzcT + nh2 * t), P<u16>(ws, L.dzgT + 2 * nh2 * t), dbc, dbg, s);
    DISPATCH_VH(c, launch_prop_bwd, c, P<u16>(ws, L.dXT), P<u16>(adj, AL.AbT), P<float>(adj, AL.deg),
                P<u16>(pack, PL.WT), dB, dA, P<u16>(ws, L.dMT + (size_t)c.C * nh2 * t), use_bias ? dbeta : nullptr, s);
  }
  { Prof p_(2, s); hipLaunchKernelGGL(k_unpad_state, dim3(grid1d((long)c.b * c.vin * H)), dim3(256), 0, s, dA, c.vin, c.V, c.H, dh0, (long)c.b); }

  // weight gradients: out[m][n] += sum_{t,rows} P_t[m][row] Q_t[n][row]
  WgArgs a; memset(&a, 0, sizeof(a));
  int np = 0, tiles = 0;
  auto add = [&](const u16* Pp, long stepP, const u16* Qp, long stepQ, float* out, int ldO, int M, int Nn) {
    WgProb& p = a.p[np++];
    p.P = Pp; p.Q = Qp; p.out = out; p.ldP = N; p.ldQ = N; p.stepP = stepP; p.stepQ = stepQ;
    p.ldO = ldO; p.M = M; p.N = Nn; p.tiles_n = Nn / 128 > 0 ? Nn / 128 : 1; p.tile_begin = tiles;
    tiles += (M / 128 > 0 ? M / 128 : 1) * p.tiles_n;
  };
  if (c.C + 4 > WG_MAXP) return fail(GGNN_EUNSUP, "too many channels for the grouped weight-gradient launch");
  // d gates_kernel rows [0,H) from X, rows [H,2H) from h ;  cols = dzg (2H)
  add(P<u16>(ws, L.XT), nh2 / 2, P<u16>(ws, L.dzgT), nh2, dWg, 2 * H, H, 2 * H);
  add(P<u16>(ws, L.hT), nh2 / 2, P<u16>(ws, L.dzgT), nh2, dWg + H * 2 * H, 2 * H, H, 2 * H);
  // d candidate_kernel rows [0,H) from X, rows [H,2H) from r*h ; cols = dzc (H)
  add(P<u16>(ws, L.XT), nh2 / 2, P<u16>(ws, L.dzcT), nh2 / 2, dWc, H, H, H);
  add(P<u16>(ws, L.rhT), nh2 / 2, P<u16>(ws, L.dzcT), nh2 / 2, dWc + H * H, H, H, H);
  // d edge_weights[c] = sum h^T dM_c
  for (int ch = 0; ch < c.C; ++ch)
    add(P<u16>(ws, L.hT), nh2 / 2, P<u16>(ws, L.dMT + (size_t)ch * nh2), c.C * nh2 / 2, dW + (long)ch * H * H, H, H, H);
  a.nprob = np;
  a.T = c.T;
  // K chunking: rows per chunk, a divisor of N
  int KC = 4096;
  while (KC > 32 && (N % KC) != 0) KC /= 2;
  while (KC > 256 && (long)tiles * (N / KC) < 256) KC /= 2;
  if (N % KC) return fail(GGNN_EUNSUP, "rows not divisible into weight-gradient chunks");
  a.KC = KC;
  a.nchunks = (int)(N / KC);
  const int grid = tiles * a.nchunks;
  if (H < 128) {
    // M / N below one 128 tile are not supported by k_wgrad
    return fail(GGNN_EUNSUP, "weight gradients need hidden >= 128");
  }
  Prof p(7, s);
  if (KC % 64 == 0) hipLaunchKernelGGL(k_wgrad<64>, dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_wgrad<32>, dim3(grid), dim3(256), 0, s, a);
  LAUNCHCHK();
  return GGNN_OK;
}

}  // extern "C"
