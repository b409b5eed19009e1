// MX-fp8 limb-correction probe (round 6): can the fp32-parity limb split
//   a.b ~= a_hi.b_hi + a_hi.b_lo + a_lo.b_hi          (3 f16 MFMAs per K = 16)
// put its two correction terms on the block-scaled fp8 MFMA instead?
//   a.b ~= a_hi.b_hi  (f16, 2 x v_mfma_f32_32x32x16_f16 per 32 K)
//        + [e4m3(a_hi) | e4m3(a_lo 2^S)] . [e4m3(b_lo 2^S) ; e4m3(b_hi)] 2^-S
//                      (one v_mfma_scale_f32_32x32x64_f8f6f4 per 32 K: its K = 64
//                       holds both correction terms of 32 k's; the 2^-S comes
//                       from the E8M0 scale operand)
// The guide's rates (MI355X_MICROARCH.md, Matrix cores): the scaled 32x32x64 fp8
// MFMA takes twice the cycles of the 32x32x16 16-bit form, so per 32 K the
// hybrid issues 2 + 2 = 4 units against 6.
//
// Part 1 (layout): one wave, random small integers exactly representable in
// e4m3, per-lane scales; the host checks D against the pairing "A lane l byte j
// meets B lane l' byte j iff l >> 5 == l' >> 5" (row = A lane & 31, column =
// B lane & 31) and "lane l's scale multiplies its own 32 bytes".
// Part 2 (rate): the message-transform loop of k_prop_bwd's phase b /
// k_fwd_fused's MT (128 rows x K = 256 per workgroup, A from a chunk-major LDS
// image, B streamed from L2, 8 waves of 32 columns), 3-product f16 vs hybrid,
// same LDS and L2 bytes per K; TFLOP/s counted as the 3-product FLOPs.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mx_hybrid_probe tools/mx_hybrid_probe.hip
//   tools/mx_hybrid_probe [secs] [rounds]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef unsigned short u16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

// ---------------------------------------------------------------- part 1
__global__ void k_layout(const i32x8* __restrict__ a, const i32x8* __restrict__ b, const int* __restrict__ sa,
                         const int* __restrict__ sb, float* __restrict__ d) {
  // one MFMA per wave; wave w reads its own operands (a, b: [w][64] lanes)
  const int l = threadIdx.x & 63, w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[w * 64 + l], b[w * 64 + l], acc, 0, 0, 0, sa[w * 64 + l],
                                                         0, sb[w * 64 + l]);
  for (int i = 0; i < 16; ++i) d[((long)w * 64 + l) * 16 + i] = acc[i];
}

// OCP e4m3fn encode of an exactly representable value (host, by search)
static uint8_t e4m3(float x) {
  if (x == 0.f) return 0;
  if (x == 1.f) return 0x38;
  for (int c = 0; c < 256; ++c) {
    if ((c & 0x7F) == 0x7F) continue;  // NaN
    const int s = c >> 7, e = (c >> 3) & 15, m = c & 7;
    const float v = (e == 0 ? ldexpf((float)m / 8.f, -6) : ldexpf(1.f + m / 8.f, e - 7)) * (s ? -1.f : 1.f);
    if (v == x) return (uint8_t)c;
  }
  fprintf(stderr, "not exact in e4m3: %g\n", x);
  exit(1);
}

// runs nw MFMAs: A[w][lane][byte], B likewise (float values, e4m3-exact), scales
static std::vector<float> run_mfma(int nw, const std::vector<float>& Av, const std::vector<float>& Bv,
                                   const std::vector<int>& sa, const std::vector<int>& sb) {
  std::vector<uint8_t> A(nw * 64 * 32), B(nw * 64 * 32);
  for (size_t i = 0; i < A.size(); ++i) {
    A[i] = e4m3(Av[i]);
    B[i] = e4m3(Bv[i]);
  }
  i32x8 *da, *db;
  int *dsa, *dsb;
  float* dd;
  CHK(hipMalloc(&da, A.size()));
  CHK(hipMalloc(&db, B.size()));
  CHK(hipMalloc(&dsa, nw * 64 * 4));
  CHK(hipMalloc(&dsb, nw * 64 * 4));
  CHK(hipMalloc(&dd, (size_t)nw * 64 * 16 * 4));
  CHK(hipMemcpy(da, A.data(), A.size(), hipMemcpyHostToDevice));
  CHK(hipMemcpy(db, B.data(), B.size(), hipMemcpyHostToDevice));
  CHK(hipMemcpy(dsa, sa.data(), nw * 64 * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dsb, sb.data(), nw * 64 * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_layout, dim3(nw), dim3(64), 0, 0, da, db, dsa, dsb, dd);
  CHK(hipDeviceSynchronize());
  std::vector<float> D((size_t)nw * 64 * 16);
  CHK(hipMemcpy(D.data(), dd, D.size() * 4, hipMemcpyDeviceToHost));
  CHK(hipFree(da));
  CHK(hipFree(db));
  CHK(hipFree(dsa));
  CHK(hipFree(dsb));
  CHK(hipFree(dd));
  return D;
}

static inline int drow(int l, int i) { return (i & 3) + 8 * (i >> 2) + 4 * (l >> 5); }

static int part1() {
  // E1: one-hot A positions against B = 1 everywhere -> the row of each A (lane, byte)
  //     one-hot B positions against A = 1 everywhere -> the column of each B (lane, byte)
  const int P = 64 * 32;
  std::vector<float> Av((size_t)P * P, 0.f), Bv((size_t)P * P, 1.f);
  std::vector<int> s127((size_t)P * 64, 127);
  for (int p = 0; p < P; ++p) Av[(size_t)p * P + p] = 1.f;
  std::vector<float> D = run_mfma(P, Av, Bv, s127, s127);
  std::vector<int> rowA(P, -1), colB(P, -1);
  int amb = 0;
  for (int p = 0; p < P; ++p) {
    int cnt = 0;
    for (int l = 0; l < 64; ++l)
      for (int i = 0; i < 16; ++i)
        if (D[((size_t)p * 64 + l) * 16 + i] != 0.f) {
          if (rowA[p] != drow(l, i) && rowA[p] >= 0) ++amb;
          rowA[p] = drow(l, i);
          ++cnt;
        }
    if (cnt != 32) ++amb;
  }
  std::fill(Av.begin(), Av.end(), 1.f);
  std::fill(Bv.begin(), Bv.end(), 0.f);
  for (int p = 0; p < P; ++p) Bv[(size_t)p * P + p] = 1.f;
  D = run_mfma(P, Av, Bv, s127, s127);
  for (int p = 0; p < P; ++p) {
    int cnt = 0;
    for (int l = 0; l < 64; ++l)
      for (int i = 0; i < 16; ++i)
        if (D[((size_t)p * 64 + l) * 16 + i] != 0.f) {
          if (colB[p] != (l & 31) && colB[p] >= 0) ++amb;
          colB[p] = l & 31;
          ++cnt;
        }
    if (cnt != 32) ++amb;
  }
  // E2: pairing. A one-hot at (la, ja); B[lb][jb] = bit bit of (64 * ... ) code
  //     code(lb, jb) = (lb >> 5) * 32 + jb (6 bits), one run per bit
  std::vector<int> pairA(P, 0);
  for (int bit = 0; bit < 6; ++bit) {
    std::fill(Av.begin(), Av.end(), 0.f);
    for (int p = 0; p < P; ++p) {
      Av[(size_t)p * P + p] = 1.f;
      for (int q = 0; q < P; ++q) {
        const int code = ((q / 32) >> 5) * 32 + (q % 32);
        Bv[(size_t)p * P + q] = ((code >> bit) & 1) ? 1.f : 0.f;
      }
    }
    D = run_mfma(P, Av, Bv, s127, s127);
    for (int p = 0; p < P; ++p) {
      // any output of A's row: take column 0's entry (lane 0.. of the row)
      float v = 0.f;
      for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 16; ++i)
          if (drow(l, i) == rowA[p] && (l & 31) == 0) v = D[((size_t)p * 64 + l) * 16 + i];
      if (v != 0.f) pairA[p] |= 1 << bit;
    }
  }
  printf("{\"part\": \"layout_onehot\", \"ambiguous\": %d,\n \"rowA_lane\": [", amb);
  for (int l = 0; l < 64; ++l) printf("%d%s", rowA[l * 32], l < 63 ? "," : "]");
  printf(",\n \"colB_lane\": [");
  for (int l = 0; l < 64; ++l) printf("%d%s", colB[l * 32], l < 63 ? "," : "]");
  int rowvar = 0, colvar = 0;
  for (int p = 0; p < P; ++p) {
    rowvar += rowA[p] != rowA[(p / 32) * 32];
    colvar += colB[p] != colB[(p / 32) * 32];
  }
  printf(",\n \"row_varies_within_lane\": %d, \"col_varies_within_lane\": %d", rowvar, colvar);
  for (int la : {0, 1, 31, 32, 33, 63}) {
    printf(",\n \"pair_of_A_lane%d\": [", la);  // B (half, byte) code = half*32 + byte, per A byte j
    for (int j = 0; j < 32; ++j) printf("%d%s", pairA[la * 32 + j], j < 31 ? "," : "]");
  }
  printf("}\n");
  fflush(stdout);
  // E3: random values, per-lane scales, the decoded pairing
  const int NW = 1;
  std::vector<float> Ar(64 * 32), Br(64 * 32);
  std::vector<int> sa(64), sb(64);
  srand(7);
  const float vals[] = {0.f, 1.f, -1.f, 2.f, -2.f, 3.f, -3.f, 4.f, 0.5f, -0.5f, 1.5f};
  for (int i = 0; i < 64 * 32; ++i) {
    Ar[i] = vals[rand() % 11];
    Br[i] = vals[rand() % 11];
  }
  int bad[2] = {0, 0};
  for (int sc = 0; sc < 2; ++sc) {
    for (int l = 0; l < 64; ++l) {
      sa[l] = sc ? 127 + (rand() % 5) - 2 : 127;
      sb[l] = sc ? 127 + (rand() % 5) - 2 : 127;
    }
    std::vector<float> Dr = run_mfma(NW, Ar, Br, sa, sb);
    // B position of code: lane = half * 32 + col, byte
    for (int l = 0; l < 64; ++l)
      for (int i = 0; i < 16; ++i) {
        const int col = l & 31, row = drow(l, i);
        double ref = 0;
        for (int p = 0; p < P; ++p) {
          if (rowA[p] != row) continue;
          const int code = pairA[p], lb = (code >> 5) * 32 + col, jb = code & 31;
          ref += (double)Ar[p] * ldexp(1.0, sa[p / 32] - 127) * Br[lb * 32 + jb] * ldexp(1.0, sb[lb] - 127);
        }
        if (fabs(ref - Dr[l * 16 + i]) > 1e-6 * std::max(1.0, fabs(ref))) ++bad[sc];
      }
  }
  // E4: which lane's scale multiplies an A / B byte: lane l's scale = 2^(l - 27)
  {
    const int js[4] = {0, 15, 16, 31};
    const int NR = 2 * 64 * 4;
    std::vector<float> Ae((size_t)NR * P, 0.f), Be((size_t)NR * P, 0.f);
    std::vector<int> se((size_t)NR * 64), s1((size_t)NR * 64, 127);
    for (int w = 0; w < NR; ++w) {
      const int side = w / 256, la = (w / 4) % 64, ja = js[w % 4];
      for (int q = 0; q < P; ++q) (side ? Ae : Be)[(size_t)w * P + q] = 1.f;
      (side ? Be : Ae)[(size_t)w * P + la * 32 + ja] = 1.f;
      for (int l = 0; l < 64; ++l) se[(size_t)w * 64 + l] = 100 + l;
    }
    std::vector<float> Da = run_mfma(NR / 2, std::vector<float>(Ae.begin(), Ae.begin() + (size_t)NR / 2 * P),
                                     std::vector<float>(Be.begin(), Be.begin() + (size_t)NR / 2 * P),
                                     std::vector<int>(se.begin(), se.begin() + NR / 2 * 64),
                                     std::vector<int>(s1.begin(), s1.begin() + NR / 2 * 64));
    std::vector<float> Db = run_mfma(NR / 2, std::vector<float>(Ae.begin() + (size_t)NR / 2 * P, Ae.end()),
                                     std::vector<float>(Be.begin() + (size_t)NR / 2 * P, Be.end()),
                                     std::vector<int>(s1.begin(), s1.begin() + NR / 2 * 64),
                                     std::vector<int>(se.begin(), se.begin() + NR / 2 * 64));
    printf("{\"part\": \"scale_lane\", \"note\": \"[A or B lane, byte] -> lane whose scale applied (-1: none/other)\",\n \"A\": [");
    for (int w = 0; w < NR / 2; ++w) {
      float mx = 0.f;
      for (int i = 0; i < 64 * 16; ++i) mx = std::max(mx, fabsf(Da[(size_t)w * 1024 + i]));
      const int used = mx > 0.f ? (int)lrint(log2(mx)) + 27 : -1;
      printf("[%d,%d,%d]%s", (w / 4) % 64, js[w % 4], used, w < NR / 2 - 1 ? "," : "]");
    }
    printf(",\n \"B\": [");
    for (int w = 0; w < NR / 2; ++w) {
      float mx = 0.f;
      for (int i = 0; i < 64 * 16; ++i) mx = std::max(mx, fabsf(Db[(size_t)w * 1024 + i]));
      const int used = mx > 0.f ? (int)lrint(log2(mx)) + 27 : -1;
      printf("[%d,%d,%d]%s", (w / 4) % 64, js[w % 4], used, w < NR / 2 - 1 ? "," : "]");
    }
    printf("}\n");
  }
  printf("{\"part\": \"layout_random\", \"mismatches_scale127\": %d, \"mismatches_lane_scales\": %d}\n", bad[0], bad[1]);
  fflush(stdout);
  return amb + bad[0] + bad[1];
}

// ---------------------------------------------------------------- part 1b
// byte order of the packed converts the kernels use (ggnn_common.h pk4_bf8,
// pk4_fp8, f16x8_to_fp8): element i of the source -> byte i of the result
typedef short v2i16_t __attribute__((ext_vector_type(2)));
typedef _Float16 v2f16_t __attribute__((ext_vector_type(2)));
__global__ void k_cvt_order(unsigned* o) {
  unsigned w = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(1.0f, 2.0f, 0, false);
  o[0] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(3.0f, 4.0f, (int)w, true);
  w = (unsigned)__builtin_amdgcn_cvt_pk_bf8_f32(1.0f, 2.0f, 0, false);
  o[1] = (unsigned)__builtin_amdgcn_cvt_pk_bf8_f32(3.0f, 4.0f, (int)w, true);
  v2i16_t r = {0, 0};
  const v2f16_t a = {(_Float16)1.0f, (_Float16)2.0f}, b = {(_Float16)3.0f, (_Float16)4.0f};
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(r, a, 1.0f, false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(r, b, 1.0f, true);
  o[2] = __builtin_bit_cast(unsigned, r);
}
static int part1b() {
  unsigned* d;
  CHK(hipMalloc(&d, 16));
  hipLaunchKernelGGL(k_cvt_order, dim3(1), dim3(1), 0, 0, d);
  unsigned h[3];
  CHK(hipMemcpy(h, d, 12, hipMemcpyDeviceToHost));
  // e4m3 1,2,3,4 = 0x38 0x40 0x44 0x48; e5m2 1,2,3,4 = 0x3C 0x40 0x42 0x44
  const bool ok = h[0] == 0x48444038u && h[1] == 0x4442403Cu && h[2] == 0x48444038u;
  printf("{\"part\": \"cvt_order\", \"fp8_f32\": \"0x%08x\", \"bf8_f32\": \"0x%08x\", \"fp8_f16\": \"0x%08x\", "
         "\"element_i_to_byte_i\": %s}\n", h[0], h[1], h[2], ok ? "true" : "false");
  fflush(stdout);
  return ok ? 0 : 1;
}

// ---------------------------------------------------------------- part 2
constexpr int R = 128, K = 256, NT = 512, NITER = 64;
constexpr int IMG = R * K * 2;  // one f16 limb image, bytes (= the fp8 [hi | lo] image)

__device__ inline uint4 ld16(const void* p) { return *(const uint4*)p; }
__device__ inline int kimg(int row, int ch) { return ch * (R * 16) + row * 16; }

template <int MODE>  // 0: 3 x f16, 1: 2 x f16 + 1 x MX fp8 (K 64) per 32 K
__global__ void __launch_bounds__(NT) k_rate(const u16* __restrict__ Ah, const u16* __restrict__ Al,
                                             const u16* __restrict__ Bh, const u16* __restrict__ Bl,
                                             float* __restrict__ out, unsigned long long* __restrict__ clk) {
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG];
  char* ih = smem;
  char* il = smem + IMG;  // MODE 1: the fp8 image, 4 chunks per (row, 32-K block): hi0 hi1 lo0 lo1
  const int tid = threadIdx.x, lane = tid & 63, ns = tid >> 6;
  for (int q = tid; q < R * K / 8; q += NT) {
    const int row = q % R, ch = q / R;
    *(uint4*)(ih + kimg(row, ch)) = ld16(Ah + row * K + ch * 8);
    *(uint4*)(il + kimg(row, ch)) = ld16(Al + row * K + ch * 8);
  }
  __syncthreads();
  unsigned long long rt0 = __builtin_amdgcn_s_memrealtime(), mt0 = __builtin_amdgcn_s_memtime();
  constexpr int KS = K / 16, RT = R / 32;
  f32x16 acc[RT];
  for (int i = 0; i < RT; ++i)
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  const u16* bh = Bh + (size_t)ns * KS * 512 + lane * 8;
  const u16* bl = Bl + (size_t)ns * KS * 512 + lane * 8;
  const int l32 = lane & 31, hh = lane >> 5;
  for (int it = 0; it < NITER; ++it) {
    if constexpr (MODE == 0) {
      uint4 wh = ld16(bh), wl = ld16(bl);
#pragma unroll 2
      for (int ks = 0; ks < KS; ++ks) {
        const int kn = ks + 1 < KS ? ks + 1 : 0;
        const uint4 nh = ld16(bh + kn * 512), nl = ld16(bl + kn * 512);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int off = kimg(rt * 32 + l32, 2 * ks + hh);
          const uint4 ah = ld16(ih + off), al = ld16(il + off);
          const f16x8 A = __builtin_bit_cast(f16x8, ah), AL = __builtin_bit_cast(f16x8, al);
          const f16x8 B = __builtin_bit_cast(f16x8, wh), BL = __builtin_bit_cast(f16x8, wl);
          acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AL, B, acc[rt], 0, 0, 0);
          acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, BL, acc[rt], 0, 0, 0);
          acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, B, acc[rt], 0, 0, 0);
        }
        wh = nh;
        wl = nl;
      }
    } else {
      // per 32-K block kb: f16 hi fragments of k-steps 2kb, 2kb+1 (2 x 16 B) and
      // one 32 B fp8 fragment, from the same bytes per K as MODE 0
      constexpr int KB = K / 32;
      uint4 w0 = ld16(bh), w1 = ld16(bh + 512), f0 = ld16(bl), f1 = ld16(bl + 512);
#pragma unroll 2
      for (int kb = 0; kb < KB; ++kb) {
        const int kn = kb + 1 < KB ? kb + 1 : 0;
        const uint4 n0 = ld16(bh + 2 * kn * 512), n1 = ld16(bh + (2 * kn + 1) * 512);
        const uint4 g0 = ld16(bl + 2 * kn * 512), g1 = ld16(bl + (2 * kn + 1) * 512);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int row = rt * 32 + l32;
          const uint4 a0 = ld16(ih + kimg(row, 4 * kb + hh)), a1 = ld16(ih + kimg(row, 4 * kb + 2 + hh));
          const uint4 p0 = ld16(il + kimg(row, 4 * kb + 2 * hh)), p1 = ld16(il + kimg(row, 4 * kb + 2 * hh + 1));
          acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a0), __builtin_bit_cast(f16x8, w0),
                                                            acc[rt], 0, 0, 0);
          acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a1), __builtin_bit_cast(f16x8, w1),
                                                            acc[rt], 0, 0, 0);
          const i32x8 fa = {(int)p0.x, (int)p0.y, (int)p0.z, (int)p0.w, (int)p1.x, (int)p1.y, (int)p1.z, (int)p1.w};
          const i32x8 fb = {(int)f0.x, (int)f0.y, (int)f0.z, (int)f0.w, (int)f1.x, (int)f1.y, (int)f1.z, (int)f1.w};
          acc[rt] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa, fb, acc[rt], 0, 0, 0, 127 - 16, 0, 127);
        }
        w0 = n0;
        w1 = n1;
        f0 = g0;
        f1 = g1;
      }
    }
  }
  float s = 0.f;
  for (int i = 0; i < RT; ++i)
    for (int j = 0; j < 16; ++j) s += acc[i][j];
  out[blockIdx.x * NT + tid] = s;
  unsigned long long rt1 = __builtin_amdgcn_s_memrealtime(), mt1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) {
    clk[blockIdx.x * 2] = rt1 - rt0;
    clk[blockIdx.x * 2 + 1] = mt1 - mt0;
  }
}

static u16 f2h(float x) {
  _Float16 h = (_Float16)x;
  return *(u16*)&h;
}

int main(int argc, char** argv) {
  const double secs = argc > 1 ? atof(argv[1]) : 3.0;
  const int rounds = argc > 2 ? atoi(argv[2]) : 2;
  if (argc > 3 && argv[3][0] == 'c') return part1b();
  const int p1 = part1() + part1b();
  if (argc > 3) return p1;
  const int NWG = 256;
  std::vector<u16> ah(R * K), al(R * K), bh(K * K), bl(K * K);
  srand(1);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  // MODE 1 reads the "lo" arrays as fp8 bytes: any bit pattern but NaN (0x7F / 0xFF) is fine for a rate
  for (auto& x : ah) x = f2h(rnd());
  for (auto& x : al) x = f2h(rnd() * 1e-3f) & 0x7E7E;
  for (auto& x : bh) x = f2h(rnd());
  for (auto& x : bl) x = f2h(rnd() * 1e-3f) & 0x7E7E;
  u16 *dAh, *dAl, *dBh, *dBl;
  float* dout;
  unsigned long long* dclk;
  CHK(hipMalloc(&dAh, ah.size() * 2));
  CHK(hipMalloc(&dAl, al.size() * 2));
  CHK(hipMalloc(&dBh, bh.size() * 2));
  CHK(hipMalloc(&dBl, bl.size() * 2));
  CHK(hipMalloc(&dout, NWG * NT * 4));
  CHK(hipMalloc(&dclk, NWG * 16));
  CHK(hipMemcpy(dAh, ah.data(), ah.size() * 2, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dAl, al.data(), al.size() * 2, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dBh, bh.data(), bh.size() * 2, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dBl, bl.data(), bl.size() * 2, hipMemcpyHostToDevice));
  const double flops = (double)NWG * NITER * 2.0 * R * K * K * 3;  // 3-product FLOPs for both modes
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r) {
    for (int mode : {0, 1}) {
      auto launch = [&] {
        if (mode == 0) hipLaunchKernelGGL(k_rate<0>, dim3(NWG), dim3(NT), 0, 0, dAh, dAl, dBh, dBl, dout, dclk);
        else hipLaunchKernelGGL(k_rate<1>, dim3(NWG), dim3(NT), 0, 0, dAh, dAl, dBh, dBl, dout, dclk);
      };
      launch();
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      launch();
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms1;
      CHK(hipEventElapsedTime(&ms1, e0, e1));
      const int warm = std::max(1, (int)(secs * 1e3 / std::max(ms1, 1e-3f)));
      for (int i = 0; i < warm; ++i) launch();
      const int nt = 50;
      CHK(hipEventRecord(e0));
      for (int i = 0; i < nt; ++i) launch();
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      ms /= nt;
      std::vector<unsigned long long> clk(NWG * 2);
      CHK(hipMemcpy(clk.data(), dclk, NWG * 16, hipMemcpyDeviceToHost));
      std::vector<double> ghz;
      for (int w = 0; w < NWG; ++w)
        if (clk[2 * w]) ghz.push_back((double)clk[2 * w + 1] / clk[2 * w] * 0.1);
      std::sort(ghz.begin(), ghz.end());
      printf("{\"round\": %d, \"mode\": \"%s\", \"ms\": %.4f, \"tflops_3product_equiv\": %.1f, "
             "\"clock_ghz_median\": %.3f, \"warm_launches\": %d}\n",
             r, mode == 0 ? "f16x3" : "f16+mxfp8", ms, flops / (ms * 1e-3) / 1e12, ghz[ghz.size() / 2], warm);
      fflush(stdout);
    }
  }
  return 0;
}
