// MFMA shape probe: the message-transform loop of
// k_fwd_fused / k_prop_bwd's phase b -- A operand from a chunk-major f16 hi/lo
// LDS image (128 rows x K = 256), B operand (hi/lo weight fragments) streamed
// from L2, 3 MFMAs per product (fp32-parity limb split), 8 waves of 32 output
// columns each -- built once with v_mfma_f32_32x32x16_f16 (4 row tiles of 32)
// and once with v_mfma_f32_16x16x32_f16 (8 row tiles x 2 column strips of 16).
// Same FLOPs, same LDS and L2 bytes per FLOP.  Runs each variant back to back
// for >= `secs` seconds on random data (MI355X_MICROARCH.md "DVFS give-back":
// the clock the chip holds depends on the MFMA shape) and reports TFLOP/s from
// HIP events and the in-kernel clock (s_memtime / s_memrealtime around the
// loop, median over workgroups).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mfma_shape_probe tools/mfma_shape_probe.hip
//   tools/mfma_shape_probe [secs] [rounds]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef unsigned short u16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

constexpr int R = 128, K = 256, NT = 512, NITER = 64;
constexpr int IMG = R * K * 2;  // one limb image, bytes

__device__ inline uint4 ld16(const void* p) { return *(const uint4*)p; }
__device__ inline int kimg(int row, int ch) { return ch * (R * 16) + row * 16; }

template <int SHAPE>  // 32: 32x32x16, 16: 16x16x32
__global__ void __launch_bounds__(NT) k_probe(const u16* __restrict__ Ah, const u16* __restrict__ Al,
                                              const u16* __restrict__ Bh, const u16* __restrict__ Bl,
                                              float* __restrict__ out, unsigned long long* __restrict__ clk) {
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG];
  char* ih = smem;
  char* il = smem + IMG;
  const int tid = threadIdx.x, lane = tid & 63, ns = tid >> 6;
  for (int q = tid; q < R * K / 8; q += NT) {  // stage the A image (chunk-major), row-major source
    const int row = q % R, ch = q / R;
    *(uint4*)(ih + kimg(row, ch)) = ld16(Ah + row * K + ch * 8);
    *(uint4*)(il + kimg(row, ch)) = ld16(Al + row * K + ch * 8);
  }
  __syncthreads();
  unsigned long long rt0 = __builtin_amdgcn_s_memrealtime(), mt0 = __builtin_amdgcn_s_memtime();
  if constexpr (SHAPE == 32) {
    constexpr int KS = K / 16, RT = R / 32;
    f32x16 acc[RT];
    for (int i = 0; i < RT; ++i)
      for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
    // B fragments [strip ns][kstep][64][8]
    const u16* bh = Bh + (size_t)ns * KS * 512 + lane * 8;
    const u16* bl = Bl + (size_t)ns * KS * 512 + lane * 8;
    for (int it = 0; it < NITER; ++it) {
      uint4 wh = ld16(bh), wl = ld16(bl);
#pragma unroll 2
      for (int ks = 0; ks < KS; ++ks) {
        const int kn = ks + 1 < KS ? ks + 1 : 0;
        const uint4 nh = ld16(bh + kn * 512), nl = ld16(bl + kn * 512);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int off = kimg(rt * 32 + (lane & 31), 2 * ks + (lane >> 5));
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
    }
    float s = 0.f;
    for (int i = 0; i < RT; ++i)
      for (int j = 0; j < 16; ++j) s += acc[i][j];
    out[blockIdx.x * NT + tid] = s;
  } else {
    constexpr int KS = K / 32, RT = R / 16, CS = 2;
    f32x4 acc[RT][CS];
    for (int i = 0; i < RT; ++i)
      for (int c = 0; c < CS; ++c)
        for (int j = 0; j < 4; ++j) acc[i][c][j] = 0.f;
    // B fragments [strip (2 ns + c)][kstep][64][8]
    const u16* bh = Bh + (size_t)(2 * ns) * KS * 512 + lane * 8;
    const u16* bl = Bl + (size_t)(2 * ns) * KS * 512 + lane * 8;
    for (int it = 0; it < NITER; ++it) {
      uint4 wh[CS], wl[CS];
      for (int c = 0; c < CS; ++c) {
        wh[c] = ld16(bh + c * KS * 512);
        wl[c] = ld16(bl + c * KS * 512);
      }
#pragma unroll 2
      for (int ks = 0; ks < KS; ++ks) {
        const int kn = ks + 1 < KS ? ks + 1 : 0;
        uint4 nh[CS], nl[CS];
#pragma unroll
        for (int c = 0; c < CS; ++c) {
          nh[c] = ld16(bh + (c * KS + kn) * 512);
          nl[c] = ld16(bl + (c * KS + kn) * 512);
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int off = kimg(rt * 16 + (lane & 15), 4 * ks + (lane >> 4));
          const uint4 ah = ld16(ih + off), al = ld16(il + off);
          const f16x8 A = __builtin_bit_cast(f16x8, ah), AL = __builtin_bit_cast(f16x8, al);
#pragma unroll
          for (int c = 0; c < CS; ++c) {
            const f16x8 B = __builtin_bit_cast(f16x8, wh[c]), BL = __builtin_bit_cast(f16x8, wl[c]);
            acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AL, B, acc[rt][c], 0, 0, 0);
            acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, BL, acc[rt][c], 0, 0, 0);
            acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, acc[rt][c], 0, 0, 0);
          }
        }
#pragma unroll
        for (int c = 0; c < CS; ++c) {
          wh[c] = nh[c];
          wl[c] = nl[c];
        }
      }
    }
    float s = 0.f;
    for (int i = 0; i < RT; ++i)
      for (int c = 0; c < CS; ++c)
        for (int j = 0; j < 4; ++j) s += acc[i][c][j];
    out[blockIdx.x * NT + tid] = s;
  }
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
  const int NWG = 256;
  std::vector<u16> ah(R * K), al(R * K), bh(K * K), bl(K * K);
  srand(1);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  for (auto& x : ah) x = f2h(rnd());
  for (auto& x : al) x = f2h(rnd() * 1e-3f);
  for (auto& x : bh) x = f2h(rnd());
  for (auto& x : bl) x = f2h(rnd() * 1e-3f);
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
  const double flops = (double)NWG * NITER * 2.0 * R * K * K * 3;  // 3 products per limb-split product
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r) {
    for (int shape : {32, 16}) {
      auto launch = [&] {
        if (shape == 32) hipLaunchKernelGGL(k_probe<32>, dim3(NWG), dim3(NT), 0, 0, dAh, dAl, dBh, dBl, dout, dclk);
        else hipLaunchKernelGGL(k_probe<16>, dim3(NWG), dim3(NT), 0, 0, dAh, dAl, dBh, dBl, dout, dclk);
      };
      // >= secs of back-to-back launches, then 50 timed ones
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
      printf("{\"round\": %d, \"shape\": \"%s\", \"ms\": %.4f, \"tflops\": %.1f, \"clock_ghz_median\": %.3f, "
             "\"warm_launches\": %d}\n",
             r, shape == 32 ? "32x32x16" : "16x16x32", ms, flops / (ms * 1e-3) / 1e12, ghz[ghz.size() / 2], warm);
      fflush(stdout);
    }
  }
  return 0;
}
