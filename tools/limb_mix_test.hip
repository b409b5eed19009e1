// GPU check that the library's f16 limb residual (ggnn_common.h pk_lo<true>:
// v_fma_mix{lo,hi}_f16) gives the same bits as convert / subtract / convert
// over 2^24 pairs of random and special fp32 values.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/limb_mix_test tools/limb_mix_test.hip
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../ggnn_amd/csrc/ggnn_common.h"

__global__ void k_limbs(const float* x, uint32_t* lo, uint32_t* lo_ref, uint32_t* slo, uint32_t* slo_ref, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = x[2 * i], b = x[2 * i + 1];
  const f32x2v v = {a, b};
  const f32x2v back = __builtin_convertvector(__builtin_convertvector(v, f16x2v), f32x2v);
  const f32x2v d = v - back;
  lo_ref[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(d, f16x2v));
  lo[i] = pk_lo<true>(a, b);
  slo[i] = lo_limb16(a);  // the one-element form (img_put)
  slo_ref[i] = to_limb<true>(a - (float)(_Float16)a);
}

int main() {
  const int n = 1 << 24;
  float* hx = (float*)malloc(8L * n);
  uint32_t s = 12345;
  for (long i = 0; i < 2L * n; ++i) {
    s = s * 1664525u + 1013904223u;
    uint32_t bits = s;
    const uint32_t e = 127 - 40 + ((s >> 8) % 60);  // magnitudes 2^-40 .. 2^20
    bits = (bits & 0x807fffffu) | (e << 23);
    if (i % 97 == 0) bits = s;  // raw bit patterns: inf, nan, denormals, huge
    std::memcpy(&hx[i], &bits, 4);
  }
  const float special[] = {0.f, -0.f, 65504.f, 65519.f, 1e-8f, 6.1e-5f, 5.96e-8f, -3.0e-5f};
  for (int j = 0; j < 8; ++j) hx[j] = special[j];
  float* dx;
  uint32_t *dl, *dr, *ds, *dsr;
  if (hipMalloc(&dx, 8L * n) || hipMalloc(&dl, 4L * n) || hipMalloc(&dr, 4L * n) || hipMalloc(&ds, 4L * n) ||
      hipMalloc(&dsr, 4L * n))
    return 2;
  hipMemcpy(dx, hx, 8L * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_limbs, dim3(n / 256), dim3(256), 0, 0, dx, dl, dr, ds, dsr, n);
  uint32_t* l = (uint32_t*)malloc(4L * n);
  uint32_t* r = (uint32_t*)malloc(4L * n);
  hipMemcpy(l, dl, 4L * n, hipMemcpyDeviceToHost);
  hipMemcpy(r, dr, 4L * n, hipMemcpyDeviceToHost);
  long bad = 0, badfin = 0;
  for (long i = 0; i < n; ++i)
    if (l[i] != r[i]) {
      ++bad;
      const float a = hx[2 * i], b = hx[2 * i + 1];
      if (std::isfinite(a) && std::isfinite(b) && std::fabs(a) < 65504.f && std::fabs(b) < 65504.f) {
        if (badfin < 5) printf("mismatch %ld a=%g b=%g mix=%08x ref=%08x\n", i, a, b, l[i], r[i]);
        ++badfin;
      }
    }
  uint32_t* sl = (uint32_t*)malloc(4L * n);
  uint32_t* sr = (uint32_t*)malloc(4L * n);
  hipMemcpy(sl, ds, 4L * n, hipMemcpyDeviceToHost);
  hipMemcpy(sr, dsr, 4L * n, hipMemcpyDeviceToHost);
  long sbad = 0;
  for (long i = 0; i < n; ++i) {
    const float a = hx[2 * i];
    if ((sl[i] & 0xffffu) != (sr[i] & 0xffffu) && std::isfinite(a) && std::fabs(a) < 65504.f) {
      if (sbad < 5) printf("element mismatch %ld a=%g mix=%04x ref=%04x\n", i, a, sl[i] & 0xffffu, sr[i] & 0xffffu);
      ++sbad;
    }
  }
  printf("pairs %d, mismatches %ld (finite, within the f16 range: %ld); one-element form: %ld\n", n, bad, badfin,
         sbad);
  return badfin != 0 || sbad != 0;
}
