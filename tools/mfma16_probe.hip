// (round 5) v_mfma_f32_16x16x16_bf16 vs v_mfma_f32_16x16x32_bf16 on gfx950: issue rate (4
// independent accumulators per wave, register operands, 4 waves per SIMD) and the SrcC hand-off
// between the two shapes (a 16x16x32 result used at once as the 16x16x16 accumulator: the
// compiler inserted no wait state there; this checks what the hardware returns).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma16_probe.hip -o build/mfma16_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

template <int SHAPE>
__global__ void __launch_bounds__(256) rate(float* out, int iters, float seed) {
  bf16x8_t a, b;
  s16x4_t a4, b4;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(seed * (threadIdx.x + i)); b[i] = (__bf16)(seed * (i - (int)threadIdx.x)); }
  for (int i = 0; i < 4; ++i) { a4[i] = __builtin_bit_cast(short, a[i]); b4[i] = __builtin_bit_cast(short, b[i]); }
  f32x4_t acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (SHAPE == 32) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
      else acc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[i], 0, 0, 0);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
}

// D = mfma16(A16, B16, mfma32(A32, B32, 0)) with the 16x16x32 result fed straight in
template <int ORDER>
__global__ void chain(const float* A, const float* B, float* D) {   // A [16][48], B [48][16] (k-major mix)
  const int l = threadIdx.x, i = l & 15, g = l >> 4;
  bf16x8_t a32, b32;
  s16x4_t a16, b16;
  for (int j = 0; j < 8; ++j) { a32[j] = (__bf16)A[i * 48 + 8 * g + j]; b32[j] = (__bf16)B[(8 * g + j) * 16 + i]; }
  for (int j = 0; j < 4; ++j) {
    a16[j] = __builtin_bit_cast(short, (__bf16)A[i * 48 + 32 + 4 * g + j]);
    b16[j] = __builtin_bit_cast(short, (__bf16)B[(32 + 4 * g + j) * 16 + i]);
  }
  f32x4_t z = {0.f, 0.f, 0.f, 0.f};
  if constexpr (ORDER == 0) {
    z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a32, b32, z, 0, 0, 0);
    z = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a16, b16, z, 0, 0, 0);
  } else {
    z = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a16, b16, z, 0, 0, 0);
    z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a32, b32, z, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + i] = z[r];
}

int main() {
  float* d_out;
  CK(hipMalloc(&d_out, 4096 * 256 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20000, blocks = 4096;
  for (int rep = 0; rep < 3; ++rep)
    for (int shape : {32, 16}) {
      if (shape == 32) hipLaunchKernelGGL(rate<32>, dim3(blocks), dim3(256), 0, 0, d_out, 100, 0.001f);
      else hipLaunchKernelGGL(rate<16>, dim3(blocks), dim3(256), 0, 0, d_out, 100, 0.001f);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      if (shape == 32) hipLaunchKernelGGL(rate<32>, dim3(blocks), dim3(256), 0, 0, d_out, iters, 0.001f);
      else hipLaunchKernelGGL(rate<16>, dim3(blocks), dim3(256), 0, 0, d_out, iters, 0.001f);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double mfmas_per_simd = (double)blocks * 4 /*waves*/ * iters * 4 / 1024.0;
      const double flop = (double)blocks * 4 * iters * 4 * 2.0 * 16 * 16 * shape;
      printf("{\"mfma\": \"16x16x%d_bf16\", \"ms\": %.3f, \"tflops\": %.1f, \"ns_per_mfma_per_simd\": %.3f}\n", shape, ms,
             flop / ms / 1e9, ms * 1e6 / mfmas_per_simd);
    }
  // hazard check
  std::vector<float> A(16 * 48), B(48 * 16), D(256);
  unsigned s = 7u;
  for (auto& v : A) { s = s * 1664525u + 1013904223u; v = (float)((int)(s >> 27) - 16); }
  for (auto& v : B) { s = s * 1664525u + 1013904223u; v = (float)((int)(s >> 27) - 16); }
  float *dA, *dB, *dD;
  CK(hipMalloc(&dA, A.size() * 4)); CK(hipMalloc(&dB, B.size() * 4)); CK(hipMalloc(&dD, 256 * 4));
  CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
  for (int order = 0; order < 2; ++order) {
    if (order == 0) hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    else hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    CK(hipMemcpy(D.data(), dD, 256 * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    double maxerr = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double ref = 0;
        for (int k = 0; k < 48; ++k) ref += (double)A[i * 48 + k] * B[k * 16 + j];
        double e = fabs(ref - D[i * 16 + j]);
        maxerr = e > maxerr ? e : maxerr;
        bad += e > 0.5;
      }
    printf("{\"chain\": \"%s\", \"bad\": %d, \"max_abs_err\": %.1f}\n", order == 0 ? "32->16" : "16->32", bad, maxerr);
  }
  return 0;
}
