// (round 6) Does a polynomial exp2 on the FMA path pay on gfx950?  VERDICT r5 item 2 proposed
// evaluating part of each attention tile's exp2 as a Cody-Waite split + degree-3 polynomial so
// that "the transcendental and FMA pipes run in parallel".  This probe measures, per wave and
// iteration of 16 independent values per lane:
//   exp   : 16 v_exp_f32
//   fma   : 16 v_fma_f32
//   mix   : 16 v_exp_f32 + 16 v_fma_f32 on independent registers (overlap of the two?)
//   poly  : 16 x (floor, sub, 3 fma, cvt, lshl_add): the FMA-path exp2
//   poly8 : 8 v_exp_f32 + 8 poly (the proposed split)
// at 1 and 2 waves per SIMD.  s_memtime cycles per iteration (100 MHz-independent: the same
// counter for all variants), averaged over the grid.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp_pipe_probe.hip -o build/exp_pipe_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ float poly_exp2(float x) {
  // x <= 0 here; 2^x = 2^floor(x) * 2^f, f in [0, 1): degree-3 minimax of 2^f (rel err ~1e-4)
  const float fl = __builtin_floorf(x);
  const float f = x - fl;
  float p = fmaf(fmaf(fmaf(0.0790209f, f, 0.2249340f), f, 0.6960656f), f, 1.0000011f);
  const int e = (int)fl;
  return __int_as_float(__float_as_int(p) + (e << 23));
}

template <int MODE>
__global__ void __launch_bounds__(512) probe(float* out, unsigned long long* cyc, int iters, float seed) {
  float r[16], s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { r[i] = -0.25f - 0.01f * i - seed * threadIdx.x; s[i] = 0.5f + 0.001f * i; }
  const float a = 0.999f, b = 1e-4f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (MODE == 0) r[i] = __builtin_amdgcn_exp2f(-r[i]);
      if constexpr (MODE == 1) s[i] = fmaf(s[i], a, b);
      if constexpr (MODE == 2) { r[i] = __builtin_amdgcn_exp2f(-r[i]); s[i] = fmaf(s[i], a, b); }
      if constexpr (MODE == 3) r[i] = poly_exp2(-r[i]);
      if constexpr (MODE == 4) r[i] = (i & 1) ? poly_exp2(-r[i]) : __builtin_amdgcn_exp2f(-r[i]);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += r[i] + s[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
double run(int waves_per_simd, int iters) {
  const int threads = 256 * waves_per_simd;        // 4 SIMDs per CU, one block per CU
  const int blocks = 256;
  float* out;
  unsigned long long* cyc;
  CK(hipMalloc(&out, sizeof(float) * blocks * threads));
  CK(hipMalloc(&cyc, sizeof(unsigned long long) * blocks * threads / 64));
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 10, 0.001f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 0.001f);
  CK(hipEventRecord(e1));
  CK(hipDeviceSynchronize());
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(blocks * threads / 64);
  CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  double mean = 0;
  for (auto v : h) mean += (double)v;
  mean /= h.size();
  CK(hipFree(out));
  CK(hipFree(cyc));
  // wall ns per iteration per wave is what matters (the SIMD's issue port is shared by its waves)
  return 1e6 * ms / iters;
}

int main() {
  const int iters = 20000;
  const char* names[] = {"exp16", "fma16", "exp16+fma16", "poly16", "exp8+poly8"};
  for (int w = 1; w <= 2; ++w) {
    double t[5] = {run<0>(w, iters), run<1>(w, iters), run<2>(w, iters), run<3>(w, iters), run<4>(w, iters)};
    for (int m = 0; m < 5; ++m)
      printf("{\"waves_per_simd\": %d, \"variant\": \"%s\", \"ns_per_iter\": %.3f, \"rel_exp16\": %.3f}\n", w, names[m], t[m],
             t[m] / t[0]);
  }
  // accuracy of the polynomial against v_exp_f32 on the host-side reference
  double worst = 0;
  for (int i = 0; i < 100000; ++i) {
    const float x = -20.f * i / 100000.f;
    const float fl = floorf(x), f = x - fl;
    const float p = fmaf(fmaf(fmaf(0.0790209f, f, 0.2249340f), f, 0.6960656f), f, 1.0000011f);
    const double v = ldexp((double)p, (int)fl), ref = exp2((double)x);
    const double rel = fabs(v - ref) / ref;
    if (rel > worst) worst = rel;
  }
  printf("{\"poly_exp2_max_rel_err\": %.3e, \"bf16_half_ulp\": %.3e}\n", worst, 1.0 / 512);
  return 0;
}
