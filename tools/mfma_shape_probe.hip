// MFMA shape probe (verdict r2 item 1a: "32x32x16 fragments for the GEMM tiles").
//
// The GEMM mainloop body in isolation: 8 waves per CU-resident block (2 per SIMD, as in the
// ping-pong GEMM), every operand fragment re-read from an XOR-swizzled LDS tile by ds_read_b128
// (the 128-byte-row image gemm_pp.h stages), random bf16 data, the same 64 x 64 output tile per
// wave and the same LDS bytes per FLOP in both arms:
//   arm 16: per 32-deep k-step 4 A + 4 B fragments (16 rows x 32 k), 16 x v_mfma_f32_16x16x32_bf16
//   arm 32: per 16-deep k-step 2 A + 2 B fragments (32 rows x 16 k),  4 x v_mfma_f32_32x32x16_bf16
// Both do 2 x 64^2 x 64 FLOP per wave per 64-deep k-tile from 16 KiB of fragment reads.
// Arms are interleaved over rounds in one process; prints TFLOP/s per arm and round.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_shape_probe.hip -o build/mfma_shape_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int ROWS = 256;            // LDS tile: 256 rows x 64 k bf16 (128-byte rows) = 32 KiB

__device__ inline bf16x8_t rd(const uint4* s, int row, int chunk) {
  const uint4 v = s[row * 8 + (chunk ^ ((row >> 1) & 7))];
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int SHAPE>
__global__ void __launch_bounds__(512, 1) probe(const uint4* __restrict__ src, float* __restrict__ out, int iters) {
  __shared__ uint4 s[ROWS * 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < ROWS * 8; i += 512) s[i] = src[(blockIdx.x * 97 + i) % (1 << 16)];
  __syncthreads();
  // wave (wm, wn) in a 2 x 4 grid: A rows 64 wm.., B rows 128 + 32 wn.. (overlapping reads are fine)
  const int a0 = 64 * (wave & 1), b0 = 128 + 32 * (wave >> 1) % 128;
  float sum = 0.f;
  if constexpr (SHAPE == 16) {
    f32x4_t acc[4][4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fq = lane >> 4;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = rd(s, a0 + 16 * i + fr, 4 * ks + fq);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = rd(s, (b0 + 16 * j + fr) & (ROWS - 1), 4 * ks + fq);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  } else {
    f32x16_t acc[2][2];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    const int fr = lane & 31, fq = lane >> 5;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8_t a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = rd(s, a0 + 32 * i + fr, 2 * ks + fq);
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = rd(s, (b0 + 32 * j + fr) & (ROWS - 1), 2 * ks + fq);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int e = 0; e < 16; ++e) sum += acc[i][j][e];
  }
  out[blockIdx.x * 512 + tid] = sum;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const int blocks = 256 * 4;
  std::vector<uint16_t> h(1 << 19);
  unsigned s = 12345u;
  for (auto& v : h) {            // uniform random bf16 in [-1, 1)
    s = s * 1664525u + 1013904223u;
    float f = ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
    v = (uint16_t)(__builtin_bit_cast(uint32_t, f) >> 16);
  }
  uint4* d_src;
  float* d_out;
  CK(hipMalloc(&d_src, h.size() * 2));
  CK(hipMalloc(&d_out, blocks * 512 * 4));
  CK(hipMemcpy(d_src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flop = 2.0 * 64 * 64 * 64 * 8 * (double)blocks * iters;   // per launch
  for (int w = 0; w < 3; ++w) {
    hipLaunchKernelGGL(probe<16>, dim3(blocks), dim3(512), 0, 0, d_src, d_out, iters);
    hipLaunchKernelGGL(probe<32>, dim3(blocks), dim3(512), 0, 0, d_src, d_out, iters);
  }
  CK(hipDeviceSynchronize());
  for (int round = 0; round < 5; ++round) {
    for (int arm : {16, 32}) {
      CK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) {
        if (arm == 16) hipLaunchKernelGGL(probe<16>, dim3(blocks), dim3(512), 0, 0, d_src, d_out, iters);
        else hipLaunchKernelGGL(probe<32>, dim3(blocks), dim3(512), 0, 0, d_src, d_out, iters);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"round\": %d, \"mfma\": \"%s\", \"ms_per_launch\": %.3f, \"tflops\": %.1f}\n", round,
             arm == 16 ? "16x16x32_bf16" : "32x32x16_bf16", ms / 5, flop / (ms / 5 * 1e-3) / 1e12);
    }
  }
  CK(hipFree(d_src));
  CK(hipFree(d_out));
  return 0;
}
