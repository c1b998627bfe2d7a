// Timing diagnostics of the ping-pong GEMM mainloop (ops/csrc/gemm_pp.h DIAG template bit):
// the same kernel with its mainloop DMA and/or barriers removed, on the SD-1.5 level-1 conv and
// a 4096^3 GEMM, so the cost of each part of the phase skeleton can be read off (results of the
// DIAG != 0 arms are wrong by construction; only their time is printed).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I cassmantle_amd/ops/csrc \
//         -mllvm -pragma-unroll-threshold=100000 tools/ppdiag.hip -o build/ppdiag
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "gemm_pp.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int BM, int BN, int WM, int WN, int CONV, int SCHED, int DIAG>
float run(GemmArgs p, int iters) {
  constexpr size_t lds = pp_lds_bytes<BM, BN, WM, WN, false>();
  auto* kfn = &gemm_pp_kernel<BM, BN, WM, WN, CONV, false, SCHED, DIAG>;
  CK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int nN = (p.N + BN - 1) / BN, nM = (p.M + BM - 1) / BM;
  dim3 grid(nN * nM, 1, 1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kfn, grid, dim3(512), lds, 0, p, nullptr);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(kfn, grid, dim3(512), lds, 0, p, nullptr);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / iters;
}

static uint16_t* rnd_bf16(size_t n, float scale, unsigned seed) {
  std::vector<uint16_t> h(n);
  unsigned s = seed;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    float f = (((s >> 8) & 0xFFFF) / 32768.0f - 1.0f) * scale;
    unsigned u;
    memcpy(&u, &f, 4);
    h[i] = (uint16_t)(u >> 16);
  }
  uint16_t* d;
  CK(hipMalloc(&d, n * 2));
  CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
  return d;
}

template <int BM, int BN, int WM, int WN, int CONV, int SCHED>
long long mismatches(GemmArgs p, size_t n_out) {
  // bitwise comparison of this schedule's output against SCHED 0 (same MFMA sequence per element)
  std::vector<uint16_t> a(n_out), b(n_out);
  run<BM, BN, WM, WN, CONV, 0, 0>(p, 1);
  CK(hipMemcpy(a.data(), p.C, n_out * 2, hipMemcpyDeviceToHost));
  CK(hipMemset(p.C, 0, n_out * 2));
  run<BM, BN, WM, WN, CONV, SCHED, 0>(p, 1);
  CK(hipMemcpy(b.data(), p.C, n_out * 2, hipMemcpyDeviceToHost));
  long long bad = 0;
  for (size_t i = 0; i < n_out; ++i) bad += a[i] != b[i];
  return bad;
}

template <int BM, int BN, int WM, int WN, int CONV, int SCHED>
void arms(const char* name, GemmArgs p, double flop, int iters) {
  const long long bad = mismatches<BM, BN, WM, WN, CONV, SCHED>(p, (size_t)p.M * p.N);
  float t[4];
  // interleaved rounds, median of 3
  std::vector<float> r[4];
  for (int k = 0; k < 3; ++k) {
    r[0].push_back(run<BM, BN, WM, WN, CONV, SCHED, 0>(p, iters));
    r[1].push_back(run<BM, BN, WM, WN, CONV, SCHED, 1>(p, iters));
    r[2].push_back(run<BM, BN, WM, WN, CONV, SCHED, 2>(p, iters));
    r[3].push_back(run<BM, BN, WM, WN, CONV, SCHED, 3>(p, iters));
  }
  for (int a = 0; a < 4; ++a) {
    std::vector<float> v = r[a];
    std::sort(v.begin(), v.end());
    t[a] = v[1];
  }
  printf("{\"case\": \"%s\", \"tile\": \"%dx%d\", \"sched\": %d, \"full_us\": %.1f, \"no_dma_us\": %.1f, "
         "\"no_barrier_us\": %.1f, \"neither_us\": %.1f, \"full_tflops\": %.1f, \"mismatch_vs_sched0\": %lld}\n",
         name, BM, BN, SCHED, t[0], t[1], t[2], t[3], flop / t[0] / 1e6, bad);
  fflush(stdout);
}

int main() {
  // SD-1.5 level-1 3x3 conv: [8,64,64,320] -> 320, K = 2880
  {
    const int B = 8, H = 64, C = 320;
    GemmArgs p;
    p.conv = 1;
    p.A = rnd_bf16((size_t)B * H * H * C, 1.f, 1);
    p.W = rnd_bf16((size_t)C * 9 * C, 0.02f, 2);
    uint16_t* out;
    CK(hipMalloc(&out, (size_t)B * H * H * C * 2));
    p.C = out;
    p.IH = H; p.IW = H; p.Cin = C; p.ksize = 3; p.Ho = H; p.Wo = H; p.N = C; p.Nw = C;
    p.M = B * H * H; p.K = 9 * C; p.lda = C; p.ldc = C; p.stride = 1; p.pad = 1;
    const double fl = 2.0 * p.M * p.N * p.K;
    for (int rep = 0; rep < 2; ++rep) {
      arms<256, 160, 4, 2, 2, 2>("conv64_320", p, fl, 20);
      arms<256, 128, 4, 2, 2, 2>("conv64_320", p, fl, 20);
      arms<256, 256, 4, 2, 2, 2>("conv64_320", p, fl, 20);
    }
  }
  {
    const int M = 4096, N = 4096, K = 4096;
    GemmArgs p;
    p.A = rnd_bf16((size_t)M * K, 1.f, 3);
    p.W = rnd_bf16((size_t)N * K, 0.02f, 4);
    uint16_t* out;
    CK(hipMalloc(&out, (size_t)M * N * 2));
    p.C = out;
    p.M = M; p.N = N; p.Nw = N; p.K = K; p.lda = K; p.ldc = N;
    const double fl = 2.0 * M * N * K;
    for (int rep = 0; rep < 2; ++rep) {
      arms<256, 256, 4, 2, 0, 2>("gemm4096", p, fl, 10);
      arms<256, 160, 4, 2, 0, 2>("gemm4096", p, fl, 10);
      arms<128, 256, 2, 4, 0, 2>("gemm4096", p, fl, 10);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
