// L2 -> LDS fill-rate probe: how many bytes per cycle can one CU stream into LDS by LDS-DMA
// (buffer_load_dwordx4 ... lds), and does it depend on waves per CU or on DMAs in flight?
//
// Every GEMM tile in this repo moves ~20-22 B/cycle/CU (profiles/r3_dma_bound.txt) and the
// latency-bound level-3 GEMMs (M 2048, N 1280, K 1280) take ~0.5 us per 64-deep k-tile while their
// MFMAs need ~0.15: if ~22 B/cycle/CU is the fill ceiling, those GEMMs sit at their floor.
//
// Kernel: one workgroup per CU (grid = 256 x REP), WAVES waves; each wave streams 1 KiB pieces
// (64 lanes x 16 B) of an L2/MALL-resident source window into a private LDS ring of DEPTH pieces,
// keeping DEPTH - 1 in flight (counted vmcnt), for ITERS pieces.  No compute.  Reports B/cycle/CU
// from wall time and the shader clock read by s_memtime (median over workgroups).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lds_fill_probe.hip -o /tmp/lds_fill_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int WAVES, int DEPTH, bool ROWS>
__global__ void __launch_bounds__(64 * WAVES, 1) fill(const uint4* __restrict__ src, long long window_bytes, int iters,
                                                      long long* __restrict__ cyc) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(src), (short)0, (int)window_bytes, 0x00020000);
  // each workgroup streams its own window slice (distinct lines per CU, L2/MALL-resident overall)
  const long long slice = window_bytes / gridDim.x;
  const int base = (int)(blockIdx.x * slice) & ~1023;
  const int pieces = (int)(slice / 1024);
  uint4* ring = lds + wave * DEPTH * 64;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  int p = wave;
#pragma unroll 1
  for (int i = 0; i < iters; ++i) {
    // ROWS: a GEMM tile's access pattern: one piece = 8 rows x 128 B (64 bf16 of K) of a
    // row-major [rows, 1280] bf16 matrix (2560 B row stride), k-chunks of a row block in order
    const int q = ROWS ? p % (pieces / 20 * 20) : p % pieces;
    const int off = ROWS ? base + ((q / 20) * 8 + (lane >> 3)) * 2560 + (q % 20) * 128 + (lane & 7) * 16
                         : base + q * 1024 + lane * 16;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(ring + (i % DEPTH) * 64), 16, off, 0, 0, 0);
    wait_vm<DEPTH - 1>();
    p += WAVES;
  }
  wait_vm<0>();
  __syncthreads();
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int WAVES, int DEPTH, bool ROWS = false>
void run(const uint4* src, long long window, long long* d_cyc, int nblk) {
  const int iters = 4096;
  auto* k = &fill<WAVES, DEPTH, ROWS>;
  const size_t lds = (size_t)WAVES * DEPTH * 1024;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(nblk), dim3(64 * WAVES), lds, 0, src, window, iters, d_cyc);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(nblk), dim3(64 * WAVES), lds, 0, src, window, iters, d_cyc);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<long long> cyc(nblk);
  CK(hipMemcpy(cyc.data(), d_cyc, nblk * sizeof(long long), hipMemcpyDeviceToHost));
  std::sort(cyc.begin(), cyc.end());
  const double bytes_per_wg = (double)WAVES * iters * 1024;
  const double med = (double)cyc[nblk / 2];
  printf("{\"access\": \"%s\", \"waves\": %d, \"depth\": %d, \"in_flight_kib_per_cu\": %d, \"window_mib\": %.0f, \"B_per_cycle_per_cu\": %.1f, "
         "\"chip_TBps\": %.2f}\n",
         ROWS ? "8x128B-rows" : "1KiB-contiguous", WAVES, DEPTH, WAVES * (DEPTH - 1), window / 1048576.0, bytes_per_wg / med,
         bytes_per_wg * nblk * reps / (ms * 1e-3) / 1e12);
}

int main() {
  const int nblk = 256;
  const long long window = 64LL << 20;   // 64 MiB: fits the 256 MiB Infinity Cache, 2x the L2s
  uint4* src;
  long long* d_cyc;
  CK(hipMalloc(&src, window));
  CK(hipMemset(src, 1, window));
  CK(hipMalloc(&d_cyc, nblk * sizeof(long long)));
  run<1, 8>(src, window, d_cyc, nblk);
  run<4, 4>(src, window, d_cyc, nblk);
  run<16, 8>(src, window, d_cyc, nblk);
  const long long small = 8LL << 20;     // 8 MiB: L2-resident (4 MiB per XCD, 32 CUs each)
  run<1, 2>(src, small, d_cyc, nblk);
  run<1, 4>(src, small, d_cyc, nblk);
  run<1, 8>(src, small, d_cyc, nblk);
  run<1, 16>(src, small, d_cyc, nblk);
  run<2, 8>(src, small, d_cyc, nblk);
  run<4, 2>(src, small, d_cyc, nblk);
  run<4, 4>(src, small, d_cyc, nblk);
  run<4, 8>(src, small, d_cyc, nblk);
  run<4, 16>(src, small, d_cyc, nblk);
  run<8, 4>(src, small, d_cyc, nblk);
  run<8, 8>(src, small, d_cyc, nblk);
  run<16, 8>(src, small, d_cyc, nblk);
  run<4, 4, true>(src, small, d_cyc, nblk);
  run<4, 8, true>(src, small, d_cyc, nblk);
  run<8, 8, true>(src, small, d_cyc, nblk);
  run<16, 8, true>(src, small, d_cyc, nblk);
  CK(hipFree(src));
  CK(hipFree(d_cyc));
  return 0;
}
