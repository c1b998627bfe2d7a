// (round 6) What is the ~6 us "fixed" part of a small-grid GEMM launch made of?
// probe_small_gemm.py fits the 128x80 producer-wave tile (256 blocks x 1024 threads, 106 KiB of
// dynamic LDS) as ~6 us per launch + 0.40 us per 64-deep k-tile.  This probe times, inside a
// replayed hipGraph of 200 back-to-back launches (the serving path), kernels that do nothing
// but what every GEMM launch does regardless of K:
//   empty : no memory traffic
//   touch : every thread loads 16 B of a 64 MiB source and stores 16 B (first-touch ramp, the
//           shape of a k-tile's first DMA + the epilogue store), source rotated per launch
// over grid {256, 512, 1024} blocks x block {256, 512, 1024} threads x dynamic LDS {0, 64 KiB,
// 104 KiB, 156 KiB}.  Output: one JSON line per case, us per launch (graph replay).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_cost_probe.hip -o tools/bin/launch_cost_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void empty_kernel(int* sink) {
  extern __shared__ int lds[];
  (void)lds;
  (void)sink;
}

__global__ void touch_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, long long n, long long off) {
  extern __shared__ int lds[];
  (void)lds;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long j = (i + off) % n;
  dst[i] = src[j];
}

static double time_graph(hipStream_t s, int launches, int replays, void (*enq)(hipStream_t, int, void*), void* ctx) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < launches; ++i) enq(s, i, ctx);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));   // warm-up
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  for (int r = 0; r < replays; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 1000.0 * ms / ((double)launches * replays);
}

struct Ctx {
  int blocks, threads;
  size_t lds;
  int* sink;
  const uint4* src;
  uint4* dst;
  long long n;
};

static void enq_empty(hipStream_t s, int, void* p) {
  Ctx* c = (Ctx*)p;
  hipLaunchKernelGGL(empty_kernel, dim3(c->blocks), dim3(c->threads), c->lds, s, c->sink);
}

static void enq_touch(hipStream_t s, int i, void* p) {
  Ctx* c = (Ctx*)p;
  const long long per = (long long)c->blocks * c->threads;
  hipLaunchKernelGGL(touch_kernel, dim3(c->blocks), dim3(c->threads), c->lds, s, c->src, c->dst, c->n,
                     (long long)i * per * 7 % c->n);
}

int main() {
  CK(hipFuncSetAttribute((const void*)empty_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)touch_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const long long n = (64ll << 20) / 16;
  uint4 *src, *dst;
  int* sink;
  CK(hipMalloc(&src, n * 16));
  CK(hipMalloc(&dst, 1024ll * 1024 * 16));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(src, 1, n * 16));
  const int grids[] = {256, 512, 1024};
  const int blocks_t[] = {256, 512, 1024};
  const size_t ldss[] = {0, 64 * 1024, 104 * 1024, 156 * 1024};
  for (int gi = 0; gi < 3; ++gi)
    for (int ti = 0; ti < 3; ++ti)
      for (int li = 0; li < 4; ++li) {
        Ctx c{grids[gi], blocks_t[ti], ldss[li], sink, src, dst, n};
        const double e = time_graph(s, 200, 10, enq_empty, &c);
        const double t = time_graph(s, 200, 10, enq_touch, &c);
        printf("{\"blocks\": %d, \"threads\": %d, \"lds_kib\": %zu, \"empty_us\": %.2f, \"touch_us\": %.2f}\n",
               c.blocks, c.threads, c.lds / 1024, e, t);
        fflush(stdout);
      }
  CK(hipFree(src));
  CK(hipFree(dst));
  CK(hipFree(sink));
  CK(hipStreamDestroy(s));
  return 0;
}
