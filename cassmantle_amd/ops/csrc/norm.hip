// GroupNorm(+SiLU) for NHWC activations and LayerNorm.
//
// GroupNorm over NHWC: a group is Cg = C/G consecutive channels of every pixel, so the
// statistics are a strided reduction.  Three small kernels, all 16-byte vectorised:
//   1. partial sums: grid (B, chunks); each thread owns ONE 8-channel vector position of the
//      row (blockDim = multiple of C/8) and walks rows -> per-channel sum / sum-of-squares in
//      registers, reduced across the block's row-lanes in LDS; per-(b, chunk, channel) partials
//      go to a small fp32 workspace.  Chunks are sized so B*chunks fills all 256 CUs even for
//      the 512x512 VAE levels.
//   2. finalize: per (b, group) combine partials in fp64 -> per-(b, channel) scale/shift
//      (gamma*rstd, beta - mean*gamma*rstd).
//   3. apply: y = x*scale + shift (+ SiLU) streamed at HBM rate.
// LayerNorm: one wave per row, the row held in registers (two-pass mean/variance).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int GN_THREADS = 256;

template <int VPT>
__global__ void gn_partial_kernel(const uint16_t* __restrict__ x, float* __restrict__ part,
                                  long long S, int C, int chunks, long long rows_per_chunk) {
  extern __shared__ float sh[];              // [16][GN_THREADS] (row-lane reduction)
  const int V = C / 8;                       // 8-channel vectors per row
  const int tid = threadIdx.x;
  const int b = blockIdx.y, ck = blockIdx.x;
  const long long rbeg = (long long)ck * rows_per_chunk;
  const long long rend = min(S, rbeg + rows_per_chunk);
  const uint16_t* base = x + ((long long)b * S) * C;
  if (VPT > 1 || V > GN_THREADS / 2) {
    // wide rows: each thread owns whole vector columns, no cross-thread reduction
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = tid + GN_THREADS * j;
      if (v >= V) continue;
      float s[8], ss[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] = 0.f; ss[i] = 0.f; }
      for (long long r = rbeg; r < rend; ++r) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(base + r * C + v * 8), f);
#pragma unroll
        for (int i = 0; i < 8; ++i) { s[i] += f[i]; ss[i] = fmaf(f[i], f[i], ss[i]); }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        part[(((long long)b * chunks + ck) * 2 + 0) * C + v * 8 + i] = s[i];
        part[(((long long)b * chunks + ck) * 2 + 1) * C + v * 8 + i] = ss[i];
      }
    }
    return;
  }
  const int R = GN_THREADS / V;              // row lanes sharing a vector column
  const bool active = tid < R * V;
  const int v = tid % V, r0 = tid / V;
  float s[8], ss[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = 0.f; ss[i] = 0.f; }
  if (active) {
    for (long long r = rbeg + r0; r < rend; r += R) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(base + r * C + v * 8), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] += f[i]; ss[i] = fmaf(f[i], f[i], ss[i]); }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sh[i * GN_THREADS + tid] = active ? s[i] : 0.f;
    sh[(8 + i) * GN_THREADS + tid] = active ? ss[i] : 0.f;
  }
  __syncthreads();
  for (int job = tid; job < V * 16; job += GN_THREADS) {
    const int vv = job % V, comp = job / V;  // comp = stat*8 + i
    float acc = 0.f;
    for (int rr = 0; rr < R; ++rr) acc += sh[comp * GN_THREADS + rr * V + vv];
    const int stat = comp / 8, i = comp % 8;
    part[(((long long)b * chunks + ck) * 2 + stat) * C + vv * 8 + i] = acc;
  }
}

// one 64-thread block per (b, group): the chunks x Cg partials are summed in fp64 across lanes
__global__ void gn_finalize_kernel(const float* __restrict__ part, const uint16_t* __restrict__ gamma,
                                   const uint16_t* __restrict__ beta, float* __restrict__ scale,
                                   float* __restrict__ shift, long long S, int C, int G, int chunks, float eps) {
  const int g = blockIdx.x, b = blockIdx.y;
  const int Cg = C / G;
  const int lane = threadIdx.x;
  double sum = 0.0, sq = 0.0;
  for (int j = lane; j < chunks * Cg; j += 64) {
    const int ck = j / Cg, c = j - ck * Cg;
    const int ch = g * Cg + c;
    sum += part[(((long long)b * chunks + ck) * 2 + 0) * C + ch];
    sq += part[(((long long)b * chunks + ck) * 2 + 1) * C + ch];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sum += __shfl_xor(sum, o, 64);
    sq += __shfl_xor(sq, o, 64);
  }
  const double n = (double)S * Cg;
  const double mean = sum / n;
  double var = sq / n - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  for (int c = lane; c < Cg; c += 64) {
    const int ch = g * Cg + c;
    const float ga = bf2f(gamma[ch]), be = bf2f(beta[ch]);
    scale[b * C + ch] = ga * rstd;
    shift[b * C + ch] = be - (float)mean * ga * rstd;
  }
}

__global__ void gn_apply_kernel(const uint16_t* __restrict__ x, const float* __restrict__ scale,
                                const float* __restrict__ shift, uint16_t* __restrict__ y,
                                long long S, int C, int B, int silu) {
  const long long nvec = (long long)B * S * C / 8;
  const int V = C / 8;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (long long)gridDim.x * blockDim.x) {
    long long row = i / V;
    int v = (int)(i - row * V);
    int b = (int)(row / S);
    uint4 u = reinterpret_cast<const uint4*>(x)[i];
    float f[8];
    unpack8(u, f);
    const float4* sc = reinterpret_cast<const float4*>(scale + (long long)b * C + v * 8);
    const float4* sh = reinterpret_cast<const float4*>(shift + (long long)b * C + v * 8);
    float4 s0 = sc[0], s1 = sc[1], h0 = sh[0], h1 = sh[1];
    float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float o = fmaf(f[k], sv[k], hv[k]);
      f[k] = silu ? silu_f(o) : o;
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
}

// LayerNorm / RMSNorm (RMS: no mean subtraction, no beta): one wave per row; D <= 64*8*MAXV
template <int MAXV, bool RMS>
__global__ void ln_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ gamma,
                          const uint16_t* __restrict__ beta, uint16_t* __restrict__ y,
                          long long rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int V = D / 8;
  const uint4* xr = reinterpret_cast<const uint4*>(x + row * D);
  float f[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int v = lane + 64 * j;
    if (v < V) {
      unpack8(xr[v], f[j]);
#pragma unroll
      for (int k = 0; k < 8; ++k) s += f[j][k];
    }
  }
  const float mean = RMS ? 0.f : wave_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int v = lane + 64 * j;
    if (v < V) {
#pragma unroll
      for (int k = 0; k < 8; ++k) { float t = f[j][k] - mean; ss = fmaf(t, t, ss); }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / D + eps);
  uint4* yr = reinterpret_cast<uint4*>(y + row * D);
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    int v = lane + 64 * j;
    if (v < V) {
      uint4 gu = reinterpret_cast<const uint4*>(gamma)[v];
      float g[8], bb[8];
      unpack8(gu, g);
      if (beta) unpack8(reinterpret_cast<const uint4*>(beta)[v], bb);
      else for (int k = 0; k < 8; ++k) bb[k] = 0.f;
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaf((f[j][k] - mean) * rstd, g[k], bb[k]);
      yr[v] = pack8(o);
    }
  }
}

int gn_chunks(int B, long long S) {
  long long want = (1024 + B - 1) / B;             // ~4 blocks per CU in total
  long long maxc = (S + 63) / 64;                  // at least 64 rows per chunk
  long long ch = want < maxc ? want : maxc;
  return (int)(ch < 1 ? 1 : ch);
}

}  // namespace

long long group_norm_workspace(int B, long long S, int C) {
  int chunks = gn_chunks(B, S);
  return (long long)B * chunks * 2 * C + 2LL * B * C;   // floats
}

void launch_group_norm(const uint16_t* x, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                       float* ws, int B, long long S, int C, int G, float eps, int silu, hipStream_t s) {
  const int chunks = gn_chunks(B, S);
  const long long rpc = (S + chunks - 1) / chunks;
  float* part = ws;
  float* scale = ws + (long long)B * chunks * 2 * C;
  float* shift = scale + (long long)B * C;
  const int V = C / 8;
  dim3 g1(chunks, B);
  size_t sh = sizeof(float) * 16 * GN_THREADS;
  if (V <= GN_THREADS)
    hipLaunchKernelGGL(gn_partial_kernel<1>, g1, dim3(GN_THREADS), sh, s, x, part, S, C, chunks, rpc);
  else
    hipLaunchKernelGGL(gn_partial_kernel<2>, g1, dim3(GN_THREADS), sh, s, x, part, S, C, chunks, rpc);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(G, B), dim3(64), 0, s, part, gamma, beta, scale, shift, S, C, G, chunks, eps);
  long long nvec = (long long)B * S * C / 8;
  long long blocks = (nvec + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gn_apply_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, scale, shift, y, S, C, B, silu);
}

template <bool RMS>
static void launch_ln(const uint16_t* x, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                      long long rows, int D, float eps, hipStream_t s) {
  const int V = D / 8;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (V <= 64) hipLaunchKernelGGL((ln_kernel<1, RMS>), grid, dim3(256), 0, s, x, gamma, beta, y, rows, D, eps);
  else if (V <= 128) hipLaunchKernelGGL((ln_kernel<2, RMS>), grid, dim3(256), 0, s, x, gamma, beta, y, rows, D, eps);
  else if (V <= 256) hipLaunchKernelGGL((ln_kernel<4, RMS>), grid, dim3(256), 0, s, x, gamma, beta, y, rows, D, eps);
  else hipLaunchKernelGGL((ln_kernel<8, RMS>), grid, dim3(256), 0, s, x, gamma, beta, y, rows, D, eps);
}

void launch_layer_norm(const uint16_t* x, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                       long long rows, int D, float eps, hipStream_t s) {
  launch_ln<false>(x, gamma, beta, y, rows, D, eps, s);
}

void launch_rms_norm(const uint16_t* x, const uint16_t* gamma, uint16_t* y, long long rows, int D, float eps,
                     hipStream_t s) {
  launch_ln<true>(x, gamma, nullptr, y, rows, D, eps, s);
}
