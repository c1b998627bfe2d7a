// GroupNorm(+SiLU) for NHWC activations and LayerNorm.
//
// GroupNorm over NHWC: a group is Cg = C/G consecutive channels of every pixel, so the
// statistics are a strided reduction.  Three kernels, all 16-byte vectorised:
//   1. stats: grid (chunks, B), 256 threads = R row-lanes x T vector-lanes (T*VPT 8-channel
//      vectors cover a row); each thread keeps 4 rows of loads in flight and accumulates
//      per-channel sum / sum-of-squares in registers; the block reduces row-lanes and then the
//      Cg channels of each group in LDS and writes ONE (sum, sumsq) pair per (b, chunk, group).
//      Chunks are sized so B*chunks ~ 512 blocks: every CU streams (the per-channel, per-chunk
//      partials of v0 made the finalize pass read chunks*C floats per group, 5.7 us a call).
//   2. finalize: one wave per (b, group): lane-strided chunk partials, fp64 shuffle reduce ->
//      (mean, rstd).
//   3. apply: grid (row-blocks, B); each thread derives the scale/shift of its channels once
//      (gamma*rstd, beta - mean*gamma*rstd) and streams rows with no per-element index math
//      (v0 decoded row/batch with 64-bit divisions per vector: 2.9 TB/s).
// LayerNorm: T = 2..64 lanes per row (T*8*VPL >= D), 64/T rows per wave, row held in
// registers, two-pass mean/variance, xor-shuffle reductions inside the T-lane segment
// (v0 used one wave per row: 40 of 64 lanes busy at D = 320).
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int GN_THREADS = 256;
constexpr int GN_UNROLL = 4;

struct GnGeom { int V, VPT, T, R; };
GnGeom gn_geom(int C) {
  GnGeom g;
  g.V = C / 8;
  g.VPT = (g.V + GN_THREADS - 1) / GN_THREADS;
  g.T = (g.V + g.VPT - 1) / g.VPT;
  g.R = GN_THREADS / g.T;
  if (g.R < 1) g.R = 1;
  return g;
}

template <int VPT>
__global__ void __launch_bounds__(GN_THREADS) gn_stats_kernel(const uint16_t* __restrict__ x, float* __restrict__ part,
                                                              long long S, int C, int G, int T, int R, int chunks,
                                                              long long rows_per_chunk) {
  extern __shared__ float sh[];              // [2][R][C] row-lane partials, then [2][C] channel sums
  const int V = C / 8;
  const int tid = threadIdx.x;
  const int b = blockIdx.y, ck = blockIdx.x;
  const long long rbeg = (long long)ck * rows_per_chunk;
  const long long rend = min(S, rbeg + rows_per_chunk);
  const uint16_t* base = x + (long long)b * S * C;
  const int tv = tid % T, rl = tid / T;
  const bool active = rl < R;
  float s[VPT][8], q[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) { s[j][i] = 0.f; q[j][i] = 0.f; }
  if (active) {
    long long r = rbeg + rl;
    for (; r + (GN_UNROLL - 1) * R < rend; r += GN_UNROLL * R) {
      uint4 u[GN_UNROLL][VPT];
#pragma unroll
      for (int k = 0; k < GN_UNROLL; ++k)
#pragma unroll
        for (int j = 0; j < VPT; ++j) {
          const int v = tv + T * j;
          u[k][j] = v < V ? *reinterpret_cast<const uint4*>(base + (r + (long long)k * R) * C + v * 8) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
      for (int k = 0; k < GN_UNROLL; ++k)
#pragma unroll
        for (int j = 0; j < VPT; ++j) {
          float f[8];
          unpack8(u[k][j], f);
#pragma unroll
          for (int i = 0; i < 8; ++i) { s[j][i] += f[i]; q[j][i] = fmaf(f[i], f[i], q[j][i]); }
        }
    }
    for (; r < rend; r += R) {
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int v = tv + T * j;
        if (v >= V) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(base + r * C + v * 8), f);
#pragma unroll
        for (int i = 0; i < 8; ++i) { s[j][i] += f[i]; q[j][i] = fmaf(f[i], f[i], q[j][i]); }
      }
    }
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = tv + T * j;
      if (v >= V) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sh[(long long)rl * C + v * 8 + i] = s[j][i];
        sh[(long long)(R + rl) * C + v * 8 + i] = q[j][i];
      }
    }
  }
  __syncthreads();
  float* cs = sh + 2LL * R * C;              // [2][C]
  for (int c = tid; c < 2 * C; c += GN_THREADS) {
    const int stat = c / C, ch = c - stat * C;
    float acc = 0.f;
    for (int k = 0; k < R; ++k) acc += sh[(long long)(stat * R + k) * C + ch];
    cs[c] = acc;
  }
  __syncthreads();
  const int Cg = C / G;
  for (int j = tid; j < 2 * G; j += GN_THREADS) {
    const int stat = j / G, g = j - stat * G;
    float acc = 0.f;
    for (int c = 0; c < Cg; ++c) acc += cs[stat * C + g * Cg + c];
    part[(((long long)b * chunks + ck) * G + g) * 2 + stat] = acc;
  }
}

// one wave per (b, group): chunk partials summed in fp64 -> (mean, rstd)
__global__ void gn_finalize_kernel(const float* __restrict__ part, float* __restrict__ stats, long long S, int C,
                                   int G, int chunks, float eps) {
  const int g = blockIdx.x, b = blockIdx.y;
  const int lane = threadIdx.x;
  double sum = 0.0, sq = 0.0;
  for (int ck = lane; ck < chunks; ck += 64) {
    const float2 v = *reinterpret_cast<const float2*>(part + (((long long)b * chunks + ck) * G + g) * 2);
    sum += v.x;
    sq += v.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sum += __shfl_xor(sum, o, 64);
    sq += __shfl_xor(sq, o, 64);
  }
  if (lane == 0) {
    const double n = (double)S * (C / G);
    const double mean = sum / n;
    double var = sq / n - mean * mean;
    if (var < 0) var = 0;
    stats[((long long)b * G + g) * 2 + 0] = (float)mean;
    stats[((long long)b * G + g) * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

template <int VPT>
__global__ void __launch_bounds__(GN_THREADS) gn_apply_kernel(const uint16_t* __restrict__ x,
                                                              const float* __restrict__ stats,
                                                              const uint16_t* __restrict__ gamma,
                                                              const uint16_t* __restrict__ beta,
                                                              uint16_t* __restrict__ y, long long S, int C, int G,
                                                              int T, int R, long long rows_per_block, int silu) {
  const int V = C / 8;
  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const int tv = tid % T, rl = tid / T;
  if (rl >= R) return;
  const int Cg = C / G;
  float sc[VPT][8], sf[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int v = tv + T * j;
    if (v >= V) continue;
    float ga[8], be[8];
    unpack8(*reinterpret_cast<const uint4*>(gamma + v * 8), ga);
    unpack8(*reinterpret_cast<const uint4*>(beta + v * 8), be);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int g = (v * 8 + i) / Cg;
      const float2 ms = *reinterpret_cast<const float2*>(stats + ((long long)b * G + g) * 2);
      sc[j][i] = ga[i] * ms.y;
      sf[j][i] = be[i] - ms.x * sc[j][i];
    }
  }
  const long long rbeg = (long long)blockIdx.x * rows_per_block;
  const long long rend = min(S, rbeg + rows_per_block);
  const long long off = (long long)b * S * C;
  const uint16_t* xb = x + off;
  uint16_t* yb = y + off;
  auto emit = [&](long long r, int j, uint4 u) {
    float f[8];
    unpack8(u, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float o = fmaf(f[i], sc[j][i], sf[j][i]);
      f[i] = silu ? silu_f(o) : o;
    }
    *reinterpret_cast<uint4*>(yb + r * C + (tv + T * j) * 8) = pack8(f);
  };
  long long r = rbeg + rl;
  for (; r + (GN_UNROLL - 1) * R < rend; r += GN_UNROLL * R) {
    uint4 u[GN_UNROLL][VPT];
#pragma unroll
    for (int k = 0; k < GN_UNROLL; ++k)
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int v = tv + T * j;
        if (v < V) u[k][j] = *reinterpret_cast<const uint4*>(xb + (r + (long long)k * R) * C + v * 8);
      }
#pragma unroll
    for (int k = 0; k < GN_UNROLL; ++k)
#pragma unroll
      for (int j = 0; j < VPT; ++j)
        if (tv + T * j < V) emit(r + (long long)k * R, j, u[k][j]);
  }
  for (; r < rend; r += R)
#pragma unroll
    for (int j = 0; j < VPT; ++j)
      if (tv + T * j < V) emit(r, j, *reinterpret_cast<const uint4*>(xb + r * C + (tv + T * j) * 8));
}

// GroupNorm apply from producer-accumulated per-channel statistics (GEMM epilogue, p.stats):
// each block folds the Cg channel sums of every group of its image into (mean, rstd) in LDS
// (fp64), then streams rows.  A channel concatenation (UNet up-block skips) reads channels >= Ca
// from the second producer's statistics.
//
// Latency structure (round 4): these applies are short (2.6-21 MB) and were bound by three
// SERIAL memory round trips per block -- statistics fold, then gamma / beta, then the first rows
// -- not by bandwidth (0.5-5 TB/s, profiles/r3_membound_bandwidth.jsonl).  Now the block's first
// row group and gamma / beta are issued BEFORE the statistics loads, so the three latencies
// overlap, and the row loop is software-pipelined (the next row group's loads are issued before
// the current one is normalised and stored).
template <int VPT, int U>
__global__ void __launch_bounds__(GN_THREADS) gn_apply_cs_kernel(const uint16_t* __restrict__ x,
                                                                 const uint16_t* __restrict__ x2,
                                                                 const long long* __restrict__ sa, int Ca,
                                                                 const long long* __restrict__ sb,
                                                                 const uint16_t* __restrict__ gamma,
                                                                 const uint16_t* __restrict__ beta,
                                                                 uint16_t* __restrict__ y, long long S, int C,
                                                                 int G, int T, int R, long long rows_per_block,
                                                                 float eps, int silu) {
  extern __shared__ float gst[];           // [G][2] mean, rstd
  const int V = C / 8;
  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const int Cg = C / G;
  const int Cb = C - Ca;
  const int tv = tid % T, rl = tid / T;
  const bool act = rl < R;                 // row lanes beyond R only help with the fold
  const long long rbeg = (long long)blockIdx.x * rows_per_block;
  const long long rend = min(S, rbeg + rows_per_block);
  uint16_t* yb = y + (long long)b * S * C;
  // source of each of this thread's 8-channel vectors: the input itself, or for a channel
  // concatenation [x | x2] (UNet up-block skips, never materialised) x rows of Ca channels and
  // x2 rows of C - Ca channels (Ca % 8 == 0: a vector never straddles the two)
  const uint16_t* src[VPT];
  int lds_[VPT];
  bool von[VPT];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    von[j] = act && (tv + T * j) < V;
    const int c0 = (von[j] ? tv + T * j : 0) * 8;     // (idle lanes read a valid vector)
    if (x2 == nullptr) {
      src[j] = x + (long long)b * S * C + c0;
      lds_[j] = C;
    } else if (c0 < Ca) {
      src[j] = x + (long long)b * S * Ca + c0;
      lds_[j] = Ca;
    } else {
      src[j] = x2 + (long long)b * S * Cb + (c0 - Ca);
      lds_[j] = Cb;
    }
  }
  // ---- 1. the first row group and gamma / beta in flight before anything else
  uint4 u[U][VPT];
  long long r = rbeg + rl;
  // unconditional loads at clamped rows (a per-element "load or zero" select makes hipcc branch
  // around every load and wait for each in turn)
  auto load_group = [&](long long r0) {
#pragma unroll
    for (int k = 0; k < U; ++k)
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const long long rr = min(r0 + (long long)k * R, rend - 1);
        u[k][j] = *reinterpret_cast<const uint4*>(src[j] + rr * lds_[j]);
      }
  };
  load_group(r);
  uint4 gv[VPT], bv[VPT];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int v = von[j] ? tv + T * j : 0;
    gv[j] = *reinterpret_cast<const uint4*>(gamma + v * 8);
    bv[j] = *reinterpret_cast<const uint4*>(beta + v * 8);
  }
  // ---- 2. fold the Cg channel (sum, sumsq) pairs of every group with TPG threads per group (all
  // loads of a thread in flight together), exact int64 sums combined across the TPG lanes by
  // shuffles, then fp64 mean / rstd
  const int tpg = G >= GN_THREADS ? 1 : (GN_THREADS / G >= 8 ? 8 : (GN_THREADS / G >= 4 ? 4 : (GN_THREADS / G >= 2 ? 2 : 1)));
  for (int g0 = 0; g0 < G; g0 += GN_THREADS / tpg) {
    const int g = g0 + tid / tpg, sub = tid % tpg;
    long long si = 0, qi = 0;
    if (g < G) {
      const int c0 = g * Cg + sub, c1 = (g + 1) * Cg;
      longlong2 v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {          // unconditional loads (clamped index) ...
        const int c = min(c0 + q * tpg, c1 - 1);
        const long long* sp = c < Ca ? sa + ((long long)b * Ca + c) * 2 : sb + ((long long)b * Cb + (c - Ca)) * 2;
        v[q] = *reinterpret_cast<const longlong2*>(sp);
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {          // ... then the sums of the live ones
        const bool live = c0 + q * tpg < c1;
        si += live ? v[q].x : 0;
        qi += live ? v[q].y : 0;
      }
      for (int c = c0 + 16 * tpg; c < c1; c += tpg) {
        const long long* sp = c < Ca ? sa + ((long long)b * Ca + c) * 2 : sb + ((long long)b * Cb + (c - Ca)) * 2;
        const longlong2 vv = *reinterpret_cast<const longlong2*>(sp);
        si += vv.x;
        qi += vv.y;
      }
    }
    for (int o = 1; o < tpg; o <<= 1) {    // tpg lanes of a group are adjacent within one wave
      si += __shfl_xor(si, o, 64);
      qi += __shfl_xor(qi, o, 64);
    }
    if (g < G && sub == 0) {
      const double sm = stat_decode(si, 0), q = stat_decode(qi, 1);
      const double n = (double)S * Cg;
      const double mean = sm / n;
      double var = q / n - mean * mean;
      if (var < 0) var = 0;
      gst[2 * g] = (float)mean;
      gst[2 * g + 1] = (float)(1.0 / sqrt(var + (double)eps));
    }
  }
  __syncthreads();
  if (!act) return;
  float sc[VPT][8], sf[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int v = tv + T * j;
    float ga[8], be[8];
    unpack8(gv[j], ga);
    unpack8(bv[j], be);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int g = von[j] ? (v * 8 + i) / Cg : 0;
      sc[j][i] = ga[i] * gst[2 * g + 1];
      sf[j][i] = be[i] - gst[2 * g] * sc[j][i];
    }
  }
  auto emit = [&](long long rr, int j, uint4 w) {
    float f[8];
    unpack8(w, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float o = fmaf(f[i], sc[j][i], sf[j][i]);
      f[i] = silu ? silu_f(o) : o;
    }
#if GN_NT_STORE
    // (A/B knob) streaming store: no write-allocate in L2 / MALL for outputs larger than them
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_nt;
    const uint4 pk = pack8(f);
    __builtin_nontemporal_store(u32x4_nt{pk.x, pk.y, pk.z, pk.w}, reinterpret_cast<u32x4_nt*>(yb + rr * C + (tv + T * j) * 8));
#else
    *reinterpret_cast<uint4*>(yb + rr * C + (tv + T * j) * 8) = pack8(f);
#endif
  };
  // ---- 3. software-pipelined row loop: group i + 1 is in flight while group i is stored
  for (; r < rend; r += U * R) {
    uint4 cur[U][VPT];
#pragma unroll
    for (int k = 0; k < U; ++k)
#pragma unroll
      for (int j = 0; j < VPT; ++j) cur[k][j] = u[k][j];
    const long long rn = r + (long long)U * R;
    if (rn < rend) load_group(rn);
#pragma unroll
    for (int k = 0; k < U; ++k)
#pragma unroll
      for (int j = 0; j < VPT; ++j)
        if (von[j] && r + (long long)k * R < rend) emit(r + (long long)k * R, j, cur[k][j]);
  }
}

// per-channel sum / sum-of-squares of an NHWC tensor, atomically added into [B][C][2]
template <int VPT>
__global__ void __launch_bounds__(GN_THREADS) channel_stats_kernel(const uint16_t* __restrict__ x,
                                                                   long long* __restrict__ stats, long long S, int C,
                                                                   int T, int R, long long rows_per_chunk) {
  extern __shared__ float sh[];              // [2][R][C]
  const int V = C / 8;
  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const long long rbeg = (long long)blockIdx.x * rows_per_chunk;
  const long long rend = min(S, rbeg + rows_per_chunk);
  const uint16_t* base = x + (long long)b * S * C;
  const int tv = tid % T, rl = tid / T;
  float s[VPT][8], q[VPT][8];
#pragma unroll
  for (int j = 0; j < VPT; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) { s[j][i] = 0.f; q[j][i] = 0.f; }
  if (rl < R) {
    for (long long r = rbeg + rl; r < rend; r += R)
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int v = tv + T * j;
        if (v >= V) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(base + r * C + v * 8), f);
#pragma unroll
        for (int i = 0; i < 8; ++i) { s[j][i] += f[i]; q[j][i] = fmaf(f[i], f[i], q[j][i]); }
      }
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int v = tv + T * j;
      if (v >= V) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sh[(long long)rl * C + v * 8 + i] = s[j][i];
        sh[(long long)(R + rl) * C + v * 8 + i] = q[j][i];
      }
    }
  }
  __syncthreads();
  for (int c = tid; c < 2 * C; c += GN_THREADS) {
    const int stat = c / C, ch = c - stat * C;
    float acc = 0.f;
    for (int k = 0; k < R; ++k) acc += sh[(long long)(stat * R + k) * C + ch];
    stat_atomic_add(stats + ((long long)b * C + ch) * 2 + stat, stat, acc);
  }
}

// LayerNorm / RMSNorm (RMS: no mean subtraction, no beta): T lanes per row, VPL vectors per lane
// STATS: write only the row (mean, rstd) as float2 into y (LayerNorm folded into the next GEMM,
// whose epilogue applies them: no normalised copy of the activation is written or re-read)
// EMB: the row is the token-embedding sum of an encoder's input layer, gathered here instead of
// read from x: word[ids[row]] + pos[row % seq] + add (MiniLM / BERT: word + position + token
// type 0), so the scorer's embedding step is ONE kernel (gather + add + LayerNorm) instead of
// three ATen index/add launches plus the LayerNorm.
struct EmbArgs {
  const long long* ids = nullptr;     // [rows] token ids
  const uint16_t* pos = nullptr;      // [>= seq][D]
  const uint16_t* add = nullptr;      // [D] (nullable)
  int seq = 1;
};

template <int VPL, bool RMS, bool STATS = false, bool EMB = false>
__global__ void ln_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ gamma,
                          const uint16_t* __restrict__ beta, uint16_t* __restrict__ y,
                          long long rows, int D, int T, float eps, EmbArgs e = EmbArgs()) {
  const int lane = threadIdx.x & 63;
  const int seg = lane / T, sl = lane - seg * T;
  const int rows_per_wave = 64 / T;
  const long long row = ((long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * rows_per_wave + seg;
  const bool ok = row < rows;
  const int V = D / 8;
  const long long src_row = EMB ? (ok ? e.ids[row] : 0) : (ok ? row : 0);
  const uint4* xr = reinterpret_cast<const uint4*>(x + src_row * D);
  float f[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int v = sl + T * j;
    if (ok && v < V) {
      unpack8(xr[v], f[j]);
      if constexpr (EMB) {
        float a[8];
        unpack8(reinterpret_cast<const uint4*>(e.pos + (row % e.seq) * D)[v], a);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[j][k] = bf2f(f2bf(f[j][k] + a[k]));   // bf16 adds, as the
        if (e.add) {                                                         // eager model rounds
          unpack8(reinterpret_cast<const uint4*>(e.add)[v], a);
#pragma unroll
          for (int k = 0; k < 8; ++k) f[j][k] = bf2f(f2bf(f[j][k] + a[k]));
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += f[j][k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) f[j][k] = 0.f;
    }
  }
  // segment reductions: xor offsets < T stay inside the T-lane segment
  for (int o = T >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = RMS ? 0.f : s / D;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int v = sl + T * j;
    if (v < V) {
#pragma unroll
      for (int k = 0; k < 8; ++k) { const float t = f[j][k] - mean; ss = fmaf(t, t, ss); }
    }
  }
  for (int o = T >> 1; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float rstd = rsqrtf(ss / D + eps);
  if (!ok) return;
  if constexpr (STATS) {
    if (sl == 0) reinterpret_cast<float2*>(y)[row] = make_float2(mean, rstd);
    return;
  }
  uint4* yr = reinterpret_cast<uint4*>(y + row * D);
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int v = sl + T * j;
    if (v < V) {
      float g[8], bb[8];
      unpack8(reinterpret_cast<const uint4*>(gamma)[v], g);
      if (beta) unpack8(reinterpret_cast<const uint4*>(beta)[v], bb);
      else for (int k = 0; k < 8; ++k) bb[k] = 0.f;
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaf((f[j][k] - mean) * rstd, g[k], bb[k]);
      yr[v] = pack8(o);
    }
  }
}

int gn_chunks(int B, long long S, int R) {
  long long want = (512 + B - 1) / B;                      // ~2 blocks per CU in total
  long long maxc = (S + 4LL * R - 1) / (4LL * R);          // >= one unrolled row group per lane
  long long ch = want < maxc ? want : maxc;
  return (int)(ch < 1 ? 1 : ch);
}

}  // namespace

long long group_norm_workspace(int B, long long S, int C) {
  const GnGeom g = gn_geom(C);
  const int chunks = gn_chunks(B, S, g.R);
  return (long long)B * chunks * 2 * C + 2LL * B * C;   // floats (>= partials + stats for any G)
}

void launch_group_norm(const uint16_t* x, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                       float* ws, int B, long long S, int C, int G, float eps, int silu, hipStream_t s) {
  const GnGeom g = gn_geom(C);
  const int chunks = gn_chunks(B, S, g.R);
  const long long rpc = (S + chunks - 1) / chunks;
  float* part = ws;
  float* stats = ws + (long long)B * chunks * G * 2;
  const size_t shs = sizeof(float) * (2LL * g.R * C + 2LL * C);
  if (g.VPT == 1)
    hipLaunchKernelGGL(gn_stats_kernel<1>, dim3(chunks, B), dim3(GN_THREADS), shs, s, x, part, S, C, G, g.T, g.R,
                       chunks, rpc);
  else
    hipLaunchKernelGGL(gn_stats_kernel<2>, dim3(chunks, B), dim3(GN_THREADS), shs, s, x, part, S, C, G, g.T, g.R,
                       chunks, rpc);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(G, B), dim3(64), 0, s, part, stats, S, C, G, chunks, eps);
  // apply: ~8 rows per row-lane per block
  long long rpb = 2LL * GN_UNROLL * g.R;                   // whole GN_UNROLL-row iterations per thread
  long long nb = (S + rpb - 1) / rpb;
  if (nb * B < 2048) {                                     // small images: shorter blocks, more of them
    rpb = (long long)GN_UNROLL * g.R;
    nb = (S + rpb - 1) / rpb;
  }
  if (g.VPT == 1)
    hipLaunchKernelGGL(gn_apply_kernel<1>, dim3((unsigned)nb, B), dim3(GN_THREADS), 0, s, x, stats, gamma, beta, y, S,
                       C, G, g.T, g.R, rpb, silu);
  else
    hipLaunchKernelGGL(gn_apply_kernel<2>, dim3((unsigned)nb, B), dim3(GN_THREADS), 0, s, x, stats, gamma, beta, y, S,
                       C, G, g.T, g.R, rpb, silu);
}

// Apply geometry: 8-channel vectors per thread (VPT in {1, 2}) chosen for the most active threads
// of the 256 (V = 160 at C = 1280 left 96 idle at VPT 1), U rows per thread in flight, and
// ~GN_APPLY_BLOCKS blocks over the chip (the round-3 rule of >= 32 rows per block left ~2 blocks
// per CU at the 64^2 level).  Same-box A/B of the variants (profiles/r4_gn_apply_variants.txt):
// 64^2 x 320 16.8 -> 13.0 us, 32^2 x 1280 15.5 -> 14.7, the 16^2 / 8^2 applies unchanged; 8 rows
// per thread or 2048 blocks were slower on the small levels.
#ifndef GN_APPLY_GEOM
#define GN_APPLY_GEOM 1
#endif
// Output stores non-temporal (round 6, profiles/r6_gn_apply_variants.txt: 64^2 x 320 at batch 8
// 12.9 -> 11.3 us, the VAE 256^2 x 512 / 512^2 x 128 applies 114 / 111 -> 87 / 83 us = 6.2-6.5
// TB/s); GN_U8_RULE: 8 rows per thread in flight for 512..1024-channel tensors of >= 4096 rows
// per image (64^2 x 640 16.7 vs 18.4 us, the VAE 64^2 x 512 9.2 vs 11.4), 4 elsewhere (the
// small levels lose with 8)
#ifndef GN_NT_STORE
#define GN_NT_STORE 1
#endif
#ifndef GN_U8_RULE
#define GN_U8_RULE 1
#endif
#ifndef GN_APPLY_U
#define GN_APPLY_U 4
#endif
#ifndef GN_APPLY_BLOCKS
#define GN_APPLY_BLOCKS 1024
#endif
static GnGeom gn_apply_geom(int C) {
  GnGeom g = gn_geom(C);
  if (!GN_APPLY_GEOM) return g;
  int best = -1;
  for (int vpt = 1; vpt <= 2; vpt *= 2) {      // (VPT 4 measured 1.1-1.6x slower at C = 2560)
    const int T = (g.V + vpt - 1) / vpt;
    if (T > GN_THREADS) continue;
    const int R = GN_THREADS / T;
    const int active = R * T;
    if (active * 10 > best * 11) { best = active; g.VPT = vpt; g.T = T; g.R = R; }   // > 10 % more

  }
  return g;
}

template <int VPT, int U>
static void launch_apply(const uint16_t* x, const uint16_t* x2, const long long* stats_a, int Ca, const long long* stats_b,
                         const uint16_t* gamma, const uint16_t* beta, uint16_t* y, int B, long long S, int C, int G,
                         float eps, int silu, const GnGeom& g, hipStream_t s) {
  const long long step = (long long)U * g.R;                       // rows per block iteration
  long long rpb;
  if (GN_APPLY_GEOM) {
    // tensors of >= CASSMANTLE_GN_BIG_MB MiB may take CASSMANTLE_GN_BIG_BLOCKS blocks (A/B knob)
    static const int big_mb = [] { const char* e = getenv("CASSMANTLE_GN_BIG_MB"); return e ? atoi(e) : 0; }();
    static const int big_blocks = [] { const char* e = getenv("CASSMANTLE_GN_BIG_BLOCKS"); return e ? atoi(e) : GN_APPLY_BLOCKS; }();
    const bool big = big_mb > 0 && (long long)B * S * C * 2 >= ((long long)big_mb << 20);
    const long long blocks = big ? big_blocks : GN_APPLY_BLOCKS;
    const long long per_img = (blocks + B - 1) / B;
    const long long want = (S + per_img - 1) / per_img;
    rpb = step * ((want + step - 1) / step);
  } else {
    long long want = 32;
    if (want < (32LL << 10) / (2LL * C)) want = (32LL << 10) / (2LL * C);
    rpb = step * ((want + step - 1) / step);
    while (rpb > step && ((S + rpb - 1) / rpb) * B < 1024) rpb -= step;
    if (rpb == step && ((S + rpb - 1) / rpb) * B < 256) rpb = step / 2 >= g.R ? step / 2 : g.R;
  }
  const long long nb = (S + rpb - 1) / rpb;
  const size_t shs = sizeof(float) * 2 * G;
  hipLaunchKernelGGL((gn_apply_cs_kernel<VPT, U>), dim3((unsigned)nb, B), dim3(GN_THREADS), shs, s, x, x2, stats_a, Ca,
                     stats_b, gamma, beta, y, S, C, G, g.T, g.R, rpb, eps, silu);
}

void launch_group_norm_cs(const uint16_t* x, const uint16_t* x2, const long long* stats_a, int Ca, const long long* stats_b,
                          const uint16_t* gamma, const uint16_t* beta, uint16_t* y, int B, long long S, int C,
                          int G, float eps, int silu, hipStream_t s) {
  const GnGeom g = gn_apply_geom(C);
  if (stats_b == nullptr) Ca = C;
  // U rows per thread, at most 16 vector loads (VPT x U) in flight per thread
  constexpr int U = GN_APPLY_U;
  constexpr int U2 = U * 2 > 16 ? 8 : U, U4 = U * 4 > 16 ? 4 : U;
  if (GN_U8_RULE && C >= 512 && C <= 1024 && S >= 4096) {
    if (g.VPT == 1) launch_apply<1, 8>(x, x2, stats_a, Ca, stats_b, gamma, beta, y, B, S, C, G, eps, silu, g, s);
    else launch_apply<2, 8>(x, x2, stats_a, Ca, stats_b, gamma, beta, y, B, S, C, G, eps, silu, g, s);
    return;
  }
  if (g.VPT == 1) launch_apply<1, U>(x, x2, stats_a, Ca, stats_b, gamma, beta, y, B, S, C, G, eps, silu, g, s);
  else if (g.VPT == 2) launch_apply<2, U2>(x, x2, stats_a, Ca, stats_b, gamma, beta, y, B, S, C, G, eps, silu, g, s);
  else launch_apply<4, U4>(x, x2, stats_a, Ca, stats_b, gamma, beta, y, B, S, C, G, eps, silu, g, s);
}

void launch_channel_stats(const uint16_t* x, long long* stats, int B, long long S, int C, hipStream_t s) {
  const GnGeom g = gn_geom(C);
  const int chunks = gn_chunks(B, S, g.R);
  const long long rpc = (S + chunks - 1) / chunks;
  const size_t shs = sizeof(float) * 2LL * g.R * C;
  if (g.VPT == 1)
    hipLaunchKernelGGL(channel_stats_kernel<1>, dim3(chunks, B), dim3(GN_THREADS), shs, s, x, stats, S, C, g.T, g.R,
                       rpc);
  else
    hipLaunchKernelGGL(channel_stats_kernel<2>, dim3(chunks, B), dim3(GN_THREADS), shs, s, x, stats, S, C, g.T, g.R,
                       rpc);
}

template <int VPL, bool RMS, bool STATS, bool EMB>
static void launch_ln_t(const uint16_t* x, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                        long long rows, int D, int T, float eps, const EmbArgs& e, hipStream_t s) {
  const long long rows_per_block = 4LL * (64 / T);
  dim3 grid((unsigned)((rows + rows_per_block - 1) / rows_per_block));
  hipLaunchKernelGGL((ln_kernel<VPL, RMS, STATS, EMB>), grid, dim3(256), 0, s, x, gamma, beta, y, rows, D, T, eps, e);
}

template <bool RMS, bool STATS = false, bool EMB = false>
static void launch_ln(const uint16_t* x, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                      long long rows, int D, float eps, hipStream_t s, const EmbArgs& e = EmbArgs()) {
  const int V = D / 8;
  int T = 1;
  while (T < 64 && T * 8 < V) T <<= 1;                 // VPL <= 8 (D <= 4096)
  const int VPL = (V + T - 1) / T;
  switch (VPL) {
    case 1: launch_ln_t<1, RMS, STATS, EMB>(x, gamma, beta, y, rows, D, T, eps, e, s); break;
    case 2: launch_ln_t<2, RMS, STATS, EMB>(x, gamma, beta, y, rows, D, T, eps, e, s); break;
    case 3: launch_ln_t<3, RMS, STATS, EMB>(x, gamma, beta, y, rows, D, T, eps, e, s); break;
    case 4: launch_ln_t<4, RMS, STATS, EMB>(x, gamma, beta, y, rows, D, T, eps, e, s); break;
    case 5: launch_ln_t<5, RMS, STATS, EMB>(x, gamma, beta, y, rows, D, T, eps, e, s); break;
    case 6: launch_ln_t<6, RMS, STATS, EMB>(x, gamma, beta, y, rows, D, T, eps, e, s); break;
    case 7: launch_ln_t<7, RMS, STATS, EMB>(x, gamma, beta, y, rows, D, T, eps, e, s); break;
    default: launch_ln_t<8, RMS, STATS, EMB>(x, gamma, beta, y, rows, D, T, eps, e, s); break;
  }
}

void launch_embed_layer_norm(const uint16_t* word, const long long* ids, const uint16_t* pos, int seq,
                             const uint16_t* add, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                             long long rows, int D, float eps, hipStream_t s) {
  EmbArgs e;
  e.ids = ids; e.pos = pos; e.add = add; e.seq = seq;
  launch_ln<false, false, true>(word, gamma, beta, y, rows, D, eps, s, e);
}

void launch_row_stats(const uint16_t* x, float* stats, long long rows, int D, float eps, hipStream_t s) {
  launch_ln<false, true>(x, nullptr, nullptr, reinterpret_cast<uint16_t*>(stats), rows, D, eps, s);
}

void launch_layer_norm(const uint16_t* x, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                       long long rows, int D, float eps, hipStream_t s) {
  launch_ln<false>(x, gamma, beta, y, rows, D, eps, s);
}

void launch_rms_norm(const uint16_t* x, const uint16_t* gamma, uint16_t* y, long long rows, int D, float eps,
                     hipStream_t s) {
  launch_ln<true>(x, gamma, nullptr, y, rows, D, eps, s);
}
