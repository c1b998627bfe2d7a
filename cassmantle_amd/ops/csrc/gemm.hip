// MFMA GEMM / implicit-GEMM conv: tile planner and dispatch (kernels: gemm_impl.h, instantiated
// per A-operand mode in gemm_c*.hip).
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

void gemm_c0_buf_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c0_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c1_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c2_buf_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c2_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c3_launch(const GemmArgs& p, float* ws, hipStream_t s);

namespace {

constexpr int BK = 64;

// Tile menu.  4 waves, 2 blocks per CU by LDS, 2 stages:
//   0: 128x128 (2x2)   1: 128x160 (2x2, wave 80x64)   2: 256x64 (4x1)   3: 128x64 (2x2)   4: 256x16 (4x1)
// 8 waves, 1 block per CU, 3-stage ring:
//   5: 256x160 (4x2, wave 64x80)   6: 256x128 (4x2, wave 64x64)
struct TileCfg { int BM, BN; float eff; int slots; };
constexpr int kNumTiles = 7;
// slots = resident blocks on the chip: 128x64 needs 48 KiB of LDS per block, so 3 blocks fit a
// CU (768 slots); with 512 the model undercounted it and missed the measured best on the
// level-2..4 plain GEMMs (profiles/r1_gemm_plan_sweep.jsonl: 14.5 vs 17.8 us at 8192x640x640)
constexpr TileCfg kTiles[kNumTiles] = {{128, 128, 1.00f, 512}, {128, 160, 1.02f, 512}, {256, 64, 0.95f, 512},
                                       {128, 64, 0.80f, 768},  {256, 16, 0.25f, 512},  {256, 160, 1.02f, 256},
                                       {256, 128, 1.00f, 256}};

// buffer-resource LDS-DMA path: K in whole k-tiles and every byte range addressable by a
// 31-bit buffer offset (num_records), plain GEMMs and Cin % 64 convolutions without upsample
bool buf_ok(const GemmArgs& p) {
  static int force = -1;
  if (force < 0) {
    const char* e = getenv("CASSMANTLE_GEMM_BUF");
    force = e ? atoi(e) : 1;
  }
  if (p.A2 != nullptr) return true;   // two-source A exists only on this path (host-checked sizes)
  if (!force || p.K % BK != 0) return false;
  const long long ldw = p.ldw ? p.ldw : p.K;
  const long long lim = (1LL << 31) - 1;
  if (((long long)(p.Nw - 1) * ldw + p.K) * 2 > lim) return false;
  if (!p.conv) return ((long long)(p.M - 1) * p.lda + p.K) * 2 <= lim;
  if (p.upsample || p.Cin % 64 != 0) return false;
  const long long bias = ((long long)p.pad * p.IW + p.pad) * p.Cin * 2;
  return (long long)p.M / (p.Ho * p.Wo) * p.IH * p.IW * p.Cin * 2 + bias <= lim;
}

// SIMT fallback for shapes the MFMA path does not take (K % 8 != 0 linear layers: the
// 4 -> 4 post_quant_conv).  One thread per output element.
template <int CONV>
__global__ void gemm_simt_kernel(GemmArgs p) {
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)p.M * p.N;
  if (idx >= total) return;
  int m = (int)(idx / p.N), n = (int)(idx - (long long)m * p.N);
  const int batch = blockIdx.z;
  const uint16_t* A = p.A + (long long)batch * p.sA;
  const uint16_t* W = p.W + (long long)batch * p.sW + (long long)n * (p.ldw ? p.ldw : p.K);
  float s = 0.f;
  if constexpr (CONV == 0) {
    const uint16_t* a = A + (long long)m * p.lda;
    for (int k = 0; k < p.K; ++k) s += bf2f(a[k]) * bf2f(W[k]);
  } else {
    int hw = p.Ho * p.Wo;
    int b = m / hw, r = m - b * hw, oy = r / p.Wo, ox = r - oy * p.Wo;
    int Hv = p.upsample ? 2 * p.IH : p.IH, Wv = p.upsample ? 2 * p.IW : p.IW;
    for (int ky = 0; ky < p.ksize; ++ky) {
      int iy = oy * p.stride - p.pad + ky;
      if (iy < 0 || iy >= Hv) continue;
      for (int kx = 0; kx < p.ksize; ++kx) {
        int ix = ox * p.stride - p.pad + kx;
        if (ix < 0 || ix >= Wv) continue;
        int sy = p.upsample ? iy >> 1 : iy, sx = p.upsample ? ix >> 1 : ix;
        const uint16_t* a = A + (((long long)b * p.IH + sy) * p.IW + sx) * p.Cin;
        const uint16_t* w = W + (ky * p.ksize + kx) * p.Cin;
        for (int c = 0; c < p.Cin; ++c) s += bf2f(a[c]) * bf2f(w[c]);
      }
    }
  }
  float o = s * p.alpha;
  if (p.bias) o += bf2f(p.bias[n]);
  if (p.chan_bias) o += bf2f(p.chan_bias[(long long)(m / (p.Ho * p.Wo)) * (p.ldcb ? p.ldcb : p.N) + n]);
  o = apply_act(o, p.act);
  if (p.residual) o += bf2f(p.residual[(long long)m * p.ldc + n]);
  if (p.out_f32)
    reinterpret_cast<float*>(p.C)[(long long)batch * p.sC + (long long)m * p.ldc + n] = o;
  else
    reinterpret_cast<uint16_t*>(p.C)[(long long)batch * p.sC + (long long)m * p.ldc + n] = f2bf(o);
}

}  // namespace

// Choose tile config + split-K by an occupancy-round cost model: the kernel is latency-bound
// per k-tile, so time ~ rounds(blocks / 512) x k-tiles-per-block x tile-cost; split-K adds a
// reduction pass over split x M x N fp32.  Wave quantisation (e.g. 640 blocks = 1.25 rounds)
// was the single largest loss on the SD shapes (M = 32768 / 8192 / 2048 / 512).
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// A/B knobs for the microbenchmark / tile sweeps: CASSMANTLE_GEMM_CFG=<tile index>,
// CASSMANTLE_GEMM_SPLIT=<k slices>, or at run time gemm_set_override (tools/sweep_gemm.py)
static int g_force_cfg = -2, g_force_split = 0;   // -2: not yet read from the environment
void gemm_set_override(int cfg, int split) {
  g_force_cfg = cfg;
  g_force_split = split;
}

GemmPlan gemm_plan(const GemmArgs& p) {
  GemmPlan best{0, 1};
  if (g_force_cfg == -2) {
    g_force_cfg = env_int("CASSMANTLE_GEMM_CFG", -1);
    g_force_split = env_int("CASSMANTLE_GEMM_SPLIT", 0);
  }
  const int force_cfg = g_force_cfg, force_split = g_force_split;
  static const int use_big = env_int("CASSMANTLE_GEMM_8WAVE", 0);
  const bool gated = p.act == ACT_GEGLU || p.act == ACT_SWIGLU;
  int only = -1;                         // forced tile (cost model still picks the split)
  if (force_cfg >= 0 && force_cfg < kNumTiles && ((force_cfg == 4) == (p.N <= 16))) {
    if (gated) {
      if (force_cfg == 0 || force_cfg == 6) best.cfg = force_cfg;
      return best;
    }
    only = force_cfg;
  }
  if (gated) return best;
  const int nk = (p.K + BK - 1) / BK;
  // M <= 8 goes to the GEMV path; short prompts (M = tens of rows) need split-K to fill the chip
  const bool can_split = p.batch == 1 && p.N % 4 == 0 && p.K % 8 == 0 && p.M > 8;
  double best_t = 1e30;
  for (int c = 0; c < kNumTiles; ++c) {
    const TileCfg& tc = kTiles[c];
    if (only >= 0 ? c != only : (c >= 5 && !use_big)) continue;
    if (c == 4 && p.N > 16) continue;
    if (c != 4 && p.N <= 16) continue;
    const long long tiles = (long long)((p.N + tc.BN - 1) / tc.BN) * ((p.M + tc.BM - 1) / tc.BM) * p.batch;
    const double waste = (double)tc.BN * ((p.N + tc.BN - 1) / tc.BN) / p.N;   // padded columns
    for (int split = 1; split <= GEMM_MAX_SPLIT; ++split) {
      if (split > 1 && (!can_split || nk / split < 4)) break;
      const long long blocks = tiles * split;
      const long long rounds = (blocks + tc.slots - 1) / tc.slots;
      const int kper = (nk + split - 1) / split;
      // per-k-tile cost: fixed latency part + size part (normalised to a 128x128 tile)
      const double tile_cost = (0.55 + 0.45 * (tc.BM * tc.BN) / 16384.0) / tc.eff;
      // calibrated on MI355X: ~1.8 us per 128x128x64 k-tile per occupancy round (2 blocks/CU)
      double t = 1.8 * rounds * (kper + 2) * tile_cost * (waste > 1.3 ? waste : 1.0);
      // split-K: slab write + read at ~3 TB/s plus the extra reduce launch (~6 us in a graph)
      if (split > 1) t += 6.0 + 2.0 * (double)split * p.M * p.N * 4 / 3.0e6;
      if (only >= 0 && force_split > 0 && split != force_split) continue;
      if (t < best_t - 1e-9) { best_t = t; best = GemmPlan{c, split}; }
    }
  }
  return best;
}

int gemm_plan_split(const GemmArgs& p) { return gemm_plan(p).split; }

void launch_gemm(const GemmArgs& p, float* ws, hipStream_t s) {
  const bool mfma_ok = (p.K % 8 == 0) && (!p.conv || p.Cin % 8 == 0) &&
                       (p.conv || p.lda % 8 == 0) && (p.ldw % 8 == 0);
  // skinny M (decode tokens, time-embedding / pooled projections): a weight-streaming GEMV
  if (launch_gemv(p, s)) return;
  if (!mfma_ok) {
    if (p.act == ACT_GEGLU || p.act == ACT_SWIGLU) return;  // host guarantees gated shapes are MFMA-able
    long long total = (long long)p.M * p.N;
    dim3 grid((unsigned)((total + 255) / 256), 1, p.batch);
    if (p.conv)
      hipLaunchKernelGGL(gemm_simt_kernel<1>, grid, dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL(gemm_simt_kernel<0>, grid, dim3(256), 0, s, p);
    return;
  }
  const bool buf = buf_ok(p);
  if (!p.conv) {
    if (buf) gemm_c0_buf_launch(p, ws, s);
    else gemm_c0_launch(p, ws, s);
  } else if (p.Cin % 64 == 0) {
    if (p.upsample) gemm_c3_launch(p, ws, s);
    else if (buf) gemm_c2_buf_launch(p, ws, s);
    else gemm_c2_launch(p, ws, s);
  } else {
    gemm_c1_launch(p, ws, s);
  }
}
