// MFMA GEMM / implicit-GEMM conv: tile planner and dispatch (kernels: gemm_impl.h, instantiated
// per A-operand mode in gemm_c*.hip).
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>

#include "common.h"
#include "kernels.h"

void gemm_c0_buf_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c0_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c1_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c2_buf_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c2_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_c3_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_pp_c0_launch(const GemmArgs& p, float* ws, hipStream_t s);
void gemm_pp_c2_launch(const GemmArgs& p, float* ws, hipStream_t s);

namespace {

constexpr int BK = 64;

// Tile menu.  4 waves, 2 blocks per CU by LDS, 2 stages:
//   0: 128x128 (2x2)   1: 128x160 (2x2, wave 80x64)   2: 256x64 (4x1)   3: 128x64 (2x2)   4: 256x16 (4x1)
// 8 waves, 1 block per CU, 3-stage ring:
//   5: 256x160 (4x2, wave 64x80)   6: 256x128 (4x2, wave 64x64)
// 8-wave ping-pong kernel (gemm_pp.h; 1 block per CU, 4 phases per k-tile, counted vmcnt):
//   7: 256x256   8: 256x160   9: 256x128   10: 128x256
// deep LDS ring (gemm_impl.h STAGES 3-5, one block per CU; buffer-resource modes, bf16 out):
//   12: 128x128 4w S4 (also gated)   13: 128x64 4w S5   14: 128x160 8w S4
//   15: A-in-registers short-K kernel (gemm_areg.hip: K = 320 / 640, W streamed in chunks)
//   16: 128x80 4w (4x1, wave 32x80) S4: M = 2048 x N = 1280 is exactly 256 tiles, one per CU
//       (the 128x64 tile's 320 blocks ran as 1.25 rounds; the deep rings are one block per CU)
//   20: ping-pong 128x160 (4x2 waves, wave 32x80): twice the blocks of 256x160 without split-K
//       (M = 8192 x N = 640: 256 tiles)
//   21: ping-pong 128x128 (4x2 waves, wave 32x64, 64 KiB LDS: 2 blocks per CU)
//   22: ping-pong 128x64 (4x2 waves, 48 KiB LDS)
//   26 / 27: 8-wave 128x80 (8x1 waves, wave 16x80, 4-stage ring) / 128x64 (4x2 waves, 3 stages):
//       the small-grid tiles with twice the waves issuing LDS-DMA.  A CU's LDS-DMA fill rate is
//       set by the number of waves issuing it, not by the bytes in flight (4 waves: 22 B/cycle
//       on the GEMM row pattern at any ring depth, 8 waves: 37; profiles/r3_lds_fill_probe.jsonl)
//   31 / 32 / 33: warp-specialised deep rings, 8 MFMA waves + 8 DMA-only producer waves (1024
//       threads, 4 stages): 128x80 (8x1), 128x64 (4x2), 128x160 (4x2).  (256x128 / 128x256 / 128x128
//       and the gated 128x160 8x1 producer-wave tiles: bench-neutral in situ, removed;
//       profiles/r4_producer_waves_ab.txt)
// Removed in round 4 (measured, picked by no shape of the SD-1.5 / SDXL census; results kept in
// profiles/ and in git history): 11 (128x160 4w S4), 17-19 (register-staged 4-wave tiles,
// profiles/r2_regstage_ab.txt), 23 (ping-pong 256x64), 24/25 (halo-staged 3x3 conv,
// profiles/r3_bench_halo.jsonl), 28 (16-wave 128x64, profiles/r3_probe_16wave.jsonl), 29/30 (8-wave
// 128x128 / 256x80 and the gated 128x128, profiles/r3_tune_8wave_b_ab.txt,
// profiles/r3_tune_8wave_gated.txt).  Their indices stay reserved so table keys keep their meaning.
// Configs >= 11 are chosen only from the measured tuning table (gemm_tune_*) or when forced.
struct TileCfg { int BM, BN; float eff; int slots; };
constexpr int kNumTiles = 34;
constexpr int kPP128 = 20, kPP128x128 = 21;
// ping-pong configs outside the 7..10 block (dispatch and eligibility)
constexpr bool is_pp_cfg(int c) { return (c >= 7 && c < 11) || c == 20 || c == 21 || c == 22; }
// configs with a kernel behind them (the reserved indices above have none)
constexpr bool is_live_cfg(int c) {
  return (c >= 0 && c <= 10) || (c >= 12 && c <= 16) || (c >= 20 && c <= 22) || c == 26 || c == 27 ||
         (c >= 31 && c <= 33);
}
constexpr int kAreg = 15;
constexpr int kFirstPP = 7;
constexpr int kFirstDeep = 11;
// slots = resident blocks on the chip: 128x64 needs 48 KiB of LDS per block, so 3 blocks fit a
// CU (768 slots); with 512 the model undercounted it and missed the measured best on the
// level-2..4 plain GEMMs (profiles/r1_gemm_plan_sweep.jsonl: 14.5 vs 17.8 us at 8192x640x640)
constexpr TileCfg kTiles[kNumTiles] = {{128, 128, 1.00f, 512}, {128, 160, 1.02f, 512}, {256, 64, 0.95f, 512},
                                       {128, 64, 0.80f, 768},  {256, 16, 0.25f, 512},  {256, 160, 1.02f, 256},
                                       {256, 128, 1.00f, 256}, {256, 256, 1.60f, 256}, {256, 160, 1.55f, 256},
                                       {256, 128, 1.45f, 256}, {128, 256, 1.45f, 256}, {128, 160, 1.f, 256},
                                       {128, 128, 1.f, 256},   {128, 64, 1.f, 256},    {128, 160, 1.f, 256},
                                       {128, 64, 1.f, 256},    {128, 80, 1.f, 256},    {128, 64, 1.f, 768},
                                       {128, 128, 1.f, 512},   {128, 160, 1.f, 512},   {128, 160, 1.f, 256},
                                       {128, 128, 1.f, 512},   {128, 64, 1.f, 768},    {256, 64, 1.f, 512},
                                       {256, 160, 1.f, 256},   {128, 160, 1.f, 256},   {128, 80, 1.f, 256},
                                       {128, 64, 1.f, 256},    {128, 64, 1.f, 256},    {128, 128, 1.f, 256},
                                       {256, 80, 1.f, 256},    {128, 80, 1.f, 256},    {128, 64, 1.f, 256},
                                       {128, 160, 1.f, 256}};

// buffer-resource LDS-DMA path: K in whole k-tiles and every byte range addressable by a
// 31-bit buffer offset (num_records), plain GEMMs and Cin % 64 convolutions without upsample
bool buf_ok(const GemmArgs& p) {
  static const int force = [] {
    const char* e = getenv("CASSMANTLE_GEMM_BUF");
    return e ? atoi(e) : 1;
  }();
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

// the ping-pong kernel takes the buffer-resource modes (plain / two-source A, Cin % 64 convs
// without the fused upsample) with bf16 output
bool pp_ok(const GemmArgs& p) {
  // bf16 outputs the LDS-staged epilogue takes (the kernel's direct path only stores split-K slabs)
  const int cbs = p.ldcb ? p.ldcb : p.N;
  if (p.N % 8 != 0 || p.ldc % 8 != 0 || cbs % 4 != 0) return false;
  if (p.out_f32 || !buf_ok(p) || p.K % BK != 0) return false;
  if (p.conv && (p.upsample || p.Cin % 64 != 0)) return false;
  return p.N > 16;
}

bool deep_ok(const GemmArgs& p) {
  return !p.out_f32 && buf_ok(p) && p.K % BK == 0 && (!p.conv || (!p.upsample && p.Cin % 64 == 0)) && p.N > 16;
}

// ---- measured per-shape tuning table (tools/autotune_gemm.py -> ops/gemm_tuning.json, loaded by
// ops/__init__.py): shape key -> (tile config, split-K).  Consulted before the cost model.
std::mutex g_tune_mu;
std::unordered_map<std::string, GemmPlan> g_tune;
// per calling thread: the generation thread and the scorer thread both launch GEMMs, and these
// are written on every plan (tests/test_native_sanitizers.py runs the planner under TSan)
thread_local std::string g_last_key;
thread_local GemmPlan g_last_plan{0, 1};
std::atomic<bool> g_record_key{false};

}  // namespace

std::string gemm_key(const GemmArgs& p) {
  char buf[192];
  snprintf(buf, sizeof(buf), "m%d n%d k%d w%d b%d c%d:%d:%d:%d:%d:%d:%d:%d p%d a%d g%d s%d r%d cb%d ln%d f%d",
           p.M, p.N, p.K, p.Nw, p.batch, p.conv, p.IH, p.IW, p.Cin, p.stride, p.ksize, p.pad, p.upsample, p.parity,
           p.A2 != nullptr, is_gated(p.act) ? 1 : 0, p.stats != nullptr, p.residual != nullptr, p.chan_bias != nullptr,
           (p.ln_rows != nullptr || p.ln_rows_fx != nullptr) ? 1 : (p.ln_wsum != nullptr ? 2 : (p.gn_stats ? 3 : 0)),
           p.out_f32);
  return std::string(buf);
}

void gemm_tune_set(const std::string& key, int cfg, int split) {
  std::lock_guard<std::mutex> g(g_tune_mu);
  g_tune[key] = GemmPlan{cfg, split};
}
void gemm_tune_clear() {
  std::lock_guard<std::mutex> g(g_tune_mu);
  g_tune.clear();
}
int gemm_tune_size() {
  std::lock_guard<std::mutex> g(g_tune_mu);
  return (int)g_tune.size();
}
void gemm_record_keys(bool on) { g_record_key = on; }
std::string gemm_last_key() { return g_last_key; }
void gemm_last_plan(int* cfg, int* split) { *cfg = g_last_plan.cfg; *split = g_last_plan.split; }

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
static std::atomic<int> g_force_cfg{-2}, g_force_split{0};   // -2: not yet read from the environment
void gemm_set_override(int cfg, int split) {
  g_force_cfg = cfg;
  g_force_split = split;
}

static GemmPlan gemm_plan_impl(const GemmArgs& p);
GemmPlan gemm_plan(const GemmArgs& p) {
  GemmPlan r = gemm_plan_impl(p);
  if (p.row_stats != nullptr) {
    // output row statistics exist only in the shared LDS-staged epilogue (tile_epilogue):
    // no split-K, not the A-in-registers kernel
    if (r.cfg == kAreg) r.cfg = 3;
    r.split = 1;
  }
  g_last_plan = r;
  return r;
}

static GemmPlan gemm_plan_impl(const GemmArgs& p) {
  GemmPlan best{0, 1};
  if (g_force_cfg.load(std::memory_order_acquire) == -2) {
    static const bool from_env = [] {
      g_force_split.store(env_int("CASSMANTLE_GEMM_SPLIT", 0));
      int expect = -2;
      g_force_cfg.compare_exchange_strong(expect, env_int("CASSMANTLE_GEMM_CFG", -1));
      return true;
    }();
    (void)from_env;
  }
  const int force_cfg = g_force_cfg.load(), force_split = g_force_split.load();
  if (g_record_key) g_last_key = gemm_key(p);
  // in-kernel LayerNorm statistics exist only in the A-in-registers kernel (the binding checked
  // eligibility, so neither the table nor a forced config may pick anything else)
  if (p.ln_wsum != nullptr && p.ln_rows == nullptr && p.ln_rows_fx == nullptr) return GemmPlan{kAreg, 1};
  // GroupNorm folded into the A rows: only the A-in-registers kernel applies it (the binding
  // checked eligibility)
  if (p.gn_stats != nullptr) return GemmPlan{kAreg, 1};
  if (force_cfg < 0) {
    bool have = false;
    GemmPlan tp{0, 1};
    {
      std::lock_guard<std::mutex> g(g_tune_mu);
      if (!g_tune.empty()) {
        auto it = g_tune.find(gemm_key(p));
        if (it != g_tune.end()) { tp = it->second; have = true; }
      }
    }
    // a table entry is only taken if the kernel family can run this call (same checks as a
    // forced config), so a stale table never selects an unsupported path
    const bool elig = is_live_cfg(tp.cfg) &&
                      (tp.cfg < kFirstPP || (is_pp_cfg(tp.cfg) ? pp_ok(p) : (tp.cfg == kAreg ? gemm_areg_ok(p) : deep_ok(p))));
    if (have && elig) return tp;
  }
  static const int use_big = env_int("CASSMANTLE_GEMM_8WAVE", 0);
  const bool gated = p.act == ACT_GEGLU || p.act == ACT_SWIGLU;
  int only = -1;                         // forced tile (cost model still picks the split)
  const bool pp_elig = pp_ok(p);
  // CASSMANTLE_GEMM_PP=0 keeps the planner on the 4-wave kernel (A/B knob); forced configs
  // (CASSMANTLE_GEMM_CFG / gemm_set_override) only need eligibility
  static const int pp_auto = env_int("CASSMANTLE_GEMM_PP", 0);
  const bool pp = pp_elig && pp_auto;
  const bool deep_elig = deep_ok(p);
  if (force_cfg == kAreg) {
    if (gemm_areg_ok(p)) return GemmPlan{kAreg, 1};
  } else if (force_cfg >= 0 && is_live_cfg(force_cfg) && ((force_cfg == 4) == (p.N <= 16)) &&
      (force_cfg < kFirstPP || (is_pp_cfg(force_cfg) ? pp_elig : deep_elig))) {
    if (gated) {
      if (force_cfg == 0 || force_cfg == 6) best.cfg = force_cfg;
      else if (force_cfg >= kFirstDeep) best.cfg = 12;    // the deep-ring gated tile
      else if (force_cfg >= kFirstPP) best.cfg = force_cfg == 8 ? 8 : 9;   // the ping-pong gated tiles
      return best;
    }
    only = force_cfg;
  }
  if (gated) {
    if (pp && (p.N % 64 == 0) && (long long)(p.N / 64) * ((p.M + 255) / 256) >= 256) best.cfg = 9;
    return best;
  }
  const int nk = (p.K + BK - 1) / BK;
  // M <= 8 goes to the GEMV path; short prompts (M = tens of rows) need split-K to fill the chip
  // (batched calls -- the upsampling conv's 4 parity classes -- split per batch: slabs [z][split])
  const bool can_split = p.N % 4 == 0 && p.K % 8 == 0 && p.M > 8;
  double best_t = 1e30;
  for (int c = 0; c < kNumTiles; ++c) {
    const TileCfg& tc = kTiles[c];
    if (only >= 0 ? c != only : ((c == 5 || c == 6) && !use_big)) continue;
    if (c >= kFirstDeep && only != c) continue;   // table / forced only
    if (c == kAreg) continue;
    if (c >= kFirstPP && c < kFirstDeep && !(only >= 0 ? pp_elig : pp)) continue;
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
      if (split > 1) t += 6.0 + 2.0 * (double)split * p.batch * p.M * p.N * 4 / 3.0e6;
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
  if (p.cfg == kAreg && gemm_areg_ok(p)) {
    launch_gemm_areg(p, s);
    return;
  }
  if (is_pp_cfg(p.cfg) && pp_ok(p)) {
    if (!p.conv) gemm_pp_c0_launch(p, ws, s);
    else gemm_pp_c2_launch(p, ws, s);
    return;
  }
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
