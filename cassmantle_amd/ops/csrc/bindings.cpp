// pybind11 bindings of the gfx950 kernel library: tensor checks (fail loudly on wrong dtype,
// device, layout or alignment), output allocation stays in Python, every launch goes to the
// current HIP stream (so torch.cuda.graph capture records it).
#include <torch/extension.h>
#include <atomic>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_ext.h>

#include "kernels.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")

const uint16_t* bptr(const at::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* bptr_mut(at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
const uint16_t* opt_bptr(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_DEV(*t);
  CHECK_BF16(*t);
  CHECK_CONTIG(*t);
  return bptr(*t);
}

// plans split-K and allocates its fp32 partial slabs from the caching allocator (graph-pool
// safe inside a capture), then launches on the current stream
long long* opt_stats(const c10::optional<at::Tensor>& t, long long images, int N) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_DEV(*t);
  CHECK_CONTIG(*t);
  TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() == images * N * 2,
              "stats must be a zeroed int64 fixed-point [images, N, 2] tensor (ops.new_stats)");
  return reinterpret_cast<long long*>(t->data_ptr<int64_t>());
}

// tile raster group of every GEMM launch (gemm_impl.h tile_of): 0 = the compiled default;
// separate values for gated (GEGLU / SwiGLU) calls.  CASSMANTLE_GEMM_RASTER="G" or "G,Ggated",
// or gemm_set_raster at run time (A/B knob)
static std::atomic<int> g_raster[2] = {{-1}, {-1}};   // read by every GEMM launch thread
static void raster_from_env() {
  static const bool once = [] {
    const char* e = getenv("CASSMANTLE_GEMM_RASTER");
    int a = 0, b = -1;
    if (e != nullptr) {
      if (sscanf(e, "%d,%d", &a, &b) < 2) b = a;
    } else {
      b = 0;
    }
    int expect = -1;
    g_raster[0].compare_exchange_strong(expect, a);
    expect = -1;
    g_raster[1].compare_exchange_strong(expect, b);
    return true;
  }();
  (void)once;
}
void gemm_set_raster(int64_t plain, int64_t gated) {
  raster_from_env();
  g_raster[0].store((int)plain);
  g_raster[1].store((int)gated);
}

void run_gemm(GemmArgs& p, const at::Tensor& like) {
  raster_from_env();
  p.raster = g_raster[(p.act == 4 || p.act == 6) ? 1 : 0].load(std::memory_order_relaxed);   // gated: GEGLU (4) / SwiGLU (6)
  // output statistics are fused into the LDS-staged bf16 epilogue; shapes that take another
  // path (fp32 out, GEMV rows, batched, gated) get a separate per-channel statistics pass over
  // the output; split-K shapes accumulate them in the reduce pass
  TORCH_CHECK(p.stats == nullptr || (p.N % 8 == 0 && p.ldc == p.N),
              "gemm/conv2d stats: the output channel count must be a multiple of 8 (GroupNorm consumers)");
  const GemmPlan plan = gemm_plan(p);
  p.cfg = plan.cfg;
  p.split = plan.split;
  // fp8 K/V emission runs in the LDS-staged epilogue (V transposed through the tile in LDS);
  // the split-K reduce would scatter V byte by byte
  if (p.kv8 != nullptr) p.split = 1;
  long long* post_stats = nullptr;
  if (p.stats != nullptr && (p.out_f32 || p.M <= 8 || (p.batch != 1 && !p.parity) || p.act == 4 || p.act == 6)) {
    post_stats = p.stats;
    p.stats = nullptr;
  }
  if (p.split > 1) {
    auto ws = at::empty({(long long)p.split * p.batch * p.M * p.N}, like.options().dtype(at::kFloat));
    launch_gemm(p, ws.data_ptr<float>(), cur_stream());
  } else {
    launch_gemm(p, nullptr, cur_stream());
  }
  if (post_stats != nullptr)
    launch_channel_stats(reinterpret_cast<const uint16_t*>(p.C), post_stats, p.M / p.stats_hw, p.stats_hw, p.N,
                         cur_stream());
}

void gemm(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
          const c10::optional<at::Tensor>& residual, at::Tensor& out, int64_t act,
          const c10::optional<at::Tensor>& stats, int64_t stats_hw,
          const c10::optional<at::Tensor>& ln_rows, const c10::optional<at::Tensor>& ln_wsum, double ln_eps,
          const c10::optional<at::Tensor>& kv8, int64_t kv8_col0, int64_t kv8_ntok, int64_t kv8_hk,
          const c10::optional<at::Tensor>& ln_rows_fx, const c10::optional<at::Tensor>& row_stats,
          const c10::optional<at::Tensor>& gn_stats, const c10::optional<at::Tensor>& gn_gamma,
          const c10::optional<at::Tensor>& gn_beta, int64_t gn_groups, int64_t gn_hw, double gn_eps) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "gemm: 2-D operands expected");
  TORCH_CHECK(x.stride(1) == 1, "gemm: x rows must be contiguous");
  GemmArgs p;
  p.A = bptr(x); p.W = bptr(w); p.bias = opt_bptr(bias); p.residual = opt_bptr(residual);
  p.M = (int)x.size(0); p.K = (int)x.size(1); p.N = (int)out.size(1); p.Nw = (int)w.size(0);
  p.lda = (int)x.stride(0); p.ldc = p.N; p.act = (int)act;
  TORCH_CHECK(w.size(1) == p.K, "gemm: K mismatch");
  TORCH_CHECK(out.size(0) == p.M, "gemm: M mismatch");
  if (act == 4 || act == 6) {
    TORCH_CHECK(p.Nw == 2 * p.N && p.K % 8 == 0 && p.N % 4 == 0, "geglu/swiglu: W must be [2N,K], K%8==0, N%4==0");
  } else {
    TORCH_CHECK(p.Nw == p.N, "gemm: N mismatch");
  }
  if (residual.has_value() && residual->defined()) TORCH_CHECK(residual->numel() == out.numel(), "gemm: residual shape");
  if (out.scalar_type() == at::kFloat) {
    p.out_f32 = 1;
  } else {
    CHECK_BF16(out);
  }
  p.C = out.data_ptr();
  if (kv8.has_value() && kv8->defined()) {
    // e4m3 K/V image of the fp8 attention kernel written by the epilogue (columns >= kv8_col0)
    CHECK_DEV(*kv8); CHECK_CONTIG(*kv8);
    TORCH_CHECK(kv8->scalar_type() == at::kByte && kv8_ntok > 0 && kv8_ntok % 64 == 0 && p.M % kv8_ntok == 0 &&
                    kv8_hk > 0 && kv8_col0 % 8 == 0 && kv8_col0 + 128 * kv8_hk == p.N && act == 0 &&
                    !p.out_f32 && !(residual.has_value() && residual->defined()) && !(stats.has_value() && stats->defined()),
                "gemm kv8: uint8 image, 64-aligned tokens per image, K|V heads ending the output, plain epilogue");
    TORCH_CHECK(kv8->numel() == 2LL * p.M * kv8_hk * 64, "gemm kv8: image size");
    p.kv8 = kv8->data_ptr<uint8_t>();
    p.kv8_col0 = (int)kv8_col0; p.kv8_ntok = (int)kv8_ntok; p.kv8_hk = (int)kv8_hk;
  }
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats_hw > 0 && p.M % stats_hw == 0, "gemm: stats_hw must divide the rows");
    p.stats_hw = (int)stats_hw;
    p.stats = opt_stats(stats, p.M / stats_hw, p.N);
  }
  if (gn_stats.has_value() && gn_stats->defined()) {
    // GroupNorm (no SiLU) of x folded into the A-in-registers GEMM (transformer GroupNorm ->
    // proj_in); shapes that kernel does not take run the stats-driven GroupNorm apply + GEMM
    TORCH_CHECK(gn_gamma.has_value() && gn_beta.has_value() && gn_groups > 0 && gn_hw > 0 && p.M % gn_hw == 0,
                "gemm: gn_stats needs gamma, beta, groups and rows per image");
    CHECK_DEV(*gn_stats); CHECK_CONTIG(*gn_stats);
    TORCH_CHECK(gn_stats->scalar_type() == at::kLong && gn_stats->numel() == 2LL * (p.M / gn_hw) * p.K,
                "gemm: gn_stats int64 [images, K, 2]");
    TORCH_CHECK(!(ln_wsum.has_value() && ln_wsum->defined()) && !(row_stats.has_value() && row_stats->defined()) &&
                    !(kv8.has_value() && kv8->defined()) && !(stats.has_value() && stats->defined()),
                "gemm: gn_stats excludes LayerNorm folds, row / GroupNorm output statistics and kv8");
    p.gn_stats = reinterpret_cast<const long long*>(gn_stats->data_ptr<int64_t>());
    p.gn_gamma = opt_bptr(gn_gamma);
    p.gn_beta = opt_bptr(gn_beta);
    p.gn_groups = (int)gn_groups;
    p.gn_hw = (int)gn_hw;
    p.gn_eps = (float)gn_eps;
    if (gemm_areg_ok(p)) {
      run_gemm(p, out);                           // the planner maps gn_stats to the A-in-registers kernel
      return;
    }
    TORCH_CHECK(x.is_contiguous() && p.K % 8 == 0 && p.K % gn_groups == 0, "gemm gn fallback: contiguous rows");
    at::Tensor xn = at::empty_like(x);
    launch_group_norm_cs(bptr(x), nullptr, p.gn_stats, p.K, nullptr, p.gn_gamma, p.gn_beta, bptr_mut(xn),
                         p.M / gn_hw, gn_hw, p.K, (int)gn_groups, (float)gn_eps, 0, cur_stream());
    p.gn_stats = nullptr; p.gn_gamma = nullptr; p.gn_beta = nullptr;
    p.A = bptr(xn);
    run_gemm(p, out);
    return;
  }
  if (row_stats.has_value() && row_stats->defined()) {
    // LayerNorm row statistics of this output for a folded consumer (the LDS-staged epilogue
    // accumulates them; the planner then never splits K)
    CHECK_DEV(*row_stats); CHECK_CONTIG(*row_stats);
    TORCH_CHECK(row_stats->scalar_type() == at::kLong && row_stats->numel() == 2LL * p.M,
                "gemm: row_stats zeroed int64 [M, 2]");
    TORCH_CHECK(p.stats == nullptr && p.kv8 == nullptr && !p.out_f32 && p.batch == 1 && p.M > 8 && p.N % 8 == 0 &&
                    p.ldc % 8 == 0 && p.K % 8 == 0 && p.lda % 8 == 0,
                "gemm: row_stats needs the LDS-staged bf16 epilogue (no GroupNorm stats / kv8, N % 8 == 0, M > 8)");
    p.row_stats = reinterpret_cast<long long*>(row_stats->data_ptr<int64_t>());
  }
  if (ln_rows_fx.has_value() && ln_rows_fx->defined()) {
    // folded LayerNorm on row statistics a producer epilogue accumulated (no statistics pass)
    TORCH_CHECK(ln_wsum.has_value() && ln_wsum->defined() && ln_eps > 0 && !(ln_rows.has_value() && ln_rows->defined()),
                "gemm: ln_rows_fx needs ln_wsum and ln_eps, and excludes ln_rows");
    CHECK_DEV(*ln_rows_fx); CHECK_CONTIG(*ln_rows_fx); CHECK_DEV(*ln_wsum); CHECK_CONTIG(*ln_wsum);
    TORCH_CHECK(ln_rows_fx->scalar_type() == at::kLong && ln_rows_fx->numel() == 2LL * p.M, "gemm: ln_rows_fx int64 [M, 2]");
    TORCH_CHECK(ln_wsum->scalar_type() == at::kFloat && ln_wsum->numel() == p.Nw, "gemm: ln_wsum fp32 [Nw]");
    TORCH_CHECK(p.M > 8 && p.K % 8 == 0 && p.lda % 8 == 0 && !p.out_f32, "gemm: folded LayerNorm needs the MFMA path");
    p.ln_rows_fx = reinterpret_cast<const long long*>(ln_rows_fx->data_ptr<int64_t>());
    p.ln_wsum = ln_wsum->data_ptr<float>();
    p.ln_eps = (float)ln_eps;
    run_gemm(p, out);
    return;
  }
  if (ln_rows.has_value() && ln_rows->defined()) {
    // folded LayerNorm: raw rows in, per-row (mean, rstd) + column sums of the folded weights
    TORCH_CHECK(ln_wsum.has_value() && ln_wsum->defined(), "gemm: ln_rows needs ln_wsum");
    CHECK_DEV(*ln_rows); CHECK_CONTIG(*ln_rows); CHECK_DEV(*ln_wsum); CHECK_CONTIG(*ln_wsum);
    TORCH_CHECK(ln_rows->scalar_type() == at::kFloat && ln_rows->numel() == 2LL * p.M, "gemm: ln_rows fp32 [M, 2]");
    TORCH_CHECK(ln_wsum->scalar_type() == at::kFloat && ln_wsum->numel() == p.Nw, "gemm: ln_wsum fp32 [Nw]");
    TORCH_CHECK(p.M > 8 && p.K % 8 == 0 && p.lda % 8 == 0, "gemm: folded LayerNorm needs the MFMA path (M > 8)");
    TORCH_CHECK(!p.out_f32 || p.act == 0, "gemm: folded LayerNorm with fp32 output supports no activation");
    p.ln_rows = ln_rows->data_ptr<float>();
    p.ln_wsum = ln_wsum->data_ptr<float>();
  } else if (ln_wsum.has_value() && ln_wsum->defined() && ln_eps > 0) {
    // folded LayerNorm with the row statistics computed where they are cheapest: inside the
    // A-in-registers kernel when it takes the shape (K = 320 / 640), else a row-stats pass
    CHECK_DEV(*ln_wsum); CHECK_CONTIG(*ln_wsum);
    TORCH_CHECK(ln_wsum->scalar_type() == at::kFloat && ln_wsum->numel() == p.Nw, "gemm: ln_wsum fp32 [Nw]");
    TORCH_CHECK(p.M > 8 && p.K % 8 == 0 && p.lda % 8 == 0 && !p.out_f32, "gemm: folded LayerNorm needs the MFMA path");
    p.ln_wsum = ln_wsum->data_ptr<float>();
    p.ln_eps = (float)ln_eps;
    // CASSMANTLE_LN_INKERNEL=0 forces the row-statistics pass (A/B and debugging knob)
    static const bool inkernel = [] { const char* e = getenv("CASSMANTLE_LN_INKERNEL"); return !(e && e[0] == '0'); }();
    if (!inkernel || !gemm_areg_ok(p)) {
      TORCH_CHECK(x.is_contiguous() && p.K <= 4096, "gemm: folded LayerNorm row statistics need contiguous rows");
      at::Tensor rows = at::empty({p.M, 2}, x.options().dtype(at::kFloat));
      launch_row_stats(bptr(x), rows.data_ptr<float>(), p.M, p.K, (float)ln_eps, cur_stream());
      p.ln_rows = rows.data_ptr<float>();
      p.ln_eps = 0.f;
      run_gemm(p, out);
      return;
    }
  }
  run_gemm(p, out);
}

// per-row LayerNorm statistics (mean, rstd) of x [..., D] -> out fp32 [rows, 2]
void row_stats(const at::Tensor& x, at::Tensor& out, double eps) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_CONTIG(out);
  const int D = (int)x.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 4096, "row_stats: D % 8 == 0 and D <= 4096");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() == 2 * (x.numel() / D), "row_stats: out fp32 [rows, 2]");
  launch_row_stats(bptr(x), out.data_ptr<float>(), x.numel() / D, D, (float)eps, cur_stream());
}

// y = [x | x2] @ w^T + bias (+ residual, + output statistics) without materialising the channel
// concatenation: the GEMM stages k-tiles < Ca from x and the rest from x2 (UNet up-block
// ResNet shortcut over [h | skip]); Ca and K multiples of 64, M > 8
void gemm_cat(const at::Tensor& x, const at::Tensor& x2, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
              const c10::optional<at::Tensor>& residual, at::Tensor& out, const c10::optional<at::Tensor>& stats,
              int64_t stats_hw) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(x2); CHECK_CONTIG(x2); CHECK_BF16(w); CHECK_CONTIG(w);
  CHECK_BF16(out); CHECK_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && x2.dim() == 2 && w.dim() == 2 && out.dim() == 2 && x.size(0) == x2.size(0),
              "gemm_cat: 2-D operands with equal rows expected");
  GemmArgs p;
  p.A = bptr(x); p.A2 = bptr(x2); p.W = bptr(w); p.bias = opt_bptr(bias); p.residual = opt_bptr(residual);
  p.M = (int)x.size(0); p.ka = (int)x.size(1); p.K = p.ka + (int)x2.size(1);
  p.N = (int)out.size(1); p.Nw = (int)w.size(0);
  p.lda = p.ka; p.lda2 = (int)x2.size(1); p.ldc = p.N;
  TORCH_CHECK(w.size(1) == p.K && p.Nw == p.N && out.size(0) == p.M, "gemm_cat: shape mismatch");
  TORCH_CHECK(p.ka % 64 == 0 && p.K % 64 == 0 && p.M > 8, "gemm_cat: Ca and K must be multiples of 64, M > 8");
  const long long lim = (1LL << 31) - 1;
  TORCH_CHECK(x.numel() * 2 <= lim && x2.numel() * 2 <= lim && w.numel() * 2 <= lim, "gemm_cat: operand too large");
  if (residual.has_value() && residual->defined()) TORCH_CHECK(residual->numel() == out.numel(), "gemm_cat: residual shape");
  p.C = out.data_ptr();
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats_hw > 0 && p.M % stats_hw == 0, "gemm_cat: stats_hw must divide the rows");
    p.stats_hw = (int)stats_hw;
    p.stats = opt_stats(stats, p.M / stats_hw, p.N);
  }
  run_gemm(p, out);
}

// y = act(rmsnorm(x) @ w^T + bias) + residual for skinny x (<= 8 rows): the norm is fused into
// the weight-streaming GEMV (decode path of the causal LM)
void gemm_rms(const at::Tensor& x, const at::Tensor& gamma, double eps, const at::Tensor& w,
              const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& residual, at::Tensor& out,
              int64_t act) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(gamma); CHECK_CONTIG(gamma); CHECK_BF16(w); CHECK_CONTIG(w);
  CHECK_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(0) <= 8, "gemm_rms: x [<=8, K] rows contiguous");
  GemmArgs p;
  p.A = bptr(x); p.W = bptr(w); p.bias = opt_bptr(bias); p.residual = opt_bptr(residual);
  p.M = (int)x.size(0); p.K = (int)x.size(1); p.N = (int)out.size(1); p.Nw = (int)w.size(0);
  p.lda = (int)x.stride(0); p.ldc = p.N; p.act = (int)act;
  p.rms_gamma = bptr(gamma); p.rms_eps = (float)eps;
  TORCH_CHECK(gamma.numel() == p.K && w.size(1) == p.K, "gemm_rms: K mismatch");
  TORCH_CHECK(p.Nw == ((act == 4 || act == 6) ? 2 * p.N : p.N), "gemm_rms: N mismatch");
  if (out.scalar_type() == at::kFloat) p.out_f32 = 1;
  else CHECK_BF16(out);
  p.C = out.data_ptr();
  TORCH_CHECK(launch_gemv(p, cur_stream()), "gemm_rms: shape not supported by the GEMV path (K % 8)");
}

void conv2d(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
            const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& chan_bias, at::Tensor& out,
            int64_t stride, int64_t pad, int64_t upsample, const c10::optional<at::Tensor>& stats) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_CONTIG(out); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && out.dim() == 4, "conv2d: NHWC 4-D tensors expected");
  GemmArgs p;
  p.conv = 1;
  p.A = bptr(x); p.W = bptr(w); p.bias = opt_bptr(bias); p.residual = opt_bptr(residual);
  if (chan_bias.has_value() && chan_bias->defined()) {
    CHECK_DEV(*chan_bias);
    CHECK_BF16(*chan_bias);
    TORCH_CHECK(chan_bias->dim() == 2 && chan_bias->stride(1) == 1, "conv2d: chan_bias must be [B, Cout] rows");
    p.chan_bias = bptr(*chan_bias);
    p.ldcb = (int)chan_bias->stride(0);
  }
  p.IH = (int)x.size(1); p.IW = (int)x.size(2); p.Cin = (int)x.size(3);
  p.ksize = (int)w.size(1);
  TORCH_CHECK(w.size(2) == p.ksize && w.size(3) == p.Cin, "conv2d: weight must be [Cout,k,k,Cin]");
  p.Ho = (int)out.size(1); p.Wo = (int)out.size(2);
  p.N = (int)out.size(3); p.Nw = (int)w.size(0);
  TORCH_CHECK(p.Nw == p.N && out.size(0) == x.size(0), "conv2d: shape mismatch");
  p.M = (int)(x.size(0) * p.Ho * p.Wo);
  p.K = p.ksize * p.ksize * p.Cin;
  p.lda = p.Cin; p.ldc = p.N;
  p.stride = (int)stride; p.pad = (int)pad; p.upsample = (int)upsample;
  if (residual.has_value() && residual->defined()) TORCH_CHECK(residual->numel() == out.numel(), "conv2d: residual shape");
  if (chan_bias.has_value() && chan_bias->defined())
    TORCH_CHECK(chan_bias->size(0) == x.size(0) && chan_bias->size(1) == p.N, "conv2d: chan_bias must be [B, Cout]");
  p.C = out.data_ptr();
  p.stats_hw = p.Ho * p.Wo;
  p.stats = opt_stats(stats, x.size(0), p.N);
  run_gemm(p, out);
}

// nearest-2x upsample + 3x3 conv (pad 1) as four 2x2 convs on the low-res input, one per output
// parity class (4/9 of the MACs of the upsampled conv): w4 [4, Cout, 2, 2, Cin] are the folded
// weights (ops.fold_upsample_weights), out [B, 2H, 2W, Cout]
void conv2d_up2(const at::Tensor& x, const at::Tensor& w4, const c10::optional<at::Tensor>& bias,
                const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& chan_bias, at::Tensor& out,
                const c10::optional<at::Tensor>& stats) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w4); CHECK_CONTIG(w4); CHECK_CONTIG(out); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 4 && w4.dim() == 5 && w4.size(0) == 4 && w4.size(2) == 2 && w4.size(3) == 2 &&
              w4.size(4) == x.size(3), "conv2d_up2: x [B,H,W,Cin], w4 [4,Cout,2,2,Cin]");
  TORCH_CHECK(out.dim() == 4 && out.size(0) == x.size(0) && out.size(1) == 2 * x.size(1) &&
              out.size(2) == 2 * x.size(2) && out.size(3) == w4.size(1), "conv2d_up2: out [B,2H,2W,Cout]");
  GemmArgs p;
  p.conv = 1;
  p.parity = 1;
  p.A = bptr(x); p.W = bptr(w4); p.bias = opt_bptr(bias); p.residual = opt_bptr(residual);
  if (chan_bias.has_value() && chan_bias->defined()) {
    CHECK_DEV(*chan_bias);
    CHECK_BF16(*chan_bias);
    TORCH_CHECK(chan_bias->dim() == 2 && chan_bias->stride(1) == 1 && chan_bias->size(0) == x.size(0) &&
                chan_bias->size(1) == out.size(3), "conv2d_up2: chan_bias must be [B, Cout] rows");
    p.chan_bias = bptr(*chan_bias);
    p.ldcb = (int)chan_bias->stride(0);
  }
  p.IH = (int)x.size(1); p.IW = (int)x.size(2); p.Cin = (int)x.size(3);
  p.ksize = 2; p.stride = 1; p.pad = 1; p.upsample = 0;
  p.Ho = p.IH; p.Wo = p.IW;                       // GEMM rows: the low-res grid of each class
  p.N = (int)out.size(3); p.Nw = p.N;
  p.M = (int)(x.size(0) * p.Ho * p.Wo);
  p.K = 4 * p.Cin;
  p.lda = p.Cin; p.ldc = p.N;
  p.batch = 4;                                    // grid z = parity class
  p.sA = 0; p.sW = (long long)p.N * 4 * p.Cin; p.sC = 0;
  TORCH_CHECK(p.Cin % 64 == 0, "conv2d_up2: Cin % 64 == 0 (buffer-DMA conv path)");
  if (residual.has_value() && residual->defined()) TORCH_CHECK(residual->numel() == out.numel(), "conv2d_up2: residual shape");
  p.C = out.data_ptr();
  p.stats_hw = p.Ho * p.Wo;                       // per image: every class adds its quarter
  p.stats = opt_stats(stats, x.size(0), p.N);
  run_gemm(p, out);
}

// batched C[b] = alpha * A[b] @ B[b]^T ; A [Bt, M, K] (row stride free), B [Bt, N, K], C [Bt, M, N]
void bmm_nt(const at::Tensor& a, const at::Tensor& b, at::Tensor& out, double alpha) {
  CHECK_DEV(a); CHECK_BF16(a); CHECK_BF16(b); CHECK_CONTIG(out);
  TORCH_CHECK(a.dim() == 3 && b.dim() == 3 && out.dim() == 3, "bmm_nt: 3-D operands");
  TORCH_CHECK(a.stride(2) == 1 && b.stride(2) == 1, "bmm_nt: K must be contiguous");
  GemmArgs p;
  p.A = bptr(a); p.W = bptr(b);
  p.batch = (int)a.size(0);
  p.M = (int)a.size(1); p.K = (int)a.size(2); p.N = (int)b.size(1); p.Nw = p.N;
  p.lda = (int)a.stride(1); p.ldw = (int)b.stride(1); p.sA = a.stride(0); p.sW = b.stride(0);
  p.ldc = p.N; p.sC = (long long)p.M * p.N;
  p.alpha = (float)alpha;
  if (out.scalar_type() == at::kFloat) {
    p.out_f32 = 1;
  } else {
    CHECK_BF16(out);
  }
  p.C = out.data_ptr();
  run_gemm(p, out);
}

void group_norm(const at::Tensor& x, const at::Tensor& gamma, const at::Tensor& beta, at::Tensor& out,
                int64_t groups, double eps, int64_t silu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(gamma); CHECK_BF16(beta); CHECK_CONTIG(out);
  const int B = (int)x.size(0);
  const int C = (int)x.size(-1);
  const long long S = x.numel() / ((long long)B * C);
  TORCH_CHECK(C % 8 == 0 && C % groups == 0, "group_norm: C must be a multiple of 8 and of groups");
  auto ws = at::empty({group_norm_workspace(B, S, C)}, x.options().dtype(at::kFloat));
  launch_group_norm(bptr(x), bptr(gamma), bptr(beta), bptr_mut(out), ws.data_ptr<float>(), B, S, C, (int)groups,
                    (float)eps, (int)silu, cur_stream());
}

// GroupNorm from producer statistics: stats_a [B, Ca, 2] (+ stats_b [B, C - Ca, 2] for a
// channel concatenation), as accumulated by gemm/conv2d(stats=...)
void group_norm_stats(const at::Tensor& x, const at::Tensor& stats_a, const c10::optional<at::Tensor>& stats_b,
                      const at::Tensor& gamma, const at::Tensor& beta, at::Tensor& out, int64_t groups, double eps,
                      int64_t silu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(gamma); CHECK_BF16(beta); CHECK_CONTIG(out);
  const int B = (int)x.size(0);
  const int C = (int)x.size(-1);
  const long long S = x.numel() / ((long long)B * C);
  TORCH_CHECK(C % 8 == 0 && C % groups == 0, "group_norm_stats: C must be a multiple of 8 and of groups");
  TORCH_CHECK(stats_a.scalar_type() == at::kLong && stats_a.is_contiguous() && stats_a.dim() == 3 &&
              stats_a.size(0) == B && stats_a.size(2) == 2, "group_norm_stats: stats_a must be int64 [B, Ca, 2]");
  const int Ca = (int)stats_a.size(1);
  const long long* sb = nullptr;
  if (stats_b.has_value() && stats_b->defined()) {
    TORCH_CHECK(stats_b->scalar_type() == at::kLong && stats_b->is_contiguous() && stats_b->dim() == 3 &&
                stats_b->size(0) == B && stats_b->size(1) == C - Ca && stats_b->size(2) == 2,
                "group_norm_stats: stats_b must be int64 [B, C - Ca, 2]");
    sb = reinterpret_cast<const long long*>(stats_b->data_ptr<int64_t>());
  } else {
    TORCH_CHECK(Ca == C, "group_norm_stats: stats_a must cover every channel");
  }
  launch_group_norm_cs(bptr(x), nullptr, reinterpret_cast<const long long*>(stats_a.data_ptr<int64_t>()), Ca, sb, bptr(gamma), bptr(beta), bptr_mut(out), B, S, C,
                       (int)groups, (float)eps, (int)silu, cur_stream());
}

// GroupNorm(+SiLU) of the channel concatenation [x | x2] (NHWC, same B and pixels) from the
// producers' statistics, written as one contiguous [.., Ca + Cb] output; the concatenation
// itself is never materialised
void group_norm_cat(const at::Tensor& x, const at::Tensor& x2, const at::Tensor& stats_a, const at::Tensor& stats_b,
                    const at::Tensor& gamma, const at::Tensor& beta, at::Tensor& out, int64_t groups, double eps,
                    int64_t silu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(x2); CHECK_CONTIG(x2); CHECK_BF16(gamma); CHECK_BF16(beta);
  CHECK_CONTIG(out); CHECK_BF16(out);
  const int B = (int)x.size(0);
  const int Ca = (int)x.size(-1), Cb = (int)x2.size(-1), C = Ca + Cb;
  const long long S = x.numel() / ((long long)B * Ca);
  TORCH_CHECK(x2.size(0) == B && x2.numel() == (long long)B * S * Cb && out.numel() == (long long)B * S * C &&
              out.size(-1) == C, "group_norm_cat: shapes must agree on batch and pixels");
  TORCH_CHECK(Ca % 8 == 0 && Cb % 8 == 0 && C % groups == 0, "group_norm_cat: channel counts");
  TORCH_CHECK(stats_a.scalar_type() == at::kLong && stats_a.is_contiguous() && stats_a.numel() == (long long)B * Ca * 2 &&
              stats_b.scalar_type() == at::kLong && stats_b.is_contiguous() && stats_b.numel() == (long long)B * Cb * 2,
              "group_norm_cat: int64 [B, C, 2] statistics of both inputs expected");
  launch_group_norm_cs(bptr(x), bptr(x2), reinterpret_cast<const long long*>(stats_a.data_ptr<int64_t>()), Ca, reinterpret_cast<const long long*>(stats_b.data_ptr<int64_t>()), bptr(gamma),
                       bptr(beta), bptr_mut(out), B, S, C, (int)groups, (float)eps, (int)silu, cur_stream());
}

void channel_stats(const at::Tensor& x, at::Tensor& stats) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x);
  const int B = (int)x.size(0);
  const int C = (int)x.size(-1);
  const long long S = x.numel() / ((long long)B * C);
  TORCH_CHECK(C % 8 == 0, "channel_stats: C % 8 == 0");
  launch_channel_stats(bptr(x), opt_stats(stats, B, C), B, S, C, cur_stream());
}

void layer_norm(const at::Tensor& x, const at::Tensor& gamma, const c10::optional<at::Tensor>& beta, at::Tensor& out,
                double eps) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(gamma); CHECK_CONTIG(out);
  const int D = (int)x.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 4096, "layer_norm: D % 8 == 0 and D <= 4096");
  launch_layer_norm(bptr(x), bptr(gamma), opt_bptr(beta), bptr_mut(out), x.numel() / D, D, (float)eps, cur_stream());
}

// encoder input layer: out[r] = LN(word[ids[r]] + pos[r % seq] + add); ids int64 [rows]
void embed_layer_norm(const at::Tensor& word, const at::Tensor& ids, const at::Tensor& pos, int64_t seq,
                      const c10::optional<at::Tensor>& add, const at::Tensor& gamma,
                      const c10::optional<at::Tensor>& beta, at::Tensor& out, double eps) {
  CHECK_DEV(word); CHECK_BF16(word); CHECK_CONTIG(word); CHECK_DEV(ids); CHECK_CONTIG(ids);
  CHECK_BF16(pos); CHECK_CONTIG(pos); CHECK_BF16(gamma); CHECK_BF16(out); CHECK_CONTIG(out);
  TORCH_CHECK(ids.scalar_type() == at::kLong, "embed_layer_norm: int64 ids");
  const int D = (int)word.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 4096 && pos.size(-1) == D && out.numel() == ids.numel() * D,
              "embed_layer_norm: D % 8 == 0, D <= 4096, out [rows, D]");
  TORCH_CHECK(seq > 0 && pos.size(0) >= seq, "embed_layer_norm: position table shorter than seq");
  launch_embed_layer_norm(bptr(word), reinterpret_cast<const long long*>(ids.data_ptr<int64_t>()), bptr(pos), (int)seq,
                          opt_bptr(add), bptr(gamma), opt_bptr(beta), bptr_mut(out), ids.numel(), D, (float)eps,
                          cur_stream());
}

static AttnArgs attn_args(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& out, double scale,
                          int64_t causal, const c10::optional<at::Tensor>& kv_lens) {
  CHECK_DEV(q); CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v); CHECK_BF16(out);
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4 && out.dim() == 4, "attention: [B,N,H,d] tensors");
  TORCH_CHECK(q.stride(3) == 1 && k.stride(3) == 1 && v.stride(3) == 1 && out.stride(3) == 1,
              "attention: head dim must be contiguous");
  AttnArgs a;
  a.q = bptr(q); a.k = bptr(k); a.v = bptr(v); a.o = bptr_mut(out);
  a.q_sb = q.stride(0); a.q_sn = q.stride(1); a.q_sh = q.stride(2);
  a.k_sb = k.stride(0); a.k_sn = k.stride(1); a.k_sh = k.stride(2);
  a.v_sb = v.stride(0); a.v_sn = v.stride(1); a.v_sh = v.stride(2);
  a.o_sb = out.stride(0); a.o_sn = out.stride(1); a.o_sh = out.stride(2);
  a.B = (int)q.size(0); a.Nq = (int)q.size(1); a.H = (int)q.size(2); a.d = (int)q.size(3);
  a.Nk = (int)k.size(1);
  TORCH_CHECK(a.d % 8 == 0 && (a.d <= 160 || a.d == 512), "attention: head dim must be a multiple of 8 and <= 160, or 512");
  TORCH_CHECK(k.size(2) == v.size(2) && a.H % k.size(2) == 0, "attention: query heads must be a multiple of kv heads");
  a.group = a.H / (int)k.size(2);
  for (long long st : {a.q_sb, a.q_sn, a.q_sh, a.k_sb, a.k_sn, a.k_sh, a.v_sb, a.v_sn, a.v_sh})
    TORCH_CHECK(st % 8 == 0, "attention: q/k/v strides must be 16-byte aligned");
  for (long long st : {a.o_sb, a.o_sn, a.o_sh}) TORCH_CHECK(st % 4 == 0, "attention: out strides must be 8-byte aligned");
  a.scale = (float)scale;
  a.causal = (int)causal;
  a.kv_lens = nullptr;
  if (kv_lens.has_value() && kv_lens->defined()) {
    TORCH_CHECK(kv_lens->scalar_type() == at::kInt && kv_lens->is_cuda(), "kv_lens must be int32 on device");
    a.kv_lens = kv_lens->data_ptr<int>();
  }
  return a;
}

// K8 / V8t bytes of an fp8 attention over these K/V (B x kv heads x keys rounded to 64 x 64 x 2)
int64_t attention_fp8_bytes(int64_t B, int64_t Nk, int64_t Hk) { return 2 * B * Hk * ((Nk + 63) / 64 * 64) * 64; }

// pack K/V [B, Nk, Hk, 64] (any strides, last dim contiguous) into kv8 once -- the cross-attention
// K/V are constant over a whole generation (UNet.set_context)
void attention_fp8_pack(const at::Tensor& k, const at::Tensor& v, const c10::optional<at::Tensor>& kv_lens,
                        at::Tensor& kv8) {
  at::Tensor out = at::empty({1, 1, 1, k.size(3)}, k.options());
  AttnArgs a = attn_args(k, k, v, out, 1.0, 0, kv_lens);
  TORCH_CHECK(a.d == 64, "fp8 attention: head dim 64 only");
  const int Hk = (int)k.size(2);
  TORCH_CHECK(kv8.is_cuda() && kv8.scalar_type() == at::kByte && kv8.is_contiguous() &&
                  kv8.numel() == attention_fp8_bytes(a.B, a.Nk, Hk), "kv8: contiguous uint8 of attention_fp8_bytes");
  launch_attention_fp8_pack(a, Hk, kv8.data_ptr<uint8_t>(), cur_stream());
}

void attention(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& out, double scale,
               int64_t causal, const c10::optional<at::Tensor>& kv_lens, int64_t fp8,
               const c10::optional<at::Tensor>& kv8) {
  AttnArgs a = attn_args(q, k, v, out, scale, causal, kv_lens);
  if (a.d == 512) {
    const long long wsb = attention_d512_workspace(a);
    at::Tensor ws;
    if (wsb > 0) ws = at::empty({wsb / 4}, q.options().dtype(at::kFloat));
    launch_attention_d512(a, wsb > 0 ? ws.data_ptr<float>() : nullptr, cur_stream());
    return;
  }
  if (fp8 && a.d == 64) {
    const int Hk = (int)k.size(2);
    if (kv8.has_value() && kv8->defined()) {          // K/V packed earlier (cross-attention)
      TORCH_CHECK(kv8->is_cuda() && kv8->scalar_type() == at::kByte &&
                      kv8->numel() == attention_fp8_bytes(a.B, a.Nk, Hk), "kv8 does not match K/V");
      launch_attention_fp8(a, Hk, kv8->data_ptr<uint8_t>(), cur_stream(), true);
      return;
    }
    // OCP e4m3 K/V packed per call (workspace from the caching allocator: graph-safe)
    auto ws = at::empty({attention_fp8_workspace(a, Hk)}, q.options().dtype(at::kByte));
    launch_attention_fp8(a, Hk, ws.data_ptr<uint8_t>(), cur_stream());
    return;
  }
  launch_attention(a, cur_stream());
}

void gather_cosine(const at::Tensor& table, const at::Tensor& ia, const at::Tensor& ib, at::Tensor& out) {
  CHECK_DEV(table); CHECK_CONTIG(table);
  TORCH_CHECK(ia.scalar_type() == at::kInt && ib.scalar_type() == at::kInt, "indices must be int32");
  int f32 = table.scalar_type() == at::kFloat;
  if (!f32) {
    CHECK_BF16(table);
  }
  launch_gather_cosine(table.data_ptr(), f32, (int)table.size(1), ia.data_ptr<int>(), ib.data_ptr<int>(),
                       out.data_ptr<float>(), (int)ia.size(0), cur_stream());
}

void pair_cosine(const at::Tensor& a, const at::Tensor& b, at::Tensor& out) {
  CHECK_DEV(a);
  TORCH_CHECK(a.scalar_type() == at::kFloat && b.scalar_type() == at::kFloat, "pair_cosine: f32 inputs");
  CHECK_CONTIG(a); CHECK_CONTIG(b);
  launch_pair_cosine(a.data_ptr<float>(), b.data_ptr<float>(), (int)a.size(1), out.data_ptr<float>(), (int)a.size(0),
                     cur_stream());
}

void cosine_gemv(const at::Tensor& table, const at::Tensor& vec, at::Tensor& out) {
  CHECK_DEV(table); CHECK_CONTIG(table); CHECK_CONTIG(vec);
  int tf = table.scalar_type() == at::kFloat, vf = vec.scalar_type() == at::kFloat;
  launch_cosine_gemv(table.data_ptr(), tf, (int)table.size(0), (int)table.size(1), vec.data_ptr(), vf,
                     out.data_ptr<float>(), cur_stream());
}

// K15 most_similar: fused cosine GEMV + block top-k + merge passes (misc.hip), no ATen sort
std::vector<at::Tensor> cosine_topk(const at::Tensor& table, const at::Tensor& vec, int64_t k) {
  CHECK_DEV(table); CHECK_CONTIG(table); CHECK_CONTIG(vec);
  TORCH_CHECK(table.dim() == 2 && vec.numel() == table.size(1), "cosine_topk: table [V, D], vec [D]");
  TORCH_CHECK(table.size(0) < (1ll << 31), "cosine_topk: V must fit int32");
  TORCH_CHECK(k >= 1 && k <= 1024 && k <= table.size(0), "cosine_topk: 1 <= k <= min(1024, V)");
  int tf = table.scalar_type() == at::kFloat, vf = vec.scalar_type() == at::kFloat;
  TORCH_CHECK(tf || table.scalar_type() == at::kBFloat16, "cosine_topk: table f32 or bf16");
  TORCH_CHECK(vf || vec.scalar_type() == at::kBFloat16, "cosine_topk: vec f32 or bf16");
  const int V = (int)table.size(0);
  auto ws = at::empty({(int64_t)cosine_topk_workspace(V, (int)k)}, table.options().dtype(at::kLong));
  auto vals = at::empty({k}, table.options().dtype(at::kFloat));
  auto idx = at::empty({k}, table.options().dtype(at::kLong));
  launch_cosine_topk(table.data_ptr(), tf, V, (int)table.size(1), vec.data_ptr(), vf, (int)k,
                     reinterpret_cast<unsigned long long*>(ws.data_ptr<int64_t>()), vals.data_ptr<float>(),
                     reinterpret_cast<long long*>(idx.data_ptr<int64_t>()), cur_stream());
  return {vals, idx};
}

void mean_pool_l2(const at::Tensor& h, const at::Tensor& lens, at::Tensor& out) {
  CHECK_DEV(h); CHECK_BF16(h); CHECK_CONTIG(h);
  TORCH_CHECK(lens.scalar_type() == at::kInt, "lens must be int32");
  launch_mean_pool_l2(bptr(h), lens.data_ptr<int>(), out.data_ptr<float>(), (int)h.size(0), (int)h.size(1),
                      (int)h.size(2), cur_stream());
}

void gaussian_blur(const at::Tensor& img, const at::Tensor& w, at::Tensor& out) {
  CHECK_DEV(img); CHECK_CONTIG(img);
  TORCH_CHECK(img.dim() == 3, "gaussian_blur: [H, W, C]");
  int u8 = img.scalar_type() == at::kByte;
  if (!u8) {
    TORCH_CHECK(img.scalar_type() == at::kFloat, "gaussian_blur: uint8 or f32");
  }
  auto wf = w.to(at::kFloat).contiguous();
  int R = (int)(wf.numel() - 1) / 2;
  const int C = (int)img.size(2);
  // the LDS-tiled uint8 kernel (R <= 48, C in {1,3,4}) needs no global scratch
  const bool tiled = u8 && R <= 48 && (C == 1 || C == 3 || C == 4);
  at::Tensor tmp;
  if (!tiled) tmp = at::empty({img.numel()}, img.options().dtype(at::kFloat));
  launch_gaussian_blur(img.data_ptr(), u8, (int)img.size(0), (int)img.size(1), C, wf.data_ptr<float>(), R,
                       tiled ? nullptr : tmp.data_ptr<float>(), out.data_ptr(), cur_stream());
}

void to_uint8(const at::Tensor& x, at::Tensor& out) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x);
  launch_to_uint8(bptr(x), out.data_ptr<uint8_t>(), x.numel(), cur_stream());
}

void timestep_embedding(const at::Tensor& t, at::Tensor& out, int64_t flip, double shift) {
  CHECK_DEV(t); CHECK_CONTIG(t); CHECK_CONTIG(out);
  TORCH_CHECK(t.scalar_type() == at::kFloat && out.dim() == 2 && out.size(0) == t.numel() && out.size(1) % 2 == 0,
              "timestep_embedding: t f32 [B], out [B, dim]");
  const int bf = out.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || out.scalar_type() == at::kFloat, "timestep_embedding: out f32 or bf16");
  launch_timestep_embedding(t.data_ptr<float>(), out.data_ptr(), (int)t.size(0), (int)out.size(1), (int)flip,
                            (float)shift, bf, cur_stream());
}

void gather_add(const at::Tensor& table, const at::Tensor& ids, const c10::optional<at::Tensor>& pos, int64_t seq,
                at::Tensor& out) {
  CHECK_DEV(table); CHECK_BF16(table); CHECK_CONTIG(table); CHECK_CONTIG(ids); CHECK_BF16(out); CHECK_CONTIG(out);
  TORCH_CHECK(ids.scalar_type() == at::kInt && ids.is_cuda(), "gather_add: int32 device ids");
  const int D = (int)table.size(-1);
  const long long rows = ids.numel();
  TORCH_CHECK(D % 8 == 0 && out.numel() == rows * D, "gather_add: D % 8 == 0, out [rows, D]");
  const uint16_t* pp = opt_bptr(pos);
  TORCH_CHECK(pp == nullptr || (seq > 0 && pos->size(-1) == D && pos->numel() >= seq * D), "gather_add: pos [>= seq, D]");
  launch_gather_add(bptr(table), ids.data_ptr<int>(), pp, (int)(seq > 0 ? seq : 1), D, rows, bptr_mut(out),
                    cur_stream());
}

void concat2(const at::Tensor& a, const at::Tensor& b, at::Tensor& out) {
  CHECK_DEV(a); CHECK_BF16(a); CHECK_CONTIG(a); CHECK_DEV(b); CHECK_CONTIG(b); CHECK_BF16(out); CHECK_CONTIG(out);
  const int Da = (int)a.size(-1), Db = (int)b.size(-1);
  const long long rows = a.numel() / Da;
  const int f32 = b.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || b.scalar_type() == at::kBFloat16, "concat2: b bf16 or f32");
  TORCH_CHECK(Da % 8 == 0 && Db % 8 == 0 && b.numel() == rows * Db && out.numel() == rows * (Da + Db),
              "concat2: [rows, Da] + [rows, Db] -> [rows, Da + Db], D % 8 == 0");
  launch_concat2(bptr(a), Da, b.data_ptr(), Db, f32, rows, bptr_mut(out), cur_stream());
}

void silu_(at::Tensor& x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.numel() % 8 == 0, "silu_: numel % 8 == 0");
  launch_silu_bf16(bptr_mut(x), x.numel(), cur_stream());
}

void latent_init(const at::Tensor& x0, double c_in0, at::Tensor& x, at::Tensor& xs, at::Tensor& hist, at::Tensor& unet_in,
                 int64_t cfg) {
  CHECK_DEV(x0); CHECK_CONTIG(x0); CHECK_CONTIG(x); CHECK_CONTIG(xs); CHECK_CONTIG(hist); CHECK_BF16(unet_in);
  CHECK_CONTIG(unet_in);
  TORCH_CHECK(x0.scalar_type() == at::kFloat && x.scalar_type() == at::kFloat && xs.scalar_type() == at::kFloat &&
              hist.scalar_type() == at::kFloat, "latent_init: f32 latents");
  const long long n = x.numel();
  const int cin = (int)x.size(-1), cstride = (int)unet_in.size(-1);
  TORCH_CHECK(x0.numel() == n && xs.numel() == n && hist.numel() % n == 0 && cstride >= cin &&
              unet_in.numel() == (cfg ? 2 : 1) * (n / cin) * cstride, "latent_init: shape mismatch");
  launch_latent_init(x0.data_ptr<float>(), (float)c_in0, x.data_ptr<float>(), xs.data_ptr<float>(),
                     hist.data_ptr<float>(), (int)(hist.numel() / n), bptr_mut(unet_in), n, (int)cfg, cin, cstride,
                     cur_stream());
}

void dcopy(const at::Tensor& src, at::Tensor& dst) {
  CHECK_DEV(src); CHECK_CONTIG(src); CHECK_DEV(dst); CHECK_CONTIG(dst);
  TORCH_CHECK(src.scalar_type() == dst.scalar_type() && src.numel() == dst.numel(), "dcopy: same dtype and size");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
              "dcopy: 16-byte aligned");
  launch_copy(src.data_ptr(), dst.data_ptr(), (long long)src.numel() * src.element_size(), cur_stream());
}

void finalize_latents(const at::Tensor& x, at::Tensor& z, at::Tensor& finite) {
  CHECK_DEV(x); CHECK_CONTIG(x); CHECK_BF16(z); CHECK_CONTIG(z);
  TORCH_CHECK(x.scalar_type() == at::kFloat && z.numel() == x.numel() && finite.scalar_type() == at::kByte &&
              finite.numel() >= 1 && finite.is_cuda(), "finalize_latents: f32 x -> bf16 z, uint8 flag");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(z.data_ptr()) % 8 == 0,
              "finalize_latents: x 16-byte / z 8-byte aligned");
  launch_finalize_latents(x.data_ptr<float>(), bptr_mut(z), x.numel(), finite.data_ptr<uint8_t>(), cur_stream());
}

void latent_step(const at::Tensor& eps, at::Tensor& x, at::Tensor& hist, at::Tensor& xs, const at::Tensor& coef,
                 const at::Tensor& step, at::Tensor& unet_in, int64_t cfg, const c10::optional<at::Tensor>& tab0,
                 const c10::optional<at::Tensor>& buf0, const c10::optional<at::Tensor>& tab1,
                 const c10::optional<at::Tensor>& buf1) {
  CHECK_DEV(x); CHECK_BF16(eps); CHECK_CONTIG(eps); CHECK_BF16(unet_in); CHECK_CONTIG(unet_in);
  TORCH_CHECK(x.scalar_type() == at::kFloat && hist.scalar_type() == at::kFloat && xs.scalar_type() == at::kFloat,
              "latent_step: f32 master latents");
  TORCH_CHECK(step.scalar_type() == at::kInt, "latent_step: int32 step counter");
  const long long n = x.numel();
  const int cin = (int)x.size(-1), cstride = (int)unet_in.size(-1);
  TORCH_CHECK(cstride >= cin && eps.numel() == (cfg ? 2 * n : n) && hist.numel() == 4 * n &&
              unet_in.numel() == eps.numel() / cin * cstride, "latent_step: shape mismatch");
  auto tab_ok = [&](const c10::optional<at::Tensor>& t, const c10::optional<at::Tensor>& b) {
    if (!t.has_value() || !t->defined()) return false;
    TORCH_CHECK(b.has_value() && b->defined() && t->is_contiguous() && b->is_contiguous() &&
                t->numel() % t->size(0) == 0 && b->numel() * b->element_size() * t->size(0) == t->numel() * t->element_size() &&
                (b->numel() * b->element_size()) % 16 == 0, "latent_step: tables [rows, ...] and row buffers, 16-B rows");
    return true;
  };
  const bool h0 = tab_ok(tab0, buf0), h1 = tab_ok(tab1, buf1);
  const int rows = h0 ? (int)tab0->size(0) : (h1 ? (int)tab1->size(0) : 0);
  TORCH_CHECK(!(h0 && h1) || tab1->size(0) == rows, "latent_step: tables of equal row count");
  launch_latent_step(bptr(eps), x.data_ptr<float>(), hist.data_ptr<float>(), xs.data_ptr<float>(),
                     coef.data_ptr<float>(), step.data_ptr<int>(), bptr_mut(unet_in), n, (int)cfg, cin, cstride,
                     h0 ? tab0->data_ptr() : nullptr, h0 ? buf0->data_ptr() : nullptr,
                     h0 ? buf0->numel() * buf0->element_size() : 0, h1 ? tab1->data_ptr() : nullptr,
                     h1 ? buf1->data_ptr() : nullptr, h1 ? buf1->numel() * buf1->element_size() : 0, rows,
                     cur_stream());
}

// A HIP stream whose kernels may only run on the CUs of ``mask`` (bit i of word i / 32 = CU i):
// the serving scorer gets a few CUs of its own and the generation stream the rest, so a guess is
// never queued behind a wave of denoise workgroups (verdict r2 item 6).  Returned as the raw
// handle for torch.cuda.ExternalStream; it lives for the process.
int64_t cu_mask_stream(int64_t device, const std::vector<int64_t>& mask) {
  TORCH_CHECK(!mask.empty(), "cu_mask_stream: empty mask");
  std::vector<uint32_t> m(mask.begin(), mask.end());
  int prev = 0;
  TORCH_CHECK(hipGetDevice(&prev) == hipSuccess, "hipGetDevice");
  TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "hipSetDevice");
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data());
  (void)hipSetDevice(prev);
  TORCH_CHECK(e == hipSuccess, "hipExtStreamCreateWithCUMask failed: ", hipGetErrorString(e));
  return reinterpret_cast<int64_t>(s);
}

int64_t cu_count(int64_t device) {
  hipDeviceProp_t p;
  TORCH_CHECK(hipGetDeviceProperties(&p, (int)device) == hipSuccess, "hipGetDeviceProperties");
  return p.multiProcessorCount;
}

void advance_step(at::Tensor& step) { launch_advance_step(step.data_ptr<int>(), cur_stream()); }
void zero_(at::Tensor& t) {
  CHECK_DEV(t);
  CHECK_CONTIG(t);
  TORCH_CHECK(((uintptr_t)t.data_ptr() & 15) == 0, "zero_: 16-byte aligned storage expected");
  launch_zero(t.data_ptr(), (long long)t.numel() * (long long)t.element_size(), cur_stream());
}

void prefetch(const at::Tensor& t, at::Tensor& sink, int64_t blocks) {
  CHECK_DEV(t);
  CHECK_CONTIG(t);
  CHECK_DEV(sink);
  TORCH_CHECK(((uintptr_t)t.data_ptr() & 3) == 0 && sink.numel() * sink.element_size() >= 4, "prefetch: aligned tensor, 4-B sink");
  launch_prefetch(t.data_ptr(), (long long)t.numel() * (long long)t.element_size(), (int)blocks, sink.data_ptr(),
                  cur_stream());
}

void softmax_rows(const at::Tensor& S, at::Tensor& P, int64_t causal, const c10::optional<at::Tensor>& kv_lens) {
  CHECK_DEV(S); CHECK_CONTIG(S); CHECK_CONTIG(P);
  TORCH_CHECK(S.scalar_type() == at::kFloat, "softmax_rows: f32 scores");
  const int cols = (int)S.size(-1);
  const int Nq = (int)S.size(-2);
  const int rows = (int)(S.numel() / cols);
  const int* kl = nullptr;
  if (kv_lens.has_value() && kv_lens->defined()) kl = kv_lens->data_ptr<int>();
  launch_softmax_rows(S.data_ptr<float>(), bptr_mut(P), rows, cols, Nq, (int)causal, kl, cur_stream());
}

void rms_norm(const at::Tensor& x, const at::Tensor& gamma, at::Tensor& out, double eps) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(gamma); CHECK_CONTIG(out);
  const int D = (int)x.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 4096 && gamma.numel() == D, "rms_norm: D % 8 == 0, D <= 4096");
  launch_rms_norm(bptr(x), bptr(gamma), bptr_mut(out), x.numel() / D, D, (float)eps, cur_stream());
}

// qkv [B, T, (H + 2Hk) * d] -> q_out [B, T, H, d] (rotated), K (rotated) / V into the caches
// [B, L, Hk, d] at positions pos0[b] + t
void rope_kv(const at::Tensor& qkv, const at::Tensor& pos0, at::Tensor& q_out, at::Tensor& k_cache,
             at::Tensor& v_cache, int64_t H, int64_t Hk, double theta) {
  CHECK_DEV(qkv); CHECK_BF16(qkv); CHECK_BF16(q_out); CHECK_CONTIG(q_out);
  CHECK_BF16(k_cache); CHECK_CONTIG(k_cache); CHECK_BF16(v_cache); CHECK_CONTIG(v_cache);
  TORCH_CHECK(qkv.dim() == 3 && qkv.stride(2) == 1, "rope_kv: qkv [B, T, C] with contiguous rows");
  TORCH_CHECK(pos0.scalar_type() == at::kInt && pos0.is_cuda(), "rope_kv: pos0 int32 on device");
  RopeArgs a;
  a.B = (int)qkv.size(0); a.T = (int)qkv.size(1); a.H = (int)H; a.Hk = (int)Hk;
  a.d = (int)q_out.size(3); a.L = (int)k_cache.size(1);
  TORCH_CHECK(qkv.size(2) == (H + 2 * Hk) * a.d && a.d % 2 == 0, "rope_kv: qkv width");
  TORCH_CHECK(qkv.stride(1) * a.T == qkv.stride(0), "rope_kv: qkv tokens must be packed per batch");
  TORCH_CHECK(k_cache.size(0) == a.B && k_cache.size(2) == Hk && k_cache.size(3) == a.d, "rope_kv: cache shape");
  a.qkv = bptr(qkv); a.ld = qkv.stride(1); a.pos0 = pos0.data_ptr<int>();
  a.q_out = bptr_mut(q_out); a.k_cache = bptr_mut(k_cache); a.v_cache = bptr_mut(v_cache);
  a.log2_theta = (float)std::log2(theta);
  launch_rope_kv(a, cur_stream());
}

// one query token per sequence: q [B, H, d], caches [B, L, Hk, d], lens [B] -> out [B, H, d]
void lm_sample(const at::Tensor& logits, const at::Tensor& noise, const at::Tensor& eos_bias, int64_t eos,
               double temperature, int64_t k, at::Tensor& step, at::Tensor& out, at::Tensor& tok, at::Tensor& pos,
               at::Tensor& lens) {
  CHECK_DEV(logits); CHECK_CONTIG(logits); CHECK_CONTIG(noise); CHECK_CONTIG(out);
  const int64_t V = logits.size(-1);
  TORCH_CHECK(logits.numel() == V, "lm_sample: batch-1 logits [1, V]");
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16, "lm_sample: f32 / bf16 logits");
  TORCH_CHECK(noise.scalar_type() == at::kFloat && noise.numel() % V == 0, "lm_sample: noise [steps, 1, V] f32");
  TORCH_CHECK(eos_bias.scalar_type() == at::kFloat && eos_bias.numel() == noise.numel() / V,
              "lm_sample: eos_bias [steps] f32");
  TORCH_CHECK(out.scalar_type() == at::kLong && out.numel() == eos_bias.numel(), "lm_sample: out [steps, 1] int64");
  TORCH_CHECK(step.scalar_type() == at::kLong && tok.scalar_type() == at::kLong && step.numel() == 1 && tok.numel() == 1,
              "lm_sample: step / token int64 scalars");
  TORCH_CHECK(pos.scalar_type() == at::kInt && lens.scalar_type() == at::kInt, "lm_sample: pos / lens int32");
  TORCH_CHECK(k >= 1 && temperature > 0, "lm_sample: k >= 1, temperature > 0");
  launch_lm_sample(logits.data_ptr(), logits.scalar_type() == at::kFloat, (int)V, noise.data_ptr<float>(),
                   eos_bias.data_ptr<float>(), (int)eos, (float)temperature, (int)k,
                   reinterpret_cast<long long*>(step.data_ptr<int64_t>()), reinterpret_cast<long long*>(out.data_ptr<int64_t>()),
                   reinterpret_cast<long long*>(tok.data_ptr<int64_t>()), pos.data_ptr<int>(), lens.data_ptr<int>(),
                   cur_stream());
}

void decode_attention(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                      const at::Tensor& lens, at::Tensor& out, double scale) {
  CHECK_DEV(q); CHECK_BF16(q); CHECK_BF16(k_cache); CHECK_CONTIG(k_cache); CHECK_CONTIG(v_cache);
  CHECK_BF16(out);
  TORCH_CHECK(lens.scalar_type() == at::kInt && lens.is_cuda(), "decode_attention: lens int32 on device");
  DecodeArgs a;
  a.B = (int)q.size(0); a.H = (int)q.size(1); a.d = (int)q.size(2);
  a.L = (int)k_cache.size(1); a.Hk = (int)k_cache.size(2);
  TORCH_CHECK(q.stride(2) == 1 && q.stride(1) == a.d && out.stride(2) == 1 && out.stride(1) == a.d,
              "decode_attention: heads must be packed");
  TORCH_CHECK(a.d == 64 || a.d == 128, "decode_attention: head dim 64 or 128");
  TORCH_CHECK(a.H % a.Hk == 0 && a.H / a.Hk <= 8, "decode_attention: 1..8 query heads per kv head");
  a.q = bptr(q); a.q_sb = q.stride(0); a.k_cache = bptr(k_cache); a.v_cache = bptr(v_cache);
  a.lens = lens.data_ptr<int>(); a.o = bptr_mut(out); a.o_sb = out.stride(0); a.scale = (float)scale;
  const int ns = decode_splits(a.B, a.Hk, a.L);
  at::Tensor ws;
  a.ws = nullptr;
  a.tickets = nullptr;
  if (ns > 1) {
    ws = at::empty({(long long)a.B * a.H * ns * (a.d + 2)}, q.options().dtype(at::kFloat));
    a.ws = ws.data_ptr<float>();
    // arrival tickets: zeroed once per device, every kernel re-arms the ones it used
    static std::vector<at::Tensor> tickets;
    const int dev = q.get_device();
    if ((int)tickets.size() <= dev) tickets.resize(dev + 1);
    // never reallocated: a captured graph keeps pointing at it
    if (!tickets[dev].defined()) tickets[dev] = at::zeros({65536}, q.options().dtype(at::kInt));
    TORCH_CHECK((long long)a.B * a.Hk <= 65536, "decode_attention: B * kv_heads <= 65536");
    a.tickets = tickets[dev].data_ptr<int>();
  }
  launch_decode_attention(a, ns, cur_stream());
}

}  // namespace

using nogil = py::call_guard<py::gil_scoped_release>;

PYBIND11_MODULE(_C, m) {
  m.doc() = "cassmantle_amd gfx950 (CDNA4) HIP kernel library";
  // Every launcher runs without the GIL: a kernel launch can block while the device queue is
  // full behind a long generation (hundreds of eager VAE / encoder launches after a denoise
  // graph), and holding the GIL there froze the scorer thread of a serving process for the
  // whole wait (~110 ms spikes in test_legacy_stream_scorer_not_blocked_by_generation).
  m.def("gemm", &gemm, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("residual"), py::arg("out"),
        py::arg("act"), py::arg("stats"), py::arg("stats_hw"), py::arg("ln_rows") = py::none(),
        py::arg("ln_wsum") = py::none(), py::arg("ln_eps") = 0.0, py::arg("kv8") = py::none(),
        py::arg("kv8_col0") = 0, py::arg("kv8_ntok") = 0, py::arg("kv8_hk") = 0, py::arg("ln_rows_fx") = py::none(),
        py::arg("row_stats") = py::none(), py::arg("gn_stats") = py::none(), py::arg("gn_gamma") = py::none(),
        py::arg("gn_beta") = py::none(), py::arg("gn_groups") = 0, py::arg("gn_hw") = 0, py::arg("gn_eps") = 0.0, nogil());
  m.def("row_stats", &row_stats, nogil());
  m.def("gemm_cat", &gemm_cat, nogil());
  m.def("group_norm_cat", &group_norm_cat, nogil());
  m.def("gemm_set_override", [](int64_t cfg, int64_t split) { gemm_set_override((int)cfg, (int)split); });
  m.def("gemm_tune_set", [](const std::string& key, int64_t cfg, int64_t split) { gemm_tune_set(key, (int)cfg, (int)split); });
  m.def("gemm_tune_clear", []() { gemm_tune_clear(); });
  m.def("gemm_tune_size", []() { return (int64_t)gemm_tune_size(); });
  m.def("gemm_record_keys", [](bool on) { gemm_record_keys(on); });
  m.def("gemm_last_key", []() { return gemm_last_key(); });
  m.def("gemm_last_plan", []() { int c, sp; gemm_last_plan(&c, &sp); return std::vector<int64_t>{c, sp}; });
  m.def("gemm_rms", &gemm_rms, nogil());
  m.def("conv2d", &conv2d, nogil());
  m.def("conv2d_up2", &conv2d_up2, nogil());
  m.def("bmm_nt", &bmm_nt, nogil());
  m.def("group_norm", &group_norm, nogil());
  m.def("layer_norm", &layer_norm, nogil());
  m.def("embed_layer_norm", &embed_layer_norm, nogil());
  m.def("group_norm_stats", &group_norm_stats, nogil());
  m.def("channel_stats", &channel_stats, nogil());
  m.def("attention", &attention, nogil());
  m.def("attention_fp8_pack", &attention_fp8_pack, nogil());
  m.def("attention_fp8_bytes", &attention_fp8_bytes, nogil());
  m.def("gather_cosine", &gather_cosine, nogil());
  m.def("pair_cosine", &pair_cosine, nogil());
  m.def("cosine_gemv", &cosine_gemv, nogil());
  m.def("cosine_topk", &cosine_topk, nogil());
  m.def("mean_pool_l2", &mean_pool_l2, nogil());
  m.def("gaussian_blur", &gaussian_blur, nogil());
  m.def("to_uint8", &to_uint8, nogil());
  m.def("timestep_embedding", &timestep_embedding, nogil());
  m.def("gather_add", &gather_add, nogil());
  m.def("concat2", &concat2, nogil());
  m.def("silu_", &silu_, nogil());
  m.def("latent_init", &latent_init, nogil());
  m.def("finalize_latents", &finalize_latents, nogil());
  m.def("dcopy", &dcopy, nogil());
  m.def("set_fp8_attn_variant", [](int64_t v) { set_fp8_attn_variant((int)v); });
  m.def("set_attn_d40_variant", [](int64_t v) { set_attn_d40_variant((int)v); });
  m.def("gemm_set_raster", &gemm_set_raster);
  m.def("latent_step", &latent_step, nogil());
  m.def("advance_step", &advance_step, nogil());
  m.def("zero_", &zero_, nogil());
  m.def("prefetch", &prefetch, nogil());
  m.def("lm_sample", &lm_sample, nogil());
  m.def("cu_mask_stream", &cu_mask_stream);
  m.def("cu_count", &cu_count);
  m.def("softmax_rows", &softmax_rows, nogil());
  m.def("rms_norm", &rms_norm, nogil());
  m.def("rope_kv", &rope_kv, nogil());
  m.def("decode_attention", &decode_attention, nogil());
  m.attr("arch") = "gfx950";
}
