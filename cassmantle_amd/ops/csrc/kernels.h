// Host-visible launcher declarations of the gfx950 kernel library.  Kernel translation units
// (*.hip) are compiled without torch headers; bindings.cpp converts tensors to these structs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct GemmArgs {
  const uint16_t* A = nullptr;          // activations [batch][M][lda] or NHWC conv input
  const uint16_t* W = nullptr;          // weights [batch][Nw][K], K contiguous
  const uint16_t* bias = nullptr;       // [Nw] (geglu: [2N])
  const uint16_t* residual = nullptr;   // [M][ldc]
  const uint16_t* chan_bias = nullptr;  // [B][N] per-image bias (ResNet time embedding)
  int ldcb = 0;                         // chan_bias row stride (0 -> N): slices of one batched GEMM
  void* C = nullptr;                    // [batch][M][ldc] bf16 or f32
  int M = 0, N = 0, K = 0, Nw = 0;
  int lda = 0, ldc = 0, ldw = 0;      // ldw = W row stride (0 -> K)
  long long sA = 0, sW = 0, sC = 0;
  int batch = 1;
  float alpha = 1.f;
  int act = 0;
  int out_f32 = 0;
  int split = 1;                       // split-K slices (gemm_plan)
  int cfg = 0;                         // tile config index (gemm_plan)
  int raster = 0;                      // tile raster group (gemm_impl.h tile_of; 0 = compiled default)
  // implicit-GEMM convolution (conv != 0)
  int conv = 0, IH = 0, IW = 0, Cin = 0, Ho = 0, Wo = 0, stride = 1, pad = 0, ksize = 1, upsample = 0;
  // parity-upsample conv (nearest-2x upsample + 3x3 conv as four 2x2 convs on the low-res input,
  // 4/9 of the MACs): grid z = parity class 2a+b, W = [4][Cout][2][2][Cin] folded weights
  // (sW = one class), Ho/Wo = low-res size, output written at pixel (2i+a, 2j+b)
  int parity = 0;
  // fused RMSNorm of A's rows (GEMV path only): A <- A * gamma / rms(A)
  const uint16_t* rms_gamma = nullptr;
  float rms_eps = 0.f;
  // second A source (1x1 conv / linear over a channel concatenation [A | A2]): k < ka reads A
  // (row stride lda), k >= ka reads A2 (row stride lda2); ka % 64 == 0 (whole k-tiles)
  const uint16_t* A2 = nullptr;
  int lda2 = 0, ka = 0;
  // LayerNorm folded into this GEMM (A = raw rows x, W = W * gamma, bias = bias + W . beta):
  // out[m][n] = rstd[m] * (acc - mean[m] * wsum[n]) + bias[n] ...; ln_rows [M] (mean, rstd)
  // float2, ln_wsum [Nw] fp32 column sums of the folded W
  const float* ln_rows = nullptr;
  const float* ln_wsum = nullptr;
  // ln_wsum set, ln_rows null, ln_eps > 0: the row statistics are computed INSIDE the kernel from
  // the register-resident A rows (A-in-registers short-K GEMM, gemm_areg.hip, only)
  float ln_eps = 0.f;
  // folded LayerNorm whose row statistics a PRODUCER epilogue accumulated (row_stats below):
  // [M][2] int64 fixed-point (sum, sum of squares) over the K columns; mean / rstd (with ln_eps)
  // are derived in this GEMM's epilogue -- no row-statistics pass
  const long long* ln_rows_fx = nullptr;
  // row statistics of THIS GEMM's stored output (after bias / residual), for a LayerNorm-folded
  // consumer: atomically accumulated [M][2] int64 fixed-point (sum, sum of squares) over the N
  // columns (zeroed by the caller); LDS-staged bf16 epilogue only (no split-K, no GroupNorm stats)
  long long* row_stats = nullptr;
  // GroupNorm (no SiLU) of the A rows folded into the A-in-registers kernel (gemm_areg.hip only):
  // A = the raw input x, gn_stats = its producer-accumulated per-(image, channel) int64 (sum,
  // sum of squares) [M / gn_hw][K][2]; the kernel folds them to per-group mean / rstd and applies
  // x * gamma * rstd + (beta - mean * gamma * rstd) to the register-resident fragments
  const long long* gn_stats = nullptr;
  const uint16_t* gn_gamma = nullptr;
  const uint16_t* gn_beta = nullptr;
  int gn_groups = 0, gn_hw = 0;
  float gn_eps = 0.f;
  // GroupNorm statistics of the output: atomically accumulated per-(image, column) sum and
  // sum-of-squares [M / stats_hw][N][2] int64 fixed point (common.h; zeroed by the caller);
  // stats_hw = rows per image
  long long* stats = nullptr;
  int stats_hw = 0;
  // e4m3 K/V emission for the fp8 attention kernel (SDXL self-attention): output columns
  // [kv8_col0, kv8_col0 + 128 kv8_hk) are the K then V heads (64 wide) of images of kv8_ntok
  // tokens (kv8_ntok % 64 == 0); they are stored as K8 [B][Hk][ntok][64] and V8t [B][Hk][64][ntok]
  // (slot-permuted key blocks) in kv8 instead of bf16 in C (attention.hip's packed image)
  uint8_t* kv8 = nullptr;
  int kv8_col0 = 0, kv8_ntok = 0, kv8_hk = 0;
};
#define GEMM_MAX_SPLIT 16
struct GemmPlan { int cfg; int split; };
GemmPlan gemm_plan(const GemmArgs& p);
int gemm_plan_split(const GemmArgs& p);
// force a tile config (-1: cost model) and split-K factor (0: cost model) for every later plan
void gemm_set_override(int cfg, int split);
// measured tuning table: shape key (gemm_key) -> plan; key recording for the autotuner
#include <string>
std::string gemm_key(const GemmArgs& p);
void gemm_tune_set(const std::string& key, int cfg, int split);
void gemm_tune_clear();
int gemm_tune_size();
void gemm_record_keys(bool on);
std::string gemm_last_key();
void gemm_last_plan(int* cfg, int* split);
// ws: fp32 workspace of split * M * N floats when split > 1 (else may be null)
void launch_gemm(const GemmArgs& p, float* ws, hipStream_t s);

struct AttnArgs {
  const uint16_t* q; const uint16_t* k; const uint16_t* v; uint16_t* o;
  long long q_sb, q_sn, q_sh;     // element strides: batch, token, head
  long long k_sb, k_sn, k_sh;
  long long v_sb, v_sn, v_sh;
  long long o_sb, o_sn, o_sh;
  int B, H, Nq, Nk, d;
  float scale;
  int causal;
  const int* kv_lens;             // [B] or null
  int group = 1;                  // query heads per K/V head (GQA)
};
void launch_attention(const AttnArgs& a, hipStream_t s);
// head dim 512 (VAE mid-block): flash kernel; ws = attention_d512_workspace bytes (key-split
// partials for short grids, 0 otherwise)
long long attention_d512_workspace(const AttnArgs& a);
void launch_attention_d512(const AttnArgs& a, float* ws, hipStream_t s);
// fp8 (OCP e4m3) attention for head dim 64: ws = attention_fp8_workspace bytes (K8 + V8t)
long long attention_fp8_workspace(const AttnArgs& a, int Hk);
// packed = true: ws already holds K8/V8t of these K/V (attention_fp8_pack once per text
// context for cross-attention), only the attention kernel runs
void set_fp8_attn_variant(int v);
void set_attn_d40_variant(int v);
void launch_attention_fp8(const AttnArgs& a, int Hk, uint8_t* ws, hipStream_t s, bool packed = false);
void launch_attention_fp8_pack(const AttnArgs& a, int Hk, uint8_t* ws, hipStream_t s);

// norms
void launch_group_norm(const uint16_t* x, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                       float* ws, int B, long long S, int C, int G, float eps, int silu, hipStream_t s);
// GroupNorm from producer-accumulated per-channel stats ([B][Ca][2] for channels < Ca, then
// [B][C-Ca][2] from stats_b when the input is a channel concatenation); no statistics pass.
// x2 != null: the input is the concatenation [x (Ca channels) | x2 (C - Ca channels)] read from
// the two tensors (the concatenated tensor is never materialised)
void launch_group_norm_cs(const uint16_t* x, const uint16_t* x2, const long long* stats_a, int Ca, const long long* stats_b,
                          const uint16_t* gamma, const uint16_t* beta, uint16_t* y, int B, long long S, int C,
                          int G, float eps, int silu, hipStream_t s);
// per-channel stats of an NHWC tensor into zeroed int64 fixed-point [B][C][2] (for producers
// without a fused path)
void launch_channel_stats(const uint16_t* x, long long* stats, int B, long long S, int C, hipStream_t s);
long long group_norm_workspace(int B, long long S, int C);
void launch_layer_norm(const uint16_t* x, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                       long long rows, int D, float eps, hipStream_t s);
// per-row (mean, rstd) float2 of [rows][D] (LayerNorm statistics for a folded-LN GEMM)
// A-in-registers short-K GEMM (gemm_areg.hip): shapes it takes, and the launch
bool gemm_areg_ok(const GemmArgs& p);
void launch_gemm_areg(const GemmArgs& p, hipStream_t s);
void launch_row_stats(const uint16_t* x, float* stats, long long rows, int D, float eps, hipStream_t s);
// fused encoder input layer: y[r] = LN(word[ids[r]] + pos[r % seq] + add) (bf16, D % 8 == 0)
void launch_embed_layer_norm(const uint16_t* word, const long long* ids, const uint16_t* pos, int seq,
                             const uint16_t* add, const uint16_t* gamma, const uint16_t* beta, uint16_t* y,
                             long long rows, int D, float eps, hipStream_t s);
void launch_rms_norm(const uint16_t* x, const uint16_t* gamma, uint16_t* y, long long rows, int D, float eps,
                     hipStream_t s);

// decode path (lm.hip)
bool launch_gemv(const GemmArgs& p, hipStream_t s);   // false -> shape not handled (M > 8, conv, ...)
struct RopeArgs {
  const uint16_t* qkv; long long ld;   // [B*T][ld], heads [q | k | v] x d
  const int* pos0;                     // [B] first position of this chunk (null -> 0)
  uint16_t* q_out;                     // [B][T][H][d]
  uint16_t* k_cache; uint16_t* v_cache;   // [B][L][Hk][d]
  int B, T, H, Hk, d, L;
  float log2_theta;
};
void launch_rope_kv(const RopeArgs& a, hipStream_t s);
struct DecodeArgs {
  const uint16_t* q; long long q_sb;   // [B][H][d] (batch stride q_sb)
  const uint16_t* k_cache; const uint16_t* v_cache;   // [B][L][Hk][d]
  const int* lens;                     // [B] valid keys (device)
  uint16_t* o; long long o_sb;         // [B][H][d]
  float* ws;                           // split partials [B*H][ns][d+2]
  int* tickets;                        // [B*Hk] zeroed arrival counters (re-armed by the kernel)
  int B, H, Hk, d, L;
  float scale;
};
int decode_splits(int B, int Hk, int L);
// decode-step sampler (batch 1): top-k of logits / T (+ EOS bias of the step) + Gumbel-max with
// the step's noise row, then token / position / length / step counter updated on the device
void launch_lm_sample(const void* logits, int logits_f32, int V, const float* noise, const float* eos_bias, int eos,
                      float temperature, int k, long long* step, long long* out, long long* tok, int* pos, int* lens,
                      hipStream_t s);
void launch_decode_attention(const DecodeArgs& a, int ns, hipStream_t s);

// scorer
void launch_gather_cosine(const void* table, int table_f32, int D, const int* ia, const int* ib,
                          float* out, int n, hipStream_t s);
void launch_pair_cosine(const float* a, const float* b, int D, float* out, int n, hipStream_t s);
void launch_cosine_gemv(const void* table, int table_f32, int V, int D, const void* vec, int vec_f32,
                        float* out, hipStream_t s);
int cosine_topk_workspace(int V, int k);
void launch_cosine_topk(const void* table, int table_f32, int V, int D, const void* vec, int vec_f32, int k,
                        unsigned long long* ws, float* vals, long long* idx, hipStream_t s);
void launch_mean_pool_l2(const uint16_t* h, const int* lens, float* out, int B, int T, int D, hipStream_t s);

// image / diffusion glue
void launch_gaussian_blur(const void* img, int u8, int H, int W, int C, const float* w, int R,
                          float* tmp, void* out, hipStream_t s);
void launch_to_uint8(const uint16_t* x, uint8_t* out, long long n, hipStream_t s);
void launch_timestep_embedding(const float* t, void* out, int B, int dim, int flip, float shift, int out_bf16,
                               hipStream_t s);
void launch_gather_add(const uint16_t* table, const int* ids, const uint16_t* pos, int seq, int D, long long rows,
                       uint16_t* out, hipStream_t s);
void launch_concat2(const uint16_t* a, int Da, const void* b, int Db, int b_f32, long long rows, uint16_t* out,
                    hipStream_t s);
void launch_silu_bf16(uint16_t* x, long long n, hipStream_t s);
void launch_latent_init(const float* x0, float c_in0, float* x, float* xs, float* hist, int nhist, uint16_t* unet_in,
                        long long n, int cfg, int cin, int cstride, hipStream_t s);
void launch_copy(const void* src, void* dst, long long bytes, hipStream_t s);
void launch_finalize_latents(const float* x, uint16_t* z, long long n, uint8_t* finite, hipStream_t s);
// CFG combine + scheduler update + next UNet input (channel-padded to cstride); the optional
// tables' rows for step+1 (time conditioning) are copied into buf0/buf1 by extra blocks
void launch_latent_step(const uint16_t* eps, float* x, float* hist, float* xs, const float* coef, const int* step,
                        uint16_t* unet_in, long long n, int cfg, int cin, int cstride, const void* tab0, void* buf0,
                        long long row_bytes0, const void* tab1, void* buf1, long long row_bytes1, int rows,
                        hipStream_t s);
void launch_advance_step(int* step, hipStream_t s);
void launch_zero(void* p, long long bytes, hipStream_t s);
void launch_prefetch(const void* p, long long bytes, int blocks, void* sink, hipStream_t s);
void launch_softmax_rows(const float* S, uint16_t* P, int rows, int cols, int Nq, int causal,
                         const int* kv_lens, hipStream_t s);
