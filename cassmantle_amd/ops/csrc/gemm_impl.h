// MFMA bf16 GEMM / implicit-GEMM convolution with fused epilogues.
//
//   D[n][m] = sum_k W[n][k] * A[m][k]          (computed transposed so each lane owns 4
//   C[m][n] = act(alpha*D + bias[n] + cb[b][n])  consecutive output channels of one row ->
//             (+ residual[m][n])                 8-byte NHWC stores)
//
// * A is either a row-major activation matrix (linear layers, 1x1 convs) or an NHWC image read
//   through an implicit im2col (3x3 convs, stride-2 downsamplers, and the nearest-2x upsample
//   fused into the address generation: the upsampled tensor never exists).
// * W rows are K-contiguous ([Cout][kh][kw][Cin] for convs), so both operands are read from
//   LDS as 16-byte k-chunks: mfma_f32_16x16x32_bf16 fragments straight from ds_read_b128.
// * Global -> LDS by LDS-DMA (global_load_lds_dwordx4, cdna_hip_programming.md §5): no VGPR
//   staging, no ds_write; each wave-instruction fills 8 rows x 128 B.  Out-of-range rows and
//   conv padding point their lane at a 16-byte zero page.
//   - STAGES=2: the next k-tile's DMA is issued before the current tile's MFMAs; one
//     __syncthreads (= vmcnt(0) + barrier) per k-tile.
//   - STAGES=3: two tiles in flight; a counted `s_waitcnt vmcnt(N)` retires only the tile about
//     to be read and a raw s_barrier publishes it, so one DMA stays in flight across every
//     barrier ("Pipelining across barriers", guide §5).
// * LDS rows are 128 B; logical chunk c of row r lives in slot c ^ ((r >> 1) & 7).  The DMA
//   image is lane-linear, so the swizzle is applied on the SOURCE address (rule 21) and the
//   same XOR on the ds_read; each 16-lane ds_read_b128 group then hits 16 distinct bank slots.
// * Tiles (BM x BN x 64, 4 waves as WM x WN): 128x128 (2x2), 256x64 (4x1) for N = 64 (mod
//   128), 256x16 (4x1) for the 3/4-channel conv_out layers.
// * Split-K: grids that cannot fill the 256 CUs (the 16x16 / 8x8 UNet levels: M = 2048 / 512
//   with K = 11520) split the k-tiles over blockIdx.y; fp32 partial slabs are summed by a
//   second kernel that applies the epilogue (cheaper than a sub-occupied chip).
// * GroupNorm statistics of the output (p.stats) are accumulated in the epilogue, so a
//   following GroupNorm needs no statistics pass over the activation.
// * GEGLU (transformer FF): W tile rows interleave 16-row value/gate blocks, so each lane
//   holds h and g of the same output column and computes h * gelu(g) in registers.
// * Block ids are remapped XCD-aware so tiles that share an A panel run on one XCD's L2.
#pragma once
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

#ifndef GEMM_DIAG_APRO
#define GEMM_DIAG_APRO 0
#endif
#ifndef GEMM_FRAG_PREFETCH
#define GEMM_FRAG_PREFETCH 0
#endif

namespace {

__device__ uint4 g_zero_page[4];   // zero-initialised (per translation unit); padded / out-of-range chunks

constexpr int BK = 64;

CM_DEVICE int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// tile of linear (XCD-remapped) index lin: rows of N-tiles (G = 1: tm = lin / nN), or groups of G
// M-tiles walked column by column, so the 32 consecutive tiles an XCD runs cover G M-panels x
// 32/G N-panels instead of 2 x 16 (less A+W per XCD L2 on small grids).  G = p.raster, or
// GEMM_RASTER_G when 0.  G = 4 measured 524.9 -> 521.6 ms/step on the bench, same box x2
// (profiles/r5_raster_ab.txt)
// Warp-specialised tiles (NP > 0): the MFMA waves issue no global loads in the mainloop, so at the
// kernel start they read their block's W panel once (one dword per 64-B line, the block's k
// range; GEMM_PF_SELF 2: only the quarter selected by tm & 3, the M tiles of one XCD's raster
// group sharing the panel) to bring the weights to L2 / MALL while the DMA ring starts.  The
// loads are waited for only at the end (their XOR feeds an empty asm): a cold weight's HBM
// latency then overlaps the ring instead of stalling k-tiles.
#ifndef GEMM_PF_SELF
#define GEMM_PF_SELF 0
#endif
#ifndef GEMM_RASTER_G
#define GEMM_RASTER_G 4
#endif
CM_DEVICE void tile_of(int lin, int nM, int nN, int raster, int& tm, int& tn) {
  const int G = min(raster > 0 ? raster : GEMM_RASTER_G, nM);
  if (G > 1) {
    const int grp = lin / (G * nN);
    const int gs = min(G, nM - grp * G);
    const int r = lin - grp * G * nN;
    tm = grp * G + r % gs;
    tn = r / gs;
  } else {
    tn = lin % nN;
    tm = lin / nN;
  }
}

typedef __attribute__((address_space(3))) void lds_void;

CM_DEVICE void glds16(const void* src, uint4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_void*)lds_wave_base, 16, 0, 0);
}

// buffer-resource LDS-DMA: 16 B per lane to lds_wave_base + 16*lane, source rsrc + voff + soff
// (device-only helper: the address-space cast must not appear in a host-instantiated body)
CM_DEVICE void blds16(__amdgpu_buffer_rsrc_t rs, uint4* lds_wave_base, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds_wave_base, 16, voff, soff, 0, 0);
}

CM_DEVICE __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <int N>
CM_DEVICE void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

CM_DEVICE void add4(float* o, uint2 v) {
  o[0] += bf2f(v.x & 0xffff); o[1] += bf2f(v.x >> 16); o[2] += bf2f(v.y & 0xffff); o[3] += bf2f(v.y >> 16);
}

// folded LayerNorm (p.ln_rows, or p.ln_rows_fx from a producer epilogue): o = rstd_m * (acc -
// mean_m * wsum[n..n+3]) for the W rows n..n+3
// inv_k = 1 / K (callers hoist it: an fp64 division per row was a ~20-instruction sequence)
CM_DEVICE float2 ln_row(const GemmArgs& p, int m, double inv_k) {
  if (p.ln_rows_fx != nullptr) {
    // the fixed-point sums are exact; mean and var = q / K - mean^2 are formed in fp64, so rows
    // with |mean| >> std keep their variance (fp32 lost ~log2(mean^2 / var) bits of it to the
    // cancellation).  This runs once per ROW of the LDS-staged epilogue (the per-4-
    // column form of round 3 pushed the 256x256 ping-pong tiles into scratch;
    // tests/test_kernel_registers.py guards it)
    const longlong2 v = reinterpret_cast<const longlong2*>(p.ln_rows_fx)[m];
    const double mean = (double)v.x * (inv_k * (1.0 / STAT_SCALE_SUM));
    const double var = fmax((double)v.y * (inv_k * (1.0 / STAT_SCALE_SQ)) - mean * mean, 0.0);
    return make_float2((float)mean, rsqrtf((float)var + p.ln_eps));
  }
  return reinterpret_cast<const float2*>(p.ln_rows)[m];
}
CM_DEVICE void ln_apply4(float2 ms, const float* __restrict__ wsum, float* o) {
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = ms.y * fmaf(-ms.x, wsum[r], o[r]);
}
CM_DEVICE void ln_fold4(const GemmArgs& p, int m, int wn, float* o) {
  const float2 ms = ln_row(p, m, 1.0 / (double)p.K);
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = ms.y * fmaf(-ms.x, p.ln_wsum[wn + r], o[r]);
}

// output row of GEMM row m.  Parity-upsample mode (p.parity, nearest-2x upsample + 3x3 conv as
// four 2x2 convs on the low-res input, one per output parity class z = 2a + b = blockIdx.z):
// GEMM row m = (image, i, j) of the low-res grid writes output pixel (2i + a, 2j + b).
CM_DEVICE long long out_row(const GemmArgs& p, int m, int z) {
  if (!p.parity) return m;
  const int hw = p.Ho * p.Wo;
  const int img = m / hw;
  const int r = m - img * hw;
  const int i = r / p.Wo, j = r - i * p.Wo;
  return ((long long)img * 2 * p.Ho + 2 * i + (z >> 1)) * (2 * p.Wo) + 2 * j + (z & 1);
}

// epilogue for 4 consecutive output columns n..n+3 of row m (raw accumulators in o)
template <bool OUTF32>
CM_DEVICE void epilogue4(const GemmArgs& p, int batch, int m, int n, float* o) {
  const int hw = p.Ho * p.Wo;
  const int bimg = (p.chan_bias != nullptr) ? (m / hw) : 0;
  const long long cbs = p.ldcb ? p.ldcb : p.N;
  const bool full = (n + 4 <= p.N) && (p.N % 4 == 0) && (p.ldc % 4 == 0) && (cbs % 4 == 0);
  const long long om = out_row(p, m, batch);
  if (p.ln_rows || p.ln_rows_fx) ln_fold4(p, m, n, o);
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] *= p.alpha;
  if (full) {
    if (p.bias) add4(o, *reinterpret_cast<const uint2*>(p.bias + n));
    if (p.chan_bias) add4(o, *reinterpret_cast<const uint2*>(p.chan_bias + (long long)bimg * cbs + n));
    if (p.act != ACT_NONE) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = apply_act(o[r], p.act);
    }
    if (p.residual) add4(o, *reinterpret_cast<const uint2*>(p.residual + om * p.ldc + n));
    if (!OUTF32 && kv8_store4(p, m, n, o)) return;
    if constexpr (OUTF32) {
      float* C = reinterpret_cast<float*>(p.C) + (long long)batch * p.sC + om * p.ldc + n;
      *reinterpret_cast<float4*>(C) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
      uint16_t* C = reinterpret_cast<uint16_t*>(p.C) + (long long)batch * p.sC + om * p.ldc + n;
      *reinterpret_cast<uint2*>(C) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
    }
  } else {   // ragged N (3-channel conv_out): element-wise tail
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (n + r >= p.N) break;
      float v = o[r];
      if (p.bias) v += bf2f(p.bias[n + r]);
      if (p.chan_bias) v += bf2f(p.chan_bias[(long long)bimg * cbs + n + r]);
      v = apply_act(v, p.act);
      if (p.residual) v += bf2f(p.residual[om * p.ldc + n + r]);
      if constexpr (OUTF32)
        reinterpret_cast<float*>(p.C)[(long long)batch * p.sC + om * p.ldc + n + r] = v;
      else
        reinterpret_cast<uint16_t*>(p.C)[(long long)batch * p.sC + om * p.ldc + n + r] = f2bf(v);
    }
  }
}

// Per-fragment forms of the direct epilogue.  They stay INLINE: an out-of-line call gives the
// kernel a stack (scratch) and measured 1.5-2x slower on every GEMM; the unrolled loop they sit
// in exceeds the default pragma-unroll size limit, so build.py raises it
// (-mllvm -pragma-unroll-threshold) rather than let the accumulators go to scratch.
template <bool OUTF32>
CM_DEVICE void epilogue4_call(const GemmArgs& p, int batch, int m, int n, f32x4_t v) {
  float o[4] = {v[0], v[1], v[2], v[3]};
  epilogue4<OUTF32>(p, batch, m, n, o);
}

CM_DEVICE void gated_epilogue4_call(const GemmArgs& p, int batch, int m, int n, f32x4_t hv, f32x4_t gv) {
  float o[4], hh[4] = {hv[0], hv[1], hv[2], hv[3]}, gg[4] = {gv[0], gv[1], gv[2], gv[3]};
  if (p.ln_rows || p.ln_rows_fx) { ln_fold4(p, m, n, hh); ln_fold4(p, m, p.N + n, gg); }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float h = hh[r], g = gg[r];
    if (p.bias) { h += bf2f(p.bias[n + r]); g += bf2f(p.bias[p.N + n + r]); }
    o[r] = gate_f(h, g, p.act);
  }
  uint16_t* C = reinterpret_cast<uint16_t*>(p.C) + (long long)batch * p.sC + (long long)m * p.ldc + n;
  if (p.residual) add4(o, *reinterpret_cast<const uint2*>(p.residual + (long long)m * p.ldc + n));
  *reinterpret_cast<uint2*>(C) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
}

// Shared tile epilogue of the MFMA GEMM kernels: acc[TI][TJ] holds, for W subtile i and A
// subtile j of wave (wm, wn), D[n][m] with n = n0 + wn*(BN/WN) + 16i + 4*(lane>>4) + r and
// m = m0 + wm*(BM/WM) + 16j + (lane&15).  bf16 outputs without split are staged through LDS
// (smem, >= BM*(OBN+8)*2 bytes) and stored as full 16-byte row chunks (+ residual, + GroupNorm
// statistics); fp32 / split-K / ragged outputs take the direct path.
// SPLIT_DIRECT: the caller guarantees the direct path only ever stores split-K partial slabs
// (bf16, N % 8 == 0 outputs always take the LDS path), which keeps the kernel small.
// has_acc: false for the DMA-only producer waves of a warp-specialised tile (no accumulators;
// they still take part in the LDS-staged store pass)
template <int BM, int BN, int WM, int WN, bool GEGLU, bool OUTF32, int TI, int TJ, int THREADS, bool SPLIT_DIRECT = false>
CM_DEVICE void tile_epilogue(const GemmArgs& p, f32x4_t (&acc)[TI][TJ], uint4* smem, float* __restrict__ partial,
                             int m0, int n0, int batch, int wm, int wn, int tid, int nsplit, int split_id,
                             bool has_acc = true) {
  const int lane = tid & 63;
  const int fr = lane & 15, fq = lane >> 4;
  // ---- LDS-staged epilogue (bf16 output, no split): the MFMA layout gives each lane 4
  // consecutive columns of one row (8-byte stores, 32 B per row per instruction); instead the
  // tile is written to LDS (bias / time-bias / activation applied in registers) and streamed out
  // as full rows of 16-byte stores, residual added in the same coalesced pass.
  if constexpr (!OUTF32) {
    constexpr int OBN = GEGLU ? BN / 2 : BN;   // output columns of this tile
    constexpr int OST = OBN + 8;               // LDS row stride (elements): 16-B pad
    const long long cbs = p.ldcb ? p.ldcb : p.N;
    const bool lds_ok = nsplit == 1 && (p.N % 8 == 0) && (p.ldc % 8 == 0) && (cbs % 4 == 0);
    if (lds_ok) {
      __syncthreads();                        // every wave is done with the staging buffers
      uint16_t* T = reinterpret_cast<uint16_t*>(smem);
      const int hw = p.Ho * p.Wo;
      const double inv_k = 1.0 / (double)p.K;
      if (has_acc) {
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int ml = wm * (BM / WM) + 16 * j + fr;
        const int m = m0 + ml;
        const int bimg = (p.chan_bias != nullptr && m < p.M) ? (m / hw) : 0;
        // folded LayerNorm: this row's (mean, rstd), once per row (not per 4-column group)
        const bool lnf = (p.ln_rows != nullptr || p.ln_rows_fx != nullptr) && m < p.M;
        const float2 lnm = lnf ? ln_row(p, m, inv_k) : make_float2(0.f, 1.f);
        if constexpr (GEGLU) {
#pragma unroll
          for (int pi = 0; pi < TI / 2; ++pi) {
            const int nl = wn * (BN / WN / 2) + 16 * pi + 4 * fq;
            const int n = n0 + nl;
            float o[4], hh[4], gg[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) { hh[r] = acc[2 * pi][j][r]; gg[r] = acc[2 * pi + 1][j][r]; }
            if (lnf && n < p.N) { ln_apply4(lnm, p.ln_wsum + n, hh); ln_apply4(lnm, p.ln_wsum + p.N + n, gg); }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float h = hh[r], g = gg[r];
              if (p.bias && n < p.N) { h += bf2f(p.bias[n + r]); g += bf2f(p.bias[p.N + n + r]); }
              o[r] = gate_f(h, g, p.act);
            }
            *reinterpret_cast<uint2*>(T + ml * OST + nl) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
          }
        } else {
#pragma unroll
          for (int i = 0; i < TI; ++i) {
            const int nl = wn * (BN / WN) + 16 * i + 4 * fq;
            const int n = n0 + nl;
            float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            if (lnf && n < p.N) ln_apply4(lnm, p.ln_wsum + n, o);
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] *= p.alpha;
            if (n < p.N && m < p.M) {
              if (p.bias) add4(o, *reinterpret_cast<const uint2*>(p.bias + n));
              if (p.chan_bias) add4(o, *reinterpret_cast<const uint2*>(p.chan_bias + (long long)bimg * cbs + n));
              if (p.act != ACT_NONE) {
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = apply_act(o[r], p.act);
              }
            }
            *reinterpret_cast<uint2*>(T + ml * OST + nl) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
          }
        }
      }
      }
      __syncthreads();
      constexpr int CPR = OBN / 8;              // 16-byte chunks per tile row
      uint16_t* Cb = reinterpret_cast<uint16_t*>(p.C) + (long long)batch * p.sC;
      auto finish = [&](int row, int c8) -> uint4 {   // residual add + store of one 16-B chunk
        const int m = m0 + row, n = n0 + c8 * 8;
        const long long om = out_row(p, m, batch);
        uint4 v = *reinterpret_cast<const uint4*>(T + row * OST + c8 * 8);
        if (p.residual) {
          const uint4 rv = *reinterpret_cast<const uint4*>(p.residual + om * p.ldc + n);
          float a[8], b[8];
          unpack8(v, a);
          unpack8(rv, b);
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] += b[e];
          v = pack8(a);
        }
        if (p.kv8 != nullptr && n >= p.kv8_col0) {   // K / V columns: e4m3 attention image only
          if (n < p.kv8_col0 + 64 * p.kv8_hk) {       // K: 8 bytes of key m's 64-byte row
            float a[8];
            unpack8(v, a);
            const int rel = n - p.kv8_col0, b = m / p.kv8_ntok, key = m - b * p.kv8_ntok;
            const long long bh = (long long)b * p.kv8_hk + (rel >> 6);
            *reinterpret_cast<uint2*>(p.kv8 + (bh * p.kv8_ntok + key) * 64 + (rel & 63)) =
                make_uint2(f8x4(a[0], a[1], a[2], a[3]), f8x4(a[4], a[5], a[6], a[7]));
          }                                            // V: transposed pass below
          return v;
        }
        *reinterpret_cast<uint4*>(Cb + om * p.ldc + n) = v;
        return v;
      };
      if (p.stats == nullptr) {
        for (int c = tid; c < BM * CPR; c += THREADS) {
          const int row = c / CPR, c8 = c - row * CPR;
          if (m0 + row >= p.M || n0 + c8 * 8 >= p.N) continue;
          const uint4 v = finish(row, c8);
          if (p.row_stats != nullptr) *reinterpret_cast<uint4*>(T + row * OST + c8 * 8) = v;   // stored values
        }
        if (p.row_stats != nullptr) {
          // LayerNorm row statistics of the stored tile for a folded consumer (p.ln_rows_fx there):
          // one thread per row sums its OBN stored values, one fixed-point atomic pair per row
          __syncthreads();
          for (int row = tid; row < BM; row += THREADS) {
            const int m = m0 + row;
            if (m >= p.M) break;
            float sm = 0.f, sq = 0.f;
            for (int c8 = 0; c8 < CPR && n0 + c8 * 8 < p.N; ++c8) {
              float f[8];
              unpack8(*reinterpret_cast<const uint4*>(T + row * OST + c8 * 8), f);
#pragma unroll
              for (int e = 0; e < 8; ++e) { sm += f[e]; sq = fmaf(f[e], f[e], sq); }
            }
            stat_atomic_add(p.row_stats + 2LL * m, 0, sm);
            stat_atomic_add(p.row_stats + 2LL * m + 1, 1, sq);
          }
        }
        if (p.kv8 != nullptr && n0 + OBN > p.kv8_col0 + 64 * p.kv8_hk) {
          // V columns -> V8t rows: d-row of a 64-key block = 64 slot-ordered bytes, written as
          // 16-byte runs of 16 slots gathered from the bf16 tile in LDS (key blocks never
          // straddle images: tokens per image and BM are multiples of 64)
          const int vc0 = p.kv8_col0 + 64 * p.kv8_hk;
          const long long Bimg = p.M / p.kv8_ntok;
          uint8_t* V8t = p.kv8 + Bimg * p.kv8_hk * p.kv8_ntok * 64;
          for (int it = tid; it < OBN * (BM / 64) * 4; it += THREADS) {
            const int col = it % OBN, sg = (it / OBN) & 3, kb = it / (OBN * 4);
            const int n = n0 + col, mb = m0 + kb * 64;
            if (n < vc0 || n >= p.N || mb >= p.M) continue;
            uint32_t w[4];
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
              float f[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int j = sg * 16 + q4 * 4 + e;           // slot 32h + j' of the block
                const int h = j >> 5, jj = j & 31;
                const int kk = 32 * (jj >> 4) + (jj & 3) + 8 * ((jj & 15) >> 2) + 4 * h;
                f[e] = bf2f(T[(kb * 64 + kk) * OST + col]);
              }
              w[q4] = f8x4(f[0], f[1], f[2], f[3]);
            }
            const int b = mb / p.kv8_ntok, key0 = mb - b * p.kv8_ntok;
            const long long bh = (long long)b * p.kv8_hk + ((n - vc0) >> 6);
            *reinterpret_cast<uint4*>(V8t + (bh * 64 + ((n - vc0) & 63)) * p.kv8_ntok + key0 + sg * 16) =
                make_uint4(w[0], w[1], w[2], w[3]);
          }
        }
        return;
      }
      // GroupNorm statistics of the stored output (consumer: group_norm with stats): each thread
      // owns one 8-column chunk and walks rows; per-(image, column) sum / sum-of-squares are
      // reduced over the row lanes in LDS and added to p.stats[image][n][2] with one atomic per
      // column per tile (tiles that straddle images flush per thread instead).
      constexpr int RL = THREADS / CPR;          // row lanes
      const int c8 = tid % CPR, r0 = tid / CPR;
      const int n = n0 + c8 * 8;
      const bool lane_on = r0 < RL && n < p.N;
      const int shw = p.stats_hw;
      const int mlast = min(m0 + BM, p.M) - 1;
      const int img0 = m0 / shw;
      const bool single = img0 == mlast / shw;
      float s8[8], q8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { s8[e] = 0.f; q8[e] = 0.f; }
      int cur = -1;
      auto flush = [&]() {
        if (cur < 0) return;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          stat_atomic_add(p.stats + ((long long)cur * p.N + n + e) * 2 + 0, 0, s8[e]);
          stat_atomic_add(p.stats + ((long long)cur * p.N + n + e) * 2 + 1, 1, q8[e]);
          s8[e] = 0.f;
          q8[e] = 0.f;
        }
      };
      if (lane_on) {
        for (int row = r0; row < BM; row += RL) {
          const int m = m0 + row;
          if (m >= p.M) break;
          const uint4 v = finish(row, c8);
          if (!single) {
            const int img = m / shw;
            if (img != cur) { flush(); cur = img; }
          }
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) { s8[e] += f[e]; q8[e] = fmaf(f[e], f[e], q8[e]); }
        }
      }
      if (!single) {
        flush();
        return;
      }
      __syncthreads();                          // T fully consumed: reuse LDS for the reduction
      float* R = reinterpret_cast<float*>(smem);   // [2][RL][OBN]
      if (r0 < RL) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          R[r0 * OBN + c8 * 8 + e] = s8[e];
          R[(RL + r0) * OBN + c8 * 8 + e] = q8[e];
        }
      }
      __syncthreads();
      for (int c = tid; c < 2 * OBN; c += THREADS) {
        const int stat = c / OBN, col = c - stat * OBN;
        if (n0 + col >= p.N) continue;
        float a = 0.f;
        for (int r = 0; r < RL; ++r) a += R[(stat * RL + r) * OBN + col];
        stat_atomic_add(p.stats + ((long long)img0 * p.N + n0 + col) * 2 + stat, stat, a);
      }
      return;
    }
  }

  // ---- direct epilogue (fp32 outputs, split-K partial slabs, ragged N)
  if (!has_acc) return;
  if constexpr (SPLIT_DIRECT) {
    if constexpr (!GEGLU) {
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int m = m0 + wm * (BM / WM) + 16 * j + fr;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int n = n0 + wn * (BN / WN) + 16 * i + 4 * fq;
          if (m < p.M && n < p.N) {
            float* dst = partial + (((long long)batch * nsplit + split_id) * p.M + m) * p.N + n;
            *reinterpret_cast<float4*>(dst) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int m = m0 + wm * (BM / WM) + 16 * j + fr;
    if (m >= p.M) continue;
    if constexpr (GEGLU) {
#pragma unroll
      for (int pi = 0; pi < TI / 2; ++pi) {
        const int n = n0 + wn * (BN / WN / 2) + 16 * pi + 4 * fq;
        if (n >= p.N) continue;
        gated_epilogue4_call(p, batch, m, n, acc[2 * pi][j], acc[2 * pi + 1][j]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int n = n0 + wn * (BN / WN) + 16 * i + 4 * fq;
        if (n >= p.N) continue;
        float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (nsplit > 1) {               // split-K: raw fp32 partial slab
          float* dst = partial + (((long long)batch * nsplit + split_id) * p.M + m) * p.N + n;
          *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
          epilogue4_call<OUTF32>(p, batch, m, n, acc[i][j]);
        }
      }
    }
  }
}

// 4-wave blocks with 2 LDS stages run 2 per CU; deeper rings (STAGES 3-5, one block per CU)
// keep STAGES-2 k-tiles of DMA in flight across every barrier: the short-K / small-grid UNet
// GEMMs (K = 320..1280, <= 2 tiles per CU) are bound by the per-k-tile DMA latency, not by
// MFMA, and a 2-stage loop exposes that latency once per k-tile.
//
// NP > 0 (deep rings only): a warp-specialised block of NW MFMA waves plus NP DMA-only producer
// waves.  The LDS-DMA fill rate of a CU is set by the waves issuing it (22 / 37 / 48 B/cycle for
// 4 / 8 / 16 issuing waves, profiles/r3_lds_fill_probe.jsonl), and on the small-grid tiles the MFMA
// waves also issued the DMA between their fragment reads and MFMAs; with producers the MFMA waves
// only read LDS and run MFMAs, and the producers only stage (same ring, same barrier per k-tile).
template <int BM, int BN, int WM, int WN, int CONV, bool GEGLU, bool OUTF32, int STAGES, bool BUF, int NP = 0>
__global__ void __launch_bounds__(64 * (WM * WN + NP), (WM * WN == 4 && STAGES == 2 && NP == 0) ? 2 : 1)
gemm_kernel(GemmArgs p, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  constexpr int NW = WM * WN;
  constexpr int THREADS = 64 * (NW + NP);
  constexpr int NSW = NP ? NP : NW;        // staging waves
  static_assert(NP == 0 || (STAGES >= 3 && BUF), "producer waves: buffer-resource deep rings only");
  constexpr int RR = 8 * NSW;              // rows covered by one DMA round (8 per staging wave)
  constexpr int TILE = (BM + BN) * 8;      // uint4 per buffer
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int TI = BN / WN / 16;         // n-subtiles per wave
  constexpr int TJ = BM / WM / 16;         // m-subtiles per wave
  static_assert(!GEGLU || (TI % 2 == 0), "geglu pairs");
  static_assert(BM % RR == 0, "A rows in whole DMA rounds");
  constexpr int AR = BM / RR;              // A DMA rounds
  constexpr int WR = (BN + RR - 1) / RR;   // W DMA rounds (the last may cover only some waves)
  static_assert(STAGES >= 2 && STAGES <= 5, "stages");
  constexpr int NPT = AR + WR;             // DMA instructions per k-tile of a wave in every round

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform
  const int wm = wave % WM, wn = wave / WM;
  const bool mma_wave = NP == 0 || wave < NW;                  // has accumulators / runs MFMAs
  const bool dma_wave = NP == 0 || wave >= NW;                 // stages k-tiles
  const int swave = NP ? (dma_wave ? wave - NW : 0) : wave;    // index among the staging waves

  const int nN = GEGLU ? (p.N + BN / 2 - 1) / (BN / 2) : (p.N + BN - 1) / BN;
  const int nM = (p.M + BM - 1) / BM;
  const int lin = xcd_remap(blockIdx.x, nN * nM);
  int tn, tm;
  tile_of(lin, nM, nN, p.raster, tm, tn);
  const int batch = blockIdx.z;
  const int m0 = tm * BM;
  const int n0 = GEGLU ? tn * (BN / 2) : tn * BN;   // output-column origin

  const uint16_t* __restrict__ A = p.A + (long long)batch * p.sA;
  const uint16_t* __restrict__ W = p.W + (long long)batch * p.sW;
  const int ldw = p.ldw ? p.ldw : p.K;
  const void* zp = (const void*)g_zero_page;

  // ---- this lane's DMA rows: round i covers rows 32i + 8*wave + (lane>>3), slot lane&7
  const int slot = lane & 7;
  const int rsub = 8 * swave + (lane >> 3);
  const bool w_last_round = (RR * (WR - 1) + 8 * swave) < BN;  // this wave stages the last W round
  // Per-row state is computed ONCE; the per-k-tile address work is then a few VALU ops per DMA
  // (the first version recomputed divisions per tile and was issue-bound on SALU/VALU:
  // 15 SALU + 9 VALU per MFMA in the rocprof counters).
  int a_chunk[AR];
  long long a_off[AR];       // plain: row*lda + chunk*8 ; conv: element offset of pixel (b,cy,cx) + chunk*8
  int cy_[AR], cx_[AR], cbh_[AR];
  bool a_ok[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int r = RR * i + rsub;
    const int row = m0 + r;
    a_chunk[i] = slot ^ ((r >> 1) & 7);
    a_ok[i] = row < p.M;
    if constexpr (CONV == 0) {
      a_off[i] = (long long)row * p.lda + a_chunk[i] * 8;
    } else {
      const int m = a_ok[i] ? row : 0;
      const int hw = p.Ho * p.Wo;
      const int b = m / hw;
      const int rr = m - b * hw;
      const int oy = rr / p.Wo;
      const int ox = rr - oy * p.Wo;
      // parity-upsample mode: 2x2 taps at offsets {a-1, a} x {b-1, b} (pad 1-a / 1-b)
      const int pad_y = p.parity ? 1 - (batch >> 1) : p.pad;
      const int pad_x = p.parity ? 1 - (batch & 1) : p.pad;
      cy_[i] = oy * p.stride - pad_y;
      cx_[i] = ox * p.stride - pad_x;
      cbh_[i] = b * p.IH;
      a_off[i] = (((long long)b * p.IH + cy_[i]) * p.IW + cx_[i]) * p.Cin + a_chunk[i] * 8;
      if (!a_ok[i]) cy_[i] = -(1 << 28);   // never in bounds
    }
  }
  int w_row[WR], w_chunk[WR];
#pragma unroll
  for (int i = 0; i < WR; ++i) {
    const int r = RR * i + rsub;
    w_chunk[i] = slot ^ ((r >> 1) & 7);
    int gr = -1;
    if (r < BN) {
      if constexpr (GEGLU) {
        const int blk = r >> 4, within = r & 15;
        const int nout = n0 + (blk >> 1) * 16 + within;
        gr = (nout < p.N) ? ((blk & 1) ? p.N + nout : nout) : -1;
      } else {
        const int n = n0 + r;
        gr = n < p.Nw ? n : -1;
      }
    }
    w_row[i] = gr;
  }
  long long w_off[WR];
#pragma unroll
  for (int i = 0; i < WR; ++i) w_off[i] = (long long)(w_row[i] < 0 ? 0 : w_row[i]) * ldw + w_chunk[i] * 8;
  const int Hv = p.upsample ? 2 * p.IH : p.IH;
  const int Wv = p.upsample ? 2 * p.IW : p.IW;
  const bool kfull = (p.K % BK) == 0;     // no k bound checks needed

  // ---- BUF: LDS-DMA through buffer resources (buffer_load_dwordx4 ... lds).  The per-lane
  // part of every source address is a constant 32-bit voffset computed here once; the per-k-tile
  // part (k0, or the conv tap offset) is a wave-uniform SGPR soffset, so staging a k-tile costs
  // no VALU address math (the global_load_lds path spent ~4 VALU + 3.6 SALU per MFMA on it,
  // rocprof PMC).  Invalid rows / conv padding use voffset 0x80000000 >= num_records: the
  // buffer unit returns zeros (no zero page, no per-tile select).  Conv tap validity is a
  // per-lane bitmask over the ksize^2 taps.
  __amdgpu_buffer_rsrc_t rsA, rsW, rsA2;
  int a_vo[BUF ? AR : 1], a_mask[BUF ? AR : 1], w_vo[BUF ? WR : 1];
  int a_vo2[(BUF && CONV == 0) ? AR : 1];   // second A source (channel concatenation, p.A2)
  if constexpr (BUF) {
    constexpr int OOB = (int)0x80000000;
    long long biasA = 0;   // bytes: lowest pixel offset a conv tap can address is -bias
    if constexpr (CONV == 2) biasA = ((long long)p.pad * p.IW + p.pad) * p.Cin * 2;
    const long long a_bytes = CONV ? (long long)p.M / (p.Ho * p.Wo) * p.IH * p.IW * p.Cin * 2
                                   : ((long long)(p.M - 1) * p.lda + (p.A2 ? p.ka : p.K)) * 2;
    rsA = make_rsrc((const char*)A - biasA, a_bytes + biasA);
    const long long w_bytes = ((long long)(p.Nw - 1) * ldw + p.K) * 2;
    rsW = make_rsrc(W, w_bytes);
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      if constexpr (CONV == 0) {
        a_vo[i] = a_ok[i] ? (int)(a_off[i] * 2) : OOB;
        a_mask[i] = 0;
      } else {
        a_vo[i] = a_ok[i] ? (int)(a_off[i] * 2 + biasA) : OOB;
        int mk = 0;
        for (int ky = 0; ky < p.ksize; ++ky)
          for (int kx = 0; kx < p.ksize; ++kx) {
            const int iy = cy_[i] + ky, ix = cx_[i] + kx;
            if ((unsigned)iy < (unsigned)Hv && (unsigned)ix < (unsigned)Wv) mk |= 1 << (ky * p.ksize + kx);
          }
        a_mask[i] = a_ok[i] ? mk : 0;
      }
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) w_vo[i] = w_row[i] >= 0 ? (int)(w_off[i] * 2) : OOB;
    if constexpr (CONV == 0) {
      if (p.A2 != nullptr) {   // k >= ka: rows of A2 (row stride lda2), k offset k0 - ka
        rsA2 = make_rsrc(p.A2, ((long long)(p.M - 1) * p.lda2 + (p.K - p.ka)) * 2);
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          const int r = RR * i + rsub;
          a_vo2[i] = a_ok[i] ? (int)(((long long)(m0 + r) * p.lda2 + a_chunk[i] * 8) * 2) : OOB;
        }
      }
    }
  }

  // wave-uniform conv tap state for CONV >= 2 (Cin % 64 == 0: a k-tile is 64 channels of one
  // tap), advanced incrementally as the k-tiles are staged in order
  int t_ci = 0, t_kx = 0, t_ky = 0;
  auto tap_init = [&](int kt) {
    const int k0 = kt * BK;
    const int tap = k0 / p.Cin;
    t_ci = k0 - tap * p.Cin;
    t_ky = tap / p.ksize;
    t_kx = tap - t_ky * p.ksize;
  };
  auto tap_next = [&]() {
    t_ci += BK;
    if (t_ci == p.Cin) {
      t_ci = 0;
      if (++t_kx == p.ksize) { t_kx = 0; ++t_ky; }
    }
  };

  auto stage = [&](int kt, int buf) {
    const int k0 = kt * BK;
    const bool kin = kfull || (k0 + BK <= p.K);   // whole tile inside K (uniform)
    uint4* As = smem + buf * TILE;
    uint4* Ws = As + BM * 8;
    if constexpr (BUF) {                           // (host guarantees K % BK == 0)
      int soffA = k0 * 2, tap = 0;
      if constexpr (CONV == 2) {
        soffA = ((t_ky * p.IW + t_kx) * p.Cin + t_ci) * 2;
        tap = t_ky * p.ksize + t_kx;
      }
      if constexpr (CONV == 0) {
        if (p.A2 != nullptr && k0 >= p.ka) {        // wave-uniform: this k-tile lies in A2
#pragma unroll
          for (int i = 0; i < AR; ++i) blds16(rsA2, As + (RR * i + 8 * swave) * 8, a_vo2[i], (k0 - p.ka) * 2);
        } else {
#pragma unroll
          for (int i = 0; i < AR; ++i) blds16(rsA, As + (RR * i + 8 * swave) * 8, a_vo[i], soffA);
        }
      } else {
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          int vo = a_vo[i];
          if constexpr (CONV == 2) vo = ((a_mask[i] >> tap) & 1) ? vo : (int)0x80000000;
          blds16(rsA, As + (RR * i + 8 * swave) * 8, vo, soffA);
        }
      }
#pragma unroll
      for (int i = 0; i < WR; ++i) {
        if (RR * i + 8 * swave < BN)
          blds16(rsW, Ws + (RR * i + 8 * swave) * 8, w_vo[i], k0 * 2);
      }
      if constexpr (CONV >= 2) tap_next();
      return;
    }
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const void* src = zp;
      if constexpr (CONV == 0) {
        if (a_ok[i] && (kin || k0 + a_chunk[i] * 8 < p.K)) src = A + a_off[i] + k0;
      } else if constexpr (CONV == 1) {            // general (Cin % 8): per-lane tap decode
        const int k = k0 + a_chunk[i] * 8;
        if (k < p.K) {
          const int tap = k / p.Cin;
          const int ci = k - tap * p.Cin;
          const int ky = tap / p.ksize;
          const int kx = tap - ky * p.ksize;
          int iy = cy_[i] + ky, ix = cx_[i] + kx;
          if ((unsigned)iy < (unsigned)Hv && (unsigned)ix < (unsigned)Wv) {
            if (p.upsample) { iy >>= 1; ix >>= 1; }
            src = A + (((long long)cbh_[i] + iy) * p.IW + ix) * p.Cin + ci;
          }
        }
      } else if constexpr (CONV == 2) {            // Cin % 64, no upsample: linear tap offset
        const int iy = cy_[i] + t_ky, ix = cx_[i] + t_kx;
        const long long toff = ((long long)t_ky * p.IW + t_kx) * p.Cin + t_ci;   // uniform
        if ((unsigned)iy < (unsigned)Hv && (unsigned)ix < (unsigned)Wv) src = A + a_off[i] + toff;
      } else {                                     // CONV == 3: Cin % 64 with fused 2x upsample
        int iy = cy_[i] + t_ky, ix = cx_[i] + t_kx;
        if ((unsigned)iy < (unsigned)Hv && (unsigned)ix < (unsigned)Wv) {
          iy >>= 1; ix >>= 1;
          src = A + (((long long)cbh_[i] + iy) * p.IW + ix) * p.Cin + t_ci + a_chunk[i] * 8;
        }
      }
      glds16(src, As + (RR * i + 8 * swave) * 8);
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      if (RR * i + 8 * swave < BN) {          // wave-uniform
        const void* src = (w_row[i] >= 0 && (kin || k0 + w_chunk[i] * 8 < p.K)) ? (const void*)(W + w_off[i] + k0) : zp;
        glds16(src, Ws + (RR * i + 8 * swave) * 8);
      }
    }
    if constexpr (CONV >= 2) tap_next();
  };

  f32x4_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15;      // fragment row within 16
  const int fq = lane >> 4;      // k-chunk within a 32-k step
  // fragment read addresses are loop-invariant: rows 16*i + r0 share the swizzle of r0
  // ((r0 + 16 i) >> 1) & 7 == (r0 >> 1) & 7), so each k-step needs ONE lane offset per operand
  // and the per-fragment / per-buffer parts are ds_read immediates
  const int w_r0 = wn * (BN / WN) + fr, a_r0 = wm * (BM / WM) + fr;
  int w_rd[2], a_rd[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    w_rd[ks] = BM * 8 + w_r0 * 8 + swz(w_r0, ks * 4 + fq);
    a_rd[ks] = a_r0 * 8 + swz(a_r0, ks * 4 + fq);
  }
  auto compute = [&](int buf) {
    const uint4* Bs = smem + buf * TILE;
#if GEMM_FRAG_PREFETCH && !GEMM_DIAG_APRO
    // both 32-deep k-steps' fragments are read before the first MFMA: the second step's LDS
    // latency hides under the first step's MFMAs (reading them step by step left the matrix
    // pipe idle for one LDS round trip per step, the two waves of a SIMD in lockstep after the
    // k-tile barrier: 0.40 us per 64-deep k-tile at 128x80 against 320 MFMA cycles per SIMD)
    bf16x8_t wf2[2][TI], af2[2][TJ];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < TI; ++i) wf2[ks][i] = as_bf16x8(Bs[w_rd[ks] + 16 * 8 * i]);
#pragma unroll
      for (int j = 0; j < TJ; ++j) af2[ks][j] = as_bf16x8(Bs[a_rd[ks] + 16 * 8 * j]);
    }
    // (without this the scheduler sinks the second step's reads below the first step's MFMAs:
    // the round-5 A/B of this path, profiles/r5_frag_prefetch_ab.txt, compiled to the old order)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf2[ks][i], af2[ks][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    return;
#endif
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t wf[TI], af[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) wf[i] = as_bf16x8(Bs[w_rd[ks] + 16 * 8 * i]);
#pragma unroll
      for (int j = 0; j < TJ; ++j) af[j] = as_bf16x8(Bs[a_rd[ks] + 16 * 8 * j]);
#if GEMM_DIAG_APRO
      // cost probe of a GroupNorm+SiLU prologue on the A operand (results are wrong; variant
      // builds only, profiles/r4_gn_prologue_probe.txt): scale / shift as lane constants
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        float f[8];
        unpack8(__builtin_bit_cast(uint4, af[j]), f);
        const float sc = 1.f + 0.001f * (lane & 7), sh = 0.01f * (lane >> 3);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = silu_f(fmaf(f[e], sc, sh));
        af[j] = as_bf16x8(pack8(f));
      }
#endif
      // raised wave priority while issuing the MFMA cluster (guide T5): with 2 blocks per CU the
      // wave that has MFMA work keeps the pipe busy while the other waits on its LDS-DMA
      // (+1..13 % on the SD convs / GEMMs, profiles/r1_ops_setprio_ab.txt)
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  // ---- k range of this split
  const int nk_all = (p.K + BK - 1) / BK;
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int kt0 = blockIdx.y * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
  if constexpr (CONV >= 2) tap_init(kt0);

#if GEMM_PF_SELF
  uint32_t pf_acc = 0;
  if constexpr (NP > 0 && !GEGLU) {
    if (mma_wave && nk > 0) {
      const int kb = kt0 * BK, ke = min(p.K, (kt0 + nk) * BK);
      const int lpr = ((ke - kb) * 2 + 63) / 64;          // 64-B lines per W row in this k range
      const int rows = min(BN, p.Nw - n0);
      int l0 = 0, l1 = rows * lpr;
      if (GEMM_PF_SELF == 2) {
        const int part = (l1 + 3) / 4;
        l0 = (tm & 3) * part;
        l1 = min(l1, l0 + part);
      }
      const uint32_t* Wp = reinterpret_cast<const uint32_t*>(W);
      for (int l = l0 + tid; l < l1; l += 64 * NW) {
        const int r = l / lpr, c = l - r * lpr;
        pf_acc ^= Wp[((long long)(n0 + r) * ldw + kb) / 2 + c * 16];
      }
    }
  }
#endif

  if constexpr (STAGES == 2) {
    if (nk > 0) stage(kt0, 0);
    __syncthreads();                       // drains the DMA (vmcnt(0)) and publishes the tile
    // unrolled by two so the LDS buffer of every stage/compute is a compile-time offset
    for (int t = 0; t < nk; t += 2) {
      if (t + 1 < nk) stage(kt0 + t + 1, 1);
      compute(0);
      __syncthreads();                     // next tile landed and everyone is done with this one
      if (t + 1 >= nk) break;
      if (t + 2 < nk) stage(kt0 + t + 2, 0);
      compute(1);
      __syncthreads();
    }
  } else {
    // STAGES-deep ring: tiles t+1 .. t+STAGES-2 stay in flight while tile t is consumed
    constexpr int S = STAGES;
    const int npt = w_last_round ? NPT : NPT - 1;   // this wave's DMAs per k-tile (uniform)
    auto wait_tiles = [&](int k) {                  // leave k tiles' DMAs outstanding
      if (npt == NPT) {
        if (k <= 0) wait_vmcnt<0>();
        else if (k == 1) wait_vmcnt<NPT>();
        else if (k == 2) wait_vmcnt<2 * NPT>();
        else wait_vmcnt<3 * NPT>();
      } else {
        if (k <= 0) wait_vmcnt<0>();
        else if (k == 1) wait_vmcnt<NPT - 1>();
        else if (k == 2) wait_vmcnt<2 * (NPT - 1)>();
        else wait_vmcnt<3 * (NPT - 1)>();
      }
    };
    if (dma_wave) {
#pragma unroll
      for (int s0 = 0; s0 < S - 1; ++s0)
        if (s0 < nk) stage(kt0 + s0, s0);
    }
    for (int t = 0; t < nk; ++t) {
      if (dma_wave) wait_tiles(min(S - 2, nk - 1 - t));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();        // every wave's share of tile t landed; tile t-1 is free
      if (dma_wave && t + S - 1 < nk) stage(kt0 + t + S - 1, (t + S - 1) % S);
      if (mma_wave) compute(t % S);
    }
  }

  tile_epilogue<BM, BN, WM, WN, GEGLU, OUTF32, TI, TJ, THREADS>(p, acc, smem, partial, m0, n0, batch, wm, wn, tid,
                                                               gridDim.y, blockIdx.y, mma_wave);
#if GEMM_PF_SELF
  asm volatile("" ::"v"(pf_acc));         // keeps the warm-up loads; their wait lands here
#endif
}

// split-K: a second, fully parallel pass sums the slices' fp32 slabs and applies the epilogue
// (an in-kernel last-arriver reduction was measured 1.3-2.4x slower on the split shapes: one
// block serially reading up to 15 slabs of its tile)
template <bool OUTF32>
__global__ void splitk_reduce_kernel(GemmArgs p, const float* __restrict__ partial, int split) {
  // slabs of batch z (parity class of the upsampling conv) start at z * split * M * N
  const int bz = blockIdx.y;
  partial += (long long)bz * split * p.M * p.N;
  const long long nq = (long long)p.M * (p.N / 4);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(i / (p.N / 4));
    const int n = (int)(i - (long long)m * (p.N / 4)) * 4;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < split; ++s) {
      const float4 v = *reinterpret_cast<const float4*>(partial + ((long long)s * p.M + m) * p.N + n);
      o[0] += v.x; o[1] += v.y; o[2] += v.z; o[3] += v.w;
    }
    epilogue4<OUTF32>(p, bz, m, n, o);
  }
}

// split-K reduce + GroupNorm statistics of the output (p.stats): block = 16 column quads (64
// columns) x 16 row lanes over SK_RB = 64 rows; each thread sums the slabs of its quad for 4 rows
// (4 slab loads in flight), runs the epilogue and accumulates (sum, sumsq) of the stored bf16
// values; the 16 row lanes are folded in LDS and added with one atomic per (column, statistic)
// per block (per-thread flushes when a block's rows straddle images).  The fp32 atomics, not the
// slab reads, bound this pass when blocks are small: 4 row lanes x 16 rows cost +9 us on the
// 16x16-level conv (327k atomics), 16 x 64 is ~4x fewer.
constexpr int SK_RB = 64;
constexpr int SK_QB = 16;                  // column quads per block
constexpr int SK_RL = 256 / SK_QB;         // row lanes
template <bool OUTF32>
__global__ void __launch_bounds__(256) splitk_reduce_stats_kernel(GemmArgs p, const float* __restrict__ partial,
                                                                  int split, int rb) {
  __shared__ float red[2][SK_RL][SK_QB * 4];
  const int bz = blockIdx.z;
  partial += (long long)bz * split * p.M * p.N;
  const int qd = threadIdx.x % SK_QB, rl = threadIdx.x / SK_QB;
  const int n = (blockIdx.x * SK_QB + qd) * 4;
  const int m0 = blockIdx.y * rb;
  const int m1 = min(p.M, m0 + rb);
  const bool on = n < p.N;
  const int shw = p.stats_hw;
  const bool single = (m0 / shw) == ((m1 - 1) / shw);
  float s4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f};
  int cur = -1;
  auto flush = [&]() {
    if (cur < 0) return;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      stat_atomic_add(p.stats + ((long long)cur * p.N + n + e) * 2 + 0, 0, s4[e]);
      stat_atomic_add(p.stats + ((long long)cur * p.N + n + e) * 2 + 1, 1, q4[e]);
      s4[e] = 0.f;
      q4[e] = 0.f;
    }
  };
  if (on) {
    for (int m = m0 + rl; m < m1; m += SK_RL) {
      float o[4] = {0.f, 0.f, 0.f, 0.f};
      const float* src = partial + (long long)m * p.N + n;
      const long long slab = (long long)p.M * p.N;
      int sl = 0;
      for (; sl + 4 <= split; sl += 4) {     // 4 slab loads in flight per thread
        const float4 v0 = *reinterpret_cast<const float4*>(src + (sl + 0) * slab);
        const float4 v1 = *reinterpret_cast<const float4*>(src + (sl + 1) * slab);
        const float4 v2 = *reinterpret_cast<const float4*>(src + (sl + 2) * slab);
        const float4 v3 = *reinterpret_cast<const float4*>(src + (sl + 3) * slab);
        o[0] += (v0.x + v1.x) + (v2.x + v3.x);
        o[1] += (v0.y + v1.y) + (v2.y + v3.y);
        o[2] += (v0.z + v1.z) + (v2.z + v3.z);
        o[3] += (v0.w + v1.w) + (v2.w + v3.w);
      }
      for (; sl < split; ++sl) {
        const float4 v = *reinterpret_cast<const float4*>(src + sl * slab);
        o[0] += v.x; o[1] += v.y; o[2] += v.z; o[3] += v.w;
      }
      epilogue4<OUTF32>(p, bz, m, n, o);     // (N % 8 == 0: o holds the final values)
      if (!single) {
        const int img = m / shw;
        if (img != cur) { flush(); cur = img; }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float f = OUTF32 ? o[e] : bf2f(f2bf(o[e]));
        s4[e] += f;
        q4[e] = fmaf(f, f, q4[e]);
      }
    }
  }
  if (!single) {
    flush();
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][rl][qd * 4 + e] = s4[e];
    red[1][rl][qd * 4 + e] = q4[e];
  }
  __syncthreads();
  const int img = m0 / shw;
  if (threadIdx.x < 2 * SK_QB * 4) {
    const int st = threadIdx.x / (SK_QB * 4), col = threadIdx.x % (SK_QB * 4);
    const int nn = blockIdx.x * SK_QB * 4 + col;
    if (nn < p.N) {
      float a = 0.f;
#pragma unroll
      for (int r = 0; r < SK_RL; ++r) a += red[st][r][col];
      stat_atomic_add(p.stats + ((long long)img * p.N + nn) * 2 + st, st, a);
    }
  }
}

// the split-K second pass (slabs [batch][split][M][N] fp32)
template <bool OUTF32>
void launch_splitk_reduce(const GemmArgs& p, float* ws, int split, hipStream_t s) {
  if (p.stats != nullptr) {
    // rows per block: SK_RB, halved (down to one row per row lane) while the grid has fewer than
    // 512 blocks -- the small-M reduces (batch-1 levels 3 / 4: 160 blocks at M 512) are bound by
    // each thread's serial rows, not by the statistics atomics that larger blocks save
    // (CASSMANTLE_SK_ADAPT=0: fixed SK_RB, A/B knob)
    static const int adapt = [] { const char* e = getenv("CASSMANTLE_SK_ADAPT"); return e ? atoi(e) : 1; }();
    const long long cols = (p.N / 4 + SK_QB - 1) / SK_QB;
    int rb = SK_RB;
    while (adapt && rb > SK_RL && cols * ((p.M + rb - 1) / rb) * p.batch < 512) rb /= 2;
    dim3 g2((unsigned)cols, (unsigned)((p.M + rb - 1) / rb), (unsigned)p.batch);
    hipLaunchKernelGGL(splitk_reduce_stats_kernel<OUTF32>, g2, dim3(256), 0, s, p, ws, split, rb);
  } else {
    const long long nq = (long long)p.M * (p.N / 4);
    const long long nb = (nq + 255) / 256;
    const unsigned rb = (unsigned)(nb < 2048 ? nb : 2048);
    hipLaunchKernelGGL(splitk_reduce_kernel<OUTF32>, dim3(rb, (unsigned)p.batch), dim3(256), 0, s, p, ws, split);
  }
}

template <int BM, int BN, int WM, int WN, int CONV, bool GEGLU, bool OUTF32, int STAGES, bool BUF, int NP = 0>
void launch_t(const GemmArgs& p, float* ws, hipStream_t s) {
  const int nN = GEGLU ? (p.N + BN / 2 - 1) / (BN / 2) : (p.N + BN - 1) / BN;
  const int nM = (p.M + BM - 1) / BM;
  const int split = (ws != nullptr && p.split > 1) ? p.split : 1;
  dim3 grid(nN * nM, split, p.batch);
  constexpr size_t lds_stage = (size_t)STAGES * (BM + BN) * BK * 2;
  constexpr size_t lds_epi = (size_t)BM * ((GEGLU ? BN / 2 : BN) + 8) * 2;
  constexpr size_t lds = lds_stage > lds_epi ? lds_stage : lds_epi;
  // (the kernel is named once, outside any lambda: a kernel template referenced only from a
  // lambda inside this function template was left uninstantiated by hipcc)
  auto* kfn = &gemm_kernel<BM, BN, WM, WN, CONV, GEGLU, OUTF32, STAGES, BUF, NP>;
  if constexpr (lds > 65536) {
    // > 64 KiB dynamic LDS must be opted into once (first call happens before any graph capture)
    // > 64 KiB dynamic LDS opt-in, once per process (thread-safe static init)
    static const bool once = [&] {
      (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      return true;
    }();
    (void)once;
  }
  hipLaunchKernelGGL(kfn, grid, dim3(64 * (WM * WN + NP)), lds, s, p, ws);
  if (split > 1) launch_splitk_reduce<OUTF32>(p, ws, split, s);
}

template <int BM, int BN, int WM, int WN, int CONV, bool GEGLU, bool OUTF32, bool BUF>
void launch_st(const GemmArgs& p, float* ws, hipStream_t s) {
  if constexpr (WM * WN == 8) {
    launch_t<BM, BN, WM, WN, CONV, GEGLU, OUTF32, 3, BUF>(p, ws, s);
  } else {
    // (4-wave tiles: STAGES=3 at one block/CU measured 1.3-1.7x SLOWER than 2 stages at 2
    // blocks/CU on every SD shape, profiles/r1_ops_stages_ab.txt)
    launch_t<BM, BN, WM, WN, CONV, GEGLU, OUTF32, 2, BUF>(p, ws, s);
  }
}

template <int CONV, bool OUTF32, bool BUF>
void launch_cfg(const GemmArgs& p, float* ws, hipStream_t s) {
  // deep-ring tiles (buffer-resource modes, bf16 out): one block per CU, STAGES-2 k-tiles ahead
  if constexpr (BUF && !OUTF32) {
    switch (p.cfg) {
      case 12: return launch_t<128, 128, 2, 2, CONV, false, false, 4, true>(p, ws, s);
      case 13: return launch_t<128, 64, 2, 2, CONV, false, false, 5, true>(p, ws, s);
      case 14: return launch_t<128, 160, 4, 2, CONV, false, false, 4, true>(p, ws, s);
      case 16: return launch_t<128, 80, 4, 1, CONV, false, false, 4, true>(p, ws, s);
      case 26: return launch_t<128, 80, 8, 1, CONV, false, false, 4, true>(p, ws, s);
      case 27: return launch_t<128, 64, 4, 2, CONV, false, false, 3, true>(p, ws, s);
      // warp-specialised: 8 MFMA waves + 8 DMA-only producer waves (1024 threads)
      case 31: return launch_t<128, 80, 8, 1, CONV, false, false, 4, true, 8>(p, ws, s);
      case 32: return launch_t<128, 64, 4, 2, CONV, false, false, 4, true, 8>(p, ws, s);
      case 33: return launch_t<128, 160, 4, 2, CONV, false, false, 4, true, 8>(p, ws, s);
      // (256x128 / 128x256 / 128x128 and 128x160 8x1 (also gated) producer-wave tiles were tuned
      // in situ in round 4: bench-neutral, removed; profiles/r4_producer_waves_ab.txt.  6-stage
      // rings of 31 / 32: no faster with weights from HBM on every call,
      // profiles/r4_cold_weight_probe.jsonl.  31-33 with the MFMA waves staging too: 3-15 % slower
      // per call, bench-neutral, profiles/r4_producer_waves_ab.txt)
      default: break;
    }
  }
  switch (p.cfg) {
    case 1: launch_st<128, 160, 2, 2, CONV, false, OUTF32, BUF>(p, ws, s); break;
    case 2: launch_st<256, 64, 4, 1, CONV, false, OUTF32, BUF>(p, ws, s); break;
    case 3: launch_st<128, 64, 2, 2, CONV, false, OUTF32, BUF>(p, ws, s); break;
    case 4: launch_st<256, 16, 4, 1, CONV, false, OUTF32, BUF>(p, ws, s); break;
    case 5: launch_st<256, 160, 4, 2, CONV, false, OUTF32, BUF>(p, ws, s); break;
    case 6: launch_st<256, 128, 4, 2, CONV, false, OUTF32, BUF>(p, ws, s); break;
    default: launch_st<128, 128, 2, 2, CONV, false, OUTF32, BUF>(p, ws, s); break;
  }
}

template <int CONV, bool BUF>
void launch_tiles(const GemmArgs& p, float* ws, hipStream_t s) {
  if (p.act == ACT_GEGLU || p.act == ACT_SWIGLU) {
    if constexpr (BUF) {
      if (p.cfg == 12) return launch_t<128, 128, 2, 2, CONV, true, false, 4, true>(p, ws, s);
    }
    if (p.cfg == 6) launch_st<256, 128, 4, 2, CONV, true, false, BUF>(p, ws, s);
    else launch_st<128, 128, 2, 2, CONV, true, false, BUF>(p, ws, s);
  }
  else if (p.out_f32) launch_cfg<CONV, true, BUF>(p, ws, s);
  else launch_cfg<CONV, false, BUF>(p, ws, s);
}

}  // namespace

// per-translation-unit entry points (gemm_c*.hip): the tile menu of one A-operand mode
#define GEMM_TU_ENTRY(NAME, CONV, BUF) \
  void NAME(const GemmArgs& p, float* ws, hipStream_t s) { launch_tiles<CONV, BUF>(p, ws, s); }
