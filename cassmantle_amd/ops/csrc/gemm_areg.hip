// Short-K GEMM with the A operand held in REGISTERS (the UNet's level-1
// transformer projections, QKV and GEGLU feed-forward, K = 320..640).
//
// Why a separate kernel: at K = 320 a tiled GEMM runs only 5 k-tiles per output tile, so every
// tile pays its DMA prologue latency and its epilogue serially (measured 126 us for the
// 32768 x 2560 x 320 GEGLU = 3.3 PF-equivalent 4.7x off its MFMA floor; profiles/
// r2_autotune_sd15.jsonl).  Here a block owns BM = 128 rows and keeps their ENTIRE K extent as
// MFMA B-operand fragments in VGPRs (each wave 32 rows: 2 x K/32 fragments, loaded once from
// global memory), then streams the W matrix through a 2-3 deep LDS ring in chunks of BNC rows:
// per chunk every wave runs K/32 x TI x 2 MFMAs against that chunk and writes its 32 x BNC
// outputs straight from the accumulators (bias / GEGLU / residual / GroupNorm statistics
// fused).  The next chunks' LDS-DMA overlaps the current chunk's MFMAs; the block never
// returns to a prologue until all of its N range is done.
//
// Layout: D[n][m] = W[n][:] . A[m][:] as in gemm_impl.h (W rows on the MFMA row axis: each lane
// owns 4 consecutive output columns of one row -> 8-byte stores).  W chunk LDS image: K/64
// k-tiles of [BNC][64] bf16 (128-byte rows, chunk XOR-swizzled by (row >> 1) & 7 on the DMA
// source address and the ds_read, conflict-free for the 16-row fragment reads).
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;

CM_DEVICE void areg_blds16(__amdgpu_buffer_rsrc_t rs, uint4* lds_wave_base, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds_wave_base, 16, voff, soff, 0, 0);
}

// sum over lanes l, l ^ 16, l ^ 32, l ^ 48 (the 4 lanes holding one A row) with the gfx950
// permlane swaps: pure VALU, no ds_bpermute through the LDS unit.
//
// The in-kernel LayerNorm race (round 2: whole 16-row fragment groups came out with slightly
// different LayerNorm statistics, only while a workgroup of another kernel shared the CU; the
// round-2 "fix" built this file with -fno-slp-vectorize) -- what the round-3 screens showed
// (tools/race_lnk_{concurrency,rows}.py, profiles/r3_lnk_race_rootcause.txt):
//   * the failures are confined to the LAST fragment group of a wave (j = RW - 1) and need
//     packed fp32 (v_pk_add/mul/fma_f32, produced by SLP vectorisation) in the statistics /
//     normalisation PROLOGUE.  There hipcc pairs the (sum, sum of squares) reductions of that
//     group into packed ops and reads their results at its one-wait-state minimum
//     (v_pk_add_f32 v[82:83] ; s_nop 0 ; v_pk_mul_f32 v[82:83], v[82:83] ; s_nop 0 ; v_fma_f32
//     v84, -v83, v83, v82); in the first group's reductions the same readers sit >= 2
//     instructions away;
//   * padding the permlane swaps alone (the first hypothesis, kept below) still failed;
//   * a prologue in scalar fp32 (scalar_f) with SLP ON for the rest of the kernel (the epilogue
//     keeps its packed ops) passed every screen: 0 / 1440 concurrent runs of the row screen and
//     0 / 40 x 10 concurrency arms, where the round-2 source built with SLP failed 1-2 / 40 and
//     dozens of row-screen iterations on the same box.
// So the mechanism is a read of a packed-fp32 result that the compiler's hazard padding does
// not protect under issue contention from a co-resident workgroup (a hardware / hazard-table
// issue we could bracket but not observe at instruction level); the fix lives in the source:
// no packed fp32 before the first DMA, plus generously padded swaps.
CM_DEVICE void permlane16_swap_padded(unsigned& a, unsigned& b) {
  asm volatile("s_nop 4\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
}
CM_DEVICE void permlane32_swap_padded(unsigned& a, unsigned& b) {
  asm volatile("s_nop 4\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
}
// An opaque scalar fp32 value: the SLP vectoriser cannot pair two of these into one packed
// v_pk_*_f32 instruction (the LayerNorm statistics and normalisation prologue, see above)
CM_DEVICE float scalar_f(float x) {
  asm volatile("" : "+v"(x));
  return x;
}

CM_DEVICE float sum_row_groups(float v) {
  unsigned a0 = __float_as_uint(v), a1 = a0;
  permlane16_swap_padded(a0, a1);                                          // rows (0,0,2,2) | (1,1,3,3)
  const float s = __uint_as_float(a0) + __uint_as_float(a1);
  unsigned b0 = __float_as_uint(s), b1 = b0;
  permlane32_swap_padded(b0, b1);                                          // halves (lo,lo) | (hi,hi)
  return __uint_as_float(b0) + __uint_as_float(b1);
}

template <int N>
CM_DEVICE void areg_wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

constexpr int AR_THREADS = 256;        // 4 waves, each owning 16 * RW rows

// KS = K / 32 k-steps; TI = BNC / 16 W subtiles per chunk; RING = LDS chunk buffers;
// RW = 16-row A fragments per wave (each W fragment read from LDS feeds RW MFMAs)
template <int KS, int TI, int RING>
constexpr int areg_minb() {
  return RING * 16 * TI * (KS / 2) * 128 <= 52 * 1024 ? 3 : (RING * 16 * TI * (KS / 2) * 128 <= 80 * 1024 ? 2 : 1);
}

// LNK: LayerNorm applied to the A rows already resident in registers (W = W * gamma,
// bias = bias + W . beta folded offline): row statistics from the fragments, then every
// fragment is normalised in place to bf16 -- exactly the LayerNorm kernel's output, with no
// LayerNorm kernel, no normalised copy in HBM, no stats pass, and a plain epilogue
// GNK: GroupNorm (p.gn_stats) applied to the resident A rows, see the prologue below
template <int KS, int TI, int RING, int RW, bool GEGLU, bool LNK, bool GNK = false>
__global__ void __launch_bounds__(AR_THREADS, (areg_minb<KS, TI, RING>())) gemm_areg_kernel(GemmArgs p, int chunks_per_block) {
  constexpr int AR_BM = 64 * RW;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  constexpr int BNC = 16 * TI;                 // W rows per chunk
  constexpr int KT = KS / 2;                   // 64-deep k-tiles
  constexpr int CHUNK = BNC * KT * 8;          // uint4 per chunk buffer
  constexpr int DMA_PER_CHUNK = (BNC * KT) / 32;   // 1 KiB pieces per wave (4 waves x 8 rows)
  static_assert(KS % 2 == 0 && (BNC * KT) % 32 == 0, "whole DMA rounds");
  static_assert(!GEGLU || TI % 2 == 0, "geglu value/gate pairs");
  constexpr int OOB = (int)0x80000000;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int m0 = blockIdx.x * AR_BM + wave * 16 * RW;     // this wave's 16 * RW rows
  const int nchunks = GEGLU ? (2 * p.N) / BNC : p.N / BNC;
  const int c_begin = blockIdx.y * chunks_per_block;
  const int c_end = min(nchunks, c_begin + chunks_per_block);
  const int ldw = p.ldw ? p.ldw : p.K;

  // ---- A fragments into registers: afr[j][ks] = 8 bf16 of row m0 + 16 j + fr, k = 32 ks + 8 fq
  bf16x8_t afr[RW][KS];
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    const int row = m0 + 16 * j + fr;
    const bool ok = row < p.M;
    const uint4* src = reinterpret_cast<const uint4*>(p.A + (long long)(ok ? row : 0) * p.lda) + fq;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint4 v = src[4 * ks];
      if (!ok) v = make_uint4(0, 0, 0, 0);
      afr[j][ks] = as_bf16x8(v);
    }
  }
  // ---- LayerNorm row statistics: a row's K values sit in the 4 lanes fr, fr+16, fr+32, fr+48.
  // Scalar fp32 only (scalar_f): see the race note above sum_row_groups.
  float ln_mean[RW], ln_rstd[RW];
  if constexpr (LNK) {
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      // one pass (sum, sum of squares): a second pass re-unpacked the same fragments and the
      // compiler kept all K/4 unpacked floats live between the passes (spills)
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const uint4 u = __builtin_bit_cast(uint4, afr[j][ks]);
        const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = __uint_as_float(w4[e] << 16), hi = __uint_as_float(w4[e] & 0xffff0000u);
          s1 = scalar_f(s1 + scalar_f(lo + hi));
          s2 = scalar_f(fmaf(lo, lo, scalar_f(fmaf(hi, hi, s2))));
        }
      }
      s1 = sum_row_groups(s1);
      s2 = sum_row_groups(s2);
      const float mu = scalar_f(s1 * (1.f / (32 * KS)));
      const float var = scalar_f(fmaxf(scalar_f(s2 * (1.f / (32 * KS))) - scalar_f(mu * mu), 0.f));
      ln_mean[j] = mu;
      ln_rstd[j] = scalar_f(rsqrtf(var + p.ln_eps));
    }
    // opaque re-definition of the fragments: otherwise hipcc reuses the statistics pass's
    // unpacked floats here and keeps all K / 4 of them live (spills)
#pragma unroll
    for (int j = 0; j < RW; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        i32x4_t t = __builtin_bit_cast(i32x4_t, afr[j][ks]);
        asm volatile("" : "+v"(t));
        afr[j][ks] = __builtin_bit_cast(bf16x8_t, t);
      }
#pragma unroll
    for (int j = 0; j < RW; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float f[8];
        unpack8(__builtin_bit_cast(uint4, afr[j][ks]), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = scalar_f((f[e] - ln_mean[j]) * ln_rstd[j]);
        afr[j][ks] = as_bf16x8(pack8(f));
      }
    // Finish the statistics before the first W-chunk LDS-DMA.  Their cross-lane sums are
    // ds_bpermute (__shfl_xor) reads through the LDS unit, and the scheduler used to place them
    // after the first LDS-DMAs.  While those DMAs were in flight, the shuffles' partial lgkmcnt
    // waits did not cover them.  Whole 16-row groups then came out with a wrong mean/rstd (up to
    // 0.1 abs), but only when another kernel slowed the DMA down: a 4-wave GEMM on a second
    // stream, or stage-overlapped VAE decode (tools/dbg_conc_matrix.py, tools/dbg_overlap.py).
    // The opaque asm below makes the normalised fragments inputs of a memory-clobbering
    // statement, so no DMA can be scheduled above the statistics.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < RW; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        i32x4_t t = __builtin_bit_cast(i32x4_t, afr[j][ks]);
        asm volatile("" : "+v"(t) : : "memory");
        afr[j][ks] = __builtin_bit_cast(bf16x8_t, t);
      }
  }

  // ---- GroupNorm of the A rows (p.gn_stats; transformer GroupNorm -> proj_in, no SiLU): the
  // block's rows lie in one image (host: gn_hw % (64 RW) == 0).  Fold the image's K channel
  // (sum, sum of squares) into per-group (mean, rstd) in LDS (8 threads per group), then scale /
  // shift every resident fragment in place.  Scalar fp32 and finished before the first DMA, as
  // the LayerNorm prologue above (race note at sum_row_groups); the LDS scratch is released by
  // a barrier before the ring is staged.
  if constexpr (GNK) {
    float* gs = reinterpret_cast<float*>(smem);            // [G][2] mean, rstd
    const int G = p.gn_groups;
    constexpr int K = 32 * KS;
    const int img = (blockIdx.x * AR_BM) / p.gn_hw;
    const long long* st = p.gn_stats + (long long)img * K * 2;
    const int Cg = K / G;
    for (int g0 = 0; g0 < G; g0 += AR_THREADS / 8) {
      const int g = g0 + tid / 8, sub = tid % 8;
      long long si = 0, qi = 0;
      if (g < G)
        for (int c = g * Cg + sub; c < (g + 1) * Cg; c += 8) {
          si += st[2 * c];
          qi += st[2 * c + 1];
        }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        si += __shfl_xor(si, o, 64);
        qi += __shfl_xor(qi, o, 64);
      }
      if (g < G && sub == 0) {
        const double n = (double)p.gn_hw * Cg;
        const double mean = stat_decode(si, 0) / n;
        double var = stat_decode(qi, 1) / n - mean * mean;
        var = var > 0.0 ? var : 0.0;
        gs[2 * g] = (float)mean;
        gs[2 * g + 1] = (float)(1.0 / sqrt(var + (double)p.gn_eps));
      }
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c0 = 32 * ks + 8 * fq;                     // this lane's 8 channels of k-step ks
      float ga[8], be[8], sc[8], sh[8];
      unpack8(*reinterpret_cast<const uint4*>(p.gn_gamma + c0), ga);
      unpack8(*reinterpret_cast<const uint4*>(p.gn_beta + c0), be);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int g = ((c0 + e) * G) / K;                   // K is a compile-time constant
        sc[e] = scalar_f(ga[e] * gs[2 * g + 1]);
        sh[e] = scalar_f(be[e] - scalar_f(gs[2 * g] * sc[e]));
      }
#pragma unroll
      for (int j = 0; j < RW; ++j) {
        float f[8];
        unpack8(__builtin_bit_cast(uint4, afr[j][ks]), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = scalar_f(fmaf(f[e], sc[e], sh[e]));
        afr[j][ks] = as_bf16x8(pack8(f));
      }
    }
    __syncthreads();                                       // gs consumed: the ring may overwrite it
#pragma unroll
    for (int j = 0; j < RW; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        i32x4_t t = __builtin_bit_cast(i32x4_t, afr[j][ks]);
        asm volatile("" : "+v"(t) : : "memory");
        afr[j][ks] = __builtin_bit_cast(bf16x8_t, t);
      }
  }

  // ---- W chunk staging: chunk c, LDS row (k-tile t, chunk row r) <- W row of (c, r), k 64 t..
  __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.W), (short)0,
                                                                  (int)(((long long)(p.Nw - 1) * ldw + p.K) * 2),
                                                                  0x00020000);
  // piece q of a chunk (q = 0 .. DMA_PER_CHUNK-1) covers LDS rows 32 q + 8 wave + (lane >> 3) of
  // the [KT][BNC] row space; its lane moves chunk (lane & 7) ^ swz of that row
  int w_vo_base[DMA_PER_CHUNK], w_koff[DMA_PER_CHUNK];
  const int slot = lane & 7;
#pragma unroll
  for (int q = 0; q < DMA_PER_CHUNK; ++q) {
    const int lr = 32 * q + 8 * wave + (lane >> 3);      // LDS row in the chunk image
    const int t = lr / BNC, r = lr - t * BNC;             // k-tile, chunk row
    const int ch = slot ^ ((r >> 1) & 7);
    w_koff[q] = (t * 64 + ch * 8) * 2;                    // bytes within the W row
    w_vo_base[q] = r;                                     // chunk row (W row resolved per chunk)
  }
  auto w_row_of = [&](int c, int r) -> int {              // W row for chunk c, chunk row r
    if constexpr (GEGLU) {
      // chunk c covers output columns [c * BNC/2, ...): 16-row blocks alternate value / gate
      const int blk = r >> 4, within = r & 15;
      const int nout = c * (BNC / 2) + (blk >> 1) * 16 + within;
      return nout < p.N ? ((blk & 1) ? p.N + nout : nout) : -1;
    } else {
      const int n = c * BNC + r;
      return n < p.Nw ? n : -1;
    }
  };
  // every stage() issues exactly DMA_PER_CHUNK loads per wave (a chunk past the block's range
  // moves zeros into a free buffer) so the vmcnt bookkeeping is static on every path
  auto stage = [&](int c, int buf) {
    uint4* base = smem + buf * CHUNK;
    const bool live = c < c_end;
#pragma unroll
    for (int q = 0; q < DMA_PER_CHUNK; ++q) {
      const int wr = live ? w_row_of(c, w_vo_base[q]) : -1;
      const int vo = wr >= 0 ? (int)((long long)wr * ldw * 2 + w_koff[q]) : OOB;
      areg_blds16(rsW, base + (32 * q + 8 * wave) * 8, vo, 0);
    }
  };

  // fragment read offsets (uint4 units) within a chunk buffer: W subtile i rows 16 i + fr,
  // k-step ks -> k-tile ks >> 1, logical 16-byte chunk 4 (ks & 1) + fq
  auto w_off = [&](int i, int ks) {
    const int r = 16 * i + fr;
    return ((ks >> 1) * BNC + r) * 8 + ((4 * (ks & 1) + fq) ^ ((r >> 1) & 7));
  };

  const int hw = p.stats_hw > 0 ? p.stats_hw : 1;
  // RING 3: one chunk in flight behind the one being retired.  RING 2 (plain double buffer):
  // the next chunk's DMA overlaps this chunk's MFMAs and epilogue and is retired at the top of
  // the next iteration; 2/3 of the LDS, so the K = 640 tiles fit 2 blocks per CU
  static_assert(RING == 2 || RING == 3, "2- or 3-deep ring");
  stage(c_begin, 0);
  if constexpr (RING == 3) stage(c_begin + 1, 1);

  constexpr int NQ = GEGLU ? TI / 2 : TI;          // output column quads per row per chunk
  for (int c = c_begin; c < c_end; ++c) {
    const int rel = c - c_begin;
    const int buf = rel % RING;
    // retire chunk c (chunk c + 1 stays in flight), publish it.  After the first chunk this is
    // already satisfied by the previous chunk's epilogue wait.
    areg_wait_vmcnt<(RING - 2) * DMA_PER_CHUNK>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();            // chunk c landed; every wave is done with c-1's buffer

    // epilogue operands of THIS chunk, loaded BEFORE the next DMA so that waiting for them
    // (loads retire in order) leaves that DMA in flight
    uint2 bq[NQ], gq[GEGLU ? NQ : 1], rq[RW][NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int n = GEGLU ? c * (BNC / 2) + 16 * i + 4 * fq : c * BNC + 16 * i + 4 * fq;
      const bool nok = n < p.N;
      bq[i] = make_uint2(0, 0);
      if (GEGLU) gq[GEGLU ? i : 0] = make_uint2(0, 0);
      if (p.bias && nok) {
        bq[i] = *reinterpret_cast<const uint2*>(p.bias + n);
        if (GEGLU) gq[GEGLU ? i : 0] = *reinterpret_cast<const uint2*>(p.bias + p.N + n);
      }

#pragma unroll
      for (int j = 0; j < RW; ++j) {
        const int m = m0 + 16 * j + fr;
        rq[j][i] = make_uint2(0, 0);
        if (p.residual && nok && m < p.M) rq[j][i] = *reinterpret_cast<const uint2*>(p.residual + (long long)m * p.ldc + n);
      }
    }
    stage(c + RING - 1, (rel + RING - 1) % RING);

    const uint4* Bs = smem + buf * CHUNK;
    f32x4_t acc[TI][RW];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < RW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // W fragments software-pipelined one k-step ahead of the MFMAs that consume them
    bf16x8_t wf[2][TI];
#pragma unroll
    for (int i = 0; i < TI; ++i) wf[0][i] = as_bf16x8(Bs[w_off(i, 0)]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
#pragma unroll
        for (int i = 0; i < TI; ++i) wf[(ks + 1) & 1][i] = as_bf16x8(Bs[w_off(i, ks + 1)]);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < RW; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks & 1][i], afr[j][ks], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    areg_wait_vmcnt<DMA_PER_CHUNK>();   // this chunk's epilogue operands (and chunk c + 1) landed

    // ---- epilogue straight from the accumulators: row m, columns n .. n+3
    float ssum[TI][4], ssq[TI][4];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) { ssum[i][e] = 0.f; ssq[i][e] = 0.f; }
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      const int m = m0 + 16 * j + fr;
      const bool mok = m < p.M;
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int n = GEGLU ? c * (BNC / 2) + 16 * i + 4 * fq : c * BNC + 16 * i + 4 * fq;
        if (!mok || n >= p.N) continue;
        const float b[4] = {bf2f(bq[i].x & 0xffff), bf2f(bq[i].x >> 16), bf2f(bq[i].y & 0xffff), bf2f(bq[i].y >> 16)};
        const float r[4] = {bf2f(rq[j][i].x & 0xffff), bf2f(rq[j][i].x >> 16), bf2f(rq[j][i].y & 0xffff),
                            bf2f(rq[j][i].y >> 16)};
        float o[4];
        if constexpr (GEGLU) {
          const uint2 g2 = gq[GEGLU ? i : 0];
          const float gb[4] = {bf2f(g2.x & 0xffff), bf2f(g2.x >> 16), bf2f(g2.y & 0xffff), bf2f(g2.y >> 16)};
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = gate_f(acc[2 * i][j][e] + b[e], acc[2 * i + 1][j][e] + gb[e], p.act) + r[e];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = acc[i][j][e] * p.alpha + b[e];
          if (p.act != ACT_NONE) {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = apply_act(o[e], p.act);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] += r[e];
        }
        const uint2 pk = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
        if (GEGLU || !kv8_store4(p, m, n, o))
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.C) + (long long)m * p.ldc + n) = pk;
        if (!GEGLU && p.stats) {   // statistics of the STORED (bf16-rounded) values
          const float q0 = bf2f(pk.x & 0xffff), q1 = bf2f(pk.x >> 16), q2 = bf2f(pk.y & 0xffff), q3 = bf2f(pk.y >> 16);
          ssum[i][0] += q0; ssum[i][1] += q1; ssum[i][2] += q2; ssum[i][3] += q3;
          ssq[i][0] = fmaf(q0, q0, ssq[i][0]); ssq[i][1] = fmaf(q1, q1, ssq[i][1]);
          ssq[i][2] = fmaf(q2, q2, ssq[i][2]); ssq[i][3] = fmaf(q3, q3, ssq[i][3]);
        }
      }
    }
    if constexpr (!GEGLU) {
      // GroupNorm statistics: a wave's 16 RW rows lie in one image (hw % 64 == 0, host-checked);
      // reduce over the 16 row lanes sharing a column quad, one atomic per (column, stat)
      if (p.stats && m0 < p.M) {
        const int img = m0 / hw;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float a = ssum[i][e], b = ssq[i][e];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) { a += __shfl_xor(a, o, 64); b += __shfl_xor(b, o, 64); }
            const int n = c * BNC + 16 * i + 4 * fq + e;
            if (fr == 0 && n < p.N) {
              stat_atomic_add(p.stats + ((long long)img * p.N + n) * 2 + 0, 0, a);
              stat_atomic_add(p.stats + ((long long)img * p.N + n) * 2 + 1, 1, b);
            }
          }
      }
    }
  }
  // the ring always has a chunk's DMA in flight (the zero-filled stage past the block's range
  // included): drain it before the workgroup retires, or it lands in the LDS of the next
  // workgroup placed on this CU (a run-to-run race: tools/dbg_det_ops.py)
  areg_wait_vmcnt<0>();
}

template <int KS, int TI, int RING, int RW, bool GEGLU, bool LNK, bool GNK = false>
void launch_areg_t(const GemmArgs& p, hipStream_t s) {
  constexpr int AR_BM = 64 * RW;
  constexpr int BNC = 16 * TI;
  const int nchunks = GEGLU ? (2 * p.N) / BNC : p.N / BNC;
  const int mblocks = (p.M + AR_BM - 1) / AR_BM;
  // split the chunks over blocks until the grid covers the chip (each split re-loads its A rows
  // into registers; they come from L2)
  int groups = 1;
  const int target = 256 * areg_minb<KS, TI, RING>();
  while (mblocks * groups < target && nchunks / (groups * 2) >= 2) groups *= 2;
  const int per = (nchunks + groups - 1) / groups;
  groups = (nchunks + per - 1) / per;   // no block without chunks
  const size_t lds = (size_t)RING * BNC * (KS / 2) * 128;
  auto* kfn = &gemm_areg_kernel<KS, TI, RING, RW, GEGLU, LNK, GNK>;
  // > 64 KiB dynamic LDS opt-in, once per process (thread-safe static init)
  static const bool once = [&] {
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return true;
  }();
  (void)once;
  hipLaunchKernelGGL(kfn, dim3(mblocks, groups), dim3(AR_THREADS), lds, s, p, per);
}

}  // namespace

// K = 320: 64-row chunks, 3-deep ring (120 KiB); K = 640: 32-row chunks, 3-deep ring (120 KiB)
bool gemm_areg_ok(const GemmArgs& p) {
  if (p.conv || p.A2 || p.batch != 1 || p.out_f32 || p.ln_rows || p.chan_bias || p.split > 1) return false;
  if (p.ln_rows_fx != nullptr || p.row_stats != nullptr) return false;
  if (p.gn_stats != nullptr) {
    // GroupNorm fold: K = 320 / 640 tiles (not the K = 1280 variant), no LayerNorm, every
    // block's rows in one image (64 RW <= 256 rows), 8-channel vectors inside the groups
    if (p.ln_wsum || is_gated(p.act) || !(p.K == 320 || p.K == 640) || p.gn_hw <= 0 || p.gn_hw % 256 ||
        p.M % p.gn_hw)
      return false;
    if (p.gn_groups <= 0 || p.K % p.gn_groups || p.gn_gamma == nullptr || p.gn_beta == nullptr) return false;
  }
  if (p.ln_wsum && !(p.ln_eps > 0.f)) return false;
  if (!(p.K == 320 || p.K == 640) || p.lda % 8 || p.ldc % 8 || p.N % 8) return false;
  const bool gated = is_gated(p.act);
  const int bnc = p.K == 320 ? 64 : 32;
  if ((gated ? 2 * p.N : p.N) % bnc) return false;
  if (gated && p.stats) return false;
  if (p.stats && (p.stats_hw % 64 != 0)) return false;
  // 16-byte A fragment loads, 8-byte bias / residual / output quads
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.C & 7) || ((uintptr_t)p.residual & 7) || ((uintptr_t)p.bias & 7))
    return false;
  const long long lim = (1LL << 31) - 1;
  return ((long long)(p.Nw - 1) * (p.ldw ? p.ldw : p.K) + p.K) * 2 <= lim;
}

// Tiles (measured on the SD-1.5 batch-8 level-1/2 shapes, profiles/r2_areg_variants.jsonl,
// profiles/r2_areg_ring2_ab.txt): K = 320 on 64-row W chunks through a 3-deep ring (2 blocks per
// CU), 64 A rows per wave for the gated tiles (each LDS W fragment feeds 4 MFMAs); K = 640 on
// 32-row chunks through a 2-deep ring (80 KiB: 2 blocks per CU).  The measured-slower variants
// (1 block per CU, 3 blocks per CU, 16-row chunks, a K = 1280 tile) were removed in round 4
// (profiles/r2_areg_v4_ab.txt, profiles/r2_areg_k1280.txt; git history).
template <bool LNK>
void launch_gemm_areg_t(const GemmArgs& p, hipStream_t s) {
  const bool gated = is_gated(p.act);
  if (p.K == 320) {
    if (gated) launch_areg_t<10, 2, 3, 4, true, LNK>(p, s);   // RW = 4 spills without the gate pairing
    else launch_areg_t<10, 2, 3, 2, false, LNK>(p, s);
  } else {
    if (gated) launch_areg_t<20, 2, 2, 2, true, LNK>(p, s);
    else launch_areg_t<20, 2, 2, 2, false, LNK>(p, s);
  }
}

void launch_gemm_areg(const GemmArgs& p, hipStream_t s) {
  if (p.gn_stats != nullptr) {
    // GroupNorm-folded proj_in (non-gated, K = 320 / 640): the default tiles of those shapes
    if (p.K == 320) launch_areg_t<10, 2, 3, 2, false, false, true>(p, s);
    else launch_areg_t<20, 2, 2, 2, false, false, true>(p, s);
    return;
  }
  if (p.ln_wsum != nullptr) launch_gemm_areg_t<true>(p, s);
  else launch_gemm_areg_t<false>(p, s);
}
