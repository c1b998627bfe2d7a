// Halo-staged 3x3 convolution on the ping-pong 8-wave MFMA mainloop (the
// UNet / VAE 3x3 convs, reference hot loop /root/reference/src/backend.py:270-295).
//
// Why it exists: the ping-pong implicit-GEMM conv (gemm_pp.h CONV 2) stages, for every 64-deep
// k-tile (one tap x 64 input channels), the BM shifted input rows of that tap plus BN weight rows
// by LDS-DMA, so 8 of every 9 A rows it stages are a neighbouring tap's rows again.
//
// What: a block owns BM output pixels that are whole output rows of one image (BM % Wo == 0);
// per 64-channel chunk c it stages ONE halo tile -- the (BM/Wo + 2) x (Wo + 2) input pixels
// those rows read through any tap, zero outside the image (buffer-resource OOB) -- and then runs
// the chunk's 9 taps as 9 k-tiles whose A fragments are read from the halo at a per-tap row
// offset ky (Wo + 2) + kx.  Per k-tile the DMA carries BN weight rows plus 1/9 of a halo:
// 25.6 KB instead of 52 KB at 256x160 on the 64^2 level.
//
// Measured (profiles/r3_bench_halo.jsonl, profiles/r3_dma_bound.txt): NOT faster than the CONV-2
// tiles on any SD-1.5 shape (level-1 68.9 vs 65.4 us): the convs are not bound by DMA bytes.
// Kept as opt-in tile configs 24/25 that the autotuner weighs for every shape.
//
// Pipeline (two phases per k-tile, as gemm_pp.h SCHED 2): P0 reads the W-a and all A fragments of
// k-tile t and issues W of t+1 into the other W buffer; P1 reads W-b of t and issues ONE 64-row
// round of the NEXT chunk's halo into the other halo buffer (rounds 0..NRH-1 at taps 0..NRH-1,
// NRH <= 8, so the last round is waited one phase and read two phases after its issue); every
// phase waits for all DMA but its own before its barrier, so data issued in phase q is visible
// from phase q+2 on.  The halo buffer a chunk writes was last read in the previous chunk (>= 3
// phases earlier).  Waves 4-7 run one barrier behind waves 0-3 (stagger), s_setprio around the
// MFMA clusters, counted vmcnt only (DMA stays in flight across barriers).
// Split-K splits the chunks (each slice: whole chunks x 9 taps); epilogue: tile_epilogue.
#pragma once
#include "gemm_impl.h"

namespace {

template <int N>
CM_DEVICE void halo_wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }

constexpr int HALO_MAX_ROUNDS = 8;   // 64-row DMA rounds per halo (<= 8: see the pipeline note)

// LDS geometry: [W buffer 0][W buffer 1][64 junk rows][halo 0][halo 1], rows of 128 bytes
template <int BN>
struct HaloGeom {
  static constexpr int WROWS = BN;
  static constexpr int JUNK = 2 * BN;                 // 64 junk rows (partial DMA rounds)
  static constexpr int H0 = 2 * BN + 64;              // first halo buffer
};

__host__ __device__ inline int halo_rows(int BM, int Wo) { return (BM / Wo + 2) * (Wo + 2); }
// halo buffer rows: whole 8-row wave pieces
__host__ __device__ inline int halo_stride(int BM, int Wo) { return (halo_rows(BM, Wo) + 7) / 8 * 8; }
__host__ __device__ inline size_t halo_lds_bytes(int BM, int BN, int Wo) {
  const size_t st = ((size_t)2 * BN + 64 + 2 * (size_t)halo_stride(BM, Wo)) * 128;
  const size_t ep = (size_t)BM * (BN + 8) * 2;
  return st > ep ? st : ep;
}

template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(512, 1) gemm_halo_kernel(GemmArgs p, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  using H = HaloGeom<BN>;
  static_assert(WM * WN == 8, "8 waves");
  constexpr int TI = BN / WN / 16, TJ = BM / WM / 16;
  constexpr int TIa = (TI + 1) / 2, TIb = TI / 2;
  static_assert(TIb >= 1, "two W halves");
  // W parts: a = the first TIa subtiles of every wave's n range, b = the rest
  constexpr int R1 = WN * 16 * TIa, R3 = WN * 16 * TIb;
  constexpr int NR1 = (R1 + 63) / 64, NR3 = (R3 + 63) / 64, NRW = NR1 + NR3;
  constexpr int O1 = 0, O3 = R1;                       // rows inside a W buffer
  constexpr int OOB = (int)0x80000000;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const bool late = wave >= 4;

  const int nN = (p.N + BN - 1) / BN;
  const int nM = p.M / BM;                             // host: (Ho*Wo) % BM == 0
  const int lin = xcd_remap(blockIdx.x, nN * nM);
  const int tn = lin % nN, tm = lin / nN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int hw = p.Ho * p.Wo;
  const int img = m0 / hw;
  const int y0 = (m0 - img * hw) / p.Wo;               // first output row of the tile
  const int HW2 = p.Wo + 2;
  const int HR = halo_rows(BM, p.Wo);
  const int HS = halo_stride(BM, p.Wo);
  const int NRH = (HR + 63) / 64;                       // host: <= HALO_MAX_ROUNDS
  const int ldw = p.ldw ? p.ldw : p.K;

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A, (long long)p.M / hw * p.IH * p.IW * p.Cin * 2);
  const __amdgpu_buffer_rsrc_t rsW = make_rsrc(p.W, ((long long)(p.Nw - 1) * ldw + p.K) * 2);

  // ---- DMA lane geometry: LDS row rho of round r = 64 r + 8 wave + (lane >> 3); the lane moves
  // logical 16-byte chunk (lane & 7) ^ swz of that row (source-side swizzle)
  const int slot = lane & 7;
  const int rsub = 8 * wave + (lane >> 3);
  auto chunk_of = [&](int ldsrow) { return slot ^ ((ldsrow >> 1) & 7); };

  // halo source offsets (bytes, channel chunk 0) of this lane for every round
  int h_vo[HALO_MAX_ROUNDS];
#pragma unroll
  for (int r = 0; r < HALO_MAX_ROUNDS; ++r) {
    const int rho = 64 * r + rsub;
    const int hy = rho / HW2, hx = rho - hy * HW2;
    const int iy = y0 - 1 + hy, ix = hx - 1;
    const bool ok = rho < HR && (unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW;
    h_vo[r] = ok ? (int)((((long long)img * p.IH + iy) * p.IW + ix) * p.Cin * 2 + chunk_of(rho) * 16) : OOB;
  }
  // W source offsets (bytes, k 0) of this lane for the rounds of parts a and b
  int w_vo[NRW];
#pragma unroll
  for (int q = 0; q < NRW; ++q) {
    const int h = q < NR1 ? 0 : 1;
    const int r = h ? q - NR1 : q;
    const int R = h ? R3 : R1;
    const int rho = 64 * r + rsub;
    const int per = 16 * (h ? TIb : TIa);
    const int w = rho / per, rem = rho - w * per;
    const int br = w * (BN / WN) + (h ? 16 * TIa : 0) + rem;   // block W row
    const int n = n0 + br;
    w_vo[q] = (rho < R && n < p.Nw) ? (int)(((long long)n * ldw + chunk_of((h ? O3 : O1) + rho) * 8) * 2) : OOB;
  }

  // chunk range of this split-K slice
  const int nchunk_all = p.Cin / 64;
  const int cper = (nchunk_all + gridDim.y - 1) / gridDim.y;
  const int cbeg = blockIdx.y * cper;
  const int cend = min(nchunk_all, cbeg + cper);
  const int nk = max(0, cend - cbeg) * 9;

  // W part PT (1: a, 3: b) of local k-tile u into W buffer b
  auto stage_w = [&](auto PTc, int u, int b) {
    constexpr int PT = decltype(PTc)::value;
    constexpr int h = PT == 3;
    constexpr int NR = h ? NR3 : NR1, QB = h ? NR1 : 0, R = h ? R3 : R1, OFF = h ? O3 : O1;
    const int c = cbeg + u / 9, tap = u - (u / 9) * 9;
    const int soff = (tap * p.Cin + c * 64) * 2;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const bool real = 64 * r + 8 * wave < R;         // wave-uniform
      uint4* d = real ? smem + (b * H::WROWS + OFF + 64 * r + 8 * wave) * 8 : smem + (H::JUNK + 8 * wave) * 8;
      blds16(rsW, d, w_vo[QB + r], soff);
    }
  };
  // round r of the halo of local chunk cl into halo buffer hb.  r is wave-uniform: one scalar
  // branch per round keeps every voffset a compile-time-indexed register (a select chain over
  // h_vo was folded back into a runtime-indexed array in scratch, whose load then drained the
  // DMA queue through vmcnt)
  auto stage_h = [&](int r, int cl, int hb) {
    const bool real = 64 * r + 8 * wave < HR;          // wave-uniform
    uint4* d = real ? smem + (H::H0 + hb * HS + 64 * r + 8 * wave) * 8 : smem + (H::JUNK + 8 * wave) * 8;
    const int soff = (cbeg + cl) * 128;
    switch (r) {
      case 0: blds16(rsA, d, h_vo[0], soff); break;
      case 1: blds16(rsA, d, h_vo[1], soff); break;
      case 2: blds16(rsA, d, h_vo[2], soff); break;
      case 3: blds16(rsA, d, h_vo[3], soff); break;
      case 4: blds16(rsA, d, h_vo[4], soff); break;
      case 5: blds16(rsA, d, h_vo[5], soff); break;
      case 6: blds16(rsA, d, h_vo[6], soff); break;
      default: blds16(rsA, d, h_vo[7], soff); break;
    }
  };

  // ---- fragment addressing: W as gemm_pp.h; A rows of fragment j at halo row hb_j + tap offset
  const int fr = lane & 15, fq = lane >> 4;
  int lo[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) lo[ks] = fr * 8 + ((4 * ks + fq) ^ ((fr >> 1) & 7));
  const int wbase_a = (O1 + wn * 16 * TIa) * 8, wbase_b = (O3 + wn * 16 * TIb) * 8;
  int hrow[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int ml = wm * (BM / WM) + 16 * j + fr;
    hrow[j] = (ml / p.Wo) * HW2 + (ml - (ml / p.Wo) * p.Wo);
  }

  f32x4_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t wfa[TIa][2], wfb[TIb][2], af[TJ][2];

  using I1 = std::integral_constant<int, 1>;
  using I3 = std::integral_constant<int, 3>;
  // ---- prologue: the first chunk's whole halo and k-tile 0's W, all landed
  if (nk > 0) {
    for (int r = 0; r < NRH; ++r) stage_h(r, 0, 0);
    stage_w(I1{}, 0, 0);
    stage_w(I3{}, 0, 0);
  }
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  if (late) __builtin_amdgcn_s_barrier();

  // one k-tile t (W buffer B, compile-time): P0 then P1
  auto ktile = [&](auto Bc, int t) {
    constexpr int B = decltype(Bc)::value;
    const int cl = t / 9, tap = t - cl * 9;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int toff = ky * HW2 + kx;
    const uint4* Ws = smem + B * H::WROWS * 8;
    const uint4* Hs = smem + (H::H0 + (cl & 1) * HS) * 8;
    // ---- P0: W-a and every A fragment of t; issue W of t+1
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < TIa; ++i) wfa[i][ks] = as_bf16x8(Ws[wbase_a + 128 * i + lo[ks]]);
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int row = hrow[j] + toff;
        af[j][ks] = as_bf16x8(Hs[row * 8 + ((4 * ks + fq) ^ ((row >> 1) & 7))]);
      }
    }
    if (t + 1 < nk) {
      stage_w(I1{}, t + 1, B ^ 1);
      stage_w(I3{}, t + 1, B ^ 1);
      wait_vmcnt<NRW>();
    } else {
      wait_vmcnt<0>();
    }
    halo_wait_lgkm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TIa; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfa[i][ks], af[j][ks], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- P1: W-b of t; issue round `tap` of the next chunk's halo
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TIb; ++i) wfb[i][ks] = as_bf16x8(Ws[wbase_b + 128 * i + lo[ks]]);
    if (tap < NRH && (cl + 1) * 9 < nk) {
      stage_h(tap, cl + 1, (cl + 1) & 1);
      wait_vmcnt<1>();
    } else {
      wait_vmcnt<0>();
    }
    halo_wait_lgkm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TIb; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[TIa + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfb[i][ks], af[j][ks], acc[TIa + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  for (int t = 0; t < nk; t += 2) {
    ktile(I0{}, t);
    if (t + 1 >= nk) break;
    ktile(I1{}, t + 1);
  }
  if (!late) __builtin_amdgcn_s_barrier();   // re-align the two halves
  wait_vmcnt<0>();
  __syncthreads();

  tile_epilogue<BM, BN, WM, WN, false, false, TI, TJ, 512, true>(p, acc, smem, partial, m0, n0, 0, wm, wn, tid,
                                                                gridDim.y, blockIdx.y);
}

template <int BM, int BN, int WM, int WN>
void launch_halo_t(const GemmArgs& p, float* ws, hipStream_t s) {
  const int nN = (p.N + BN - 1) / BN;
  const int nM = p.M / BM;
  const int split = (ws != nullptr && p.split > 1) ? p.split : 1;
  dim3 grid(nN * nM, split, 1);
  const size_t lds = halo_lds_bytes(BM, BN, p.Wo);
  auto* kfn = &gemm_halo_kernel<BM, BN, WM, WN>;
  static const bool once = [&] {
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)once;
  hipLaunchKernelGGL(kfn, grid, dim3(512), lds, s, p, ws);
  if (split > 1) launch_splitk_reduce<false>(p, ws, split, s);
}

}  // namespace

// tile of halo config c (gemm.hip kHalo*): 0 = 256x160 (4x2 waves), 1 = 128x160 (4x2)
inline int halo_bm(int c) { return c == 1 ? 128 : 256; }
inline int halo_bn(int) { return 160; }

// eligibility: NHWC 3x3, stride 1, pad 1, no upsample / parity, Cin % 64 == 0, single batch
// slice, output tiles of whole rows of one image, halo within 8 DMA rounds and the LDS budget
inline bool halo_ok(const GemmArgs& p, int BM, int BN) {
  if (!p.conv || p.ksize != 3 || p.stride != 1 || p.pad != 1 || p.upsample || p.parity || p.batch != 1) return false;
  if (p.Cin % 64 != 0 || p.K != 9 * p.Cin || p.out_f32 || p.A2 != nullptr) return false;
  if (p.Ho != p.IH || p.Wo != p.IW || p.Wo % 16 != 0 || BM % p.Wo != 0 || (p.Ho * p.Wo) % BM != 0) return false;
  if (p.N % 8 != 0 || p.ldc % 8 != 0 || p.N <= 16) return false;
  const int cbs = p.ldcb ? p.ldcb : p.N;
  if (cbs % 4 != 0 || p.ln_rows != nullptr || p.ln_wsum != nullptr || p.kv8 != nullptr) return false;
  if ((halo_rows(BM, p.Wo) + 63) / 64 > HALO_MAX_ROUNDS) return false;
  if (halo_lds_bytes(BM, BN, p.Wo) > 160 * 1024) return false;
  const long long a_bytes = (long long)p.M * p.Cin * 2;     // input pixels = output pixels
  const long long w_bytes = ((long long)(p.Nw - 1) * (p.ldw ? p.ldw : p.K) + p.K) * 2;
  return a_bytes < (1LL << 31) && w_bytes < (1LL << 31);
}

void gemm_halo_launch(const GemmArgs& p, float* ws, hipStream_t s) {
  if (halo_bm(p.cfg - 24) == 128) launch_halo_t<128, 160, 4, 2>(p, ws, s);
  else launch_halo_t<256, 160, 4, 2>(p, ws, s);
}
