// Ping-pong 8-wave MFMA GEMM / implicit-GEMM convolution.
//
// Same contract as gemm_kernel (gemm_impl.h: D[n][m] = W[n][:] . A[m][:], W rows on the MFMA
// row axis so each lane owns 4 consecutive output channels; shared epilogue tile_epilogue), with
// the mainloop rebuilt around what the round-1 PMC counters showed (s_waitcnt waits 33 % of wave
// cycles: every k-tile drained its LDS-DMA at a __syncthreads):
//
// * one 512-thread block per CU (8 waves, 2 per SIMD), tile BM x BN x 64, 2 LDS buffers;
// * each k-tile runs as 4 PHASES, one per quadrant of the wave's output tile
//   (n-half, m-half) = (a,a) (a,b) (b,b) (b,a): the W fragments of an n-half are read once and
//   used twice, the A fragments of both m-halves stay in registers for the whole k-tile, so a
//   wave issues TI + TJ ds_read_b128 per 32-deep k-step for TI * TJ MFMAs;
// * the staging is split into 4 PARTS per k-tile (LDS regions A-m-half-a, W-n-half-a,
//   A-m-half-b, W-n-half-b), one part issued per phase by buffer-resource LDS-DMA, 5-6 phases
//   ahead of its first read and >= 2 phases after the last read of the bytes it overwrites;
//   a COUNTED `s_waitcnt vmcnt` (never 0 in the steady state) + raw s_barrier publish it, so DMA
//   stays in flight across every barrier (cdna_hip_programming.md §5 "Pipelining across
//   barriers", the 8-phase template);
// * waves 4-7 run one barrier behind waves 0-3 (stagger), so on every SIMD one wave's MFMA
//   cluster overlaps its partner's fragment reads / DMA issue;
// * regions whose row count is not a multiple of 64 (one DMA round = 8 rows per wave) let the
//   idle waves of the partial round DMA an out-of-range (zero) row into a junk LDS slab, so every
//   wave issues the same number of DMAs per part and the vmcnt counts are compile-time.
//
// Supported A modes: CONV 0 (row-major, optional second source A2 for a channel concatenation)
// and CONV 2 (NHWC 3x3 / strided conv with Cin % 64 == 0, parity-upsample classes); bf16 out;
// GEGLU/SwiGLU; split-K through the partial-slab path of gemm_impl.h.
#pragma once
#include <type_traits>

#include "gemm_impl.h"

namespace {

template <int N>
CM_DEVICE void wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }

template <int BM, int BN, int WM, int WN>
struct PPGeom {
  static constexpr int TI = BN / WN / 16, TJ = BM / WM / 16;
  static constexpr int TIa = (TI + 1) / 2, TIb = TI / 2, TJa = (TJ + 1) / 2, TJb = TJ / 2;
  // region rows (part types 0..3 = A m-half a, W n-half a, A m-half b, W n-half b)
  static constexpr int R0 = WM * 16 * TJa, R1 = WN * 16 * TIa, R2 = WM * 16 * TJb, R3 = WN * 16 * TIb;
  // region row offsets inside one buffer (rows of 128 B)
  static constexpr int O0 = 0, O2 = R0, O1 = BM, O3 = BM + R1;
  static constexpr int TILE_ROWS = BM + BN;
  static constexpr int NR0 = (R0 + 63) / 64, NR1 = (R1 + 63) / 64, NR2 = (R2 + 63) / 64, NR3 = (R3 + 63) / 64;
  static constexpr bool JUNK = (R0 % 64) || (R1 % 64) || (R2 % 64) || (R3 % 64);
  static constexpr int JUNK_ROW = 2 * TILE_ROWS;           // 64 junk rows after the two buffers
  static constexpr int STAGE_ROWS = 2 * TILE_ROWS + (JUNK ? 64 : 0);
  static constexpr int PERIOD = NR0 + NR1 + NR2 + NR3;     // DMAs per wave per k-tile
  static constexpr int OBN_ = BN;                          // (GEGLU halves it in the epilogue)
};

template <int BM, int BN, int WM, int WN, bool GEGLU>
constexpr size_t pp_lds_bytes() {
  using G = PPGeom<BM, BN, WM, WN>;
  constexpr size_t st = (size_t)G::STAGE_ROWS * 128;
  constexpr size_t ep = (size_t)BM * ((GEGLU ? BN / 2 : BN) + 8) * 2;
  return st > ep ? st : ep;
}

// DIAG bit 2 probe: x -> silu(x * s + t) on one 8-element A fragment (s, t lane constants)
CM_DEVICE bf16x8_t gn_silu_probe(bf16x8_t a, int lane) {
  float f[8];
  unpack8(__builtin_bit_cast(uint4, a), f);
  const float sc = 1.f + 0.001f * (lane & 7), sh = 0.01f * (lane >> 3);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = silu_f(fmaf(f[e], sc, sh));
  return as_bf16x8(pack8(f));
}

#ifndef PP_DIAG_DEFAULT
#define PP_DIAG_DEFAULT 0
#endif

// SCHED: 0 = four quadrant phases per k-tile (J0 loads W-a and A-a), 1 = four phases with the
// W-a load moved to J3 of the previous k-tile, 2 = two phases per k-tile (W-a x A, W-b x A).
// (Reading the next phase's fragments inside the current MFMA cluster was tried: slower on every
// tile, and the early half would read parts the late half has not waited for; profiles/r2_ppdiag_sched3.jsonl.)
// (Issuing the LDS-DMA parts inside the MFMA clusters instead of the load segments was tried in
// round 4: 3-11 % slower on every conv, profiles/r4_pp_sched3_ab.txt.)
// (A gated 256x160 tile on 4x2 waves -- value / gate rows interleaved at 8-row granularity, paired
// by v_permlane32_swap in the epilogue -- was correct but no faster than the 8x1 gated tile on the
// level-3 GEGLU, 68.3 us; round 4, profiles/r4_producer_waves_ab.txt.)
// (8 LDS-DMA-only producer waves beside the 8 MFMA waves of the 128x160 / 128x128 tiles, issuing
// the parts at the same barrier points, 1 block per CU: correct, picked for 9 shapes in situ, but
// the bench step was 0.7 % slower; round 4, profiles/r4_producer_waves_ab.txt.)
// DIAG (timing diagnostics only, tools/ppdiag.hip; results are wrong): bit 0 drops the mainloop
// DMA, bit 1 its barriers, bit 2 adds a GroupNorm+SiLU cost probe on the A fragments (variant
// builds with -DPP_DIAG_DEFAULT=4, profiles/r4_gn_prologue_probe.txt)
template <int BM, int BN, int WM, int WN, int CONV, bool GEGLU, int SCHED, int DIAG = 0>
__global__ void __launch_bounds__(512, 1) gemm_pp_kernel(GemmArgs p, float* __restrict__ partial) {
  constexpr bool SPREAD = SCHED == 1;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  using G = PPGeom<BM, BN, WM, WN>;
  static_assert(WM * WN == 8, "8 waves");
  static_assert(CONV == 0 || CONV == 2, "buffer-resource A modes only");
  constexpr int TI = G::TI, TJ = G::TJ, TIa = G::TIa, TIb = G::TIb, TJa = G::TJa, TJb = G::TJb;
  static_assert(TIb >= 1 && TJb >= 1, "each wave tile splits into 2 x 2 quadrants");
  static_assert(!GEGLU || (TI % 2 == 0), "geglu pairs");
  constexpr int TILE = G::TILE_ROWS * 8;   // uint4 per buffer
  constexpr int OOB = (int)0x80000000;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const bool late = wave >= 4;             // staggered half (one barrier behind)

  const int nN = GEGLU ? (p.N + BN / 2 - 1) / (BN / 2) : (p.N + BN - 1) / BN;
  const int nM = (p.M + BM - 1) / BM;
  const int lin = xcd_remap(blockIdx.x, nN * nM);
  int tn, tm;
  tile_of(lin, nM, nN, p.raster, tm, tn);
  const int batch = blockIdx.z;
  const int m0 = tm * BM;
  const int n0 = GEGLU ? tn * (BN / 2) : tn * BN;

  const uint16_t* __restrict__ A = p.A + (long long)batch * p.sA;
  const uint16_t* __restrict__ W = p.W + (long long)batch * p.sW;
  const int ldw = p.ldw ? p.ldw : p.K;

  // ---- per-lane DMA state.  LDS region row rho of round r: 64 r + 8 wave + (lane >> 3); the
  // lane moves logical chunk (lane & 7) ^ swz of that row (source-side swizzle, rule 21).
  const int slot = lane & 7;
  const int rsub = 8 * wave + (lane >> 3);
  auto chunk_of = [&](int ldsrow) { return slot ^ ((ldsrow >> 1) & 7); };
  // block row (0..BM) of A region h (0: m-half a, 1: m-half b), region row rho
  auto a_row = [&](int h, int rho) {
    const int per = 16 * (h ? TJb : TJa);
    const int w = rho / per, rem = rho - w * per;
    return w * (BM / WM) + (h ? 16 * TJa : 0) + rem;
  };
  auto w_row = [&](int h, int rho) {
    const int per = 16 * (h ? TIb : TIa);
    const int w = rho / per, rem = rho - w * per;
    return w * (BN / WN) + (h ? 16 * TIa : 0) + rem;
  };

  // A operand: buffer resource + per-round voffset / conv tap mask (regions 0 and 2)
  __amdgpu_buffer_rsrc_t rsA, rsW, rsA2;
  long long biasA = 0;
  if constexpr (CONV == 2) biasA = ((long long)p.pad * p.IW + p.pad) * p.Cin * 2;
  {
    const long long a_bytes = CONV ? (long long)p.M / (p.Ho * p.Wo) * p.IH * p.IW * p.Cin * 2
                                   : ((long long)(p.M - 1) * p.lda + (p.A2 ? p.ka : p.K)) * 2;
    rsA = make_rsrc((const char*)A - biasA, a_bytes + biasA);
    rsW = make_rsrc(W, ((long long)(p.Nw - 1) * ldw + p.K) * 2);
    if constexpr (CONV == 0) {
      if (p.A2 != nullptr) rsA2 = make_rsrc(p.A2, ((long long)(p.M - 1) * p.lda2 + (p.K - p.ka)) * 2);
    }
  }
  constexpr int NRA = G::NR0 + G::NR2;
  int a_vo[NRA], a_mask[CONV == 2 ? NRA : 1], a_vo2[CONV == 0 ? NRA : 1];
  {
    const int pad_y = p.parity ? 1 - (batch >> 1) : p.pad;
    const int pad_x = p.parity ? 1 - (batch & 1) : p.pad;
#pragma unroll
    for (int q = 0; q < NRA; ++q) {
      const int h = q < G::NR0 ? 0 : 1;
      const int r = h ? q - G::NR0 : q;
      const int R = h ? G::R2 : G::R0;
      const int rho = 64 * r + rsub;
      const int ldsrow = (h ? G::O2 : G::O0) + rho;
      const int row = m0 + a_row(h, rho);
      const int ch = chunk_of(ldsrow);
      const bool ok = rho < R && row < p.M;
      if constexpr (CONV == 0) {
        a_vo[q] = ok ? (int)(((long long)row * p.lda + ch * 8) * 2) : OOB;
        a_vo2[q] = ok ? (int)(((long long)row * p.lda2 + ch * 8) * 2) : OOB;
      } else {
        const int m = ok ? row : 0;
        const int hw = p.Ho * p.Wo;
        const int b = m / hw;
        const int rr = m - b * hw;
        const int oy = rr / p.Wo;
        const int ox = rr - oy * p.Wo;
        const int cy = oy * p.stride - pad_y, cx = ox * p.stride - pad_x;
        a_vo[q] = ok ? (int)(((((long long)b * p.IH + cy) * p.IW + cx) * p.Cin + ch * 8) * 2 + biasA) : OOB;
        int mk = 0;
        for (int ky = 0; ky < p.ksize; ++ky)
          for (int kx = 0; kx < p.ksize; ++kx) {
            const int iy = cy + ky, ix = cx + kx;
            if ((unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW) mk |= 1 << (ky * p.ksize + kx);
          }
        a_mask[q] = ok ? mk : 0;
      }
    }
  }
  constexpr int NRW = G::NR1 + G::NR3;
  int w_vo[NRW];
#pragma unroll
  for (int q = 0; q < NRW; ++q) {
    const int h = q < G::NR1 ? 0 : 1;
    const int r = h ? q - G::NR1 : q;
    const int R = h ? G::R3 : G::R1;
    const int rho = 64 * r + rsub;
    const int ldsrow = (h ? G::O3 : G::O1) + rho;
    const int br = w_row(h, rho);   // block n row
    int gr = -1;
    if (rho < R && br < BN) {
      if constexpr (GEGLU) {
        const int blk = br >> 4, within = br & 15;
        const int nout = n0 + (blk >> 1) * 16 + within;
        gr = (nout < p.N) ? ((blk & 1) ? p.N + nout : nout) : -1;
      } else {
        const int n = n0 + br;
        gr = n < p.Nw ? n : -1;
      }
    }
    w_vo[q] = gr >= 0 ? (int)(((long long)gr * ldw + chunk_of(ldsrow) * 8) * 2) : OOB;
  }

  // wave-uniform conv tap state of the A k-tile being staged (k-tiles staged in order)
  int t_ci = 0, t_kx = 0, t_ky = 0, tap_tile = 0;
  const int nk_all = p.K / BK;
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int kt0 = blockIdx.y * per;
  const int kend = min(nk_all, kt0 + per);
  const int nk = max(0, kend - kt0);
  if constexpr (CONV == 2) {
    const int k0 = kt0 * BK;
    const int tap = k0 / p.Cin;
    t_ci = k0 - tap * p.Cin;
    t_ky = tap / p.ksize;
    t_kx = tap - t_ky * p.ksize;
    tap_tile = kt0;
  }

  // ---- stage part PT of k-tile u into buffer b (every wave issues exactly NR_PT DMAs)
  auto dst = [&](int b, int regoff, int r, int R) -> uint4* {
    const bool real = 64 * r + 8 * wave < R;   // wave-uniform
    return real ? smem + b * TILE + (regoff + 64 * r + 8 * wave) * 8 : smem + (G::JUNK_ROW + 8 * wave) * 8;
  };
  auto stage = [&](auto PTc, int u, int b) {
    constexpr int PT = decltype(PTc)::value;
    const int k0 = u * BK;
    if constexpr (PT == 0 || PT == 2) {
      constexpr int h = PT == 2;
      constexpr int NR = h ? G::NR2 : G::NR0;
      constexpr int QB = h ? G::NR0 : 0;
      constexpr int R = h ? G::R2 : G::R0;
      constexpr int OFF = h ? G::O2 : G::O0;
      if constexpr (CONV == 0) {
        if (p.A2 != nullptr && k0 >= p.ka) {
#pragma unroll
          for (int r = 0; r < NR; ++r) blds16(rsA2, dst(b, OFF, r, R), a_vo2[QB + r], (k0 - p.ka) * 2);
        } else {
#pragma unroll
          for (int r = 0; r < NR; ++r) blds16(rsA, dst(b, OFF, r, R), a_vo[QB + r], k0 * 2);
        }
      } else {
        if constexpr (PT == 0) {
          if (tap_tile < u) {   // advance to k-tile u (one step: A parts are staged in tile order)
            t_ci += BK;
            if (t_ci == p.Cin) {
              t_ci = 0;
              if (++t_kx == p.ksize) { t_kx = 0; ++t_ky; }
            }
            tap_tile = u;
          }
        }
        const int soff = ((t_ky * p.IW + t_kx) * p.Cin + t_ci) * 2;
        const int tap = t_ky * p.ksize + t_kx;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int vo = ((a_mask[QB + r] >> tap) & 1) ? a_vo[QB + r] : OOB;
          blds16(rsA, dst(b, OFF, r, R), vo, soff);
        }
      }
    } else {
      constexpr int h = PT == 3;
      constexpr int NR = h ? G::NR3 : G::NR1;
      constexpr int QB = h ? G::NR1 : 0;
      constexpr int R = h ? G::R3 : G::R1;
      constexpr int OFF = h ? G::O3 : G::O1;
#pragma unroll
      for (int r = 0; r < NR; ++r) blds16(rsW, dst(b, OFF, r, R), w_vo[QB + r], k0 * 2);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // ---- fragment reads: lane offset (uint4 units) of row fr, logical chunk 4 ks + fq; the
  // region / subtile / buffer parts are compile-time immediates
  const int fr = lane & 15, fq = lane >> 4;
  int lo[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) lo[ks] = fr * 8 + ((4 * ks + fq) ^ ((fr >> 1) & 7));
  const int wbase_a = (G::O1 + wn * 16 * TIa) * 8, wbase_b = (G::O3 + wn * 16 * TIb) * 8;
  const int abase_a = (G::O0 + wm * 16 * TJa) * 8, abase_b = (G::O2 + wm * 16 * TJb) * 8;

  f32x4_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t wfa[TIa][2], wfb[TIb][2];      // W fragments of both n-halves
  bf16x8_t afa[TJa][2], afb[TJb][2];       // A fragments of both m-halves

  // ---- prologue: parts 0..5 (k-tile 0 whole, k-tile 1 A-a / W-a), then retire k-tile 0's
  // first two parts (PERIOD DMAs = one of each part type may stay in flight)
  if (nk > 0) {
    stage(I0{}, kt0, 0);
    stage(I1{}, kt0, 0);
    stage(I2{}, kt0, 0);
    stage(I3{}, kt0, 0);
  }
  if (nk > 1) {
    if constexpr (SCHED >= 2) {            // k-tile 1's A halves (issued by "P1 of k-tile -1")
      stage(I0{}, kt0 + 1, 1);
      stage(I2{}, kt0 + 1, 1);
      wait_vmcnt<G::NR0 + G::NR2>();
    } else if constexpr (SPREAD) {
      stage(I1{}, kt0 + 1, 1);
      stage(I0{}, kt0 + 1, 1);
      wait_vmcnt<G::PERIOD>();
    } else {
      stage(I0{}, kt0 + 1, 1);
      stage(I1{}, kt0 + 1, 1);
      wait_vmcnt<G::PERIOD>();
    }
  } else {
    wait_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();
  if (late) __builtin_amdgcn_s_barrier();
  if constexpr (SPREAD) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TIa; ++i) wfa[i][ks] = as_bf16x8(smem[wbase_a + 128 * i + lo[ks]]);
  }

  // one phase: quadrant J of local k-tile t (buffer B).  Fragment reads are spread so no phase
  // carries more than one operand half: J0 A-a, J1 A-b, J2 W-b, J3 W-a of the NEXT k-tile (from
  // the other buffer; the quadrant order (a,a) (a,b) (b,b) (b,a) leaves W-a idle in J2/J3), which
  // is why W-a of tile t+2 is staged in J2 and A-a in J3.  Issues the part scheduled 5-6 phases
  // ahead of its first read and >= 3 phases after the last read of the bytes it overwrites;
  // waits so that every part issued >= 4 phases ago has landed (reads of phase q+1)
  auto phase = [&](auto Jc, auto Bc, int t) {
    constexpr int J = decltype(Jc)::value;
    constexpr int B = decltype(Bc)::value;
    const uint4* Bs = smem + B * TILE;
    if constexpr (J == 0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (!SPREAD) {
#pragma unroll
          for (int i = 0; i < TIa; ++i) wfa[i][ks] = as_bf16x8(Bs[wbase_a + 128 * i + lo[ks]]);
        }
#pragma unroll
        for (int j = 0; j < TJa; ++j) afa[j][ks] = as_bf16x8(Bs[abase_a + 128 * j + lo[ks]]);
      }
    } else if constexpr (J == 1) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < TJb; ++j) afb[j][ks] = as_bf16x8(Bs[abase_b + 128 * j + lo[ks]]);
    } else if constexpr (J == 2) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TIb; ++i) wfb[i][ks] = as_bf16x8(Bs[wbase_b + 128 * i + lo[ks]]);
    } else if constexpr (SPREAD) {           // W-a of the next k-tile (other buffer; garbage past nk)
      const uint4* Bn = smem + (B ^ 1) * TILE;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TIa; ++i) wfa[i][ks] = as_bf16x8(Bn[wbase_a + 128 * i + lo[ks]]);
    }
    // part issued now: J=0 -> A-b of tile t+1, J=1 -> W-b of t+1, J=2 -> W-a of t+2, J=3 -> A-a of t+2
    constexpr int DU = (J + 2) >> 2 ? 2 : 1;
    const int u = t + DU;                  // local tile index of the part
    const bool issue = !(DIAG & 1) && u < nk;
    if (issue) {
      if constexpr (J == 0) stage(I2{}, kt0 + u, B ^ 1);
      else if constexpr (J == 1) stage(I3{}, kt0 + u, B ^ 1);
      else if constexpr (J == 2) { if constexpr (SPREAD) stage(I1{}, kt0 + u, B); else stage(I0{}, kt0 + u, B); }
      else { if constexpr (SPREAD) stage(I0{}, kt0 + u, B); else stage(I1{}, kt0 + u, B); }
      wait_vmcnt<G::PERIOD>();
    } else {
      wait_vmcnt<0>();
    }
    if constexpr (!(DIAG & 2)) __builtin_amdgcn_s_barrier();
    wait_lgkm<0>();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if constexpr (J == 0 || J == 1) {
#pragma unroll
        for (int i = 0; i < TIa; ++i) {
          if constexpr (J == 0) {
#pragma unroll
            for (int j = 0; j < TJa; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfa[i][ks], afa[j][ks], acc[i][j], 0, 0, 0);
          } else {
#pragma unroll
            for (int j = 0; j < TJb; ++j)
              acc[i][TJa + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfa[i][ks], afb[j][ks], acc[i][TJa + j], 0, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < TIb; ++i) {
          if constexpr (J == 3) {
#pragma unroll
            for (int j = 0; j < TJa; ++j)
              acc[TIa + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfb[i][ks], afa[j][ks], acc[TIa + i][j], 0, 0, 0);
          } else {
#pragma unroll
            for (int j = 0; j < TJb; ++j)
              acc[TIa + i][TJa + j] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfb[i][ks], afb[j][ks], acc[TIa + i][TJa + j], 0, 0, 0);
          }
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (!(DIAG & 2)) __builtin_amdgcn_s_barrier();
  };

  // SCHED 2: two phases per k-tile t (buffer B), each one MFMA cluster twice as long as a
  // quadrant's.  P0 reads W-a, A-a, A-b of t and issues W-a, W-b of t+1 (other buffer, whose W
  // regions were last read in P0 / P1 of t-1); P1 reads W-b of t and issues A-a, A-b of t+2 (this
  // buffer, A regions last read in P0 of t).  Every phase waits for all parts but its own, so the
  // parts the next phase reads have landed before the barrier that publishes them; the reads wait
  // for their data BEFORE the barrier because the other half overwrites bytes read in phase q
  // right after the barrier of phase q+1.
  auto mphase = [&](auto Pc, auto Bc, int t) {
    constexpr int P = decltype(Pc)::value;
    constexpr int B = decltype(Bc)::value;
    const uint4* Bs = smem + B * TILE;
    if constexpr (P == 0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < TIa; ++i) wfa[i][ks] = as_bf16x8(Bs[wbase_a + 128 * i + lo[ks]]);
#pragma unroll
        for (int j = 0; j < TJa; ++j) afa[j][ks] = as_bf16x8(Bs[abase_a + 128 * j + lo[ks]]);
#pragma unroll
        for (int j = 0; j < TJb; ++j) afb[j][ks] = as_bf16x8(Bs[abase_b + 128 * j + lo[ks]]);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TIb; ++i) wfb[i][ks] = as_bf16x8(Bs[wbase_b + 128 * i + lo[ks]]);
    }
    const int u = t + (P == 0 ? 1 : 2);
    if (!(DIAG & 1) && u < nk) {
      if constexpr (P == 0) {
        stage(I1{}, kt0 + u, B ^ 1);
        stage(I3{}, kt0 + u, B ^ 1);
        wait_vmcnt<G::NR1 + G::NR3>();
      } else {
        stage(I0{}, kt0 + u, B);
        stage(I2{}, kt0 + u, B);
        wait_vmcnt<G::NR0 + G::NR2>();
      }
    } else {
      wait_vmcnt<0>();
    }
    wait_lgkm<0>();
    if constexpr ((DIAG & 4) && P == 0) {
      // cost probe of a GroupNorm+SiLU prologue on the A operand (results are wrong): every A
      // fragment read this k-tile is normalised and SiLU'd in registers before its MFMAs (the
      // per-channel scale / shift as lane constants: a LOWER bound of the fused prologue's VALU)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int j = 0; j < TJa; ++j) afa[j][ks] = gn_silu_probe(afa[j][ks], lane);
#pragma unroll
        for (int j = 0; j < TJb; ++j) afb[j][ks] = gn_silu_probe(afb[j][ks], lane);
      }
    }
    if constexpr (!(DIAG & 2)) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if constexpr (P == 0) {
#pragma unroll
        for (int i = 0; i < TIa; ++i) {
#pragma unroll
          for (int j = 0; j < TJa; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfa[i][ks], afa[j][ks], acc[i][j], 0, 0, 0);
#pragma unroll
          for (int j = 0; j < TJb; ++j)
            acc[i][TJa + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfa[i][ks], afb[j][ks], acc[i][TJa + j], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < TIb; ++i) {
#pragma unroll
          for (int j = 0; j < TJb; ++j)
            acc[TIa + i][TJa + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfb[i][ks], afb[j][ks], acc[TIa + i][TJa + j], 0, 0, 0);
#pragma unroll
          for (int j = 0; j < TJa; ++j)
            acc[TIa + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfb[i][ks], afa[j][ks], acc[TIa + i][j], 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (!(DIAG & 2)) __builtin_amdgcn_s_barrier();
  };

  // two k-tiles per iteration so the buffer of every phase is a compile-time offset
  if constexpr (SCHED == 2) {
    for (int t = 0; t < nk; t += 2) {
      mphase(I0{}, I0{}, t);
      mphase(I1{}, I0{}, t);
      if (t + 1 >= nk) break;
      mphase(I0{}, I1{}, t + 1);
      mphase(I1{}, I1{}, t + 1);
    }
  } else {
    for (int t = 0; t < nk; t += 2) {
      phase(I0{}, I0{}, t);
      phase(I1{}, I0{}, t);
      phase(I2{}, I0{}, t);
      phase(I3{}, I0{}, t);
      if (t + 1 >= nk) break;
      phase(I0{}, I1{}, t + 1);
      phase(I1{}, I1{}, t + 1);
      phase(I2{}, I1{}, t + 1);
      phase(I3{}, I1{}, t + 1);
    }
  }
  if (!late) __builtin_amdgcn_s_barrier();   // re-align the two halves
  wait_vmcnt<0>();
  __syncthreads();

  tile_epilogue<BM, BN, WM, WN, GEGLU, false, TI, TJ, 512, true>(p, acc, smem, partial, m0, n0, batch, wm, wn, tid,
                                                          gridDim.y, blockIdx.y);
}

template <int BM, int BN, int WM, int WN, int CONV, bool GEGLU>
void launch_pp(const GemmArgs& p, float* ws, hipStream_t s) {
  const int nN = GEGLU ? (p.N + BN / 2 - 1) / (BN / 2) : (p.N + BN - 1) / BN;
  const int nM = (p.M + BM - 1) / BM;
  const int split = (ws != nullptr && p.split > 1) ? p.split : 1;
  dim3 grid(nN * nM, split, p.batch);
  constexpr size_t lds = pp_lds_bytes<BM, BN, WM, WN, GEGLU>();
  // the two-phase schedule (SCHED 2; 593 -> 573 ms/step, commit 88fbe5c).  SCHED 0 / 1 are no
  // longer instantiated in the library (tools/ppdiag.hip still builds them for diagnostics)
  auto* kfn = &gemm_pp_kernel<BM, BN, WM, WN, CONV, GEGLU, 2, PP_DIAG_DEFAULT>;
  // > 64 KiB dynamic LDS opt-in, once per process (thread-safe static init)
  static const bool once = [&] {
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return true;
  }();
  (void)once;
  hipLaunchKernelGGL(kfn, grid, dim3(512), lds, s, p, ws);
  if (split > 1) launch_splitk_reduce<false>(p, ws, split, s);
}

// ping-pong tile menu (gemm.hip kPP* configs)
template <int CONV>
void launch_pp_cfg(const GemmArgs& p, float* ws, hipStream_t s) {
  if (is_gated(p.act)) {
    // (256x256 gated spills: 256 VGPRs).  cfg 8: 256 x 160 with the 8 waves stacked along M
    // (wave tile 32 x 160: 5 value/gate pairs), 80 outputs per block -- at M = 2048 x 5120 that
    // is 512 blocks = 2 full rounds instead of 640 = 2.5 rounds of the 64-output 256 x 128 tile
    if (p.cfg == 8) launch_pp<256, 160, 8, 1, CONV, true>(p, ws, s);
    else launch_pp<256, 128, 4, 2, CONV, true>(p, ws, s);
    return;
  }
  switch (p.cfg) {
    case 8: launch_pp<256, 160, 4, 2, CONV, false>(p, ws, s); break;
    case 9: launch_pp<256, 128, 4, 2, CONV, false>(p, ws, s); break;
    case 10: launch_pp<128, 256, 2, 4, CONV, false>(p, ws, s); break;
    case 20: launch_pp<128, 160, 4, 2, CONV, false>(p, ws, s); break;
    case 21: launch_pp<128, 128, 4, 2, CONV, false>(p, ws, s); break;
    case 22: launch_pp<128, 64, 4, 2, CONV, false>(p, ws, s); break;
    default: launch_pp<256, 256, 4, 2, CONV, false>(p, ws, s); break;
  }
}

}  // namespace

#define GEMM_PP_TU_ENTRY(NAME, CONV) \
  void NAME(const GemmArgs& p, float* ws, hipStream_t s) { launch_pp_cfg<CONV>(p, ws, s); }
