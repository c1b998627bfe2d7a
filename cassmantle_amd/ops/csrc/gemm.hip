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
//   staging, no ds_write; each wave-instruction fills 8 rows x 128 B.  The next k-tile's DMA is
//   issued before the current tile's MFMAs into the other of two LDS buffers; one barrier per
//   k-tile.  Out-of-range rows / conv padding point their lane at a 16-byte zero page.
// * LDS rows are 128 B; logical chunk c of row r lives in slot c ^ ((r >> 1) & 7).  The DMA
//   image is lane-linear, so the swizzle is applied on the SOURCE address (rule 21) and the
//   same XOR on the ds_read; each 16-lane ds_read_b128 group then hits 16 distinct bank slots.
// * Tiles (BM x BN x 64, 4 waves as WM x WN): 128x128 (2x2), 256x64 (4x1) for N = 64 (mod
//   128), 256x16 (4x1) for the 3/4-channel conv_out layers.
// * GEGLU (transformer FF): W tile rows interleave 16-row value/gate blocks, so each lane
//   holds h and g of the same output column and computes h * gelu(g) in registers.
// * Block ids are remapped XCD-aware so tiles that share an A panel run on one XCD's L2.
#include "common.h"
#include "kernels.h"

__device__ uint4 g_zero_page[4];   // zero-initialised; source of padded / out-of-range chunks

namespace {

constexpr int BK = 64;
constexpr int THREADS = 256;

CM_DEVICE int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

typedef __attribute__((address_space(3))) void lds_void;

CM_DEVICE void glds16(const void* src, uint4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_void*)lds_wave_base, 16, 0, 0);
}

template <int BM, int BN, int WM, int WN, int CONV, bool GEGLU, bool OUTF32>
__global__ void __launch_bounds__(THREADS, 2) gemm_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  constexpr int TILE = (BM + BN) * 8;      // uint4 per buffer
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TI = BN / WN / 16;         // n-subtiles per wave
  constexpr int TJ = BM / WM / 16;         // m-subtiles per wave
  static_assert(!GEGLU || (TI % 2 == 0), "geglu pairs");
  constexpr int AR = BM / 32;              // A DMA rounds (32 rows each, 8 per wave)
  constexpr int WR = (BN + 31) / 32;       // W DMA rounds

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;

  const int nN = GEGLU ? (p.N + BN / 2 - 1) / (BN / 2) : (p.N + BN - 1) / BN;
  const int nM = (p.M + BM - 1) / BM;
  const int lin = xcd_remap(blockIdx.x, nN * nM);
  const int tn = lin % nN, tm = lin / nN;
  const int batch = blockIdx.z;
  const int m0 = tm * BM;
  const int n0 = GEGLU ? tn * (BN / 2) : tn * BN;   // output-column origin

  const uint16_t* __restrict__ A = p.A + (long long)batch * p.sA;
  const uint16_t* __restrict__ W = p.W + (long long)batch * p.sW;
  const int ldw = p.ldw ? p.ldw : p.K;
  const void* zp = (const void*)g_zero_page;

  // ---- this lane's DMA rows: round i covers rows 32i + 8*wave + (lane>>3), slot lane&7
  const int slot = lane & 7;
  const int rsub = 8 * wave + (lane >> 3);
  int a_row[AR], a_chunk[AR];
  int cb_[AR], cy_[AR], cx_[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int r = 32 * i + rsub;
    a_row[i] = m0 + r;
    a_chunk[i] = slot ^ ((r >> 1) & 7);
    if constexpr (CONV != 0) {
      const int m = a_row[i] < p.M ? a_row[i] : 0;
      const int hw = p.Ho * p.Wo;
      const int b = m / hw;
      const int rr = m - b * hw;
      const int oy = rr / p.Wo;
      const int ox = rr - oy * p.Wo;
      cb_[i] = b;
      cy_[i] = oy * p.stride - p.pad;
      cx_[i] = ox * p.stride - p.pad;
    }
  }
  int w_row[WR], w_chunk[WR];
#pragma unroll
  for (int i = 0; i < WR; ++i) {
    const int r = 32 * i + rsub;
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
  const int Hv = p.upsample ? 2 * p.IH : p.IH;
  const int Wv = p.upsample ? 2 * p.IW : p.IW;

  auto stage = [&](int kt, int buf) {
    const int k0 = kt * BK;
    uint4* As = smem + buf * TILE;
    uint4* Ws = As + BM * 8;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int k = k0 + a_chunk[i] * 8;
      const void* src = zp;
      if constexpr (CONV == 0) {
        if (a_row[i] < p.M && k < p.K) src = A + (long long)a_row[i] * p.lda + k;
      } else {
        if (a_row[i] < p.M && k < p.K) {
          int tap, ci;
          if constexpr (CONV == 2) {   // Cin % 64 == 0: one tap per k-tile (uniform)
            tap = k0 / p.Cin;
            ci = k - tap * p.Cin;
          } else {
            tap = k / p.Cin;
            ci = k - tap * p.Cin;
          }
          const int ky = tap / p.ksize;
          const int kx = tap - ky * p.ksize;
          int iy = cy_[i] + ky, ix = cx_[i] + kx;
          if (iy >= 0 && iy < Hv && ix >= 0 && ix < Wv) {
            if (p.upsample) { iy >>= 1; ix >>= 1; }
            src = A + (((long long)cb_[i] * p.IH + iy) * p.IW + ix) * p.Cin + ci;
          }
        }
      }
      glds16(src, As + (32 * i + 8 * wave) * 8);
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      if (32 * i + 8 * wave < BN) {          // wave-uniform
        const int k = k0 + w_chunk[i] * 8;
        const void* src = (w_row[i] >= 0 && k < p.K) ? (const void*)(W + (long long)w_row[i] * ldw + k) : zp;
        glds16(src, Ws + (32 * i + 8 * wave) * 8);
      }
    }
  };

  f32x4_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  stage(0, 0);
  __syncthreads();   // drains the DMA (vmcnt(0)) and publishes the tile

  const int fr = lane & 15;      // fragment row within 16
  const int fq = lane >> 4;      // k-chunk within a 32-k step
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const uint4* As = smem + cur * TILE;
    const uint4* Ws = As + BM * 8;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fq;
      bf16x8_t wf[TI], af[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wn * (BN / WN) + 16 * i + fr;
        wf[i] = as_bf16x8(Ws[r * 8 + swz(r, ch)]);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = wm * (BM / WM) + 16 * j + fr;
        af[j] = as_bf16x8(As[r * 8 + swz(r, ch)]);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();   // next tile landed (vmcnt(0)) and everyone is done with this one
  }

  // ---- epilogue
  const int hw = p.Ho * p.Wo;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int m = m0 + wm * (BM / WM) + 16 * j + fr;
    if (m >= p.M) continue;
    const int bimg = (p.chan_bias != nullptr) ? (m / hw) : 0;
    if constexpr (GEGLU) {
#pragma unroll
      for (int pi = 0; pi < TI / 2; ++pi) {
        const int n = n0 + wn * (BN / WN / 2) + 16 * pi + 4 * fq;
        if (n >= p.N) continue;
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float h = acc[2 * pi][j][r], g = acc[2 * pi + 1][j][r];
          if (p.bias) { h += bf2f(p.bias[n + r]); g += bf2f(p.bias[p.N + n + r]); }
          o[r] = h * gelu_f(g);
        }
        uint16_t* C = reinterpret_cast<uint16_t*>(p.C) + (long long)batch * p.sC + (long long)m * p.ldc + n;
        if (p.residual) {
          uint2 rv = *reinterpret_cast<const uint2*>(p.residual + (long long)m * p.ldc + n);
          o[0] += bf2f(rv.x & 0xffff); o[1] += bf2f(rv.x >> 16); o[2] += bf2f(rv.y & 0xffff); o[3] += bf2f(rv.y >> 16);
        }
        *reinterpret_cast<uint2*>(C) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    } else {
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int n = n0 + wn * (BN / WN) + 16 * i + 4 * fq;
        if (n >= p.N) continue;
        const bool full = (n + 4 <= p.N) && (p.N % 4 == 0) && (p.ldc % 4 == 0);
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = acc[i][j][r] * p.alpha;
        if (full) {
          if (p.bias) {
            uint2 bv = *reinterpret_cast<const uint2*>(p.bias + n);
            o[0] += bf2f(bv.x & 0xffff); o[1] += bf2f(bv.x >> 16); o[2] += bf2f(bv.y & 0xffff); o[3] += bf2f(bv.y >> 16);
          }
          if (p.chan_bias) {
            uint2 bv = *reinterpret_cast<const uint2*>(p.chan_bias + (long long)bimg * p.N + n);
            o[0] += bf2f(bv.x & 0xffff); o[1] += bf2f(bv.x >> 16); o[2] += bf2f(bv.y & 0xffff); o[3] += bf2f(bv.y >> 16);
          }
          if (p.act != ACT_NONE) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = apply_act(o[r], p.act);
          }
          if (p.residual) {
            uint2 rv = *reinterpret_cast<const uint2*>(p.residual + (long long)m * p.ldc + n);
            o[0] += bf2f(rv.x & 0xffff); o[1] += bf2f(rv.x >> 16); o[2] += bf2f(rv.y & 0xffff); o[3] += bf2f(rv.y >> 16);
          }
          if constexpr (OUTF32) {
            float* C = reinterpret_cast<float*>(p.C) + (long long)batch * p.sC + (long long)m * p.ldc + n;
            *reinterpret_cast<float4*>(C) = make_float4(o[0], o[1], o[2], o[3]);
          } else {
            uint16_t* C = reinterpret_cast<uint16_t*>(p.C) + (long long)batch * p.sC + (long long)m * p.ldc + n;
            *reinterpret_cast<uint2*>(C) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
          }
        } else {   // ragged N (3-channel conv_out): element-wise tail
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (n + r >= p.N) break;
            float v = o[r];
            if (p.bias) v += bf2f(p.bias[n + r]);
            if (p.chan_bias) v += bf2f(p.chan_bias[(long long)bimg * p.N + n + r]);
            v = apply_act(v, p.act);
            if (p.residual) v += bf2f(p.residual[(long long)m * p.ldc + n + r]);
            if constexpr (OUTF32)
              reinterpret_cast<float*>(p.C)[(long long)batch * p.sC + (long long)m * p.ldc + n + r] = v;
            else
              reinterpret_cast<uint16_t*>(p.C)[(long long)batch * p.sC + (long long)m * p.ldc + n + r] = f2bf(v);
          }
        }
      }
    }
  }
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
  if (p.chan_bias) o += bf2f(p.chan_bias[(long long)(m / (p.Ho * p.Wo)) * p.N + n]);
  o = apply_act(o, p.act);
  if (p.residual) o += bf2f(p.residual[(long long)m * p.ldc + n]);
  if (p.out_f32)
    reinterpret_cast<float*>(p.C)[(long long)batch * p.sC + (long long)m * p.ldc + n] = o;
  else
    reinterpret_cast<uint16_t*>(p.C)[(long long)batch * p.sC + (long long)m * p.ldc + n] = f2bf(o);
}

template <int BM, int BN, int WM, int WN, int CONV, bool GEGLU, bool OUTF32>
void launch_t(const GemmArgs& p, hipStream_t s) {
  const int nN = GEGLU ? (p.N + BN / 2 - 1) / (BN / 2) : (p.N + BN - 1) / BN;
  const int nM = (p.M + BM - 1) / BM;
  dim3 grid(nN * nM, 1, p.batch);
  constexpr size_t lds = 2 * (size_t)(BM + BN) * BK * 2;
  if constexpr (lds > 65536) {
    // > 64 KiB dynamic LDS must be opted into once (first call happens before any graph capture)
    static const bool once = [] {
      (void)hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, WM, WN, CONV, GEGLU, OUTF32>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      return true;
    }();
    (void)once;
  }
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, CONV, GEGLU, OUTF32>), grid, dim3(THREADS), lds, s, p);
}

template <int CONV, bool OUTF32>
void launch_shape(const GemmArgs& p, hipStream_t s) {
  if (p.N <= 16) launch_t<256, 16, 4, 1, CONV, false, OUTF32>(p, s);
  else if (p.N % 128 != 0 && p.N % 64 == 0) launch_t<256, 64, 4, 1, CONV, false, OUTF32>(p, s);
  else launch_t<128, 128, 2, 2, CONV, false, OUTF32>(p, s);
}

template <int CONV>
void launch_tiles(const GemmArgs& p, hipStream_t s) {
  if (p.act == ACT_GEGLU) launch_t<128, 128, 2, 2, CONV, true, false>(p, s);
  else if (p.out_f32) launch_shape<CONV, true>(p, s);
  else launch_shape<CONV, false>(p, s);
}

}  // namespace

void launch_gemm(const GemmArgs& p, hipStream_t s) {
  const bool mfma_ok = (p.K % 8 == 0) && (!p.conv || p.Cin % 8 == 0) &&
                       (p.conv || p.lda % 8 == 0) && (p.ldw % 8 == 0);
  if (!mfma_ok) {
    if (p.act == ACT_GEGLU) return;  // host side guarantees geglu shapes are MFMA-able
    long long total = (long long)p.M * p.N;
    dim3 grid((unsigned)((total + 255) / 256), 1, p.batch);
    if (p.conv)
      hipLaunchKernelGGL(gemm_simt_kernel<1>, grid, dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL(gemm_simt_kernel<0>, grid, dim3(256), 0, s, p);
    return;
  }
  if (!p.conv) launch_tiles<0>(p, s);
  else if (p.Cin % 64 == 0) launch_tiles<2>(p, s);
  else launch_tiles<1>(p, s);
}
