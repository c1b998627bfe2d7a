// MFMA bf16 GEMM / implicit-GEMM convolution with fused epilogues.
//
//   D[n][m] = sum_k W[n][k] * A[m][k]          (computed transposed so each lane owns 4
//   C[m][n] = act(alpha*D + bias[n] + cb[b][n])  consecutive output channels of one row ->
//             (+ residual[m][n])                 8-byte NHWC stores)
//
// * A is either a row-major activation matrix (linear layers, 1x1 convs) or an NHWC image read
//   through an implicit im2col (3x3 convs, stride 2 downsamplers, nearest-2x upsample fused
//   into the address generation: the upsampled tensor never exists).
// * W rows are K-contiguous ([Cout][kh][kw][Cin] for convs), so both operands are read from
//   LDS as 16-byte k-chunks: mfma_f32_16x16x32_bf16 fragments straight from ds_read_b128.
// * Tiles: BM x BN x 64, 256 threads = 4 waves (2 x 2), each wave 64 x 64 = 4 x 4 MFMA tiles.
//   Global->LDS by register staging with the next k-tile's loads issued before the current
//   tile's MFMAs (issue early / write late, cdna_hip_programming.md T14).
// * LDS rows are 128 B; 16-B chunk c of row r is stored at chunk c ^ ((r >> 1) & 7), which
//   makes the 16 rows read by each ds_read_b128 lane group hit 16 distinct bank slots.
// * GEGLU (transformer FF): W tile rows interleave 16-row value/gate blocks, so each lane
//   holds h and g of the same output column and computes h * gelu(g) in registers.
// * Block ids are remapped XCD-aware so tiles that share an A panel run on one XCD's L2.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int BK = 64;
constexpr int THREADS = 256;

CM_DEVICE int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int BM, int BN, int CONV, bool GEGLU, bool OUTF32>
__global__ void __launch_bounds__(THREADS, 2) gemm_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  uint4* As = smem;                    // [BM][8] 16-B chunks
  uint4* Ws = smem + BM * 8;           // [BN][8]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  const int nN = (GEGLU ? (p.N + BN / 2 - 1) / (BN / 2) : (p.N + BN - 1) / BN);
  const int nM = (p.M + BM - 1) / BM;
  const int tiles = nN * nM;
  const int lin = xcd_remap(blockIdx.x, tiles);
  const int tn = lin % nN, tm = lin / nN;
  const int batch = blockIdx.z;
  const int m0 = tm * BM;
  const int n0 = GEGLU ? tn * (BN / 2) : tn * BN;   // output-column origin

  const uint16_t* __restrict__ A = p.A + (long long)batch * p.sA;
  const uint16_t* __restrict__ W = p.W + (long long)batch * p.sW;
  const int ldw = p.ldw ? p.ldw : p.K;

  // ---- per-thread load assignment: chunk c, rows r0 + 32*i
  constexpr int AR = BM / 32, WR = BN / 32;
  const int lc = tid & 7;
  const int lr = tid >> 3;

  // conv row decode (output pixel -> batch, input origin)
  int cb_[AR], cy_[AR], cx_[AR];
  bool cv_[AR];
  if constexpr (CONV != 0) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      int m = m0 + lr + 32 * i;
      cv_[i] = m < p.M;
      int mm = cv_[i] ? m : 0;
      int hw = p.Ho * p.Wo;
      int b = mm / hw;
      int r = mm - b * hw;
      int oy = r / p.Wo;
      int ox = r - oy * p.Wo;
      cb_[i] = b;
      cy_[i] = oy * p.stride - p.pad;
      cx_[i] = ox * p.stride - p.pad;
    }
  }
  // W row mapping
  int wrow_[WR];
#pragma unroll
  for (int i = 0; i < WR; ++i) {
    int r = lr + 32 * i;
    int gr;
    if constexpr (GEGLU) {
      int blk = r >> 4, within = r & 15;
      int nout = n0 + (blk >> 1) * 16 + within;
      gr = (nout < p.N) ? ((blk & 1) ? p.N + nout : nout) : -1;
    } else {
      int n = n0 + r;
      gr = n < p.Nw ? n : -1;
    }
    wrow_[i] = gr;
  }

  const int Hv = p.upsample ? 2 * p.IH : p.IH;
  const int Wv = p.upsample ? 2 * p.IW : p.IW;

  auto load_a = [&](int k0, uint4* ra) {
    const int k = k0 + lc * 8;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if constexpr (CONV == 0) {
        int m = m0 + lr + 32 * i;
        if (m < p.M && k < p.K) v = *reinterpret_cast<const uint4*>(A + (long long)m * p.lda + k);
      } else {
        if (cv_[i] && k < p.K) {
          int tap, ci;
          if constexpr (CONV == 2) {   // Cin % 64 == 0: one tap per k-tile
            tap = k0 / p.Cin;
            ci = k - tap * p.Cin;
          } else {
            tap = k / p.Cin;
            ci = k - tap * p.Cin;
          }
          int ky = tap / p.ksize;
          int kx = tap - ky * p.ksize;
          int iy = cy_[i] + ky, ix = cx_[i] + kx;
          if (iy >= 0 && iy < Hv && ix >= 0 && ix < Wv) {
            if (p.upsample) { iy >>= 1; ix >>= 1; }
            v = *reinterpret_cast<const uint4*>(A + (((long long)cb_[i] * p.IH + iy) * p.IW + ix) * p.Cin + ci);
          }
        }
      }
      ra[i] = v;
    }
  };
  auto load_w = [&](int k0, uint4* rw) {
    const int k = k0 + lc * 8;
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (wrow_[i] >= 0 && k < p.K) v = *reinterpret_cast<const uint4*>(W + (long long)wrow_[i] * ldw + k);
      rw[i] = v;
    }
  };
  auto store_tiles = [&](const uint4* ra, const uint4* rw) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      int r = lr + 32 * i;
      As[r * 8 + swz(r, lc)] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      int r = lr + 32 * i;
      Ws[r * 8 + swz(r, lc)] = rw[i];
    }
  };

  constexpr int TI = BN / 2 / 16;   // n-subtiles per wave
  constexpr int TJ = BM / 2 / 16;   // m-subtiles per wave
  f32x4_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 ra[AR], rw[WR];
  const int nk = (p.K + BK - 1) / BK;
  load_a(0, ra);
  load_w(0, rw);
  store_tiles(ra, rw);
  __syncthreads();

  const int fr = lane & 15;      // fragment row within 16
  const int fq = lane >> 4;      // k-chunk within a 32-k step
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      load_a((kt + 1) * BK, ra);
      load_w((kt + 1) * BK, rw);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fq;
      bf16x8_t wf[TI], af[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        int r = wn * (BN / 2) + 16 * i + fr;
        wf[i] = as_bf16x8(Ws[r * 8 + swz(r, ch)]);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        int r = wm * (BM / 2) + 16 * j + fr;
        af[j] = as_bf16x8(As[r * 8 + swz(r, ch)]);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (more) {
      store_tiles(ra, rw);
      __syncthreads();
    }
  }

  // ---- epilogue
  const int hw = p.Ho * p.Wo;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int m = m0 + wm * (BM / 2) + 16 * j + fr;
    if (m >= p.M) continue;
    const int bimg = (p.chan_bias != nullptr) ? (m / hw) : 0;
    if constexpr (GEGLU) {
#pragma unroll
      for (int pi = 0; pi < TI / 2; ++pi) {
        const int n = n0 + wn * (BN / 4) + 16 * pi + 4 * fq;
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
        const int n = n0 + wn * (BN / 2) + 16 * i + 4 * fq;
        if (n >= p.N) continue;
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = acc[i][j][r] * p.alpha;
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
      }
    }
  }
}

// SIMT fallback for shapes the MFMA path does not take (N % 4 != 0, K % 8 != 0: conv_in with 4
// latent channels, VAE conv_out with 3 RGB channels).  One thread per output element.
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

template <int BM, int BN, int CONV, bool GEGLU, bool OUTF32>
void launch_t(const GemmArgs& p, hipStream_t s) {
  int nN = GEGLU ? (p.N + BN / 2 - 1) / (BN / 2) : (p.N + BN - 1) / BN;
  int nM = (p.M + BM - 1) / BM;
  dim3 grid(nN * nM, 1, p.batch);
  size_t lds = (size_t)(BM + BN) * BK * 2;
  hipLaunchKernelGGL((gemm_kernel<BM, BN, CONV, GEGLU, OUTF32>), grid, dim3(THREADS), lds, s, p);
}

template <int CONV>
void launch_tiles(const GemmArgs& p, hipStream_t s) {
  const bool geglu = p.act == ACT_GEGLU;
  if (geglu) {
    launch_t<128, 128, CONV, true, false>(p, s);
  } else if (p.out_f32) {
    launch_t<128, 128, CONV, false, true>(p, s);
  } else {
    launch_t<128, 128, CONV, false, false>(p, s);
  }
}

}  // namespace

void launch_gemm(const GemmArgs& p, hipStream_t s) {
  const bool mfma_ok = (p.K % 8 == 0) && (p.N % 4 == 0) && (p.ldc % 4 == 0) &&
                       (!p.conv || p.Cin % 8 == 0) && (p.conv || p.lda % 8 == 0) &&
                       (p.ldw % 8 == 0);
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
