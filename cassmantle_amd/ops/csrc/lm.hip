// Decode-path kernels (gfx950): skinny-M GEMV, RoPE + KV-cache write, split-KV decode attention.
//
// These serve the optional local causal LM prompt generator (models/lm.py; it replaces the
// reference's remote Mistral-7B call, src/backend.py:240-268) and every other GEMM whose M is a
// handful of rows (UNet time-embedding projections, pooled text projections):
//
// * gemv_kernel: M <= 8 rows.  A GEMM tile would run 1/16..1/128 of its MFMA lanes and stage W
//   through LDS for nothing; decode is a pure weight stream (7B bf16 = 14.5 GB per token, the
//   HBM3E bound is ~1.8 ms/token), so each block streams R weight rows with 16-byte loads (a
//   wave covers 1 KiB of a row per instruction), the 4 waves split K, and partial sums are
//   combined with a halving "transpose" butterfly (V values over 64 lanes in ~2V shuffles instead
//   of 6V) then across waves through LDS.  Gated activations (GEGLU / SwiGLU) read the value row
//   n and gate row N+n in the same pass.
// * rope_kv_kernel: fused QKV projection output -> rotary-embedded Q, rotary K and V appended to
//   the KV cache at each sequence's device-side position (graph-capturable: no host positions).
// * decode_attn_kernel: one query token per sequence against the cache, GQA (a block serves the
//   G query heads of one KV head so K/V rows are read once), split over the key axis so a batch-1
//   decode still fills the chip, exp2-domain online softmax, then decode_combine_kernel.
#include "common.h"
#include "kernels.h"

namespace {

// ------------------------------------------------------------------------------------ GEMV
// Halving butterfly over the wave: V partial sums per lane -> lane l ends with the full sum of
// value index idx(l) (V <= 64, power of two).  Lanes differing only in the low log2(64/V) bits
// hold the same index.
template <int V>
CM_DEVICE float transpose_reduce(float (&v)[V], int lane, int& idx) {
  idx = 0;
  int c = V;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    if (c > 1) {
      const bool up = (lane & o) != 0;
#pragma unroll
      for (int i = 0; i < V / 2; ++i) {
        if (i < c / 2) {
          const float send = up ? v[i] : v[i + c / 2];
          const float keep = up ? v[i + c / 2] : v[i];
          v[i] = keep + __shfl_xor(send, o);
        }
      }
      if (up) idx += c / 2;
      c /= 2;
    } else {
      v[0] += __shfl_xor(v[0], o);
    }
  }
  return v[0];
}

// output columns per block: 4, or 2 for gated M=8 (keeps the 64 partial sums + operands in VGPRs)
template <int MM, bool GATED> constexpr int gemv_r() { return (GATED && MM >= 8) ? 2 : 4; }
constexpr int GEMV_THREADS = 256;

template <int MM, bool GATED>
__global__ __launch_bounds__(GEMV_THREADS) void gemv_kernel(GemmArgs p) {
  constexpr int GEMV_R = gemv_r<MM, GATED>();
  constexpr int NR = GATED ? 2 * GEMV_R : GEMV_R;   // weight rows streamed by this block
  constexpr int V = NR * MM;                          // partial sums per lane
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * GEMV_R;
  const int batch = blockIdx.z;
  const uint16_t* A = p.A + (long long)batch * p.sA;
  const uint16_t* W = p.W + (long long)batch * p.sW;
  const long long ldw = p.ldw ? p.ldw : p.K;

  const uint16_t* wr[NR];
#pragma unroll
  for (int r = 0; r < GEMV_R; ++r) {
    const int n = n0 + r < p.N ? n0 + r : p.N - 1;   // clamp (result discarded)
    wr[r] = W + (long long)n * ldw;
    if constexpr (GATED) wr[GEMV_R + r] = W + (long long)(p.N + n) * ldw;
  }
  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.f;

  for (int k = (wave * 64 + lane) * 8; k < p.K; k += GEMV_THREADS * 8) {
    uint4 wv[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) wv[r] = *reinterpret_cast<const uint4*>(wr[r] + k);
    float wf[NR][8];
#pragma unroll
    for (int r = 0; r < NR; ++r) unpack8(wv[r], wf[r]);
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      if (m < p.M) {
        float af[8];
        unpack8(*reinterpret_cast<const uint4*>(A + (long long)m * p.lda + k), af);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          float s = acc[r * MM + m];
#pragma unroll
          for (int e = 0; e < 8; ++e) s = fmaf(af[e], wf[r][e], s);
          acc[r * MM + m] = s;
        }
      }
    }
  }

  int idx;
  const float tot = transpose_reduce<V>(acc, lane, idx);
  __shared__ float red[GEMV_THREADS / 64][V];
  if ((lane & (64 / V - 1)) == 0) red[wave][idx] = tot;
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= GEMV_R * MM) return;
  const int r = t / MM, m = t - r * MM;
  const int n = n0 + r;
  if (n >= p.N || m >= p.M) return;
  float o = 0.f;
#pragma unroll
  for (int w = 0; w < GEMV_THREADS / 64; ++w) o += red[w][t];
  o *= p.alpha;
  if constexpr (GATED) {
    float g = 0.f;
#pragma unroll
    for (int w = 0; w < GEMV_THREADS / 64; ++w) g += red[w][GEMV_R * MM + t];
    g *= p.alpha;
    if (p.bias) { o += bf2f(p.bias[n]); g += bf2f(p.bias[p.N + n]); }
    o = gate_f(o, g, p.act);
  } else {
    if (p.bias) o += bf2f(p.bias[n]);
    o = apply_act(o, p.act);
  }
  if (p.residual) o += bf2f(p.residual[(long long)m * p.ldc + n]);
  const long long off = (long long)batch * p.sC + (long long)m * p.ldc + n;
  if (p.out_f32) reinterpret_cast<float*>(p.C)[off] = o;
  else reinterpret_cast<uint16_t*>(p.C)[off] = f2bf(o);
}

template <int MM>
void gemv_launch(const GemmArgs& p, hipStream_t s) {
  if (is_gated(p.act)) {
    constexpr int R = gemv_r<MM, true>();
    hipLaunchKernelGGL((gemv_kernel<MM, true>), dim3((p.N + R - 1) / R, 1, p.batch), dim3(GEMV_THREADS), 0, s, p);
  } else {
    constexpr int R = gemv_r<MM, false>();
    hipLaunchKernelGGL((gemv_kernel<MM, false>), dim3((p.N + R - 1) / R, 1, p.batch), dim3(GEMV_THREADS), 0, s, p);
  }
}

// ------------------------------------------------------------------------------------ RoPE
// qkv [B*T][ld] rows = [q heads | k heads | v heads] x d.  Rotate-half RoPE (pairs i, i+d/2).
__global__ void rope_kv_kernel(RopeArgs a) {
  const int half = a.d / 2;
  const int slots = a.H + 2 * a.Hk;
  const long long total = (long long)a.B * a.T * slots * half;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int e = (int)(i % half);
  long long r = i / half;
  const int slot = (int)(r % slots);
  r /= slots;
  const int t = (int)(r % a.T);
  const int b = (int)(r / a.T);
  const int pos = (a.pos0 ? a.pos0[b] : 0) + t;
  const uint16_t* src = a.qkv + ((long long)b * a.T + t) * a.ld + (long long)slot * a.d;
  float x0 = bf2f(src[e]), x1 = bf2f(src[e + half]);
  if (slot < a.H + a.Hk) {
    // inv_freq = theta^(-2e/d); fp32 angle is exact enough for the LM's context lengths
    const float inv = exp2f(-(2.0f * e / a.d) * a.log2_theta);
    float sn, cs;
    sincosf((float)pos * inv, &sn, &cs);
    const float y0 = x0 * cs - x1 * sn, y1 = x1 * cs + x0 * sn;
    x0 = y0; x1 = y1;
  }
  uint16_t* dst;
  if (slot < a.H) {
    dst = a.q_out + (((long long)b * a.T + t) * a.H + slot) * a.d;
  } else {
    if (pos >= a.L) return;   // cache full: the host never schedules past capacity
    const int hk = slot < a.H + a.Hk ? slot - a.H : slot - a.H - a.Hk;
    uint16_t* cache = slot < a.H + a.Hk ? a.k_cache : a.v_cache;
    dst = cache + (((long long)b * a.L + pos) * a.Hk + hk) * a.d;
  }
  dst[e] = f2bf(x0);
  dst[e + half] = f2bf(x1);
}

// --------------------------------------------------------------------------- decode attention
constexpr int DEC_THREADS = 256;
constexpr int DEC_MAXG = 8;

template <int D>
__global__ __launch_bounds__(DEC_THREADS) void decode_attn_kernel(DecodeArgs a) {
  constexpr int DL = D / 64;        // head-dim elements per lane
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x / a.Hk, hk = blockIdx.x - b * a.Hk;
  const int G = a.H / a.Hk;
  const int len = a.lens[b];
  const int chunk = (a.L + gridDim.y - 1) / gridDim.y;
  const int k0 = blockIdx.y * chunk;
  const int k1 = min(len, k0 + chunk);

  float q[DEC_MAXG][DL];
  float m_run[DEC_MAXG], l_run[DEC_MAXG], acc[DEC_MAXG][DL];
  const float qs = a.scale * 1.4426950408889634f;   // exp2 domain
#pragma unroll
  for (int g = 0; g < DEC_MAXG; ++g) {
    m_run[g] = -INFINITY; l_run[g] = 0.f;
#pragma unroll
    for (int e = 0; e < DL; ++e) {
      acc[g][e] = 0.f;
      q[g][e] = g < G ? bf2f(a.q[(long long)b * a.q_sb + (long long)(hk * G + g) * a.d + lane * DL + e]) * qs : 0.f;
    }
  }
  for (int key = k0 + wave; key < k1; key += DEC_THREADS / 64) {
    const long long base = (((long long)b * a.L + key) * a.Hk + hk) * a.d + lane * DL;
    float kf[DL], vf[DL];
#pragma unroll
    for (int e = 0; e < DL; ++e) { kf[e] = bf2f(a.k_cache[base + e]); vf[e] = bf2f(a.v_cache[base + e]); }
#pragma unroll
    for (int g = 0; g < DEC_MAXG; ++g) {
      if (g < G) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < DL; ++e) s = fmaf(q[g][e], kf[e], s);
        s = wave_sum(s);
        const float mn = fmaxf(m_run[g], s);
        const float corr = exp2f(m_run[g] - mn);
        const float pr = exp2f(s - mn);
        l_run[g] = l_run[g] * corr + pr;
#pragma unroll
        for (int e = 0; e < DL; ++e) acc[g][e] = fmaf(acc[g][e], corr, pr * vf[e]);
        m_run[g] = mn;
      }
    }
  }
  // merge the 4 waves
  __shared__ float sm[DEC_THREADS / 64][DEC_MAXG], sl[DEC_THREADS / 64][DEC_MAXG];
  __shared__ float sacc[DEC_THREADS / 64][DEC_MAXG][D];
#pragma unroll
  for (int g = 0; g < DEC_MAXG; ++g) {
    if (g < G) {
      if (lane == 0) { sm[wave][g] = m_run[g]; sl[wave][g] = l_run[g]; }
#pragma unroll
      for (int e = 0; e < DL; ++e) sacc[wave][g][lane * DL + e] = acc[g][e];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += DEC_THREADS) {
    const int g = i / D, e = i - g * D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < DEC_THREADS / 64; ++w) M = fmaxf(M, sm[w][g]);
    float l = 0.f, o = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < DEC_THREADS / 64; ++w) {
        const float c = exp2f(sm[w][g] - M);
        l += sl[w][g] * c;
        o += sacc[w][g][e] * c;
      }
    }
    const int h = hk * G + g;
    if (gridDim.y == 1) {
      a.o[(long long)b * a.o_sb + (long long)h * a.d + e] = f2bf(l > 0.f ? o / l : 0.f);
    } else {
      const long long slot = ((long long)(b * a.H + h) * gridDim.y + blockIdx.y);
      a.ws[slot * (D + 2) + e] = o;
      if (e == 0) { a.ws[slot * (D + 2) + D] = M; a.ws[slot * (D + 2) + D + 1] = l; }
    }
  }
}

template <int D>
__global__ void decode_combine_kernel(DecodeArgs a, int ns) {
  const int bh = blockIdx.x;                 // b * H + h
  const int b = bh / a.H, h = bh - b * a.H;
  const int e = threadIdx.x;
  if (e >= D) return;
  const float* w = a.ws + (long long)bh * ns * (D + 2);
  float M = -INFINITY;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, w[s * (D + 2) + D]);
  float l = 0.f, o = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < ns; ++s) {
      const float c = exp2f(w[s * (D + 2) + D] - M);
      l += w[s * (D + 2) + D + 1] * c;
      o += w[s * (D + 2) + e] * c;
    }
  }
  a.o[(long long)b * a.o_sb + (long long)h * a.d + e] = f2bf(l > 0.f ? o / l : 0.f);
}

}  // namespace

bool launch_gemv(const GemmArgs& p, hipStream_t s) {
  const long long ldw = p.ldw ? p.ldw : p.K;
  if (p.conv || p.M > 8 || p.M < 1 || p.chan_bias != nullptr) return false;
  if (p.K % 8 != 0 || p.lda % 8 != 0 || ldw % 8 != 0) return false;
  if (p.M <= 1) gemv_launch<1>(p, s);
  else if (p.M <= 2) gemv_launch<2>(p, s);
  else if (p.M <= 4) gemv_launch<4>(p, s);
  else gemv_launch<8>(p, s);
  return true;
}

void launch_rope_kv(const RopeArgs& a, hipStream_t s) {
  const long long total = (long long)a.B * a.T * (a.H + 2 * a.Hk) * (a.d / 2);
  if (total == 0) return;
  hipLaunchKernelGGL(rope_kv_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
}

int decode_splits(int B, int Hk, int L) {
  // enough blocks to cover the CUs for batch-1 decode, >= 64 keys per split
  int want = (512 + B * Hk - 1) / (B * Hk);
  int maxs = (L + 63) / 64;
  int ns = want < maxs ? want : maxs;
  if (ns > 32) ns = 32;
  return ns < 1 ? 1 : ns;
}

void launch_decode_attention(const DecodeArgs& a, int ns, hipStream_t s) {
  dim3 grid(a.B * a.Hk, ns);
  if (a.d == 64) {
    hipLaunchKernelGGL(decode_attn_kernel<64>, grid, dim3(DEC_THREADS), 0, s, a);
    if (ns > 1) hipLaunchKernelGGL(decode_combine_kernel<64>, dim3(a.B * a.H), dim3(64), 0, s, a, ns);
  } else {
    hipLaunchKernelGGL(decode_attn_kernel<128>, grid, dim3(DEC_THREADS), 0, s, a);
    if (ns > 1) hipLaunchKernelGGL(decode_combine_kernel<128>, dim3(a.B * a.H), dim3(128), 0, s, a, ns);
  }
}
