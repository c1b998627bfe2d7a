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
// * lm_sample_kernel: the decode step's sampler in ONE launch (was ATen topk + gather + argmax +
//   index_copy inside the captured graph): logits / T (+ the step's EOS bias), the top-k set by a
//   4-pass 8-bit radix select on order-preserving float keys (ties at the k-th value resolved to
//   the lowest vocabulary ids), Gumbel-max over the set with the step's noise row, and the
//   device-side state update (token, position, cache length, step counter).
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

// one 8-element k-chunk of every row: acc[r*MM+m] += A[m][k..k+7] . W[r][k..k+7]; with
// gamma (fused RMSNorm) also ss[m] += A^2 and A is scaled by gamma first
template <int MM, int NR>
CM_DEVICE void gemv_chunk(const uint4 (&wv)[NR], const uint16_t* A, int lda, int M, int k, const uint16_t* gamma,
                          float (&acc)[NR * MM], float (&ss)[MM]) {
  float gf[8];
  if (gamma) unpack8(*reinterpret_cast<const uint4*>(gamma + k), gf);
#pragma unroll
  for (int m = 0; m < MM; ++m) {
    if (m < M) {
      float af[8];
      unpack8(*reinterpret_cast<const uint4*>(A + (long long)m * lda + k), af);
      if (gamma) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { ss[m] = fmaf(af[e], af[e], ss[m]); af[e] *= gf[e]; }
      }
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        float wf[8];
        unpack8(wv[r], wf);
        float s = acc[r * MM + m];
#pragma unroll
        for (int e = 0; e < 8; ++e) s = fmaf(af[e], wf[e], s);
        acc[r * MM + m] = s;
      }
    }
  }
}

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
  // fused RMSNorm prologue (p.rms_gamma): the block covers all of K for its rows, so it owns the
  // row statistics: sum(x^2) accumulates from the same A loads, gamma scales A in registers and
  // 1/rms is applied to the finished dot products (no normalised copy of x in HBM)
  const bool rms = p.rms_gamma != nullptr;
  float ss[MM];
#pragma unroll
  for (int m = 0; m < MM; ++m) ss[m] = 0.f;

  // two k-chunks per iteration: all 2*NR weight loads are issued before any FMA (the kernel is a
  // pure HBM stream, no LDS staging)
  constexpr int STEP = GEMV_THREADS * 8;
  int k = (wave * 64 + lane) * 8;
  for (; NR * MM <= 8 && k + STEP < p.K; k += 2 * STEP) {   // (wide blocks: keep occupancy)
    uint4 w0[NR], w1[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) w0[r] = *reinterpret_cast<const uint4*>(wr[r] + k);
#pragma unroll
    for (int r = 0; r < NR; ++r) w1[r] = *reinterpret_cast<const uint4*>(wr[r] + k + STEP);
    gemv_chunk<MM, NR>(w0, A, p.lda, p.M, k, p.rms_gamma, acc, ss);
    gemv_chunk<MM, NR>(w1, A, p.lda, p.M, k + STEP, p.rms_gamma, acc, ss);
  }
  for (; k < p.K; k += STEP) {
    uint4 w0[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) w0[r] = *reinterpret_cast<const uint4*>(wr[r] + k);
    gemv_chunk<MM, NR>(w0, A, p.lda, p.M, k, p.rms_gamma, acc, ss);
  }

  int idx;
  const float tot = transpose_reduce<V>(acc, lane, idx);
  __shared__ float red[GEMV_THREADS / 64][V];
  __shared__ float red_ss[GEMV_THREADS / 64][MM];
  if ((lane & (64 / V - 1)) == 0) red[wave][idx] = tot;
  if (rms) {
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      const float v = wave_sum(ss[m]);
      if (lane == 0) red_ss[wave][m] = v;
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= GEMV_R * MM) return;
  const int r = t / MM, m = t - r * MM;
  const int n = n0 + r;
  if (n >= p.N || m >= p.M) return;
  float scale = p.alpha;
  if (rms) {
    float s2 = 0.f;
#pragma unroll
    for (int w = 0; w < GEMV_THREADS / 64; ++w) s2 += red_ss[w][m];
    scale *= rsqrtf(s2 / p.K + p.rms_eps);
  }
  float o = 0.f;
#pragma unroll
  for (int w = 0; w < GEMV_THREADS / 64; ++w) o += red[w][t];
  o *= scale;
  if constexpr (GATED) {
    float g = 0.f;
#pragma unroll
    for (int w = 0; w < GEMV_THREADS / 64; ++w) g += red[w][GEMV_R * MM + t];
    g *= scale;
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
constexpr int DEC_THREADS = 128;   // 2 waves: a 64-key V tile per wave staged in LDS
constexpr int DEC_MAXG = 8;

// Merge per-split partials (m, l, acc[D]) of G heads -> normalised bf16 output
template <int D>
__device__ void decode_combine(const DecodeArgs& a, int b, int hk, int G, int ns, int nact) {
  for (int i = threadIdx.x; i < G * D; i += DEC_THREADS) {
    const int g = i / D, e = i - g * D;
    const int h = hk * G + g;
    const float* w = a.ws + (long long)(b * a.H + h) * ns * (D + 2);
    float M = -INFINITY;
#pragma unroll 4
    for (int s = 0; s < nact; ++s) M = fmaxf(M, __builtin_nontemporal_load(w + s * (D + 2) + D));
    float l = 0.f, o = 0.f;
    if (M != -INFINITY) {
#pragma unroll 4
      for (int s = 0; s < nact; ++s) {
        const float c = exp2f(__builtin_nontemporal_load(w + s * (D + 2) + D) - M);
        l += __builtin_nontemporal_load(w + s * (D + 2) + D + 1) * c;
        o += __builtin_nontemporal_load(w + s * (D + 2) + e) * c;
      }
    }
    a.o[(long long)b * a.o_sb + (long long)h * a.d + e] = f2bf(l > 0.f ? o / l : 0.f);
  }
}

// grid (B*Hk, ns): block = one KV head of one sequence x one key span (multiple of 128 keys).
// Scores with lane = key (each lane dots its K row with the G queries broadcast from LDS: all of
// a row's 16-byte loads issue at once), one wave max/sum per 64 keys and head, then P.V with
// lane = head-dim element over coalesced V rows.  Split partials are merged by the LAST block of
// each (sequence, kv head) to finish (atomic ticket), so there is no second launch.
template <int D, int G>
__global__ __launch_bounds__(DEC_THREADS) void decode_attn_kernel(DecodeArgs a) {
  constexpr int DL = D / 64;          // head-dim elements per lane in P.V
  constexpr int NW = DEC_THREADS / 64;
  constexpr int NCH = D / 8;          // 16-byte chunks per K/V row
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x / a.Hk, hk = blockIdx.x - b * a.Hk;
  const int ns = gridDim.y;
  const int span = ((a.L + ns - 1) / ns + NW * 64 - 1) / (NW * 64) * (NW * 64);
  const int k0 = blockIdx.y * span;
  const long long row = (long long)a.Hk * a.d;            // elements between consecutive keys
  const uint16_t* Kb = a.k_cache + ((long long)b * a.L * a.Hk + hk) * a.d;
  const uint16_t* Vb = a.v_cache + ((long long)b * a.L * a.Hk + hk) * a.d;

  // Decode is a latency chain: the length and the G query rows are fetched in one round.
  const int len_raw = a.lens[b];
  // the G query rows of this kv head are contiguous: [G*D] bf16, 4 per thread and round
  const int nq4 = G * D / 4;
  const uint16_t* qb = a.q + (long long)b * a.q_sb + (long long)hk * G * a.d;
  const int i0 = threadIdx.x, i1 = threadIdx.x + DEC_THREADS;
  const uint2 qv0 = i0 < nq4 ? *reinterpret_cast<const uint2*>(qb + 4 * i0) : make_uint2(0, 0);
  const uint2 qv1 = i1 < nq4 ? *reinterpret_cast<const uint2*>(qb + 4 * i1) : make_uint2(0, 0);
  const int len = min(len_raw, a.L);
  const int k1 = min(len, k0 + span);
  // only the splits that hold keys take part (short contexts: one block, no merge at all)
  const int nact = min(ns, (len + span - 1) / span);
  if (blockIdx.y >= max(nact, 1)) return;
  if (nact == 0) {
    for (int i = threadIdx.x; i < G * D; i += DEC_THREADS)
      a.o[(long long)b * a.o_sb + (long long)(hk * G + i / D) * a.d + i % D] = 0;
    return;
  }

  __shared__ float qs[G][D];
  __shared__ float ps[NW][G][64];
  __shared__ uint4 vs[NW][64][NCH + 1];   // +16 B row pad: conflict-light stores, free row reads
  const float qscale = a.scale * 1.4426950408889634f;   // exp2 domain
  float* qsf = &qs[0][0];
  if (i0 < nq4) {
    qsf[4 * i0 + 0] = __uint_as_float(qv0.x << 16) * qscale;
    qsf[4 * i0 + 1] = __uint_as_float(qv0.x & 0xffff0000u) * qscale;
    qsf[4 * i0 + 2] = __uint_as_float(qv0.y << 16) * qscale;
    qsf[4 * i0 + 3] = __uint_as_float(qv0.y & 0xffff0000u) * qscale;
  }
  if (i1 < nq4) {
    qsf[4 * i1 + 0] = __uint_as_float(qv1.x << 16) * qscale;
    qsf[4 * i1 + 1] = __uint_as_float(qv1.x & 0xffff0000u) * qscale;
    qsf[4 * i1 + 2] = __uint_as_float(qv1.y << 16) * qscale;
    qsf[4 * i1 + 3] = __uint_as_float(qv1.y & 0xffff0000u) * qscale;
  }
  __syncthreads();

  float m_run[G], l_run[G], acc[G][DL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m_run[g] = -INFINITY; l_run[g] = 0.f;
#pragma unroll
    for (int e = 0; e < DL; ++e) acc[g][e] = 0.f;
  }

  for (int t0 = k0 + wave * 64; t0 < k1; t0 += NW * 64) {
    const bool valid = t0 + lane < k1;
    // this lane's whole K and V rows in flight at once (one memory latency per 64-key tile)
    uint4 kv[NCH], vv[NCH];
    {
      const long long ro = (long long)min(t0 + lane, a.L - 1) * row;
#pragma unroll
      for (int c = 0; c < NCH; ++c) kv[c] = reinterpret_cast<const uint4*>(Kb + ro)[c];
#pragma unroll
      for (int c = 0; c < NCH; ++c) vv[c] = reinterpret_cast<const uint4*>(Vb + ro)[c];
    }
    float sc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) sc[g] = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      float kf[8];
      unpack8(kv[c], kf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        {
#pragma unroll
          for (int e = 0; e < 8; ++e) sc[g] = fmaf(qs[g][c * 8 + e], kf[e], sc[g]);
        }
      }
    }
    // V tile -> LDS (row = key) for the P.V pass over head-dim lanes
#pragma unroll
    for (int c = 0; c < NCH; ++c) vs[wave][lane][c] = vv[c];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      {
        const float s = valid ? sc[g] : -INFINITY;
        const float mn = fmaxf(m_run[g], wave_max(s));    // lane 0 is always a valid key
        const float corr = exp2f(m_run[g] - mn);
        const float p = exp2f(s - mn);
        l_run[g] = l_run[g] * corr + wave_sum(p);
        ps[wave][g][lane] = p;
#pragma unroll
        for (int e = 0; e < DL; ++e) acc[g][e] *= corr;
        m_run[g] = mn;
      }
    }
    __builtin_amdgcn_wave_barrier();
    const int nv = min(64, k1 - t0);
    const int mych = (lane * DL) / 8, myoff = (lane * DL) & 7;   // this lane's d elements
#pragma unroll 8
    for (int j = 0; j < nv; ++j) {
      const uint16_t* rp = reinterpret_cast<const uint16_t*>(&vs[wave][j][mych]) + myoff;
      float vf[DL];
      if constexpr (DL == 2) {
        const uint32_t u = *reinterpret_cast<const uint32_t*>(rp);
        vf[0] = __uint_as_float(u << 16);
        vf[1] = __uint_as_float(u & 0xffff0000u);
      } else {
        vf[0] = bf2f(*rp);
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        {
          const float pj = ps[wave][g][j];
#pragma unroll
          for (int e = 0; e < DL; ++e) acc[g][e] = fmaf(pj, vf[e], acc[g][e]);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  // merge the waves of this block
  __shared__ float sm[NW][G], sl[NW][G];
  __shared__ float sacc[NW][G][D];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    {
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
    for (int w = 0; w < NW; ++w) M = fmaxf(M, sm[w][g]);
    float l = 0.f, o = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float c = exp2f(sm[w][g] - M);
        l += sl[w][g] * c;
        o += sacc[w][g][e] * c;
      }
    }
    const int h = hk * G + g;
    if (nact == 1) {
      a.o[(long long)b * a.o_sb + (long long)h * a.d + e] = f2bf(l > 0.f ? o / l : 0.f);
    } else {
      float* w = a.ws + ((long long)(b * a.H + h) * ns + blockIdx.y) * (D + 2);
      w[e] = o;
      if (e == 0) { w[D] = M; w[D + 1] = l; }
    }
  }
  if (nact == 1) return;
  // last block of this (b, hk) to finish merges the splits and re-arms the ticket
  __shared__ int last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = atomicAdd(a.tickets + blockIdx.x, 1);
    last = (t == nact - 1);
    if (last) a.tickets[blockIdx.x] = 0;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  decode_combine<D>(a, b, hk, G, ns, nact);
}

// ------------------------------------------------------------------------------------ sampler
// Contract (ops/reference.py lm_sample): v = logit / T, v[eos] += eos_bias[step]; the k largest v
// with ties broken by the LOWER id; among them the id maximising v + noise[step][id] (ties: larger
// v, then lower id); out[step] = tok = id; pos, lens, step += 1.  One block, batch 1.
constexpr int SAMPLE_THREADS = 1024;

CM_DEVICE unsigned fkey(float f) {                  // order-preserving float -> uint32
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <bool F32>
__global__ void __launch_bounds__(SAMPLE_THREADS) lm_sample_kernel(const void* __restrict__ logits, int V,
                                                                   const float* __restrict__ noise,
                                                                   const float* __restrict__ eos_bias, int eos,
                                                                   float temp, int k, long long* __restrict__ step_p,
                                                                   long long* __restrict__ out,
                                                                   long long* __restrict__ tok,
                                                                   int* __restrict__ pos, int* __restrict__ lens) {
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_rem, s_eq, s_cut;
  __shared__ float r_sc[SAMPLE_THREADS / 64], r_v[SAMPLE_THREADS / 64];
  __shared__ int r_id[SAMPLE_THREADS / 64];
  const int tid = threadIdx.x;
  const long long step = *step_p;
  const float eb = eos_bias[step];
  auto value = [&](int i) -> float {
    const float l = F32 ? reinterpret_cast<const float*>(logits)[i] : bf2f(reinterpret_cast<const uint16_t*>(logits)[i]);
    float v = l / temp;
    if (i == eos) v += eb;
    return v;
  };
  // ---- radix select of the k-th largest key, 8 bits per pass from the top
  unsigned prefix = 0, mask = 0, rem = (unsigned)min(k, V);
  for (int shift = 24; shift >= 0; shift -= 8) {
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < V; i += SAMPLE_THREADS) {
      const unsigned key = fkey(value(i));
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned above = 0;
      int d = 255;
      for (; d > 0; --d) {                         // digits from the top until rem is reached
        if (above + hist[d] >= rem) break;
        above += hist[d];
      }
      s_prefix = prefix | ((unsigned)d << shift);
      s_rem = rem - above;
      s_eq = hist[d];                              // after the last pass: keys equal to the k-th
    }
    __syncthreads();
    prefix = s_prefix;
    rem = s_rem;
    mask |= 255u << shift;
  }
  // ---- ties at the k-th key: keep the `rem` lowest ids (only when more keys equal it)
  if (tid == 0) s_cut = 0x7fffffff;
  __syncthreads();
  if (s_eq > rem) {
    __shared__ unsigned wcnt[SAMPLE_THREADS / 64];
    unsigned need = rem;
    for (int base = 0; base < V && need > 0; base += SAMPLE_THREADS) {
      const int i = base + tid;
      const bool eq = i < V && fkey(value(i)) == prefix;
      const unsigned long long bal = __ballot(eq);
      const int lane = tid & 63, w = tid >> 6;
      if (lane == 0) wcnt[w] = (unsigned)__popcll(bal);
      __syncthreads();
      unsigned before = 0, total = 0;
      for (int j = 0; j < SAMPLE_THREADS / 64; ++j) {
        if (j < w) before += wcnt[j];
        total += wcnt[j];
      }
      const unsigned rank = before + (unsigned)__popcll(bal & ((1ull << lane) - 1ull));
      if (eq && rank == need - 1) s_cut = (unsigned)i;   // the last tied id that is kept
      __syncthreads();
      if (total >= need) break;
      need -= total;
    }
    __syncthreads();
  }
  const unsigned cut = s_cut;
  // ---- Gumbel-max over the top-k set
  float best = -INFINITY, bv = -INFINITY;
  int bid = 0x7fffffff;
  const float* g = noise + step * (long long)V;
  for (int i = tid; i < V; i += SAMPLE_THREADS) {
    const float v = value(i);
    const unsigned key = fkey(v);
    if (key > prefix || (key == prefix && (unsigned)i <= cut)) {
      const float sc = v + g[i];
      if (sc > best || (sc == best && (v > bv || (v == bv && i < bid)))) { best = sc; bv = v; bid = i; }
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64), ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bid, o, 64);
    if (ob > best || (ob == best && (ov > bv || (ov == bv && oi < bid)))) { best = ob; bv = ov; bid = oi; }
  }
  if ((tid & 63) == 0) { r_sc[tid >> 6] = best; r_v[tid >> 6] = bv; r_id[tid >> 6] = bid; }
  __syncthreads();
  if (tid == 0) {
    for (int j = 1; j < SAMPLE_THREADS / 64; ++j)
      if (r_sc[j] > best || (r_sc[j] == best && (r_v[j] > bv || (r_v[j] == bv && r_id[j] < bid)))) {
        best = r_sc[j]; bv = r_v[j]; bid = r_id[j];
      }
    out[step] = bid;
    tok[0] = bid;
    pos[0] += 1;
    lens[0] += 1;
    *step_p = step + 1;
  }
}

}  // namespace

void launch_lm_sample(const void* logits, int logits_f32, int V, const float* noise, const float* eos_bias, int eos,
                      float temperature, int k, long long* step, long long* out, long long* tok, int* pos, int* lens,
                      hipStream_t s) {
  if (logits_f32)
    hipLaunchKernelGGL(lm_sample_kernel<true>, dim3(1), dim3(SAMPLE_THREADS), 0, s, logits, V, noise, eos_bias, eos,
                       temperature, k, step, out, tok, pos, lens);
  else
    hipLaunchKernelGGL(lm_sample_kernel<false>, dim3(1), dim3(SAMPLE_THREADS), 0, s, logits, V, noise, eos_bias, eos,
                       temperature, k, step, out, tok, pos, lens);
}

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
  // one split per 128 keys (one 64-key tile per wave), at most 32
  (void)B; (void)Hk;
  int ns = (L + 127) / 128;
  if (ns > 32) ns = 32;
  return ns < 1 ? 1 : ns;
}

template <int D>
static void launch_dec_d(const DecodeArgs& a, dim3 grid, hipStream_t s) {
  // the query-group size is a template argument: the score loop is then a fixed unrolled set of
  // broadcast LDS reads + FMAs (no per-head branches)
  switch (a.H / a.Hk) {
    case 1: hipLaunchKernelGGL((decode_attn_kernel<D, 1>), grid, dim3(DEC_THREADS), 0, s, a); break;
    case 2: hipLaunchKernelGGL((decode_attn_kernel<D, 2>), grid, dim3(DEC_THREADS), 0, s, a); break;
    case 3: hipLaunchKernelGGL((decode_attn_kernel<D, 3>), grid, dim3(DEC_THREADS), 0, s, a); break;
    case 4: hipLaunchKernelGGL((decode_attn_kernel<D, 4>), grid, dim3(DEC_THREADS), 0, s, a); break;
    case 5: hipLaunchKernelGGL((decode_attn_kernel<D, 5>), grid, dim3(DEC_THREADS), 0, s, a); break;
    case 6: hipLaunchKernelGGL((decode_attn_kernel<D, 6>), grid, dim3(DEC_THREADS), 0, s, a); break;
    case 7: hipLaunchKernelGGL((decode_attn_kernel<D, 7>), grid, dim3(DEC_THREADS), 0, s, a); break;
    default: hipLaunchKernelGGL((decode_attn_kernel<D, 8>), grid, dim3(DEC_THREADS), 0, s, a); break;
  }
}

void launch_decode_attention(const DecodeArgs& a, int ns, hipStream_t s) {
  dim3 grid(a.B * a.Hk, ns);
  if (a.d == 64) launch_dec_d<64>(a, grid, s);
  else launch_dec_d<128>(a, grid, s);
}
