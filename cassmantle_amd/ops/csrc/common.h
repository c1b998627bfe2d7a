// Shared device helpers for the cassmantle_amd gfx950 (CDNA4) kernel library.
//
// Conventions: bf16 tensors are handled as raw 16-bit words (uint16_t) and moved 16 bytes per
// lane (8 x bf16, `uint4`), never element by element (cdna_hip_programming.md G13).  MFMA
// operands use the gfx950 bf16 vector types; accumulators are f32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;

#define CM_DEVICE __device__ __forceinline__

CM_DEVICE float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// f32 -> bf16, round-to-nearest-even.  A plain cast lowers to the gfx950 hardware converter
// (v_cvt_pk_bf16_f32, NaN-preserving; MI355X_MICROARCH.md 'Correctness boundaries').
CM_DEVICE uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// two floats -> one packed dword in ONE v_cvt_pk_bf16_f32
CM_DEVICE uint32_t pack2(float a, float b) {
  bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// four fp32 -> four OCP e4m3 bytes (little-endian)
// (one asm pair: through the builtin, hipcc zero-fills the destination before the first
// half-word write -- a v_mov per packed word, 8 per fp8 attention tile, round 6 ISA)
CM_DEVICE uint32_t f8x4(float a, float b, float c, float d) {
  uint32_t w;
  asm("v_cvt_pk_fp8_f32 %0, %1, %2\n\tv_cvt_pk_fp8_f32 %0, %3, %4 op_sel:[0,0,1]"
      : "=&v"(w) : "v"(a), "v"(b), "v"(c), "v"(d));
  return w;
}

// slot of key offset kk (0..63) inside its 64-key block of the fp8 attention kernel's V8t image
// (attention.hip: slot 32h + j of a block holds the key of S accumulator register j&15 of key
// half j>>4 in lane half h)
CM_DEVICE int f8_slot(int kk) {
  const int hf = kk >> 5, w = kk & 31;
  const int h = (w >> 2) & 1, r = (w & 3) + 4 * (w >> 3);
  return 32 * h + 16 * hf + r;
}

// e4m3 K/V emission (GemmArgs::kv8): stores final values o[0..3] of row m, columns n..n+3 into
// the fp8 attention image when they are K or V columns; false for every other column
template <class Args>   // GemmArgs (kernels.h)
CM_DEVICE bool kv8_store4(const Args& p, int m, int n, const float* o) {
  if (p.kv8 == nullptr || n < p.kv8_col0) return false;
  const int C = p.kv8_hk * 64, rel = n - p.kv8_col0;
  const int b = m / p.kv8_ntok, key = m - b * p.kv8_ntok;
  const uint32_t w = f8x4(o[0], o[1], o[2], o[3]);
  if (rel < C) {
    const long long bh = (long long)b * p.kv8_hk + (rel >> 6);
    *reinterpret_cast<uint32_t*>(p.kv8 + (bh * p.kv8_ntok + key) * 64 + (rel & 63)) = w;
  } else {
    const long long B = p.M / p.kv8_ntok;
    uint8_t* V8t = p.kv8 + B * p.kv8_hk * p.kv8_ntok * 64;
    const long long bh = (long long)b * p.kv8_hk + ((rel - C) >> 6);
    const long long col = (key & ~63) + f8_slot(key & 63);
    uint8_t* dst = V8t + (bh * 64 + ((rel - C) & 63)) * p.kv8_ntok + col;
#pragma unroll
    for (int e = 0; e < 4; ++e) dst[(long long)e * p.kv8_ntok] = (uint8_t)(w >> (8 * e));
  }
  return true;
}


CM_DEVICE void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

CM_DEVICE uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]); v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]); v.w = pack2(f[6], f[7]);
  return v;
}

CM_DEVICE bf16x8_t as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8_t, v); }

// Four pairs of ds_read_b64_tr_b16 (T10 hardware-transposed LDS reads) and their lgkmcnt(0) in
// ONE asm statement (early-clobber outputs, so no output register is read, copied or reused
// before the data lands: cdna_hip_programming.md §5.7 item 1 form (i)).  Pair e reads at lds
// byte address a[e] and a[e] + HI_OFF.  hipcc's waitcnt pass treats the builtin form as aliasing
// every LDS-DMA still in flight and emits s_waitcnt vmcnt(0) in front of it -- in a kernel that
// keeps the next tile's buffer_load ... lds in flight that drains it every tile.
template <int HI_OFF>
CM_DEVICE void ds_read_tr16_x4x2(const uint32_t (&a)[4], s16x4_t (&lo)[4], s16x4_t (&hi)[4]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8\n\t"
      "ds_read_b64_tr_b16 %1, %8 offset:%c12\n\t"
      "ds_read_b64_tr_b16 %2, %9\n\t"
      "ds_read_b64_tr_b16 %3, %9 offset:%c12\n\t"
      "ds_read_b64_tr_b16 %4, %10\n\t"
      "ds_read_b64_tr_b16 %5, %10 offset:%c12\n\t"
      "ds_read_b64_tr_b16 %6, %11\n\t"
      "ds_read_b64_tr_b16 %7, %11 offset:%c12\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(lo[0]), "=&v"(hi[0]), "=&v"(lo[1]), "=&v"(hi[1]), "=&v"(lo[2]), "=&v"(hi[2]), "=&v"(lo[3]), "=&v"(hi[3])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "i"(HI_OFF)
      : "memory");
}
CM_DEVICE uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <typename T>
CM_DEVICE void lds_use(T& v) { asm volatile("" : "+v"(v)); }

// SiLU / quick-GELU with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE divide:
// the GroupNorm+SiLU apply and activation epilogues evaluate them per element
CM_DEVICE float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// exact-GELU with erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below bf16's 2^-9):
// one reciprocal + one exp + 5 FMAs instead of the libm erff (GEGLU epilogues evaluate it on every
// FF hidden element: 42M per level-1 call)
CM_DEVICE float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float y = fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t, 0.254829592f) * t;
  y = 1.0f - y * __expf(-ax * ax);
  return copysignf(y, x);
}
CM_DEVICE float gelu_f(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
CM_DEVICE float gelu_tanh_f(float x) {
  const float k = 0.7978845608028654f;
  return 0.5f * x * (1.0f + tanhf(k * (x + 0.044715f * x * x * x)));
}
CM_DEVICE float quick_gelu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * x)); }

// activation codes shared with python (ops/__init__.py _ACT)
// Gated acts (GEGLU: h*gelu(g), SWIGLU: h*silu(g)) read a [value; gate] weight of 2N rows.
// GroupNorm statistics are accumulated as 64-bit FIXED-POINT integers (sum x 2^24, sum of squares
// x 2^16): integer atomics are exact and order-independent, so the fused-statistics path is
// bit-deterministic run to run (fp32 atomics made whole denoise runs differ at the bf16 level).
// Range: |sum| < 5e11, sumsq < 1.4e14 per (image, channel); resolution 6e-8 / 1.5e-5.
constexpr double STAT_SCALE_SUM = 16777216.0;
constexpr double STAT_SCALE_SQ = 65536.0;
CM_DEVICE void stat_atomic_add(long long* st, int which, float v) {
  const double sc = which ? STAT_SCALE_SQ : STAT_SCALE_SUM;
  atomicAdd(reinterpret_cast<unsigned long long*>(st), (unsigned long long)__double2ll_rn((double)v * sc));
}
CM_DEVICE double stat_decode(long long v, int which) {
  return (double)v * (which ? (1.0 / STAT_SCALE_SQ) : (1.0 / STAT_SCALE_SUM));
}

enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_SILU = 2, ACT_QUICK_GELU = 3, ACT_GEGLU = 4, ACT_GELU_TANH = 5,
           ACT_SWIGLU = 6 };

__host__ __device__ inline bool is_gated(int act) { return act == ACT_GEGLU || act == ACT_SWIGLU; }
// GEGLU's GELU (the UNet feed-forward: 42M gate elements per eval at every level, evaluated in
// the GEMM epilogue beside the MFMAs): x * sigmoid(x * P(x^2)) with an odd degree-5 argument,
// fitted to the exact erf GELU (max |error| 3.0e-5 on [-9, 9], 0.04 % relative where
// |gelu| > 0.05 -- below bf16's half-ulp), 9 VALU with 2 transcendentals against ~18 with 2 for
// erf_fast: the A-in-registers GEGLU epilogue issued ~5 VALU per MFMA and was VALU-bound.
// The argument is clamped to |x| <= 8, where the sigmoid has saturated (< 2e-12) and before
// the polynomial turns over.  -DCASSMANTLE_GELU_EXACT restores erf_fast (A/B builds).
CM_DEVICE float gelu_geglu_f(float x) {
#ifdef CASSMANTLE_GELU_EXACT
  return gelu_f(x);
#else
  const float xc = __builtin_amdgcn_fmed3f(x, -8.f, 8.f);
  const float x2 = xc * xc;
  // coefficients pre-scaled by -log2(e): exp2 of this is exp(-x * P(x^2))
  const float z = xc * fmaf(x2, fmaf(x2, 0.0010350826722789555f, -0.10690469751684778f), -2.300978763043183f);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z));
#endif
}

CM_DEVICE float gate_f(float h, float g, int act) { return h * (act == ACT_SWIGLU ? silu_f(g) : gelu_geglu_f(g)); }

CM_DEVICE float apply_act(float x, int act) {
  switch (act) {
    case ACT_GELU: return gelu_f(x);
    case ACT_SILU: return silu_f(x);
    case ACT_QUICK_GELU: return quick_gelu_f(x);
    case ACT_GELU_TANH: return gelu_tanh_f(x);
    default: return x;
  }
}

CM_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
CM_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware bijective remap of a linear block id (cdna_hip_programming.md §5 / T1):
// consecutive logical tiles land on the same XCD (shared L2) under round-robin dispatch.
CM_DEVICE int xcd_remap(int bid, int nblocks) {
  const int nx = 8;
  int q = nblocks / nx, r = nblocks % nx;
  int xcd = bid % nx, idx = bid / nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
