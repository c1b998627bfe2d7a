// Flash attention for head dim 512 (the VAE decoder's single-head mid-block
// self-attention, 4096 tokens at SD-1.5 512^2 and 16384 at SDXL 1024^2).  Replaces the
// S = QK^T GEMM -> row softmax -> PV GEMM path that materialised S in HBM (1 GiB per image at
// 16384 tokens) and ran at 0.73x stock SDPA (profiles/r1_attn_variants_ab.txt).
//
// Same MFMA formulation as attention.hip (v_mfma_f32_32x32x16_bf16, lane-local softmax):
//   S^T[key][q] = K[key][:] . Q[q][:]    A = K rows from LDS (ds_read_b128), B = Q^T in VGPRs
//   O^T[d][q]  += V^T[d][key] . P^T      B = P^T straight from the S^T accumulator registers,
//                                        A = V^T via ds_read_b64_tr_b16 transposed reads
// At d = 512 one wave cannot hold both the Q^T fragments of 32 queries (128 VGPRs) and their
// O^T accumulator (256 AGPRs) next to the S tile, so the head dim is split over a PAIR of waves:
// wave (pair p, half e) holds Q[:, 256 e .. 256 e + 255] of the pair's 32 queries (64 VGPRs) and
// O^T rows 256 e .. 256 e + 255 (8 x 32x32 tiles = 128 AGPRs).  Per 32-key tile each wave forms
// the partial S^T over its d half, the pair exchanges the partials through LDS (4 KiB per wave)
// and both sum them -- bit-identical S, so the pair's softmax state never diverges -- and each
// wave then accumulates P.V for its own d half.  Block = 8 waves = 4 pairs = 128 queries, two
// waves per SIMD, sharing 32-key K/V tiles (32 KiB each) double-buffered in LDS; with the S
// exchange the block declares all 160 KiB.
// The tiles move by LDS-DMA (buffer_load ... lds, one 1-KiB key row per wave instruction) with
// the XOR swizzle applied on the source address:
//   K rows: 16-byte chunk c at c ^ (key & 15)      -> the 32 row reads of a k-step hit 16
//                                                    distinct chunks per lane group
//   V rows: 16-byte chunk c at c ^ 4 (key & 3)     -> the 4-row x 16-column transposed reads
//                                                    of a 32-lane half cover all 64 banks
// Short grids (B x Nq/128 < 256 blocks, e.g. 4 images x 4096 tokens) split the keys over
// blocks; the unnormalised fp32 O and (m, l) per split are merged by attn_d512_merge_kernel.
#include "common.h"
#include "kernels.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
constexpr int D5 = 512;
constexpr int DH5 = D5 / 2;             // head dims per wave
constexpr int KT5 = 32;                 // keys per tile
constexpr int NW5 = 8;                  // waves per block (two per SIMD)
constexpr int QB5 = 32 * NW5 / 2;       // queries per block (one 32-query group per wave pair)
constexpr int ROWB = D5 * 2;            // bytes per K / V row
constexpr int TILEB = KT5 * ROWB;       // 32 KiB
constexpr int XB = 16 * 64 * 4;         // S partial exchange bytes per wave
constexpr int LDS5 = 4 * TILEB + NW5 * XB;   // {K, V} x 2 buffers + exchange = 160 KiB

__global__ void __launch_bounds__(64 * NW5, 1) attn_d512_kernel(AttnArgs a, float* __restrict__ ws, int nsplit,
                                                                int keys_per_split) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds5[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pr = wave >> 1, dh = wave & 1;       // query group, head-dim half
  const int hlf = lane >> 5, ql = lane & 31;

  const int nqb = (a.Nq + QB5 - 1) / QB5;
  // XCD-aware order: the q-blocks of one (batch, head, split) run on one XCD and share its L2
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb;
  const int rest = bid / nqb;
  const int sp = rest % nsplit;
  const int bh = rest / nsplit;
  const int h = bh % a.H, b = bh / a.H;
  const int q0 = qb * QB5 + pr * 32;
  const int q = q0 + ql;

  int nk = a.Nk;
  if (a.kv_lens) nk = min(nk, a.kv_lens[b]);
  const int k_begin = sp * keys_per_split;
  int k_end = min(nk, k_begin + keys_per_split);
  if (a.causal) k_end = min(k_end, qb * QB5 + QB5);
  const int ntiles = k_end > k_begin ? (k_end - k_begin + KT5 - 1) / KT5 : 0;

  const uint16_t* Qp = a.q + (long long)b * a.q_sb + (long long)h * a.q_sh;
  const int hk = a.group > 1 ? h / a.group : h;
  const uint16_t* Kp = a.k + (long long)b * a.k_sb + (long long)hk * a.k_sh;
  const uint16_t* Vp = a.v + (long long)b * a.v_sb + (long long)hk * a.v_sh;

  // Q^T fragments of this wave's d half (pre-scaled by scale * log2 e):
  // lane holds Q[q][256 dh + 16 ks + 8 hlf .. +7]
  bf16x8_t qf[DH5 / 16];
  {
    const bool ok = q < a.Nq;
    const uint16_t* src = Qp + (long long)(ok ? q : 0) * a.q_sn + DH5 * dh + 8 * hlf;
    const float sc = a.scale * 1.4426950408889634f;
#pragma unroll
    for (int ks = 0; ks < DH5 / 16; ++ks) {
      uint4 v = *reinterpret_cast<const uint4*>(src + ks * 16);
      if (!ok) v = make_uint4(0, 0, 0, 0);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sc;
      qf[ks] = as_bf16x8(pack8(f));
    }
  }

  // ---- LDS-DMA staging: wave w moves key rows w and w + 8 ... (4 K rows + 4 V rows per tile)
  const long long k_rows = (long long)(nk - 1) * a.k_sn + D5;     // elements reachable
  const long long v_rows = (long long)(nk - 1) * a.v_sn + D5;
  __amdgpu_buffer_rsrc_t rsK = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(Kp), (short)0,
                                                                  (int)(k_rows * 2), 0x00020000);
  __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(Vp), (short)0,
                                                                  (int)(v_rows * 2), 0x00020000);
  constexpr int OOB = (int)0x80000000;
  auto stage = [&](int t, int buf) {
    const int kb = k_begin + t * KT5;
    uint16_t* Kb = lds5 + (size_t)buf * TILEB;
    uint16_t* Vb = Kb + TILEB / 2;
    // an opaque copy of the lane id: the per-row source offsets are recomputed per tile (2 VALU
    // each) instead of being hoisted into registers, which spilled and put serial scratch
    // reloads in front of every tile's DMA issue
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < KT5 / NW5; ++i) {
      const int r = wave + NW5 * i;                 // tile row (uniform)
      const int key = kb + r;
      const bool live = key < k_end;
      const int kc = ln ^ (r & 15), vc = ln ^ (4 * (r & 3));
      const int ko = live ? (int)((long long)key * a.k_sn * 2 + kc * 16) : OOB;
      const int vo = live ? (int)((long long)key * a.v_sn * 2 + vc * 16) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsK, (lds_void*)(Kb + r * D5), 16, ko, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsV, (lds_void*)(Vb + r * D5), 16, vo, 0, 0, 0);
    }
  };
  float* Xs = reinterpret_cast<float*>(lds5 + 2 * TILEB);     // [wave][16 regs][64 lanes]
  float* Xmine = Xs + wave * (16 * 64) + lane;
  const float* Xpart = Xs + (wave ^ 1) * (16 * 64) + lane;

  f32x16_t oacc[DH5 / 32];
#pragma unroll
  for (int i = 0; i < DH5 / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  float m_run = 0.f, l_run = 0.f;

  // transposed-read lane geometry (T10): group g = lane >> 4, i = lane & 15
  const int tg = lane >> 4, ti = lane & 15;
  const int tr_row = 4 * (tg >> 1) + (ti >> 2);                    // key row within the k-step
  const int tr_chunk = 2 * (tg & 1) + ((ti & 3) >> 1);             // logical chunk within 32 d
  const int tr_byte = 8 * (ti & 1);
  const int tr_swz = 4 * (tr_row & 3);

  if (ntiles > 0) stage(0, 0);
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // tile t landed for every wave; tile t-1's buffer is free
    if (t + 1 < ntiles) stage(t + 1, buf ^ 1);
    const uint16_t* Kb = lds5 + (size_t)buf * TILEB;
    const uint16_t* Vb = Kb + TILEB / 2;

    // ---- partial S^T = K Q^T over this wave's d half: K rows ql, logical chunk 32 dh + 2 ks + hlf
    f32x16_t sacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
    {
      // (opaque per-tile copies of the lane-dependent address terms: hoisted out of the loop they
      // cost 16+ VGPRs and spilled; recomputed they are one v_xor per fragment read)
      int qlv = ql;
      asm volatile("" : "+v"(qlv));
      const char* krow = reinterpret_cast<const char*>(Kb + qlv * D5);
      const int sw = qlv & 15;
#pragma unroll
      for (int ks = 0; ks < DH5 / 16; ++ks) {
        const int pc = (32 * dh + 2 * ks + hlf) ^ sw;
        const bf16x8_t kf = as_bf16x8(*reinterpret_cast<const uint4*>(krow + pc * 16));
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], sacc, 0, 0, 0);
        if ((ks & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // bound the fragment read-ahead
      }
    }
    // ---- exchange the partials within the pair; both waves form the identical sum
#pragma unroll
    for (int r = 0; r < 16; ++r) Xmine[r * 64] = sacc[r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float o = Xpart[r * 64];
      sacc[r] = (dh == 0 ? sacc[r] + o : o + sacc[r]) - m_run;
    }
    // ---- masking (ragged key range, kv_lens, causal)
    const int kbase = k_begin + t * KT5;
    if (kbase + KT5 > k_end || (a.causal && kbase + KT5 - 1 > q0)) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kbase + (r & 3) + 8 * (r >> 2) + 4 * hlf;
        if (key >= k_end || (a.causal && key > q)) sacc[r] = -INFINITY;
      }
    }
    // ---- online softmax, deferred max (attention.hip): rescale only when a query's max moves
    // by more than 2^8, so the common tile is one v_exp per score and no O traffic
    constexpr float RESCALE_THR = 8.f;
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (__builtin_expect(t == 0 || !__all(mx <= RESCALE_THR), 0)) {
      // a real branch: without the volatile asm hipcc if-converts this block and rescales O
      // and S by alpha = 1 on EVERY tile (a v_pk_mul per two O registers per tile)
      asm volatile("" ::: "memory");
      float delta = (t == 0) ? mx : fmaxf(mx, 0.f);
      if (!(delta > -1e30f)) delta = 0.f;
      m_run += delta;
      const float alpha = __builtin_amdgcn_exp2f(-delta);
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < DH5 / 32; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[i][r] *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[r] -= delta;
    }
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = __builtin_amdgcn_exp2f(sacc[r]);
      sacc[r] = pv;
      rs += pv;
    }
    rs += __shfl_xor(rs, 32, 64);
    l_run += rs;
    // ---- P^T fragments: k-step s uses accumulator registers 8 s .. 8 s + 7
    bf16x8_t pf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint4 u;
      u.x = pack2(sacc[8 * s + 0], sacc[8 * s + 1]);
      u.y = pack2(sacc[8 * s + 2], sacc[8 * s + 3]);
      u.z = pack2(sacc[8 * s + 4], sacc[8 * s + 5]);
      u.w = pack2(sacc[8 * s + 6], sacc[8 * s + 7]);
      pf[s] = as_bf16x8(u);
    }
    // ---- O^T += V^T P^T over this wave's d half (element j of lane half h pairs with key
    // 16 s + 8 (j >> 2) + 4 h + (j & 3))
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      int trr = tr_row;
      asm volatile("" : "+v"(trr));
      const char* vlo = reinterpret_cast<const char*>(Vb + (16 * s + trr) * D5) + tr_byte;
#pragma unroll
      for (int g = 0; g < DH5 / 32; g += 4) {
        // transposed reads + their wait in one asm statement (common.h ds_read_tr16_x4x2: the
        // builtin made hipcc drain the next tile's in-flight DMA before every read)
        uint32_t ad[4];
        s16x4_t lo[4], hi[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) ad[e] = lds_addr(vlo + ((4 * (8 * dh + g + e) + tr_chunk) ^ tr_swz) * 16);
        ds_read_tr16_x4x2<8 * ROWB>(ad, lo, hi);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          typedef __attribute__((ext_vector_type(8))) short s16x8_t;
          const s16x8_t vv = {lo[e][0], lo[e][1], lo[e][2], lo[e][3], hi[e][0], hi[e][1], hi[e][2], hi[e][3]};
          oacc[g + e] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, vv), pf[s], oacc[g + e], 0, 0, 0);
        }
      }
    }
  }

  if (q >= a.Nq) return;
  if (nsplit == 1) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    uint16_t* Op = a.o + (long long)b * a.o_sb + (long long)q * a.o_sn + (long long)h * a.o_sh + DH5 * dh;
#pragma unroll
    for (int dc = 0; dc < DH5 / 32; ++dc)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int dd = 32 * dc + 8 * g4 + 4 * hlf;
        uint2 w;
        w.x = pack2(oacc[dc][4 * g4 + 0] * inv, oacc[dc][4 * g4 + 1] * inv);
        w.y = pack2(oacc[dc][4 * g4 + 2] * inv, oacc[dc][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(Op + dd) = w;
      }
    return;
  }
  // split keys: unnormalised O (fp32) + (m, l) of this split, merged by attn_d512_merge_kernel
  const long long row = ((long long)sp * a.B * a.H + (long long)b * a.H + h) * a.Nq + q;
  float* Ow = ws + row * D5 + DH5 * dh;
#pragma unroll
  for (int dc = 0; dc < DH5 / 32; ++dc)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int dd = 32 * dc + 8 * g4 + 4 * hlf;
      *reinterpret_cast<float4*>(Ow + dd) =
          make_float4(oacc[dc][4 * g4 + 0], oacc[dc][4 * g4 + 1], oacc[dc][4 * g4 + 2], oacc[dc][4 * g4 + 3]);
    }
  if (hlf == 0 && dh == 0) {
    float* ml = ws + (long long)nsplit * a.B * a.H * a.Nq * D5 + row * 2;
    *reinterpret_cast<float2*>(ml) = make_float2(m_run, l_run);
  }
}

// one block of 128 threads per (b, h, q) row: 4 head dims per thread
__global__ void __launch_bounds__(128) attn_d512_merge_kernel(AttnArgs a, const float* __restrict__ ws, int nsplit) {
  const long long rows = (long long)a.B * a.H * a.Nq;
  const long long r = blockIdx.x;
  const int q = (int)(r % a.Nq);
  const int bh = (int)(r / a.Nq);
  const int h = bh % a.H, b = bh / a.H;
  const float* ml = ws + (long long)nsplit * rows * D5;
  float mmax = -INFINITY;
  for (int s = 0; s < nsplit; ++s) {
    const float2 v = *reinterpret_cast<const float2*>(ml + (s * rows + r) * 2);
    if (v.y > 0.f) mmax = fmaxf(mmax, v.x);
  }
  float o[4] = {0.f, 0.f, 0.f, 0.f}, l = 0.f;
  const int dd = threadIdx.x * 4;
  for (int s = 0; s < nsplit; ++s) {
    const float2 v = *reinterpret_cast<const float2*>(ml + (s * rows + r) * 2);
    if (!(v.y > 0.f)) continue;
    const float w = __builtin_amdgcn_exp2f(v.x - mmax);
    l += w * v.y;
    const float4 ov = *reinterpret_cast<const float4*>(ws + (s * rows + r) * D5 + dd);
    o[0] += w * ov.x; o[1] += w * ov.y; o[2] += w * ov.z; o[3] += w * ov.w;
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  uint16_t* Op = a.o + (long long)b * a.o_sb + (long long)q * a.o_sn + (long long)h * a.o_sh + dd;
  *reinterpret_cast<uint2*>(Op) = make_uint2(pack2(o[0] * inv, o[1] * inv), pack2(o[2] * inv, o[3] * inv));
}

int d512_splits(const AttnArgs& a) {
  const long long blocks = (long long)((a.Nq + QB5 - 1) / QB5) * a.H * a.B;
  int ns = 1;
  while (blocks * ns < 256 && ns < 8 && (a.Nk / (ns * 2)) >= 4 * KT5) ns *= 2;
  return ns;
}

}  // namespace

long long attention_d512_workspace(const AttnArgs& a) {
  const int ns = d512_splits(a);
  if (ns == 1) return 0;
  return (long long)ns * a.B * a.H * a.Nq * (D5 + 2) * 4;
}

void launch_attention_d512(const AttnArgs& a, float* ws, hipStream_t s) {
  // > 64 KiB dynamic LDS opt-in, once per process (thread-safe static init)
  static const bool once = [&] {
    (void)hipFuncSetAttribute((const void*)&attn_d512_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS5);
    return true;
  }();
  (void)once;
  const int ns = ws ? d512_splits(a) : 1;
  int kps = (a.Nk + ns - 1) / ns;
  kps = (kps + KT5 - 1) / KT5 * KT5;
  const int nqb = (a.Nq + QB5 - 1) / QB5;
  dim3 grid((unsigned)(nqb * ns * a.H * a.B));
  hipLaunchKernelGGL(attn_d512_kernel, grid, dim3(64 * NW5), LDS5, s, a, ws, ns, kps);
  if (ns > 1)
    hipLaunchKernelGGL(attn_d512_merge_kernel, dim3((unsigned)((long long)a.B * a.H * a.Nq)), dim3(128), 0, s, a,
                       ws, ns);
}
