// Flash-attention forward for gfx950 (SURVEY §2.3 K1 self-attn, K2 cross-attn, K13/K16 text
// encoders): softmax(Q K^T * scale) V with online softmax, no score matrix in HBM.
//
// MFMA formulation (v_mfma_f32_32x32x16_bf16), chosen so every softmax quantity is lane-local:
//   S^T[key][q] = K[key][:] . Q[q][:]      A = K tile from LDS (ds_read_b128 rows),
//                                          B = Q^T fragments held in registers for the whole loop
//   -> each lane owns ONE query column (q = lane & 31) and 16 of the tile's keys; the other 16
//      keys of that query sit in lane ^ 32, so a row max / row sum is 31 VALU ops + one
//      cross-half shuffle (cdna_hip_programming.md Appendix B 'swapped QK^T').
//   O^T[d][q] += V^T[d][key] . P^T[key][q]  B = P^T taken straight from the S^T accumulator
//                                           registers (converted to bf16, permuted k order;
//                                           guide §3 'accumulator tile as next MFMA operand'),
//                                           A = V^T via ds_read_b64_tr_b16 hardware-transposed
//                                           LDS reads of the row-major V tile (T10).
//   -> the O accumulator is also query-per-lane, so the online-softmax rescale and the final
//      1/l normalisation are lane-local multiplies.
// Head dims 40/80/160 (SD-1.5), 64 (SDXL, CLIP), 32 (MiniLM): QK^T runs over d padded to 16,
// P.V over d padded to 32; padding is zero-filled in LDS.  Ragged key counts (77-token cross
// attention, padded MiniLM batches via kv_lens) and causal masking (CLIP) are masked to -inf.
// K/V tiles of 64 keys are staged global->registers->LDS with the next tile's loads issued
// before the current tile's MFMAs (T14).  LDS strides are padded so the K row reads
// (16 distinct rows per lane group) and the V transposed reads are bank-conflict-free.
#include <atomic>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int KT = 64;  // keys per tile

// A/B switches of the round-4 micro-changes, each measured alone on one box
// (profiles/r4_attn_switches_ab.txt): the permlane cross-half max/sum and the static priority
// of the younger half are 1-4 % faster and on; branch-free staging loads (value selects) were
// 4-12 % SLOWER (their selects are VALU, the contended pipe of this kernel) and are off
#ifndef ATTN_KBATCH
#define ATTN_KBATCH 1
#endif
#ifndef ATTN_PERMLANE
#define ATTN_PERMLANE 1
#endif
#ifndef ATTN_BRANCHLESS
#define ATTN_BRANCHLESS 0
#endif
#ifndef ATTN_PRIO
#define ATTN_PRIO 1
#endif
#ifndef F8_ONES_SUM
#define F8_ONES_SUM 1
#endif

// v_permlane32_swap of a value with itself: one of the two results is this lane's own value and
// the other lane l ^ 32's (lanes 0-31 get it in .y, lanes 32-63 in .x), so a cross-half max or
// sum is fmax(.x, .y) / .x + .y in every lane -- a VALU op instead of __shfl_xor's ds_bpermute
// round trip through the LDS unit (guide T12)
CM_DEVICE float2 both_halves(float v) {
  const unsigned u = __float_as_uint(v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return make_float2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

template <int DQK, int DO>
struct AttnGeom {
  static constexpr int KCH = DQK / 8;                         // 16B chunks per K row
  static constexpr int KSTR = (KCH % 2 == 0 ? KCH + 1 : KCH) * 8;  // elements; odd chunk count
  static constexpr int VCH = DO / 8;
  static constexpr int VB = DO * 2;                            // bytes per V row
  static constexpr int VSTR = ((VB % 256 == 64) || (VB % 256 == 192)) ? DO : DO + 32;
  static constexpr int LDS_BYTES = KT * KSTR * 2 + KT * VSTR * 2;
};

// DB: K/V double-buffered in LDS, so the next tile is stored into the other buffer while this
// one is read and each tile needs ONE barrier (single buffer: one before the store -- everyone
// is done reading -- and one after it)
// (Measured and removed in round 4, kept in git history: software-pipelined tiles on 3 buffers,
// profiles/r2_attn_pipe_ab.txt; staggered wave halves, profiles/r3_attn_stag_ab.txt.)
template <int DQK, int DO, int NW, bool DB>
// min blocks 8 / NW caps the kernel at 256 registers: the compiler then keeps the MFMA
// accumulators in VGPRs, where the softmax reads and writes them (with a 512-register budget it
// chose AGPRs and paid a v_accvgpr_read + write per score per pass: ~144 of ~300 VALU per tile)
__global__ void __launch_bounds__(64 * NW, NW >= 4 ? 8 / NW : (DO >= 128 ? 1 : 2)) attn_fwd_kernel(AttnArgs a) {
  using G = AttnGeom<DQK, DO>;
  constexpr int THREADS = 64 * NW;
  constexpr int QB = 32 * NW;
  constexpr int NKS = DQK / 16;       // k-steps of QK^T
  constexpr int NDC = DO / 32;        // 32-row chunks of O^T
  constexpr int KLD = (KT * G::KCH + THREADS - 1) / THREADS;
  constexpr int VLD = (KT * G::VCH + THREADS - 1) / THREADS;

  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  constexpr int BUF = KT * G::KSTR + KT * G::VSTR;   // elements of one K/V buffer
  uint16_t* Ks = lds;
  uint16_t* Vs = lds + KT * G::KSTR;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hlf = lane >> 5;          // lane half
  const int ql = lane & 31;

  const int nqb = (a.Nq + QB - 1) / QB;
  // XCD-aware order: the q-blocks of one (batch, head) run on one XCD, so its K/V (<= 1 MB)
  // is fetched into that XCD's L2 once instead of once per XCD
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb;
  const int bh = bid / nqb;
  const int h = bh % a.H;
  const int b = bh / a.H;
  const int q0 = qb * QB + wave * 32;
  const int q = q0 + ql;

  int nk = a.Nk;
  if (a.kv_lens) nk = min(nk, a.kv_lens[b]);
  int ntiles = (nk + KT - 1) / KT;
  if (a.causal) ntiles = min(ntiles, (qb * QB + QB + KT - 1) / KT);

  const uint16_t* Qp = a.q + (long long)b * a.q_sb + (long long)h * a.q_sh;
  const int hk = a.group > 1 ? h / a.group : h;   // grouped-query attention (LM prefill)
  const uint16_t* Kp = a.k + (long long)b * a.k_sb + (long long)hk * a.k_sh;
  const uint16_t* Vp = a.v + (long long)b * a.v_sb + (long long)hk * a.v_sh;
  const int d = a.d;

  // Q^T fragments: lane holds Q[q][ks*16 + 8*hlf .. +7]
  bf16x8_t qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    uint4 v = make_uint4(0, 0, 0, 0);
    int d0 = ks * 16 + 8 * hlf;
    if (q < a.Nq && d0 < d) v = *reinterpret_cast<const uint4*>(Qp + (long long)q * a.q_sn + d0);
    // pre-scale Q by scale*log2(e): S comes out of the MFMA in log2 units, so softmax needs
    // no per-element multiply
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= a.scale * 1.4426950408889634f;
    qf[ks] = as_bf16x8(pack8(f));
  }

  f32x16_t oacc[NDC];
#pragma unroll
  for (int i = 0; i < NDC; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  float m_run = 0.f, l_run = 0.f;   // m_run: reference max in log2 units (set on the first tile)
  // padded head dims (40 -> 64, 80 -> 96): the first padding column of V carries ones, so the
  // row sum of P comes out of the P.V MFMAs (rescaled with O for free) instead of 32 VALU adds
  // and a cross-half shuffle per tile
  constexpr bool ones = DO > DQK;   // d <= DQK < DO: at least one zero-padded V column
  // head dim 40 (QK^T over 48): the first padding column also carries the running max, so
  // S - m comes out of the MFMA -- K[:, 40] = 1 and Q^T[40][q] = -m (bf16, kept exact by
  // tracking m as a bf16 value): no per-score accumulator initialisation
  constexpr bool MF = (DQK == 48 && DO == 64);

  // staging geometry is tile-invariant: decode (key, chunk) once per thread; per tile only the
  // uniform key base moves (the first version re-derived it per tile: ~40 VALU per tile)
  uint4 kr[KLD], vr[VLD];
  int k_key[KLD], v_key[VLD], k_lds[KLD], v_lds[VLD];
  const uint16_t* k_src[KLD];
  const uint16_t* v_src[VLD];
  bool k_use[KLD], v_use[VLD], v_one[VLD], k_one[KLD];
#pragma unroll
  for (int i = 0; i < KLD; ++i) {
    const int idx = tid + i * THREADS;
    const int key = idx / G::KCH, ch = idx - key * G::KCH;
    k_key[i] = key;
    k_use[i] = key < KT && ch * 8 < d;
    k_one[i] = MF && key < KT && ch * 8 == d;     // K[:, d] = 1.0 -> the -m column of Q^T
    k_lds[i] = key < KT ? key * G::KSTR + ch * 8 : -1;
    k_src[i] = Kp + (long long)key * a.k_sn + ch * 8;
  }
#pragma unroll
  for (int i = 0; i < VLD; ++i) {
    const int idx = tid + i * THREADS;
    const int key = idx / G::VCH, ch = idx - key * G::VCH;
    v_key[i] = key;
    v_use[i] = key < KT && ch * 8 < d;
    v_one[i] = ones && key < KT && ch * 8 == d;   // V[:, d] = 1.0 -> P.V accumulates the row sum
    v_lds[i] = key < KT ? key * G::VSTR + ch * 8 : -1;
    v_src[i] = Vp + (long long)key * a.v_sn + ch * 8;
  }
  // branch-free staging loads: every lane loads (an out-of-range or padding chunk reads the
  // K / V base row instead) and the padding value is selected afterwards -- a conditional load
  // made hipcc wrap every load in an exec-mask branch (s_and_saveexec / s_cbranch_execz)
  auto gload = [&](int t) {
    const int kbase = t * KT;
    const long long ko = (long long)kbase * a.k_sn, vo = (long long)kbase * a.v_sn;
#pragma unroll
    for (int i = 0; i < KLD; ++i) {
      if constexpr (ATTN_BRANCHLESS) {
        const bool ok = k_use[i] && kbase + k_key[i] < nk;
        const uint4 v = *reinterpret_cast<const uint4*>(ok ? k_src[i] + ko : Kp);
        const uint4 z = make_uint4(k_one[i] ? 0x3F80u : 0u, 0, 0, 0);
        kr[i] = make_uint4(ok ? v.x : z.x, ok ? v.y : z.y, ok ? v.z : z.z, ok ? v.w : z.w);
      } else {
        uint4 v = make_uint4(k_one[i] ? 0x3F80u : 0u, 0, 0, 0);
        if (k_use[i] && kbase + k_key[i] < nk) v = *reinterpret_cast<const uint4*>(k_src[i] + ko);
        kr[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < VLD; ++i) {
      if constexpr (ATTN_BRANCHLESS) {
        const bool ok = v_use[i] && kbase + v_key[i] < nk;
        const uint4 v = *reinterpret_cast<const uint4*>(ok ? v_src[i] + vo : Vp);
        const uint4 z = make_uint4(v_one[i] ? 0x3F80u : 0u, 0, 0, 0);
        vr[i] = make_uint4(ok ? v.x : z.x, ok ? v.y : z.y, ok ? v.z : z.z, ok ? v.w : z.w);
      } else {
        uint4 v = make_uint4(v_one[i] ? 0x3F80u : 0u, 0, 0, 0);
        if (v_use[i] && kbase + v_key[i] < nk) v = *reinterpret_cast<const uint4*>(v_src[i] + vo);
        vr[i] = v;
      }
    }
  };
  auto lstore = [&](int bo) {   // bo: element offset of the target buffer
#pragma unroll
    for (int i = 0; i < KLD; ++i)
      if (k_lds[i] >= 0) *reinterpret_cast<uint4*>(Ks + bo + k_lds[i]) = kr[i];
#pragma unroll
    for (int i = 0; i < VLD; ++i)
      if (v_lds[i] >= 0) *reinterpret_cast<uint4*>(Vs + bo + v_lds[i]) = vr[i];
  };

  if (ntiles > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  // static priority for the second-dispatched half of an 8-wave block (MI355X_MICROARCH.md
  // "Two waves per SIMD" item 4): it otherwise loses every VALU arbitration to its older partner
  if constexpr (NW == 8 && ATTN_PRIO) {
    if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  }

  // tr-read lane geometry (T10): group g = lane>>4, i = lane&15 -> row q' = i>>2, col 4*(i&3)
  const int tg = lane >> 4, ti = lane & 15;
  const int tr_row = 4 * (tg >> 1) + (ti >> 2);
  const int tr_col = 16 * (tg & 1) + 4 * (ti & 3);

  for (int t = 0; t < ntiles; ++t) {
    const bool more = t + 1 < ntiles;
    if (more) gload(t + 1);                          // staged during this tile
    const int bo = DB ? (t & 1) * BUF : 0;           // this tile's buffer

    // ---- S^T = K Q^T for 64 keys (two 32-key accumulators)
    f32x16_t sacc[2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[hf][r] = MF ? 0.f : -m_run;   // S - m folded into the MFMA
      const uint16_t* krow = Ks + bo + (hf * 32 + ql) * G::KSTR + 8 * hlf;
      if constexpr (ATTN_KBATCH && NKS <= 5) {
        // all NKS K fragments of this half in flight before its MFMA chain: hipcc otherwise
        // issues read, wait, MFMA per k-step and every MFMA waits out a full LDS latency
        // (ATTN_KBATCH=0: the per-step form, A/B knob)
        // (d <= 80 only: the d = 160 blocks sit at 250 VGPRs and spill with the extra fragments)
        bf16x8_t kf[NKS];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) kf[ks] = as_bf16x8(*reinterpret_cast<const uint4*>(krow + ks * 16));
        __builtin_amdgcn_sched_barrier(0);   // (the scheduler would sink each read to its MFMA)
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) sacc[hf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ks], qf[ks], sacc[hf], 0, 0, 0);
      } else {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          bf16x8_t kf = as_bf16x8(*reinterpret_cast<const uint4*>(krow + ks * 16));
          sacc[hf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], sacc[hf], 0, 0, 0);
        }
      }
    }

    // ---- masking
    const int kbase = t * KT;
    const bool need_mask = (kbase + KT > nk) || (a.causal && kbase + KT - 1 > q0);
    if (need_mask) {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int key = kbase + hf * 32 + (r & 3) + 8 * (r >> 2) + 4 * hlf;
          bool bad = key >= nk || (a.causal && key > q);
          if (bad) sacc[hf][r] = -INFINITY;
        }
    }

    // ---- online softmax with a deferred max (lane-local query; lane ^32 holds the other 32
    // keys).  sacc already holds S - m_run (log2 units).  The reference max only moves when a
    // query's tile max exceeds it by more than RESCALE_THR (and always on the first tile, whose
    // m_run = 0 is a placeholder), so p <= 2^THR and the common tile costs one v_exp per score.
    // At a rescale every quantity still at the old max — O, l and this tile's scores — is
    // shifted exactly once, before any P of this tile is formed (guide T13 hazard).
    constexpr float RESCALE_THR = 8.f;
    float mx = -INFINITY;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[hf][r]);
    if constexpr (ATTN_PERMLANE) {
      const float2 hm = both_halves(mx);
      mx = fmaxf(hm.x, hm.y);
    } else {
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    }
    if (__builtin_expect(t == 0 || !__all(mx <= RESCALE_THR), 0)) {
      // a real branch: without the volatile asm hipcc if-converts this block and rescales O
      // and S by alpha = 1 on EVERY tile (a v_pk_mul per two O registers per tile)
      asm volatile("" ::: "memory");
      float delta = (t == 0) ? mx : fmaxf(mx, 0.f);
      if (!(delta > -1e30f)) delta = 0.f;            // fully masked tile for this query
      if constexpr (MF) {
        // the new reference max as a bf16 value (it is an MFMA operand); only the rounded
        // shift is applied, so every quantity stays consistent
        const float mn = (float)(__bf16)(m_run + delta);
        delta = mn - m_run;
        m_run = mn;
        qf[2][0] = hlf ? (__bf16)(-m_run) : qf[2][0];
      } else {
        m_run += delta;
      }
      const float alpha = __builtin_amdgcn_exp2f(-delta);
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < NDC; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[i][r] *= alpha;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[hf][r] -= delta;
    }
    float rs = 0.f;
    if constexpr (ones) {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[hf][r] = __builtin_amdgcn_exp2f(sacc[hf][r]);
    } else {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = __builtin_amdgcn_exp2f(sacc[hf][r]);
          sacc[hf][r] = pv;
          rs += pv;
        }
      if constexpr (ATTN_PERMLANE) {
        const float2 hs = both_halves(rs);
        rs = hs.x + hs.y;
      } else {
        rs += __shfl_xor(rs, 32, 64);
      }
    }
    l_run += rs;

    // ---- P^T fragments (bf16), k-step kk = 2*hf + s uses regs 8s..8s+7 of sacc[hf]
    bf16x8_t pf[4];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        uint4 u;
        u.x = pack2(sacc[hf][8 * s + 0], sacc[hf][8 * s + 1]);
        u.y = pack2(sacc[hf][8 * s + 2], sacc[hf][8 * s + 3]);
        u.z = pack2(sacc[hf][8 * s + 4], sacc[hf][8 * s + 5]);
        u.w = pack2(sacc[hf][8 * s + 6], sacc[hf][8 * s + 7]);
        pf[2 * hf + s] = as_bf16x8(u);
      }

    // ---- O^T += V^T P^T
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
      for (int dc = 0; dc < NDC; ++dc) {
        const uint16_t* base = Vs + bo + (16 * kk + tr_row) * G::VSTR + 32 * dc + tr_col;
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(base));
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(base + 8 * G::VSTR));
        typedef __attribute__((ext_vector_type(8))) short s16x8_t;
        s16x8_t vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bf16x8_t vf = __builtin_bit_cast(bf16x8_t, vv);
        oacc[dc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kk], oacc[dc], 0, 0, 0);
      }
    }

    if constexpr (DB) {
      // the other buffer was last read in tile t - 1, which every wave finished before the
      // previous barrier
      if (more) lstore(BUF - bo);
      __syncthreads();
    } else {
      __syncthreads();
      if (more) {
        lstore(0);
        __syncthreads();
      }
    }
  }

  // ---- epilogue: O[q][d] = O^T[d][q] / l
  if constexpr (ones) {
    // row sum sits in O^T row d: chunk d/32, register 4*((d%32)/8) of the lane half 0
    const int dcl = d >> 5, rgl = ((d & 31) >> 3) << 2;
    float ls = 0.f;
#pragma unroll
    for (int dc = 0; dc < NDC; ++dc)
#pragma unroll
      for (int r = 0; r < 16; r += 4)
        if (dc == dcl && r == rgl) ls = oacc[dc][r];
    l_run = __shfl(ls, ql, 64);
  }
  if (q < a.Nq) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    uint16_t* Op = a.o + (long long)b * a.o_sb + (long long)q * a.o_sn + (long long)h * a.o_sh;
#pragma unroll
    for (int dc = 0; dc < NDC; ++dc)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        int dd = 32 * dc + 8 * g4 + 4 * hlf;
        if (dd < d) {
          uint2 w;
          w.x = pack2(oacc[dc][4 * g4 + 0] * inv, oacc[dc][4 * g4 + 1] * inv);
          w.y = pack2(oacc[dc][4 * g4 + 2] * inv, oacc[dc][4 * g4 + 3] * inv);
          *reinterpret_cast<uint2*>(Op + dd) = w;
        }
      }
  }
}

// ======================================================================= head dim 40, 16x16 MFMAs
// The SD-1.5 level-1 attention (d = 40) on the 32x32x16 kernel above pays for P.V over 64 O^T
// rows (40 real + ones column + 23 zero rows: 37.5 % of its MFMA cycles are padding).  Here every
// product is a 16x16 block, so O^T needs only 48 rows (3 blocks):
//   S^T[16 keys][16 q] = K . Q^T     two 16x16x32 steps: d 0..31, then d 32..39 plus the -m
//                                    column (K[:, 40] = 1, Q^T[40][q] = -m, as above)
//   O^T[16 d][16 q] += V^T . P^T     16x16x32 over 32 keys; P^T straight from the S accumulators
//                                    of two 16-key blocks (k order permuted, see below), V^T by
//                                    ds_read_b64_tr_b16 of the row-major V tile (T10)
// Per wave: 32 queries (two 16-query blocks), 64-key tiles: QK^T 8 x 2 and P.V 12 16x16x32 MFMAs,
// the 448 cycles per tile of the 32x32 layout, but on the 16x16 shape (MI355X_MICROARCH.md DVFS
// item 7: the chip holds a higher clock on it) and with no padded O^T rows.  Lane l (g = l >> 4, i = l & 15) holds
// S^T[key 16 kb + 4 g + r][query 16 qb + i], r = 0..3: a query's 64 keys sit in 4 lanes x 16
// registers.  The deferred-max test only needs each lane's OWN max (all lanes <= THR <=> every
// query's max <= THR), so the common tile has no cross-lane op; a rescale reduces over the 4
// lanes (xor 16, xor 32).  The P.V contraction index k = 8 g + j of a k-step s pairs
//   B = P^T: element j of lane (g, q) = P[q][32 s + 16 (j >> 2) + 4 g + (j & 3)]  (S registers)
//   A = V^T: element j of lane (g, d) = V[32 s + 16 (j >> 2) + 4 g + (j & 3)][d]  (two tr reads)
// Row sums come out of O^T row 40 (V[:, 40] = 1), rescaled with O for free.  Column 40 of K and
// V (1.0) and 41..47 (0) are written once per LDS buffer; only d 0..39 is staged per tile.
constexpr int A16_STR = 48;          // LDS row (elements): conflict-free b128 K reads and V tr reads
constexpr int A16_NCH = 5;           // staged 16-B chunks per key row (d = 40)
#ifndef A16_KSTR
#define A16_KSTR 48                  // K row (elements) of the 16x16 kernel (56 measured slower: r5_attn_d40_mixed_ab)
#endif
// A16_BUFLD: K/V staging loads through per-tile buffer resources (base = the tile's first key,
// num_records = the bytes of its valid keys), so keys past nk and idle lanes read zeros from the
// buffer unit's range check: no zero-fill moves, compares, exec masking or 64-bit address VALU
// per tile.  A16_UNROLL2: the tile loop unrolled by two, so both LDS buffers' addresses are
// compile-time immediates.  The kernel is bound by the SIMD's issue slots (v_exp_f32 8 cycles,
// MFMA 8 of its 16, VALU 4: ~800 issue cycles per wave-tile against 448 of MFMA), so every VALU
// taken off the tile counts (round 6).
#ifndef A16_BUFLD
#define A16_BUFLD 1
#endif
#ifndef A16_UNROLL2
#define A16_UNROLL2 1
#endif

template <int NW>
__global__ void __launch_bounds__(64 * NW, 2) attn16_d40_kernel(AttnArgs a) {
  constexpr int THREADS = 64 * NW;
  constexpr int QB = 32 * NW;
  // K row stride A16_KSTR (48; 56 -- a bank model's conflict-free choice -- measured 1.5 % slower
  // and with MORE LDS bank conflicts, profiles/r5_attn_d40_mixed_ab.jsonl), V rows of 48
  constexpr int KSTR = A16_KSTR;
  constexpr int KTILE = KT * KSTR;
  constexpr int BUF = KTILE + KT * A16_STR;   // K + V
  constexpr int CH = KT * A16_NCH;     // 16-B chunks per operand per tile
  constexpr int LD = (CH + THREADS - 1) / THREADS;
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;

  const int nqb = (a.Nq + QB - 1) / QB;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qblk = bid % nqb;
  const int bh = bid / nqb;
  const int h = bh % a.H;
  const int b = bh / a.H;
  const int q0 = qblk * QB + wave * 32;

  int nk = a.Nk;
  if (a.kv_lens) nk = min(nk, a.kv_lens[b]);
  const int ntiles = (nk + KT - 1) / KT;

  const uint16_t* Qp = a.q + (long long)b * a.q_sb + (long long)h * a.q_sh;
  const int hk = a.group > 1 ? h / a.group : h;
  const uint16_t* Kp = a.k + (long long)b * a.k_sb + (long long)hk * a.k_sh;
  const uint16_t* Vp = a.v + (long long)b * a.v_sb + (long long)hk * a.v_sh;

  // Q^T fragments of the two query blocks, pre-scaled by scale*log2(e) (S in log2 units).
  // k-step 0: d 0..31 (lane group g: d 8g..8g+7).  k-step 1: group 0 = d 32..39, group 1 = the
  // -m column (element 0) against K's constant chunk d 40..47, groups 2-3 zero (their K slots
  // re-read that chunk; a zero Q slot makes them inert).  Both steps are 16x16x32 MFMAs chained
  // on one accumulator: a 16x16x32 result fed straight into a 16x16x16 MFMA as its accumulator
  // came out wrong (the compiler placed no wait between the two shapes), and the 16x16x16 form
  // costs ~0.8 of a 16x16x32 on gfx950 (tools/mfma16_probe.hip), so it would save little anyway.
  const float qs = a.scale * 1.4426950408889634f;
  bf16x8_t qA[2], qB[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = q0 + 16 * qb + li;
    uint4 v = make_uint4(0, 0, 0, 0), w = make_uint4(0, 0, 0, 0);
    if (q < a.Nq) {
      v = *reinterpret_cast<const uint4*>(Qp + (long long)q * a.q_sn + 8 * g);
      if (g == 0) w = *reinterpret_cast<const uint4*>(Qp + (long long)q * a.q_sn + 32);
    }
    float f[8], e[8];
    unpack8(v, f);
    unpack8(w, e);
#pragma unroll
    for (int j = 0; j < 8; ++j) { f[j] *= qs; e[j] *= qs; }
    qA[qb] = as_bf16x8(pack8(f));
    qB[qb] = as_bf16x8(pack8(e));
  }

  // the constant column chunk (d 40 = 1.0, 41..47 = 0) of every row of both buffers' K and V
  for (int r = tid; r < 2 * 2 * KT; r += THREADS) {
    const int buf = r / (2 * KT), rr = r % (2 * KT);
    const int off = buf * BUF + (rr < KT ? rr * KSTR : KTILE + (rr - KT) * A16_STR);
    *reinterpret_cast<uint4*>(lds + off + 40) = make_uint4(0x3F80u, 0, 0, 0);
  }

  // staging: chunk c -> key c / 5, 16-B chunk c % 5 of d 0..39 (tile-invariant, decoded once)
  uint4 kr[LD], vr[LD];
  int c_key[LD], c_lds[LD], c_vlds[LD];
  long long c_ks[LD], c_vs[LD];
#pragma unroll
  for (int i = 0; i < LD; ++i) {
    const int c = tid + i * THREADS;
    const int key = c / A16_NCH, ch = c - key * A16_NCH;
    c_key[i] = c < CH ? key : (1 << 30);
    c_lds[i] = c < CH ? key * KSTR + ch * 8 : -1;
    c_vlds[i] = c < CH ? KTILE + key * A16_STR + ch * 8 : -1;
    c_ks[i] = (long long)key * a.k_sn + ch * 8;
    c_vs[i] = (long long)key * a.v_sn + ch * 8;
  }
  int c_kvo[LD], c_vvo[LD];                 // A16_BUFLD: byte voffsets (idle lanes out of range)
#pragma unroll
  for (int i = 0; i < LD; ++i) {
    const bool on = tid + i * THREADS < CH;
    c_kvo[i] = on ? (int)(c_ks[i] * 2) : (int)0x80000000;
    c_vvo[i] = on ? (int)(c_vs[i] * 2) : (int)0x80000000;
  }
  auto gload = [&](int t) {
    const int kbase = t * KT;
    const long long ko = (long long)kbase * a.k_sn, vo = (long long)kbase * a.v_sn;
    if constexpr (A16_BUFLD) {
      // wave-uniform resources: all scalar work; the range check covers voffset only
      const int left = nk - kbase;
      const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint16_t*>(Kp + ko), (short)0, (int)((long long)left * a.k_sn * 2), 0x00020000);
      const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint16_t*>(Vp + vo), (short)0, (int)((long long)left * a.v_sn * 2), 0x00020000);
#pragma unroll
      for (int i = 0; i < LD; ++i) {
        typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
        const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(rk, c_kvo[i], 0, 0);
        const u32x4_t y = __builtin_amdgcn_raw_buffer_load_b128(rv, c_vvo[i], 0, 0);
        kr[i] = make_uint4(x.x, x.y, x.z, x.w);
        vr[i] = make_uint4(y.x, y.y, y.z, y.w);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      uint4 x = make_uint4(0, 0, 0, 0), y = make_uint4(0, 0, 0, 0);
      if (kbase + c_key[i] < nk) {
        x = *reinterpret_cast<const uint4*>(Kp + ko + c_ks[i]);
        y = *reinterpret_cast<const uint4*>(Vp + vo + c_vs[i]);
      }
      kr[i] = x;
      vr[i] = y;
    }
  };
  auto lstore = [&](int bo) {
#pragma unroll
    for (int i = 0; i < LD; ++i)
      if (c_lds[i] >= 0) {
        *reinterpret_cast<uint4*>(lds + bo + c_lds[i]) = kr[i];
        *reinterpret_cast<uint4*>(lds + bo + c_vlds[i]) = vr[i];
      }
  };

  if (ntiles > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  if constexpr (NW == 8 && ATTN_PRIO) {
    if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  }

  f32x4_t oacc[3][2];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) oacc[i][qb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {0.f, 0.f};
  constexpr float RESCALE_THR = 8.f;
  // tr-read geometry: lane 4q'+p of a 16-lane group addresses row q', columns 4p..4p+3
  const int tr_off = (4 * g + (li >> 2)) * A16_STR + 4 * (li & 3);

  auto tile = [&](const int t, const int bo) {
    const bool more = t + 1 < ntiles;
    if (more) gload(t + 1);
    const uint16_t* Ks = lds + bo;
    const uint16_t* Vs = lds + bo + KTILE;

    // ---- S^T - m for 64 keys x 32 queries
    f32x4_t sacc[4][2];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const uint16_t* krow = Ks + (16 * kb + li) * KSTR;
      const bf16x8_t kA = as_bf16x8(*reinterpret_cast<const uint4*>(krow + 8 * g));
      const bf16x8_t kB = as_bf16x8(*reinterpret_cast<const uint4*>(krow + (g == 0 ? 32 : 40)));
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kA, qA[qb], z, 0, 0, 0);
        sacc[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kB, qB[qb], z, 0, 0, 0);
      }
    }
    const int kbase = t * KT;
    if (__builtin_expect(kbase + KT > nk, 0)) {
      // a real branch: without the volatile asm hipcc if-converts this block and pays its 16
      // compares + 32 v_cndmask on EVERY tile (round 6, ISA of attn16_d40_kernel<8>)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool bad = kbase + 16 * kb + 4 * g + r >= nk;
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
            if (bad) sacc[kb][qb][r] = -INFINITY;
        }
    }

    // ---- deferred-max online softmax (lane-local test, see above)
    float mx[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float m = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) m = fmaxf(m, sacc[kb][qb][r]);
      mx[qb] = m;
    }
    if (__builtin_expect(t == 0 || !__all(fmaxf(mx[0], mx[1]) <= RESCALE_THR), 0)) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        float m = fmaxf(mx[qb], __shfl_xor(mx[qb], 16, 64));
        const float2 hm = both_halves(m);
        m = fmaxf(hm.x, hm.y);
        float delta = (t == 0) ? m : fmaxf(m, 0.f);
        if (!(delta > -1e30f)) delta = 0.f;            // fully masked tile for this query
        const float mn = (float)(__bf16)(m_run[qb] + delta);   // an MFMA operand: keep it bf16-exact
        delta = mn - m_run[qb];
        m_run[qb] = mn;
        if (g == 1) qB[qb][0] = (__bf16)(-mn);
        const float alpha = __builtin_amdgcn_exp2f(-delta);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) oacc[i][qb][r] *= alpha;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) sacc[kb][qb][r] -= delta;
      }
    }
    // ---- P^T fragments: k-step s = key blocks 2s, 2s+1 of this lane's 4-key groups
    bf16x8_t pf[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        float p[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[r] = __builtin_amdgcn_exp2f(sacc[2 * s2][qb][r]);
          p[4 + r] = __builtin_amdgcn_exp2f(sacc[2 * s2 + 1][qb][r]);
        }
        pf[s2][qb] = as_bf16x8(pack8(p));
      }
    // ---- O^T += V^T P^T over 48 d rows
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int db = 0; db < 3; ++db) {
        const uint16_t* base = Vs + 32 * s2 * A16_STR + 16 * db + tr_off;
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(base));
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(base + 16 * A16_STR));
        typedef __attribute__((ext_vector_type(8))) short s16x8_t;
        s16x8_t vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8_t vf = __builtin_bit_cast(bf16x8_t, vv);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
          oacc[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[s2][qb], oacc[db][qb], 0, 0, 0);
      }
    // the other buffer was last read in tile t - 1, which every wave finished before the
    // previous barrier
    if (more) lstore(BUF - bo);
    __syncthreads();
  };
  if constexpr (A16_UNROLL2) {
    for (int t = 0; t < ntiles; t += 2) {
      tile(t, 0);
      if (t + 1 < ntiles) tile(t + 1, BUF);
    }
  } else {
    for (int t = 0; t < ntiles; ++t) tile(t, (t & 1) * BUF);
  }

  // ---- epilogue: O[q][d] = O^T[d][q] / l, l = O^T row 40 (lanes 32..47, register 0 of block 2)
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const float ls = __shfl(oacc[2][qb][0], 32 + li, 64);
    const int q = q0 + 16 * qb + li;
    if (q >= a.Nq) continue;
    const float inv = ls > 0.f ? 1.f / ls : 0.f;
    uint16_t* Op = a.o + (long long)b * a.o_sb + (long long)q * a.o_sn + (long long)h * a.o_sh;
#pragma unroll
    for (int db = 0; db < 3; ++db) {
      const int dd = 16 * db + 4 * g;
      if (dd < 40) {
        uint2 w;
        w.x = pack2(oacc[db][qb][0] * inv, oacc[db][qb][1] * inv);
        w.y = pack2(oacc[db][qb][2] * inv, oacc[db][qb][3] * inv);
        *reinterpret_cast<uint2*>(Op + dd) = w;
      }
    }
  }
}

template <int NW>
void launch_a16(const AttnArgs& a, hipStream_t s) {
  const int nqb = (a.Nq + 32 * NW - 1) / (32 * NW);
  hipLaunchKernelGGL((attn16_d40_kernel<NW>), dim3(nqb * a.H * a.B), dim3(64 * NW), 0, s, a);
}

template <int DQK, int DO, int NW>
void launch_t(const AttnArgs& a, hipStream_t s) {
  using G = AttnGeom<DQK, DO>;
  constexpr int QB = 32 * NW;
  int nqb = (a.Nq + QB - 1) / QB;
  dim3 grid(nqb * a.H * a.B);
  // K/V double-buffered in LDS (level-1 self-attention 247 -> 240 us, 568.7 -> 566.7 ms/step
  // same box x3, profiles/r2_attn_db_ab.txt; the single-buffer variant was removed in round 4)
  auto* kfn = &attn_fwd_kernel<DQK, DO, NW, true>;
  if constexpr (2 * G::LDS_BYTES > 65536) {
    // > 64 KiB dynamic LDS opt-in, once per process (thread-safe static init)
    static const bool once = [&] {
      (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * G::LDS_BYTES);
      return true;
    }();
    (void)once;
  }
  hipLaunchKernelGGL(kfn, grid, dim3(64 * NW), 2 * G::LDS_BYTES, s, a);
}

template <int DQK, int DO>
void launch_nw(const AttnArgs& a, hipStream_t s) {
  // enough workgroups to fill 256 CUs: fall back to fewer waves per block for short sequences
  long long blocks4 = (long long)((a.Nq + 127) / 128) * a.H * a.B;
  long long blocks8 = (long long)((a.Nq + 255) / 256) * a.H * a.B;
  // CASSMANTLE_ATTN_NW=4: never the 8-wave block (A/B knob: two 4-wave blocks per CU are not
  // lock-stepped by one block's per-tile barrier, at twice the K/V tile loads)
  static const int nw_cap = [] { const char* e = getenv("CASSMANTLE_ATTN_NW"); return e ? atoi(e) : 8; }();
  // 4-wave blocks from 512 of them, or -- UNet-sized sequences (>= 256 queries) -- from 16: at
  // batch 1 (levels 2 / 3 of SD-1.5: 128 / 32 four-wave blocks) the 4-wave block shares each K/V
  // tile over twice the queries and ran 9-15 % faster than twice as many 2-wave blocks
  // (profiles/r5_attn_nw4_batch1_ab.txt); text-encoder / scorer shapes keep the 512 rule.
  // CASSMANTLE_ATTN_NW4_MIN overrides the 16 (A/B knob)
  static const int nw4_min = [] { const char* e = getenv("CASSMANTLE_ATTN_NW4_MIN"); return e ? atoi(e) : 16; }();
  if (DO <= 96 && blocks8 >= 1024 && nw_cap >= 8) launch_t<DQK, DO, 8>(a, s);   // 8 waves share each K/V tile
  else if (blocks4 >= 512 || (a.Nq >= 256 && blocks4 >= nw4_min)) launch_t<DQK, DO, 4>(a, s);
  else launch_t<DQK, DO, 2>(a, s);
}

// ================================================================================ fp8 (OCP e4m3)
// BASELINE config 4 (SDXL, head dim 64): both attention GEMMs on the block-scaled fp8 MFMA
// v_mfma_scale_f32_32x32x64_f8f6f4 (scales fixed at 2^0), which does a 32x32 tile over 64 head
// dims / 64 keys in ONE instruction at twice the bf16 rate:
//   S^T = K8 . Q8^T       A = 32 key rows x 64 d (32 B per lane from LDS), B = Q8 in registers
//   O^T += V8^T . P8^T    B = P^T from the S accumulator (fp8 packed, k order = accumulator order)
//                         A = V^T rows from a pre-transposed fp8 V whose 64-key blocks are stored
//                             in exactly that k order, so the A fragment is 32 contiguous bytes.
// K and V are packed once per call by attn_fp8_pack_kernel (K8 [B,Hk,Nkp,64], V8t [B,Hk,64,Nkp],
// Nkp = keys rounded up to 64, zero padded); Q is quantised in registers after the
// scale*log2(e) prescale.  P <= 2^RESCALE_THR (deferred max) stays inside e4m3's range.
// Element j (0..31) of lane half h of a 32x32x64 operand is paired with the same (h, j) of the
// other operand, so only the P <-> V^T correspondence has to be fixed: slot 32h + j of a key
// block holds key kappa(h, j) = 32(j>>4) + (j&3) + 8((j&15)>>2) + 4h, the key of S accumulator
// register j&15 of key-half j>>4 in lane half h.
#ifndef F8_VEARLY
#define F8_VEARLY 1
#endif
// F8_PIPE (two-stage blocks): the P.V MFMAs of tile t are issued in the NEXT step, right after
// tile t+1's S MFMAs, so they fill the S latency and tile t+1's softmax runs while they retire
// (P and the V fragments of tile t are carried across the step's barrier in registers).
// Measured 4 % SLOWER on the SDXL self-attention (80.3 -> 83.8 us at 4096 keys, same box,
// profiles/r6_fp8_pipe_negative.txt): off; kept selectable for A/B builds
#ifndef F8_PIPE
#define F8_PIPE 0
#endif
constexpr int F8_KSTR = 80;   // LDS row stride (bytes) of the 64-byte fp8 rows: 16-lane groups
                              // of ds_read_b128 hit disjoint banks (20 r mod 64 distinct)

// (f8x4 / f8_slot: common.h, shared with the GEMM epilogues that emit this image directly)

// one block per (64-key tile, kv head, batch): K rows convert straight to K8 (8 B per thread,
// 64-B rows); V goes through a 64 x 64-byte LDS image in the V8t slot order and leaves as
// 64-byte d-rows (16 B per thread).  The round-1 version wrote V8t one BYTE per store (13.4 us
// for 2 x 4096 x 10 heads; profiles/r2_attn_fp8_kernel_trace.txt)
__global__ void __launch_bounds__(256) attn_fp8_pack_kernel(AttnArgs a, int Hk, int Nkp, uint8_t* __restrict__ K8,
                                                            uint8_t* __restrict__ V8t) {
  __shared__ __attribute__((aligned(16))) uint8_t vt[64][64 + 16];
  const int kb = blockIdx.x * 64, hh = blockIdx.y, b = blockIdx.z;
  int nk = a.Nk;
  if (a.kv_lens) nk = min(nk, a.kv_lens[b]);
  const long long bh = (long long)b * Hk + hh;
  const uint16_t* Kp = a.k + (long long)b * a.k_sb + (long long)hh * a.k_sh;
  const uint16_t* Vp = a.v + (long long)b * a.v_sb + (long long)hh * a.v_sh;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = threadIdx.x + 256 * it;          // 512 chunks = 64 keys x 8 chunks of 8 d
    const int kk = c >> 3, ch = c & 7;
    const int key = kb + kk;
    uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (key < nk && ch * 8 < a.d) {
      kv = *reinterpret_cast<const uint4*>(Kp + (long long)key * a.k_sn + ch * 8);
      vv = *reinterpret_cast<const uint4*>(Vp + (long long)key * a.v_sn + ch * 8);
    }
    float kf[8], vf[8];
    unpack8(kv, kf);
    unpack8(vv, vf);
    *reinterpret_cast<uint2*>(K8 + (bh * Nkp + key) * 64 + ch * 8) =
        make_uint2(f8x4(kf[0], kf[1], kf[2], kf[3]), f8x4(kf[4], kf[5], kf[6], kf[7]));
    const uint32_t v0 = f8x4(vf[0], vf[1], vf[2], vf[3]), v1 = f8x4(vf[4], vf[5], vf[6], vf[7]);
    const int slot = f8_slot(kk);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      vt[ch * 8 + e][slot] = (uint8_t)(v0 >> (8 * e));
      vt[ch * 8 + e + 4][slot] = (uint8_t)(v1 >> (8 * e));
    }
  }
  __syncthreads();
  const int dr = threadIdx.x >> 2, seg = threadIdx.x & 3;
  *reinterpret_cast<uint4*>(V8t + (bh * 64 + dr) * Nkp + kb + seg * 16) = *reinterpret_cast<const uint4*>(&vt[dr][seg * 16]);
}

typedef __attribute__((ext_vector_type(8))) int i32x8_t;

// Block = NQ query groups (32 queries each, one wave per group and key split) x NS key splits.
// Wave (qg, ks) runs tiles ks, ks + NS, ks + 2 NS, ... of its group's keys, so each step stages
// NS consecutive K/V tiles in LDS, each shared by the NQ waves of one split; at the end the
// splits' partial (O, m, l) are merged through LDS by the ks = 0 wave.  NS > 1 is for the short
// grids of SDXL (1024 queries x 20 heads x 2 CFG images = 1280 query groups for 1024 SIMDs: with
// one split every wave walks all 16 key tiles at one wave per SIMD, a latency-bound chain);
// splitting the keys multiplies the waves and divides the chain without a second kernel.
// staging of one step's K/V tiles through registers: chunk slot I (0..3) of this thread as
// plain variables (an array here was put in scratch memory by hipcc once LD > 1)
#define F8_GSLOT(I, ST, KR, VR)                                                                  \
  if constexpr (I < LD) {                                                                        \
    const int c = tid + I * THREADS;                                                             \
    if (c < CH) {                                                                                \
      const int tt = c / (KT * 4), row = (c >> 2) % KT, cc = c & 3;                              \
      const int t_ = (ST) * NS + tt;                                                             \
      if (t_ < ntiles) {                                                                         \
        KR = *reinterpret_cast<const uint4*>(Kg + (long long)(t_ * KT + row) * 64 + cc * 16);    \
        VR = *reinterpret_cast<const uint4*>(Vg + (long long)row * Nkp + t_ * KT + cc * 16);     \
      }                                                                                          \
    }                                                                                            \
  }
#define F8_LSLOT(I, KR, VR)                                                                      \
  if constexpr (I < LD) {                                                                        \
    const int c = tid + I * THREADS;                                                             \
    if (c < CH) {                                                                                \
      const int tt = c / (KT * 4), row = (c >> 2) % KT, cc = c & 3;                              \
      *reinterpret_cast<uint4*>(Ks + tt * TILE_B + row * F8_KSTR + cc * 16) = KR;                \
      *reinterpret_cast<uint4*>(Vs + tt * TILE_B + row * F8_KSTR + cc * 16) = VR;                \
    }                                                                                            \
  }
#define F8_GLOAD(ST) \
  F8_GSLOT(0, ST, kr0, vr0) F8_GSLOT(1, ST, kr1, vr1) F8_GSLOT(2, ST, kr2, vr2) F8_GSLOT(3, ST, kr3, vr3)
#define F8_LSTORE() F8_LSLOT(0, kr0, vr0) F8_LSLOT(1, kr1, vr1) F8_LSLOT(2, kr2, vr2) F8_LSLOT(3, kr3, vr3)

// DB: two LDS stages.  The next step's K/V (already in registers) go to the other stage right
// after this step's MFMAs, so a step ends with ONE barrier instead of barrier + store + barrier
// (the stage written in step st was last read in step st - 1, which every wave has left).
template <int NQ, int NS, bool DB>
__global__ void __launch_bounds__(64 * NQ * NS, (NQ * NS >= 4) ? 8 / (NQ * NS) > 0 ? 8 / (NQ * NS) : 1 : 2)
attn_fp8_kernel(AttnArgs a, int Hk, int Nkp, const uint8_t* __restrict__ K8, const uint8_t* __restrict__ V8t) {
  constexpr int NWV = NQ * NS;
  constexpr int THREADS = 64 * NWV;
  constexpr int QB = 32 * NQ;
  constexpr int TILE_B = KT * F8_KSTR;   // one 64-row fp8 tile in LDS
  constexpr int STAGE_B = 2 * NS * TILE_B;
  constexpr int MREC = 34;               // merge record per lane: 32 O registers, m, l
  constexpr int MERGE_B = (NS - 1) * NQ * 64 * MREC * 4;
  constexpr int STAGES_B = (DB ? 2 : 1) * STAGE_B;
  constexpr int LDS_B = STAGES_B > MERGE_B ? STAGES_B : MERGE_B;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_B];
  uint8_t* Ks = lds;                       // the stage F8_LSTORE writes
  uint8_t* Vs = lds + NS * TILE_B;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qg = wave % NQ, ks = wave / NQ;
  const int hlf = lane >> 5, ql = lane & 31;
  const int nqb = (a.Nq + QB - 1) / QB;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb, bh = bid / nqb;
  const int h = bh % a.H, b = bh / a.H;
  const int hk = a.group > 1 ? h / a.group : h;
  const int q0 = qb * QB + qg * 32, q = q0 + ql;

  int nk = a.Nk;
  if (a.kv_lens) nk = min(nk, a.kv_lens[b]);
  int ntiles = (nk + KT - 1) / KT;
  if (a.causal) ntiles = min(ntiles, (qb * QB + QB + KT - 1) / KT);
  const int nsteps = (ntiles + NS - 1) / NS;

  // Q8 fragment: lane holds Q[q][32*hlf .. +31] * scale*log2e as e4m3
  i32x8_t qf;
  {
    const uint16_t* Qp = a.q + (long long)b * a.q_sb + (long long)h * a.q_sh + (long long)q * a.q_sn + 32 * hlf;
    const float sc = a.scale * 1.4426950408889634f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (q < a.Nq) v = *reinterpret_cast<const uint4*>(Qp + 8 * c);
      float f[8];
      unpack8(v, f);
      qf[2 * c] = (int)f8x4(f[0] * sc, f[1] * sc, f[2] * sc, f[3] * sc);
      qf[2 * c + 1] = (int)f8x4(f[4] * sc, f[5] * sc, f[6] * sc, f[7] * sc);
    }
  }
  const uint8_t* Kg = K8 + ((long long)b * Hk + hk) * Nkp * 64;
  const uint8_t* Vg = V8t + ((long long)b * Hk + hk) * 64 * Nkp;
  // staging: per step NS tiles x 256 16-byte chunks per operand (row = chunk >> 2, 4 per row)
  constexpr int CH = NS * KT * 4;
  constexpr int LD = (CH + THREADS - 1) / THREADS;
  static_assert(LD <= 4, "fp8 attention staging: at most 4 chunks per thread");
  uint4 kr0 = {}, kr1 = {}, kr2 = {}, kr3 = {}, vr0 = {}, vr1 = {}, vr2 = {}, vr3 = {};
  if (nsteps > 0) { F8_GLOAD(0) F8_LSTORE() }
  __syncthreads();

  f32x16_t oacc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  float m_run = 0.f, l_run = 0.f;
  constexpr float RESCALE_THR = 8.f;
  // F8_ONES_SUM: the row sums of P come from one more MFMA per tile against an all-ones e4m3 A
  // operand (every row of lsum = the query's sum over the tile's 64 keys, of the same fp8 P the
  // P.V MFMAs use) instead of 32 VALU adds + a cross-half shuffle per tile.  Key-split variants
  // only (the self-attention shapes): on the NS = 1 blocks (77-key cross-attention, 2 tiles) its
  // 16 accumulator registers would cost a wave per SIMD (117 -> 132 registers)
  constexpr bool ONES = F8_ONES_SUM && NS > 1;
  f32x16_t lsum;
#pragma unroll
  for (int r = 0; r < 16; ++r) lsum[r] = 0.f;
  const i32x8_t ones8 = {0x38383838, 0x38383838, 0x38383838, 0x38383838,
                         0x38383838, 0x38383838, 0x38383838, 0x38383838};   // e4m3 1.0
  constexpr bool PIPE = F8_PIPE && DB && F8_VEARLY;
  i32x8_t pf_prev, vf_prev[2];             // PIPE: the previous tile's P and V fragments
  bool pend = false;
  auto pv_mfmas = [&](const i32x8_t& p8, const i32x8_t* v8) {
#pragma unroll
    for (int dc = 0; dc < 2; ++dc)
      oacc[dc] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(v8[dc], p8, oacc[dc], 0, 0, 0, 127, 0, 127);
    if constexpr (ONES)
      lsum = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ones8, p8, lsum, 0, 0, 0, 127, 0, 127);
  };
  for (int st = 0; st < nsteps; ++st) {
    const bool more = st + 1 < nsteps;
    if (more) { F8_GLOAD(st + 1) }
    const int cur = DB ? (st & 1) * STAGE_B : 0;   // the stage this step reads
    const uint8_t* const Kw = lds + cur + ks * TILE_B;
    const uint8_t* const Vw = lds + cur + NS * TILE_B + ks * TILE_B;
    const int t = st * NS + ks;
    if (PIPE && !(t < ntiles) && pend) {   // this split's last tile was the previous one
      pv_mfmas(pf_prev, vf_prev);
      pend = false;
    }
    if (t < ntiles) {                      // wave-uniform: the last step may not reach every split
      f32x16_t sacc[2];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[hf][r] = -m_run;
        const uint8_t* kp = Kw + (hf * 32 + ql) * F8_KSTR + 32 * hlf;
        const uint4 k0 = *reinterpret_cast<const uint4*>(kp);
        const uint4 k1 = *reinterpret_cast<const uint4*>(kp + 16);
        const i32x8_t kf = {(int)k0.x, (int)k0.y, (int)k0.z, (int)k0.w, (int)k1.x, (int)k1.y, (int)k1.z, (int)k1.w};
        sacc[hf] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kf, qf, sacc[hf], 0, 0, 0, 127, 0, 127);
      }
      // V fragments of this tile issued now (F8_VEARLY): their LDS latency hides behind the softmax
      i32x8_t vfe[2];
      if constexpr (F8_VEARLY) {
#pragma unroll
        for (int dc = 0; dc < 2; ++dc) {
          const uint8_t* vp = Vw + (dc * 32 + ql) * F8_KSTR + 32 * hlf;
          const uint4 v0 = *reinterpret_cast<const uint4*>(vp);
          const uint4 v1 = *reinterpret_cast<const uint4*>(vp + 16);
          vfe[dc] = i32x8_t{(int)v0.x, (int)v0.y, (int)v0.z, (int)v0.w, (int)v1.x, (int)v1.y, (int)v1.z, (int)v1.w};
        }
      }
      if constexpr (PIPE) {                // the previous tile's P.V behind this tile's S MFMAs
        if (pend) pv_mfmas(pf_prev, vf_prev);
        pend = false;
      }
      const int kbase = t * KT;
      const bool need_mask = (kbase + KT > nk) || (a.causal && kbase + KT - 1 > q0);
      if (__builtin_expect(need_mask, 0)) {
        // a real branch (see attn16_d40_kernel): if-converted, this mask cost ~130 VALU + 66 SALU
        // per 64-key tile on unmasked tiles, more than the softmax itself (round 6 ISA count)
        asm volatile("" ::: "memory");
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kbase + hf * 32 + (r & 3) + 8 * (r >> 2) + 4 * hlf;
            if (key >= nk || (a.causal && key > q)) sacc[hf][r] = -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[hf][r]);
      if constexpr (ATTN_PERMLANE) {    // cross-half max by v_permlane32_swap, not ds_bpermute
        const float2 hm = both_halves(mx);
        mx = fmaxf(hm.x, hm.y);
      } else {
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      }
      if (__builtin_expect(st == 0 || !__all(mx <= RESCALE_THR), 0)) {
        // a real branch: without the volatile asm hipcc if-converts this block and rescales O
        // and S by alpha = 1 on EVERY tile (a v_pk_mul per two O registers per tile)
        asm volatile("" ::: "memory");
        float delta = (st == 0) ? mx : fmaxf(mx, 0.f);
        if (!(delta > -1e30f)) delta = 0.f;
        m_run += delta;
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        l_run *= alpha;
        if constexpr (ONES) {
#pragma unroll
          for (int r = 0; r < 16; ++r) lsum[r] *= alpha;
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) oacc[i][r] *= alpha;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc[hf][r] -= delta;
      }
      if constexpr (ONES) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc[hf][r] = __builtin_amdgcn_exp2f(sacc[hf][r]);
      } else {
        float rs = 0.f;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float pv = __builtin_amdgcn_exp2f(sacc[hf][r]);
            sacc[hf][r] = pv;
            rs += pv;
          }
        if constexpr (ATTN_PERMLANE) {
          const float2 hs = both_halves(rs);
          rs = hs.x + hs.y;
        } else {
          rs += __shfl_xor(rs, 32, 64);
        }
        l_run += rs;
      }
      // P^T fragment: element j = sacc[j >> 4][j & 15]
      i32x8_t pf;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          pf[4 * hf + c] = (int)f8x4(sacc[hf][4 * c], sacc[hf][4 * c + 1], sacc[hf][4 * c + 2], sacc[hf][4 * c + 3]);
      if constexpr (PIPE) {
        pf_prev = pf;
        vf_prev[0] = vfe[0];
        vf_prev[1] = vfe[1];
        pend = true;
      } else {
#pragma unroll
        for (int dc = 0; dc < 2; ++dc) {
          i32x8_t vf;
          if constexpr (F8_VEARLY) {
            vf = vfe[dc];
          } else {
            const uint8_t* vp = Vw + (dc * 32 + ql) * F8_KSTR + 32 * hlf;
            const uint4 v0 = *reinterpret_cast<const uint4*>(vp);
            const uint4 v1 = *reinterpret_cast<const uint4*>(vp + 16);
            vf = i32x8_t{(int)v0.x, (int)v0.y, (int)v0.z, (int)v0.w, (int)v1.x, (int)v1.y, (int)v1.z, (int)v1.w};
          }
          oacc[dc] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf, pf, oacc[dc], 0, 0, 0, 127, 0, 127);
        }
        if constexpr (ONES)
          lsum = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ones8, pf, lsum, 0, 0, 0, 127, 0, 127);
      }
    }
    if constexpr (DB) {
      if (more) {
        Ks = lds + (cur ^ STAGE_B);
        Vs = Ks + NS * TILE_B;
        F8_LSTORE()
      }
      __syncthreads();
    } else {
      __syncthreads();
      if (more) {
        F8_LSTORE()
        __syncthreads();
      }
    }
  }
  if (PIPE && pend) pv_mfmas(pf_prev, vf_prev);   // the last tile's P.V
  if constexpr (ONES) l_run = lsum[0];
  if constexpr (NS > 1) {
    // merge the key splits: every wave is past the loop's last barrier, so the staging LDS is
    // free; splits 1.. publish (O, m, l) per lane (lane-contiguous records: no bank conflicts)
    float* const mg = reinterpret_cast<float*>(lds);
    if (ks > 0) {
      float* dst = mg + ((ks - 1) * NQ + qg) * 64 * MREC;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dst[r * 64 + lane] = oacc[0][r];
        dst[(16 + r) * 64 + lane] = oacc[1][r];
      }
      dst[32 * 64 + lane] = m_run;
      dst[33 * 64 + lane] = l_run;
    }
    __syncthreads();
    if (ks > 0) return;                    // no barrier follows
    // an empty split (no tile reached it, or every key masked) has l = 0 and takes no part
    float mm = l_run > 0.f ? m_run : -INFINITY;
#pragma unroll
    for (int j = 1; j < NS; ++j) {
      const float* src = mg + ((j - 1) * NQ + qg) * 64 * MREC;
      if (src[33 * 64 + lane] > 0.f) mm = fmaxf(mm, src[32 * 64 + lane]);
    }
    if (mm > -INFINITY) {
      const float a0 = l_run > 0.f ? __builtin_amdgcn_exp2f(m_run - mm) : 0.f;
      l_run *= a0;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[i][r] *= a0;
#pragma unroll
      for (int j = 1; j < NS; ++j) {
        const float* src = mg + ((j - 1) * NQ + qg) * 64 * MREC;
        const float lj = src[33 * 64 + lane];
        const float aj = lj > 0.f ? __builtin_amdgcn_exp2f(src[32 * 64 + lane] - mm) : 0.f;
        l_run = fmaf(aj, lj, l_run);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          oacc[0][r] = fmaf(aj, src[r * 64 + lane], oacc[0][r]);
          oacc[1][r] = fmaf(aj, src[(16 + r) * 64 + lane], oacc[1][r]);
        }
      }
    }
  }
  if (q < a.Nq) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    uint16_t* Op = a.o + (long long)b * a.o_sb + (long long)q * a.o_sn + (long long)h * a.o_sh;
#pragma unroll
    for (int dc = 0; dc < 2; ++dc)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int dd = 32 * dc + 8 * g4 + 4 * hlf;
        uint2 w;
        w.x = pack2(oacc[dc][4 * g4 + 0] * inv, oacc[dc][4 * g4 + 1] * inv);
        w.y = pack2(oacc[dc][4 * g4 + 2] * inv, oacc[dc][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(Op + dd) = w;
      }
  }
}

template <int NQ, int NS>
void launch_fp8_t(const AttnArgs& a, int Hk, int Nkp, const uint8_t* K8, const uint8_t* V8t, hipStream_t s) {
  const int nqb = (a.Nq + 32 * NQ - 1) / (32 * NQ);
  // two LDS stages on the 2-split blocks unless CASSMANTLE_FP8_DBUF=0 (A/B knob; =2 forces every
  // variant).  Same box (profiles/r5_fp8_attn_dbuf_ab.txt): 2x2 self-attention 1.0-1.6 % faster,
  // 4x2 3-5 %; the one-step cross-attention blocks (NS 1) +1 %, the 80 KB 1x4 stages 12-30 % slower
  static const int dbuf = [] { const char* e = getenv("CASSMANTLE_FP8_DBUF"); return e ? atoi(e) : 1; }();
  if (dbuf == 2 || (dbuf == 1 && NS == 2))
    hipLaunchKernelGGL((attn_fp8_kernel<NQ, NS, true>), dim3(nqb * a.H * a.B), dim3(64 * NQ * NS), 0, s, a, Hk, Nkp, K8, V8t);
  else
    hipLaunchKernelGGL((attn_fp8_kernel<NQ, NS, false>), dim3(nqb * a.H * a.B), dim3(64 * NQ * NS), 0, s, a, Hk, Nkp, K8, V8t);
}

}  // namespace

long long attention_fp8_workspace(const AttnArgs& a, int Hk) {
  const long long Nkp = (a.Nk + KT - 1) / KT * KT;
  return 2LL * a.B * Hk * Nkp * 64;   // bytes: K8 + V8t
}

void launch_attention_fp8_pack(const AttnArgs& a, int Hk, uint8_t* ws, hipStream_t s) {
  const int Nkp = (a.Nk + KT - 1) / KT * KT;
  hipLaunchKernelGGL(attn_fp8_pack_kernel, dim3((unsigned)(Nkp / 64), (unsigned)Hk, (unsigned)a.B), dim3(256), 0, s, a, Hk,
                     Nkp, ws, ws + (long long)a.B * Hk * Nkp * 64);
}

// forced fp8 variant NQ*10 + NS (0: the shape rule); set by ops.set_fp8_attention_variant
static std::atomic<int> g_fp8_attn_variant{0};   // A/B knob, read by every launch thread
void set_fp8_attn_variant(int v) { g_fp8_attn_variant = v; }

void launch_attention_fp8(const AttnArgs& a, int Hk, uint8_t* ws, hipStream_t s, bool packed) {
  const int Nkp = (a.Nk + KT - 1) / KT * KT;
  uint8_t* K8 = ws;
  uint8_t* V8t = ws + (long long)a.B * Hk * Nkp * 64;
  if (!packed) launch_attention_fp8_pack(a, Hk, ws, s);
  // query groups of 32 over the chip's 1024 SIMDs: short grids split the keys too (NS), so
  // every SIMD gets several waves.  CASSMANTLE_FP8_ATTN="NQxNS" forces a variant (A/B knob).
  static const int env_forced = [] {
    const char* e = getenv("CASSMANTLE_FP8_ATTN");
    if (!e) return 0;
    int nq = 0, ns = 0;
    return sscanf(e, "%dx%d", &nq, &ns) == 2 ? nq * 10 + ns : 0;
  }();
  const int fv = g_fp8_attn_variant.load(std::memory_order_relaxed);
  const int forced = fv > 0 ? fv : env_forced;
  const long long groups = (long long)((a.Nq + 31) / 32) * a.H * a.B;
  const int nkt = (a.Nk + KT - 1) / KT;
  int v = forced;
  // measured (tools/bench_attn_fp8.py, profiles/r3_attn_fp8_variants.jsonl): 2 query groups x
  // 2 key splits is fastest at both SDXL self-attention shapes (1024 keys x 20 heads: 19.2 us vs
  // 21.5 for 4x1; 4096 x 10: 84.5 vs 89.4); the 77-key cross-attention (2 tiles) keeps 4x1
  if (v == 0) v = groups >= 8192 ? 81 : (nkt < 4 ? 41 : 22);
  switch (v) {
    case 81: return launch_fp8_t<8, 1>(a, Hk, Nkp, K8, V8t, s);
    case 41: return launch_fp8_t<4, 1>(a, Hk, Nkp, K8, V8t, s);
    case 22: return launch_fp8_t<2, 2>(a, Hk, Nkp, K8, V8t, s);
    case 42: return launch_fp8_t<4, 2>(a, Hk, Nkp, K8, V8t, s);
    case 14: return launch_fp8_t<1, 4>(a, Hk, Nkp, K8, V8t, s);
    case 24: return launch_fp8_t<2, 4>(a, Hk, Nkp, K8, V8t, s);
    default: return launch_fp8_t<4, 1>(a, Hk, Nkp, K8, V8t, s);
  }
}

// d = 40 kernel: 1 = 16x16-block kernel, 0 = the 32x32x16 kernel, -1 = CASSMANTLE_ATTN16 (default 1)
static std::atomic<int> g_attn_d40_variant{-1};   // A/B knob, read by every launch thread
void set_attn_d40_variant(int v) { g_attn_d40_variant = v; }

void launch_attention(const AttnArgs& a, hipStream_t s) {
  switch (a.d) {
    case 32: launch_nw<32, 32>(a, s); break;
    case 40: {
      // 16x16-block kernel (round 5) unless CASSMANTLE_ATTN16=0 (A/B knob) or causal masking
      static const int a16_env = [] { const char* e = getenv("CASSMANTLE_ATTN16"); return e ? atoi(e) : 1; }();
      const int dv = g_attn_d40_variant.load(std::memory_order_relaxed);
      const int a16 = dv >= 0 ? dv : a16_env;
      const long long blocks8 = (long long)((a.Nq + 255) / 256) * a.H * a.B;
      // (variant 2, the mixed 32x32 QK^T / 16x16 P.V kernel, is archived: tools/archive/attn_mx_d40.hip.txt)
      // (the 16x16 kernel's per-tile buffer resources address a (batch, head)'s keys with 32-bit
      // byte counts: spans of 2 GiB or more take the 32x32 kernel)
      const bool span_ok = (long long)a.Nk * a.k_sn * 2 < (1LL << 31) && (long long)a.Nk * a.v_sn * 2 < (1LL << 31);
      if (a16 && !a.causal && (span_ok || !A16_BUFLD)) {
        // 8-wave blocks from 256 of them: the 4-wave build takes 130 registers (3 waves per SIMD),
        // and at batch 1 (B = 2, 256 eight-wave blocks) the 8-wave block is 10 % faster
        // (profiles/r5_attn_d40_nw8_batch1_ab.txt).  CASSMANTLE_ATTN16_NW8_MIN overrides (A/B knob)
        static const int nw8_min = [] { const char* e = getenv("CASSMANTLE_ATTN16_NW8_MIN"); return e ? atoi(e) : 256; }();
        if (blocks8 >= nw8_min) launch_a16<8>(a, s);
        else launch_a16<4>(a, s);
      } else {
        launch_nw<48, 64>(a, s);
      }
      break;
    }
    case 64: launch_nw<64, 64>(a, s); break;
    case 80: launch_nw<80, 96>(a, s); break;
    case 128: launch_nw<128, 128>(a, s); break;
    case 160: launch_nw<160, 160>(a, s); break;
    default: {
      // generic: round up (d must be a multiple of 8, <= 256)
      if (a.d <= 32) launch_nw<32, 32>(a, s);
      else if (a.d <= 64) launch_nw<64, 64>(a, s);
      else if (a.d <= 96) launch_nw<96, 96>(a, s);
      else if (a.d <= 128) launch_nw<128, 128>(a, s);
      else if (a.d <= 160) launch_nw<160, 160>(a, s);
      // d > 160 never reaches this kernel: ops.attention routes it to the GEMM path
    }
  }
}
