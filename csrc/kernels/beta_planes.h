// Fused beta-divergence MU on the bf16 matrix cores, fp32-accurate through split operands
// (gfx950 / CDNA4), replicate-batched.  The hot loop of online/batch KL and IS NMF
// (sklearn/decomposition/_nmf.py:526-728 is the math nmf-torch
// runs as three eager ops per MU step: h@W, x/(hW), (.)@W^T).
//
// One workgroup owns one replicate and a strip of "fixed-axis" columns (cells on the
// usage side H, genes on the spectra side W) and streams the other factor -- the
// "streamed" operand, reduced over -- through LDS in chunks of 64 rows:
//
//   P   = S^T F + eps            (Ls x cols, never in memory: two 16 x 16 accumulator tiles
//                                 per 32 streamed rows and 16 columns)
//   Q   = X * P^(beta-2)         D = P^(beta-1)                      (VALU, registers)
//   num = S Q   (K x cols)       den = S D   (beta != 1; KL: den = S 1, a host vector)
//
// H side: S = W (K x G), F = H^T, X as stored (cells x genes); W side: S = H^T of the
// chunk, F = W, X^T.  Both products run on v_mfma_f32_16x16x32_bf16:
//
// * P is EXACT to fp32 rounding: every fp32 value v splits into three bf16 planes
//   v = v0 + v1 + v2 (each residual exact), and the six plane products with i + j <= 2,
//   {S0F0, S0F1, S1F0, S0F2, S1F1, S2F0}, are packed along the 32-deep MFMA reduction:
//   slot s = t*K + k of term t, so K <= 10 costs two MFMAs per 16 x 16 tile (fp32 MFMA:
//   three of twice the cycles).  The S planes come pre-arranged ("panels", built once per
//   factor update by bp_panel_kernel), the F planes are built in registers once per step.
// * num = S Q: the P accumulator of lane (q, m) holds streamed rows 4q+i (+16) of column
//   m -- exactly the B-operand fragment of a 32-deep product over those rows, so Q goes
//   from the accumulator through the VALU straight into the next MFMA, no lane movement
//   (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand"); the
//   S panel stores its columns in the matching permuted order.  Q splits into two bf16
//   planes in registers (v_cvt_pk_bf16_f32), S into two: S0Q0 + S0Q1 + S1Q0 leaves
//   <= 3 * 2^-16 relative per term, with random sign -- inside the fp32 accumulation
//   error of the 2000-long reduction (the split-GEMM argument of gemm_planes.hip).
//
// KL (the reference CLI's common non-Frobenius loss) runs a cheaper variant of both
// products, since its VALU work per element (rcp, mul, split) bounds the kernel, not the MFMAs:
// * P from the three plane products {S0F0, S0F1, S1F0} only (relative error <= ~3 * 2^-16,
//   far below the Q rounding below): 3K slots, so K <= 10 costs ONE MFMA per tile.
// * Q = X / P goes into ONE fp16 plane (v_cvt_pk_f16_f32: half an instruction per element
//   instead of the two-plane split's three), S into two fp16 planes scaled per row k by a
//   power of two 2^-e_k (its max -> [0.5, 1): bp_rowscale_kernel), num = S0 Q + S1 Q on
//   v_mfma_f32_16x16x32_f16.  Per term the error is <= 2^-11 relative (random sign):
//   simulated over 200 batch KL MU iterations (2000 x 2000, K = 10) the factors drift
//   1.8e-5 relative from an fp32 run and the objective 1e-8 (tests/test_kernels_gpu.py
//   pins the online solver against the fp32 torch path).  fp16 has a narrower range than fp32:
//   Q is computed as x / (2^s P) with a per-column shift s (F's planes and eps scaled
//   by 2^s, exactly), s = 0 to start with (x / P stays below ~200 on count data), and a
//   step whose numerator comes out non-finite for some column is redone with that
//   column's s raised by 12 (at most 6 times), so overflow never reaches the result.
//
// The H-side kernel runs `nsteps` MU steps per launch: every workgroup's cells only
// depend on their own usages and on W, so the steps need no cross-workgroup
// synchronisation; the updated usages go back into the B-operand planes through a small
// per-wave LDS exchange.  The block-objective stopping rule (beta-divergence of the chunk
// every `nsteps` steps) is decided by the last-arriving workgroup of the replicate.  One
// launch thus replaces `check_every` launches of the first-generation kernel
// (beta_mu.hip), and the loss is only evaluated where the rule reads it.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace cnmf {

typedef short bp_v8 __attribute__((ext_vector_type(8)));
typedef __bf16 bp_b8 __attribute__((ext_vector_type(8)));
typedef _Float16 bp_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 bp_h4 __attribute__((ext_vector_type(4)));
typedef float bp_f4 __attribute__((ext_vector_type(4)));
typedef unsigned int bp_u4 __attribute__((ext_vector_type(4)));

constexpr int kBpCH = 64;          // streamed rows per panel chunk (two 32-row blocks)
constexpr int kBpWaves = 4;        // waves per workgroup
constexpr int kBpThreads = 64 * kBpWaves;
// N-panel row stride (bf16 elements): 160-B rows put the 16 lanes of every ds_read_b128
// lane group on 16 distinct 4-bank slots (144-B rows: 2-way conflicts on most groups;
// MI355X_MICROARCH.md §LDS lane groups, profiles/r3k_pmc_beta_kl_fp16.txt
// SQ_LDS_BANK_CONFLICT 1.3x the LDS-active cycles)
constexpr int kBpNS = kBpCH + 16;

// kBpKLX: KL with the fp32-accurate numerator (the default KL mode): P from KL's three
// plane products, Q = X / P split into two bf16 planes and S into two (num = S0 Q0 +
// S0 Q1 + S1 Q0, <= 3 * 2^-16 relative per term with random sign -- inside the fp32
// accumulation error of the reduction, as for IS / general beta), den = S 1 a host vector
// as for KL.  kBpKL is the opt-in fp16 numerator (CNMF_KL_FP16=1, see the file comment).
enum BpMode { kBpKL = 0, kBpIS = 1, kBpGeneral = 2, kBpKLX = 3 };

__host__ __device__ constexpr bool bp_is_kl(int mode) { return mode == kBpKL || mode == kBpKLX; }

// plane-product terms of P: KL 3, IS / general beta 6 (exact to fp32 rounding)
__host__ __device__ constexpr int bp_nt(int mode) { return bp_is_kl(mode) ? 3 : 6; }
__host__ __device__ constexpr int bp_np(int K, int mode = kBpIS) {
  return (bp_nt(mode) * K + 31) / 32;
}
// per-replicate panel tail (KL): kBpMaxK row scales 2^-e_k and their inverses, fp32
constexpr int kBpTail = 256;
// ranks the kernels take (the engine pads K > 32 to a multiple of 8, models.nmf.native_rank)
constexpr int kBpMaxK = 64;
__host__ __device__ constexpr int bp_t(int K) { return (K + 15) / 16; }
// P-panel row stride: 32 NP + 16 bf16 (96, 160, 224 B rows) is conflict-free for the
// ds_read_b128 fragment reads; 32 NP + 8 (80 B at NP = 1) was 2-way
__host__ __device__ constexpr int bp_ps(int NP) { return 32 * NP + 16; }
// chunk stride (bf16 elements), padded to whole 16-byte pieces per thread so the staging
// loads are unconditional (the tail of a chunk is never written nor read by the MFMAs)
__host__ __device__ constexpr int bp_chunk(int NP, int T) {
  return (kBpCH * bp_ps(NP) + 2 * 16 * T * kBpNS + kBpThreads * 8 - 1) / (kBpThreads * 8) *
         (kBpThreads * 8);
}
// column tiles per wave: 2 (4: 820 vs 510 us per usage step; 1 for KL -- fewer live
// registers, twice the workgroups -- measured 290 vs 325 rep/s: the panel chunks in LDS
// then serve 64 columns instead of 128, profiles/r3l_*).  1 from T = 3 (K > 32): the
// fixed operand's planes and the accumulators of two tiles would not fit the registers
__host__ __device__ constexpr int bp_ct(int T) { return T >= 3 ? 1 : 2; }
__host__ __device__ constexpr int bp_ks(int T) { return 16 * T + 1; }     // exchange stride

// plane of the streamed (a) / fixed (b) operand in product term t (0..5)
__device__ __forceinline__ int bp_pa(int t) { return (0x210100 >> (4 * t)) & 15; }
__device__ __forceinline__ int bp_pb(int t) { return (0x012010 >> (4 * t)) & 15; }

__device__ __forceinline__ unsigned short bp_bits(__bf16 h) {
  return __builtin_bit_cast(unsigned short, h);
}

// v = p0 + p1 + p2 exactly (finite v, away from the subnormal range)
__device__ __forceinline__ void bp_split3(float v, unsigned short& p0, unsigned short& p1,
                                          unsigned short& p2) {
  const __bf16 h0 = (__bf16)v;
  const float r1 = v - (float)h0;
  const __bf16 h1 = (__bf16)r1;
  const float r2 = r1 - (float)h1;
  p0 = bp_bits(h0);
  p1 = bp_bits(h1);
  p2 = bp_bits((__bf16)r2);
}

// -------------------------------------------------------------------------------- panels
// Per replicate r the panel buffer is nchunks x bp_chunk(NP, T) bf16: chunk c covers
// streamed rows [64c, 64c + 64), zero beyond L:
//   P panel  [64 rows][bp_ps(NP)]:  row l, slot t*K + k = plane bp_pa(t) of F[k][l]
//   N panel  [2 planes][16T rows k][kBpNS]: plane p of F[k][l] at the permuted column of l
//            (within a 32-row block: offset o = 16h + 4q + i  ->  8q + 4h + i); KL: the
//            two fp16 planes of F[k][l] * 2^-e_k instead
//   (KL) tail [kBpTail]: fp32 2^-e_k (k < kBpMaxK), then 2^e_k
// ------------------------------------------------------------------------------ main op
struct BpParams {
  const float* X;              // element (fixed col c, streamed row j) at X[c * ldx + j]
  long long ldx;
  int xvec;                    // ldx % 4 == 0 and X 16-byte aligned: float4 loads
  // KL on fp16 counts (x = c * u_g, c <= 2048 exact in fp16): X points at the counts
  // (_Float16); the H side's P panel was built from S / u (so c / P' = x / P), the loss
  // weights x by uvec (per streamed row); the W side scales its fixed operand by fscale
  const float* uvec;
  const float* fscale;
  const unsigned short* panel; // streamed operand panels, replicate r at panel + r*panel_rs
  long long panel_rs;
  float* F;                    // fixed operand, replicate r: F + r*f_rs, row k stride ldf
  long long f_rs, ldf;
  int K, Lf, Ls, R;
  int n_strips, splits, chunks_per_split;
  float beta, eps;
  float* num;                  // side W: (splits, R, K, Lf)
  float* den;                  //   same (beta != 1)
  int nsteps;                  // side H: MU steps this launch (0: loss only)
  int loss_entry, loss_exit;   // evaluate D(X | P) before the first / after the last step
  const float* den_vec;        // KL: (R, K) row sums of W
  float l1, l2, gamma, tol;
  int conv_mode;               // 0: |dh|/|h| of the last step < tol; 1: block objective
  double* hstate;              // (R, 2): objective at the last check, checks done
  double* part;                // (R, n_strips, 4) partials: |dh|^2, |h|^2, f_entry, f_exit
  int* counter;                // (R) arrival counters, zero between launches
  int* act;                    // (R) active flags cleared by the stopping rule
  int* iters;                  // (R) MU steps taken
  const int* active;           // gate (0: workgroup exits)
  double* loss;                // loss-only launches: (R, n_strips) partial objectives
  double xsum;                 // KL: sum of X over the rows (the objective's -sum x term)
};

template <int MODE>
__device__ __forceinline__ void bp_terms(float x, float p, float beta, float& q, float& d) {
  if (bp_is_kl(MODE)) {
    q = x * __builtin_amdgcn_rcpf(p);
    d = 1.f;
  } else if (MODE == kBpIS) {
    const float r = __builtin_amdgcn_rcpf(p);
    d = r;
    q = x * r * r;
  } else {
    const float lp = __builtin_amdgcn_logf(p);  // log2
    d = __builtin_amdgcn_exp2f((beta - 1.f) * lp);
    q = x * __builtin_amdgcn_exp2f((beta - 2.f) * lp);
  }
}

// D_beta term of (x, p); q = x P^(beta-2) and d = P^(beta-1) as bp_terms left them
template <int MODE>
__device__ __forceinline__ float bp_loss(float x, float p, float q, float d, float beta,
                                         float eps) {
  if (bp_is_kl(MODE)) {
    // x log2(x / p) only (q = x / p): the linear part sum(p) - sum(x) of the KL objective
    // is added per workgroup from the usage and spectra sums (bp_kernel)
    return x > 0.f ? x * __builtin_amdgcn_logf(q) : 0.f;
  } else if (MODE == kBpIS) {
    const float r = fmaxf(x * d, eps);                // d = 1 / p
    return r - __logf(r) - 1.f;
  } else {
    return (__powf(x, beta) + (beta - 1.f) * __powf(p, beta) - beta * x * __powf(p, beta - 1.f)) /
           (beta * (beta - 1.f));
  }
}

// 8 fp32 values -> two bf16 planes (hi, residual)
__device__ __forceinline__ void bp_split2(const float (&v)[8], bp_v8& b0, bp_v8& b1) {
  bp_b8 h, l;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h[e] = (__bf16)v[e];
    l[e] = (__bf16)(v[e] - (float)h[e]);
  }
  b0 = __builtin_bit_cast(bp_v8, h);
  b1 = __builtin_bit_cast(bp_v8, l);
}

__device__ __forceinline__ bp_f4 bp_mfma(bp_v8 a, bp_v8 b, bp_f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// x[col][j .. j+3] (zero beyond Ls / for an invalid column)
__device__ __forceinline__ void bp_load4(const float* __restrict__ row, int j, int Ls, bool ok,
                                         int xvec, float* out) {
  if (ok && xvec && j + 3 < Ls) {
    const float4 v = *reinterpret_cast<const float4*>(row + j);
    out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = (ok && j + i < Ls) ? row[j + i] : 0.f;
  }
}

// OCC: waves per SIMD the register allocation targets (2: the compiler's choice, ~235
// VGPRs for the usage-side kernels; 3: <= 168, with spills outside the hot loop)
template <int NP, int T, int MODE, bool UPD, int CT, bool XH, int OCC = 2>
__global__ void __launch_bounds__(kBpThreads) __attribute__((amdgpu_waves_per_eu(OCC)))
bp_kernel(BpParams p) {
  constexpr int PS = bp_ps(NP);
  constexpr int CE = bp_chunk(NP, T);
  constexpr int PIECES = CE * 2 / 16;
  constexpr int PER_T = (PIECES + kBpThreads - 1) / kBpThreads;
  constexpr int COLS = kBpWaves * CT * 16;
  constexpr int KS = bp_ks(T);
  constexpr bool kH = MODE == kBpKL;   // fp16 numerator path (see the file comment)
  constexpr bool kKL = bp_is_kl(MODE); // den = S 1 (host vector), KL objective
  constexpr int NT = bp_nt(MODE);
  static_assert(PIECES == PER_T * kBpThreads, "chunk must be whole pieces per thread");
  extern __shared__ __attribute__((aligned(16))) unsigned char bp_smem[];
  __shared__ double sred[4 * kBpWaves];
  __shared__ int s_last;

  // XCD-aware unit map: the replicates of one unit (strip, split) run back to back on one
  // XCD, so its X rows stay in that L2
  const int b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int rep = local % p.R;
  const int unit = (local / p.R) * 8 + xcd;
  if (unit >= p.n_strips * p.splits) return;
  if (p.active && p.active[rep] == 0) return;
  const int strip = unit % p.n_strips, split = unit / p.n_strips;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, m = lane & 15;
  const int K = p.K;
  const int col_w = strip * COLS + wave * CT * 16;
  float* __restrict__ F = p.F + (long long)rep * p.f_rs;
  const unsigned short* __restrict__ pan = p.panel + (long long)rep * p.panel_rs;
  const int nch_all = (p.Ls + kBpCH - 1) / kBpCH;
  const int c_begin = split * p.chunks_per_split;
  const int c_end = min(nch_all, c_begin + p.chunks_per_split);
  unsigned short* sbuf = reinterpret_cast<unsigned short*>(bp_smem);
  float* sx = reinterpret_cast<float*>(bp_smem + 2 * CE * 2) + wave * (CT * 16) * KS;

  bool cok[CT];
  const float* xrow[CT];
  const _Float16* xhrow[CT];
  float fsc[CT];   // XH, W side: 1 / u of the column's gene
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int col = col_w + 16 * ct + m;
    cok[ct] = col < p.Lf;
    xrow[ct] = p.X + (long long)(cok[ct] ? col : 0) * p.ldx;
    xhrow[ct] = reinterpret_cast<const _Float16*>(p.X) + (long long)(cok[ct] ? col : 0) * p.ldx;
    fsc[ct] = (XH && !UPD && cok[ct]) ? p.fscale[col] : 1.f;
  }

  // KL: per-column shift 2^s of F (csc) and s (csg); inverse panel row scales 2^e_k
  float csc[CT], csg[CT], rinv[T][4];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    csc[ct] = 1.f;
    csg[ct] = 0.f;
  }
  if (kH) {
    const float* tail = reinterpret_cast<const float*>(pan + (long long)nch_all * CE);
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 16 * t + 4 * q + i;
        rinv[t][i] = k < K ? tail[kBpMaxK + k] : 0.f;
      }
  }

  // fixed operand in the accumulator layout: hc[ct][t][i] = F[16t + 4q + i][col]
  bp_f4 hc[CT][T];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 16 * t + 4 * q + i;
        hc[ct][t][i] = (k < K && cok[ct]) ? F[(long long)k * p.ldf + col_w + 16 * ct + m] : 0.f;
      }

  // B-operand planes of the fixed operand: slot s = 32j + 8q + e holds plane bp_pb(s / K)
  // of F[s % K][col]; rebuilt through the wave's LDS exchange rows after every update
  bp_v8 freg[CT][NP];
  auto build_freg = [&]() {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          sx[(16 * ct + m) * KS + 16 * t + 4 * q + i] =
              (kH || XH) ? hc[ct][t][i] * (csc[ct] * fsc[ct]) : hc[ct][t][i];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int s0 = 32 * j + 8 * q;
      int tt = s0 / K, kk = s0 - tt * K;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int pl = bp_pb(tt < NT ? tt : 0);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          unsigned short a0 = 0, a1 = 0, a2 = 0;
          if (tt < NT) bp_split3(sx[(16 * ct + m) * KS + kk], a0, a1, a2);
          freg[ct][j][e] = (short)(pl == 0 ? a0 : (pl == 1 ? a1 : a2));
        }
        if (++kk == K) { kk = 0; ++tt; }
      }
    }
    __syncthreads();
  };
  build_freg();

  // The exit objective is read off the P pass of the block's LAST step (the iterate
  // before that step's update, so no extra pass over X); with a single step per launch
  // it would coincide with the entry objective, so it gets a P pass of its own then.
  const bool exit_in_last = p.nsteps >= 2;
  const int n_it = UPD ? p.nsteps + ((p.loss_exit && !exit_in_last) || p.nsteps == 0 ? 1 : 0)
                       : 1;
  double f_entry = 0.0, f_exit = 0.0;
  float d2 = 0.f, o2 = 0.f;
  // panel chunk c -> registers -> LDS buffer bi (plain loads: the compiler counts them,
  // so waiting for this block's X loads leaves the next chunk's panels in flight)
  bp_u4 stg[PER_T];
  auto load_chunk = [&](int c) {
    const bp_u4* src = reinterpret_cast<const bp_u4*>(pan + (long long)c * CE);
#pragma unroll
    for (int u = 0; u < PER_T; ++u) stg[u] = src[u * kBpThreads + tid];
  };
  auto store_chunk = [&](int bi) {
    bp_u4* dst = reinterpret_cast<bp_u4*>(sbuf + bi * CE);
#pragma unroll
    for (int u = 0; u < PER_T; ++u) dst[u * kBpThreads + tid] = stg[u];
  };

  for (int it = 0; it < n_it; ++it) {
    const bool want_num = !UPD || it < p.nsteps;
    const bool is_exit = it == (exit_in_last ? p.nsteps - 1 : p.nsteps);
    const bool is_entry = it == 0 && p.loss_entry && p.nsteps > 0;
    const bool want_loss = UPD && (is_entry || (is_exit && (p.loss_exit || p.nsteps == 0)));
    bp_f4 num[CT][T], den[CT][T];
    float lsum = 0.f;
    // X of block b (32 streamed rows) for this lane's columns: float4 loads while the
    // block is inside X (invalid columns read row 0 -- their F is zero and their outputs
    // are discarded), guarded scalar loads at the tail
    auto load_x = [&](int b, float (&dst)[CT][8]) {
      const int j0 = (c_begin + (b >> 1)) * kBpCH + (b & 1) * 32;
      if constexpr (XH) {
        if (p.xvec && j0 + 32 <= p.Ls) {
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            const bp_h4 v0 = *reinterpret_cast<const bp_h4*>(xhrow[ct] + j0 + 4 * q);
            const bp_h4 v1 = *reinterpret_cast<const bp_h4*>(xhrow[ct] + j0 + 16 + 4 * q);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              dst[ct][i] = (float)v0[i];
              dst[ct][4 + i] = (float)v1[i];
            }
          }
        } else {
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int ja = j0 + 4 * q + i, jb = j0 + 16 + 4 * q + i;
              dst[ct][i] = (cok[ct] && ja < p.Ls) ? (float)xhrow[ct][ja] : 0.f;
              dst[ct][4 + i] = (cok[ct] && jb < p.Ls) ? (float)xhrow[ct][jb] : 0.f;
            }
        }
        return;
      }
      if (p.xvec && j0 + 32 <= p.Ls) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const bp_f4 v0 = *reinterpret_cast<const bp_f4*>(xrow[ct] + j0 + 4 * q);
          const bp_f4 v1 = *reinterpret_cast<const bp_f4*>(xrow[ct] + j0 + 16 + 4 * q);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            dst[ct][i] = v0[i];
            dst[ct][4 + i] = v1[i];
          }
        }
      } else {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          bp_load4(xrow[ct], j0 + 4 * q, p.Ls, cok[ct], 0, &dst[ct][0]);
          bp_load4(xrow[ct], j0 + 16 + 4 * q, p.Ls, cok[ct], 0, &dst[ct][4]);
        }
      }
    };
    // one 32-row block of the streamed axis: P tiles, elementwise terms, loss, numerator
    // (WN, WL: numerator / loss wanted, as compile-time constants so that the hot
    // variant -- numerator only -- is one straight-line block over both column tiles)
    auto compute_block = [&](auto WN, auto WL, auto SAT, const float (&xv)[CT][8], int blk,
                             const unsigned short* pb, int j0) {
      constexpr bool kNum = decltype(WN)::value, kLoss = decltype(WL)::value;
      const unsigned short* nb0 = pb + kBpCH * PS;
      const unsigned short* nb1 = nb0 + 16 * T * kBpNS;
        bp_v8 ap[2][NP];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int jj = 0; jj < NP; ++jj)
            ap[a][jj] = *reinterpret_cast<const bp_v8*>(pb + (blk * 32 + 16 * a + m) * PS +
                                                         32 * jj + 8 * q);
        bp_v8 an0[T], an1[T];
        if (kNum) {
#pragma unroll
          for (int t = 0; t < T; ++t) {
            const int off = (16 * t + m) * kBpNS + blk * 32 + 8 * q;
            an0[t] = *reinterpret_cast<const bp_v8*>(nb0 + off);
            an1[t] = *reinterpret_cast<const bp_v8*>(nb1 + off);
          }
        }
        // phase 1: the P tiles of every column tile (independent MFMA chains), so the
        // elementwise work of tile 0 overlaps the MFMAs of tile 1
        bp_f4 P0[CT], P1[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const float e0 = kH ? p.eps * csc[ct] : p.eps;
          P0[ct] = bp_f4{e0, e0, e0, e0};
          P1[ct] = P0[ct];
#pragma unroll
          for (int jj = 0; jj < NP; ++jj) {
            P0[ct] = bp_mfma(ap[0][jj], freg[ct][jj], P0[ct]);
            P1[ct] = bp_mfma(ap[1][jj], freg[ct][jj], P1[ct]);
          }
        }
        // phase 2: elementwise terms, loss, operand planes; phase 3: numerator MFMAs
        if constexpr (kH) {
          bp_h8 qh[CT];
          // XH: the loss weight x = c u_j of each streamed row (u from L1)
          float uw[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) uw[e] = 1.f;
          if (XH && kLoss) {
            if (j0 + 32 <= p.Ls) {
              const float4 u0 = *reinterpret_cast<const float4*>(p.uvec + j0 + 4 * q);
              const float4 u1 = *reinterpret_cast<const float4*>(p.uvec + j0 + 16 + 4 * q);
              uw[0] = u0.x; uw[1] = u0.y; uw[2] = u0.z; uw[3] = u0.w;
              uw[4] = u1.x; uw[5] = u1.y; uw[6] = u1.z; uw[7] = u1.w;
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const int j = j0 + (e >> 2) * 16 + 4 * q + (e & 3);
                uw[e] = j < p.Ls ? p.uvec[j] : 0.f;
              }
            }
          }
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float x = xv[ct][e];
              const float qv = x * __builtin_amdgcn_rcpf(e < 4 ? P0[ct][e] : P1[ct][e - 4]);
              if (kLoss) {
                // x log2(x / p) with q' = q 2^-s: log2 q = log2 q' + s
                const int j = j0 + (e >> 2) * 16 + 4 * q + (e & 3);
                const float t = x > 0.f ? (x * uw[e]) * (__builtin_amdgcn_logf(qv) + csg[ct])
                                        : 0.f;
                lsum += (cok[ct] && j < p.Ls) ? t : 0.f;
              }
              if (kNum) qh[ct][e] = (_Float16)qv;
            }
            // the redo pass after an overflow saturates instead (x / p beyond 2^40)
            if (decltype(SAT)::value) qh[ct] = __builtin_elementwise_min(qh[ct], bp_h8(65504.f16));
          }
          if (kNum) {
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
              for (int t = 0; t < T; ++t) {
                num[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                    __builtin_bit_cast(bp_h8, an0[t]), qh[ct], num[ct][t], 0, 0, 0);
                num[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                    __builtin_bit_cast(bp_h8, an1[t]), qh[ct], num[ct][t], 0, 0, 0);
              }
          }
        } else {
          bp_v8 qb0[CT], qb1[CT], db0[CT], db1[CT];
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            float qv[8], dv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e)
              bp_terms<MODE>(xv[ct][e], e < 4 ? P0[ct][e] : P1[ct][e - 4], p.beta, qv[e], dv[e]);
            if (kLoss) {
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const int j = j0 + (e >> 2) * 16 + 4 * q + (e & 3);
                const float t = bp_loss<MODE>(xv[ct][e], e < 4 ? P0[ct][e] : P1[ct][e - 4], qv[e],
                                              dv[e], p.beta, p.eps);
                lsum += (cok[ct] && j < p.Ls) ? t : 0.f;
              }
            }
            if (kNum) {
              bp_split2(qv, qb0[ct], qb1[ct]);
              if (!kKL) bp_split2(dv, db0[ct], db1[ct]);
            }
          }
          if (kNum) {
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
              for (int t = 0; t < T; ++t) {
                num[ct][t] = bp_mfma(an0[t], qb0[ct], num[ct][t]);
                num[ct][t] = bp_mfma(an0[t], qb1[ct], num[ct][t]);
                num[ct][t] = bp_mfma(an1[t], qb0[ct], num[ct][t]);
                if (!kKL) {
                  den[ct][t] = bp_mfma(an0[t], db0[ct], den[ct][t]);
                  den[ct][t] = bp_mfma(an0[t], db1[ct], den[ct][t]);
                  den[ct][t] = bp_mfma(an1[t], db0[ct], den[ct][t]);
                }
              }
          }
        }
    };
    // one pass over the streamed axis into num / den / lsum.  Software pipeline over the
    // chunks: block 0's X (xa) arrived during the previous chunk; block 1's X (xb), the
    // next chunk's block-0 X and panels load behind the compute (the last chunk reloads
    // itself into the idle buffer: no branch around the staging registers)
    using kT = std::integral_constant<bool, true>;
    using kF = std::integral_constant<bool, false>;
    auto stream_pass = [&](auto SAT) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int t = 0; t < T; ++t) {
          num[ct][t] = bp_f4{0.f, 0.f, 0.f, 0.f};
          den[ct][t] = bp_f4{0.f, 0.f, 0.f, 0.f};
        }
      lsum = 0.f;
      if (c_begin < c_end) {
        load_chunk(c_begin);
        store_chunk(0);
      }
      __syncthreads();
      const int nblk = 2 * (c_end - c_begin);
      float xa[CT][8], xb[CT][8];
      if (nblk > 0) load_x(0, xa);
      for (int c = c_begin; c < c_end; ++c) {
        const int i2 = 2 * (c - c_begin), bi = (c - c_begin) & 1;
        const unsigned short* pb = sbuf + bi * CE;
        load_x(i2 + 1, xb);
        load_chunk(min(c + 1, c_end - 1));
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (h == 1 && i2 + 2 < nblk) load_x(i2 + 2, xa);
          const float(&xv)[CT][8] = h == 0 ? xa : xb;
          const int j0 = c * kBpCH + 32 * h;
          if (want_num && !want_loss) compute_block(kT{}, kF{}, SAT, xv, h, pb, j0);
          else if (want_num) compute_block(kT{}, kT{}, SAT, xv, h, pb, j0);
          else compute_block(kF{}, kT{}, SAT, xv, h, pb, j0);
        }
        store_chunk(bi ^ 1);
        __syncthreads();
      }
    };
    stream_pass(kF{});

    if (kH && want_num) {
      // fp16 overflow of some column's Q: redo the step with that column's shift raised
      // (ballot over the lanes of one column: lane 16q + m, all q; padded columns ignored)
      bool bad[CT];
      int any = 0;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        bool b = false;
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) b |= !(fabsf(num[ct][t][i]) <= 3.0e38f);
        const unsigned long long bal = __ballot(b && cok[ct]);
        const unsigned c16 = (unsigned)((bal | (bal >> 16) | (bal >> 32) | (bal >> 48)) & 0xffffu);
        bad[ct] = (c16 >> m) & 1u;
        any |= c16 != 0u;
      }
      if (__syncthreads_or(any)) {
        // rare: a second copy of the pass (no loop back-edge: a retry loop around the
        // pass kept ~40 more VGPRs live in the hot loop) with the columns' shift raised
        // by 2^24 for the rest of the launch, saturating what still overflows
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
          if (bad[ct]) {
            csc[ct] *= 16777216.f;
            csg[ct] += 24.f;
          }
        build_freg();
        stream_pass(kT{});
      }
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) num[ct][t][i] *= rinv[t][i] * csc[ct];
    }

    if (want_loss) {
      double l = (double)lsum;
      if (kKL) {
        // sum x log(x/p) = ln 2 * sum x log2(x/p);  sum p = sum_k (sum_cols h_k) (sum_g w_k)
        // (+ eps per element, negligible); - sum x is subtracted once per replicate
        l *= 0.69314718055994530942;
        float hp = 0.f;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int t = 0; t < T; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int k = 16 * t + 4 * q + i;
              if (k < K && cok[ct]) hp = fmaf(hc[ct][t][i], p.den_vec[(long long)rep * K + k], hp);
            }
        l += (double)hp;
      }
      if (is_entry) f_entry += l;
      if (is_exit) f_exit += l;
    }
    if (UPD && want_num) {
      const bool last = it + 1 == p.nsteps;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int k = 16 * t + 4 * q + i;
            if (k < K && cok[ct]) {
              const float h = hc[ct][t][i];
              float dn = kKL ? p.den_vec[(long long)rep * K + k] : den[ct][t][i];
              dn = dn + p.l1 + p.l2 * h;
              if (dn == 0.f) dn = p.eps;
              float delta = num[ct][t][i] / dn;
              if (p.gamma != 1.f) delta = __powf(delta, p.gamma);
              const float hn = h * delta;
              if (last) {
                d2 = fmaf(hn - h, hn - h, d2);
                o2 = fmaf(h, h, o2);
              }
              hc[ct][t][i] = hn;
            }
          }
      if (it + 1 < n_it) build_freg();
    }
    if (!UPD) {
      const long long base = ((long long)split * p.R + rep) * K * p.Lf;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int k = 16 * t + 4 * q + i;
            if (k < K && cok[ct]) {
              const long long o = base + (long long)k * p.Lf + col_w + 16 * ct + m;
              p.num[o] = num[ct][t][i];
              if (!kKL) p.den[o] = den[ct][t][i];
            }
          }
    }
  }

  if (!UPD) return;
  if (p.nsteps > 0) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 16 * t + 4 * q + i;
          if (k < K && cok[ct]) F[(long long)k * p.ldf + col_w + 16 * ct + m] = hc[ct][t][i];
        }
  }
  // workgroup partials: |dh|^2, |h|^2 (last step), objective at entry / exit
  {
    const double v0 = wave_sum((double)d2), v1 = wave_sum((double)o2);
    const double v2 = wave_sum(f_entry), v3 = wave_sum(f_exit);
    if (lane == 0) {
      sred[wave * 4 + 0] = v0;
      sred[wave * 4 + 1] = v1;
      sred[wave * 4 + 2] = v2;
      sred[wave * 4 + 3] = v3;
    }
    __syncthreads();
  }
  if (p.loss && tid == 0) {
    double tot = 0.0;
    for (int w = 0; w < kBpWaves; ++w) tot += sred[w * 4 + 3];
    p.loss[(long long)rep * p.n_strips + strip] = tot;
  }
  if (!p.part) return;
  if (tid == 0) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int w = 0; w < kBpWaves; ++w)
      for (int v = 0; v < 4; ++v) acc[v] += sred[w * 4 + v];
    // publish (cdna_hip_programming.md G16): plain stores -> drain -> agent release ->
    // drain -> arrival counter
    double* pp = p.part + ((long long)rep * p.n_strips + strip) * 4;
    for (int v = 0; v < 4; ++v) pp[v] = acc[v];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(p.counter + rep, 1, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    s_last = (prev == p.n_strips - 1);
  }
  __syncthreads();
  if (s_last && tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    double tot[4] = {0.0, 0.0, 0.0, 0.0};
    const double* pr = p.part + (long long)rep * p.n_strips * 4;
    for (int s2 = 0; s2 < p.n_strips; ++s2)
      for (int v = 0; v < 4; ++v)
        tot[v] += __hip_atomic_load(pr + 4 * s2 + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (kKL) {
      tot[2] -= p.xsum;
      tot[3] -= p.xsum;
    }
    if (p.conv_mode == 1) {
      double* hs = p.hstate + 2 * (long long)rep;
      const double f_prev = p.loss_entry ? tot[2] : hs[0];
      if ((p.loss_entry || hs[1] > 0.0) && fabs(f_prev - tot[3]) <= (double)p.tol * fabs(f_prev))
        p.act[rep] = 0;
      hs[0] = tot[3];
      hs[1] = hs[1] + 1.0;
    } else if (p.nsteps > 0) {
      const double rel = sqrt(tot[0]) / (sqrt(tot[1]) + (double)p.eps);
      if (rel < (double)p.tol) p.act[rep] = 0;
    }
    if (p.iters) p.iters[rep] += p.nsteps;
    p.counter[rep] = 0;
  }
}

template <int NP, int T, int MODE, bool UPD, bool XH, int CT, int OCC>
hipError_t bp_launch_occ(const BpParams& p, hipStream_t s) {
  const size_t lds = (size_t)2 * bp_chunk(NP, T) * 2 +
                     (size_t)kBpWaves * CT * 16 * bp_ks(T) * sizeof(float);
  static bool attr_done = false;
  if (!attr_done) {
    const hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&bp_kernel<NP, T, MODE, UPD, CT, XH, OCC>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_done = true;
  }
  const int units = p.n_strips * p.splits;
  const int per_xcd = (units + 7) / 8;
  const dim3 grid((unsigned)(per_xcd * p.R * 8));
  hipLaunchKernelGGL((bp_kernel<NP, T, MODE, UPD, CT, XH, OCC>), grid, dim3(kBpThreads), lds, s,
                     p);
  return hipGetLastError();
}

template <int NP, int T, int MODE, bool UPD, bool XH = false, int CT = bp_ct(T)>
hipError_t bp_launch(const BpParams& p, hipStream_t s) {
  // K > 32: two panel chunks (74-156 KB of LDS) already hold a CU per workgroup, so the
  // register budget of one wave per SIMD costs no occupancy (at two waves the usage-side
  // kernels spilled 300-1500 bytes per lane)
  if constexpr (T >= 3) return bp_launch_occ<NP, T, MODE, UPD, XH, CT, 1>(p, s);
  else return bp_launch_occ<NP, T, MODE, UPD, XH, CT, 2>(p, s);
}


// wide ranks (K in 33..64, padded to a multiple of 8): instantiated in their own units
// (beta_planes_wide*.hip) so the K <= 32 kernels keep compiling in parallel
hipError_t bp_launch_wide_kl(bool upd, bool xh, int np, int t, const BpParams& p, hipStream_t s);
hipError_t bp_launch_wide_klx(bool upd, bool xh, int np, int t, const BpParams& p, hipStream_t s);
hipError_t bp_launch_wide_gen(int mode, bool upd, int np, int t, const BpParams& p,
                              hipStream_t s);

}  // namespace cnmf
