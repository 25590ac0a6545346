// Fused, replicate-batched NNLS-style inner solvers for NMF.
//
// Both halves of a Frobenius NMF step reduce to the same problem, independently per
// column j, with a convergence test on the WHOLE (replicate, chunk) block:
//   H-side  (cnmf.py:352-381 fit_H_online; nmf-torch online H step):
//       x = h^T (K x c), numer = W x^T (K x c), Gram = W W^T
//   W-side  (nmf-torch online/batch W step):
//       x = W (K x G),   numer = B = sum h^T x,  Gram = A = sum h^T h
// One workgroup owns one replicate's block and iterates the update in place (the block
// stays L2-resident), reducing ||dx||, ||x|| or the block objective on device.  There is
// no per-iteration kernel launch and no host sync (the reference syncs every iteration
// at cnmf.py:377).  A grid covers every active replicate of a batch, so one launch
// drives the whole replicate grid.
//
// ALGO 0 = multiplicative update (MU):  x <- x * numer / (Gram x + l2 x + l1_den),
//          rate := 0 where the denominator < eps (cnmf.py:370-372).
// ALGO 1 = HALS (Gauss-Seidel over components):
//          x_k <- max(0, x_k + (numer_k - l1_den - (Gram x)_k - l2 x_k) / (Gram_kk + l2)).
// Optional epilogue: lin_out[r] = <numer, x>, quad_out[r] = sum_j x_j^T Gram x_j, which
// give the exact Frobenius loss from sufficient statistics (trace trick, G7).
//
// Memory path: each sweep a thread handles U columns at a time and issues all 2*U*K
// loads of the group before any arithmetic (U*K loads in flight per lane hide the L2
// latency that dominated the one-column-at-a-time version: 273 us/solve in
// profiles/r1_bench_v0_kernel_stats.txt).  Loads/stores are buffer operations: the
// column is the per-lane VGPR offset, component k*ld the SGPR soffset, so the K
// addresses of a column cost no VGPRs.  Gram products read one LDS row per component
// (every lane the same word: broadcast), row by row behind a compiler memory fence and
// an opaque LDS base, so the K*K loop-invariant Gram values are never hoisted into
// registers (that hoisting spilled hundreds of VGPRs at K >= 7).
#pragma once
#include <hip/hip_runtime.h>
#include "common.h"
#include "solve_params.h"

namespace cnmf {

// cooperative slices per replicate (coop_sum2: one wave watches the 2 S granules)
constexpr int kCoopMaxSlices = 32;

template <int K>
constexpr int solve_max_threads() { return 1024; }

// Gram rows live in LDS padded to a multiple of 4 floats, so a row is read with KP/4
// ds_read_b128 broadcasts (every lane the same address) instead of K ds_read_b32.
__host__ __device__ constexpr int gram_pad(int K) { return (K + 3) & ~3; }

// Register-resident variant with U columns per thread: x and x_new live in VGPRs, the
// numerator is staged once in LDS (thread-major, odd row stride: conflict-free b32
// reads).  U is capped where the 1024-thread (128-VGPR) instantiation still compiles
// without spills (hipcc -Rpass-analysis=kernel-resource-usage, ROCm 7.2): U*K <= 33,
// except K = 15 (U = 2 spills 20 VGPRs).
__host__ __device__ constexpr int res_max_cols(int K) {
  return K == 15 ? 1 : ((33 / K) < 1 ? 1 : ((33 / K) > 4 ? 4 : (33 / K)));
}

// Columns per thread per group: keep ~(2U+1)K live floats well under the 128-VGPR cap.
__host__ __device__ constexpr int cols_per_group_rt(int K) {
  return (16 / K) < 1 ? 1 : ((16 / K) > 4 ? 4 : (16 / K));
}
template <int K>
constexpr int cols_per_group() { return cols_per_group_rt(K); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff,
                                           0x00020000);
}

#define CNMF_MEMBAR() asm volatile("" ::: "memory")

// raw_buffer_{load,store}_b32 move 32-bit integers: bit-cast, never value-convert.
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, int vo, int so) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}
__device__ __forceinline__ void buf_st(float v, __amdgpu_buffer_rsrc_t r, int vo, int so) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, vo, so, 0);
}

// A zero the compiler cannot see through, produced inside the column loop: indexing the
// LDS Gram with it stops LICM from hoisting all K*K loop-invariant Gram reads into
// registers (K*K VGPRs -> spills at K >= 7).  Every lane reads the same LDS word.
typedef __attribute__((address_space(3))) float lds_float;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f32x4 lds_f32x4;

__device__ __forceinline__ const lds_float* opaque(const lds_float* p) {
  asm volatile("" : "+v"(p));
  return p;
}

template <int K, int U, bool HasN = true>
struct ColGroup {
  float x[U][K];
  float n[HasN ? U : 1][HasN ? K : 1];
  int vo[U];
  bool ok[U];
};

template <int K, int U>
__device__ __forceinline__ void load_group(ColGroup<K, U>& cg, int j, int T, int end,
                                           __amdgpu_buffer_rsrc_t rx, int sx,
                                           __amdgpu_buffer_rsrc_t rn, int sn, float l1n) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = j + u * T;
    cg.ok[u] = c < end;
    cg.vo[u] = cg.ok[u] ? c * 4 : 0;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      cg.x[u][k] = buf_ld(rx, cg.vo[u], k * sx);
      cg.n[u][k] = buf_ld(rn, cg.vo[u], k * sn);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      cg.x[u][k] = cg.ok[u] ? cg.x[u][k] : 0.f;
      float t = cg.ok[u] ? cg.n[u][k] : 0.f;
      if (l1n > 0.f) t = fmaxf(t - l1n, 0.f);
      cg.n[u][k] = t;
    }
  }
}

// Cross-workgroup sum of (a, b) for the S workgroups of one replicate, epoch `e`.
// The data IS the flag (cdna_hip_programming.md Guideline 16, form R2): each workgroup
// publishes its two block totals as 8-byte {tag, value} granules with agent-scope atomic
// (write-through) stores into its own slots of epoch e; one wave of every workgroup
// re-reads the 2 S granules of the epoch (one lane each, relaxed agent-scope loads, no
// fence) until every tag is this launch's, then sums the S slices in slice order ->
// identical, deterministic totals everywhere.  No counter and no release/acquire fence:
// those (a CAS arrival + an L2 writeback/invalidate per workgroup) made one exchange cost
// ~3 us at S = 2 and ~15 us at S = 9.  Slots are never zeroed between eager launches (the
// tag is the launch generation, strictly increasing per workspace); under a HIP graph
// the captured memset zeroes them and the tag is 0xFFFFFFFF.  Spins are bounded: on
// timeout the flag is raised and the host fails.  Returns false once the launch's
// timeout flag is up (this or any earlier exchange gave up): the caller then stops
// iterating, so slices that diverged never wait for each other again.
typedef __attribute__((address_space(1))) unsigned long long gran_t;

__device__ __forceinline__ bool coop_sum2_tag(const SolveParams& p, unsigned gen, int rep,
                                              int e, float& a, float& b, float* sred);
__device__ __forceinline__ bool coop_sum2(const SolveParams& p, int rep, int e, float& a,
                                          float& b, float* sred) {
  return coop_sum2_tag(p, p.coop_gen, rep, e, a, b, sred);
}
__device__ __forceinline__ bool coop_sum2_tag_s(const SolveParams& p, unsigned gen, int rep,
                                                int e, float& a, float& b, float* sred, int S,
                                                int slice);
__device__ __forceinline__ bool coop_sum2_tag(const SolveParams& p, unsigned gen, int rep,
                                              int e, float& a, float& b, float* sred) {
  return coop_sum2_tag_s(p, gen, rep, e, a, b, sred, (int)gridDim.y, (int)blockIdx.y);
}
// (S slices; this workgroup is slice `slice` of replicate rep)
__device__ __forceinline__ bool coop_sum2_tag_s(const SolveParams& p, unsigned gen, int rep,
                                                int e, float& a, float& b, float* sred, int S,
                                                int slice) {
  if (S <= 1) return true;
  if (e >= p.coop_epochs) {  // workspace too small: treat as timeout (host sizes it)
    if (threadIdx.x == 0) atomicExch(p.coop_timeout, 2);
    return false;
  }
  gran_t* g = (gran_t*)(p.coop_slots + (((long long)rep * p.coop_epochs + e) * S) * 2);
  const unsigned long long tag = (unsigned long long)gen << 32;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (lane == 0) {
      __hip_atomic_store(g + 2 * slice, tag | __float_as_uint(a), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(g + 2 * slice + 1, tag | __float_as_uint(b), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    int ok = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(p.coop_timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0);
    // lane i < 2 S watches granule i (S <= 32: one wave covers every slot)
    unsigned long long v = tag;
    unsigned spins = 0;
    while (ok) {
      if (lane < 2 * S) v = __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all((v & 0xffffffff00000000ull) == tag)) break;
      __builtin_amdgcn_s_sleep(2);
      ++spins;
      if ((spins & 1023u) == 0 &&
          __builtin_amdgcn_readfirstlane(__hip_atomic_load(p.coop_timeout, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT)) != 0)
        ok = 0;   // another replicate's exchange already gave up: stop waiting (uniform)
      if (spins > (1u << 22)) {
        if (lane == 0) atomicExch(p.coop_timeout, 1);
        ok = 0;
      }
    }
    // slice-ordered sums through LDS (sred[3 ..]): deterministic on every workgroup
    if (lane < 2 * S) sred[3 + lane] = __uint_as_float((unsigned)v);
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      float ta = 0.f, tb = 0.f;
      if (ok) {
        for (int s2 = 0; s2 < S; ++s2) {
          ta += sred[3 + 2 * s2];
          tb += sred[3 + 2 * s2 + 1];
        }
      }
      sred[0] = ta;
      sred[1] = tb;
      sred[2] = ok ? 1.f : 0.f;
    }
  }
  __syncthreads();
  a = sred[0];
  b = sred[1];
  const bool good = sred[2] != 0.f;
  __syncthreads();
  return good;
}

__device__ __forceinline__ unsigned short solve_f2bf_rn(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

// Final x of this block's columns [j0, n) as three exact bf16 planes (x = hi + mid + lo,
// each residual exact in fp32), times pl_colmul; the last slice also zeroes the GEMM's
// k padding [ncols, pl_cols).  Reads x back from L2 (just stored by this block).
template <int K>
__device__ __forceinline__ void emit_planes(const SolveParams& p, int rep, int j0, int n,
                                            bool last_slice) {
  const float* __restrict__ x = p.x + (long long)rep * p.x_rs;
  unsigned short* __restrict__ pl = p.planes + (long long)rep * p.pl_rs;
  // this block's columns [j0, n), then (last slice only) the padding [ncols, pl_cols)
  const int pad = last_slice ? max(0, p.pl_cols - p.ncols) : 0;
  const int span = (n - j0) + pad;
  for (int i = threadIdx.x; i < span; i += blockDim.x) {
    const bool real = i < n - j0;
    const int c = real ? j0 + i : p.ncols + (i - (n - j0));
    const float m = (real && p.pl_colmul) ? p.pl_colmul[c] : 1.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float v = real ? x[(long long)k * p.ldx + c] * m : 0.f;
      const unsigned short h0 = solve_f2bf_rn(v);
      const float r1 = v - __uint_as_float((unsigned)h0 << 16);
      const unsigned short h1 = solve_f2bf_rn(r1);
      const float r2 = r1 - __uint_as_float((unsigned)h1 << 16);
      const long long o = (long long)k * p.pl_ld + c;
      pl[o] = h0;
      if (p.pl_n > 1) pl[p.pl_plane + o] = h1;
      if (p.pl_n > 2) pl[2 * p.pl_plane + o] = solve_f2bf_rn(r2);
    }
  }
}

// Row k of the padded LDS Gram into row[KP] (KP/4 broadcast b128 reads).
#define CNMF_GRAM_ROW(GZ, k, row)                                                                 \
  float row[KP];                                                                                  \
  do {                                                                                            \
    const lds_f32x4* rp_ = (const lds_f32x4*)((GZ) + (k) * KP);                                   \
_Pragma("unroll")                                                                                    \
    for (int q_ = 0; q_ < KP / 4; ++q_) {                                                         \
      const f32x4 v_ = rp_[q_];                                                                   \
      row[4 * q_] = v_.x; row[4 * q_ + 1] = v_.y; row[4 * q_ + 2] = v_.z; row[4 * q_ + 3] = v_.w; \
    }                                                                                             \
  } while (0)

// Per-group pieces shared by the streaming and the register-resident paths.  They are
// macros on purpose: as __forceinline__ functions taking the ColGroup by reference the
// compiler inlines them too late to scalarise the group, and the K=20 kernel went from
// 111 VGPRs / 0 spills to 128 VGPRs / 148 spills.  They expect K, KP, U, ALGO, sG, l1,
// l2, eps and the accumulators (q, l / d2, x2 / lin, quad) in scope; NV(u, k) names the
// numerator of column u, component k (a register of the group, or the LDS stage).
// Objective / epilogue loop order: Gram row k is read once (KP/4 broadcast b128) and
// used for all U columns.
// Objective terms (x2, dropping the constant ||X||^2):
//   f(x) = sum_j x_j^T Gram x_j - 2 numer_j . x_j + 2 l1 |x_j|_1 + l2 |x_j|^2
#define CNMF_OBJECTIVE_GROUP(CG, NV)                                                              \
  do {                                                                                            \
  const lds_float* gz = opaque(sG);                                                               \
_Pragma("unroll")                                                                                    \
  for (int k = 0; k < K; ++k) {                                                                   \
    CNMF_MEMBAR();                                                                                \
    CNMF_GRAM_ROW(gz, k, row);                                                                    \
_Pragma("unroll")                                                                                    \
    for (int u = 0; u < U; ++u) {                                                                 \
      float gx = 0.f;                                                                             \
_Pragma("unroll")                                                                                    \
      for (int kk = 0; kk < K; ++kk) gx = fmaf(row[kk], (CG).x[u][kk], gx);                       \
      q = fmaf((CG).x[u][k], gx + l2 * (CG).x[u][k], q);                                          \
      l = fmaf((CG).x[u][k], NV(u, k) - l1, l);                                                   \
    }                                                                                             \
  }                                                                                               \
  } while (0)


// One MU (Jacobi, row-wise) or HALS (Gauss-Seidel) sweep over the group's columns,
// accumulating |dx|^2 and |x_old|^2.  Padded columns hold x = numer = 0 and stay 0.
// Column-outer: only one column's K new values are live at a time (U*K would spill the
// resident variant); the Gram rows are re-read per column as b128 broadcasts.
#define CNMF_UPDATE_GROUP(CG, NV)                                                                 \
  do {                                                                                            \
  const lds_float* gz = opaque(sG);                                                               \
_Pragma("unroll")                                                                                    \
  for (int u = 0; u < U; ++u) {                                                                   \
    if (ALGO == 0) {                                                                              \
      float xn[K];                                                                                \
_Pragma("unroll")                                                                                    \
      for (int k = 0; k < K; ++k) {                                                               \
        CNMF_MEMBAR();                                                                            \
        CNMF_GRAM_ROW(gz, k, row);                                                                \
        float den = 0.f;                                                                          \
_Pragma("unroll")                                                                                    \
        for (int kk = 0; kk < K; ++kk) den = fmaf(row[kk], (CG).x[u][kk], den);                   \
        den = fmaf(l2, (CG).x[u][k], den) + l1;                                                   \
        xn[k] = (den < eps) ? 0.f : (CG).x[u][k] * (NV(u, k) * __builtin_amdgcn_rcpf(den));       \
      }                                                                                           \
_Pragma("unroll")                                                                                    \
      for (int k = 0; k < K; ++k) {                                                               \
        const float d = xn[k] - (CG).x[u][k];                                                     \
        d2 = fmaf(d, d, d2);                                                                      \
        x2 = fmaf((CG).x[u][k], (CG).x[u][k], x2);                                                \
        (CG).x[u][k] = xn[k];                                                                     \
      }                                                                                           \
    } else {                                                                                      \
_Pragma("unroll")                                                                                    \
      for (int k = 0; k < K; ++k) {                                                               \
        CNMF_MEMBAR();                                                                            \
        CNMF_GRAM_ROW(gz, k, row);                                                                \
        float gx = 0.f;                                                                           \
_Pragma("unroll")                                                                                    \
        for (int kk = 0; kk < K; ++kk) gx = fmaf(row[kk], (CG).x[u][kk], gx);                     \
        const float diag = row[k] + l2;                                                           \
        const float old = (CG).x[u][k];                                                           \
        float xn = old;                                                                           \
        if (diag > eps) xn = fmaxf(old + (NV(u, k) - l1 - gx - l2 * old) / diag, 0.f);            \
        const float d = xn - old;                                                                 \
        d2 = fmaf(d, d, d2);                                                                      \
        x2 = fmaf(old, old, x2);                                                                  \
        (CG).x[u][k] = xn;                                                                        \
      }                                                                                           \
    }                                                                                             \
  }                                                                                               \
  } while (0)


#define CNMF_LINQUAD_GROUP(CG, NV)                                                                \
  do {                                                                                            \
  const lds_float* gz = opaque(sG);                                                               \
_Pragma("unroll")                                                                                    \
  for (int k = 0; k < K; ++k) {                                                                   \
    CNMF_MEMBAR();                                                                                \
    CNMF_GRAM_ROW(gz, k, row);                                                                    \
_Pragma("unroll")                                                                                    \
    for (int u = 0; u < U; ++u) {                                                                 \
      float gx = 0.f;                                                                             \
_Pragma("unroll")                                                                                    \
      for (int kk = 0; kk < K; ++kk) gx = fmaf(row[kk], (CG).x[u][kk], gx);                       \
      lin = fmaf(NV(u, k), (CG).x[u][k], lin);                                                    \
      quad = fmaf((CG).x[u][k], gx, quad);                                                        \
    }                                                                                             \
  }                                                                                               \
  } while (0)

// numerator accessors for the macros above
#define CNMF_NREG_CG(u, k) (cg.n[u][k])
#define CNMF_NREG_RG(u, k) (rg.n[u][k])
// LDS numerator stage: thread-major rows of NS = (U*K)|1 words (odd stride: conflict-free
// b32 reads; one base VGPR, per-(u,k) immediate offsets)
#define CNMF_NLDS(u, k) (sNt[(u) * K + (k)])


template <int K, int U, bool HasN>
__device__ __forceinline__ void store_group(const ColGroup<K, U, HasN>& cg, __amdgpu_buffer_rsrc_t rx,
                                            int sx) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (cg.ok[u]) {
#pragma unroll
      for (int k = 0; k < K; ++k) buf_st(cg.x[u][k], rx, cg.vo[u], k * sx);
    }
  }
}

template <int K, int U>
__device__ __forceinline__ float block_objective(__amdgpu_buffer_rsrc_t rx, int sx,
                                                 __amdgpu_buffer_rsrc_t rn, int sn,
                                                 const lds_float* sG, int j0, int n, float l1_num,
                                                 float l1, float l2, float* sred) {
  constexpr int KP = gram_pad(K);
  float q = 0.f, l = 0.f;
  const int T = blockDim.x;
  for (int j = j0 + threadIdx.x; j < n; j += U * T) {
    CNMF_MEMBAR();
    ColGroup<K, U> cg;
    load_group<K, U>(cg, j, T, n, rx, sx, rn, sn, l1_num);
    CNMF_OBJECTIVE_GROUP(cg, CNMF_NREG_CG);
  }
  block_sum2(q, l, sred);
  return q - 2.f * l;
}

// RES = 0: streaming variant (U = cols_per_group columns per thread per sweep, x and
// numer re-read from L2 every iteration).  RES = U >= 1: register-resident variant, U
// columns per thread: x in VGPRs for the whole solve, numerator staged once in LDS.
// Launched only when every slice fits U columns per thread (host check in cnmf_solve).
// Launch bound per K: K > 32 (the padded wide ranks 40..64, streaming only) keeps a
// column's K values, its numerator and the new values live at once (~3K VGPRs), which
// only fits the 512-register budget of one wave per SIMD: 256-thread workgroups.
template <int K>
constexpr int solve_block_threads() { return K > 32 ? 256 : 1024; }

template <int K, int ALGO, int RES>
__global__ __launch_bounds__(solve_block_threads<K>()) void solve_kernel(SolveParams p) {
  constexpr int U = RES ? RES : cols_per_group<K>();
  constexpr int KP = gram_pad(K);
  constexpr bool resident = RES != 0;
  __shared__ __attribute__((aligned(16))) float sGm[K * KP];
  __shared__ float sred[3 + 2 * kCoopMaxSlices];
  constexpr int NS = (U * K) | 1;
  __shared__ float sNm[resident ? NS * 1024 : 1];
  const lds_float* sG = (const lds_float*)sGm;  // LDS (addrspace 3): ds_read, 32-bit address
  const int rep = p.rep_index ? p.rep_index[blockIdx.x] : (int)blockIdx.x;
  if (p.active && p.active[rep] == 0) return;  // converged replicate: untouched (uniform)
  float* __restrict__ x = p.x + (long long)rep * p.x_rs;
  const float* __restrict__ nu = p.numer + (long long)rep * p.n_rs;
  const float* __restrict__ g = p.gram + (long long)rep * p.g_rs;
  for (int i = threadIdx.x; i < K * KP; i += blockDim.x) {
    const int r = i / KP, c = i - r * KP;
    sGm[i] = c < K ? g[r * K + c] : 0.f;
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t rx = rsrc_of(x);
  const __amdgpu_buffer_rsrc_t rn = rsrc_of(nu);
  const int sx = (int)(p.ldx * 4), sn = (int)(p.ldn * 4);
  const int T = blockDim.x;
  // Column range of this block: the whole block, one of nsplit fixed-step slices, or one
  // of S cooperative slices (gridDim.y) that still converge together.
  int j0 = 0, n = p.ncols;
  const bool coop = p.coop_slots != nullptr && gridDim.y > 1;
  if (p.nsplit > 1 || coop) {
    const int parts = coop ? (int)gridDim.y : p.nsplit;
    const int per = (p.ncols + parts - 1) / parts;
    j0 = min(p.ncols, (int)blockIdx.y * per);
    n = min(p.ncols, j0 + per);
  }
  const bool check_conv = p.nsplit <= 1;
  int epoch = 0;
  const bool loss_conv = check_conv && p.conv_mode == 1;
  const int every = p.check_every > 0 ? p.check_every : 1;
  const float l1 = p.l1_den, l2 = p.l2, eps = p.eps;
  float f_prev = 0.f;
  bool have_prev = false;
  int it = 0;
  if constexpr (resident) {
    // Register-resident path: x stays in VGPRs for every iteration and the numerator in
    // LDS (no per-iteration global round trip -- that latency/L2 traffic, not
    // arithmetic, bounded the streaming loop).  Each thread reads back only the LDS
    // words it wrote, so staging needs no barrier.
    float* sNt = sNm + threadIdx.x * NS;
    ColGroup<K, U, false> rg;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = j0 + threadIdx.x + u * T;
      rg.ok[u] = c < n;
      rg.vo[u] = rg.ok[u] ? c * 4 : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float xv = buf_ld(rx, rg.vo[u], k * sx);
        float nv = buf_ld(rn, rg.vo[u], k * sn);
        rg.x[u][k] = rg.ok[u] ? xv : 0.f;
        nv = rg.ok[u] ? nv : 0.f;
        if (p.l1_num > 0.f) nv = fmaxf(nv - p.l1_num, 0.f);
        CNMF_NLDS(u, k) = nv;
      }
    }
    while (true) {
      if (loss_conv && it % every == 0) {
        float q = 0.f, l = 0.f;
        CNMF_OBJECTIVE_GROUP(rg, CNMF_NLDS);
        block_sum2(q, l, sred);
        float f = q - 2.f * l;
        if (coop) {
          float unused = 0.f;
          if (!coop_sum2(p, rep, epoch++, f, unused, sred)) break;
        }
        if (have_prev && fabsf(f_prev - f) <= p.tol * fabsf(f_prev)) break;
        f_prev = f;
        have_prev = true;
      }
      if (it >= p.max_iter) break;
      float d2 = 0.f, x2 = 0.f;
      CNMF_UPDATE_GROUP(rg, CNMF_NLDS);
      ++it;
      if (!check_conv || loss_conv) continue;
      block_sum2(d2, x2, sred);
      if (coop && !coop_sum2(p, rep, epoch++, d2, x2, sred)) break;
      if (sqrtf(d2) / (sqrtf(x2) + eps) < p.tol) break;
    }
    store_group<K, U>(rg, rx, sx);
    if (p.lin_out || p.quad_out) {
      float lin = 0.f, quad = 0.f;
      if (p.l1_num > 0.f) {
        // epilogue uses the raw numerator (no l1 shift), as the streaming reload does
        ColGroup<K, U> cg;
        load_group<K, U>(cg, j0 + threadIdx.x, T, n, rx, sx, rn, sn, 0.f);
        CNMF_LINQUAD_GROUP(cg, CNMF_NREG_CG);
      } else {
        CNMF_LINQUAD_GROUP(rg, CNMF_NLDS);
      }
      block_sum2(lin, quad, sred);
      if (coop) (void)coop_sum2(p, rep, epoch++, lin, quad, sred);
      if (threadIdx.x == 0 && (!coop || blockIdx.y == 0)) {
        if (check_conv) {
          if (p.lin_out) p.lin_out[rep] = lin;
          if (p.quad_out) p.quad_out[rep] = quad;
        } else {  // split columns: caller zeroed the outputs
          if (p.lin_out) atomicAdd(p.lin_out + rep, lin);
          if (p.quad_out) atomicAdd(p.quad_out + rep, quad);
        }
      }
    }
  } else {
    while (true) {
      if (loss_conv && it % every == 0) {
        float f = block_objective<K, U>(rx, sx, rn, sn, sG, j0, n, p.l1_num, l1, l2, sred);
        if (coop) {
          float unused = 0.f;
          if (!coop_sum2(p, rep, epoch++, f, unused, sred)) break;
        }
        if (have_prev && fabsf(f_prev - f) <= p.tol * fabsf(f_prev)) break;
        f_prev = f;
        have_prev = true;
      }
      if (it >= p.max_iter) break;
      float d2 = 0.f, x2 = 0.f;
      for (int j = j0 + threadIdx.x; j < n; j += U * T) {
        CNMF_MEMBAR();
        ColGroup<K, U> cg;
        load_group<K, U>(cg, j, T, n, rx, sx, rn, sn, p.l1_num);
        CNMF_UPDATE_GROUP(cg, CNMF_NREG_CG);
        store_group<K, U>(cg, rx, sx);
      }
      ++it;
      if (!check_conv || loss_conv) continue;
      block_sum2(d2, x2, sred);
      if (coop && !coop_sum2(p, rep, epoch++, d2, x2, sred)) break;
      if (sqrtf(d2) / (sqrtf(x2) + eps) < p.tol) break;
    }
    if (p.lin_out || p.quad_out) {
      float lin = 0.f, quad = 0.f;
      for (int j = j0 + threadIdx.x; j < n; j += U * T) {
        CNMF_MEMBAR();
        ColGroup<K, U> cg;
        load_group<K, U>(cg, j, T, n, rx, sx, rn, sn, 0.f);
        CNMF_LINQUAD_GROUP(cg, CNMF_NREG_CG);
      }
      block_sum2(lin, quad, sred);
      if (coop) (void)coop_sum2(p, rep, epoch++, lin, quad, sred);
      if (threadIdx.x == 0 && (!coop || blockIdx.y == 0)) {
        if (check_conv) {
          if (p.lin_out) p.lin_out[rep] = lin;
          if (p.quad_out) p.quad_out[rep] = quad;
        } else {  // split columns: caller zeroed the outputs
          if (p.lin_out) atomicAdd(p.lin_out + rep, lin);
          if (p.quad_out) atomicAdd(p.quad_out + rep, quad);
        }
      }
    }
  }
  if (p.planes) {
    __syncthreads();   // every thread's final x stores precede the re-read (same block)
    emit_planes<K>(p, rep, j0, n, gridDim.y <= 1 || blockIdx.y == gridDim.y - 1);
  }
  if (p.iters_out && threadIdx.x == 0 && blockIdx.y == 0) p.iters_out[rep] += it;
}

template <int K, int RES>
hipError_t launch_solve_k(int algo, const SolveParams& p, int nblocks, int threads,
                          hipStream_t s) {
  if (threads > solve_block_threads<K>()) threads = solve_block_threads<K>();
  const int gy = p.nsplit > 1 ? p.nsplit : (p.coop_slots ? p.coop_epochs_split : 1);
  const dim3 grid(nblocks, gy);
  if (algo == 0)
    hipLaunchKernelGGL((solve_kernel<K, 0, RES>), grid, dim3(threads), 0, s, p);
  else
    hipLaunchKernelGGL((solve_kernel<K, 1, RES>), grid, dim3(threads), 0, s, p);
  return hipGetLastError();
}

#define CNMF_SOLVE_K_SWITCH(RES)                                                          \
  switch (K) {                                                                            \
    case 1: return launch_solve_k<1, RES>(algo, p, nblocks, threads, s);                  \
    case 2: return launch_solve_k<2, RES>(algo, p, nblocks, threads, s);                  \
    case 3: return launch_solve_k<3, RES>(algo, p, nblocks, threads, s);                  \
    case 4: return launch_solve_k<4, RES>(algo, p, nblocks, threads, s);                  \
    case 5: return launch_solve_k<5, RES>(algo, p, nblocks, threads, s);                  \
    case 6: return launch_solve_k<6, RES>(algo, p, nblocks, threads, s);                  \
    case 7: return launch_solve_k<7, RES>(algo, p, nblocks, threads, s);                  \
    case 8: return launch_solve_k<8, RES>(algo, p, nblocks, threads, s);                  \
    case 9: return launch_solve_k<9, RES>(algo, p, nblocks, threads, s);                  \
    case 10: return launch_solve_k<10, RES>(algo, p, nblocks, threads, s);                \
    case 11: return launch_solve_k<11, RES>(algo, p, nblocks, threads, s);                \
    case 12: return launch_solve_k<12, RES>(algo, p, nblocks, threads, s);                \
    case 13: return launch_solve_k<13, RES>(algo, p, nblocks, threads, s);                \
    case 14: return launch_solve_k<14, RES>(algo, p, nblocks, threads, s);                \
    case 15: return launch_solve_k<15, RES>(algo, p, nblocks, threads, s);                \
    case 16: return launch_solve_k<16, RES>(algo, p, nblocks, threads, s);                \
    case 17: return launch_solve_k<17, RES>(algo, p, nblocks, threads, s);                \
    case 18: return launch_solve_k<18, RES>(algo, p, nblocks, threads, s);                \
    case 19: return launch_solve_k<19, RES>(algo, p, nblocks, threads, s);                \
    case 20: return launch_solve_k<20, RES>(algo, p, nblocks, threads, s);                \
    case 21: return launch_solve_k<21, RES>(algo, p, nblocks, threads, s);                \
    case 22: return launch_solve_k<22, RES>(algo, p, nblocks, threads, s);                \
    case 23: return launch_solve_k<23, RES>(algo, p, nblocks, threads, s);                \
    case 24: return launch_solve_k<24, RES>(algo, p, nblocks, threads, s);                \
    case 25: return launch_solve_k<25, RES>(algo, p, nblocks, threads, s);                \
    case 26: return launch_solve_k<26, RES>(algo, p, nblocks, threads, s);                \
    case 27: return launch_solve_k<27, RES>(algo, p, nblocks, threads, s);                \
    case 28: return launch_solve_k<28, RES>(algo, p, nblocks, threads, s);                \
    case 29: return launch_solve_k<29, RES>(algo, p, nblocks, threads, s);                \
    case 30: return launch_solve_k<30, RES>(algo, p, nblocks, threads, s);                \
    case 31: return launch_solve_k<31, RES>(algo, p, nblocks, threads, s);                \
    case 32: return launch_solve_k<32, RES>(algo, p, nblocks, threads, s);                \
    default: return hipErrorInvalidValue;                                                 \
  }

// wide ranks (K padded to a multiple of 8 by the NMF engine), streaming variant only
#define CNMF_SOLVE_WIDE_SWITCH()                                                          \
  switch (K) {                                                                            \
    case 40: return launch_solve_k<40, 0>(algo, p, nblocks, threads, s);                  \
    case 48: return launch_solve_k<48, 0>(algo, p, nblocks, threads, s);                  \
    case 56: return launch_solve_k<56, 0>(algo, p, nblocks, threads, s);                  \
    case 64: return launch_solve_k<64, 0>(algo, p, nblocks, threads, s);                  \
    default: return hipErrorInvalidValue;                                                 \
  }

// register-resident variant: K <= kResidentMaxK, U <= res_max_cols(K) columns per thread
constexpr int kResidentMaxK = 24;

// Resident launch for U columns per thread: instantiated only where U <= res_max_cols(K).
template <int K, int U>
hipError_t launch_solve_res_ku(int algo, const SolveParams& p, int nblocks, int threads,
                               hipStream_t s) {
  if constexpr (U > res_max_cols(K) || K > kResidentMaxK) {
    return hipErrorInvalidValue;
  } else {
    return launch_solve_k<K, U>(algo, p, nblocks, threads, s);
  }
}

#define CNMF_SOLVE_RES_SWITCH(U)                                                          \
  switch (K) {                                                                            \
    case 1: return launch_solve_res_ku<1, U>(algo, p, nblocks, threads, s);               \
    case 2: return launch_solve_res_ku<2, U>(algo, p, nblocks, threads, s);               \
    case 3: return launch_solve_res_ku<3, U>(algo, p, nblocks, threads, s);               \
    case 4: return launch_solve_res_ku<4, U>(algo, p, nblocks, threads, s);               \
    case 5: return launch_solve_res_ku<5, U>(algo, p, nblocks, threads, s);               \
    case 6: return launch_solve_res_ku<6, U>(algo, p, nblocks, threads, s);               \
    case 7: return launch_solve_res_ku<7, U>(algo, p, nblocks, threads, s);               \
    case 8: return launch_solve_res_ku<8, U>(algo, p, nblocks, threads, s);               \
    case 9: return launch_solve_res_ku<9, U>(algo, p, nblocks, threads, s);               \
    case 10: return launch_solve_res_ku<10, U>(algo, p, nblocks, threads, s);             \
    case 11: return launch_solve_res_ku<11, U>(algo, p, nblocks, threads, s);             \
    case 12: return launch_solve_res_ku<12, U>(algo, p, nblocks, threads, s);             \
    case 13: return launch_solve_res_ku<13, U>(algo, p, nblocks, threads, s);             \
    case 14: return launch_solve_res_ku<14, U>(algo, p, nblocks, threads, s);             \
    case 15: return launch_solve_res_ku<15, U>(algo, p, nblocks, threads, s);             \
    case 16: return launch_solve_res_ku<16, U>(algo, p, nblocks, threads, s);             \
    case 17: return launch_solve_res_ku<17, U>(algo, p, nblocks, threads, s);             \
    case 18: return launch_solve_res_ku<18, U>(algo, p, nblocks, threads, s);             \
    case 19: return launch_solve_res_ku<19, U>(algo, p, nblocks, threads, s);             \
    case 20: return launch_solve_res_ku<20, U>(algo, p, nblocks, threads, s);             \
    case 21: return launch_solve_res_ku<21, U>(algo, p, nblocks, threads, s);             \
    case 22: return launch_solve_res_ku<22, U>(algo, p, nblocks, threads, s);             \
    case 23: return launch_solve_res_ku<23, U>(algo, p, nblocks, threads, s);             \
    case 24: return launch_solve_res_ku<24, U>(algo, p, nblocks, threads, s);             \
    default: return hipErrorInvalidValue;                                                 \
  }

// one per translation unit (solve.hip / solve_res.hip / solve_res34.hip build in parallel)
hipError_t launch_solve_stream(int K, int algo, const SolveParams& p, int nblocks, int threads,
                               hipStream_t s);
hipError_t launch_solve_wide(int K, int algo, const SolveParams& p, int nblocks, int threads,
                             hipStream_t s);
hipError_t launch_solve_resident(int K, int U, int algo, const SolveParams& p, int nblocks,
                                 int threads, hipStream_t s);
hipError_t launch_solve_mfma(int K, const SolveParams& p, int nblocks, int T, hipStream_t s);
hipError_t launch_solve_pipe(int K, const SolveParams& p, int nblocks, int T, int pl_n,
                             hipStream_t s);
hipError_t launch_solve_wmfma(int K, const SolveParams& p, int nblocks, bool bf16, hipStream_t s);
hipError_t launch_solve_resident34(int K, int U, int algo, const SolveParams& p, int nblocks,
                                   int threads, hipStream_t s);

}  // namespace cnmf
