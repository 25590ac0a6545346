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
#include <hip/hip_runtime.h>
#include "common.h"
#include "solve_params.h"

namespace cnmf {

template <int K>
constexpr int solve_max_threads() { return 1024; }

// Columns per thread per group: keep ~(2U+1)K live floats well under the 128-VGPR cap.
template <int K>
constexpr int cols_per_group() { return (20 / K) < 1 ? 1 : ((20 / K) > 4 ? 4 : (20 / K)); }

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

__device__ __forceinline__ const lds_float* opaque(const lds_float* p) {
  asm volatile("" : "+v"(p));
  return p;
}

template <int K, int U>
struct ColGroup {
  float x[U][K];
  float n[U][K];
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
// Each workgroup stores its block totals to its own slot (plain store), drains, then
// arrives on the epoch counter with an agent-scope release; after all S arrived every
// workgroup sums the S slots in slice order -> identical, deterministic totals
// everywhere.  Spins are bounded: on timeout the flag is raised and the host fails.
// (Recipe: cdna_hip_programming.md Guideline 16 -- release before the counter add,
// acquire after the poll, vmcnt drained around the fence.)
__device__ __forceinline__ void coop_sum2(const SolveParams& p, int rep, int e, float& a,
                                          float& b, float* sred) {
  const int S = gridDim.y;
  const int slice = blockIdx.y;
  if (S <= 1) return;
  if (e >= p.coop_epochs) {  // workspace too small: treat as timeout (host sizes it)
    if (threadIdx.x == 0) atomicExch(p.coop_timeout, 2);
    return;
  }
  float* slots = p.coop_slots + (((long long)rep * p.coop_epochs + e) * S) * 2;
  int* cnt = p.coop_count + (long long)rep * p.coop_epochs + e;
  if (threadIdx.x == 0) {
    slots[2 * slice] = a;
    slots[2 * slice + 1] = b;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 24)) {
        atomicExch(p.coop_timeout, 1);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    float ta = 0.f, tb = 0.f;
    for (int s2 = 0; s2 < S; ++s2) {
      ta += __hip_atomic_load(slots + 2 * s2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tb += __hip_atomic_load(slots + 2 * s2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    sred[0] = ta;
    sred[1] = tb;
  }
  __syncthreads();
  a = sred[0];
  b = sred[1];
  __syncthreads();
}

// Block objective (x2, dropping the constant ||X||^2):
//   f(x) = sum_j x_j^T Gram x_j - 2 numer_j . x_j + 2 l1 |x_j|_1 + l2 |x_j|^2
template <int K, int U>
__device__ __forceinline__ float block_objective(__amdgpu_buffer_rsrc_t rx, int sx,
                                                 __amdgpu_buffer_rsrc_t rn, int sn,
                                                 const lds_float* sG, int j0, int n, float l1_num,
                                                 float l1, float l2, float* sred) {
  float q = 0.f, l = 0.f;
  const int T = blockDim.x;
  for (int j = j0 + threadIdx.x; j < n; j += U * T) {
    CNMF_MEMBAR();
    ColGroup<K, U> cg;
    load_group<K, U>(cg, j, T, n, rx, sx, rn, sn, l1_num);
    const lds_float* gz = opaque(sG);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        CNMF_MEMBAR();
        float gx = 0.f;
#pragma unroll
        for (int kk = 0; kk < K; ++kk) gx = fmaf(gz[k * K + kk], cg.x[u][kk], gx);
        q = fmaf(cg.x[u][k], gx + l2 * cg.x[u][k], q);
        l = fmaf(cg.x[u][k], cg.n[u][k] - l1, l);
      }
    }
  }
  block_sum2(q, l, sred);
  return q - 2.f * l;
}

template <int K, int ALGO>
__global__ __launch_bounds__(1024) void solve_kernel(SolveParams p) {
  constexpr int U = cols_per_group<K>();
  __shared__ float sGm[K * K];
  __shared__ float sred[2 * 16];
  const lds_float* sG = (const lds_float*)sGm;  // LDS (addrspace 3): ds_read, 32-bit address
  const int rep = p.rep_index ? p.rep_index[blockIdx.x] : (int)blockIdx.x;
  if (p.active && p.active[rep] == 0) return;  // converged replicate: untouched (uniform)
  float* __restrict__ x = p.x + (long long)rep * p.x_rs;
  const float* __restrict__ nu = p.numer + (long long)rep * p.n_rs;
  const float* __restrict__ g = p.gram + (long long)rep * p.g_rs;
  for (int i = threadIdx.x; i < K * K; i += blockDim.x) sGm[i] = g[i];
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
  while (true) {
    if (loss_conv && it % every == 0) {
      float f = block_objective<K, U>(rx, sx, rn, sn, sG, j0, n, p.l1_num, l1, l2, sred);
      if (coop) {
        float unused = 0.f;
        coop_sum2(p, rep, epoch++, f, unused, sred);
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
      const lds_float* gz = opaque(sG);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ALGO == 0) {
          // Jacobi step, row-wise: xn_k from the OLD x, written back after all k
          float xn[K];
#pragma unroll
          for (int k = 0; k < K; ++k) {
            CNMF_MEMBAR();
            float den = 0.f;
#pragma unroll
            for (int kk = 0; kk < K; ++kk) den = fmaf(gz[k * K + kk], cg.x[u][kk], den);
            den = fmaf(l2, cg.x[u][k], den) + l1;
            xn[k] = (den < eps) ? 0.f : cg.x[u][k] * (cg.n[u][k] * __builtin_amdgcn_rcpf(den));
          }
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const float d = xn[k] - cg.x[u][k];
            d2 = fmaf(d, d, d2);
            x2 = fmaf(cg.x[u][k], cg.x[u][k], x2);
            cg.x[u][k] = xn[k];
          }
        } else {
#pragma unroll
          for (int k = 0; k < K; ++k) {
            CNMF_MEMBAR();
            float gx = 0.f;
#pragma unroll
            for (int kk = 0; kk < K; ++kk) gx = fmaf(gz[k * K + kk], cg.x[u][kk], gx);
            const float diag = gz[k * K + k] + l2;
            const float old = cg.x[u][k];
            float xn = old;
            if (diag > eps) xn = fmaxf(old + (cg.n[u][k] - l1 - gx - l2 * old) / diag, 0.f);
            const float d = xn - old;
            d2 = fmaf(d, d, d2);
            x2 = fmaf(old, old, x2);
            cg.x[u][k] = xn;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (cg.ok[u]) {
#pragma unroll
          for (int k = 0; k < K; ++k)
            buf_st(cg.x[u][k], rx, cg.vo[u], k * sx);
        }
      }
    }
    ++it;
    if (!check_conv || loss_conv) continue;
    block_sum2(d2, x2, sred);
    if (coop) coop_sum2(p, rep, epoch++, d2, x2, sred);
    if (sqrtf(d2) / (sqrtf(x2) + eps) < p.tol) break;
  }

  if (p.lin_out || p.quad_out) {
    float lin = 0.f, quad = 0.f;
    for (int j = j0 + threadIdx.x; j < n; j += U * T) {
      CNMF_MEMBAR();
      ColGroup<K, U> cg;
      load_group<K, U>(cg, j, T, n, rx, sx, rn, sn, 0.f);
      const lds_float* gz = opaque(sG);
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          CNMF_MEMBAR();
          float gx = 0.f;
#pragma unroll
          for (int kk = 0; kk < K; ++kk) gx = fmaf(gz[k * K + kk], cg.x[u][kk], gx);
          lin = fmaf(cg.n[u][k], cg.x[u][k], lin);
          quad = fmaf(cg.x[u][k], gx, quad);
        }
      }
    }
    block_sum2(lin, quad, sred);
    if (coop) coop_sum2(p, rep, epoch++, lin, quad, sred);
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
  if (p.iters_out && threadIdx.x == 0 && blockIdx.y == 0) p.iters_out[rep] += it;
}

template <int K>
hipError_t launch_solve_k(int algo, const SolveParams& p, int nblocks, int threads,
                          hipStream_t s) {
  const int tmax = solve_max_threads<K>();
  if (threads > tmax) threads = tmax;
  const int gy = p.nsplit > 1 ? p.nsplit : (p.coop_slots ? p.coop_epochs_split : 1);
  const dim3 grid(nblocks, gy);
  if (algo == 0)
    hipLaunchKernelGGL((solve_kernel<K, 0>), grid, dim3(threads), 0, s, p);
  else
    hipLaunchKernelGGL((solve_kernel<K, 1>), grid, dim3(threads), 0, s, p);
  return hipGetLastError();
}

}  // namespace cnmf

#define CNMF_K_CASE(KK) \
  case KK:              \
    return cnmf::launch_solve_k<KK>(algo, p, nblocks, threads, stream);

extern "C" int cnmf_solve_max_k() { return 32; }

extern "C" int cnmf_solve_max_threads(int K) { return 1024; }

extern "C" int cnmf_solve_reg_max_cols(int K) { return 0; }

extern "C" hipError_t cnmf_solve(int algo, int K, float* x, long long x_rs, long long ldx,
                                 const float* numer, long long n_rs, long long ldn,
                                 const float* gram, long long g_rs, const int* rep_index,
                                 int nblocks, int ncols, int max_iter, float tol, float l1_num,
                                 float l1_den, float l2, float eps, float* lin_out,
                                 float* quad_out, int* iters_out, int nsplit, int conv_mode,
                                 int check_every, int threads, int variant,
                                 const int* active, int coop_split, float* coop_slots,
                                 int* coop_count, int coop_epochs, int* coop_timeout,
                                 hipStream_t stream) {
  if (nblocks <= 0) return hipSuccess;
  // buffer offsets are 32-bit: a replicate's block must span < 2 GiB
  if ((long long)K * (ldx > ldn ? ldx : ldn) * 4 >= 0x7fffffffLL) return hipErrorInvalidValue;
  cnmf::SolveParams p;
  p.x = x; p.x_rs = x_rs; p.ldx = ldx;
  p.numer = numer; p.n_rs = n_rs; p.ldn = ldn;
  p.gram = gram; p.g_rs = g_rs;
  p.rep_index = rep_index;
  p.ncols = ncols; p.max_iter = max_iter;
  p.tol = tol; p.l1_num = l1_num; p.l1_den = l1_den; p.l2 = l2; p.eps = eps;
  p.lin_out = lin_out; p.quad_out = quad_out; p.iters_out = iters_out;
  p.nsplit = nsplit;
  p.conv_mode = conv_mode;
  p.check_every = check_every;
  p.active = active;
  p.coop_slots = coop_split > 1 ? coop_slots : nullptr;
  p.coop_count = coop_count;
  p.coop_epochs = coop_epochs;
  p.coop_timeout = coop_timeout;
  p.coop_epochs_split = coop_split > 1 ? coop_split : 1;
  if (coop_split > 1 && nsplit > 1) return hipErrorInvalidValue;
  (void)variant;
  switch (K) {
    CNMF_K_CASE(1) CNMF_K_CASE(2) CNMF_K_CASE(3) CNMF_K_CASE(4) CNMF_K_CASE(5) CNMF_K_CASE(6)
    CNMF_K_CASE(7) CNMF_K_CASE(8) CNMF_K_CASE(9) CNMF_K_CASE(10) CNMF_K_CASE(11)
    CNMF_K_CASE(12) CNMF_K_CASE(13) CNMF_K_CASE(14) CNMF_K_CASE(15) CNMF_K_CASE(16)
    CNMF_K_CASE(17) CNMF_K_CASE(18) CNMF_K_CASE(19) CNMF_K_CASE(20) CNMF_K_CASE(21)
    CNMF_K_CASE(22) CNMF_K_CASE(23) CNMF_K_CASE(24) CNMF_K_CASE(25) CNMF_K_CASE(26)
    CNMF_K_CASE(27) CNMF_K_CASE(28) CNMF_K_CASE(29) CNMF_K_CASE(30) CNMF_K_CASE(31)
    CNMF_K_CASE(32)
    default:
      return hipErrorInvalidValue;
  }
}
