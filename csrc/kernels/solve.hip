// Fused, replicate-batched NNLS-style inner solvers for NMF.
//
// Both halves of a Frobenius NMF step reduce to the same problem
//     minimise_x  ||numer - Gram x|| style updates, independently per column j,
// with a convergence test on the WHOLE (replicate, chunk) block:
//   H-side  (cnmf.py:352-381 fit_H_online; nmf-torch online H step):
//       x = h^T (K x c), numer = W x^T (K x c), Gram = W W^T
//   W-side  (nmf-torch online/batch W step):
//       x = W (K x G),   numer = B = sum h^T x,  Gram = A = sum h^T h
// One workgroup owns one replicate's block, iterates the update in-place from L2,
// reduces ||dx|| and ||x|| on device and stops when ||dx||/(||x||+eps) < tol.  There
// is no per-iteration kernel launch and no host sync (the reference syncs every
// iteration at cnmf.py:377).  A grid covers every active replicate of a batch, so one
// launch drives the whole replicate grid.
//
// ALGO 0 = multiplicative update (MU):  x <- x * numer / (Gram x + l2 x + l1_den),
//          rate := 0 where the denominator < eps (cnmf.py:370-372).
// ALGO 1 = HALS (Gauss-Seidel over components):
//          x_k <- max(0, x_k + (numer_k - l1_den - (Gram x)_k - l2 x_k) / (Gram_kk + l2)).
// Optional epilogue: lin_out[r] = <numer, x>, quad_out[r] = sum_j x_j^T Gram x_j, which
// give the exact Frobenius loss from sufficient statistics (trace trick, G7).
#include <hip/hip_runtime.h>
#include "common.h"

namespace cnmf {

struct SolveParams {
  float* x;
  long long x_rs, ldx;
  const float* numer;
  long long n_rs, ldn;
  const float* gram;
  long long g_rs;
  const int* rep_index;
  int ncols, max_iter;
  float tol, l1_num, l1_den, l2, eps;
  float* lin_out;
  float* quad_out;
  int* iters_out;
  int nsplit;       // >1: blockIdx.y splits the columns; single fixed step, no convergence test
  int conv_mode;    // 0: ||dx||/(||x||+eps) < tol after every step (cnmf.py:375-378)
                    // 1: block objective checked every `check_every` steps,
                    //    |f_prev - f| / |f_prev| < tol  (nmf-torch online inner loops)
  int check_every;
};

// Block objective (x2, dropping the constant ||X||^2):
//   f(x) = sum_j x_j^T Gram x_j - 2 numer_j . x_j + 2 l1 |x_j|_1 + l2 |x_j|^2
template <int K>
__device__ __forceinline__ float block_objective(const float* __restrict__ x, long long ldx,
                                                 const float* __restrict__ nu, long long ldn,
                                                 const float* sG, int j0, int n, float l1_num,
                                                 float l1, float l2, float* sred) {
  float q = 0.f, l = 0.f;
  for (int j = j0 + threadIdx.x; j < n; j += blockDim.x) {
    float xv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) xv[k] = x[k * ldx + j];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float gx = 0.f;
#pragma unroll
      for (int kk = 0; kk < K; ++kk) gx = fmaf(sG[k * K + kk], xv[kk], gx);
      float t = nu[k * ldn + j];
      if (l1_num > 0.f) t = fmaxf(t - l1_num, 0.f);
      q = fmaf(xv[k], gx + l2 * xv[k], q);
      l = fmaf(xv[k], t - l1, l);
    }
  }
  block_sum2(q, l, sred);
  return q - 2.f * l;
}

template <int K>
constexpr int solve_max_threads() { return K <= 16 ? 1024 : 512; }

template <int K, int ALGO>
__global__ __launch_bounds__(solve_max_threads<K>()) void solve_kernel(SolveParams p) {
  __shared__ float sG[K * K];
  __shared__ float sred[2 * 16];
  const int rep = p.rep_index ? p.rep_index[blockIdx.x] : (int)blockIdx.x;
  float* __restrict__ x = p.x + (long long)rep * p.x_rs;
  const float* __restrict__ nu = p.numer + (long long)rep * p.n_rs;
  const float* __restrict__ g = p.gram + (long long)rep * p.g_rs;
  for (int i = threadIdx.x; i < K * K; i += blockDim.x) sG[i] = g[i];
  __syncthreads();

  const long long ldx = p.ldx, ldn = p.ldn;
  // Column range of this block: the whole block (nsplit == 1) or one of nsplit slices.
  int j0 = 0, n = p.ncols;
  if (p.nsplit > 1) {
    const int per = (p.ncols + p.nsplit - 1) / p.nsplit;
    j0 = blockIdx.y * per;
    n = min(p.ncols, j0 + per);
  }
  const bool check_conv = p.nsplit <= 1;
  const bool loss_conv = check_conv && p.conv_mode == 1;
  const int every = p.check_every > 0 ? p.check_every : 1;
  float f_prev = 0.f;
  bool have_prev = false;
  int it = 0;
  while (true) {
    if (loss_conv && it % every == 0) {
      const float f = block_objective<K>(x, ldx, nu, ldn, sG, j0, n, p.l1_num, p.l1_den, p.l2,
                                         sred);
      if (have_prev && fabsf(f_prev - f) <= p.tol * fabsf(f_prev)) break;
      f_prev = f;
      have_prev = true;
    }
    if (it >= p.max_iter) break;
    float d2 = 0.f, x2 = 0.f;
    for (int j = j0 + threadIdx.x; j < n; j += blockDim.x) {
      float xv[K], nv[K];
#pragma unroll
      for (int k = 0; k < K; ++k) xv[k] = x[k * ldx + j];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float t = nu[k * ldn + j];
        if (p.l1_num > 0.f) t = fmaxf(t - p.l1_num, 0.f);
        nv[k] = t;
      }
      if (ALGO == 0) {
        float xn[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          float den = 0.f;
#pragma unroll
          for (int kk = 0; kk < K; ++kk) den = fmaf(sG[k * K + kk], xv[kk], den);
          den = fmaf(p.l2, xv[k], den) + p.l1_den;
          xn[k] = (den < p.eps) ? 0.f : xv[k] * (nv[k] / den);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float d = xn[k] - xv[k];
          d2 = fmaf(d, d, d2);
          x2 = fmaf(xv[k], xv[k], x2);
          x[k * ldx + j] = xn[k];
        }
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          float gx = 0.f;
#pragma unroll
          for (int kk = 0; kk < K; ++kk) gx = fmaf(sG[k * K + kk], xv[kk], gx);
          const float diag = sG[k * K + k] + p.l2;
          const float old = xv[k];
          float xn = old;
          if (diag > p.eps) xn = fmaxf(old + (nv[k] - p.l1_den - gx - p.l2 * old) / diag, 0.f);
          const float d = xn - old;
          d2 = fmaf(d, d, d2);
          x2 = fmaf(old, old, x2);
          xv[k] = xn;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) x[k * ldx + j] = xv[k];
      }
    }
    ++it;
    if (!check_conv || loss_conv) continue;
    block_sum2(d2, x2, sred);
    if (sqrtf(d2) / (sqrtf(x2) + p.eps) < p.tol) break;
  }

  if (p.lin_out || p.quad_out) {
    float lin = 0.f, quad = 0.f;
    for (int j = j0 + threadIdx.x; j < n; j += blockDim.x) {
      float xv[K];
#pragma unroll
      for (int k = 0; k < K; ++k) xv[k] = x[k * ldx + j];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        lin = fmaf(nu[k * ldn + j], xv[k], lin);
        float gx = 0.f;
#pragma unroll
        for (int kk = 0; kk < K; ++kk) gx = fmaf(sG[k * K + kk], xv[kk], gx);
        quad = fmaf(xv[k], gx, quad);
      }
    }
    block_sum2(lin, quad, sred);
    if (threadIdx.x == 0) {
      if (check_conv) {
        if (p.lin_out) p.lin_out[rep] = lin;
        if (p.quad_out) p.quad_out[rep] = quad;
      } else {  // split columns: caller zeroed the outputs
        if (p.lin_out) atomicAdd(p.lin_out + rep, lin);
        if (p.quad_out) atomicAdd(p.quad_out + rep, quad);
      }
    }
  }
  if (p.iters_out && threadIdx.x == 0 && blockIdx.y == 0) p.iters_out[rep] = it;
}

template <int K>
hipError_t launch_solve_k(int algo, const SolveParams& p, int nblocks, int threads,
                          hipStream_t s) {
  const int tmax = solve_max_threads<K>();
  if (threads > tmax) threads = tmax;
  const dim3 grid(nblocks, p.nsplit > 1 ? p.nsplit : 1);
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

extern "C" int cnmf_solve_max_threads(int K) { return K <= 16 ? 1024 : 512; }

extern "C" hipError_t cnmf_solve(int algo, int K, float* x, long long x_rs, long long ldx,
                                 const float* numer, long long n_rs, long long ldn,
                                 const float* gram, long long g_rs, const int* rep_index,
                                 int nblocks, int ncols, int max_iter, float tol, float l1_num,
                                 float l1_den, float l2, float eps, float* lin_out,
                                 float* quad_out, int* iters_out, int nsplit, int conv_mode,
                                 int check_every, int threads, hipStream_t stream) {
  if (nblocks <= 0) return hipSuccess;
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
