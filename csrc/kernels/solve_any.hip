// Rank-general inner solve: the Frobenius MU / HALS half-step at ANY K (SURVEY.md §2.4 G3;
// the reference's -k is unbounded, cnmf.py:1416-1417, and nmf-torch's inner loop is the
// same at every rank, cnmf.py:365-378).  The register-tiled solves (solve_core.h,
// solve_pipe.h, solve_wmfma.hip) are instantiated for K <= 128 (MU) / K <= 64 (HALS);
// this unit covers the ranks beyond them with one contract (ops.solve, the same as
// ops/reference.py:solve):
//
//  * the sweep's product D = Gram x is a plain batched GEMM (K x K times K x n per
//    replicate; rocBLAS / hipBLASLt through torch.bmm on the host side) -- at these ranks it
//    is a real GEMM (K^2 n flops per replicate) and the library runs it near the MFMA peak;
//  * everything around it is here, one pass over x each: the block objective of the
//    current x (any_obj_kernel), the MU update fused with the iterate-change terms
//    (any_mu_step_kernel), the Gauss-Seidel HALS sweep with the workgroup's column tile
//    resident in LDS (any_hals_step_kernel), and the per-replicate stop decisions
//    (any_conv_kernel) -- device-side flags, so a sweep never waits on the host.
//
// Every reduction is deterministic: a workgroup's partial goes to its own slot
// [entry][block][2] (float64) and any_conv_kernel sums the slots in block order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace cnmf {

struct AnyParams {
  float* x;                 // replicate rep's block at x + rep * x_rs, row stride ldx
  long long x_rs, ldx;
  const float* numer;
  long long n_rs, ldn;
  const float* D;           // (m, K, n) contiguous: Gram x of entry e
  const float* G;           // replicate rep's K x K Gram at G + rep * g_rs
  long long g_rs;
  const int* reps;          // entry -> replicate (nullptr: identity)
  int* act;                 // m live flags
  int m, K, n, per;         // per: columns per workgroup (grid.x = ceil(n / per))
  float l1_num, l1_den, l2, eps;
  double* part;             // [m][gridDim.x][2]
  int* iters;               // per replicate, += 1 per step taken (nullable)
};

__device__ __forceinline__ void any_block_sum2(double& a, double& b, double* sc) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int nw = (blockDim.x + kWave - 1) / kWave;
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) { sc[wid] = a; sc[nw + wid] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ta = 0.0, tb = 0.0;
    for (int w = 0; w < nw; ++w) { ta += sc[w]; tb += sc[nw + w]; }
    a = ta;
    b = tb;
  }
}

__device__ __forceinline__ float any_num(const AnyParams& p, float v) {
  return p.l1_num > 0.f ? fmaxf(v - p.l1_num, 0.f) : v;
}

// MODE 0: objective pieces of the current x of a live entry -- sum x (Dx + l2 x) and
// sum x (numer' - l1_den).  MODE 1: the epilogue's lin = <raw numer, x>, quad = x^T D.
template <int MODE>
__global__ __launch_bounds__(256) void any_obj_kernel(AnyParams p) {
  __shared__ double sc[8];
  const int e = blockIdx.y;
  const int rep = p.reps ? p.reps[e] : e;
  double* slot = p.part + ((long long)e * gridDim.x + blockIdx.x) * 2;
  if (MODE == 0 && p.act[e] == 0) {       // uniform per workgroup
    if (threadIdx.x == 0) { slot[0] = 0.0; slot[1] = 0.0; }
    return;
  }
  const float* x = p.x + rep * p.x_rs;
  const float* nu = p.numer + rep * p.n_rs;
  const float* d = p.D + (long long)e * p.K * p.n;
  const int j0 = blockIdx.x * p.per, j1 = min(p.n, j0 + p.per);
  double qa = 0.0, la = 0.0;
  for (int k = 0; k < p.K; ++k) {
    float q = 0.f, l = 0.f;          // one row in fp32, rows summed in fp64
    for (int j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
      const float xv = x[k * p.ldx + j], dv = d[(long long)k * p.n + j];
      const float nv = nu[k * p.ldn + j];
      if (MODE == 0) {
        q = fmaf(xv, fmaf(p.l2, xv, dv), q);
        l = fmaf(xv, any_num(p, nv) - p.l1_den, l);
      } else {
        q = fmaf(xv, dv, q);
        l = fmaf(xv, nv, l);
      }
    }
    qa += q;
    la += l;
  }
  any_block_sum2(qa, la, sc);
  if (threadIdx.x == 0) { slot[0] = qa; slot[1] = la; }
}

// x <- x * numer' / (D + l2 x + l1_den), 0 where that denominator is < eps (the rate of
// solve_core.h); TRACK: partials of |x_new - x|^2 and |x|^2 for the iterate-change stop.
template <bool TRACK>
__global__ __launch_bounds__(256) void any_mu_step_kernel(AnyParams p) {
  __shared__ double sc[8];
  const int e = blockIdx.y;
  if (p.act[e] == 0) return;
  const int rep = p.reps ? p.reps[e] : e;
  float* x = p.x + rep * p.x_rs;
  const float* nu = p.numer + rep * p.n_rs;
  const float* d = p.D + (long long)e * p.K * p.n;
  const int j0 = blockIdx.x * p.per, j1 = min(p.n, j0 + p.per);
  double da = 0.0, xa = 0.0;
  for (int k = 0; k < p.K; ++k) {
    float d2 = 0.f, x2 = 0.f;
    for (int j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
      const float xv = x[k * p.ldx + j];
      const float den = fmaf(p.l2, xv, d[(long long)k * p.n + j]) + p.l1_den;
      const float xn = den < p.eps ? 0.f : xv * (any_num(p, nu[k * p.ldn + j]) / den);
      x[k * p.ldx + j] = xn;
      if (TRACK) {
        const float dd = xn - xv;
        d2 = fmaf(dd, dd, d2);
        x2 = fmaf(xv, xv, x2);
      }
    }
    da += d2;
    xa += x2;
  }
  if (p.iters && blockIdx.x == 0 && threadIdx.x == 0) p.iters[rep] += 1;
  if (!TRACK) return;
  any_block_sum2(da, xa, sc);
  if (threadIdx.x == 0) {
    double* slot = p.part + ((long long)e * gridDim.x + blockIdx.x) * 2;
    slot[0] = da;
    slot[1] = xa;
  }
}

// One Gauss-Seidel HALS sweep over the components (reference.py _step, algo 1): lane t
// owns column j0 + t, its K values in LDS (column-major per lane: word k * 64 + t, so the
// 64 lanes hit 64 banks); x_k <- max(x_k + (numer'_k - l1_den - G_k x - l2 x_k) /
// (G_kk + l2), 0), kept when G_kk + l2 <= eps.  The Gram row G_k is wave-uniform (scalar
// loads).  One wave per workgroup, 64 columns: K <= 512 (128 KB of LDS).
template <bool TRACK>
__global__ __launch_bounds__(64) void any_hals_step_kernel(AnyParams p) {
  extern __shared__ float xs[];          // [K][64]
  const int e = blockIdx.y;
  if (p.act[e] == 0) return;
  const int rep = p.reps ? p.reps[e] : e;
  float* x = p.x + rep * p.x_rs;
  const float* nu = p.numer + rep * p.n_rs;
  const float* g = p.G + rep * p.g_rs;
  const int t = threadIdx.x, j = blockIdx.x * 64 + t;
  const bool ok = j < p.n;
  const int K = p.K;
  for (int k = 0; k < K; ++k) xs[k * 64 + t] = ok ? x[k * p.ldx + j] : 0.f;
  double da = 0.0, xa = 0.0;
  for (int k = 0; k < K; ++k) {
    const float* gk = g + (long long)k * K;
    float gx0 = 0.f, gx1 = 0.f, gx2 = 0.f, gx3 = 0.f;
    int i = 0;
    for (; i + 4 <= K; i += 4) {
      gx0 = fmaf(gk[i], xs[i * 64 + t], gx0);
      gx1 = fmaf(gk[i + 1], xs[(i + 1) * 64 + t], gx1);
      gx2 = fmaf(gk[i + 2], xs[(i + 2) * 64 + t], gx2);
      gx3 = fmaf(gk[i + 3], xs[(i + 3) * 64 + t], gx3);
    }
    for (; i < K; ++i) gx0 = fmaf(gk[i], xs[i * 64 + t], gx0);
    const float gx = (gx0 + gx1) + (gx2 + gx3);
    const float diag = gk[k] + p.l2;
    const float old = xs[k * 64 + t];
    const float nv = ok ? any_num(p, nu[k * p.ldn + j]) : 0.f;
    const float upd = fmaxf(old + (nv - p.l1_den - gx - p.l2 * old) / diag, 0.f);
    const float xn = (diag > p.eps && ok) ? upd : old;
    xs[k * 64 + t] = xn;
    if (TRACK) {
      const float dd = xn - old;
      da += (double)dd * dd;
      xa += (double)old * old;
    }
  }
  if (ok)
    for (int k = 0; k < K; ++k) x[k * p.ldx + j] = xs[k * 64 + t];
  if (p.iters && blockIdx.x == 0 && t == 0) p.iters[rep] += 1;
  if (!TRACK) return;
  da = wave_sum(da);
  xa = wave_sum(xa);
  if (t == 0) {
    double* slot = p.part + ((long long)e * gridDim.x + blockIdx.x) * 2;
    slot[0] = da;
    slot[1] = xa;
  }
}

// Per-entry decisions from the partials (summed in block order).  mode 0: block-objective
// stop (|f_prev - f| <= tol |f_prev| once a previous value exists); mode 1: iterate-change
// stop (|dx| / (|x| + eps) < tol); mode 2: write lin / quad of the entries live at entry
// (act0) to lin_out / quad_out.
__global__ void any_conv_kernel(int mode, const double* __restrict__ part, int nblk, int m,
                                int* act, const int* act0, const int* reps, double* f_prev,
                                int have_prev, float tol, float eps, float* lin_out,
                                float* quad_out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= m) return;
  if (mode == 2 ? act0[e] == 0 : act[e] == 0) return;
  double a = 0.0, b = 0.0;
  const double* s = part + (long long)e * nblk * 2;
  for (int i = 0; i < nblk; ++i) { a += s[2 * i]; b += s[2 * i + 1]; }
  if (mode == 0) {
    const float f = (float)(a - 2.0 * b);
    if (have_prev && fabsf((float)f_prev[e] - f) <= tol * fabsf((float)f_prev[e])) act[e] = 0;
    f_prev[e] = f;
  } else if (mode == 1) {
    if ((float)(sqrt(a) / (sqrt(b) + (double)eps)) < tol) act[e] = 0;
  } else {
    const int rep = reps ? reps[e] : e;
    if (lin_out) lin_out[rep] = (float)b;
    if (quad_out) quad_out[rep] = (float)a;
  }
}

}  // namespace cnmf

extern "C" int cnmf_solve_any_hals_max_k() { return 512; }

// op: 0 objective (live entries), 1 final lin / quad terms, 2 MU step, 3 MU step + change
// terms, 4 HALS sweep, 5 HALS sweep + change terms.  Returns the grid's x extent through
// *nblk_out (the partial slots per entry the decision kernel sums).
extern "C" hipError_t cnmf_solve_any(int op, float* x, long long x_rs, long long ldx,
                                     const float* numer, long long n_rs, long long ldn,
                                     const float* D, const float* G, long long g_rs,
                                     const int* reps, int* act, int m, int K, int n, int per,
                                     float l1_num, float l1_den, float l2, float eps,
                                     double* part, int* iters, hipStream_t stream) {
  if (m <= 0 || n <= 0 || K <= 0) return hipSuccess;
  if ((long long)K * (ldx > ldn ? ldx : ldn) >= 0x7fffffffLL) return hipErrorInvalidValue;
  cnmf::AnyParams p;
  p.x = x; p.x_rs = x_rs; p.ldx = ldx;
  p.numer = numer; p.n_rs = n_rs; p.ldn = ldn;
  p.D = D; p.G = G; p.g_rs = g_rs;
  p.reps = reps; p.act = act;
  p.m = m; p.K = K; p.n = n;
  p.l1_num = l1_num; p.l1_den = l1_den; p.l2 = l2; p.eps = eps;
  p.part = part; p.iters = iters;
  if (op >= 4) {
    if (K > cnmf_solve_any_hals_max_k() || !G) return hipErrorInvalidValue;
    p.per = 64;
    const dim3 grid((n + 63) / 64, m);
    const size_t lds = (size_t)K * 64 * sizeof(float);
    if (lds > (64 << 10)) {
      const void* f = op == 5 ? reinterpret_cast<const void*>(&cnmf::any_hals_step_kernel<true>)
                              : reinterpret_cast<const void*>(&cnmf::any_hals_step_kernel<false>);
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds);
      if (e != hipSuccess) return e;
    }
    if (op == 5)
      hipLaunchKernelGGL(cnmf::any_hals_step_kernel<true>, grid, dim3(64), lds, stream, p);
    else
      hipLaunchKernelGGL(cnmf::any_hals_step_kernel<false>, grid, dim3(64), lds, stream, p);
    return hipGetLastError();
  }
  if (!D || per < 1) return hipErrorInvalidValue;
  p.per = per;
  const dim3 grid((n + per - 1) / per, m);
  switch (op) {
    case 0: hipLaunchKernelGGL(cnmf::any_obj_kernel<0>, grid, dim3(256), 0, stream, p); break;
    case 1: hipLaunchKernelGGL(cnmf::any_obj_kernel<1>, grid, dim3(256), 0, stream, p); break;
    case 2: hipLaunchKernelGGL(cnmf::any_mu_step_kernel<false>, grid, dim3(256), 0, stream, p); break;
    case 3: hipLaunchKernelGGL(cnmf::any_mu_step_kernel<true>, grid, dim3(256), 0, stream, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t cnmf_solve_any_conv(int mode, const double* part, int nblk, int m,
                                          int* act, const int* act0, const int* reps,
                                          double* f_prev, int have_prev, float tol, float eps,
                                          float* lin_out, float* quad_out, hipStream_t stream) {
  if (m <= 0) return hipSuccess;
  if (mode < 0 || mode > 2) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnmf::any_conv_kernel, dim3((m + 63) / 64), dim3(64), 0, stream, mode, part,
                     nblk, m, act, act0, reps, f_prev, have_prev, tol, eps, lin_out, quad_out);
  return hipGetLastError();
}
