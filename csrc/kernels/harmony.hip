// Harmony soft-clustering R update (harmonypy's Harmony.update_R,
// reached from preprocess.py:378-379), float64, cell-major R (N x K).
//
// One block of cells (a random 1/20th of the data set) is updated at a time:
//   E -= outer(sum_n R[n,:], Pr_b);  O -= R_b^T Phi_b            (harmony_remove_kernel)
//   Pen = ((E+1)/(O+1))^theta                                     (same kernel, last WG)
//   R[n,k] ~ exp(-dist[n,k]/sigma_k - max) * sum_v Pen[k, b_v(n)],  L1-normalised over k
//   E += outer(sum_n R[n,:], Pr_b);  O += R_b^T Phi_b             (harmony_assign_kernel)
// Each kernel is one wave per workgroup: lane l owns clusters l and l+64 (K <= 128), walks
// its chunk of cells in order and keeps per-batch sums in LDS columns it alone writes, so
// the block statistics are deterministic: per-workgroup partials are reduced in workgroup
// order by the last workgroup to arrive (self-resetting arrival counter), which also
// applies the E/O update -- no host round trip and no float atomics.
#include <hip/hip_runtime.h>

#include "common.h"

namespace cnmf {

constexpr int kHarmLanes = 64;
constexpr int kHarmKPL = 2;                 // clusters per lane (K <= 128)
constexpr int kHarmMaxKB = 4096;            // K*B doubles of LDS (32 KB per table)

struct HarmonyParams {
  double* Rt;            // N x K (row stride K)
  const double* distT;   // N x K (assign only)
  const double* sigma;   // K
  const int* cells;      // block cell ids (nb)
  const int* bidx;       // nvar x N, global batch index of each cell per covariate
  int nb, N, K, B, nvar, chunk;
  double* E;             // K x B
  double* O;             // K x B
  const double* Pr_b;    // B
  const double* theta;   // B
  double* Pen;           // K x B, written by remove, read by assign
  double* part;          // (n_wg, K*(B+1)) partial sums
  int* counter;          // 1 int, zero at rest
};

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// Write this workgroup's partials; the last workgroup reduces them in order and applies
// E += sign*outer(S, Pr_b), O += sign*Osum (and the penalty table when `pen`).
__device__ void harmony_finish(const HarmonyParams& p, const double* s, const double* o_lds,
                               double sign, bool pen) {
  const int lane = threadIdx.x;
  const int K = p.K, B = p.B;
  const long long stride = (long long)K * (B + 1);
  double* mine = p.part + (long long)blockIdx.x * stride;
#pragma unroll
  for (int j = 0; j < kHarmKPL; ++j) {
    const int k = lane + kHarmLanes * j;
    if (k < K) mine[k] = s[j];
  }
  for (int e = lane; e < K * B; e += kHarmLanes) mine[K + e] = o_lds[e];
  __shared__ int s_last;
  __threadfence();
  if (lane == 0) s_last = (atomicAdd(p.counter, 1) == (int)gridDim.x - 1);
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  // totals over workgroups, in workgroup order
  for (int e = lane; e < K * (B + 1); e += kHarmLanes) {
    double t = 0.0;
    for (int w = 0; w < (int)gridDim.x; ++w)
      t += __hip_atomic_load(p.part + (long long)w * stride + e, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    if (e < K) {
      for (int b = 0; b < B; ++b) p.E[(long long)e * B + b] += sign * t * p.Pr_b[b];
    } else {
      const int ob = e - K;             // o layout: [b][k]
      const int b = ob / K, k = ob % K;
      p.O[(long long)k * B + b] += sign * t;
    }
  }
  __syncthreads();
  __threadfence();
  if (pen) {
    for (int e = lane; e < K * B; e += kHarmLanes) {
      const int b = e % B;
      const double ev = __hip_atomic_load(p.E + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const double ov = __hip_atomic_load(p.O + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      p.Pen[e] = pow((ev + 1.0) / (ov + 1.0), p.theta[b]);
    }
  }
  if (lane == 0) *p.counter = 0;
}

__global__ void __launch_bounds__(kHarmLanes) harmony_remove_kernel(HarmonyParams p) {
  __shared__ double o_lds[kHarmMaxKB];
  const int lane = threadIdx.x;
  const int K = p.K, B = p.B;
  for (int e = lane; e < K * B; e += kHarmLanes) o_lds[e] = 0.0;
  __syncthreads();
  double s[kHarmKPL] = {0.0, 0.0};
  const int i0 = blockIdx.x * p.chunk, i1 = min(p.nb, i0 + p.chunk);
  for (int i = i0; i < i1; ++i) {
    const int n = p.cells[i];
    const double* r = p.Rt + (long long)n * K;
#pragma unroll
    for (int j = 0; j < kHarmKPL; ++j) {
      const int k = lane + kHarmLanes * j;
      if (k < K) {
        const double v = r[k];
        s[j] += v;
        for (int v_ = 0; v_ < p.nvar; ++v_) o_lds[p.bidx[(long long)v_ * p.N + n] * K + k] += v;
      }
    }
  }
  __syncthreads();
  harmony_finish(p, s, o_lds, -1.0, true);
}

__global__ void __launch_bounds__(kHarmLanes) harmony_assign_kernel(HarmonyParams p) {
  __shared__ double o_lds[kHarmMaxKB];
  __shared__ double spen[kHarmMaxKB];
  const int lane = threadIdx.x;
  const int K = p.K, B = p.B;
  for (int e = lane; e < K * B; e += kHarmLanes) {
    o_lds[e] = 0.0;
    spen[e] = p.Pen[e];
  }
  __syncthreads();
  double isig[kHarmKPL];
#pragma unroll
  for (int j = 0; j < kHarmKPL; ++j) {
    const int k = lane + kHarmLanes * j;
    isig[j] = k < K ? 1.0 / p.sigma[k] : 0.0;
  }
  double s[kHarmKPL] = {0.0, 0.0};
  const int i0 = blockIdx.x * p.chunk, i1 = min(p.nb, i0 + p.chunk);
  for (int i = i0; i < i1; ++i) {
    const int n = p.cells[i];
    const double* d = p.distT + (long long)n * K;
    double sd[kHarmKPL];
    double mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < kHarmKPL; ++j) {
      const int k = lane + kHarmLanes * j;
      sd[j] = k < K ? -d[k] * isig[j] : -INFINITY;
      mx = fmax(mx, sd[j]);
    }
    mx = wave_max_d(mx);
    double r[kHarmKPL];
    double tot = 0.0;
#pragma unroll
    for (int j = 0; j < kHarmKPL; ++j) {
      const int k = lane + kHarmLanes * j;
      double pen = 0.0;
      if (k < K)
        for (int v_ = 0; v_ < p.nvar; ++v_) pen += spen[k * B + p.bidx[(long long)v_ * p.N + n]];
      r[j] = k < K ? exp(sd[j] - mx) * pen : 0.0;
      tot += fabs(r[j]);
    }
    tot = wave_sum(tot);
    const double inv = 1.0 / tot;
    double* rout = p.Rt + (long long)n * K;
#pragma unroll
    for (int j = 0; j < kHarmKPL; ++j) {
      const int k = lane + kHarmLanes * j;
      if (k < K) {
        const double v = r[j] * inv;
        rout[k] = v;
        s[j] += v;
        for (int v_ = 0; v_ < p.nvar; ++v_) o_lds[p.bidx[(long long)v_ * p.N + n] * K + k] += v;
      }
    }
  }
  __syncthreads();
  harmony_finish(p, s, o_lds, 1.0, false);
}

}  // namespace cnmf

extern "C" int cnmf_harmony_max_kb() { return cnmf::kHarmMaxKB; }

// op 0: remove + penalty table, op 1: assign + add.  part needs
// ceil(nb/chunk) * K * (B+1) doubles; counter one zeroed int.
extern "C" hipError_t cnmf_harmony_block(int op, double* Rt, const double* distT,
                                         const double* sigma, const int* cells,
                                         const int* bidx, int nb, int N, int K, int B, int nvar,
                                         int chunk, double* E, double* O, const double* Pr_b,
                                         const double* theta, double* Pen, double* part,
                                         int* counter, hipStream_t stream) {
  if (nb <= 0) return hipSuccess;
  if (K < 1 || K > cnmf::kHarmLanes * cnmf::kHarmKPL || (long long)K * B > cnmf::kHarmMaxKB ||
      chunk < 1 || nvar < 1)
    return hipErrorInvalidValue;
  cnmf::HarmonyParams p{Rt, distT, sigma, cells, bidx, nb, N, K, B, nvar, chunk,
                        E, O, Pr_b, theta, Pen, part, counter};
  const dim3 grid((nb + chunk - 1) / chunk);
  if (op == 0)
    hipLaunchKernelGGL(cnmf::harmony_remove_kernel, grid, dim3(cnmf::kHarmLanes), 0, stream, p);
  else
    hipLaunchKernelGGL(cnmf::harmony_assign_kernel, grid, dim3(cnmf::kHarmLanes), 0, stream, p);
  return hipGetLastError();
}
