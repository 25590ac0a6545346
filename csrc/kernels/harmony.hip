// Harmony soft-clustering R update (harmonypy's Harmony.update_R,
// reached from preprocess.py:378-379), float64, cell-major R (N x K).
//
// One block of cells (a random 1/20th of the data set) is updated at a time:
//   E -= outer(sum_n R[n,:], Pr_b);  O -= R_b^T Phi_b            (op 0: remove)
//   Pen = ((E+1)/(O+1))^theta                                     (op 0, reduce kernel)
//   R[n,k] ~ exp(-dist[n,k]/sigma_k - max) * sum_v Pen[k, b_v(n)],  L1-normalised over k
//   E += outer(sum_n R[n,:], Pr_b);  O += R_b^T Phi_b             (op 1: assign + add)
// harmony_block_kernel: up to 4 waves per workgroup, each wave walks its own cells (lane l
// owns clusters l and l+64, K <= 128) and keeps the per-batch sums O in an LDS table of
// its own, so no two waves touch one word; the waves' tables and cluster sums are added
// in wave order into the workgroup's partial row.  harmony_reduce_kernel: one wave per
// (k, b) sums the workgroups' partials in a fixed order and applies the E/O update (and
// the penalty table) -- deterministic, no float atomics, no host round trip.
// The first generation ran one wave per workgroup and had the last-arriving wave reduce
// every partial alone: 1.8 ms per op on a 25k-cell block (profiles/r3q_harmony_500k_*).
#include <hip/hip_runtime.h>

#include "common.h"

namespace cnmf {

constexpr int kHarmLanes = 64;
constexpr int kHarmKPL = 2;                 // clusters per lane (K <= 128)
constexpr int kHarmMaxKB = 4096;            // K*B doubles per table
constexpr int kHarmLdsBytes = 152 * 1024;   // dynamic LDS budget of the block kernel

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
  double* Pen;           // K x B, written by op 0's reduce, read by op 1
  double* part;          // (n_wg, K*(B+1)) partial sums: [k] cluster sums, then [b][k] O sums
};

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// LDS doubles of a W-wave block kernel: W O-tables, the penalty table (assign), W K-sums
__host__ __device__ constexpr long long harmony_lds_doubles(int W, int K, int B, bool assign) {
  return (long long)W * K * B + (assign ? (long long)K * B : 0) + (long long)W * K;
}

template <bool ASSIGN>
__global__ void __launch_bounds__(4 * kHarmLanes) harmony_block_kernel(HarmonyParams p) {
  extern __shared__ __attribute__((aligned(16))) double hsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, W = blockDim.x >> 6;
  const int K = p.K, B = p.B, KB = K * B;
  double* o_w = hsm + (long long)wave * KB;          // this wave's O table, [b][k]
  double* spen = hsm + (long long)W * KB;            // penalty table (assign)
  double* ksum = spen + (ASSIGN ? KB : 0);           // [W][K] cluster sums
  for (int e = threadIdx.x; e < W * KB; e += blockDim.x) hsm[e] = 0.0;
  if (ASSIGN)
    for (int e = threadIdx.x; e < KB; e += blockDim.x) spen[e] = p.Pen[e];
  __syncthreads();
  double isig[kHarmKPL];
#pragma unroll
  for (int j = 0; j < kHarmKPL; ++j) {
    const int k = lane + kHarmLanes * j;
    isig[j] = (ASSIGN && k < K) ? 1.0 / p.sigma[k] : 0.0;
  }
  double s[kHarmKPL] = {0.0, 0.0};
  const int i0 = blockIdx.x * p.chunk, i1 = min(p.nb, i0 + p.chunk);
  for (int i = i0 + wave; i < i1; i += W) {
    const int n = p.cells[i];
    double* rr = p.Rt + (long long)n * K;
    double r[kHarmKPL];
    if (ASSIGN) {
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
#pragma unroll
      for (int j = 0; j < kHarmKPL; ++j) {
        const int k = lane + kHarmLanes * j;
        r[j] *= inv;
        if (k < K) rr[k] = r[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < kHarmKPL; ++j) {
        const int k = lane + kHarmLanes * j;
        r[j] = k < K ? rr[k] : 0.0;
      }
    }
#pragma unroll
    for (int j = 0; j < kHarmKPL; ++j) {
      const int k = lane + kHarmLanes * j;
      if (k < K) {
        s[j] += r[j];
        for (int v_ = 0; v_ < p.nvar; ++v_) o_w[p.bidx[(long long)v_ * p.N + n] * K + k] += r[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kHarmKPL; ++j) {
    const int k = lane + kHarmLanes * j;
    if (k < K) ksum[wave * K + k] = s[j];
  }
  __syncthreads();
  // the waves' sums in wave order -> this workgroup's partial row
  double* mine = p.part + (long long)blockIdx.x * K * (B + 1);
  for (int e = threadIdx.x; e < K; e += blockDim.x) {
    double t = 0.0;
    for (int w = 0; w < W; ++w) t += ksum[w * K + e];
    mine[e] = t;
  }
  for (int e = threadIdx.x; e < KB; e += blockDim.x) {
    double t = 0.0;
    for (int w = 0; w < W; ++w) t += hsm[(long long)w * KB + e];
    mine[K + e] = t;
  }
}

// one wave per (b, k): E[k,b] += sign * S_k * Pr_b[b], O[k,b] += sign * O_bk with the
// workgroup partials summed lane-strided then by a fixed xor tree (deterministic); op 0
// also refreshes Pen[k,b].  (A thread per (b, k) summing all partials in sequence took
// 155 us per call at 512 partials: seven latency-bound workgroups.)
__global__ void __launch_bounds__(256) harmony_reduce_kernel(HarmonyParams p, int n_wg,
                                                             double sign, int pen) {
  const int K = p.K, B = p.B;
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);   // e = b*K + k (partial layout)
  if (e >= K * B) return;
  const int b = e / K, k = e - b * K;
  const long long stride = (long long)K * (B + 1);
  double ts = 0.0, to = 0.0;
  for (int w = lane; w < n_wg; w += 64) {
    ts += p.part[w * stride + k];
    to += p.part[w * stride + K + e];
  }
  ts = wave_sum(ts);
  to = wave_sum(to);
  if (lane != 0) return;
  const long long kb = (long long)k * B + b;
  const double ev = p.E[kb] + sign * ts * p.Pr_b[b];
  const double ov = p.O[kb] + sign * to;
  p.E[kb] = ev;
  p.O[kb] = ov;
  if (pen) p.Pen[kb] = pow((ev + 1.0) / (ov + 1.0), p.theta[b]);
}

}  // namespace cnmf

extern "C" int cnmf_harmony_max_kb() { return cnmf::kHarmMaxKB; }

// waves per workgroup of the block kernel for K, B (1..4, within the LDS budget)
static int harmony_waves(int K, int B) {
  for (int W = 4; W > 1; --W)
    if (cnmf::harmony_lds_doubles(W, K, B, true) * 8 <= cnmf::kHarmLdsBytes) return W;
  return 1;
}

// op 0: remove + penalty table, op 1: assign + add.  part needs
// ceil(nb/chunk) * K * (B+1) doubles.  `counter` is unused (kept in the C ABI).
extern "C" hipError_t cnmf_harmony_block(int op, double* Rt, const double* distT,
                                         const double* sigma, const int* cells,
                                         const int* bidx, int nb, int N, int K, int B, int nvar,
                                         int chunk, double* E, double* O, const double* Pr_b,
                                         const double* theta, double* Pen, double* part,
                                         int* counter, hipStream_t stream) {
  (void)counter;
  if (nb <= 0) return hipSuccess;
  if (K < 1 || K > cnmf::kHarmLanes * cnmf::kHarmKPL || (long long)K * B > cnmf::kHarmMaxKB ||
      chunk < 1 || nvar < 1)
    return hipErrorInvalidValue;
  cnmf::HarmonyParams p{Rt, distT, sigma, cells, bidx, nb, N, K, B, nvar, chunk,
                        E, O, Pr_b, theta, Pen, part};
  const int n_wg = (nb + chunk - 1) / chunk;
  const int W = harmony_waves(K, B);
  const bool assign = op != 0;
  const size_t lds = (size_t)cnmf::harmony_lds_doubles(W, K, B, assign) * sizeof(double);
  static bool attr_done[2] = {false, false};
  const void* fn = assign ? reinterpret_cast<const void*>(&cnmf::harmony_block_kernel<true>)
                          : reinterpret_cast<const void*>(&cnmf::harmony_block_kernel<false>);
  if (!attr_done[assign]) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             cnmf::kHarmLdsBytes);
    if (e != hipSuccess) return e;
    attr_done[assign] = true;
  }
  if (assign)
    hipLaunchKernelGGL(cnmf::harmony_block_kernel<true>, dim3(n_wg), dim3(64 * W), lds, stream, p);
  else
    hipLaunchKernelGGL(cnmf::harmony_block_kernel<false>, dim3(n_wg), dim3(64 * W), lds, stream,
                       p);
  const int KB = K * B;
  hipLaunchKernelGGL(cnmf::harmony_reduce_kernel, dim3((KB + 3) / 4), dim3(256), 0, stream, p,
                     n_wg, assign ? 1.0 : -1.0, assign ? 0 : 1);
  return hipGetLastError();
}
