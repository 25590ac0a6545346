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
  const double* distT;   // N x K (assign only; nullptr: formed on the fly from Y and Zt)
  const double* sigma;   // K
  const int* cells;      // block cell ids (nb)
  const int* bidx;       // nvar x N, global batch index of each cell per covariate
  int nb, N, K, B, nvar, chunk;
  double* E;             // K x B
  double* O;             // K x B
  const double* Pr_b;    // B
  const double* theta;   // B
  double* Pen;           // K x B, written by op 0's reduce, read by op 1
  double* part;          // (n_wg, K*(B+1) + 2) partial sums: [k] cluster sums, [b][k] O
                         // sums, then (assign) sum R dist and sum sigma R log R
  const double* Y;       // d x K normalised centroids ([dd][k]; fused-distance assign)
  const double* Zt;      // N x d cosine-normalised PCs, cell-major
  int d;
  double* obj;           // [2] objective accumulators of the round (reduce kernel adds)
};

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// LDS doubles of a W-wave block kernel: W O-tables, the penalty table (assign), W K-sums,
// and (fused-distance assign) the d x K centroids and W x 2 objective sums
__host__ __device__ constexpr long long harmony_lds_doubles(int W, int K, int B, bool assign,
                                                            int d = 0) {
  return (long long)W * K * B + (assign ? (long long)K * B : 0) + (long long)W * K +
         (assign ? (long long)d * K + 2LL * W : 0);
}

template <bool ASSIGN>
__global__ void __launch_bounds__(4 * kHarmLanes) harmony_block_kernel(HarmonyParams p) {
  extern __shared__ __attribute__((aligned(16))) double hsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, W = blockDim.x >> 6;
  const int K = p.K, B = p.B, KB = K * B;
  double* o_w = hsm + (long long)wave * KB;          // this wave's O table, [b][k]
  double* spen = hsm + (long long)W * KB;            // penalty table (assign)
  double* ksum = spen + (ASSIGN ? KB : 0);           // [W][K] cluster sums
  double* sY = ksum + (long long)W * K;              // [d][K] centroids (fused distance)
  double* sobj = sY + (ASSIGN && !p.distT ? (long long)p.d * K : 0);   // [W][2]
  const bool fused = ASSIGN && p.distT == nullptr;
  for (int e = threadIdx.x; e < W * KB; e += blockDim.x) hsm[e] = 0.0;
  if (ASSIGN)
    for (int e = threadIdx.x; e < KB; e += blockDim.x) spen[e] = p.Pen[e];
  if (fused)
    for (int e = threadIdx.x; e < p.d * K; e += blockDim.x) sY[e] = p.Y[e];
  __syncthreads();
  double okm = 0.0, oent = 0.0;     // this lane's sum R dist and sum sigma R log R
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
      // dist[n, k] = 2 (1 - Y_k . z_n): read, or formed here from the centroids in LDS
      // and the cell's PCs (every lane reads the same z_n word: one broadcast load)
      double dk[kHarmKPL];
      if (fused) {
        double dot[kHarmKPL] = {0.0, 0.0};
        const double* z = p.Zt + (long long)n * p.d;
        for (int dd = 0; dd < p.d; ++dd) {
          const double zv = z[dd];
#pragma unroll
          for (int j = 0; j < kHarmKPL; ++j) {
            const int k = lane + kHarmLanes * j;
            if (k < K) dot[j] = fma(sY[dd * K + k], zv, dot[j]);
          }
        }
#pragma unroll
        for (int j = 0; j < kHarmKPL; ++j) dk[j] = 2.0 * (1.0 - dot[j]);
      } else {
        const double* d = p.distT + (long long)n * K;
#pragma unroll
        for (int j = 0; j < kHarmKPL; ++j) {
          const int k = lane + kHarmLanes * j;
          dk[j] = k < K ? d[k] : 0.0;
        }
      }
      double sd[kHarmKPL];
      double mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < kHarmKPL; ++j) {
        const int k = lane + kHarmLanes * j;
        sd[j] = k < K ? -dk[j] * isig[j] : -INFINITY;
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
        if (k < K) {
          rr[k] = r[j];
          // the round's objective terms of this cell (harmonypy compute_objective: the
          // k-means error and the entropy, both with the assignment just made)
          okm = fma(r[j], dk[j], okm);
          if (r[j] > 0.0) oent = fma(p.sigma[k] * r[j], log(r[j]), oent);
        }
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
  if (ASSIGN) {
    const double a = wave_sum(okm), b = wave_sum(oent);
    if (lane == 0) {
      sobj[2 * wave] = a;
      sobj[2 * wave + 1] = b;
    }
  }
  __syncthreads();
  double* mine = p.part + (long long)blockIdx.x * (K * (B + 1) + 2);
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    if (ASSIGN)
      for (int w = 0; w < W; ++w) {
        a += sobj[2 * w];
        b += sobj[2 * w + 1];
      }
    mine[K * (B + 1)] = a;
    mine[K * (B + 1) + 1] = b;
  }
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
  const long long stride = (long long)K * (B + 1) + 2;
  if (e == K * B) {          // the objective partials of an assign, in the same fixed order
    if (!p.obj || sign < 0.0) return;
    double ta = 0.0, tb = 0.0;
    for (int w = lane; w < n_wg; w += 64) {
      ta += p.part[w * stride + K * (B + 1)];
      tb += p.part[w * stride + K * (B + 1) + 1];
    }
    ta = wave_sum(ta);
    tb = wave_sum(tb);
    if (lane == 0) {
      p.obj[0] += ta;
      p.obj[1] += tb;
    }
    return;
  }
  if (e > K * B) return;
  const int b = e / K, k = e - b * K;
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

// Centroid product Y = Z_cos R^T (d x K) over all cells, in two deterministic stages:
// workgroup g sums its chunk of cells into a partial (tiles of 32 cells staged in LDS,
// thread t owns outputs t, t + 256, ...), then one wave per output sums the partials
// lane-strided + xor tree.  (A library GEMM gives this long-reduction / small-output
// product one output tile: one workgroup walking every cell.)
constexpr int kHarmCenTile = 32;
constexpr int kHarmCenMaxJ = 40;             // outputs per thread: d * K <= 10240

__global__ void __launch_bounds__(256) harmony_centroid_kernel(const double* __restrict__ Zt,
                                                               const double* __restrict__ Rt,
                                                               int N, int d, int K, int chunk,
                                                               double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) double csm[];
  double* sz = csm;                                  // [tile][d]
  double* sr = csm + kHarmCenTile * d;               // [tile][K]
  const int P = d * K, tid = threadIdx.x;
  const int n0 = blockIdx.x * chunk, n1 = min(N, n0 + chunk);
  double acc[kHarmCenMaxJ];
#pragma unroll
  for (int j = 0; j < kHarmCenMaxJ; ++j) acc[j] = 0.0;
  for (int c0 = n0; c0 < n1; c0 += kHarmCenTile) {
    const int tc = min(kHarmCenTile, n1 - c0);
    for (int e = tid; e < tc * d; e += 256) sz[e] = Zt[(long long)c0 * d + e];
    for (int e = tid; e < tc * K; e += 256) sr[e] = Rt[(long long)c0 * K + e];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kHarmCenMaxJ; ++j) {
      const int q = tid + 256 * j;
      if (q < P) {
        const int dd = q / K, k = q - dd * K;
        double a = acc[j];
        for (int c = 0; c < tc; ++c) a = fma(sz[c * d + dd], sr[c * K + k], a);
        acc[j] = a;
      }
    }
    __syncthreads();
  }
  double* o = part + (long long)blockIdx.x * P;
#pragma unroll
  for (int j = 0; j < kHarmCenMaxJ; ++j) {
    const int q = tid + 256 * j;
    if (q < P) o[q] = acc[j];
  }
}

// out[q] = sum over n_part partial rows of part[.][q]: one wave per output, lane-strided
// then a fixed xor tree (deterministic)
__global__ void __launch_bounds__(256) harmony_sum_rows_kernel(const double* __restrict__ part,
                                                               int n_part, int P,
                                                               double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= P) return;
  double t = 0.0;
  for (int w = lane; w < n_part; w += 64) t += part[(long long)w * P + q];
  t = wave_sum(t);
  if (lane == 0) out[q] = t;
}

// The round's objective: the assign passes' sum R dist and sum sigma R log R (obj[0..1],
// reset here) plus the cross-entropy term, which reduces to K x B numbers because
// O = R Phi^T: sum_{k,b} sigma_k theta_b O[k,b] log((O[k,b] + 1) / (E[k,b] + 1)).
__global__ void __launch_bounds__(256) harmony_objective_kernel(const double* __restrict__ O,
                                                                const double* __restrict__ E,
                                                                const double* __restrict__ sigma,
                                                                const double* __restrict__ theta,
                                                                int K, int B, double* obj,
                                                                double* out) {
  __shared__ double sred[4];
  double t = 0.0;
  for (int e = threadIdx.x; e < K * B; e += 256) {
    const int k = e / B, b = e - k * B;
    const double o = O[e];
    t += sigma[k] * theta[b] * o * log((o + 1.0) / (E[e] + 1.0));
  }
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double cross = (sred[0] + sred[1]) + (sred[2] + sred[3]);
    out[0] = obj[0] + obj[1] + cross;
    obj[0] = 0.0;
    obj[1] = 0.0;
  }
}

}  // namespace cnmf

extern "C" int cnmf_harmony_max_kb() { return cnmf::kHarmMaxKB; }
extern "C" int cnmf_harmony_centroid_max() { return 256 * cnmf::kHarmCenMaxJ; }

// Y (d x K) = Zt^T Rt over N cells; part needs ceil(N / chunk) * d * K doubles
extern "C" hipError_t cnmf_harmony_centroid(const double* Zt, const double* Rt, int N, int d,
                                            int K, int chunk, double* part, double* Y,
                                            hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  if (d < 1 || K < 1 || (long long)d * K > 256LL * cnmf::kHarmCenMaxJ || chunk < 1)
    return hipErrorInvalidValue;
  const int n_wg = (N + chunk - 1) / chunk;
  const size_t lds = (size_t)cnmf::kHarmCenTile * (d + K) * sizeof(double);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnmf::harmony_centroid_kernel, dim3(n_wg), dim3(256), lds, stream, Zt, Rt, N,
                     d, K, chunk, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int P = d * K;
  hipLaunchKernelGGL(cnmf::harmony_sum_rows_kernel, dim3((P + 3) / 4), dim3(256), 0, stream, part,
                     n_wg, P, Y);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_harmony_objective(const double* O, const double* E,
                                             const double* sigma, const double* theta, int K,
                                             int B, double* obj, double* out, hipStream_t stream) {
  if (K < 1 || B < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnmf::harmony_objective_kernel, dim3(1), dim3(256), 0, stream, O, E, sigma,
                     theta, K, B, obj, out);
  return hipGetLastError();
}

// op 0: remove + penalty table; op 1: assign + add (distT, or -- distT null -- the
// distances formed from Y (d x K) and Zt (N x d), with the round's objective terms added
// to obj[2]).  part needs ceil(nb/chunk) * (K * (B+1) + 2) doubles.
extern "C" hipError_t cnmf_harmony_block(int op, double* Rt, const double* distT,
                                         const double* sigma, const int* cells,
                                         const int* bidx, int nb, int N, int K, int B, int nvar,
                                         int chunk, double* E, double* O, const double* Pr_b,
                                         const double* theta, double* Pen, double* part,
                                         const double* Y, const double* Zt, int d, double* obj,
                                         hipStream_t stream) {
  if (nb <= 0) return hipSuccess;
  if (K < 1 || K > cnmf::kHarmLanes * cnmf::kHarmKPL || (long long)K * B > cnmf::kHarmMaxKB ||
      chunk < 1 || nvar < 1)
    return hipErrorInvalidValue;
  if (op != 0 && !distT && (!Y || !Zt || d < 1)) return hipErrorInvalidValue;
  cnmf::HarmonyParams p{Rt, distT, sigma, cells, bidx, nb, N, K, B, nvar, chunk,
                        E, O, Pr_b, theta, Pen, part, Y, Zt, distT ? 0 : d, obj};
  const int n_wg = (nb + chunk - 1) / chunk;
  const bool assign = op != 0;
  int W = 1;
  for (int w = 4; w >= 1; --w)
    if (cnmf::harmony_lds_doubles(w, K, B, true, p.d) * 8 <= cnmf::kHarmLdsBytes) {
      W = w;
      break;
    }
  if (cnmf::harmony_lds_doubles(W, K, B, assign, p.d) * 8 > cnmf::kHarmLdsBytes)
    return hipErrorInvalidValue;
  const size_t lds = (size_t)cnmf::harmony_lds_doubles(W, K, B, assign, p.d) * sizeof(double);
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
  hipLaunchKernelGGL(cnmf::harmony_reduce_kernel, dim3((KB + 1 + 3) / 4), dim3(256), 0, stream, p,
                     n_wg, assign ? 1.0 : -1.0, assign ? 0 : 1);
  return hipGetLastError();
}
