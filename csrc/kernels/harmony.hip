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

// lane l's value of a wave-uniform lane index, as a scalar (v_readlane)
__device__ __forceinline__ int rl_i(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ double rl_d(double x, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// LDS doubles of a W-wave block kernel: W O-tables, the penalty table (assign), W K-sums
// (rounded up to an even count), and (fused-distance assign) the centroids as
// [PC, padded to 8][lane][2] -- lane l's clusters l and l + 64 side by side, one 16-byte
// read per PC -- and W x 2 objective sums
__host__ __device__ constexpr long long harmony_sy_offset(int W, int K, int B, bool assign) {
  return ((long long)W * K * B + (assign ? (long long)K * B : 0) + (long long)W * K + 1) / 2 * 2;
}
__host__ __device__ constexpr long long harmony_lds_doubles(int W, int K, int B, bool assign,
                                                            int d = 0) {
  return harmony_sy_offset(W, K, B, assign) +
         (assign && d > 0 ? (long long)(d + 7) / 8 * 8 * 128 + 2LL * W : 0);
}

template <bool ASSIGN>
__global__ void __launch_bounds__(4 * kHarmLanes) harmony_block_kernel(HarmonyParams p) {
  extern __shared__ __attribute__((aligned(16))) double hsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, W = blockDim.x >> 6;
  const int K = p.K, B = p.B, KB = K * B;
  double* o_w = hsm + (long long)wave * KB;          // this wave's O table, [b][k]
  double* spen = hsm + (long long)W * KB;            // penalty table (assign)
  double* ksum = spen + (ASSIGN ? KB : 0);           // [W][K] cluster sums
  const bool fused = ASSIGN && p.distT == nullptr;
  const int dpad = (p.d + 7) / 8 * 8;
  double* sY = hsm + harmony_sy_offset(W, K, B, ASSIGN);   // [dpad][64][2] (fused distance)
  double* sobj = sY + (fused ? (long long)dpad * 128 : 0);  // [W][2]
  for (int e = threadIdx.x; e < W * KB; e += blockDim.x) hsm[e] = 0.0;
  if (ASSIGN)
    for (int e = threadIdx.x; e < KB; e += blockDim.x) spen[e] = p.Pen[e];
  if (fused)
    for (int e = threadIdx.x; e < dpad * 128; e += blockDim.x) {
      const int dd = e >> 7, l = (e & 127) >> 1, k = l + 64 * (e & 1);
      sY[e] = (dd < p.d && k < K) ? p.Y[(long long)dd * K + k] : 0.0;
    }
  __syncthreads();
  double okm = 0.0, oent = 0.0;     // this lane's sum R dist and sum sigma R log R
  double isig[kHarmKPL];
#pragma unroll
  for (int j = 0; j < kHarmKPL; ++j) {
    const int k = lane + kHarmLanes * j;
    isig[j] = (ASSIGN && k < K) ? 1.0 / p.sigma[k] : 0.0;
  }
  double s[kHarmKPL] = {0.0, 0.0};
  double sg[kHarmKPL];
#pragma unroll
  for (int j = 0; j < kHarmKPL; ++j) {
    const int k = lane + kHarmLanes * j;
    sg[j] = (ASSIGN && k < K) ? p.sigma[k] : 0.0;
  }
  const int i0 = blockIdx.x * p.chunk, i1 = min(p.nb, i0 + p.chunk);
  // a cell's per-cell operands are fetched by the wave as ONE vector load each (lane v:
  // its batch index of covariate v; lane dd: its PC dd) and handed out with v_readlane --
  // the first version read them word by word in the loops, a dependent global load per
  // PC: ~300 us per 25k-cell block (profiles/r5j_*).  The next cell's loads are issued
  // before the current cell is processed.
  int n_nx = i0 + wave < i1 ? p.cells[i0 + wave] : 0;
  int bl_nx = 0;
  double zl_nx = 0.0;
  if (i0 + wave < i1) {
    if (lane < p.nvar) bl_nx = p.bidx[(long long)lane * p.N + n_nx];
    if (fused && lane < p.d) zl_nx = p.Zt[(long long)n_nx * p.d + lane];
  }
  for (int i = i0 + wave; i < i1; i += W) {
    const int n = n_nx;
    const int bl = bl_nx;
    const double zl = zl_nx;
    if (i + W < i1) {
      n_nx = p.cells[i + W];
      if (lane < p.nvar) bl_nx = p.bidx[(long long)lane * p.N + n_nx];
      if (fused && lane < p.d) zl_nx = p.Zt[(long long)n_nx * p.d + lane];
    }
    double* rr = p.Rt + (long long)n * K;
    double r[kHarmKPL];
    if (ASSIGN) {
      // dist[n, k] = 2 (1 - Y_k . z_n): read, or formed here from the centroids in LDS
      // and the cell's PCs
      double dk[kHarmKPL];
      if (fused) {
        double dot[kHarmKPL] = {0.0, 0.0};
        // 8 PCs per step: 8 independent 16-byte LDS reads, then the FMAs (zero padding
        // beyond d on both sides)
        for (int d0 = 0; d0 < dpad; d0 += 8) {
          double2 y[8];
#pragma unroll
          for (int u = 0; u < 8; ++u)
            y[u] = *reinterpret_cast<const double2*>(sY + (long long)(d0 + u) * 128 + 2 * lane);
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const double zv = rl_d(zl, d0 + u);
            dot[0] = fma(y[u].x, zv, dot[0]);
            dot[1] = fma(y[u].y, zv, dot[1]);
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
          for (int v_ = 0; v_ < p.nvar; ++v_) pen += spen[k * B + rl_i(bl, v_)];
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
          if (r[j] > 0.0) oent = fma(sg[j] * r[j], log(r[j]), oent);
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
        for (int v_ = 0; v_ < p.nvar; ++v_) o_w[rl_i(bl, v_) * K + k] += r[j];
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

// Centroid product Y = Z_cos R^T (d x K) over all cells, in two deterministic stages on
// the f64 matrix cores: workgroup g sums its chunk of cells into a partial d x K block --
// the cells are the MFMA reduction dimension, A = Zt rows (16 PCs x 4 cells), B = Rt rows
// (4 cells x 16 clusters), both read straight from global memory (16 consecutive doubles
// per lane group); wave w owns cluster tiles w and w + 4 for every PC tile (<= 8
// accumulators) -- then one wave per output sums the partials lane-strided + xor tree.
// (A library GEMM gives this long-reduction / small-output product one output tile: one
// workgroup walking every cell; the scalar LDS version took 1.8 ms per call at 500k x 50
// x 100, profiles/r5j_*.)
typedef double hm_f64x4 __attribute__((ext_vector_type(4)));
constexpr int kHarmCenMaxD = 64;             // 4 PC tiles
constexpr int kHarmCenMaxK = 128;            // 8 cluster tiles = 2 per wave

__global__ void __launch_bounds__(256) harmony_centroid_kernel(const double* __restrict__ Zt,
                                                               const double* __restrict__ Rt,
                                                               int N, int d, int K, int chunk,
                                                               double* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int dT = (d + 15) >> 4, kT = (K + 15) >> 4;
  const int n0 = blockIdx.x * chunk, n1 = min(N, n0 + chunk);
  hm_f64x4 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = hm_f64x4{0.0, 0.0, 0.0, 0.0};
  const int kt0 = wave, kt1 = wave + 4;
  const bool has0 = kt0 < kT, has1 = kt1 < kT;          // wave-uniform
  if (!has0) return;                                   // no LDS / barriers below
  for (int c0 = n0; c0 < n1; c0 += 4) {
    const int c = c0 + grp;
    const bool ok = c < n1;
    const double* zr = Zt + (long long)(ok ? c : 0) * d;
    const double* rr = Rt + (long long)(ok ? c : 0) * K;
    double av[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int dd = 16 * a + col;
      av[a] = (ok && a < dT && dd < d) ? zr[dd] : 0.0;
    }
    const int k0 = 16 * kt0 + col, k1 = 16 * kt1 + col;
    const double b0 = (ok && k0 < K) ? rr[k0] : 0.0;
    const double b1 = (ok && has1 && k1 < K) ? rr[k1] : 0.0;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      if (a < dT) {                                    // uniform
        acc[a][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], b0, acc[a][0], 0, 0, 0);
        if (has1) acc[a][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], b1, acc[a][1], 0, 0, 0);
      }
    }
  }
  // D (16 PCs x 16 clusters): col = cluster lane&15, row = PC (lane>>4) + 4 * reg
  double* o = part + (long long)blockIdx.x * d * K;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    if (a >= dT) break;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int kt = b == 0 ? kt0 : kt1;
      if (b == 1 && !has1) break;
      const int k = 16 * kt + col;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int dd = 16 * a + grp + 4 * q;
        if (dd < d && k < K) o[(long long)dd * K + k] = acc[a][b][q];
      }
    }
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
extern "C" int cnmf_harmony_centroid_max_d() { return cnmf::kHarmCenMaxD; }

// Y (d x K) = Zt^T Rt over N cells; part needs ceil(N / chunk) * d * K doubles
extern "C" hipError_t cnmf_harmony_centroid(const double* Zt, const double* Rt, int N, int d,
                                            int K, int chunk, double* part, double* Y,
                                            hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  if (d < 1 || K < 1 || d > cnmf::kHarmCenMaxD || K > cnmf::kHarmCenMaxK || chunk < 1)
    return hipErrorInvalidValue;
  const int n_wg = (N + chunk - 1) / chunk;
  hipLaunchKernelGGL(cnmf::harmony_centroid_kernel, dim3(n_wg), dim3(256), 0, stream, Zt, Rt, N,
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
  // (one lane per covariate / per PC for the per-cell vector loads)
  if (nvar > cnmf::kHarmLanes) return hipErrorInvalidValue;
  if (op != 0 && !distT && (!Y || !Zt || d < 1 || d > cnmf::kHarmLanes))
    return hipErrorInvalidValue;
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
