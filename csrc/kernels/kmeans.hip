// Fused Lloyd step for low-dimensional k-means (Harmony's k-means init over cells in PC
// space: harmonypy's KMeans(k ~ N/30 <= 100, n_init=10, max_iter=25) on N x d PCs,
// d <= 64; consensus k-means at K x G spectra keeps the MFMA distance path).
//
// One launch per Lloyd iteration for ALL restarts (grid.y = restart):
//   phase A  every thread owns one point per round: the point lives in registers
//            (d padded to DP, a compile-time multiple of 16), the restart's centroids sit
//            in LDS and are read as broadcast b128 loads; the thread keeps the argmin of
//            the exact squared distance sum_j (x_j - c_j)^2 (first index on ties, as numpy
//            argmin), writes its label (and the distance for the inertia).
//   phase B  the round's points are added to the workgroup's centroid accumulator in LDS:
//            a stable counting sort groups them by label, then each thread sums whole
//            (cluster, feature) segments in point order and adds them once (no float
//            atomics; the label histogram uses integer LDS atomics).
//   flush    the workgroup writes its partial sums/counts; the host sums the partials over
//            workgroups with a fixed-order reduction -> bitwise deterministic centroids.
// The (n x n_init*k) distance matrix of the MFMA path (4 GB at 500k cells x 10 x 100) is
// never materialised.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace cnmf {

constexpr int kKmThreads = 256;
constexpr int kKmRounds = 4;   // rounds of 256 points per workgroup

template <int DP>
__global__ void __launch_bounds__(kKmThreads)
    kmeans_step_kernel(const double* __restrict__ X, long long ldx, int n, int d,
                       const double* __restrict__ C, int k, const int* __restrict__ live,
                       int* __restrict__ labels, double* __restrict__ mind,
                       double* __restrict__ psum, double* __restrict__ pcnt) {
  extern __shared__ double smem[];
  double* sC = smem;                       // k * DP centroids (zero padded)
  double* sAcc = sC + (long long)k * DP;   // k * DP accumulator
  double* sCnt = sAcc + (long long)k * DP; // k counts
  int* sLab = reinterpret_cast<int*>(sCnt + k);   // 256 labels of the current round
  int* sPerm = sLab + kKmThreads;                   // round's points grouped by label
  int* sHist = sPerm + kKmThreads;                  // k: points per label this round
  int* sOff = sHist + k;                            // k: exclusive prefix of sHist
  const int r = blockIdx.y;
  const int n_init = gridDim.y;
  if (live != nullptr && live[r] == 0) return;    // frozen restart: partials unused
  const int tid = threadIdx.x;
  const double* Cr = C + (long long)r * k * d;
  for (int e = tid; e < k * DP; e += kKmThreads) {
    const int c = e / DP, j = e % DP;
    sC[e] = j < d ? Cr[(long long)c * d + j] : 0.0;
    sAcc[e] = 0.0;
  }
  for (int c = tid; c < k; c += kKmThreads) sCnt[c] = 0.0;
  __syncthreads();

  const long long base = (long long)blockIdx.x * (kKmThreads * kKmRounds);
  for (int round = 0; round < kKmRounds; ++round) {
    const long long p0 = base + (long long)round * kKmThreads;
    if (p0 >= n) break;                              // uniform across the workgroup
    const long long i = p0 + tid;
    // ---- phase A: assignment
    int arg = -1;
    if (i < n) {
      double x[DP];
      const double* xr = X + i * ldx;
#pragma unroll
      for (int j = 0; j < DP; ++j) x[j] = j < d ? xr[j] : 0.0;
      double best = 0.0;
      arg = 0;
      for (int c = 0; c < k; ++c) {
        const double2* cc = reinterpret_cast<const double2*>(sC + (long long)c * DP);
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int j = 0; j < DP / 2; ++j) {
          const double2 v = cc[j];
          const double a = x[2 * j] - v.x, b = x[2 * j + 1] - v.y;
          s0 = fma(a, a, s0);
          s1 = fma(b, b, s1);
        }
        const double s = s0 + s1;
        if (c == 0 || s < best) {
          best = s;
          arg = c;
        }
      }
      labels[(long long)r * n + i] = arg;
      if (mind != nullptr) mind[(long long)r * n + i] = best;
    }
    sLab[tid] = arg;
    __syncthreads();
    // ---- phase B: ordered accumulation (only when partial sums are wanted).  The
    // round's points are grouped by label with a stable counting sort (rank = earlier
    // points with the same label: a broadcast LDS walk), then every thread owns
    // (cluster, feature) pairs and sums its cluster's points in point order before one
    // add into the accumulator -- all 256 threads busy and no chain of dependent LDS
    // read-modify-writes (d threads walking 256 points serially took ~11 ms per Lloyd
    // step at 500k x 50 x 100, profiles/r3ae_harmony_500k_kernel_summary.txt).
    // Deterministic: fixed summation order for every (cluster, feature).
    if (psum != nullptr) {
      for (int c = tid; c < k; c += kKmThreads) sHist[c] = 0;
      __syncthreads();
      const int lab = sLab[tid];
      int rank = 0;
      if (lab >= 0) {
        for (int q = 0; q < tid; ++q) rank += sLab[q] == lab ? 1 : 0;
        atomicAdd(&sHist[lab], 1);
      }
      __syncthreads();
      if (tid == 0) {
        int o = 0;
        for (int c = 0; c < k; ++c) {
          sOff[c] = o;
          o += sHist[c];
        }
      }
      __syncthreads();
      if (lab >= 0) sPerm[sOff[lab] + rank] = tid;
      __syncthreads();
      for (int w = tid; w < k * d; w += kKmThreads) {
        const int c = w / d, j = w - c * d;
        const int cnt = sHist[c];
        if (cnt == 0) continue;
        const int o = sOff[c];
        double acc = 0.0;
        for (int t = 0; t < cnt; ++t) acc += X[(p0 + sPerm[o + t]) * ldx + j];
        sAcc[c * DP + j] += acc;
      }
      for (int c = tid; c < k; c += kKmThreads) sCnt[c] += (double)sHist[c];
    }
    __syncthreads();
  }
  if (psum != nullptr) {
    const long long slot = (long long)blockIdx.x * n_init + r;
    double* ps = psum + slot * k * d;
    for (int e = tid; e < k * d; e += kKmThreads) ps[e] = sAcc[(e / d) * DP + (e % d)];
    for (int c = tid; c < k; c += kKmThreads) pcnt[slot * k + c] = sCnt[c];
  }
}

template <int DP>
static hipError_t launch_kmeans(const double* X, long long ldx, int n, int d, const double* C,
                                int k, int n_init, const int* live, int* labels, double* mind,
                                double* psum, double* pcnt, hipStream_t stream) {
  const size_t lds = (size_t)(2 * (size_t)k * DP + k) * sizeof(double) +
                     (2 * kKmThreads + 2 * (size_t)k) * sizeof(int);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeans_step_kernel<DP>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int per = kKmThreads * kKmRounds;
  const dim3 grid((unsigned)((n + per - 1) / per), (unsigned)n_init);
  hipLaunchKernelGGL(kmeans_step_kernel<DP>, grid, dim3(kKmThreads), lds, stream, X, ldx, n, d, C,
                     k, live, labels, mind, psum, pcnt);
  return hipGetLastError();
}

// ---------------------------------------------------------------------- k-means++ step
// Greedy k-means++ (sklearn _kmeans_plusplus) for every restart at once, low-dimensional
// points (d <= 64): the M = n_init * trials candidates sit in LDS, every thread owns one
// point in registers and, for each candidate m of restart r = m / trials, takes
// min(closest[i][r], |x_i - c_m|^2).
//   mode 0  per-workgroup partial potentials pot[block][m] (summed on the host in block
//           order: deterministic) -- nothing (n x M) is materialised
//   mode 1  the candidates are the chosen centres (trials = 1): closest[i][r] is
//           lowered in place
template <int DP>
__global__ void __launch_bounds__(kKmThreads)
    kmeanspp_kernel(const double* __restrict__ X, long long ldx, int n, int d,
                    const double* __restrict__ C, int M, int trials,
                    double* __restrict__ closest, int n_init, int mode,
                    double* __restrict__ pot) {
  extern __shared__ double smem[];
  double* sC = smem;                      // M * DP candidates (zero padded)
  double* sRed = sC + (long long)M * DP;  // (kKmThreads / 64) * M wave partials
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < M * DP; e += kKmThreads) {
    const int c = e / DP, j = e % DP;
    sC[e] = j < d ? C[(long long)c * d + j] : 0.0;
  }
  __syncthreads();
  const long long i = (long long)blockIdx.x * kKmThreads + tid;
  const bool ok = i < n;
  double x[DP];
  const double* xr = X + (ok ? i : 0) * ldx;
#pragma unroll
  for (int j = 0; j < DP; ++j) x[j] = (ok && j < d) ? xr[j] : 0.0;
  double* cl = closest + (ok ? i : 0) * n_init;
  for (int m = 0; m < M; ++m) {
    const double2* cc = reinterpret_cast<const double2*>(sC + (long long)m * DP);
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < DP / 2; ++j) {
      const double2 v = cc[j];
      const double a = x[2 * j] - v.x, b = x[2 * j + 1] - v.y;
      s0 = fma(a, a, s0);
      s1 = fma(b, b, s1);
    }
    const int r = m / trials;
    const double cur = ok ? cl[r] : 0.0;
    const double v = ok ? fmin(cur, s0 + s1) : 0.0;
    if (mode == 1) {
      if (ok) cl[r] = v;
    } else {
      const double w = wave_sum(v);
      if (lane == 0) sRed[wave * M + m] = w;
    }
  }
  if (mode == 1) return;
  __syncthreads();
  for (int m = tid; m < M; m += kKmThreads) {
    double t = 0.0;
    for (int w = 0; w < kKmThreads / 64; ++w) t += sRed[w * M + m];
    pot[(long long)blockIdx.x * M + m] = t;
  }
}

template <int DP>
static hipError_t launch_kmeanspp(const double* X, long long ldx, int n, int d, const double* C,
                                  int M, int trials, double* closest, int n_init, int mode,
                                  double* pot, hipStream_t stream) {
  const size_t lds = ((size_t)M * DP + (size_t)(kKmThreads / 64) * M) * sizeof(double);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeanspp_kernel<DP>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const dim3 grid((unsigned)((n + kKmThreads - 1) / kKmThreads));
  hipLaunchKernelGGL(kmeanspp_kernel<DP>, grid, dim3(kKmThreads), lds, stream, X, ldx, n, d, C,
                     M, trials, closest, n_init, mode, pot);
  return hipGetLastError();
}

}  // namespace cnmf

extern "C" int cnmf_kmeanspp_blocks(int n) {
  return (n + cnmf::kKmThreads - 1) / cnmf::kKmThreads;
}

extern "C" int cnmf_kmeanspp_fits(int M, int d) {
  if (M < 1 || d < 1 || d > 64) return 0;
  const int dp = (d + 15) / 16 * 16;
  return ((size_t)M * dp + (size_t)(cnmf::kKmThreads / 64) * M) * sizeof(double) <= 150 * 1024;
}

extern "C" hipError_t cnmf_kmeanspp(const double* X, long long ldx, int n, int d,
                                    const double* C, int M, int trials, double* closest,
                                    int n_init, int mode, double* pot, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (!cnmf_kmeanspp_fits(M, d) || trials < 1 || M % trials || M / trials != n_init ||
      (mode == 0 && pot == nullptr) || (mode != 0 && mode != 1))
    return hipErrorInvalidValue;
  const int dp = (d + 15) / 16 * 16;
  switch (dp) {
    case 16: return cnmf::launch_kmeanspp<16>(X, ldx, n, d, C, M, trials, closest, n_init, mode, pot, stream);
    case 32: return cnmf::launch_kmeanspp<32>(X, ldx, n, d, C, M, trials, closest, n_init, mode, pot, stream);
    case 48: return cnmf::launch_kmeanspp<48>(X, ldx, n, d, C, M, trials, closest, n_init, mode, pot, stream);
    default: return cnmf::launch_kmeanspp<64>(X, ldx, n, d, C, M, trials, closest, n_init, mode, pot, stream);
  }
}

extern "C" int cnmf_kmeans_blocks(int n) {
  const int per = cnmf::kKmThreads * cnmf::kKmRounds;
  return (n + per - 1) / per;
}

// Largest k * DP the LDS budget (160 KiB per CU) holds: 2 * k * DP + k doubles + labels.
extern "C" int cnmf_kmeans_fits(int k, int d) {
  if (k < 1 || d < 1 || d > 64) return 0;
  const int dp = (d + 15) / 16 * 16;
  const size_t lds = (size_t)(2 * (size_t)k * dp + k) * sizeof(double) +
                     (2 * cnmf::kKmThreads + 2 * (size_t)k) * sizeof(int);
  return lds <= 156 * 1024 ? 1 : 0;
}

extern "C" hipError_t cnmf_kmeans_step(const double* X, long long ldx, int n, int d,
                                       const double* C, int k, int n_init, const int* live,
                                       int* labels, double* mind, double* psum, double* pcnt,
                                       hipStream_t stream) {
  if (n <= 0 || n_init <= 0) return hipSuccess;
  if (!cnmf_kmeans_fits(k, d)) return hipErrorInvalidValue;
  const int dp = (d + 15) / 16 * 16;
  switch (dp) {
    case 16: return cnmf::launch_kmeans<16>(X, ldx, n, d, C, k, n_init, live, labels, mind, psum, pcnt, stream);
    case 32: return cnmf::launch_kmeans<32>(X, ldx, n, d, C, k, n_init, live, labels, mind, psum, pcnt, stream);
    case 48: return cnmf::launch_kmeans<48>(X, ldx, n, d, C, k, n_init, live, labels, mind, psum, pcnt, stream);
    default: return cnmf::launch_kmeans<64>(X, ldx, n, d, C, k, n_init, live, labels, mind, psum, pcnt, stream);
  }
}
