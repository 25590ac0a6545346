// Segmented sums of the consensus step: the k-means centroid
// update of every batched restart and the per-cluster distance sums of the silhouette,
// without a one-hot matrix or a library GEMM (cnmf.py:1082-1084 KMeans(n_init=10),
// cnmf.py:1097 silhouette_score).  Both are float64 and deterministic: every sum runs in a
// fixed order (points in index order per wave, then the waves / lanes in a fixed tree).
//
//  * seg_colsum_kernel: out[r][c][j] = sum over points i with lab[r][i] == c of X[i][j].
//    Grid (gene tiles of 64, restarts).  Lane l of every wave owns gene j0 + l; wave w walks
//    its contiguous quarter of the points in order and adds X[i][j] into its LDS row
//    acc[w][lab[r][i]][l] (the label is wave-uniform, so one scalar load per point and no
//    bank conflict: lane-indexed words).  The waves' tables are summed in wave order.  Each
//    (restart, tile) reads a 64-column strip of X; the restarts of one strip run side by
//    side, so X streams from HBM about once and the re-reads hit L2.
//  * seg_rowsum_kernel: out[i][c] = sum over j with lab[j] == c of D[i][j].  One wave per
//    row i: lane l walks j = l, l + 64, ... (coalesced) into its LDS column acc[c][l], and
//    the 64 lane partials of each cluster are summed in a fixed xor tree.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cnmf {

constexpr int kSsTile = 64;

__global__ void __launch_bounds__(256) seg_colsum_kernel(const double* __restrict__ X, long long ldx,
                                                         int n, int d,
                                                         const int* __restrict__ lab,
                                                         long long ldl, int k,
                                                         double* __restrict__ out) {
  extern __shared__ double acc[];      // [nw][k][64]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int j = blockIdx.x * kSsTile + lane, r = blockIdx.y;
  double* mine = acc + (long long)w * k * kSsTile;
  for (int c = 0; c < k; ++c) mine[c * kSsTile + lane] = 0.0;
  const int* lr = lab + (long long)r * ldl;
  const int i0 = (int)((long long)n * w / nw), i1 = (int)((long long)n * (w + 1) / nw);
  if (j < d) {
    const double* xc = X + j;
    int i = i0;
    // four independent loads in flight per lane; the adds stay in point order
    for (; i + 4 <= i1; i += 4) {
      const double v0 = xc[(long long)i * ldx], v1 = xc[(long long)(i + 1) * ldx];
      const double v2 = xc[(long long)(i + 2) * ldx], v3 = xc[(long long)(i + 3) * ldx];
      const int c0 = lr[i], c1 = lr[i + 1], c2 = lr[i + 2], c3 = lr[i + 3];
      mine[c0 * kSsTile + lane] += v0;
      mine[c1 * kSsTile + lane] += v1;
      mine[c2 * kSsTile + lane] += v2;
      mine[c3 * kSsTile + lane] += v3;
    }
    for (; i < i1; ++i) mine[lr[i] * kSsTile + lane] += xc[(long long)i * ldx];
  }
  __syncthreads();
  if (j >= d) return;
  double* o = out + (long long)r * k * d + j;
  for (int c = w; c < k; c += nw) {
    double s = acc[c * kSsTile + lane];
    for (int v = 1; v < nw; ++v) s += acc[((long long)v * k + c) * kSsTile + lane];
    o[(long long)c * d] = s;
  }
}

__global__ void __launch_bounds__(256) seg_rowsum_kernel(const double* __restrict__ D, long long ldd,
                                                         int n, int m,
                                                         const int* __restrict__ lab, int k,
                                                         double* __restrict__ out,
                                                         long long ldo) {
  extern __shared__ double acc[];      // [waves][k][64]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const long long i = (long long)blockIdx.x * nw + w;
  double* mine = acc + (long long)w * k * 64;
  for (int c = 0; c < k; ++c) mine[c * 64 + lane] = 0.0;
  if (i < n) {
    const double* row = D + i * ldd;
    for (int jj = lane; jj < m; jj += 64) mine[lab[jj] * 64 + lane] += row[jj];
  }
  __syncthreads();
  if (i >= n) return;
  // per cluster: the 64 lane partials in a fixed xor tree (lane 0 holds the sum)
  for (int c = 0; c < k; ++c) {
    double s = mine[c * 64 + lane];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) out[i * ldo + c] = s;
  }
}


// Small Gram G = A^T A of a tall strided operand (H4-H6 helpers: the K x K Grams of the
// usage / spectra refits, the prediction error's trace term and the OLS normal matrix):
// element (i, a) of A (n x K) at A[i * s_i + a * s_a] -- so both U^T U (n x K rows) and
// S S^T (K x n, s_i = 1) take it.  Grid: row chunks; a chunk's rows are staged in LDS
// (64 at a time), thread t owns the pairs p = t, t + 256, .. of the K x K output and sums
// them over the chunk's rows in order; the per-chunk partials are reduced by the host in
// chunk order (a fixed order: deterministic).
template <typename T>
__global__ void __launch_bounds__(256) small_gram_kernel(const T* __restrict__ A, long long s_i,
                                                         long long s_a, int n, int K, int rows_per,
                                                         T* __restrict__ part) {
  extern __shared__ unsigned char sg_raw[];
  T* tile = reinterpret_cast<T*>(sg_raw);          // [64][K]
  const int i0 = blockIdx.x * rows_per, i1 = min(n, i0 + rows_per);
  const int npair = K * K;
  T acc[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) acc[u] = T(0);
  for (int r0 = i0; r0 < i1; r0 += 64) {
    const int nr = min(64, i1 - r0);
    __syncthreads();
    for (int e = threadIdx.x; e < nr * K; e += 256) {
      const int rr = e / K, a = e - rr * K;
      tile[rr * K + a] = A[(long long)(r0 + rr) * s_i + (long long)a * s_a];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int pq = threadIdx.x + 256 * u;
      if (pq < npair) {
        const int a = pq / K, b = pq - a * K;
        T v = acc[u];
        for (int rr = 0; rr < nr; ++rr) v += tile[rr * K + a] * tile[rr * K + b];
        acc[u] = v;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int pq = threadIdx.x + 256 * u;
    if (pq < npair) part[(long long)blockIdx.x * npair + pq] = acc[u];
  }
}

}  // namespace cnmf

static int ss_waves(int k) {
  // LDS: waves x k x 64 doubles within 128 KB
  int nw = 4;
  while (nw > 1 && (long long)nw * k * 64 * 8 > (128 << 10)) nw >>= 1;
  return nw;
}

extern "C" hipError_t cnmf_seg_colsum(const double* X, long long ldx, int n, int d, const int* lab,
                                      long long ldl, int nrest, int k, double* out,
                                      hipStream_t stream) {
  if (n < 0 || d < 1 || k < 1 || nrest < 1 || ldx < d || ldl < n || !X || !lab || !out ||
      (long long)k * 64 * 8 > (128 << 10))
    return hipErrorInvalidValue;
  const int nw = ss_waves(k);
  const size_t lds = (size_t)nw * k * 64 * sizeof(double);
  if (lds > (64 << 10)) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cnmf::seg_colsum_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(cnmf::seg_colsum_kernel, dim3((unsigned)((d + 63) / 64), (unsigned)nrest),
                     dim3(64 * nw), lds, stream, X, ldx, n, d, lab, ldl, k, out);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_seg_rowsum(const double* D, long long ldd, int n, int m, const int* lab,
                                      int k, double* out, long long ldo, hipStream_t stream) {
  if (n < 1 || m < 1 || k < 1 || ldd < m || ldo < k || !D || !lab || !out ||
      (long long)k * 64 * 8 > (128 << 10))
    return hipErrorInvalidValue;
  const int nw = ss_waves(k);
  const size_t lds = (size_t)nw * k * 64 * sizeof(double);
  if (lds > (64 << 10)) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cnmf::seg_rowsum_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(cnmf::seg_rowsum_kernel, dim3((unsigned)((n + nw - 1) / nw)), dim3(64 * nw),
                     lds, stream, D, ldd, n, m, lab, k, out, ldo);
  return hipGetLastError();
}

// chunks of rows_per rows; part: chunks x K x K partials (T = float / double by esz)
extern "C" hipError_t cnmf_small_gram(const void* A, long long s_i, long long s_a, int n, int K,
                                      int esz, int rows_per, void* part, hipStream_t stream) {
  if (n < 1 || K < 1 || K > 64 || rows_per < 1 || !A || !part || (esz != 4 && esz != 8))
    return hipErrorInvalidValue;
  const unsigned chunks = (unsigned)((n + rows_per - 1) / rows_per);
  const size_t lds = (size_t)64 * K * esz;
  if (esz == 8)
    hipLaunchKernelGGL(cnmf::small_gram_kernel<double>, dim3(chunks), dim3(256), lds, stream,
                       static_cast<const double*>(A), s_i, s_a, n, K, rows_per,
                       static_cast<double*>(part));
  else
    hipLaunchKernelGGL(cnmf::small_gram_kernel<float>, dim3(chunks), dim3(256), lds, stream,
                       static_cast<const float*>(A), s_i, s_a, n, K, rows_per,
                       static_cast<float*>(part));
  return hipGetLastError();
}
