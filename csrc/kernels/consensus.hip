// Consensus-step kernels (reference cnmf.py:1056-1084):
//
//  * pairdist_kernel     -- D[i][j] = sqrt(max(|a_i|^2 + |b_j|^2 - 2 a_i.b_j, 0)) (or the square)
//                           in float64 on the f64 matrix cores (v_mfma_f64_16x16x4_f64),
//                           LDS-staged 64x64 tiles; exact zeros on the diagonal for A == B
//                           (sklearn euclidean_distances semantics, cnmf.py:1065).
//  * knn_sum_kernel      -- per row, the sum of its k smallest entries by an exact 8-pass
//                           radix select on the float64 bit patterns (non-negative doubles order
//                           like their uint64 images), ties included exactly -- the
//                           argpartition + gather + sum of cnmf.py:1067-1070 in one pass per row.
//  * seg_argmin_kernel   -- k-means assignment: per point and per restart segment of k centroid
//                           columns, the argmin and its value (batched n_init restarts).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace cnmf {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kPdTile = 64;    // output tile edge
constexpr int kPdK = 16;       // k-chunk (doubles) staged per iteration
constexpr int kPdLd = kPdK + 1;

// f64 16x16x4 MFMA: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15];
// C/D (f64 map): col = lane&15, row = (lane>>4) + 4*reg.
__global__ void __launch_bounds__(256) pairdist_kernel(const double* __restrict__ A, long long lda,
                                                       const double* __restrict__ B, long long ldb,
                                                       const double* __restrict__ na,
                                                       const double* __restrict__ nb, int n, int m,
                                                       int kdim, double* __restrict__ D,
                                                       long long ldd, int same, int squared) {
  __shared__ double sA[kPdTile * kPdLd];
  __shared__ double sB[kPdTile * kPdLd];
  const int i0 = blockIdx.y * kPdTile, j0 = blockIdx.x * kPdTile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;   // wave's 32x32 sub-tile
  const int q = lane >> 4, c = lane & 15;
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};

  for (int k0 = 0; k0 < kdim; k0 += kPdK) {
    __syncthreads();
    for (int e = threadIdx.x; e < kPdTile * kPdK; e += 256) {
      const int r = e / kPdK, kk = e % kPdK;
      const int gi = i0 + r, gj = j0 + r, gk = k0 + kk;
      sA[r * kPdLd + kk] = (gi < n && gk < kdim) ? A[(long long)gi * lda + gk] : 0.0;
      sB[r * kPdLd + kk] = (gj < m && gk < kdim) ? B[(long long)gj * ldb + gk] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < kPdK; ks += 4) {
      double av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) av[a] = sA[(wr + 16 * a + c) * kPdLd + ks + q];
#pragma unroll
      for (int b = 0; b < 2; ++b) bv[b] = sB[(wc + 16 * b + c) * kPdLd + ks + q];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + wr + 16 * a + q + 4 * r;
        const int j = j0 + wc + 16 * b + c;
        if (i < n && j < m) {
          double d2 = na[i] + nb[j] - 2.0 * acc[a][b][r];
          d2 = d2 > 0.0 ? d2 : 0.0;
          if (same && i == j) d2 = 0.0;
          D[(long long)i * ldd + j] = squared ? d2 : sqrt(d2);
        }
      }
}

// One workgroup per row: exact sum of the k smallest entries of D[row, :m].
__global__ void __launch_bounds__(256) knn_sum_kernel(const double* __restrict__ D, long long ldd,
                                                      int m, int k, double* __restrict__ out) {
  __shared__ unsigned int hist[256];
  __shared__ unsigned long long s_prefix;
  __shared__ int s_need;
  __shared__ double sred[4];
  const int row = blockIdx.x;
  const unsigned long long* key =
      reinterpret_cast<const unsigned long long*>(D + (long long)row * ldd);
  if (threadIdx.x == 0) {
    s_prefix = 0ull;
    s_need = k;
  }
  unsigned long long mask = 0ull;
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    hist[threadIdx.x] = 0u;
    __syncthreads();
    const unsigned long long prefix = s_prefix;
    for (int j = threadIdx.x; j < m; j += 256) {
      const unsigned long long v = key[j];
      if ((v & mask) == prefix) atomicAdd(&hist[(v >> shift) & 255ull], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned int cum = 0;
      int need = s_need, sel = 255;
      for (int b = 0; b < 256; ++b) {
        if (cum + hist[b] >= (unsigned)need) {
          sel = b;
          break;
        }
        cum += hist[b];
      }
      s_need = need - (int)cum;
      s_prefix = prefix | ((unsigned long long)sel << shift);
    }
    mask |= 255ull << shift;
    __syncthreads();
  }
  // s_prefix = bit pattern of the k-th smallest value; s_need copies of it are taken
  const unsigned long long thr = s_prefix;
  double part = 0.0;
  for (int j = threadIdx.x; j < m; j += 256) {
    const unsigned long long v = key[j];
    if (v < thr) part += __longlong_as_double((long long)v);
  }
  part = wave_sum(part);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = part;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double tot = sred[0] + sred[1] + sred[2] + sred[3];
    out[row] = tot + (double)s_need * __longlong_as_double((long long)thr);
  }
}

__global__ void seg_argmin_kernel(const double* __restrict__ D, long long ldd, int n, int nseg,
                                  int k, const double* __restrict__ row_add,
                                  const double* __restrict__ col_add, int* __restrict__ labels,
                                  double* __restrict__ mind) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)n * nseg) return;
  const int i = (int)(t / nseg), s = (int)(t % nseg);
  const double* d = D + (long long)i * ldd + (long long)s * k;
  const double ra = row_add ? row_add[i] : 0.0;
  const double* ca = col_add ? col_add + (long long)s * k : nullptr;
  double best = 0.0;
  int arg = 0;
  for (int j = 0; j < k; ++j) {
    const double v = ra + (ca ? ca[j] : 0.0) + d[j];
    if (j == 0 || v < best) {
      best = v;
      arg = j;
    }
  }
  labels[t] = arg;
  mind[t] = best > 0.0 ? best : 0.0;
}

}  // namespace cnmf

extern "C" hipError_t cnmf_pairdist(const double* A, long long lda, const double* B, long long ldb,
                                    const double* na, const double* nb, int n, int m, int kdim,
                                    double* D, long long ldd, int same, int squared,
                                    hipStream_t stream) {
  if (n <= 0 || m <= 0) return hipSuccess;
  const dim3 grid((m + cnmf::kPdTile - 1) / cnmf::kPdTile, (n + cnmf::kPdTile - 1) / cnmf::kPdTile);
  hipLaunchKernelGGL(cnmf::pairdist_kernel, grid, dim3(256), 0, stream, A, lda, B, ldb, na, nb, n,
                     m, kdim, D, ldd, same, squared);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_knn_sum(const double* D, long long ldd, int n, int m, int k,
                                   double* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (k < 1 || k > m) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnmf::knn_sum_kernel, dim3(n), dim3(256), 0, stream, D, ldd, m, k, out);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_seg_argmin(const double* D, long long ldd, int n, int nseg, int k,
                                      const double* row_add, const double* col_add, int* labels,
                                      double* mind, hipStream_t stream) {
  const long long total = (long long)n * nseg;
  if (total <= 0) return hipSuccess;
  if (k < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnmf::seg_argmin_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     stream, D, ldd, n, nseg, k, row_add, col_add, labels, mind);
  return hipGetLastError();
}
