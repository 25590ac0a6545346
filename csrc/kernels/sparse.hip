// Device-resident CSR kernels for the preprocessing stages (SURVEY.md §2.4 H9/H12;
// reference cnmf.py:128-247, preprocess.py:21-29, 250-338 -- scanpy/sklearn on the host
// there).  Every kernel reads the matrix in its stored CSR form; nothing is densified
// unless asked (csr_densify).  Values are transformed on the fly:
//
//     v' = min(round?(data[j] * row_scale[row]) / col_div[c'], clip[c'], max_value)
//
// where c' = col_map[col] (-1 drops the entry: an implicit column subset), every factor
// is optional and round? rounds the row-scaled value to float32 when the host pipeline
// stores it as float32 in between (normalize_total then scale), so device and host
// results agree bit for bit.  This fuses normalize_total (row scale), the HVG column subset,
// scale(zero_center=False) (column scale), the max_value / quantile ceilings and the
// seurat_v3 per-gene clip into the consumer kernel instead of materialising each step.
//
//  * csr_row_sums      one wave per row, float64, fixed order.
//  * csr_col_stats     per-column sum, sum of squares (optionally centred) and nnz.
//                      Deterministic without atomics: each wave owns a private LDS tile
//                      of column accumulators and walks its rows in order (the lanes of
//                      one row touch distinct columns); waves are combined in fixed order
//                      into per-workgroup partials, summed over workgroups on the host
//                      side by a fixed-order reduction.
//  * csr_transform     the transformed value of every stored entry (dropped -> -1).
//  * csr_densify       transformed rows scattered into a zeroed dense (n x n_out) matrix.
//  * radix_hist        one pass of an exact radix select over the float32 bit patterns
//                      of non-negative values (negative values are skipped): 256-bin
//                      histogram of the byte at `shift` among values matching `prefix`;
//                      LDS histograms flushed with integer atomics (exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace cnmf {

struct CsrXform {
  const double* row_scale;  // [n_rows] or null
  const int* col_map;       // [n_cols] -> output column or -1, or null (identity)
  const double* col_div;    // [n_out] or null (divisor: scale(zero_center=False)'s std)
  const double* clip;       // [n_out] or null (per-column ceiling)
  double max_value;         // global ceiling (+inf when unused)
  int round_mid;            // round the row-scaled value to float32
};

__device__ __forceinline__ double xform(const CsrXform& t, double v, double rs, int c) {
  if (t.row_scale) {
    v *= rs;
    if (t.round_mid) v = (double)(float)v;
  }
  if (t.col_div) v = v / t.col_div[c];
  if (t.clip) v = fmin(v, t.clip[c]);
  return fmin(v, t.max_value);
}

template <class T>
__global__ void __launch_bounds__(256) csr_row_sums_kernel(const long long* __restrict__ indptr,
                                                           const T* __restrict__ data, int n,
                                                           double* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  double s = 0.0;
  for (long long j = indptr[row] + lane; j < indptr[row + 1]; j += 64) s += (double)data[j];
  s = wave_sum(s);
  if (lane == 0) out[row] = s;
}

constexpr int kCsWaves = 4;
constexpr int kCsTile = 1536;  // columns per LDS tile: 3 arrays x 4 waves x 1536 x 8 B = 144 KiB

template <class T>
__global__ void __launch_bounds__(256) csr_col_stats_kernel(
    const long long* __restrict__ indptr, const int* __restrict__ indices,
    const T* __restrict__ data, int n, int n_out, int rows_per_block, CsrXform t,
    const double* __restrict__ center, double* __restrict__ psum, double* __restrict__ psq,
    double* __restrict__ pcnt) {
  extern __shared__ double smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* aS = smem + (size_t)wave * kCsTile;
  double* aQ = smem + (size_t)(kCsWaves + wave) * kCsTile;
  double* aC = smem + (size_t)(2 * kCsWaves + wave) * kCsTile;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(n, r0 + rows_per_block);
  for (int t0 = 0; t0 < n_out; t0 += kCsTile) {
    const int tw = min(kCsTile, n_out - t0);
    for (int e = threadIdx.x; e < kCsWaves * kCsTile; e += 256) {
      smem[e] = 0.0;
      smem[kCsWaves * kCsTile + e] = 0.0;
      smem[2 * kCsWaves * kCsTile + e] = 0.0;
    }
    __syncthreads();
    // kCsU entries per lane per trip, their index / value loads issued together: one
    // wave per SIMD paid a full memory latency per entry (12 ms per call on a 500k x 3000
    // CSR, profiles/r3aa_harmony_500k_kernel_summary.txt).  A row's columns are distinct,
    // so the lanes' LDS updates never collide.
    constexpr int kCsU = 4;
    for (int row = r0 + wave; row < r1; row += kCsWaves) {
      const double rs = t.row_scale ? t.row_scale[row] : 1.0;
      const long long e = indptr[row + 1];
      for (long long j0 = indptr[row] + lane; j0 < e; j0 += 64 * kCsU) {
        int cc[kCsU];
        T vv[kCsU];
#pragma unroll
        for (int u = 0; u < kCsU; ++u) {
          const long long j = j0 + 64 * u;
          const bool ok = j < e;
          cc[u] = ok ? indices[j] : -1;
          vv[u] = ok ? data[j] : T(0);
        }
#pragma unroll
        for (int u = 0; u < kCsU; ++u) {
          int c = cc[u];
          if (c < 0) continue;
          if (t.col_map) c = t.col_map[c];
          c -= t0;
          if (c < 0 || c >= tw) continue;
          const int oc = c + t0;
          const double v = xform(t, (double)vv[u], rs, oc);
          const double dv = center ? v - center[oc] : v;
          aS[c] += v;
          aQ[c] += dv * dv;
          aC[c] += 1.0;
        }
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < tw; c += 256) {
      double s = 0.0, q = 0.0, k = 0.0;
#pragma unroll
      for (int w = 0; w < kCsWaves; ++w) {
        s += smem[(size_t)w * kCsTile + c];
        q += smem[(size_t)(kCsWaves + w) * kCsTile + c];
        k += smem[(size_t)(2 * kCsWaves + w) * kCsTile + c];
      }
      const size_t o = (size_t)blockIdx.x * n_out + t0 + c;
      psum[o] = s;
      psq[o] = q;
      pcnt[o] = k;
    }
    __syncthreads();
  }
}

template <class T, class O>
__global__ void __launch_bounds__(256) csr_transform_kernel(const long long* __restrict__ indptr,
                                                            const int* __restrict__ indices,
                                                            const T* __restrict__ data, int n,
                                                            CsrXform t, O* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const double rs = t.row_scale ? t.row_scale[row] : 1.0;
  for (long long j = indptr[row] + lane; j < indptr[row + 1]; j += 64) {
    int c = indices[j];
    if (t.col_map) c = t.col_map[c];
    out[j] = c < 0 ? (O)-1 : (O)xform(t, (double)data[j], rs, c);
  }
}

template <class T, class O>
__global__ void __launch_bounds__(256) csr_densify_kernel(const long long* __restrict__ indptr,
                                                          const int* __restrict__ indices,
                                                          const T* __restrict__ data, int n,
                                                          CsrXform t, O* __restrict__ out,
                                                          long long ldo) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const double rs = t.row_scale ? t.row_scale[row] : 1.0;
  O* orow = out + (long long)row * ldo;
  for (long long j = indptr[row] + lane; j < indptr[row + 1]; j += 64) {
    int c = indices[j];
    if (t.col_map) c = t.col_map[c];
    if (c >= 0) orow[c] = (O)xform(t, (double)data[j], rs, c);
  }
}

__global__ void __launch_bounds__(256) radix_hist_kernel(const float* __restrict__ x, long long m,
                                                         unsigned int prefix, unsigned int mask,
                                                         int shift,
                                                         unsigned long long* __restrict__ hist) {
  __shared__ unsigned int h[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < m; i += stride) {
    const float v = x[i];
    if (!(v >= 0.0f)) continue;               // dropped entries (and NaN) are skipped
    const unsigned int b = __float_as_uint(v);
    if ((b & mask) == prefix) atomicAdd(&h[(b >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// ---------------------------------------------------------------------------- SpMM
// out (n x K) = T(A) . B with B (n_out x K) dense float32: one wave per row, each lane
// accumulates K partial dot products over its entries, then K wave reductions (fixed
// order -> deterministic).  The usage refit numerator x W^T of fit_H_online (cnmf.py:
// 358-362) on a sparse / transformed (scaled HVG subset) matrix without densifying it.
template <class T, int KB>
__global__ void __launch_bounds__(256) csr_spmm_kernel(const long long* __restrict__ indptr,
                                                       const int* __restrict__ indices,
                                                       const T* __restrict__ data, int n,
                                                       CsrXform t, const float* __restrict__ B,
                                                       int K, float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const double rs = t.row_scale ? t.row_scale[row] : 1.0;
  float acc[KB];
#pragma unroll
  for (int k = 0; k < KB; ++k) acc[k] = 0.f;
  for (long long j = indptr[row] + lane; j < indptr[row + 1]; j += 64) {
    int c = indices[j];
    if (t.col_map) c = t.col_map[c];
    if (c < 0) continue;
    const float v = (float)xform(t, (double)data[j], rs, c);
    const float* b = B + (long long)c * K;
#pragma unroll
    for (int k = 0; k < KB; ++k)
      if (k < K) acc[k] = fmaf(v, b[k], acc[k]);
  }
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    if (k < K) {
      const float s = wave_sum(acc[k]);
      if (lane == k) out[(long long)row * K + k] = s;
    }
  }
}

// out (n_out x K) = T(A)^T . B with B (n x K) dense: per-wave LDS tiles of (columns x K)
// float64 accumulators, rows walked in order by their wave (distinct columns per row ->
// no conflicts), waves combined in fixed order into per-workgroup partials.  The spectra
// refit numerator U^T X (cnmf.py:994) and the OLS X^T Y (cnmf.py:103-120) on CSR.
constexpr int kTsLds = 4608;   // doubles per wave: 4 waves x 4608 x 8 B = 144 KiB
template <class T, class TB, int KB>
__global__ void __launch_bounds__(256) csr_tspmm_kernel(const long long* __restrict__ indptr,
                                                        const int* __restrict__ indices,
                                                        const T* __restrict__ data, int n,
                                                        int n_out, int rows_per_block,
                                                        CsrXform t, const TB* __restrict__ B,
                                                        int K, double* __restrict__ part) {
  extern __shared__ double smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* acc = smem + (size_t)wave * kTsLds;
  const int tc = kTsLds / K;   // columns per tile
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(n, r0 + rows_per_block);
  for (int t0 = 0; t0 < n_out; t0 += tc) {
    const int tw = min(tc, n_out - t0);
    for (int e = threadIdx.x; e < 4 * kTsLds; e += 256) smem[e] = 0.0;
    __syncthreads();
    for (int row = r0 + wave; row < r1; row += 4) {
      double bk[KB];
#pragma unroll
      for (int k = 0; k < KB; ++k) bk[k] = k < K ? (double)B[(long long)row * K + k] : 0.0;
      const double rs = t.row_scale ? t.row_scale[row] : 1.0;
      const long long e = indptr[row + 1];
      for (long long j = indptr[row] + lane; j < e; j += 64) {
        int c = indices[j];
        if (t.col_map) c = t.col_map[c];
        c -= t0;
        if (c < 0 || c >= tw) continue;
        const double v = xform(t, (double)data[j], rs, c + t0);
        double* a = acc + (long long)c * K;
#pragma unroll
        for (int k = 0; k < KB; ++k)
          if (k < K) a[k] = fma(v, bk[k], a[k]);
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < tw * K; e += 256) {
      const double s = smem[e] + smem[kTsLds + e] + smem[2 * kTsLds + e] + smem[3 * kTsLds + e];
      part[((size_t)blockIdx.x * n_out + t0) * K + e] = s;
    }
    __syncthreads();
  }
}

}  // namespace cnmf

using cnmf::CsrXform;

static CsrXform make_xform(const double* row_scale, const int* col_map, const double* col_div,
                           const double* clip, double max_value, int round_mid) {
  CsrXform t;
  t.row_scale = row_scale;
  t.col_map = col_map;
  t.col_div = col_div;
  t.clip = clip;
  t.max_value = max_value;
  t.round_mid = round_mid;
  return t;
}

extern "C" hipError_t cnmf_csr_row_sums(const long long* indptr, const void* data, int f64, int n,
                                        double* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((n + 3) / 4);
  if (f64)
    hipLaunchKernelGGL(cnmf::csr_row_sums_kernel<double>, grid, dim3(256), 0, stream, indptr,
                       (const double*)data, n, out);
  else
    hipLaunchKernelGGL(cnmf::csr_row_sums_kernel<float>, grid, dim3(256), 0, stream, indptr,
                       (const float*)data, n, out);
  return hipGetLastError();
}

extern "C" int cnmf_csr_stats_blocks(int n) {
  // ~2 workgroups per CU, at least 64 rows each
  int nb = (n + 63) / 64;
  return nb < 512 ? (nb > 0 ? nb : 1) : 512;
}

extern "C" hipError_t cnmf_csr_col_stats(const long long* indptr, const int* indices,
                                         const void* data, int f64, int n, int n_out,
                                         const double* row_scale, const int* col_map,
                                         const double* col_div, const double* clip,
                                         double max_value, int round_mid, const double* center, double* psum,
                                         double* psq, double* pcnt, hipStream_t stream) {
  if (n <= 0 || n_out <= 0) return hipSuccess;
  const int nb = cnmf_csr_stats_blocks(n);
  const int rpb = (n + nb - 1) / nb;
  const size_t lds = (size_t)3 * cnmf::kCsWaves * cnmf::kCsTile * sizeof(double);
  const CsrXform t = make_xform(row_scale, col_map, col_div, clip, max_value, round_mid);
  hipError_t e;
  if (f64) {
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cnmf::csr_col_stats_kernel<double>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cnmf::csr_col_stats_kernel<double>, dim3(nb), dim3(256), lds, stream,
                       indptr, indices, (const double*)data, n, n_out, rpb, t, center, psum, psq,
                       pcnt);
  } else {
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cnmf::csr_col_stats_kernel<float>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cnmf::csr_col_stats_kernel<float>, dim3(nb), dim3(256), lds, stream,
                       indptr, indices, (const float*)data, n, n_out, rpb, t, center, psum, psq,
                       pcnt);
  }
  return hipGetLastError();
}

extern "C" hipError_t cnmf_csr_transform(const long long* indptr, const int* indices,
                                         const void* data, int f64, int n,
                                         const double* row_scale, const int* col_map,
                                         const double* col_div, const double* clip,
                                         double max_value, int round_mid, void* out, int out_f64,
                                         hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((n + 3) / 4);
  const CsrXform t = make_xform(row_scale, col_map, col_div, clip, max_value, round_mid);
#define CNMF_XF(TI, TO)                                                                      \
  hipLaunchKernelGGL((cnmf::csr_transform_kernel<TI, TO>), grid, dim3(256), 0, stream, indptr, \
                     indices, (const TI*)data, n, t, (TO*)out)
  if (f64 && out_f64) CNMF_XF(double, double);
  else if (f64) CNMF_XF(double, float);
  else if (out_f64) CNMF_XF(float, double);
  else CNMF_XF(float, float);
#undef CNMF_XF
  return hipGetLastError();
}

extern "C" hipError_t cnmf_csr_densify(const long long* indptr, const int* indices,
                                       const void* data, int f64, int n, const double* row_scale,
                                       const int* col_map, const double* col_div,
                                       const double* clip, double max_value, int round_mid, void* out,
                                       int out_f64, long long ldo, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((n + 3) / 4);
  const CsrXform t = make_xform(row_scale, col_map, col_div, clip, max_value, round_mid);
#define CNMF_DN(TI, TO)                                                                      \
  hipLaunchKernelGGL((cnmf::csr_densify_kernel<TI, TO>), grid, dim3(256), 0, stream, indptr,   \
                     indices, (const TI*)data, n, t, (TO*)out, ldo)
  if (f64 && out_f64) CNMF_DN(double, double);
  else if (f64) CNMF_DN(double, float);
  else if (out_f64) CNMF_DN(float, double);
  else CNMF_DN(float, float);
#undef CNMF_DN
  return hipGetLastError();
}

extern "C" hipError_t cnmf_radix_hist(const float* x, long long m, unsigned int prefix,
                                      unsigned int mask, int shift, unsigned long long* hist,
                                      hipStream_t stream) {
  if (m <= 0) return hipSuccess;
  long long nb = (m + 255) / 256;
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(cnmf::radix_hist_kernel, dim3((unsigned)nb), dim3(256), 0, stream, x, m,
                     prefix, mask, shift, hist);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_csr_spmm(const long long* indptr, const int* indices, const void* data,
                                    int f64, int n, const double* row_scale, const int* col_map,
                                    const double* col_div, const double* clip, double max_value,
                                    int round_mid, const float* B, int K, float* out,
                                    hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (K < 1 || K > 64) return hipErrorInvalidValue;
  const dim3 grid((n + 3) / 4);
  const CsrXform t = make_xform(row_scale, col_map, col_div, clip, max_value, round_mid);
#define CNMF_SP(TI, KB)                                                                      \
  hipLaunchKernelGGL((cnmf::csr_spmm_kernel<TI, KB>), grid, dim3(256), 0, stream, indptr,     \
                     indices, (const TI*)data, n, t, B, K, out)
  if (f64) {
    if (K <= 16) CNMF_SP(double, 16); else if (K <= 32) CNMF_SP(double, 32); else CNMF_SP(double, 64);
  } else {
    if (K <= 16) CNMF_SP(float, 16); else if (K <= 32) CNMF_SP(float, 32); else CNMF_SP(float, 64);
  }
#undef CNMF_SP
  return hipGetLastError();
}

extern "C" int cnmf_csr_tspmm_blocks(int n) {
  int nb = (n + 255) / 256;
  return nb < 256 ? (nb > 0 ? nb : 1) : 256;
}

template <class TI, class TB, int KB>
static hipError_t launch_tspmm(const long long* indptr, const int* indices, const void* data,
                               int n, int n_out, CsrXform t, const void* B, int K, double* part,
                               hipStream_t stream) {
  const size_t lds = (size_t)4 * cnmf::kTsLds * sizeof(double);
  hipError_t e = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&cnmf::csr_tspmm_kernel<TI, TB, KB>),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int nb = cnmf_csr_tspmm_blocks(n);
  const int rpb = (n + nb - 1) / nb;
  hipLaunchKernelGGL((cnmf::csr_tspmm_kernel<TI, TB, KB>), dim3(nb), dim3(256), lds, stream,
                     indptr, indices, (const TI*)data, n, n_out, rpb, t, (const TB*)B, K, part);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_csr_tspmm(const long long* indptr, const int* indices,
                                     const void* data, int f64, int n, int n_out,
                                     const double* row_scale, const int* col_map,
                                     const double* col_div, const double* clip, double max_value,
                                     int round_mid, const void* B, int b_f64, int K,
                                     double* part, hipStream_t stream) {
  if (n <= 0 || n_out <= 0) return hipSuccess;
  if (K < 1 || K > 64) return hipErrorInvalidValue;
  const CsrXform t = make_xform(row_scale, col_map, col_div, clip, max_value, round_mid);
#define CNMF_TS(TI, TB)                                                                           \
  return K <= 16 ? launch_tspmm<TI, TB, 16>(indptr, indices, data, n, n_out, t, B, K, part, stream) \
       : K <= 32 ? launch_tspmm<TI, TB, 32>(indptr, indices, data, n, n_out, t, B, K, part, stream) \
                 : launch_tspmm<TI, TB, 64>(indptr, indices, data, n, n_out, t, B, K, part, stream)
  if (f64 && b_f64) { CNMF_TS(double, double); }
  if (f64) { CNMF_TS(double, float); }
  if (b_f64) { CNMF_TS(float, double); }
  CNMF_TS(float, float);
#undef CNMF_TS
}
