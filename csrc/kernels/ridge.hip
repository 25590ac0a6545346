// Harmony's MOE ridge correction on the f64 matrix cores (reference
// moe_correct_ridge, /root/reference/src/cnmf/preprocess.py:9-18, applied to the
// expression matrix by harmony_correct_X, :342-388):
//     W_k = (Phi_Rk Phi_moe^T + lamb)^-1 Phi_Rk X,  W_k[0] = 0,  X -= sum_k Phi_Rk^T W_k,
// Phi_Rk = Phi_moe * R[k].  Phi_moe = [1; one-hot batch levels]: every cell is in the
// intercept row and in exactly one level of each covariate, so nothing here materialises
// Phi_Rk (K x B1 x N, ~GB at 500k cells) and no dense (K B1) x N GEMM runs:
//
//  * ridge_seg_tgemm_kernel: Y[k, b, f] = sum over the cells n of level b of R[k, n] X[n, f]
//    -- one workgroup per (level, 32-cluster tile, 64-feature tile) walks that level's
//    cell list (gathered rows of X and of R^T), 4 waves splitting the cells, partials
//    added in wave order (deterministic, no atomics).  The same kernel with X := Phi_moe^T
//    gives the ridge systems' Gram part A[k, b, c].
//  * ridge_apply_kernel: cells sorted by their combination of levels; for a combination
//    the correction is one (cells x K) (K x F) product with Wc = sum of its levels' W_b,
//    so every output is X - R^T Wc rounded ONCE from float64 (the reference subtracts
//    cluster by cluster).
// f64 16x16x4 MFMA: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15];
// D: col = lane&15, row = (lane>>4) + 4*reg.
#include <hip/hip_runtime.h>

namespace cnmf {

typedef double rg_f64x4 __attribute__((ext_vector_type(4)));

// out[k][f] (row stride ldo) = sum_{i in [s0, s1)} Rt[idx[i]][k] * X[idx[i]][f], k < Kc,
// f < F; grid: (segments, k tiles of 32, f tiles of 64)
template <typename TX>
__global__ void __launch_bounds__(256) ridge_seg_tgemm_kernel(
    const double* __restrict__ Rt, long long ldr, int Kc, const TX* __restrict__ X,
    long long ldx, int F, const int* __restrict__ idx, const long long* __restrict__ seg,
    double* __restrict__ out, long long seg_stride, long long ldo) {
  __shared__ double red[4][32][64 + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sgi = blockIdx.x;
  const int k0 = blockIdx.y * 32, f0 = blockIdx.z * 64;
  const long long s0 = seg[sgi], s1 = seg[sgi + 1];
  const int ar = lane & 15, ak = lane >> 4;
  rg_f64x4 acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = rg_f64x4{0.0, 0.0, 0.0, 0.0};
  // wave w takes cell steps of 4 cells: w, w + 4, ... (step = cells s0 + 4 t .. + 3)
  for (long long t = s0 + 4 * wave; t < s1; t += 16) {
    const long long i = t + ak;
    const bool ok = i < s1;
    const long long n = ok ? (long long)idx[i] : 0;
    double av[2], bv[4];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int k = k0 + 16 * a + ar;
      av[a] = (ok && k < Kc) ? Rt[n * ldr + k] : 0.0;
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int f = f0 + 16 * b + ar;
      bv[b] = (ok && f < F) ? (double)X[n * ldx + f] : 0.0;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
  }
  // wave partials -> LDS, summed in wave order
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][16 * a + ak + 4 * r][16 * b + ar] = acc[a][b][r];
  __syncthreads();
  double* o = out + (long long)sgi * seg_stride;
  for (int e = threadIdx.x; e < 32 * 64; e += 256) {
    const int kk = e / 64, ff = e % 64;
    const int k = k0 + kk, f = f0 + ff;
    if (k < Kc && f < F) {
      const double v = ((red[0][kk][ff] + red[1][kk][ff]) + red[2][kk][ff]) + red[3][kk][ff];
      o[(long long)k * ldo + f] = v;
    }
  }
}

// Chunked segments: when (levels x tiles) gives too few workgroups to fill the chip (the
// 50-PC Harmony ridge: 16 levels x 4 cluster tiles x 1 feature tile = 64 workgroups each
// walking up to all 500k cells, 35 ms per call, profiles/r5i_*), the host cuts every
// level's cell list into chunks, ridge_seg_tgemm_kernel writes one partial per chunk and
// this kernel sums a level's chunks in chunk order (deterministic):
//   out[s][k][f] = sum_{c in [cfirst[s], cfirst[s+1])} part[c][k][f]   (part: Kc x F dense)
__global__ void __launch_bounds__(256) ridge_seg_reduce_kernel(
    const double* __restrict__ part, const int* __restrict__ cfirst, int Kc, int F,
    double* __restrict__ out, long long seg_stride, long long ldo) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long kf = (long long)Kc * F;
  if (e >= kf) return;
  const int s = blockIdx.y;
  const int k = (int)(e / F), f = (int)(e - (long long)k * F);
  double acc = 0.0;
  for (int c = cfirst[s]; c < cfirst[s + 1]; ++c) acc += part[(long long)c * kf + e];
  out[(long long)s * seg_stride + (long long)k * ldo + f] = acc;
}

// Y[n][f] = (TY)((double)X[n][f] - sum_k Rt[n][k] * Wc[combo][k][f]) for the cells of
// every block: blk[b] = (combo, first position in the combo-sorted cell order, count <= 64);
// grid (blocks, f tiles of 64); 4 waves x 16 cells
template <typename TX>
__global__ void __launch_bounds__(256) ridge_apply_kernel(
    const double* __restrict__ Rt, long long ldr, int Kc, const TX* __restrict__ X,
    long long ldx, TX* __restrict__ Y, long long ldy, int F, const int* __restrict__ order,
    const int* __restrict__ blk, const double* __restrict__ Wc, long long wc_combo,
    long long ldw) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int combo = blk[3 * blockIdx.x], p0 = blk[3 * blockIdx.x + 1], cnt = blk[3 * blockIdx.x + 2];
  const int f0 = blockIdx.y * 64;
  const int ar = lane & 15, ak = lane >> 4;
  const int cr = 16 * wave + ar;            // this lane's A row (cell) within the block
  const bool rok = cr < cnt;
  const long long nA = rok ? (long long)order[p0 + cr] : 0;
  const double* __restrict__ W = Wc + (long long)combo * wc_combo;
  rg_f64x4 acc[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) acc[b] = rg_f64x4{0.0, 0.0, 0.0, 0.0};
  for (int k4 = 0; k4 < Kc; k4 += 4) {
    const int k = k4 + ak;
    const double av = (rok && k < Kc) ? Rt[nA * ldr + k] : 0.0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int f = f0 + 16 * b + ar;
      const double bv = (k < Kc && f < F) ? W[(long long)k * ldw + f] : 0.0;
      acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[b], 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = 16 * wave + ak + 4 * r;    // D row -> cell of the block
    if (c < cnt) {
      const long long n = order[p0 + c];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int f = f0 + 16 * b + ar;
        if (f < F) Y[n * ldy + f] = (TX)((double)X[n * ldx + f] - acc[b][r]);
      }
    }
  }
}

}  // namespace cnmf

extern "C" hipError_t cnmf_ridge_seg_tgemm(const double* Rt, long long ldr, int Kc, const void* X,
                                           int x_f64, long long ldx, int F, const int* idx,
                                           const long long* seg, int nseg, double* out,
                                           long long seg_stride, long long ldo,
                                           hipStream_t stream) {
  if (nseg <= 0 || F <= 0 || Kc <= 0) return hipSuccess;
  if (ldr < Kc || ldx < F || ldo < F) return hipErrorInvalidValue;
  const dim3 grid(nseg, (Kc + 31) / 32, (F + 63) / 64);
  if (x_f64)
    hipLaunchKernelGGL(cnmf::ridge_seg_tgemm_kernel<double>, grid, dim3(256), 0, stream, Rt, ldr,
                       Kc, (const double*)X, ldx, F, idx, seg, out, seg_stride, ldo);
  else
    hipLaunchKernelGGL(cnmf::ridge_seg_tgemm_kernel<float>, grid, dim3(256), 0, stream, Rt, ldr, Kc,
                       (const float*)X, ldx, F, idx, seg, out, seg_stride, ldo);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_ridge_seg_reduce(const double* part, const int* cfirst, int nseg,
                                            int Kc, int F, double* out, long long seg_stride,
                                            long long ldo, hipStream_t stream) {
  if (nseg <= 0 || F <= 0 || Kc <= 0) return hipSuccess;
  if (ldo < F || seg_stride < (long long)(Kc - 1) * ldo + F) return hipErrorInvalidValue;
  const long long kf = (long long)Kc * F;
  const dim3 grid((unsigned)((kf + 255) / 256), (unsigned)nseg);
  hipLaunchKernelGGL(cnmf::ridge_seg_reduce_kernel, grid, dim3(256), 0, stream, part, cfirst, Kc,
                     F, out, seg_stride, ldo);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_ridge_apply(const double* Rt, long long ldr, int Kc, const void* X,
                                       int x_f64, long long ldx, void* Y, long long ldy, int F,
                                       const int* order, const int* blk, int nblk, const double* Wc,
                                       long long wc_combo, long long ldw, hipStream_t stream) {
  if (nblk <= 0 || F <= 0) return hipSuccess;
  if (ldr < Kc || ldx < F || ldy < F || ldw < F) return hipErrorInvalidValue;
  const dim3 grid(nblk, (F + 63) / 64);
  if (x_f64)
    hipLaunchKernelGGL(cnmf::ridge_apply_kernel<double>, grid, dim3(256), 0, stream, Rt, ldr, Kc,
                       (const double*)X, ldx, (double*)Y, ldy, F, order, blk, Wc, wc_combo, ldw);
  else
    hipLaunchKernelGGL(cnmf::ridge_apply_kernel<float>, grid, dim3(256), 0, stream, Rt, ldr, Kc,
                       (const float*)X, ldx, (float*)Y, ldy, F, order, blk, Wc, wc_combo, ldw);
  return hipGetLastError();
}
