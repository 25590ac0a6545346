// Fused prediction error of the consensus / k-selection step (the
// reference's ``((X - U S)**2).sum()`` at cnmf.py:1100-1104, which materialises the N x G
// reconstruction in float64 on the host).  By the trace identity
//     ||X - U S||^2 = ||X||^2 - 2 <X, U S> + <U^T U, S S^T>,
// and the first two terms are ONE streaming pass over the resident X here: each
// workgroup owns 64 rows of X, keeps the 16-row usage fragments of each of its 4 waves in
// VGPRs, and walks the genes in 64-column tiles; the tile of P = U S is formed on the f64
// matrix cores (v_mfma_f64_16x16x4_f64, U and S in float64 as the reference) straight in
// the accumulator layout, and every accumulator is folded with the X element at the same
// position: cross += x * p, xsq += x * x (float64).  U S is never written anywhere, and X
// is read once, in its own dtype (float32).  Per-workgroup float64 partials, summed by the
// host in workgroup order (deterministic).  The K x K term is a tiny host/torch product.
#include <hip/hip_runtime.h>

namespace cnmf {

typedef double pe_f64x4 __attribute__((ext_vector_type(4)));

constexpr int kPeMaxKS = 32;   // K <= 128 (k-steps of 4)

// f64 16x16x4 MFMA: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15];
// D: col = lane&15, row = (lane>>4) + 4*reg.
template <int KS>
__global__ void __launch_bounds__(256) predict_err_kernel(
    const float* __restrict__ X, long long ldx, const double* __restrict__ U, long long ldu,
    const double* __restrict__ S, long long lds, int N, int G, int K,
    double* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = blockIdx.x * 64 + wave * 16;
  const int ar = lane & 15, ak = lane >> 4;
  // this wave's 16 usage rows as A fragments: a[s] = U[r0 + ar][4 s + ak]
  double a[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + ak;
    a[s] = (r0 + ar < N && k < K) ? U[(long long)(r0 + ar) * ldu + k] : 0.0;
  }
  double cross = 0.0, xsq = 0.0;
  for (int c0 = 0; c0 < G; c0 += 64) {
    pe_f64x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = pe_f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 4 * s + ak;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = c0 + 16 * j + ar;
        const double b = (k < K && col < G) ? S[(long long)k * lds + col] : 0.0;
        acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b, acc[j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = c0 + 16 * j + ar;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + ak + 4 * r;
        if (row < N && col < G) {
          const double x = (double)X[(long long)row * ldx + col];
          cross = fma(x, acc[j][r], cross);
          xsq = fma(x, x, xsq);
        }
      }
    }
  }
  // block reduction in a fixed order (deterministic)
  __shared__ double sc[256], sx[256];
  sc[threadIdx.x] = cross;
  sx[threadIdx.x] = xsq;
  __syncthreads();
  for (int d = 128; d > 0; d >>= 1) {
    if (threadIdx.x < d) {
      sc[threadIdx.x] += sc[threadIdx.x + d];
      sx[threadIdx.x] += sx[threadIdx.x + d];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = sc[0];
    part[2 * blockIdx.x + 1] = sx[0];
  }
}

template <int KS>
static hipError_t launch_pe(const float* X, long long ldx, const double* U, long long ldu,
                            const double* S, long long lds, int N, int G, int K, double* part,
                            hipStream_t st) {
  hipLaunchKernelGGL((predict_err_kernel<KS>), dim3((N + 63) / 64), dim3(256), 0, st, X, ldx, U,
                     ldu, S, lds, N, G, K, part);
  return hipGetLastError();
}

}  // namespace cnmf

// part: 2 * ceil(N / 64) doubles (cross, xsq per workgroup)
extern "C" hipError_t cnmf_predict_err(const float* X, long long ldx, const double* U,
                                       long long ldu, const double* S, long long lds, int N,
                                       int G, int K, double* part, hipStream_t stream) {
  if (N <= 0 || G <= 0) return hipSuccess;
  if (K < 1 || K > 4 * cnmf::kPeMaxKS || ldu < K || lds < G || ldx < G)
    return hipErrorInvalidValue;
  const int ks = (K + 3) / 4;
  if (ks <= 1) return cnmf::launch_pe<1>(X, ldx, U, ldu, S, lds, N, G, K, part, stream);
  if (ks <= 2) return cnmf::launch_pe<2>(X, ldx, U, ldu, S, lds, N, G, K, part, stream);
  if (ks <= 4) return cnmf::launch_pe<4>(X, ldx, U, ldu, S, lds, N, G, K, part, stream);
  if (ks <= 8) return cnmf::launch_pe<8>(X, ldx, U, ldu, S, lds, N, G, K, part, stream);
  if (ks <= 16) return cnmf::launch_pe<16>(X, ldx, U, ldu, S, lds, N, G, K, part, stream);
  return cnmf::launch_pe<32>(X, ldx, U, ldu, S, lds, N, G, K, part, stream);
}
