// One-pass column statistics of the dense data matrix for the NMF engine (SURVEY.md §2.4
// H9 / G7): per gene the smallest positive entry, the float64 sum of squares (the
// trace-trick ||X||^2) and a negative-entry flag; then the integer-count test of the
// split-precision GEMM (models/nmf.py _count_units): is every entry of column g an
// integer multiple of min_pos_g / d, d = 1..8?
//
// X is row-major (cells x genes): a thread owns one column of a row block, so a wave reads
// 64 consecutive genes of a row (coalesced).  Row blocks write partials [block][gene]
// that a second kernel reduces in block order -- deterministic, no float atomics (the
// sum of squares feeds the convergence test).  The integer test ORs "not a multiple"
// bits with atomicOr, which is order-independent.
#include <hip/hip_runtime.h>

namespace cnmf {

__global__ void colstats_partial_kernel(const float* __restrict__ X, long long ldx, int N, int G,
                                        int rows_per_block, float* __restrict__ pmin,
                                        double* __restrict__ psq, int* __restrict__ pneg) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(N, r0 + rows_per_block);
  float mn = __builtin_inff();
  double sq = 0.0;
  int neg = 0;
  for (int r = r0; r < r1; ++r) {
    const float v = X[(long long)r * ldx + g];
    if (v > 0.f) mn = fminf(mn, v);
    neg |= v < 0.f;
    sq += (double)v * (double)v;
  }
  const long long o = (long long)blockIdx.y * G + g;
  pmin[o] = mn;
  psq[o] = sq;
  pneg[o] = neg;
}

__global__ void colstats_reduce_kernel(const float* __restrict__ pmin,
                                       const double* __restrict__ psq,
                                       const int* __restrict__ pneg, int nb, int G,
                                       float* __restrict__ mn_out, double* __restrict__ sq_out,
                                       int* __restrict__ neg_out) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  float mn = __builtin_inff();
  double sq = 0.0;
  int neg = 0;
  for (int b = 0; b < nb; ++b) {
    const long long o = (long long)b * G + g;
    mn = fminf(mn, pmin[o]);
    sq += psq[o];
    neg |= pneg[o];
  }
  mn_out[g] = mn;
  sq_out[g] = sq;
  neg_out[g] = neg;
}

// bit d-1 of bad[g] set <=> some entry x of column g is not an integer multiple of
// mn_g / d to fp32 rounding (|c - rint(c)| > 4e-7 c + 1e-4, c = x d / mn_g) or c >= 65536
__global__ void count_unit_check_kernel(const float* __restrict__ X, long long ldx, int N, int G,
                                        int rows_per_block, const float* __restrict__ mn,
                                        unsigned* __restrict__ bad) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const float m = mn[g];
  if (!(m > 0.f) || isinf(m)) return;   // empty column: unit 1, checked by the host
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(N, r0 + rows_per_block);
  unsigned b = 0;
  for (int r = r0; r < r1 && b != 0xffu; ++r) {
    const float x = X[(long long)r * ldx + g];
    if (x == 0.f) continue;
#pragma unroll
    for (int d = 1; d <= 8; ++d) {
      const float c = x / (m / (float)d);
      const bool off = fabsf(c - rintf(c)) > 4e-7f * c + 1e-4f || c >= 65535.5f;
      b |= off ? (1u << (d - 1)) : 0u;
    }
  }
  if (b) atomicOr(bad + g, b);
}

}  // namespace cnmf

extern "C" int cnmf_colstats_blocks(int N) {
  // ~4096 threads' worth of row blocks: enough waves to stream X at HBM rate
  int nb = (N + 255) / 256;
  return nb < 1 ? 1 : (nb > 512 ? 512 : nb);
}

extern "C" hipError_t cnmf_colstats(const float* X, long long ldx, int N, int G, float* pmin,
                                    double* psq, int* pneg, float* mn, double* sq, int* neg,
                                    hipStream_t stream) {
  if (G <= 0) return hipSuccess;
  const int nb = cnmf_colstats_blocks(N);
  const int rpb = (N + nb - 1) / nb;
  hipLaunchKernelGGL(cnmf::colstats_partial_kernel, dim3((G + 255) / 256, nb), dim3(256), 0,
                     stream, X, ldx, N, G, rpb > 0 ? rpb : 1, pmin, psq, pneg);
  hipLaunchKernelGGL(cnmf::colstats_reduce_kernel, dim3((G + 255) / 256), dim3(256), 0, stream,
                     pmin, psq, pneg, nb, G, mn, sq, neg);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_count_unit_check(const float* X, long long ldx, int N, int G,
                                            const float* mn, unsigned* bad, hipStream_t stream) {
  if (G <= 0 || N <= 0) return hipSuccess;
  const int nb = cnmf_colstats_blocks(N);
  const int rpb = (N + nb - 1) / nb;
  hipLaunchKernelGGL(cnmf::count_unit_check_kernel, dim3((G + 255) / 256, nb), dim3(256), 0,
                     stream, X, ldx, N, G, rpb > 0 ? rpb : 1, mn, bad);
  return hipGetLastError();
}
