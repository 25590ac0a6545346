// Exact per-column moments (sum x, sum x^2) of a dense device matrix as integer digits --
// the GPU side of models/hvg.py exact_moment_digits (host side: csrc/io/npzio.cpp
// exact_col_moments, same window and digit layout, so both produce the same integers).
// Every value x = +-m 2^e (m < 2^53) is added EXACTLY into base-2^32 digits held in int64:
// integer sums are associative, so the statistics of a sharded prepare (digits
// all-reduced over the ranks) equal the single-process ones bit for bit, on any device
// (the reference's column statistics: cnmf.py:128-131, 570-580,
// 674-681).
//
// Layout: thread (column c, row chunk y) walks its rows of column c (consecutive threads =
// consecutive columns: coalesced row-major loads) and keeps its 13 + 25 digits in LDS
// ([digit][thread]: conflict-free), then writes them to its chunk's partial; a second
// kernel sums the chunk partials (int64, exact in any order).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cnmf {

constexpr int kExLsb1 = -192, kExD1 = 13;
constexpr int kExLsb2 = -384, kExD2 = 25;
constexpr int kExD = kExD1 + kExD2;
constexpr int kExThreads = 128;

__device__ __forceinline__ bool ex_add_dev(double x, long long* s, int stride) {
  if (x == 0.0) return true;
  const unsigned long long bits = __double_as_longlong(x);
  const int ef = (int)((bits >> 52) & 0x7FF);
  // |x| in [2^-126, 2^127]: biased exponent in [897, 1150] (and the mantissa bound for
  // exactly 2^127 is handled by the upper test)
  if (ef < 897 || ef > 1150 || (ef == 1150 && (bits & 0xFFFFFFFFFFFFFull))) return false;
  const unsigned long long m = (bits & 0xFFFFFFFFFFFFFull) | (1ull << 52);
  const int e = ef - 1075;                       // |x| = m 2^e
  const long long sg = (bits >> 63) ? -1 : 1;
  {
    const int sh = e - kExLsb1, dd = sh >> 5, o = sh & 31;
    const unsigned long long lo = m << o;
    const unsigned long long hi = o ? (m >> (64 - o)) : 0ull;   // bits 64.. of m << o
    s[(dd) * stride] += sg * (long long)(lo & 0xFFFFFFFFull);
    s[(dd + 1) * stride] += sg * (long long)(lo >> 32);
    s[(dd + 2) * stride] += sg * (long long)hi;
  }
  {
    // m^2 < 2^106 as (p1:p0); shifted by o < 32 it spans < 2^138
    const unsigned long long p0 = m * m, p1 = __umul64hi(m, m);
    const int sh = 2 * e - kExLsb2, dd = sh >> 5, o = sh & 31;
    const unsigned long long q0 = p0 << o;
    const unsigned long long q1 = (p1 << o) | (o ? (p0 >> (64 - o)) : 0ull);
    const unsigned long long q2 = o ? (p1 >> (64 - o)) : 0ull;
    long long* t = s + kExD1 * stride;
    t[(dd) * stride] += (long long)(q0 & 0xFFFFFFFFull);
    t[(dd + 1) * stride] += (long long)(q0 >> 32);
    t[(dd + 2) * stride] += (long long)(q1 & 0xFFFFFFFFull);
    t[(dd + 3) * stride] += (long long)(q1 >> 32);
    t[(dd + 4) * stride] += (long long)q2;
  }
  return true;
}

template <typename T>
__global__ void __launch_bounds__(kExThreads) exact_moments_kernel(
    const T* __restrict__ X, long long ld, long long rows, int G, long long* __restrict__ part,
    unsigned long long* __restrict__ bad) {
  __shared__ long long sd[kExD * kExThreads];
  const int c = blockIdx.x * kExThreads + threadIdx.x;
  long long* s = sd + threadIdx.x;
  for (int i = 0; i < kExD; ++i) s[i * kExThreads] = 0;
  const long long r0 = rows * blockIdx.y / gridDim.y, r1 = rows * (blockIdx.y + 1) / gridDim.y;
  unsigned long long nb = 0;
  if (c < G) {
    for (long long r = r0; r < r1; ++r)
      if (!ex_add_dev((double)X[r * ld + c], s, kExThreads)) ++nb;
  }
  if (nb) atomicAdd(bad, nb);
  if (c < G) {
    long long* o = part + ((long long)blockIdx.y * G + c) * kExD;
    for (int i = 0; i < kExD; ++i) o[i] = s[i * kExThreads];
  }
}

// out[g][i] = sum over chunks of part[chunk][g][i] (int64: exact, any order)
__global__ void exact_moments_sum_kernel(const long long* __restrict__ part, int chunks, int G,
                                         long long* __restrict__ out) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long tot = (long long)G * kExD;
  if (i >= tot) return;
  long long v = 0;
  for (int ch = 0; ch < chunks; ++ch) v += part[(long long)ch * tot + i];
  out[i] = v;
}

}  // namespace cnmf

// part: chunks * G * 38 int64 scratch; out: G * 38 int64 (digits1 | digits2 per column);
// bad: one uint64 (values outside the window)
extern "C" hipError_t cnmf_exact_moments(const void* X, int is_f64, long long ld, long long rows,
                                         int G, int chunks, long long* part, long long* out,
                                         unsigned long long* bad, hipStream_t stream) {
  if (G <= 0) return hipSuccess;
  if (chunks < 1 || ld < G || rows < 0) return hipErrorInvalidValue;
  const dim3 grid((G + cnmf::kExThreads - 1) / cnmf::kExThreads, chunks);
  if (is_f64)
    hipLaunchKernelGGL(cnmf::exact_moments_kernel<double>, grid, dim3(cnmf::kExThreads), 0, stream,
                       (const double*)X, ld, rows, G, part, bad);
  else
    hipLaunchKernelGGL(cnmf::exact_moments_kernel<float>, grid, dim3(cnmf::kExThreads), 0, stream,
                       (const float*)X, ld, rows, G, part, bad);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const long long tot = (long long)G * cnmf::kExD;
  hipLaunchKernelGGL(cnmf::exact_moments_sum_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256),
                     0, stream, part, chunks, G, out);
  return hipGetLastError();
}
