// Batched small Gram matrices on MFMA: out[r] (+)= X_r X_r^T for X_r = K x n (K <= 128),
// the hh^T / WW^T products of every NMF step.
//
// hipBLASLt runs these (R x K x n)(R x n x K) batched GEMMs with a 16x16 macro tile at
// ~3 % MFMA utilisation (profiles/r1_pmc_summary.txt: 20 us per call at K=10, n=5000,
// R=100).  Here one 1024-thread workgroup owns one replicate: each wave streams 16-column
// slabs, every lane loads ONE float4 (row m = lane&15, columns 4q..4q+3 with q = lane>>4)
// and feeds each of its four elements as both the A and the B operand of
// v_mfma_f32_16x16x4_f32 -- A[row m][k q] = X[m][c], B[k q][col m] = X[m][c] -- so the
// k index is a permutation of the column order shared by both operands and
// D[i][j] = sum_c X[i][c] X[j][c] needs no data movement.  K in (16, 32] uses the 2 x 2
// tile grid.  The 16 per-wave partial tiles are summed in wave order through LDS
// (deterministic), then written or accumulated.  K in (64, 128] (the padded wide ranks):
// gridDim.z = 4 workgroups per replicate, each owning one 64 x 64 block (row block
// z / 2, column block z % 2) with the rows of its A and B operands loaded separately.
#include <hip/hip_runtime.h>

#include "common.h"

namespace cnmf {

typedef float gf32x4 __attribute__((ext_vector_type(4)));

// T = 1 (K <= 16), 2 (K <= 32) or 4 (K <= 64) tiles per dimension.  T = 4 keeps 32
// accumulator tiles per lane: 256-thread workgroups (the register budget of one wave per
// SIMD, and the per-wave LDS reduction slab fits).
template <int T>
constexpr int gram_max_threads() { return T == 4 ? 256 : 1024; }

template <int T, bool WIDE = false>
__global__ void __launch_bounds__(gram_max_threads<T>()) gram_kernel(
    const float* __restrict__ X, long long x_rs, long long ldx, int K, int n,
    float* __restrict__ out, long long o_rs, int accumulate, const int* active,
    float* __restrict__ part, int per) {
  __shared__ float red[gram_max_threads<T>() / 64][T * T * 16 * 16 + 1];
  const int rep = blockIdx.x;
  if (active && active[rep] == 0) return;
  const float* __restrict__ x = X + (long long)rep * x_rs;
  // WIDE: this workgroup's 64 x 64 block of the K x K result
  const int ro = WIDE ? 64 * (int)(blockIdx.z >> 1) : 0, co = WIDE ? 64 * (int)(blockIdx.z & 1) : 0;
  // column split (gridDim.y > 1, few replicates): slice [c_beg, c_end) -> partial K x K
  const int c_beg = part ? (int)blockIdx.y * per : 0;
  const int c_end = part ? min(n, c_beg + per) : n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int m = lane & 15, q = lane >> 4;
  // Two accumulator sets (even / odd column of each float4) halve the dependent MFMA
  // chain, and GU slabs per iteration keep GU float4 loads in flight per lane (one
  // load per dependent chain was latency-bound: 16 us for K=10, n=5000, R=100).
  constexpr int GU = WIDE ? 2 : 4;
  gf32x4 acc[2][T][T];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
      for (int b = 0; b < T; ++b) acc[h][a][b] = gf32x4{0.f, 0.f, 0.f, 0.f};
  const bool vec = (ldx & 3) == 0 && (((uintptr_t)x) & 15) == 0;
  for (int c00 = c_beg + wave * 16; c00 < c_end; c00 += GU * nw * 16) {
    constexpr int NV = WIDE ? 2 : 1;   // operand row sets: A rows ro + .., B rows co + ..
    float v[NV][GU][T][4];
#pragma unroll
    for (int h = 0; h < NV; ++h)
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int c = c00 + u * nw * 16 + 4 * q;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int row = m + 16 * t + (h ? co : ro);
        const float* xr = x + (long long)row * ldx;
        if (row < K && vec && c + 3 < c_end) {
          const float4 f = *reinterpret_cast<const float4*>(xr + c);
          v[h][u][t][0] = f.x; v[h][u][t][1] = f.y; v[h][u][t][2] = f.z; v[h][u][t][3] = f.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            v[h][u][t][j] = (row < K && c + j < c_end) ? xr[c + j] : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < GU; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
          for (int b = 0; b < T; ++b)
            acc[j & 1][a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                v[0][u][a][j], v[NV - 1][u][b][j], acc[j & 1][a][b], 0, 0, 0);
  }
  // C/D map: row 4q + i, col m (register i)
#pragma unroll
  for (int a = 0; a < T; ++a)
#pragma unroll
    for (int b = 0; b < T; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        red[wave][((a * T + b) * 16 + 4 * q + i) * 16 + m] = acc[0][a][b][i] + acc[1][a][b][i];
  __syncthreads();
  float* o = part ? part + ((long long)blockIdx.y * gridDim.x + rep) * K * K
                  : out + (long long)rep * o_rs;
  const int bk = WIDE ? 64 : K;   // this workgroup's block edge
  for (int e = threadIdx.x; e < bk * bk; e += blockDim.x) {
    const int i = e / bk, j = e % bk;
    if (i + ro >= K || j + co >= K) continue;
    const int a = i >> 4, b = j >> 4;
    const int slot = ((a * T + b) * 16 + (i & 15)) * 16 + (j & 15);
    float s = 0.f;
    for (int w = 0; w < nw; ++w) s += red[w][slot];
    const long long oe = (long long)(i + ro) * K + j + co;
    o[oe] = (accumulate && !part) ? o[oe] + s : s;
  }
}

// Second stage of the column-split Gram: out[r] (+)= sum of the S partials in split
// order (deterministic).
__global__ void gram_reduce_kernel(const float* __restrict__ part, int S, int R, int K,
                                   float* __restrict__ out, long long o_rs, int accumulate,
                                   const int* active) {
  const int rep = blockIdx.x;
  if (active && active[rep] == 0) return;
  float* o = out + (long long)rep * o_rs;
  for (int e = threadIdx.x; e < K * K; e += blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += part[((long long)z * R + rep) * K * K + e];
    o[e] = accumulate ? o[e] + s : s;
  }
}

}  // namespace cnmf

extern "C" hipError_t cnmf_gram(const float* X, long long x_rs, long long ldx, int R, int K, int n,
                                float* out, long long o_rs, int accumulate, const int* active,
                                float* part, int S, hipStream_t stream) {
  if (R <= 0) return hipSuccess;
  if (K < 1 || K > 128 || n < 0 || S < 1) return hipErrorInvalidValue;
  if (S > 1 && !part) return hipErrorInvalidValue;
  // slice width: a multiple of 16 columns keeps the float4 slabs aligned
  const int per = S > 1 ? (((n + S - 1) / S + 15) / 16) * 16 : n;
  const int cols = S > 1 ? per : n;
  const int tmax = K > 32 ? 256 : 1024;
  int threads = cols >= 16 * 16 ? 1024 : 64 * ((cols + 15) / 16 > 0 ? ((cols + 15) / 16) : 1);
  if (threads > tmax) threads = tmax;
  const dim3 grid(R, S);
  float* pp = S > 1 ? part : nullptr;
  if (K <= 16)
    hipLaunchKernelGGL((cnmf::gram_kernel<1>), grid, dim3(threads), 0, stream, X, x_rs, ldx, K,
                       n, out, o_rs, accumulate, active, pp, per);
  else if (K <= 32)
    hipLaunchKernelGGL((cnmf::gram_kernel<2>), grid, dim3(threads), 0, stream, X, x_rs, ldx, K,
                       n, out, o_rs, accumulate, active, pp, per);
  else if (K <= 64)
    hipLaunchKernelGGL((cnmf::gram_kernel<4>), grid, dim3(threads), 0, stream, X, x_rs, ldx, K,
                       n, out, o_rs, accumulate, active, pp, per);
  else
    hipLaunchKernelGGL((cnmf::gram_kernel<4, true>), dim3(R, S, 4), dim3(threads), 0, stream, X,
                       x_rs, ldx, K, n, out, o_rs, accumulate, active, pp, per);
  if (S > 1)
    hipLaunchKernelGGL(cnmf::gram_reduce_kernel, dim3(R), dim3(256), 0, stream, part, S, R, K,
                       out, o_rs, accumulate, active);
  return hipGetLastError();
}
