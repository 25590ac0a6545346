// Shared device helpers for the cnmf_torch_amd HIP kernels (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cnmf {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Block-wide sum of two values; every thread receives both totals.
// `scratch` needs 2 * (blockDim.x / 64) floats of LDS.  Contains two barriers.
__device__ __forceinline__ void block_sum2(float& a, float& b, float* scratch) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = (blockDim.x + kWave - 1) / kWave;
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) { scratch[wid] = a; scratch[nw + wid] = b; }
  __syncthreads();
  float ta = 0.f, tb = 0.f;
  for (int w = 0; w < nw; ++w) { ta += scratch[w]; tb += scratch[nw + w]; }
  __syncthreads();
  a = ta;
  b = tb;
}

__device__ __forceinline__ float block_sum1(float a, float* scratch) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = (blockDim.x + kWave - 1) / kWave;
  a = wave_sum(a);
  if (lane == 0) scratch[wid] = a;
  __syncthreads();
  float t = 0.f;
  for (int w = 0; w < nw; ++w) t += scratch[w];
  __syncthreads();
  return t;
}

}  // namespace cnmf
