// Replicate-batched random initialisation of W / H.
//
// One launch fills the init of every replicate in a batch.  Replicate r is keyed by its
// ledger seed (cnmf.py:738-741 seeds -> nmf-torch random_state, cnmf.py:885), so the
// values depend only on (seed, stream, element index), never on batch position.
//   mode 0: |N(0,1)| * scale[r]      (random init, sklearn/_nmf.py:303-314 semantics)
//   mode 1: U(0,1)  * scale[r]       (fit_H_online's torch.rand init, cnmf.py:343, now seeded)
#include <hip/hip_runtime.h>
#include "philox.h"

namespace cnmf {

// Canonical element index e = row * cols + col of a (rows x cols) matrix; Philox call
// e/4 yields 4 uniforms -> two Box-Muller pairs.  The output layout is free
// (strides), so H can be written transposed (component-major) directly.
__global__ __launch_bounds__(256) void philox_fill_kernel(
    float* __restrict__ out, long long rows, long long cols, long long s_row, long long s_col,
    long long rep_stride, long long row_offset, const unsigned long long* __restrict__ seeds,
    const float* __restrict__ scales, unsigned int stream, int mode) {
  // Rows [row_offset, row_offset + rows) of the canonical (global_rows x cols) matrix:
  // a cell-sharded rank draws exactly the values of its rows in the unsharded init.
  const int r = blockIdx.y;
  const long long total = rows * cols;
  const long long e_begin = row_offset * cols;          // first canonical element
  const long long call = e_begin / 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long e0 = call * 4;
  if (e0 >= e_begin + total) return;
  const unsigned long long seed = seeds[r];
  const float scale = scales[r];
  u32x4 ctr;
  ctr.x = (uint32_t)(call & 0xffffffffull);
  ctr.y = (uint32_t)(call >> 32);
  ctr.z = stream;
  ctr.w = 0u;
  const u32x4 v = philox4x32_10(ctr, (uint32_t)(seed & 0xffffffffull), (uint32_t)(seed >> 32));
  float vals[4];
  if (mode == 0) {
    const double two_pi = 6.283185307179586;
    const double u0 = u32_to_open01(v.x), u1 = u32_to_open01(v.y);
    const double u2 = u32_to_open01(v.z), u3 = u32_to_open01(v.w);
    const double ra = sqrt(-2.0 * log(u0)), rb = sqrt(-2.0 * log(u2));
    vals[0] = (float)fabs(ra * cos(two_pi * u1));
    vals[1] = (float)fabs(ra * sin(two_pi * u1));
    vals[2] = (float)fabs(rb * cos(two_pi * u3));
    vals[3] = (float)fabs(rb * sin(two_pi * u3));
  } else {
    vals[0] = (float)u32_to_open01(v.x);
    vals[1] = (float)u32_to_open01(v.y);
    vals[2] = (float)u32_to_open01(v.z);
    vals[3] = (float)u32_to_open01(v.w);
  }
  float* base = out + (long long)r * rep_stride;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long long e = e0 + q - e_begin;
    if (e >= 0 && e < total) {
      const long long row = e / cols, col = e - row * cols;
      base[row * s_row + col * s_col] = vals[q] * scale;
    }
  }
}

}  // namespace cnmf

extern "C" hipError_t cnmf_philox_fill(float* out, long long rows, long long cols, long long s_row,
                                       long long s_col, long long rep_stride, long long row_offset,
                                       const unsigned long long* seeds, const float* scales, int R,
                                       unsigned int stream_id, int mode, hipStream_t stream) {
  const long long e_begin = row_offset * cols;
  const long long calls = (e_begin + rows * cols + 3) / 4 - e_begin / 4;
  if (calls == 0 || R == 0) return hipSuccess;
  dim3 grid((unsigned)((calls + 255) / 256), (unsigned)R);
  hipLaunchKernelGGL(cnmf::philox_fill_kernel, grid, dim3(256), 0, stream, out, rows, cols, s_row,
                     s_col, rep_stride, row_offset, seeds, scales, stream_id, mode);
  return hipGetLastError();
}
