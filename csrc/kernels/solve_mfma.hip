// Fused MU inner solve with the Gram apply on the matrix cores (K <= 16; SURVEY.md §2.4
// G3, the Frobenius H/W step of every online pass).  Same contract as solve_kernel in
// solve_core.h (x <- x * numer / (Gram x + l2 x + l1), rate 0 where the denominator is
// < eps; block-objective or iterate-change stop; cooperative slices; lin/quad epilogue;
// bf16 planes epilogue) -- only the data layout and the K x K product differ.
//
// Why: the VALU kernel re-reads the Gram from LDS for every column (a ds_read_b128 costs
// 4 LDS cycles per wave whatever the broadcast) and spends K*K fmaf per column on one
// lane; on the bench's H-side (100 replicates x 5000 cells, K = 10) that is ~4.2 us per
// sweep against ~0.5 us of arithmetic (tools/solve_probe.py).  Here a wave owns tiles of
// 16 columns and one v_mfma_f32_16x16x4_f32 per 4 components computes (Gram x) for the
// whole tile from registers: the Gram is the A operand, loaded ONCE per workgroup, and
// the iterate never leaves VGPRs.  fp32 MFMA is exact fp32 (a k-ordered fmaf chain).
//
// Layout trick.  16x16x4 f32: lane l = 16 g + c holds A[m = c][k = g], B[k = g][n = c]
// and D[m = 4 g + r][n = c] in its 4 accumulators r.  The iterate lives in the B layout:
// register s of lane (g, c) holds component 4 s + g of column c.  Feeding the Gram with
// its rows permuted, A'[m][k] = Gram[pi(m)][k], pi(4 g + r) = 4 r + g, makes accumulator
// r of lane (g, c) equal (Gram x)[4 r + g] of column c -- the component register r of the
// same lane holds.  So the elementwise update needs no data movement at all: the output
// layout IS the input layout, and only K/4 registers per tile carry x (and numer).
//
// Columns: a workgroup of 4 waves owns one slice of a replicate (slices: cooperative S or
// fixed nsplit, as solve_kernel); wave w takes tiles w, w + 4, ... (T per wave, T <=
// TMAX, chosen by the host).  The numerator of a lane's columns sits in LDS.  Padded components / columns hold x = numer = 0 and stay 0.
#include "solve_core.h"

namespace cnmf {

typedef float f32x4m __attribute__((ext_vector_type(4)));

constexpr int kMfmaWaves = 4;      // waves per workgroup (256 threads)

// Tiles of 16 columns per wave: x stays in VGPRs (K/4 per tile, <= 128 VGPRs in all so
// 4 workgroups share a CU), the numerator in LDS (lane-private words, no barrier; 37 KB
// per workgroup at most, 4 per CU)
__host__ __device__ constexpr int mfma_tile_max(int K) { return K <= 12 ? 12 : 9; }

// LDS numerator slot of (tile i, k-step s) for this thread: conflict-free b32 reads
#define CNMF_MFMA_N(i, s) sN[((i) * KS + (s)) * (64 * kMfmaWaves) + threadIdx.x]

// TRACK: the sweep accumulates |dx|^2, |x|^2 (iterate-change stop only; as a runtime
// flag the compiler computes them speculatively under a mask on every element)
// amdgpu_waves_per_eu(4): <= 128 VGPRs, so the host's co-residency budget of
// MFMA_WG_PER_CU = 4 workgroups per CU (ops/__init__.py) holds for every instantiation
template <int K, int TMAX, bool TRACK>
__global__ __launch_bounds__(64 * kMfmaWaves) __attribute__((amdgpu_waves_per_eu(4)))
void solve_mfma_kernel(SolveParams p, int T) {
  constexpr int KS = (K + 3) / 4;   // 4-component k-steps (registers per column tile)
  __shared__ float sred[3 + 2 * kCoopMaxSlices];
  __shared__ float sN[TMAX * KS * 64 * kMfmaWaves];
  static_assert(TMAX * KS * 64 * kMfmaWaves >= kMfmaWaves * 256, "Gram scratch in sN");
  const int rep = p.rep_index ? p.rep_index[blockIdx.x] : (int)blockIdx.x;
  if (p.active && p.active[rep] == 0) return;   // converged replicate: untouched (uniform)
  float* __restrict__ x = p.x + (long long)rep * p.x_rs;
  const float* __restrict__ nu = p.numer + (long long)rep * p.n_rs;
  const float* __restrict__ gm = p.gsrc ? nullptr : p.gram + (long long)rep * p.g_rs;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;

  // Gram fragments (A operand, rows permuted by pi): a[s] = Gram[pi(c)][4 s + g]
  float a[KS];
  const int pm = 4 * (c & 3) + (c >> 2);
  if (p.gsrc) {
    // Gram = F F^T formed here (gram.hip's trick): lane (g, c) feeds F[c][col] as both
    // A[m = c][k = g] and B[k = g][n = c], so D[i][j] = sum_col F[i][col] F[j][col] with
    // the 4 columns of one float4 on the k index; waves take 16-column slabs, two
    // accumulator chains; the 4 wave partials are summed in wave order through sN (not
    // yet holding numerators), so the result is deterministic
    const float* __restrict__ f = p.gsrc + (long long)rep * p.gs_rs;
    const int gcols = p.gs_cols;
    const long long fld = p.gs_ld;
    f32x4m g0 = {0.f, 0.f, 0.f, 0.f}, g1 = {0.f, 0.f, 0.f, 0.f};
    const bool rowok = c < K;
    const bool fvec = (fld & 3) == 0 && (reinterpret_cast<uintptr_t>(f) & 15) == 0;
#pragma unroll 4
    for (int c0 = 16 * wave; c0 < gcols; c0 += 16 * kMfmaWaves) {
      const int cc = c0 + 4 * g;
      float v[4];
      if (fvec && rowok && cc + 3 < gcols) {
        const float4 t = *reinterpret_cast<const float4*>(f + (long long)c * fld + cc);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] = (rowok && cc + e < gcols) ? f[(long long)c * fld + cc + e] : 0.f;
      }
      g0 = __builtin_amdgcn_mfma_f32_16x16x4f32(v[0], v[0], g0, 0, 0, 0);
      g1 = __builtin_amdgcn_mfma_f32_16x16x4f32(v[1], v[1], g1, 0, 0, 0);
      g0 = __builtin_amdgcn_mfma_f32_16x16x4f32(v[2], v[2], g0, 0, 0, 0);
      g1 = __builtin_amdgcn_mfma_f32_16x16x4f32(v[3], v[3], g1, 0, 0, 0);
    }
    // lane (g, c) holds D[4 g + r][c]
#pragma unroll
    for (int r = 0; r < 4; ++r) sN[wave * 256 + (4 * g + r) * 16 + c] = g0[r] + g1[r];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 4 * s + g;
      float v = 0.f;
      if (pm < K && k < K) {
#pragma unroll
        for (int w = 0; w < kMfmaWaves; ++w) v += sN[w * 256 + pm * 16 + k];
      }
      a[s] = v;
    }
    __syncthreads();   // sN is refilled with numerators below
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 4 * s + g;
      a[s] = (pm < K && k < K) ? gm[pm * K + k] : 0.f;
    }
  }

  int j0 = 0, n = p.ncols;
  const bool coop = p.coop_slots != nullptr && gridDim.y > 1;
  if (p.nsplit > 1 || coop) {
    const int parts = coop ? (int)gridDim.y : p.nsplit;
    const int per = (p.ncols + parts - 1) / parts;
    j0 = min(p.ncols, (int)blockIdx.y * per);
    n = min(p.ncols, j0 + per);
  }

  // x and the (l1_num-shifted) numerator of this lane's columns, B layout.  Buffer
  // accesses: 32-bit offsets computed at each use (col0 is re-derived through an opaque
  // copy, so the compiler cannot keep TMAX * KS addresses live across the solve).
  const __amdgpu_buffer_rsrc_t rx = rsrc_of(x);
  const __amdgpu_buffer_rsrc_t rn = rsrc_of(nu);
  const int sx = (int)p.ldx, sn = (int)p.ldn;
  float xr[TMAX][KS];
  {
    int col0 = j0 + 16 * wave + c;
    asm volatile("" : "+v"(col0));
#pragma unroll
    for (int i = 0; i < TMAX; ++i) {
      const int cl = col0 + 16 * kMfmaWaves * i;
      const bool ok = i < T && cl < n;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kk = 4 * s + g;
        const bool v = ok && kk < K;
        const float xv = buf_ld(rx, v ? (kk * sx + cl) * 4 : 0, 0);
        float nv = buf_ld(rn, v ? (kk * sn + cl) * 4 : 0, 0);
        nv = v ? nv : 0.f;
        if (p.l1_num > 0.f) nv = fmaxf(nv - p.l1_num, 0.f);
        xr[i][s] = v ? xv : 0.f;
        CNMF_MFMA_N(i, s) = nv;
      }
    }
  }

  const bool check_conv = p.nsplit <= 1;
  const bool loss_conv = check_conv && p.conv_mode == 1;
  const int every = p.check_every > 0 ? p.check_every : 1;
  const float l1 = p.l1_den, l2 = p.l2, eps = p.eps;
  int epoch = 0, it = 0;
  float f_prev = 0.f;
  bool have_prev = false;
  // lin = <numer, x>, quad = sum_j x_j^T Gram x_j of the CURRENT x from the last objective
  // pass (valid until the next sweep): the epilogue then needs no extra pass
  float lin_p = 0.f, quad_p = 0.f;
  bool lq_valid = false;

  while (true) {
    if (loss_conv && it % every == 0) {
      // objective x^T Gram x + l2 |x|^2 - 2 (numer - l1) . x, accumulated as four plain
      // sums (no per-element loop invariant such as numer - l1 for LICM to pin in VGPRs)
      float qd = 0.f, xx = 0.f, ln = 0.f, sx = 0.f;
#pragma unroll
      for (int i = 0; i < TMAX; ++i) {
        if (i < T) {
          f32x4m d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s)
            d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], xr[i][s], d, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < KS; ++r) {
            const float xv = xr[i][r];
            qd = fmaf(xv, d[r], qd);
            xx = fmaf(xv, xv, xx);
            ln = fmaf(xv, CNMF_MFMA_N(i, r), ln);
            sx += xv;
          }
        }
        __builtin_amdgcn_sched_barrier(0);   // one tile's accumulators live at a time
      }
      float q = fmaf(l2, xx, qd), l = fmaf(-l1, sx, ln);
      lin_p = ln;
      quad_p = qd;
      lq_valid = true;
      block_sum2(q, l, sred);
      float f = q - 2.f * l;
      if (coop) {
        float unused = 0.f;
        if (!coop_sum2(p, rep, epoch++, f, unused, sred)) break;
      }
      if (have_prev && fabsf(f_prev - f) <= p.tol * fabsf(f_prev)) break;
      f_prev = f;
      have_prev = true;
    }
    if (it >= p.max_iter) break;
    float d2 = 0.f, x2 = 0.f;
    // numerators come from LDS one tile AHEAD (read for tile i + 1 while tile i is
    // multiplied): the ~50-cycle LDS latency is never on a tile's critical path
    float nv[2][KS];   // ping-pong by tile parity (compile-time indices: no copies)
#pragma unroll
    for (int r = 0; r < KS; ++r) nv[0][r] = CNMF_MFMA_N(0, r);
#pragma unroll
    for (int i = 0; i < TMAX; ++i) {
      if (i < T) {
        if (i + 1 < TMAX) {
#pragma unroll
          for (int r = 0; r < KS; ++r) nv[(i + 1) & 1][r] = CNMF_MFMA_N(i + 1 < TMAX ? i + 1 : i, r);
        }
        f32x4m d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
          d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], xr[i][s], d, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < KS; ++r) {
          const float xv = xr[i][r];
          const float den = fmaf(l2, xv, d[r]) + l1;
          const float xn = (den < eps) ? 0.f : xv * (nv[i & 1][r] * __builtin_amdgcn_rcpf(den));
          if constexpr (TRACK) {
            const float dd = xn - xv;
            d2 = fmaf(dd, dd, d2);
            x2 = fmaf(xv, xv, x2);
          }
          xr[i][r] = xn;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    ++it;
    lq_valid = false;
    if (!TRACK || !check_conv || loss_conv) continue;
    block_sum2(d2, x2, sred);
    if (coop && !coop_sum2(p, rep, epoch++, d2, x2, sred)) break;
    if (sqrtf(d2) / (sqrtf(x2) + eps) < p.tol) break;
  }

  // store the final iterate
  {
    int col0 = j0 + 16 * wave + c;
    asm volatile("" : "+v"(col0));
#pragma unroll
    for (int i = 0; i < TMAX; ++i) {
      const int cl = col0 + 16 * kMfmaWaves * i;
      const bool ok = i < T && cl < n;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kk = 4 * s + g;
        if (ok && kk < K) buf_st(xr[i][s], rx, (kk * sx + cl) * 4, 0);
      }
    }
  }

  if (p.lin_out || p.quad_out) {
    float lin = lin_p, quad = quad_p;
    if (!lq_valid) {   // stopped by max_iter: one more product for the final x
      lin = 0.f;
      quad = 0.f;
#pragma unroll
      for (int i = 0; i < TMAX; ++i) {
        if (i < T) {
          f32x4m d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s)
            d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], xr[i][s], d, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < KS; ++r) {
            lin = fmaf(CNMF_MFMA_N(i, r), xr[i][r], lin);
            quad = fmaf(xr[i][r], d[r], quad);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (p.l1_num > 0.f) {   // lin is <raw numerator, x>: re-read the unshifted numerator
      lin = 0.f;
      int col0 = j0 + 16 * wave + c;
      asm volatile("" : "+v"(col0));
#pragma unroll
      for (int i = 0; i < TMAX; ++i) {
        const int cl = col0 + 16 * kMfmaWaves * i;
        const bool ok = i < T && cl < n;
#pragma unroll
        for (int r = 0; r < KS; ++r) {
          const int kk = 4 * r + g;
          const bool v = ok && kk < K;
          const float nv = buf_ld(rn, v ? (kk * sn + cl) * 4 : 0, 0);
          lin = fmaf(v ? nv : 0.f, xr[i][r], lin);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    block_sum2(lin, quad, sred);
    if (coop) (void)coop_sum2(p, rep, epoch++, lin, quad, sred);
    if (threadIdx.x == 0 && (!coop || blockIdx.y == 0)) {
      if (check_conv) {
        if (p.lin_out) p.lin_out[rep] = lin;
        if (p.quad_out) p.quad_out[rep] = quad;
      } else {  // split columns: caller zeroed the outputs
        if (p.lin_out) atomicAdd(p.lin_out + rep, lin);
        if (p.quad_out) atomicAdd(p.quad_out + rep, quad);
      }
    }
  }
  if (p.planes) {
    __syncthreads();   // every lane's final x stores precede the re-read (same block)
    emit_planes<K>(p, rep, j0, n, gridDim.y <= 1 || blockIdx.y == gridDim.y - 1);
  }
  if (p.iters_out && threadIdx.x == 0 && blockIdx.y == 0) p.iters_out[rep] += it;
}

template <int K>
static hipError_t launch_mfma_k(const SolveParams& p, int nblocks, int T, hipStream_t s) {
  const int gy = p.nsplit > 1 ? p.nsplit : (p.coop_slots ? p.coop_epochs_split : 1);
  if (p.nsplit <= 1 && p.conv_mode == 0)
    hipLaunchKernelGGL((solve_mfma_kernel<K, mfma_tile_max(K), true>), dim3(nblocks, gy),
                       dim3(64 * kMfmaWaves), 0, s, p, T);
  else
    hipLaunchKernelGGL((solve_mfma_kernel<K, mfma_tile_max(K), false>), dim3(nblocks, gy),
                       dim3(64 * kMfmaWaves), 0, s, p, T);
  return hipGetLastError();
}

hipError_t launch_solve_mfma(int K, const SolveParams& p, int nblocks, int T, hipStream_t s) {
  switch (K) {
    case 1: return launch_mfma_k<1>(p, nblocks, T, s);
    case 2: return launch_mfma_k<2>(p, nblocks, T, s);
    case 3: return launch_mfma_k<3>(p, nblocks, T, s);
    case 4: return launch_mfma_k<4>(p, nblocks, T, s);
    case 5: return launch_mfma_k<5>(p, nblocks, T, s);
    case 6: return launch_mfma_k<6>(p, nblocks, T, s);
    case 7: return launch_mfma_k<7>(p, nblocks, T, s);
    case 8: return launch_mfma_k<8>(p, nblocks, T, s);
    case 9: return launch_mfma_k<9>(p, nblocks, T, s);
    case 10: return launch_mfma_k<10>(p, nblocks, T, s);
    case 11: return launch_mfma_k<11>(p, nblocks, T, s);
    case 12: return launch_mfma_k<12>(p, nblocks, T, s);
    case 13: return launch_mfma_k<13>(p, nblocks, T, s);
    case 14: return launch_mfma_k<14>(p, nblocks, T, s);
    case 15: return launch_mfma_k<15>(p, nblocks, T, s);
    case 16: return launch_mfma_k<16>(p, nblocks, T, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace cnmf

// columns one workgroup of the MFMA solve can own (0: K not covered)
extern "C" int cnmf_solve_mfma_max_cols(int K) {
  return (K >= 1 && K <= 16) ? 16 * cnmf::kMfmaWaves * cnmf::mfma_tile_max(K) : 0;
}
