// Fused MU inner solve for the wide ranks K in (64, 128] on the matrix cores (SURVEY.md
// §2.4 G3; the reference's -k is unbounded, cnmf.py:1416-1417, and nmf-torch's MU step is
// the same x <- x * numer / (Gram x + l2 x + l1) at any K, cnmf.py:365-378).  Same
// contract as solve_kernel (solve_core.h): rate 0 where the denominator is < eps,
// block-objective or iterate-change stop, fixed-step column split (nsplit), cooperative
// slices, lin/quad and bf16-planes epilogues.  The NMF engine pads such K to a multiple of
// 16 with zero components (models/nmf.py native_rank): a zero row stays zero under MU.
//
// Why a separate kernel: the VALU streaming kernel keeps a column's K values, numerator
// and result live per lane (~3K VGPRs) -- past K = 64 that no longer fits a wave.  Here a
// wave owns 16 columns at a time in the v_mfma_f32_16x16x4_f32 B layout (register s of
// lane (g, c) = component 4s + g of column c, K/4 registers per tile), and (Gram x) of the
// tile is K/16 output tiles of K/4 MFMAs each, the Gram streaming from LDS as A fragments.
// With the Gram rows permuted inside each 16-row output tile, pi(4g + r) = 4r + g (the
// solve_mfma.hip trick), accumulator r of output tile t lands on register 4t + r of the
// SAME lane: the elementwise update needs no lane movement.  The k-step loop runs outside
// the output-tile loop, so the K/16 accumulator chains are independent (no MFMA waits on
// its predecessor's result) and each A fragment is one conflict-free ds_read_b128 per 4
// k-steps.  fp32 MFMA is exact fp32 (a k-ordered fmaf chain).
//
// x and the numerator are re-read from L2 every sweep (the streaming discipline of
// solve_kernel): no cap on the columns a workgroup owns, so the cooperative and the
// fixed-split slicing of the other solves apply unchanged.  LDS: the K x K Gram (64 KB at
// K = 128), two workgroups per CU.
#include "solve_core.h"

namespace cnmf {

typedef float wf32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) wf32x4 lds_wf32x4;

constexpr int kWideWaves = 4;

// (Gram x) of one 16-column tile: acc[t][r] = (Gram x)[16t + 4r + g] of column c
template <int K>
__device__ __forceinline__ void wm_apply(const lds_wf32x4* __restrict__ sA, int lane,
                                         const float (&xr)[K / 4], wf32x4 (&acc)[K / 16]) {
  constexpr int KS = K / 4, KT = K / 16;
#pragma unroll
  for (int t = 0; t < KT; ++t) acc[t] = wf32x4{0.f, 0.f, 0.f, 0.f};
  // A fragments one k-step group ahead (two register sets): left alone, the scheduler
  // hoists every LDS read of the unrolled product to the top (K*K/64 VGPRs of operands)
  wf32x4 a[2][KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) a[0][t] = sA[(t * (KS / 4)) * 64 + lane];
#pragma unroll
  for (int s4 = 0; s4 < KS / 4; ++s4) {
    if (s4 + 1 < KS / 4) {
#pragma unroll
      for (int t = 0; t < KT; ++t) a[(s4 + 1) & 1][t] = sA[(t * (KS / 4) + s4 + 1) * 64 + lane];
    }
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s4 & 1][t][e], xr[4 * s4 + e], acc[t],
                                                      0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Split-bf16 variant (BF): the Gram apply on v_mfma_f32_16x16x32_bf16, fp32-accurate
// through split operands -- G = G_hi + G_lo and x = x_hi + x_lo (bf16 planes, each
// residual exact), Gx = G_hi x_hi + G_hi x_lo + G_lo x_hi (dropped term <= 2^-16
// relative, as the split GEMMs of gemm_planes.hip).  K is padded to KP, a multiple of
// 32, inside the kernel (components >= K are zero).  B layout: register s of lane
// (g, c) holds component 32 (s / 8) + 8 g + s % 8 of column c (8 per 32-deep k-block);
// output tile t = 2 kb + h with the Gram rows permuted so accumulator r of lane (g, c)
// is component 32 kb + 8 g + 4 h + r -- register 4 t + r of the same lane, as in the
// fp32 variant.  Per 16-column tile: KP/16 x KP/32 x 3 MFMAs of 16 cycles instead of
// KP/16 x KP/4 of 32 (5.3x fewer MFMA cycles at K = 128).
typedef short wbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 wbh8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) wbf16x8 lds_wbf16x8;

__device__ __forceinline__ unsigned short wb_bits(__bf16 h) {
  return __builtin_bit_cast(unsigned short, h);
}

template <int KP>
__device__ __forceinline__ void wb_apply(const lds_wbf16x8* __restrict__ sA, int lane,
                                         const float (&xr)[KP / 4], wf32x4 (&acc)[KP / 16]) {
  constexpr int KB = KP / 32, KT = KP / 16;
  wbf16x8 bh[KB], bl[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    wbh8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = xr[8 * kb + e];
      h[e] = (__bf16)v;
      l[e] = (__bf16)(v - (float)h[e]);
    }
    bh[kb] = __builtin_bit_cast(wbf16x8, h);
    bl[kb] = __builtin_bit_cast(wbf16x8, l);
  }
#pragma unroll
  for (int t = 0; t < KT; ++t) acc[t] = wf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const wbf16x8 ah = sA[((t * KB + kb) * 2 + 0) * 64 + lane];
      const wbf16x8 al = sA[((t * KB + kb) * 2 + 1) * 64 + lane];
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[kb], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[kb], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[kb], acc[t], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int K, bool TRACK, bool BF>
__global__ __launch_bounds__(64 * kWideWaves) void solve_wmfma_kernel(SolveParams p) {
  static_assert(K % 16 == 0 && K <= 128, "wide solve: K a multiple of 16, <= 128");
  constexpr int KP = BF ? (K + 31) / 32 * 32 : K;   // internal rank (bf16: whole k-blocks)
  constexpr int KS = KP / 4, KT = KP / 16;
  // fp32: K x K floats; bf16: KP x KP elements as two bf16 planes (the same bytes per
  // element)
  __shared__ __attribute__((aligned(16))) float sAm[KP * KP];
  __shared__ float sred[3 + 2 * kCoopMaxSlices];
  const int rep = p.rep_index ? p.rep_index[blockIdx.x] : (int)blockIdx.x;
  if (p.active && p.active[rep] == 0) return;   // converged replicate: untouched (uniform)
  float* __restrict__ x = p.x + (long long)rep * p.x_rs;
  const float* __restrict__ nu = p.numer + (long long)rep * p.n_rs;
  const float* __restrict__ gm = p.gram + (long long)rep * p.g_rs;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;

  if constexpr (BF) {
    // [t][kb][plane][lane][8]: lane (g', c') of output tile t = 2 kb_o + h, k-block kb
    // holds Gram[32 kb_o + 8 (c' >> 2) + 4 h + (c' & 3)][32 kb + 8 g' + e], split hi / lo
    unsigned short* sAh = reinterpret_cast<unsigned short*>(sAm);
    constexpr int KB = KP / 32;
    for (int i = threadIdx.x; i < KP * KP; i += blockDim.x) {
      const int e = i & 7, ln = (i >> 3) & 63, rest = i >> 9;   // rest = t * KB + kb
      const int t = rest / KB, kb = rest - t * KB;
      const int cc = ln & 15, gg = ln >> 4;
      const int row = 32 * (t >> 1) + 8 * (cc >> 2) + 4 * (t & 1) + (cc & 3);
      const int col = 32 * kb + 8 * gg + e;
      const float v = (row < K && col < K) ? gm[row * K + col] : 0.f;
      const __bf16 h = (__bf16)v;
      const int o = ((rest * 2) * 64 + ln) * 8 + e;
      sAh[o] = wb_bits(h);
      sAh[o + 64 * 8] = wb_bits((__bf16)(v - (float)h));
    }
  } else {
    // Gram -> LDS as permuted A fragments, stored [t][s4][lane][4] (s = 4 s4 + e: one
    // b128 per 4 k-steps): (t, s, lane (g', c')) = Gram[16t + pi(c')][4s + g']
    for (int i = threadIdx.x; i < K * K; i += blockDim.x) {
      const int e = i & 3, ln = (i >> 2) & 63, rest = i >> 8;   // rest = t * KS/4 + s4
      const int t = rest / (KS / 4), s = 4 * (rest - t * (KS / 4)) + e;
      const int cc = ln & 15, gg = ln >> 4;
      sAm[i] = gm[(16 * t + 4 * (cc & 3) + (cc >> 2)) * K + 4 * s + gg];
    }
  }
  __syncthreads();
  const lds_wf32x4* sA = (const lds_wf32x4*)sAm;
  const lds_wbf16x8* sAb = (const lds_wbf16x8*)sAm;
  // component of register s of this lane, and its row offset beyond the lane's base
  auto comp = [&](int s_) { return BF ? 32 * (s_ >> 3) + 8 * g + (s_ & 7) : 4 * s_ + g; };
  auto soff_rows = [&](int s_) { return BF ? 32 * (s_ >> 3) + (s_ & 7) : 4 * s_; };
  const int g_rows = BF ? 8 * g : g;
  auto apply = [&](const float (&xr_)[KS], wf32x4 (&acc_)[KT]) {
    if constexpr (BF) wb_apply<KP>(sAb, lane, xr_, acc_);
    else wm_apply<K>(sA, lane, xr_, acc_);
  };

  int j0 = 0, n = p.ncols;
  const bool coop = p.coop_slots != nullptr && gridDim.y > 1;
  if (p.nsplit > 1 || coop) {
    const int parts = coop ? (int)gridDim.y : p.nsplit;
    const int per = (p.ncols + parts - 1) / parts;
    j0 = min(p.ncols, (int)blockIdx.y * per);
    n = min(p.ncols, j0 + per);
  }
  const int ntile = (n - j0 + 15) / 16;
  const __amdgpu_buffer_rsrc_t rx = rsrc_of(x);
  const __amdgpu_buffer_rsrc_t rn = rsrc_of(nu);
  const int sx = (int)p.ldx, sn = (int)p.ldn;
  const bool check_conv = p.nsplit <= 1;
  const bool loss_conv = check_conv && p.conv_mode == 1;
  const int every = p.check_every > 0 ? p.check_every : 1;
  const float l1 = p.l1_den, l2 = p.l2, eps = p.eps;

  // x / numerator of tile i for this lane (B layout), numerator l1_num-shifted if `shift`
  // (per-lane VGPR offset of component g, k-step s as the uniform soffset 16 s ld)
  auto load_tile = [&](int i, float (&xr)[KS], float (&nr)[KS], bool shift) {
    const int cl = j0 + 16 * i + c;
    const bool ok = cl < n;
    const int vx = ok ? (g_rows * sx + cl) * 4 : 0, vn = ok ? (g_rows * sn + cl) * 4 : 0;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const bool v = ok && (!BF || comp(s) < K);
      const float xv = buf_ld(rx, v ? vx : 0, v ? 4 * soff_rows(s) * sx : 0);
      float nv = buf_ld(rn, v ? vn : 0, v ? 4 * soff_rows(s) * sn : 0);
      nv = v ? nv : 0.f;
      if (shift && p.l1_num > 0.f) nv = fmaxf(nv - p.l1_num, 0.f);
      xr[s] = v ? xv : 0.f;
      nr[s] = nv;
    }
  };
  // objective pieces of the current x: sum x^T Gram x, |x|^2, <numer, x>, sum x
  auto objective = [&](bool shift, float& qd, float& xx, float& ln, float& sxs) {
    qd = xx = ln = sxs = 0.f;
    for (int i = wave; i < ntile; i += kWideWaves) {
      float xr[KS], nr[KS];
      load_tile(i, xr, nr, shift);
      wf32x4 acc[KT];
      apply(xr, acc);
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xv = xr[4 * t + r];
          qd = fmaf(xv, acc[t][r], qd);
          xx = fmaf(xv, xv, xx);
          ln = fmaf(xv, nr[4 * t + r], ln);
          sxs += xv;
        }
    }
  };

  int epoch = 0, it = 0;
  float f_prev = 0.f;
  bool have_prev = false;
  while (true) {
    if (loss_conv && it % every == 0) {
      float qd, xx, ln, sxs;
      objective(true, qd, xx, ln, sxs);
      float q = fmaf(l2, xx, qd), l = fmaf(-l1, sxs, ln);
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
    for (int i = wave; i < ntile; i += kWideWaves) {
      CNMF_MEMBAR();
      float xr[KS], nr[KS];
      load_tile(i, xr, nr, true);
      wf32x4 acc[KT];
      apply(xr, acc);
      const int cl = j0 + 16 * i + c;
      const bool ok = cl < n;
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = 4 * t + r;
          const float xv = xr[s];
          const float den = fmaf(l2, xv, acc[t][r]) + l1;
          const float xn = (den < eps) ? 0.f : xv * (nr[s] * __builtin_amdgcn_rcpf(den));
          if constexpr (TRACK) {
            const float dd = xn - xv;
            d2 = fmaf(dd, dd, d2);
            x2 = fmaf(xv, xv, x2);
          }
          if (ok && (!BF || comp(s) < K)) buf_st(xn, rx, (g_rows * sx + cl) * 4, 4 * soff_rows(s) * sx);
        }
    }
    ++it;
    if (!TRACK || !check_conv || loss_conv) continue;
    block_sum2(d2, x2, sred);
    if (coop && !coop_sum2(p, rep, epoch++, d2, x2, sred)) break;
    if (sqrtf(d2) / (sqrtf(x2) + eps) < p.tol) break;
  }

  if (p.lin_out || p.quad_out) {
    __syncthreads();   // the lanes' final x stores precede the re-read (same block)
    float qd, xx, ln, sxs;
    objective(false, qd, xx, ln, sxs);   // lin = <raw numerator, x>, quad = x^T Gram x
    float lin = ln, quad = qd;
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
    __syncthreads();
    emit_planes<K>(p, rep, j0, n, gridDim.y <= 1 || blockIdx.y == gridDim.y - 1);
  }
  if (p.iters_out && threadIdx.x == 0 && blockIdx.y == 0) p.iters_out[rep] += it;
}

template <int K, bool BF>
static hipError_t launch_wmfma_kb(const SolveParams& p, int nblocks, hipStream_t s) {
  const int gy = p.nsplit > 1 ? p.nsplit : (p.coop_slots ? p.coop_epochs_split : 1);
  if (p.nsplit <= 1 && p.conv_mode == 0)
    hipLaunchKernelGGL((solve_wmfma_kernel<K, true, BF>), dim3(nblocks, gy),
                       dim3(64 * kWideWaves), 0, s, p);
  else
    hipLaunchKernelGGL((solve_wmfma_kernel<K, false, BF>), dim3(nblocks, gy),
                       dim3(64 * kWideWaves), 0, s, p);
  return hipGetLastError();
}

// bf16: the split-bf16 Gram apply (default); else the fp32-MFMA one (ops.solve
// variant="stream")
template <int K>
static hipError_t launch_wmfma_k(const SolveParams& p, int nblocks, bool bf16, hipStream_t s) {
  return bf16 ? launch_wmfma_kb<K, true>(p, nblocks, s) : launch_wmfma_kb<K, false>(p, nblocks, s);
}

hipError_t launch_solve_wmfma(int K, const SolveParams& p, int nblocks, bool bf16, hipStream_t s) {
  switch (K) {
    case 80: return launch_wmfma_k<80>(p, nblocks, bf16, s);
    case 96: return launch_wmfma_k<96>(p, nblocks, bf16, s);
    case 112: return launch_wmfma_k<112>(p, nblocks, bf16, s);
    case 128: return launch_wmfma_k<128>(p, nblocks, bf16, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace cnmf
