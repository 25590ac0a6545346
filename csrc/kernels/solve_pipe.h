// Software-pipelined matrix-core MU solve, K <= 64: the hot path of every Frobenius online
// pass (SURVEY.md §2.4 G3 -- the H/W inner loops of cnmf.py:365-378 and nmf-torch's online
// MU), for the common unregularised case (l1 = l2 = 0) with the block-objective stop
// (conv_mode 1, nmf-torch online_inner_conv='loss').  Same contract, data layout and
// cooperative slicing as solve_mfma_kernel (solve_mfma.hip), which keeps the regularised,
// iterate-change, fixed-split and in-prologue-Gram cases for K <= 16.  Instantiated per K
// by solve_pipe*.hip (one unit per K band, so they compile in parallel).
//
// Why pipelined.  solve_mfma_kernel walks its column tiles strictly one after the other
// (a sched_barrier per tile, a runtime tile count T with a branch per tile): each tile is a
// chain of K/4 DEPENDENT v_mfma_f32_16x16x4_f32 (40-cycle dependent latency each,
// MI355X_MICROARCH.md cycle table), an s_nop until the accumulator is readable, then ~20
// VALU of which the compiler SLP-packs half into v_pk_*_f32 (an anti-lever beside MFMAs,
// same table).  Nothing overlaps the chain inside a wave, so on the bench's H side a sweep
// took ~3.9 us against ~1.3 us of MFMA issue (docs/ARCHITECTURE.md "Solve sweeps").
//
// Here T is a template parameter (the host rounds the tile count up to an instantiated
// one; padded tiles hold zero columns, which MU keeps at zero), and the sweep is software
// pipelined: the MFMA chains of tile i+1 are issued before the elementwise update of tile
// i, whose accumulators were produced one step earlier.  The chains of consecutive tiles
// are independent, so the matrix core always has the next tile's work while the VALU
// finishes the previous one, within ONE wave.  Without l1/l2 the update is
//     den = (Gram x)_k ;  x_k <- den < eps ? 0 : x_k * (numer_k * rcp(den))
// five VALU per element (cmp, cndmask, rcp, 2 mul), all scalar f32 (-fno-slp-vectorize for
// these units), which fits the issue slots a 16x16x4 f32 MFMA leaves (32 cycles, 8 held).
//
// Layout (16x16x4 f32: lane l = 16 g + c holds A[m = c][k = g], B[k = g][n = c] and
// D[m = 4 g + r][n = c] in accumulator r).  The iterate lives in the B layout: register s
// of lane (g, c) holds component 4 s + g of column c (KS = K/4 registers per 16-column
// tile).  (Gram x) of a tile is MB = K/16 output blocks of 16 Gram rows; block b's A
// fragments are the Gram rows permuted, A_b[m][k] = Gram[16 b + pi(m)][k] with
// pi(4 g + r) = 4 r + g, so accumulator r of block b on lane (g, c) is component
// 16 b + 4 r + g of column c -- exactly the component register s = 4 b + r of the same lane
// holds.  The elementwise update needs no data movement at any K: the output layout IS the
// input layout.  The MB chains of a tile are independent (k-step outer, block inner), so
// from K = 17 on the matrix core has MB chains in flight even inside one tile.  fp32 MFMA
// is exact fp32 (a k-ordered fmaf chain), so the solve is the fp32 MU step.
//
// Occupancy.  x lives in VGPRs (T * KS), the numerators in LDS (T * KS KB per workgroup),
// the Gram fragments in VGPRs (MB * KS: 16 at K = 32, 64 at K = 64).  K <= 32: <= 128
// VGPRs, <= 36 KB of numerators, four 256-thread workgroups per CU; K in (32, 64]: <= 256
// VGPRs, <= 78 KB, two per CU (pipe_weu).  A replicate set whose slices do not all fit at
// once is launched in co-resident rounds by the host (cnmf_solve: reps_per_launch).
//
// The planes epilogue emits the final x straight from registers (no re-read from L2) and
// only the `pl_n` planes the consuming GEMM reads (2 with a >= 1024-deep reduction,
// ops.gemm_a_planes), instead of three.
#pragma once
#include "solve_core.h"

namespace cnmf {

typedef float f32x4p __attribute__((ext_vector_type(4)));

constexpr int kPipeWaves = 4;   // waves per workgroup (256 threads)

__host__ __device__ constexpr int pipe_ks(int K) { return (K + 3) / 4; }
__host__ __device__ constexpr int pipe_mb(int K) { return (K + 15) / 16; }
// waves per SIMD the instantiation is built for: 4 (<= 128 VGPRs) up to K = 32, 2 (<= 256)
// for the wide ranks, whose Gram fragments alone are up to 64 VGPRs
__host__ __device__ constexpr int pipe_weu(int K) { return K <= 32 ? 4 : 2; }
// 256-thread workgroups co-resident per CU (one wave per SIMD each): VGPR- and LDS-bound
__host__ __device__ constexpr int pipe_wg_per_cu(int K) { return pipe_weu(K); }
// tiles per wave: the numerators' LDS (T * KS KB) within 160 KB / pipe_wg_per_cu(K) minus
// scratch -- K <= 12: 12 tiles (36 KB), 13..16: 9 (36 KB), 17..32: 36 / KS (<= 36 KB),
// 40..64: 78 / KS (<= 78 KB)
__host__ __device__ constexpr int pipe_tile_max(int K) {
  return K <= 12 ? 12 : K <= 16 ? 9 : K <= 32 ? 36 / pipe_ks(K) : 78 / pipe_ks(K);
}
// LDS floats of the numerator / epilogue-scratch array: T * KS 256-float slots, and at
// least the partial-Gram epilogue's 4 waves x 16 x (16 MB + 1)
__host__ __device__ constexpr int pipe_lds_floats(int K, int T) {
  return (T * pipe_ks(K) * 64 * kPipeWaves > 64 * (16 * pipe_mb(K) + 1))
             ? T * pipe_ks(K) * 64 * kPipeWaves
             : 64 * (16 * pipe_mb(K) + 1);
}

#define CNMF_PIPE_N(i, s) sN[((i) * KS + (s)) * (64 * kPipeWaves) + threadIdx.x]

// (Gram x) of one tile: d[b][r] = component 16 b + 4 r + g of the lane's column
template <int KS, int MB>
__device__ __forceinline__ void pipe_chain(const float (&a)[MB][KS], const float (&x)[KS],
                                           f32x4p (&d)[MB]) {
#pragma unroll
  for (int b = 0; b < MB; ++b) d[b] = f32x4p{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int b = 0; b < MB; ++b) d[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[b][s], x[s], d[b], 0, 0, 0);
}

// Launch-completion bookkeeping of the device-side generation (SolveParams.coop_gen_dev):
// every workgroup arrives once; the last one resets the counter and advances the tag
// (kernels on one stream never overlap, so the next launch reads the new value).
__device__ __forceinline__ void pipe_arrive(const SolveParams& p) {
  if (!p.coop_gen_dev) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned total = gridDim.x * gridDim.y;
    const unsigned old = atomicAdd(p.coop_arrive, 1u);
    if (old + 1 == total) {
      atomicExch(p.coop_arrive, 0u);
      const unsigned g = __hip_atomic_load(p.coop_gen_dev, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.coop_gen_dev, g >= 0xFFFFFFFEu ? 0x80000000u : g + 1u,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ unsigned short pipe_bf16_rn(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

template <int K, int T>
__global__ __launch_bounds__(64 * kPipeWaves) __attribute__((amdgpu_waves_per_eu(pipe_weu(K))))
void solve_pipe_kernel(SolveParams p, int pl_n) {
  constexpr int KS = pipe_ks(K);
  constexpr int MB = pipe_mb(K);
  constexpr int KP = 16 * MB;          // Gram rows covered by the output blocks
  __shared__ float sred[3 + 2 * kCoopMaxSlices];
  // numerators of this lane's columns; also the partial-Gram scratch of the epilogue
  __shared__ float sN[pipe_lds_floats(K, T)];
  // phase stamps are compiled in only for the probe build (CNMF_PIPE_STAMPS_BUILD=1 at
  // build time, tools/pipe_stamp_probe.py): their 64-bit counters cost the production
  // kernels registers (K = 10 / 20 instantiations went to scratch with them)
#ifdef CNMF_PIPE_STAMPS
  const bool stp = p.stamps != nullptr;
#else
  constexpr bool stp = false;
#endif
  unsigned long long st0 = 0, st1 = 0, st_chk = 0, n_chk = 0, rt0 = 0, rt_x = 0;
  if (stp) {
    rt0 = __builtin_amdgcn_s_memrealtime();
    st0 = __builtin_amdgcn_s_memtime();
  }
  // (replicate block, slice) of this workgroup -- see SolveParams.pipe_map
  int blk, slc, nsg;
  if (p.pipe_map) {
    nsg = p.coop_slots ? p.coop_epochs_split : 1;
    const int w = (int)blockIdx.x, l = w >> 3;
    blk = (l / nsg) * 8 + (w & 7);
    slc = l - (l / nsg) * nsg;
    if (blk >= p.pipe_nblocks) {         // padding of the last group of 8 replicates
      pipe_arrive(p);
      return;
    }
  } else {
    blk = (int)blockIdx.x;
    slc = (int)blockIdx.y;
    nsg = (int)gridDim.y;
  }
  const int bx = p.rep0 + blk;
  const int rep = p.rep_index ? p.rep_index[bx] : bx;
  if (p.active && p.active[rep] == 0) {   // converged replicate: untouched (uniform)
    pipe_arrive(p);
    return;
  }
  // cooperative tag: the host's generation, or the device-side one (graph replays)
  const unsigned gen = p.coop_gen_dev ? __hip_atomic_load(p.coop_gen_dev, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : p.coop_gen;
  float* __restrict__ x = p.x + (long long)rep * p.x_rs;
  const float* __restrict__ nu = p.numer + (long long)rep * p.n_rs;
  const float* __restrict__ gm = p.gram ? p.gram + (long long)rep * p.g_rs : nullptr;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;

  // Gram fragments, rows permuted by pi(4g + r) = 4r + g inside each 16-row block b: the
  // accumulator register r of block b on lane (g, c) is then component 16b + 4r + g of
  // column c, the component this lane's B register 4b + r holds
  float a[MB][KS];
  const int pm = 4 * (c & 3) + (c >> 2);
#pragma unroll
  for (int b = 0; b < MB; ++b)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int row = 16 * b + pm, k = 4 * s + g;
      a[b][s] = (gm && row < K && k < K) ? gm[row * K + k] : 0.f;
    }
  if (p.gpart) {
    // + the producing solve's per-slice partial Grams, summed in slice order.  They are
    // staged through LDS (sN, free until the numerators arrive) in chunks of whole
    // partials: 256 threads load consecutive floats, 16 in flight each -- coalesced and
    // one or two memory rounds per chunk, where per-lane (row, k) gathers took one round
    // per QB partials and block (tools/pipe_stamp_probe.py: the spectra side's prologue
    // was half its launch).  Each lane then sums its elements over the chunk's partials
    // in slice order: bitwise the register version's sums.
    const float* gp = p.gpart + (long long)rep * p.gpart_rs;
    constexpr int KK = K * K;
    constexpr int QCH = pipe_lds_floats(K, T) / KK > 0 ? pipe_lds_floats(K, T) / KK : 1;
    constexpr int NTH = 64 * kPipeWaves;
    float t[MB][KS];
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int s = 0; s < KS; ++s) t[b][s] = 0.f;
    for (int q0 = 0; q0 < p.gpart_n; q0 += QCH) {
      const int qn = p.gpart_n - q0 < QCH ? p.gpart_n - q0 : QCH;
      const int tot = qn * KK;
      const float* src = gp + (long long)q0 * KK;
      for (int e0 = (int)threadIdx.x; e0 < tot; e0 += 16 * NTH) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = e0 + j * NTH < tot ? src[e0 + j * NTH] : 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (e0 + j * NTH < tot) sN[e0 + j * NTH] = v[j];
      }
      __syncthreads();
      for (int q = 0; q < qn; ++q) {
#pragma unroll
        for (int b = 0; b < MB; ++b)
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const int row = 16 * b + pm, k = 4 * s + g;
            t[b][s] += (row < K && k < K) ? sN[q * KK + row * K + k] : 0.f;   // exact + 0
          }
      }
      __syncthreads();                 // the chunk is consumed before the next overwrites
    }
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int s = 0; s < KS; ++s) a[b][s] = gm ? a[b][s] + t[b][s] : t[b][s];
  }

  int j0 = 0, n = p.ncols;
  const bool coop = p.coop_slots != nullptr && nsg > 1;
  if (coop) {
    const int per = (p.ncols + nsg - 1) / nsg;
    j0 = min(p.ncols, slc * per);
    n = min(p.ncols, j0 + per);
  }

  const __amdgpu_buffer_rsrc_t rx = rsrc_of(x);
  const __amdgpu_buffer_rsrc_t rn = rsrc_of(nu);
  const int sx = (int)p.ldx, sn = (int)p.ldn;
  float xr[T][KS];
  {
    int col0 = j0 + 16 * wave + c;
    asm volatile("" : "+v"(col0));
    const int nsl = p.nslab_n > 1 ? p.nslab_n : 1;
    const unsigned sstride = (unsigned)(p.nslab_stride * 4);   // host: < 2^31 bytes
    float* __restrict__ nb_out = p.nout ? p.nout + (long long)rep * p.nb_rs : nullptr;
    const float* __restrict__ nb_in = p.nbase ? p.nbase + (long long)rep * p.nb_rs : nullptr;
    const int sb = (int)p.ldnb;
#pragma unroll
    for (int i = 0; i < T; ++i) {
      const int cl = col0 + 16 * kPipeWaves * i;
      const bool ok = cl < n;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kk = 4 * s + g;
        const bool v = ok && kk < K;
        const float xv = buf_ld(rx, v ? (kk * sx + cl) * 4 : 0, 0);
        const float nv = buf_ld(rn, v ? (kk * sn + cl) * 4 : 0, 0);
        xr[i][s] = v ? xv : 0.f;
        CNMF_PIPE_N(i, s) = v ? nv : 0.f;
      }
    }
    if (nsl > 1 || p.n_scale || nb_in || nb_out) {
      // raw split-K slabs summed in slice order, then scaled and added to the base:
      // bitwise gemm_reduce_kernel's "C (+)= col_scale * sum_s slab[s]".
      if constexpr (3 * T * KS <= 48) {
        // few tiles (the spectra side): the loads of slabs 1..3 (clamped to the last
        // one, masked to + 0 past nsl -- exact) and of the base all go out together, one
        // memory round trip instead of one per slab (tools/pipe_stamp_probe.py: the
        // per-slab rounds were half of this side's launch)
        float sl[3][T][KS];
        float bs[T][KS];
#pragma unroll
        for (int q = 1; q < 4; ++q) {
          const unsigned so = (unsigned)(q < nsl ? q : nsl - 1) * sstride;
#pragma unroll
          for (int i = 0; i < T; ++i) {
            const int cl = col0 + 16 * kPipeWaves * i;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
              const int kk = 4 * s + g;
              const bool v = cl < n && kk < K;
              const float t = buf_ld(rn, v ? (kk * sn + cl) * 4 : 0, so);
              sl[q - 1][i][s] = v ? t : 0.f;
            }
          }
        }
#pragma unroll
        for (int i = 0; i < T; ++i) {
          const int cl = col0 + 16 * kPipeWaves * i;
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const int kk = 4 * s + g;
            bs[i][s] = (nb_in && cl < n && kk < K) ? nb_in[(long long)kk * sb + cl] : 0.f;
          }
        }
#pragma unroll
        for (int q = 1; q < 4; ++q)
#pragma unroll
          for (int i = 0; i < T; ++i)
#pragma unroll
            for (int s = 0; s < KS; ++s)
              if (q < nsl) CNMF_PIPE_N(i, s) += sl[q - 1][i][s];
        for (int q = 4; q < nsl; ++q) {       // more than 4 slabs (not produced by the engine): the rest in rounds
#pragma unroll
          for (int i = 0; i < T; ++i) {
            const int cl = col0 + 16 * kPipeWaves * i;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
              const int kk = 4 * s + g;
              const bool v = cl < n && kk < K;
              const float t = buf_ld(rn, v ? (kk * sn + cl) * 4 : 0, q * sstride);
              if (v) CNMF_PIPE_N(i, s) += t;
            }
          }
        }
#pragma unroll
        for (int i = 0; i < T; ++i) {
          const int cl = col0 + 16 * kPipeWaves * i;
          const bool ok = cl < n;
          const float scl = (ok && p.n_scale) ? p.n_scale[cl] : 1.f;
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const int kk = 4 * s + g;
            if (!(ok && kk < K)) continue;
            float nv = CNMF_PIPE_N(i, s);
            if (p.n_scale) nv *= scl;
            if (nb_in) nv = bs[i][s] + nv;
            if (nb_out) nb_out[(long long)kk * sb + cl] = nv;
            CNMF_PIPE_N(i, s) = nv;
          }
        }
      } else {
      // Slab-outer rounds: every element's load of slab q is in flight at once, the
      // running sum stays in the lane's own LDS slot
      for (int q = 1; q < nsl; ++q) {
#pragma unroll
        for (int i = 0; i < T; ++i) {
          const int cl = col0 + 16 * kPipeWaves * i;
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const int kk = 4 * s + g;
            const bool v = cl < n && kk < K;
            const float t = buf_ld(rn, v ? (kk * sn + cl) * 4 : 0, q * sstride);
            if (v) CNMF_PIPE_N(i, s) += t;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < T; ++i) {
        const int cl = col0 + 16 * kPipeWaves * i;
        const bool ok = cl < n;
        const float scl = (ok && p.n_scale) ? p.n_scale[cl] : 1.f;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int kk = 4 * s + g;
          if (!(ok && kk < K)) continue;
          float nv = CNMF_PIPE_N(i, s);
          if (p.n_scale) nv *= scl;
          if (nb_in) nv = nb_in[(long long)kk * sb + cl] + nv;
          if (nb_out) nb_out[(long long)kk * sb + cl] = nv;
          CNMF_PIPE_N(i, s) = nv;
        }
      }
      }
    }
  }
  // the summed Gram for the next solve that accumulates on it (slice 0 writes; every
  // slice summed the same values in the same order)
  if (p.gout && slc == 0 && wave == 0) {
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int row = 16 * b + pm, k = 4 * s + g;
        if (row < K && k < K) p.gout[(long long)rep * p.g_rs + row * K + k] = a[b][s];
      }
  }

  if (stp) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    st1 = __builtin_amdgcn_s_memtime();
  }
  const int every = p.check_every > 0 ? p.check_every : 1;
  const float eps = p.eps;
  int epoch = 0, it = 0;
  float f_prev = 0.f;
  bool have_prev = false;
  // <numer, x> and sum_j x_j^T Gram x_j of the CURRENT x from the last objective pass
  float lin_p = 0.f, quad_p = 0.f;
  bool lq_valid = false;
  // The objective of the initial x is only ever the reference of the first convergence
  // test: this slice's part of it is kept and exchanged together with the first real
  // check -- one cooperative exchange (a wait on the slowest slice) fewer per solve
  // (tools/pipe_stamp_probe.py: the checks were ~30 % of a launch).  (Folding its terms
  // into sweep 0 instead saved the chain pass too, but the second unrolled sweep body
  // pushed K = 20 past 128 VGPRs into scratch.)
  const bool defer0 = p.max_iter > 0;
  float f0_part = 0.f;
  bool f0_pending = false;

  while (true) {
    if (it % every == 0) {
      const unsigned long long tc0 = stp ? __builtin_amdgcn_s_memtime() : 0ull;
      // block objective x^T Gram x - 2 numer . x, pipelined like the sweep
      float qd = 0.f, ln = 0.f;
      f32x4p acc[2][MB];
      pipe_chain<KS, MB>(a, xr[0], acc[0]);
#pragma unroll
      for (int i = 0; i < T; ++i) {
        if (i + 1 < T) pipe_chain<KS, MB>(a, xr[i + 1], acc[(i + 1) & 1]);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const float xv = xr[i][s];
          qd = fmaf(xv, acc[i & 1][s >> 2][s & 3], qd);
          ln = fmaf(xv, CNMF_PIPE_N(i, s), ln);
        }
      }
      lin_p = ln;
      quad_p = qd;
      lq_valid = true;
      float q = qd, l = ln;
      block_sum2(q, l, sred);
      float f = q - 2.f * l;
      if (it == 0 && defer0) {            // kept for the first real check
        f0_part = f;
        f0_pending = true;
        if (stp) {
          st_chk += __builtin_amdgcn_s_memtime() - tc0;
          ++n_chk;
        }
        goto sweep;
      }
      float f0 = f0_part;
      if (stp && rt_x == 0) rt_x = __builtin_amdgcn_s_memrealtime();   // first arrival
      if (coop) {
        if (!coop_sum2_tag_s(p, gen, rep, epoch++, f, f0, sred, nsg, slc)) break;
      }
      if (f0_pending) {       // the initial objective, summed over the slices like f
        f_prev = f0;
        have_prev = true;
        f0_pending = false;
      }
      if (stp) {
        st_chk += __builtin_amdgcn_s_memtime() - tc0;
        ++n_chk;
      }
      if (have_prev && fabsf(f_prev - f) <= p.tol * fabsf(f_prev)) break;
      f_prev = f;
      have_prev = true;
    }
  sweep:
    if (it >= p.max_iter) break;
    // one MU sweep, software pipelined: chain(i + 1) in flight while tile i updates
    {
    f32x4p acc[2][MB];
    pipe_chain<KS, MB>(a, xr[0], acc[0]);
#pragma unroll
    for (int i = 0; i < T; ++i) {
      if (i + 1 < T) pipe_chain<KS, MB>(a, xr[i + 1], acc[(i + 1) & 1]);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float den = acc[i & 1][s >> 2][s & 3];
        const float xv = xr[i][s];
        const float rt = CNMF_PIPE_N(i, s) * __builtin_amdgcn_rcpf(den);
        xr[i][s] = (den < eps) ? 0.f : xv * rt;
      }
    }
    }
    ++it;
    lq_valid = false;
  }

  const unsigned long long st2 = stp ? __builtin_amdgcn_s_memtime() : 0ull;
  // the final iterate, and (optionally) its bf16 planes straight from the registers
  {
    int col0 = j0 + 16 * wave + c;
    asm volatile("" : "+v"(col0));
    unsigned short* __restrict__ pl =
        p.planes ? p.planes + (long long)rep * p.pl_rs : nullptr;
#pragma unroll
    for (int i = 0; i < T; ++i) {
      const int cl = col0 + 16 * kPipeWaves * i;
      const bool ok = cl < n;
      const float m = (pl && ok && p.pl_colmul) ? p.pl_colmul[cl] : 1.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kk = 4 * s + g;
        if (ok && kk < K) {
          buf_st(xr[i][s], rx, (kk * sx + cl) * 4, 0);
          if (pl) {
            const float v = xr[i][s] * m;
            const long long o = (long long)kk * p.pl_ld + cl;
            const unsigned short h0 = pipe_bf16_rn(v);
            pl[o] = h0;
            if (pl_n > 1) {
              const float r1 = v - __uint_as_float((unsigned)h0 << 16);
              const unsigned short h1 = pipe_bf16_rn(r1);
              pl[p.pl_plane + o] = h1;
              if (pl_n > 2)
                pl[2 * p.pl_plane + o] = pipe_bf16_rn(r1 - __uint_as_float((unsigned)h1 << 16));
            }
          }
        }
      }
    }
    // the last slice zeroes the GEMM's k padding [ncols, pl_cols) of every plane it reads
    if (pl && (!coop || slc == nsg - 1)) {
      const int pad = p.pl_cols - p.ncols;
      for (int e = threadIdx.x; e < pad * K; e += 64 * kPipeWaves) {
        const int kk = e / pad, cc = p.ncols + e % pad;
        const long long o = (long long)kk * p.pl_ld + cc;
        for (int q = 0; q < pl_n; ++q) pl[q * p.pl_plane + o] = 0;
      }
    }
  }

  if (p.lin_out || p.quad_out) {
    float lin = lin_p, quad = quad_p;
    if (!lq_valid) {   // stopped by max_iter: one more product for the final x
      lin = 0.f;
      quad = 0.f;
      f32x4p acc[2][MB];
      pipe_chain<KS, MB>(a, xr[0], acc[0]);
#pragma unroll
      for (int i = 0; i < T; ++i) {
        if (i + 1 < T) pipe_chain<KS, MB>(a, xr[i + 1], acc[(i + 1) & 1]);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          lin = fmaf(CNMF_PIPE_N(i, s), xr[i][s], lin);
          quad = fmaf(xr[i][s], acc[i & 1][s >> 2][s & 3], quad);
        }
      }
    }
    block_sum2(lin, quad, sred);
    if (coop) (void)coop_sum2_tag_s(p, gen, rep, epoch++, lin, quad, sred, nsg, slc);
    if (threadIdx.x == 0 && (!coop || slc == 0)) {
      if (p.lin_out) p.lin_out[rep] = lin;
      if (p.quad_out) p.quad_out[rep] = quad;
    }
  }
  if (p.gp_out) {
    // this slice's partial Gram sum_cols x x^T of the final x (the next solve's gpart):
    // each wave transposes its tiles through LDS into [column][component] (row stride
    // KP + 1) and runs gram.hip's trick per 16 x 16 block (b1, b2) -- lane (g, c) feeds
    // F[16 b1 + c][col 4j + g] as A[m = c][k = g] and F[16 b2 + c][col 4j + g] as
    // B[k = g][n = c], so D[m][n] = sum over the 16 columns of F[16b1 + m][col] F[16b2 + n][col]
    // (the (b2, b1) block sums the same products in the same order: bitwise symmetric)
    constexpr int KPP = KP + 1;
    __syncthreads();                       // every wave is done with the numerators
    float* sT = sN + wave * 16 * KPP;
    for (int e = lane; e < 16 * KPP; e += 64) sT[e] = 0.f;   // components >= 4 KS stay zero
    __builtin_amdgcn_wave_barrier();
    f32x4p gacc[MB][MB];
#pragma unroll
    for (int b1 = 0; b1 < MB; ++b1)
#pragma unroll
      for (int b2 = 0; b2 < MB; ++b2) gacc[b1][b2] = f32x4p{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < T; ++i) {
#pragma unroll
      for (int s = 0; s < KS; ++s) sT[c * KPP + 4 * s + g] = xr[i][s];
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the tile is in LDS
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[MB];
#pragma unroll
        for (int b = 0; b < MB; ++b) v[b] = sT[(4 * j + g) * KPP + 16 * b + c];
#pragma unroll
        for (int b1 = 0; b1 < MB; ++b1)
#pragma unroll
          for (int b2 = 0; b2 < MB; ++b2)
            gacc[b1][b2] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[b1], v[b2], gacc[b1][b2], 0, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();       // reads done before the next tile's writes
    }
    __syncthreads();
    // lane (g, c) holds D_b1b2[4 g + r][c]; per 16-row band b1 the 4 wave partials are
    // summed in wave order
    float* go = p.gp_out + (long long)rep * p.gp_rs + (long long)slc * K * K;
#pragma unroll
    for (int b1 = 0; b1 < MB; ++b1) {
#pragma unroll
      for (int b2 = 0; b2 < MB; ++b2)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sN[wave * 16 * KP + (4 * g + r) * KP + 16 * b2 + c] = gacc[b1][b2][r];
      __syncthreads();
      for (int e = threadIdx.x; e < 16 * K; e += 64 * kPipeWaves) {
        const int m = e / K, q = e - m * K;
        if (16 * b1 + m < K) {
          float v = 0.f;
#pragma unroll
          for (int w = 0; w < kPipeWaves; ++w) v += sN[w * 16 * KP + m * KP + q];
          go[(16 * b1 + m) * K + q] = v;
        }
      }
      __syncthreads();
    }
  }
  if (p.iters_out && threadIdx.x == 0 && slc == 0) p.iters_out[rep] += it;
  if (stp) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long* o = p.stamps + ((unsigned long long)slc * p.pipe_nblocks + blk) * 10;
      const unsigned long long st3 = __builtin_amdgcn_s_memtime();
      o[0] = rt0; o[1] = __builtin_amdgcn_s_memrealtime();   // 100 MHz, chip-wide
      o[2] = st1 - st0; o[3] = st2 - st1; o[4] = st_chk; o[5] = st3 - st2;   // cycles
      o[6] = rt_x; o[7] = (n_chk << 32) | (unsigned long long)(unsigned)it;
      // where this workgroup ran: HW_ID (CU / SH / SE bits) and the XCD (XCC_ID)
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
      o[8] = hw;
      o[9] = xcc;
    }
  }
  pipe_arrive(p);
}

// tile counts instantiated (the host rounds up to the next one within pipe_tile_max(K))
__host__ __device__ constexpr int pipe_t_of(int idx) {
  return idx == 0 ? 1 : idx == 1 ? 2 : idx == 2 ? 3 : idx == 3 ? 4 : idx == 4 ? 5 :
         idx == 5 ? 6 : idx == 6 ? 7 : idx == 7 ? 8 : idx == 8 ? 9 : idx == 9 ? 10 : 12;
}
constexpr int kPipeTCount = 11;

template <int K, int T>
static hipError_t launch_pipe_kt(const SolveParams& p, int nblocks, int pl_n, hipStream_t s) {
  if constexpr (T <= pipe_tile_max(K)) {
    const int gy = p.coop_slots ? p.coop_epochs_split : 1;
    SolveParams q = p;
    q.pipe_nblocks = nblocks;
    const dim3 grid = q.pipe_map ? dim3(((nblocks + 7) / 8) * 8 * gy, 1) : dim3(nblocks, gy);
    hipLaunchKernelGGL((solve_pipe_kernel<K, T>), grid, dim3(64 * kPipeWaves), 0, s, q, pl_n);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}

template <int K>
static hipError_t launch_pipe_k(const SolveParams& p, int nblocks, int T, int pl_n,
                                hipStream_t s) {
  if (T <= 1) return launch_pipe_kt<K, 1>(p, nblocks, pl_n, s);
  if (T <= 2) return launch_pipe_kt<K, 2>(p, nblocks, pl_n, s);
  if (T <= 3) return launch_pipe_kt<K, 3>(p, nblocks, pl_n, s);
  if (T <= 4) return launch_pipe_kt<K, 4>(p, nblocks, pl_n, s);
  if (T <= 5) return launch_pipe_kt<K, 5>(p, nblocks, pl_n, s);
  if (T <= 6) return launch_pipe_kt<K, 6>(p, nblocks, pl_n, s);
  if (T <= 7) return launch_pipe_kt<K, 7>(p, nblocks, pl_n, s);
  if (T <= 8) return launch_pipe_kt<K, 8>(p, nblocks, pl_n, s);
  if (T <= 9) return launch_pipe_kt<K, 9>(p, nblocks, pl_n, s);
  if (T <= 10) return launch_pipe_kt<K, 10>(p, nblocks, pl_n, s);
  if (T <= 12) return launch_pipe_kt<K, 12>(p, nblocks, pl_n, s);
  return hipErrorInvalidValue;
}

}  // namespace cnmf
