// Software-pipelined matrix-core MU solve (K <= 16): the hot path of every Frobenius
// online pass (SURVEY.md §2.4 G3 -- the H/W inner loops of cnmf.py:365-378 and nmf-torch's
// online MU), for the common unregularised case (l1 = l2 = 0) with the block-objective
// stop (conv_mode 1, nmf-torch online_inner_conv='loss').  Same contract, data layout and
// cooperative slicing as solve_mfma_kernel (solve_mfma.hip), which keeps the regularised,
// iterate-change, fixed-split and in-prologue-Gram cases.
//
// Why a second kernel.  solve_mfma_kernel walks its column tiles strictly one after the
// other (a sched_barrier per tile, a runtime tile count T with a branch per tile): each
// tile is a chain of K/4 DEPENDENT v_mfma_f32_16x16x4_f32 (40-cycle dependent latency
// each, MI355X_MICROARCH.md cycle table), an s_nop until the accumulator is readable, then
// ~20 VALU of which the compiler SLP-packs half into v_pk_*_f32 (an anti-lever beside
// MFMAs, same table).  Nothing overlaps the chain inside a wave, so on the bench's H side
// a sweep took ~3.9 us against ~1.3 us of MFMA issue (docs/ARCHITECTURE.md "Solve sweeps").
//
// Here T is a template parameter (the host rounds the tile count up to an instantiated
// one; padded tiles hold zero columns, which MU keeps at zero), and the sweep is software
// pipelined: the MFMA chain of tile i+1 is issued before the elementwise update of tile
// i, whose accumulator was produced one step earlier.  The chains of consecutive tiles
// are independent, so the matrix core always has the next tile's work while the VALU
// finishes the previous one, within ONE wave.  Without l1/l2 the update is
//     den = (Gram x)_k ;  x_k <- den < eps ? 0 : x_k * (numer_k * rcp(den))
// five VALU per element (cmp, cndmask, rcp, 2 mul), all scalar f32 (-fno-slp-vectorize for
// this unit), which fits the issue slots a 16x16x4 f32 MFMA leaves (32 cycles, 8 held).
//
// The planes epilogue emits the final x straight from registers (no re-read from L2) and
// only the `pl_n` planes the consuming GEMM reads (2 with a >= 1024-deep reduction,
// ops.gemm_a_planes), instead of three.
#include "solve_core.h"

namespace cnmf {

typedef float f32x4p __attribute__((ext_vector_type(4)));

constexpr int kPipeWaves = 4;   // waves per workgroup (256 threads)

#define CNMF_PIPE_N(i, s) sN[((i) * KS + (s)) * (64 * kPipeWaves) + threadIdx.x]

template <int K, int KS>
__device__ __forceinline__ f32x4p pipe_chain(const float (&a)[KS], const float (&x)[KS]) {
  f32x4p d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], x[s], d, 0, 0, 0);
  return d;
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

// amdgpu_waves_per_eu(4): <= 128 VGPRs, four workgroups per CU (the host's co-residency
// budget MFMA_WG_PER_CU for cooperative slices, ops/__init__.py)
template <int K, int T>
__global__ __launch_bounds__(64 * kPipeWaves) __attribute__((amdgpu_waves_per_eu(4)))
void solve_pipe_kernel(SolveParams p, int pl_n) {
  constexpr int KS = (K + 3) / 4;
  __shared__ float sred[3 + 2 * kCoopMaxSlices];
  // numerators of this lane's columns; also the partial-Gram scratch of the epilogue
  // (one 16 x 16 tile per wave), hence at least 4 x 256 floats
  __shared__ float sN[(T * KS >= 4 ? T * KS : 4) * 64 * kPipeWaves];
  const int rep = p.rep_index ? p.rep_index[blockIdx.x] : (int)blockIdx.x;
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

  // Gram fragments, rows permuted by pi(4g + r) = 4r + g (see solve_mfma.hip): the
  // accumulator register r of lane (g, c) is then component 4r + g of column c, the
  // component this lane's B register r holds -- the update needs no data movement
  float a[KS];
  const int pm = 4 * (c & 3) + (c >> 2);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + g;
    a[s] = (gm && pm < K && k < K) ? gm[pm * K + k] : 0.f;
  }
  if (p.gpart) {
    // + the producing solve's per-slice partial Grams, summed in slice order; eight
    // slices' loads in flight per round (a sequential load-add chain per element cost
    // ~gpart_n memory latencies)
    const float* gp = p.gpart + (long long)rep * p.gpart_rs + pm * K;
    float t[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) t[s] = 0.f;
    for (int q0 = 0; q0 < p.gpart_n; q0 += 8) {
      float v[8][KS];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int k = 4 * s + g;
          v[j][s] = (q0 + j < p.gpart_n && pm < K && k < K) ? gp[(q0 + j) * K * K + k] : 0.f;
        }
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int s = 0; s < KS; ++s) t[s] += v[j][s];   // + 0 for q >= gpart_n: exact
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) a[s] = gm ? a[s] + t[s] : t[s];
  }

  int j0 = 0, n = p.ncols;
  const bool coop = p.coop_slots != nullptr && gridDim.y > 1;
  if (coop) {
    const int per = (p.ncols + (int)gridDim.y - 1) / (int)gridDim.y;
    j0 = min(p.ncols, (int)blockIdx.y * per);
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
      // bitwise gemm_reduce_kernel's "C (+)= col_scale * sum_s slab[s]".  Slab-outer
      // rounds: every element's load of slab q is in flight at once, the running sum
      // stays in the lane's own LDS slot
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
  // the summed Gram for the next solve that accumulates on it (slice 0 writes; every
  // slice summed the same values in the same order)
  if (p.gout && blockIdx.y == 0 && pm < K) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 4 * s + g;
      if (k < K && wave == 0) p.gout[(long long)rep * p.g_rs + pm * K + k] = a[s];
    }
  }

  const int every = p.check_every > 0 ? p.check_every : 1;
  const float eps = p.eps;
  int epoch = 0, it = 0;
  float f_prev = 0.f;
  bool have_prev = false;
  // <numer, x> and sum_j x_j^T Gram x_j of the CURRENT x from the last objective pass
  float lin_p = 0.f, quad_p = 0.f;
  bool lq_valid = false;

  while (true) {
    if (it % every == 0) {
      // block objective x^T Gram x - 2 numer . x, pipelined like the sweep
      float qd = 0.f, ln = 0.f;
      f32x4p acc[2];
      acc[0] = pipe_chain<K, KS>(a, xr[0]);
#pragma unroll
      for (int i = 0; i < T; ++i) {
        if (i + 1 < T) acc[(i + 1) & 1] = pipe_chain<K, KS>(a, xr[i + 1]);
#pragma unroll
        for (int r = 0; r < KS; ++r) {
          const float xv = xr[i][r];
          qd = fmaf(xv, acc[i & 1][r], qd);
          ln = fmaf(xv, CNMF_PIPE_N(i, r), ln);
        }
      }
      lin_p = ln;
      quad_p = qd;
      lq_valid = true;
      float q = qd, l = ln;
      block_sum2(q, l, sred);
      float f = q - 2.f * l;
      if (coop) {
        float unused = 0.f;
        if (!coop_sum2_tag(p, gen, rep, epoch++, f, unused, sred)) break;
      }
      if (have_prev && fabsf(f_prev - f) <= p.tol * fabsf(f_prev)) break;
      f_prev = f;
      have_prev = true;
    }
    if (it >= p.max_iter) break;
    // one MU sweep, software pipelined: chain(i + 1) in flight while tile i updates
    f32x4p acc[2];
    acc[0] = pipe_chain<K, KS>(a, xr[0]);
#pragma unroll
    for (int i = 0; i < T; ++i) {
      if (i + 1 < T) acc[(i + 1) & 1] = pipe_chain<K, KS>(a, xr[i + 1]);
#pragma unroll
      for (int r = 0; r < KS; ++r) {
        const float den = acc[i & 1][r];
        const float xv = xr[i][r];
        const float rt = CNMF_PIPE_N(i, r) * __builtin_amdgcn_rcpf(den);
        xr[i][r] = (den < eps) ? 0.f : xv * rt;
      }
    }
    ++it;
    lq_valid = false;
  }

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
    if (pl && (!coop || blockIdx.y == gridDim.y - 1)) {
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
      f32x4p acc[2];
      acc[0] = pipe_chain<K, KS>(a, xr[0]);
#pragma unroll
      for (int i = 0; i < T; ++i) {
        if (i + 1 < T) acc[(i + 1) & 1] = pipe_chain<K, KS>(a, xr[i + 1]);
#pragma unroll
        for (int r = 0; r < KS; ++r) {
          lin = fmaf(CNMF_PIPE_N(i, r), xr[i][r], lin);
          quad = fmaf(xr[i][r], acc[i & 1][r], quad);
        }
      }
    }
    block_sum2(lin, quad, sred);
    if (coop) (void)coop_sum2_tag(p, gen, rep, epoch++, lin, quad, sred);
    if (threadIdx.x == 0 && (!coop || blockIdx.y == 0)) {
      if (p.lin_out) p.lin_out[rep] = lin;
      if (p.quad_out) p.quad_out[rep] = quad;
    }
  }
  if (p.gp_out) {
    // this slice's partial Gram sum_cols x x^T of the final x (the next solve's gpart):
    // each wave transposes its tiles through LDS into [column][component] and runs
    // gram.hip's trick -- lane (g, c) feeds F[c][col 4j + g] as both A[m = c][k = g] and
    // B[k = g][n = c], so D[m][n] = sum over the 16 columns of F[m][col] F[n][col]
    __syncthreads();                       // every wave is done with the numerators
    float* sT = sN + wave * 256;
    for (int e = lane; e < 256; e += 64) sT[e] = 0.f;   // components >= 4 KS stay zero
    __builtin_amdgcn_wave_barrier();
    f32x4p gacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < T; ++i) {
#pragma unroll
      for (int s = 0; s < KS; ++s) sT[c * 16 + 4 * s + g] = xr[i][s];
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the tile is in LDS
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = sT[(4 * j + g) * 16 + c];
        gacc = __builtin_amdgcn_mfma_f32_16x16x4f32(v, v, gacc, 0, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();       // reads done before the next tile's writes
    }
    __syncthreads();
    // lane (g, c) holds D[4 g + r][c]; the 4 wave partials summed in wave order
#pragma unroll
    for (int r = 0; r < 4; ++r) sN[wave * 256 + (4 * g + r) * 16 + c] = gacc[r];
    __syncthreads();
    float* go = p.gp_out + (long long)rep * p.gp_rs + (long long)blockIdx.y * K * K;
    for (int e = threadIdx.x; e < K * K; e += 64 * kPipeWaves) {
      const int m = e / K, q = e - m * K;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < kPipeWaves; ++w) v += sN[w * 256 + m * 16 + q];
      go[e] = v;
    }
  }
  if (p.iters_out && threadIdx.x == 0 && blockIdx.y == 0) p.iters_out[rep] += it;
  pipe_arrive(p);
}

// tile counts instantiated per K (the host rounds up to the next one)
__host__ __device__ constexpr int pipe_t_of(int idx) {
  return idx == 0 ? 1 : idx == 1 ? 2 : idx == 2 ? 3 : idx == 3 ? 4 : idx == 4 ? 5 :
         idx == 5 ? 6 : idx == 6 ? 8 : idx == 7 ? 9 : idx == 8 ? 10 : 12;
}
constexpr int kPipeTCount = 10;
// x in VGPRs (T * KS), numerators in LDS (T * KS * 1 KB): K <= 12 up to 12 tiles (36 KB),
// K 13..16 up to 9 (36 KB) -- four workgroups per CU either way
__host__ __device__ constexpr int pipe_tile_max(int K) { return K <= 12 ? 12 : 9; }

template <int K, int T>
static hipError_t launch_pipe_kt(const SolveParams& p, int nblocks, int pl_n, hipStream_t s) {
  const int gy = p.coop_slots ? p.coop_epochs_split : 1;
  hipLaunchKernelGGL((solve_pipe_kernel<K, T>), dim3(nblocks, gy), dim3(64 * kPipeWaves), 0, s,
                     p, pl_n);
  return hipGetLastError();
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
  if (T <= 8) return launch_pipe_kt<K, 8>(p, nblocks, pl_n, s);
  if (T <= 9) return launch_pipe_kt<K, 9>(p, nblocks, pl_n, s);
  if constexpr (pipe_tile_max(K) >= 12) {
    if (T <= 10) return launch_pipe_kt<K, 10>(p, nblocks, pl_n, s);
    if (T <= 12) return launch_pipe_kt<K, 12>(p, nblocks, pl_n, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace cnmf

namespace cnmf {
#define CNMF_PIPE_CASE(KK) \
  case KK: return launch_pipe_k<KK>(p, nblocks, T, pl_n, s);
hipError_t launch_solve_pipe(int K, const SolveParams& p, int nblocks, int T, int pl_n,
                             hipStream_t s) {
  if (T > pipe_tile_max(K)) return hipErrorInvalidValue;
  switch (K) {
    CNMF_PIPE_CASE(1) CNMF_PIPE_CASE(2) CNMF_PIPE_CASE(3) CNMF_PIPE_CASE(4)
    CNMF_PIPE_CASE(5) CNMF_PIPE_CASE(6) CNMF_PIPE_CASE(7) CNMF_PIPE_CASE(8)
    CNMF_PIPE_CASE(9) CNMF_PIPE_CASE(10) CNMF_PIPE_CASE(11) CNMF_PIPE_CASE(12)
    CNMF_PIPE_CASE(13) CNMF_PIPE_CASE(14) CNMF_PIPE_CASE(15) CNMF_PIPE_CASE(16)
    default: return hipErrorInvalidValue;
  }
}
#undef CNMF_PIPE_CASE
}  // namespace cnmf

// tile count the pipelined solve runs for `per` columns per slice (0: not covered)
extern "C" int cnmf_solve_pipe_tiles(int K, int per) {
  if (K < 1 || K > 16 || per < 1) return 0;
  const int need = (per + 16 * cnmf::kPipeWaves - 1) / (16 * cnmf::kPipeWaves);
  if (need > cnmf::pipe_tile_max(K)) return 0;
  for (int i = 0; i < cnmf::kPipeTCount; ++i)
    if (cnmf::pipe_t_of(i) >= need) return cnmf::pipe_t_of(i);
  return 0;
}
