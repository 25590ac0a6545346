// Split-precision fp32 GEMM on the bf16 matrix cores (the
// data-side products of every online NMF step, numer = W X_c^T and B += H_c^T X_c).
//
// gfx950 has no xf32/TF32 MFMA: fp32 operands run at the vector rate (157 TF), 1/16 of
// bf16 MFMA (2.5 PF).  An fp32 value splits EXACTLY into three bf16 planes
// (v = hi + mid + lo: 8 + 8 + 8 mantissa bits, each residual exact in fp32), and a
// bf16 x bf16 product is exact in the fp32 accumulator.  So
//
//     C = sum over plane pairs (i, j) with i + j <= 2 of  A_i . B_j^T      (fp32 accumulate)
//
// reproduces the fp32 GEMM to fp32 rounding (the dropped pairs are < 2^-24 relative).
// With TWO A planes (PA = 2: hi + mid, |v - hi - mid| <= 2^-16 |v|) the product error is
// <= 2^-16 sum|a b| -- inside the standard fp32 GEMM bound n 2^-24 sum|a b| for every
// reduction length n >= 256, and from n ~ 1000 on measured below hipBLASLt's fp32 GEMM
// error (tests:
// test_gemm_two_a_planes_within_fp32_library_error); the engine uses it for k >= 1024.
// The cNMF data matrix is counts / per-gene std: with the per-gene unit folded into the
// OTHER operand (A's columns for numer, C's columns for B) the count matrix is held
// exactly by ONE bf16 plane (counts <= 256) or two (< 65536), so the product costs 3 (or
// 5) bf16 MFMAs instead of one fp32 MFMA of 16x the cycles.  The operand planes are
// produced once per update by ``split_planes_kernel`` (X: once per factorisation).
//
// Tiling: 128 x 128 output tile per 256-thread workgroup (2 x 2 waves, 64 x 64 each,
// 4 x 4 accumulators of v_mfma_f32_16x16x32_bf16), BK-deep k-steps staged global -> LDS
// by LDS-DMA (global_load_lds_dwordx4, 16 B per lane) into two buffers: step k+1 is in
// flight while step k is multiplied (counted vmcnt + raw s_barrier, never a vmcnt(0)
// inside the loop -- cdna_hip_programming.md §5 "Pipelining across barriers").  LDS rows
// are 16-byte-chunk XOR-swizzled on the SOURCE address (glds writes lane-linear), which
// makes the ds_read_b128 fragment reads conflict-free.  Workgroup ids are remapped so a
// run of consecutive tiles shares one XCD's L2 (T1).  Rows of A / B beyond the matrix
// are clamped (valid memory, results discarded); the k range must be padded to BK with
// zeros in A (the caller's plane buffers are).
#include <hip/hip_runtime.h>

namespace cnmf {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

struct PlaneGemmParams {
  const unsigned short* A;  // plane p at A + p * a_plane, rows [a_rows][lda] (k contiguous)
  long long lda, a_plane;
  int a_rows;
  const unsigned short* B;  // plane p at B + p * b_plane, rows [b_rows][ldb]
  long long ldb, b_plane;
  int b_rows;
  float* C;                 // [M][ldc]
  long long ldc;
  const float* col_scale;   // optional per-output-column factor
  int M, N, Kd;             // Kd: multiple of BK
  int accumulate;           // C += instead of C =
  int tiles_m, tiles_n;
  int ksplit;               // > 1: workgroup z-slice of k; raw partials to `slab`
  float* slab;              // [ksplit][M][N] partial products (split-K only)
  int raw;                  // 1: raw partials to `slab` even at ksplit 1, and no reduce --
                            // the consuming solve sums them (solve_pipe.hip numer slabs)
  const int* gate;          // optional: *gate == 0 -> every workgroup returns at once (an
                            // online pass enqueued after every replicate had finished)
};

__device__ __forceinline__ unsigned short f2bf_rn(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);  // round to nearest even (finite inputs)
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf2f(unsigned short h) {
  return __uint_as_float((unsigned)h << 16);
}

// 16-byte chunk swizzle within a tile row (chunk count CPR): conflict-free ds_read_b128
// for the 16x16x32 fragment pattern (rows lane&15, chunk lane>>4) -- checked against the
// gfx950 ds_read_b128 lane groups.
template <int CPR>
__device__ __forceinline__ int swz(int row) {
  return CPR == 8 ? (row & 7) : ((row >> 1) & 3);
}

__device__ __forceinline__ void glds16(const unsigned short* g, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)lds, 16, 0, 0);
}

template <int PA, int PB, int BK, int WM, int WN, int NS, int MI = 4>
__global__ __launch_bounds__(64 * WM * WN) void gemm_planes_kernel(PlaneGemmParams p) {
  // gate: read now, tested after the prologue's loads are issued, so its latency hides
  // behind theirs (testing it first cost ~1 % of the headline: every GEMM waited for it)
  const int gate_v = p.gate ? *p.gate : 1;
  constexpr int NT = 64 * WM * WN;            // threads
  constexpr int WR = 16 * MI;                 // each wave owns a WR x 64 output block
  constexpr int BM = WR * WM, BN = 64 * WN;
  constexpr int CPR = BK / 8;                 // 16-byte chunks per tile row
  constexpr int A_TILE = BM * BK * 2;         // bytes per plane tile
  constexpr int B_TILE = BN * BK * 2;
  constexpr int STAGE = PA * A_TILE + PB * B_TILE;
  constexpr int A_LD = BM * CPR / NT;         // glds per thread per A plane
  constexpr int B_LD = BN * CPR / NT;
  constexpr int LOADS = PA * A_LD + PB * B_LD;
  static_assert(A_LD * NT == BM * CPR && B_LD * NT == BN * CPR, "tile / thread mismatch");
  static_assert(NS >= 2 && NS <= 4, "2..4 stages");
  static_assert((NS >= 4 ? 2 : 1) * LOADS < 64, "vmcnt is a 6-bit counter");
  static_assert(NS * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STAGE];

  // XCD-aware bijective remap; consecutive logical tiles share the M panel (the A
  // operand: three planes, the larger one), so an XCD keeps its A panels in its L2 and
  // streams B
  const int nwg = p.tiles_m * p.tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tn = wg % p.tiles_n, tm = wg / p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  // k range of this workgroup (split-K slice blockIdx.y)
  const int nk_all = p.Kd / BK;
  const int ks = blockIdx.y;
  const int kb = (int)((long long)nk_all * ks / p.ksplit);
  const int ke = (int)((long long)nk_all * (ks + 1) / p.ksplit);

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // per-thread global source offsets (elements) of its glds chunks, k excluded
  long long a_off[A_LD], b_off[B_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int qd = i * NT + t, row = qd / CPR, pos = qd % CPR;
    const int gr = min(m0 + row, p.a_rows - 1);
    a_off[i] = (long long)gr * p.lda + (pos ^ swz<CPR>(row)) * 8;
  }
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    const int qd = i * NT + t, row = qd / CPR, pos = qd % CPR;
    const int gr = min(n0 + row, p.b_rows - 1);
    b_off[i] = (long long)gr * p.ldb + (pos ^ swz<CPR>(row)) * 8;
  }

  auto issue = [&](int stage, int k0) {
    unsigned char* base = smem + stage * STAGE;
#pragma unroll
    for (int pl = 0; pl < PA; ++pl)
#pragma unroll
      for (int i = 0; i < A_LD; ++i)
        glds16(p.A + pl * p.a_plane + a_off[i] + k0,
               base + pl * A_TILE + (i * NT + wave * 64) * 16);
#pragma unroll
    for (int pl = 0; pl < PB; ++pl)
#pragma unroll
      for (int i = 0; i < B_LD; ++i)
        glds16(p.B + pl * p.b_plane + b_off[i] + k0,
               base + PA * A_TILE + pl * B_TILE + (i * NT + wave * 64) * 16);
  };

  f32x4v acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  // NS-stage ring: stage kt+NS-1 is issued right after the barrier that certifies every
  // wave has finished multiplying stage kt-1 (whose slot it refills), so ONE barrier per
  // k-step and NS-1 k-steps of loads in flight behind the MFMAs
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (kb + s < ke) issue(s, (kb + s) * BK);
  if (gate_v == 0) {   // uniform: nothing to compute; drain the LDS-DMA first
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  for (int kt = kb; kt < ke; ++kt) {
    const int cur = (kt - kb) % NS;
    // stage kt has landed once at most min(NS-2, ke-1-kt) later stages are outstanding
    const int later = min(NS - 2, ke - 1 - kt);
    if (later >= 2) {
      if constexpr (NS >= 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LOADS) : "memory");
    } else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LOADS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // this wave's fragment reads of the slot refilled below have returned
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < ke) issue((kt - kb + NS - 1) % NS, (kt + NS - 1) * BK);
    const unsigned char* As = smem + cur * STAGE;
    const unsigned char* Bs = As + PA * A_TILE;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int c = kk * 4 + (lane >> 4);
      bf16x8 bfr[PB][4];
#pragma unroll
      for (int j = 0; j < PB; ++j)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int row = wn * 64 + ni * 16 + (lane & 15);
          bfr[j][ni] = *(const bf16x8*)(Bs + j * B_TILE + row * (BK * 2) +
                                        ((c ^ swz<CPR>(row)) * 16));
        }
      bf16x8 afr[PA][MI];
#pragma unroll
      for (int i = 0; i < PA; ++i)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
          const int row = wm * WR + mi * 16 + (lane & 15);
          afr[i][mi] = *(const bf16x8*)(As + i * A_TILE + row * (BK * 2) +
                                        ((c ^ swz<CPR>(row)) * 16));
        }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int i = PA - 1; i >= 0; --i)      // small planes first
#pragma unroll
            for (int j = PB - 1; j >= 0; --j)
              if (i + j <= 2)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i][mi], bfr[j][ni],
                                                                      acc[mi][ni], 0, 0, 0);
    }
  }

  if (p.ksplit > 1 || p.raw) {   // raw partial tile -> slab ks (reduced in slice order
                                 // by gemm_reduce, or by the consumer when raw)
    float* sl = p.slab + (long long)ks * p.M * p.N;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int gn = n0 + wn * 64 + ni * 16 + (lane & 15);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int gm = m0 + wm * WR + mi * 16 + (lane >> 4) * 4 + rr;
          if (gm < p.M && gn < p.N) sl[(long long)gm * p.N + gn] = acc[mi][ni][rr];
        }
      }
    return;
  }

  // epilogue: lane holds rows (lane>>4)*4 + r of column lane&15 of each 16x16 block.
  // Accumulating: every old value is loaded (clamped addresses, no per-element branch)
  // before any is used, so the 64 loads are in flight together.
  float sc[4];
  int gn[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    gn[ni] = n0 + wn * 64 + ni * 16 + (lane & 15);
    sc[ni] = p.col_scale ? p.col_scale[min(gn[ni], p.N - 1)] : 1.f;
  }
  const int gm0 = m0 + wm * WR + (lane >> 4) * 4;
  if (p.accumulate) {
    float old[MI][4][4];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          old[mi][ni][rr] = p.C[(long long)min(gm0 + mi * 16 + rr, p.M - 1) * p.ldc +
                                min(gn[ni], p.N - 1)];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int gm = gm0 + mi * 16 + rr;
          if (gm < p.M && gn[ni] < p.N)
            p.C[(long long)gm * p.ldc + gn[ni]] = old[mi][ni][rr] + acc[mi][ni][rr] * sc[ni];
        }
  } else {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int gm = gm0 + mi * 16 + rr;
          if (gm < p.M && gn[ni] < p.N)
            p.C[(long long)gm * p.ldc + gn[ni]] = acc[mi][ni][rr] * sc[ni];
        }
  }
}

// S (rows x cols, row stride lds) [* col_mul] -> nplanes bf16 planes [rows][ldp], plane
// stride `plane`; columns [cols, cols_pad) are written as zeros (k padding of the GEMM).
// Each thread converts 4 consecutive columns.
__global__ void split_planes_kernel(const float* __restrict__ S, long long lds, int rows,
                                    int cols, int cols_pad, const float* __restrict__ col_mul,
                                    unsigned short* __restrict__ P, long long ldp,
                                    long long plane, int nplanes) {
  const int c4 = cols_pad / 4;
  const long long total = (long long)rows * c4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / c4);
    const int c = (int)(i - (long long)r * c4) * 4;
    unsigned short h[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int cc = c + e;
      float v = 0.f;
      if (cc < cols) {
        v = S[(long long)r * lds + cc];
        if (col_mul) v *= col_mul[cc];
      }
      const unsigned short h0 = f2bf_rn(v);
      const float r1 = v - bf2f(h0);
      const unsigned short h1 = f2bf_rn(r1);
      const float r2 = r1 - bf2f(h1);
      h[0][e] = h0;
      h[1][e] = h1;
      h[2][e] = f2bf_rn(r2);
    }
    for (int pl = 0; pl < nplanes; ++pl) {
      uint2 w;
      w.x = (unsigned)h[pl][0] | ((unsigned)h[pl][1] << 16);
      w.y = (unsigned)h[pl][2] | ((unsigned)h[pl][3] << 16);
      *(uint2*)(P + pl * plane + (long long)r * ldp + c) = w;
    }
  }
}

// C (+)= col_scale * sum_s slab[s] in slice order (deterministic split-K reduction)
__global__ void gemm_reduce_kernel(const float* __restrict__ slab, int ksplit, int M, int N,
                                   float* __restrict__ C, long long ldc,
                                   const float* __restrict__ col_scale, int accumulate,
                                   const int* gate) {
  // (the gate is not tested here: a reduce of a skipped product writes an output no
  // replicate reads, and waiting for the flag cost more than the rare skip saves)
  (void)gate;
  const long long total = (long long)M * N;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < ksplit; ++s) v += slab[(long long)s * total + i];
    const int m = (int)(i / N), n = (int)(i - (long long)m * N);
    if (col_scale) v *= col_scale[n];
    float* cp = C + (long long)m * ldc + n;
    *cp = accumulate ? *cp + v : v;
  }
}

template <int PA, int PB, int BK, int WM, int WN, int MI = 4>
static hipError_t launch_gemm(PlaneGemmParams p, int stages, hipStream_t s) {
  constexpr int stage_bytes = (PA * 16 * MI * WM + PB * 64 * WN) * BK * 2;
  if constexpr (BK > 32 && 2 * stage_bytes > 160 * 1024) {
    return launch_gemm<PA, PB, 32, WM, WN, MI>(p, stages, s);   // deep k-step does not fit
  } else {
  p.tiles_m = (p.M + 16 * MI * WM - 1) / (16 * MI * WM);
  p.tiles_n = (p.N + 64 * WN - 1) / (64 * WN);
  const dim3 grid(p.tiles_m * p.tiles_n, p.ksplit), block(64 * WM * WN);
  if constexpr (3 * stage_bytes <= 160 * 1024) {
    if (stages >= 3) {
      hipLaunchKernelGGL((gemm_planes_kernel<PA, PB, BK, WM, WN, 3, MI>), grid, block, 0, s, p);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_planes_kernel<PA, PB, BK, WM, WN, 2, MI>), grid, block, 0, s, p);
  return hipGetLastError();
  }
}

// tile variants: 0 = 128x128 (4 waves), 1 = 128x256 (8 waves), 2 = 256x128 (8 waves),
// 3 = 64x128 (2 waves), 4 = 64x128 (4 waves of 32 x 64: twice the waves per output),
// 5 = 128x128 (8 waves of 32 x 64)
template <int PA, int PB, int BK>
static hipError_t launch_variant_bk(int v, const PlaneGemmParams& p, int stages, hipStream_t s) {
  switch (v) {
    case 0: return launch_gemm<PA, PB, BK, 2, 2>(p, stages, s);
    case 1: return launch_gemm<PA, PB, BK, 2, 4>(p, stages, s);
    case 2: return launch_gemm<PA, PB, BK, 4, 2>(p, stages, s);
    case 4: return launch_gemm<PA, PB, BK, 2, 2, 2>(p, stages, s);   // 64 x 128, 4 waves
    case 5: return launch_gemm<PA, PB, BK, 4, 2, 2>(p, stages, s);   // 128 x 128, 8 waves
    default: return launch_gemm<PA, PB, BK, 1, 2>(p, stages, s);
  }
}

// k-step depth: 64 (two MFMA k-steps per LDS stage and barrier: the second step's
// fragment reads overlap the first step's MFMAs) where it fits and divides Kd, else 32
template <int PA, int PB>
static hipError_t launch_variant(int v, const PlaneGemmParams& p, int stages, int bk,
                                 hipStream_t s) {
  if (bk >= 64 && p.Kd % 64 == 0) return launch_variant_bk<PA, PB, 64>(v, p, stages, s);
  return launch_variant_bk<PA, PB, 32>(v, p, stages, s);
}

}  // namespace cnmf

// k granularity the caller pads the planes to (a multiple of every k-step depth)
extern "C" int cnmf_gemm_planes_bk(int pb) { return 64; }

// Tile tables: rows of (M-tile, N-tile) per variant, for the host heuristics.
extern "C" int cnmf_gemm_planes_tile(int v, int which) {
  static const int tm[6] = {128, 128, 256, 64, 64, 128};
  static const int tn[6] = {128, 256, 128, 128, 128, 128};
  return (v < 0 || v > 5) ? 0 : (which == 0 ? tm[v] : tn[v]);
}

extern "C" hipError_t cnmf_gemm_planes(const unsigned short* A, long long lda, long long a_plane,
                                       int a_rows, const unsigned short* B, long long ldb,
                                       long long b_plane, int b_rows, float* C, long long ldc,
                                       const float* col_scale, int M, int N, int Kd, int pa,
                                       int pb, int accumulate, int variant, int ksplit,
                                       float* slab, int stages, int kstep, int raw,
                                       const int* gate, hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (raw && !slab) return hipErrorInvalidValue;
  const int bk = 32;   // smallest k-step depth: Kd must be a multiple of it
  if (pa < 2 || pa > 3 || pb < 1 || pb > 3 || Kd <= 0 || Kd % bk || lda % 8 || ldb % 8 ||
      a_plane % 8 || b_plane % 8 || a_rows < 1 || b_rows < 1 || variant < 0 || variant > 5 ||
      ksplit < 1 || ksplit > Kd / (kstep >= 64 && Kd % 64 == 0 ? 64 : bk) ||
      (ksplit > 1 && !slab))
    return hipErrorInvalidValue;
  cnmf::PlaneGemmParams p;
  p.A = A; p.lda = lda; p.a_plane = a_plane; p.a_rows = a_rows;
  p.B = B; p.ldb = ldb; p.b_plane = b_plane; p.b_rows = b_rows;
  p.C = C; p.ldc = ldc; p.col_scale = col_scale;
  p.M = M; p.N = N; p.Kd = Kd; p.accumulate = accumulate;
  p.ksplit = ksplit; p.slab = slab; p.raw = raw ? 1 : 0; p.gate = gate;
  hipError_t e;
  switch (pa * 4 + pb) {
    case 9: e = cnmf::launch_variant<2, 1>(variant, p, stages, kstep, stream); break;
    case 10: e = cnmf::launch_variant<2, 2>(variant, p, stages, kstep, stream); break;
    case 11: e = cnmf::launch_variant<2, 3>(variant, p, stages, kstep, stream); break;
    case 13: e = cnmf::launch_variant<3, 1>(variant, p, stages, kstep, stream); break;
    case 14: e = cnmf::launch_variant<3, 2>(variant, p, stages, kstep, stream); break;
    default: e = cnmf::launch_variant<3, 3>(variant, p, stages, kstep, stream); break;
  }
  if (e != hipSuccess || ksplit == 1 || raw) return e;
  const long long total = (long long)M * N;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(cnmf::gemm_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, slab,
                     ksplit, M, N, C, ldc, col_scale, accumulate, gate);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_split_planes(const float* S, long long lds, int rows, int cols,
                                        int cols_pad, const float* col_mul, unsigned short* P,
                                        long long ldp, long long plane, int nplanes,
                                        hipStream_t stream) {
  if (rows <= 0 || cols_pad <= 0) return hipSuccess;
  if (cols_pad % 4 || ldp % 4 || cols > cols_pad || nplanes < 1 || nplanes > 3)
    return hipErrorInvalidValue;
  const long long total = (long long)rows * (cols_pad / 4);
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(cnmf::split_planes_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, S,
                     lds, rows, cols, cols_pad, col_mul, P, ldp, plane, nplanes);
  return hipGetLastError();
}
