// KL-divergence MU over a CSR matrix (gfx950 / CDNA4), replicate-batched: the sparse
// counterpart of beta_planes.hip for X below ~30 % density (HVG count matrices are
// typically 5-30 % non-zero).  KL is the one beta-divergence whose MU statistics only
// touch the non-zeros of X: with Q = X / P, num = S Q vanishes wherever x = 0, the
// denominator S 1 is a row sum of S, and D_KL(X | P) = sum_nz x log(x / p) - sum x +
// sum_k (sum F_k)(sum S_k).  So work and bytes scale with nnz instead of the dense
// element count (sklearn/decomposition/_nmf.py:526-728 computes the same MU step densely;
// SURVEY.md §2.4 G6, docs/ARCHITECTURE.md "Sparse KL").
//
// Layout: one 16-lane DPP row per fixed-axis column (a cell on the usage side H, a gene on
// the spectra side W), 16 columns per workgroup in flight.  The row walks its column's
// CSR entries 64 at a time (4 per lane, next batch's indices prefetched); every lane gathers the streamed operand's row S^T[j] (K
// floats, zero-padded to a multiple of 4, float4 loads, L2-resident: the replicates of
// one XCD share its L2 through the XCD-aware block map), forms p = eps + S^T[j] . f
// exactly in fp32 (v_pk_fma_f32 pairs: no MFMAs here, so packed VALU is the full-rate
// path), q = x / p, and accumulates q S^T[j]; four DPP adds (quad_perm, row_half_mirror,
// row_mirror) reduce the K sums over the row.  Unlike the dense kernel there is no shared
// panel, so the usage side runs all `nsteps` MU steps of a column back to back with the
// usages in registers.  The block-objective stopping rule is the dense kernel's (last
// workgroup of the replicate to arrive decides, cdna_hip_programming.md G16).
#include <hip/hip_runtime.h>

#include "common.h"

namespace cnmf {

typedef float sk_f2 __attribute__((ext_vector_type(2)));

constexpr int kSkThreads = 256;                 // global-gather variant
constexpr int kSkThreadsL = 512;                // LDS variant (one workgroup per CU)
constexpr int kSkRow = 16;                      // lanes per fixed column (one DPP row)
constexpr int kSkCols = kSkThreads / kSkRow;    // columns in flight per workgroup
constexpr int kSkLdsBytes = 128 * 1024;         // LDS budget for the staged S^T rows

struct SkParams {
  const int* rowptr;   // (Lf + 1): fixed column i owns entries [rowptr[i], rowptr[i+1])
  const int* col;      // streamed index of each entry
  const float* val;    // x of each entry
  const float* ST;     // streamed operand, transposed: replicate r, row l at ST + r*st_rs + l*K4
  long long st_rs;
  float* F;            // fixed operand (R, K, Lf): F + r*f_rs + k*ldf + i
  long long f_rs, ldf;
  int K, K4, Lf, Ls, R;
  int cols_per_wg, n_groups;
  float eps;
  float* num;          // side W: (R, K, Lf)
  int nsteps, loss_entry, loss_exit;
  const float* den_vec;  // (R, K) row sums of S
  float l1, l2, tol;
  int conv_mode;
  double* hstate;      // (R, 2)
  double* part;        // (R, n_groups, 4)
  int* counter;        // (R)
  int* act;            // (R)
  int* iters;          // (R)
  const int* active;   // (R) gate
  double* loss;        // loss-only launches: (R, n_groups)
  double xsum;
};

template <int CTRL>
__device__ __forceinline__ float sk_dpp(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// sum over the 16 lanes of a DPP row; every lane of the row receives it
__device__ __forceinline__ float sk_row_sum(float v) {
  v += sk_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += sk_dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += sk_dpp<0x141>(v);  // row_half_mirror
  v += sk_dpp<0x140>(v);  // row_mirror
  return v;
}

// LDS: the replicate's S^T rows [0, Ls) are staged in LDS first (gathers from LDS instead
// of L2: 48 B per non-zero at K = 10 made the L2-gather variant bandwidth-bound), 512
// threads so that one workgroup per CU still keeps two waves per SIMD
template <int NQ, bool UPD, bool LDS>
__global__ void __launch_bounds__(LDS ? kSkThreadsL : kSkThreads) sk_kernel(SkParams p) {
  constexpr int K4 = 4 * NQ;
  constexpr int NTH = LDS ? kSkThreadsL : kSkThreads;
  constexpr int NCOL = NTH / kSkRow;
  constexpr int kSkU = 4;   // entries per lane per batch (independent chains for latency)
  __shared__ double sred[4 * (NTH / 64)];
  __shared__ int s_last;
  extern __shared__ __attribute__((aligned(16))) float sk_lds[];
  // XCD-aware map: replicate r runs on XCD r % 8 (all of its workgroups), so its S^T
  // rows are gathered from one L2
  const int b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int RX = (p.R + 7) >> 3;
  const int rep = (local % RX) * 8 + xcd;
  const int grp = local / RX;
  if (rep >= p.R || grp >= p.n_groups) return;
  if (p.active && p.active[rep] == 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rl = tid & (kSkRow - 1), rc = tid / kSkRow;
  const int K = p.K;
  const float* __restrict__ ST = p.ST + (long long)rep * p.st_rs;
  if (LDS) {
    const float4* src = reinterpret_cast<const float4*>(ST);
    float4* dst = reinterpret_cast<float4*>(sk_lds);
    const int n4 = p.Ls * NQ;
    for (int i = tid; i < n4; i += NTH) dst[i] = src[i];
    __syncthreads();
    ST = sk_lds;
  }
  float* __restrict__ F = p.F + (long long)rep * p.f_rs;
  const float* dv = p.den_vec ? p.den_vec + (long long)rep * K : nullptr;
  float den[K4];
#pragma unroll
  for (int k = 0; k < K4; ++k) den[k] = (dv && k < K) ? dv[k] : 0.f;

  const bool exit_in_last = p.nsteps >= 2;
  const int n_it = UPD ? p.nsteps + ((p.loss_exit && !exit_in_last) || p.nsteps == 0 ? 1 : 0)
                       : 1;
  double f_entry = 0.0, f_exit = 0.0;
  float d2 = 0.f, o2 = 0.f;
  const int c0 = grp * p.cols_per_wg;
  const int c1 = min(p.Lf, c0 + p.cols_per_wg);
  for (int c = c0 + rc; c < c1; c += NCOL) {
    float h[K4];
#pragma unroll
    for (int k = 0; k < K4; ++k) h[k] = k < K ? F[(long long)k * p.ldf + c] : 0.f;
    sk_f2 h2[K4 / 2];
    const int beg = p.rowptr[c], end = p.rowptr[c + 1];
    const int trips = (end - beg + kSkRow * kSkU - 1) / (kSkRow * kSkU);
    for (int it = 0; it < n_it; ++it) {
      const bool want_num = !UPD || it < p.nsteps;
      const bool is_exit = it == (exit_in_last ? p.nsteps - 1 : p.nsteps);
      const bool is_entry = it == 0 && p.loss_entry && p.nsteps > 0;
      const bool want_loss = UPD && (is_entry || (is_exit && (p.loss_exit || p.nsteps == 0)));
#pragma unroll
      for (int k = 0; k < K4 / 2; ++k) h2[k] = sk_f2{h[2 * k], h[2 * k + 1]};
      // float2 pairs throughout: v_pk_fma_f32 (no MFMAs in this kernel, so the packed VALU
      // is the full-rate path)
      sk_f2 acc2[K4 / 2];
#pragma unroll
      for (int k = 0; k < K4 / 2; ++k) acc2[k] = sk_f2{0.f, 0.f};
      float acc[K4];
      float ls = 0.f;
      // batches of kSkU entries per lane: the index / value loads of batch t + 1 are in
      // flight while batch t computes, and the kSkU * NQ row gathers of a batch are
      // issued together (one L2 round trip per batch, not per entry)
      int jn[kSkU];
      float xn[kSkU];
      auto load_jx = [&](int t) {
#pragma unroll
        for (int u = 0; u < kSkU; ++u) {
          // unconditional loads (clamped into the column: trips > 0 means end > beg), so
          // the compiler counts them and batch t waits only for its own row gathers
          const int e = beg + (t * kSkU + u) * kSkRow + rl;
          const int ec = min(e, end - 1);
          jn[u] = p.col[ec];
          xn[u] = p.val[ec];     // masked where used (a select here would wait for it)
        }
      };
      if (trips > 0) load_jx(0);
      for (int t = 0; t < trips; ++t) {
        float x[kSkU];
        sk_f2 s[kSkU][K4 / 2];
#pragma unroll
        for (int u = 0; u < kSkU; ++u) {
          x[u] = beg + (t * kSkU + u) * kSkRow + rl < end ? xn[u] : 0.f;
          const float4* s4 = reinterpret_cast<const float4*>(ST + (long long)jn[u] * K4);
#pragma unroll
          for (int v = 0; v < NQ; ++v) {
            const float4 w = s4[v];
            s[u][2 * v] = sk_f2{w.x, w.y};
            s[u][2 * v + 1] = sk_f2{w.z, w.w};
          }
        }
        load_jx(min(t + 1, trips - 1));   // unconditional: the waits below stay exact
#pragma unroll
        for (int u = 0; u < kSkU; ++u) {
          sk_f2 p2 = sk_f2{p.eps, 0.f};
#pragma unroll
          for (int k = 0; k < K4 / 2; ++k) p2 = __builtin_elementwise_fma(s[u][k], h2[k], p2);
          const float q = x[u] * __builtin_amdgcn_rcpf(p2.x + p2.y);
          if (want_loss && x[u] > 0.f) ls += x[u] * __builtin_amdgcn_logf(q);
          if (want_num) {
            const sk_f2 q2 = sk_f2{q, q};
#pragma unroll
            for (int k = 0; k < K4 / 2; ++k) acc2[k] = __builtin_elementwise_fma(q2, s[u][k], acc2[k]);
          }
        }
      }
      if (want_loss) {
        // x ln(x/p) summed over the row's entries, plus sum_k h_k (sum_l S_kl) once per
        // column (the objective's linear part; -sum x is subtracted per replicate)
        double l = 0.69314718055994530942 * (double)ls;
        if (rl == 0) {
          float hp = 0.f;
#pragma unroll
          for (int k = 0; k < K4; ++k) hp = fmaf(h[k], den[k], hp);
          l += (double)hp;
        }
        if (is_entry) f_entry += l;
        if (is_exit) f_exit += l;
      }
      if (want_num) {
#pragma unroll
        for (int k = 0; k < K4 / 2; ++k) {
          acc[2 * k] = sk_row_sum(acc2[k].x);
          acc[2 * k + 1] = sk_row_sum(acc2[k].y);
        }
        if (UPD) {
          const bool last = it + 1 == p.nsteps;
#pragma unroll
          for (int k = 0; k < K4; ++k) {
            if (k < K) {
              float dn = den[k] + p.l1 + p.l2 * h[k];
              if (dn == 0.f) dn = p.eps;
              const float hn = h[k] * (acc[k] / dn);
              if (last && rl == 0) {
                d2 = fmaf(hn - h[k], hn - h[k], d2);
                o2 = fmaf(h[k], h[k], o2);
              }
              h[k] = hn;
            }
          }
        } else {
          float* o = p.num + (long long)rep * K * p.Lf + c;
#pragma unroll
          for (int k = 0; k < K4; ++k)
            if (k < K && rl == (k & (kSkRow - 1))) o[(long long)k * p.Lf] = acc[k];
        }
      }
    }
    if (UPD && p.nsteps > 0) {
#pragma unroll
      for (int k = 0; k < K4; ++k)
        if (k < K && rl == (k & (kSkRow - 1))) F[(long long)k * p.ldf + c] = h[k];
    }
  }
  if (!UPD) return;

  // workgroup partials -> the replicate's stopping rule (as beta_planes.hip bp_kernel)
  {
    const double v0 = wave_sum((double)d2), v1 = wave_sum((double)o2);
    const double v2 = wave_sum(f_entry), v3 = wave_sum(f_exit);
    if (lane == 0) {
      sred[wave * 4 + 0] = v0;
      sred[wave * 4 + 1] = v1;
      sred[wave * 4 + 2] = v2;
      sred[wave * 4 + 3] = v3;
    }
    __syncthreads();
  }
  constexpr int kW = NTH / 64;
  if (p.loss && tid == 0) {
    double tot = 0.0;
    for (int w = 0; w < kW; ++w) tot += sred[w * 4 + 3];
    p.loss[(long long)rep * p.n_groups + grp] = tot;
  }
  if (!p.part) return;
  if (tid == 0) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int w = 0; w < kW; ++w)
      for (int v = 0; v < 4; ++v) acc[v] += sred[w * 4 + v];
    double* pp = p.part + ((long long)rep * p.n_groups + grp) * 4;
    for (int v = 0; v < 4; ++v) pp[v] = acc[v];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(p.counter + rep, 1, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    s_last = (prev == p.n_groups - 1);
  }
  __syncthreads();
  if (s_last && tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    double tot[4] = {0.0, 0.0, 0.0, 0.0};
    const double* pr = p.part + (long long)rep * p.n_groups * 4;
    for (int g2 = 0; g2 < p.n_groups; ++g2)
      for (int v = 0; v < 4; ++v)
        tot[v] += __hip_atomic_load(pr + 4 * g2 + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tot[2] -= p.xsum;
    tot[3] -= p.xsum;
    if (p.conv_mode == 1) {
      double* hs = p.hstate + 2 * (long long)rep;
      const double f_prev = p.loss_entry ? tot[2] : hs[0];
      if ((p.loss_entry || hs[1] > 0.0) && fabs(f_prev - tot[3]) <= (double)p.tol * fabs(f_prev))
        p.act[rep] = 0;
      hs[0] = tot[3];
      hs[1] = hs[1] + 1.0;
    } else if (p.nsteps > 0) {
      const double rel = sqrt(tot[0]) / (sqrt(tot[1]) + (double)p.eps);
      if (rel < (double)p.tol) p.act[rep] = 0;
    }
    if (p.iters) p.iters[rep] += p.nsteps;
    p.counter[rep] = 0;
  }
}

template <int NQ, bool UPD, bool LDS>
hipError_t sk_launch(const SkParams& p, hipStream_t s) {
  const int RX = (p.R + 7) / 8;
  const dim3 grid((unsigned)(8 * RX * p.n_groups));
  const size_t lds = LDS ? (size_t)p.Ls * 16 * NQ : 0;
  if (LDS) {
    static bool attr_done = false;
    if (!attr_done) {
      const hipError_t e = hipFuncSetAttribute(
          reinterpret_cast<const void*>(&sk_kernel<NQ, UPD, LDS>),
          hipFuncAttributeMaxDynamicSharedMemorySize, kSkLdsBytes);
      if (e != hipSuccess) return e;
      attr_done = true;
    }
  }
  hipLaunchKernelGGL((sk_kernel<NQ, UPD, LDS>), grid, dim3(LDS ? kSkThreadsL : kSkThreads), lds,
                     s, p);
  return hipGetLastError();
}

template <bool UPD, bool LDS>
hipError_t sk_launch_k(const SkParams& p, hipStream_t s) {
  switch (p.K4 / 4) {
    case 1: return sk_launch<1, UPD, LDS>(p, s);
    case 2: return sk_launch<2, UPD, LDS>(p, s);
    case 3: return sk_launch<3, UPD, LDS>(p, s);
    case 4: return sk_launch<4, UPD, LDS>(p, s);
    case 5: return sk_launch<5, UPD, LDS>(p, s);
    case 6: return sk_launch<6, UPD, LDS>(p, s);
    case 7: return sk_launch<7, UPD, LDS>(p, s);
    case 8: return sk_launch<8, UPD, LDS>(p, s);
    default: return hipErrorInvalidValue;
  }
}

template <bool UPD>
hipError_t sk_launch_u(const SkParams& p, hipStream_t s) {
  return (long long)p.Ls * p.K4 * 4 <= kSkLdsBytes ? sk_launch_k<UPD, true>(p, s)
                                                    : sk_launch_k<UPD, false>(p, s);
}

}  // namespace cnmf

// padded row length of the transposed streamed operand
extern "C" int cnmf_sk_k4(int K) { return (K + 3) / 4 * 4; }

// whether a launch stages S^T (Ls rows) in LDS
extern "C" int cnmf_sk_lds(int Ls, int K) {
  return (long long)Ls * cnmf_sk_k4(K) * 4 <= cnmf::kSkLdsBytes ? 1 : 0;
}

// fixed columns per workgroup: enough workgroups to fill the chip several times over (LDS
// variant: 128, so the staging read is ~1/50 of a usage block's gathers)
extern "C" int cnmf_sk_cols_per_wg(int Lf, int R, int Ls, int K) {
  if (cnmf_sk_lds(Ls, K)) {
    int cols = 128;
    while (cols > cnmf::kSkThreadsL / cnmf::kSkRow && (long long)R * ((Lf + cols - 1) / cols) < 1024)
      cols /= 2;
    return cols;
  }
  int cols = 64;
  while (cols > cnmf::kSkCols && (long long)R * ((Lf + cols - 1) / cols) < 4096) cols /= 2;
  return cols;
}

// side 0 (H: fused nsteps MU steps of F in place + stopping rule; nsteps 0: loss only into
// `loss`), side 1 (W: num = S Q into `num`)
extern "C" hipError_t cnmf_sk_run(
    int side, const int* rowptr, const int* col, const float* val, const float* ST,
    long long st_rs, float* F, long long f_rs, long long ldf, int K, int Lf, int Ls, int R,
    float eps,
    float* num, int nsteps, int loss_entry, int loss_exit, const float* den_vec, float l1,
    float l2, float tol, int conv_mode, double* hstate, double* part, int* counter, int* act,
    int* iters, const int* active, double* loss, double xsum, hipStream_t stream) {
  if (R <= 0 || Lf <= 0) return hipSuccess;
  if (K < 1 || K > 32 || (side != 0 && side != 1) || rowptr == nullptr || ST == nullptr ||
      (reinterpret_cast<uintptr_t>(ST) & 15) != 0 || st_rs % 4 != 0)
    return hipErrorInvalidValue;
  cnmf::SkParams p;
  p.rowptr = rowptr; p.col = col; p.val = val;
  p.ST = ST; p.st_rs = st_rs;
  p.F = F; p.f_rs = f_rs; p.ldf = ldf;
  if (Ls <= 0 || st_rs < (long long)Ls * cnmf_sk_k4(K)) return hipErrorInvalidValue;
  p.K = K; p.K4 = cnmf_sk_k4(K); p.Lf = Lf; p.Ls = Ls; p.R = R;
  p.cols_per_wg = cnmf_sk_cols_per_wg(Lf, R, Ls, K);
  p.n_groups = (Lf + p.cols_per_wg - 1) / p.cols_per_wg;
  p.eps = eps; p.num = num;
  p.nsteps = nsteps; p.loss_entry = loss_entry; p.loss_exit = loss_exit;
  p.den_vec = den_vec; p.l1 = l1; p.l2 = l2; p.tol = tol; p.conv_mode = conv_mode;
  p.hstate = hstate; p.part = part; p.counter = counter; p.act = act; p.iters = iters;
  p.active = active; p.loss = loss; p.xsum = xsum;
  if (side == 1) {
    if (num == nullptr) return hipErrorInvalidValue;
    return cnmf::sk_launch_u<false>(p, stream);
  }
  if (nsteps < 0 || den_vec == nullptr || (part != nullptr && (counter == nullptr || act == nullptr)) ||
      (part != nullptr && conv_mode == 1 && hstate == nullptr) ||
      (nsteps == 0 && loss == nullptr && part == nullptr))
    return hipErrorInvalidValue;
  return cnmf::sk_launch_u<true>(p, stream);
}

extern "C" int cnmf_sk_groups(int Lf, int R, int Ls, int K) {
  const int c = cnmf_sk_cols_per_wg(Lf, R, Ls, K);
  return (Lf + c - 1) / c;
}
