// Fused beta-divergence MU contraction on MFMA (gfx950 / CDNA4), replicate-batched.
//
// For replicate r with factors HT_r (K x N, usages transposed) and W_r (K x G):
//   P   = max(HT_r^T W_r, eps)                       (N x G, never materialised)
//   Q   = X * P^(beta-2)      D = P^(beta-1)           (elementwise, in registers)
//   side H: num[r] = W_r Q^T  (K x N)   den[r] = W_r D^T   (beta != 1)
//   side W: num[r] = HT_r Q   (K x G)   den[r] = HT_r D    (beta != 1)
//   loss (side H, optional): per-workgroup partial sums of D_beta(X || P)
// This is the G6/G7 row of SURVEY.md §2.4: nmf-torch's KL/beta MU (the sklearn math at
// sklearn/decomposition/_nmf.py:526-728, loss :85-189) does h@W -> x/(hW) -> (.)@W^T as
// three eager ops with an N x G intermediate; here each 16x16 tile of P lives in four
// accumulator registers between two MFMA contractions.
//
// Tile algebra (v_mfma_f32_16x16x4_f32, lane l, q = l>>4, m = l&15):
//   A operand: A[row m][k q]   B operand: B[k q][col m]   C/D: row 4q+i, col m (reg i)
// Side H, per (16 genes x 16 cells) tile:
//   P^T[g][n] = sum_k W[k][g] HT[k][n]  (A = W^T from LDS, B = HT held in registers)
//   num[k][n] += sum_g W[k][g] Q^T[g][n]: step i feeds acc register i as B (its k index is
//   gene 4q+i, a permutation of the gene order that the A operand W[m][4q+i] matches), so
//   the accumulator becomes the next MFMA's operand without any lane movement.
// Side W is the mirror image (P[n][g] with cells on the rows, contraction over cells).
//
// Grid: 1-D, XCD-aware.  Workgroup b runs on XCD b%8; the (strip, replicate) units are
// laid out so that every replicate of one X strip lands on the same XCD back to back --
// X is read from HBM about once per call and the replicates hit it in that XCD's L2.
#include <hip/hip_runtime.h>

#include "common.h"

namespace cnmf {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBetaThreads = 256;  // 4 waves; each wave owns a 16-wide strip
constexpr int kBetaChunk = 256;    // reduction-axis chunk staged in LDS per iteration

enum BetaMode { kKL = 0, kIS = 1, kGeneral = 2 };

struct BetaParams {
  const float* X;       // N x G (row stride ldx)
  long long ldx;
  const float* HT;      // replicate r: HT + r*h_rs, row k stride ldh
  long long h_rs, ldh;
  const float* W;       // replicate r: W + r*w_rs, row k stride ldw
  long long w_rs, ldw;
  int N, G, K, R;
  float beta, eps;
  float* num;           // side H: (R, K, N) contiguous; side W: (splits, R, K, G)
  float* den;           // same layout, beta != 1 only (else nullptr)
  double* loss;         // side H only: (R, n_strips) partials or nullptr
  const int* active;    // optional per-replicate flag (0 -> skip)
  int n_strips;         // strips of 64 along the output axis
  int splits;           // side W: reduction-axis splits (grid units = strips*splits)
  // Fused in-place MU update of HT (side H, upd != 0) instead of writing num/den:
  //   h <- h * ((num / max0(den + l1 + l2 h)) ^ gamma), den = den_vec[r][k] for KL
  // plus, when part != nullptr, the usages' relative change for the inner stopping rule:
  // per-workgroup (|dh|^2, |h|^2) partials; the last workgroup of a replicate (arrival
  // counter, self-resetting) reduces them in strip order and clears act[r] when
  // |dh| / (|h| + eps) < tol, and adds one to iters[r].
  int upd;
  float* HTw;           // writable alias of HT
  const float* den_vec; // (R, K) rowsums of W for KL
  float l1, l2, gamma, tol;
  float* part;          // (R, n_strips, 3): |dh|^2, |h|^2, chunk loss
  int* counter;         // (R), zero before the first launch, left zero after every launch
  int* act;             // (R) active flags (the `active` input is usually this array)
  int* iters;           // (R)
  // Inner stopping rule.  conv_mode 0: relative iterate change |dh|/(|h|+eps) < tol after
  // every step.  conv_mode 1 (block objective, as the Frobenius solve's conv_mode 1): the
  // chunk's beta-divergence D(x | h W) -- computed from the same P tiles the step uses --
  // is recorded every `check_every` steps in hstate[r] = {f_prev, steps}; a replicate
  // stops after the step at which |f_prev - f| <= tol |f_prev|.  The host zeroes hstate
  // before each chunk solve.
  int conv_mode, check_every;
  double* hstate;       // (R, 2)
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int MODE>
__device__ __forceinline__ void beta_terms(float x, float p, float beta, float& q, float& d) {
  if (MODE == kKL) {
    q = x * __builtin_amdgcn_rcpf(p);
    d = 1.f;
  } else if (MODE == kIS) {
    const float r = __builtin_amdgcn_rcpf(p);
    d = r;
    q = x * r * r;
  } else {
    const float lp = __builtin_amdgcn_logf(p);  // log2
    d = __builtin_amdgcn_exp2f((beta - 1.f) * lp);
    q = x * __builtin_amdgcn_exp2f((beta - 2.f) * lp);
  }
}

template <int MODE>
__device__ __forceinline__ float beta_loss_term(float x, float p, float beta, float eps) {
  if (MODE == kKL) {
    const float t = x > 0.f ? x * __logf(x / p) : 0.f;
    return t - x + p;
  } else if (MODE == kIS) {
    const float d = fmaxf(x / p, eps);
    return d - __logf(d) - 1.f;
  } else {
    return (__powf(x, beta) + (beta - 1.f) * __powf(p, beta) - beta * x * __powf(p, beta - 1.f)) /
           (beta * (beta - 1.f));
  }
}

// Map the 1-D workgroup id onto (unit, replicate) so that the replicates sharing a unit
// (an X strip) run on the same XCD one after another.  Returns false for padding.
__device__ __forceinline__ bool beta_unit(int n_units, int R, int& unit, int& rep) {
  const int b = blockIdx.x;
  const int xcd = b & 7;
  const int local = b >> 3;
  rep = local % R;
  unit = (local / R) * 8 + xcd;
  return unit < n_units;
}

// ---------------------------------------------------------------------------------- side H
// Workgroup: replicate `rep`, cells [n0, n0+64) (wave w: n0+16w .. +15); loop over genes.
template <int KP4, int MODE>
__global__ void __launch_bounds__(kBetaThreads) beta_h_kernel(BetaParams p) {
  constexpr int T = (KP4 * 4 + 15) / 16;   // 16-row output tiles
  constexpr int LD = 16 * T + 4;           // LDS row stride (floats): conflict-free maps
  __shared__ float sW[kBetaChunk * LD];    // W chunk, transposed: sW[g][k]
  __shared__ double sred[kBetaThreads / 64];

  int strip, rep;
  if (!beta_unit(p.n_strips, p.R, strip, rep)) return;
  if (p.active && p.active[rep] == 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, m = lane & 15;
  const int n = strip * 64 + wave * 16 + m;          // this lane's cell (B/C column)
  const bool n_ok = n < p.N;
  const float* __restrict__ W = p.W + (long long)rep * p.w_rs;
  const float* __restrict__ HT = p.HT + (long long)rep * p.h_rs;

  // B operand of the P product: HT[k = q + 4s][n], zero-padded beyond K / N
  float hreg[KP4];
#pragma unroll
  for (int s = 0; s < KP4; ++s) {
    const int k = q + 4 * s;
    hreg[s] = (n_ok && k < p.K) ? HT[(long long)k * p.ldh + n] : 0.f;
  }
  f32x4 num[T], den[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    num[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    den[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool want_num = p.num != nullptr || p.upd;
  const bool want_loss = p.loss != nullptr || (p.upd && p.part && p.conv_mode == 1);
  float lsum = 0.f;
  const float* __restrict__ xrow = p.X + (long long)(n_ok ? n : 0) * p.ldx;

  for (int g0 = 0; g0 < p.G; g0 += kBetaChunk) {
    const int gc = min(kBetaChunk, p.G - g0);
    __syncthreads();
    for (int e = threadIdx.x; e < 16 * T * kBetaChunk; e += kBetaThreads) {
      const int k = e / kBetaChunk, g = e % kBetaChunk;
      sW[g * LD + k] = (k < p.K && g < gc) ? W[(long long)k * p.ldw + g0 + g] : 0.f;
    }
    __syncthreads();
    const int nsteps = (gc + 15) >> 4;
#pragma unroll 2
    for (int j = 0; j < nsteps; ++j) {
      const int gl = j * 16;
      f32x4 P = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KP4; ++s) P = mfma4(sW[(gl + m) * LD + q + 4 * s], hreg[s], P);
      // X[n][g0+gl+4q .. +3]
      const int gx = g0 + gl + 4 * q;
      float xv[4];
      if (n_ok && gx + 3 < p.G && (p.ldx & 3) == 0 && ((uintptr_t)p.X & 15) == 0) {
        const float4 v = *reinterpret_cast<const float4*>(xrow + gx);
        xv[0] = v.x; xv[1] = v.y; xv[2] = v.z; xv[3] = v.w;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) xv[i] = (n_ok && gx + i < p.G) ? xrow[gx + i] : 0.f;
      }
      float qv[4], dv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = n_ok && gx + i < p.G;
        const float pc = fmaxf(P[i], p.eps);
        beta_terms<MODE>(xv[i], pc, p.beta, qv[i], dv[i]);
        qv[i] = ok ? qv[i] : 0.f;
        dv[i] = ok ? dv[i] : 0.f;
        if (want_loss && ok) lsum += beta_loss_term<MODE>(xv[i], pc, p.beta, p.eps);
      }
      if (want_num) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int t = 0; t < T; ++t) {
            const float a = sW[(gl + 4 * q + i) * LD + m + 16 * t];
            num[t] = mfma4(a, qv[i], num[t]);
            if (MODE != kKL) den[t] = mfma4(a, dv[i], den[t]);
          }
        }
      }
    }
  }
  if (p.upd) {
    float d2 = 0.f, o2 = 0.f;
    if (n_ok) {
      float* hcol = p.HTw + (long long)rep * p.h_rs + n;
#pragma unroll
      for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 16 * t + 4 * q + i;
          if (k < p.K) {
            const float h = hcol[(long long)k * p.ldh];
            float dn = (MODE == kKL) ? p.den_vec[(long long)rep * p.K + k] : den[t][i];
            dn = dn + p.l1 + p.l2 * h;
            if (dn == 0.f) dn = p.eps;
            float delta = num[t][i] / dn;
            if (p.gamma != 1.f) delta = __powf(delta, p.gamma);
            const float hn = h * delta;
            hcol[(long long)k * p.ldh] = hn;
            d2 = fmaf(hn - h, hn - h, d2);
            o2 = fmaf(h, h, o2);
          }
        }
      }
    }
    if (p.part) {
      __shared__ float sp[2 * (kBetaThreads / 64)];
      __shared__ int s_last;
      __shared__ double sl[kBetaThreads / 64];
      block_sum2(d2, o2, sp);
      double lt = 0.0;
      if (p.conv_mode == 1) {
        const double v = wave_sum((double)lsum);
        if (lane == 0) sl[wave] = v;
        __syncthreads();
        for (int w = 0; w < kBetaThreads / 64; ++w) lt += sl[w];
      }
      if (threadIdx.x == 0) {
        // publish (cdna_hip_programming.md G16): plain stores -> drain -> agent release ->
        // drain -> arrival counter
        float* pp = p.part + ((long long)rep * p.n_strips + strip) * 3;
        pp[0] = d2;
        pp[1] = o2;
        pp[2] = (float)lt;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int prev = __hip_atomic_fetch_add(p.counter + rep, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        s_last = (prev == p.n_strips - 1);
      }
      __syncthreads();
      if (s_last && threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        double td = 0.0, to = 0.0, tl = 0.0;
        const float* pr = p.part + (long long)rep * p.n_strips * 3;
        for (int s2 = 0; s2 < p.n_strips; ++s2) {
          td += __hip_atomic_load(pr + 3 * s2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          to += __hip_atomic_load(pr + 3 * s2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tl += __hip_atomic_load(pr + 3 * s2 + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (p.conv_mode == 1) {
          double* hs = p.hstate + 2 * (long long)rep;
          const int steps = (int)hs[1];
          const int every = p.check_every > 0 ? p.check_every : 1;
          if (steps % every == 0) {
            if (steps > 0 && fabs(hs[0] - tl) <= (double)p.tol * fabs(hs[0])) p.act[rep] = 0;
            hs[0] = tl;
          }
          hs[1] = (double)(steps + 1);
        } else {
          const double rel = sqrt(td) / (sqrt(to) + (double)p.eps);
          if (rel < (double)p.tol) p.act[rep] = 0;
        }
        if (p.iters) p.iters[rep] += 1;
        p.counter[rep] = 0;
      }
    }
  } else if (want_num && n_ok) {
    float* out = p.num + (long long)rep * p.K * p.N;
    float* dout = p.den ? p.den + (long long)rep * p.K * p.N : nullptr;
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 16 * t + 4 * q + i;
        if (k < p.K) {
          out[(long long)k * p.N + n] = num[t][i];
          if (MODE != kKL && dout) dout[(long long)k * p.N + n] = den[t][i];
        }
      }
    }
  }
  if (p.loss) {
    double v = wave_sum((double)lsum);
    if (lane == 0) sred[wave] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      double tot = 0.0;
      for (int w = 0; w < kBetaThreads / 64; ++w) tot += sred[w];
      p.loss[(long long)rep * p.n_strips + strip] = tot;
    }
  }
}

// ---------------------------------------------------------------------------------- side W
// Workgroup: replicate `rep`, genes [g0, g0+64) (wave w: 16 genes), cells of split z.
template <int KP4, int MODE>
__global__ void __launch_bounds__(kBetaThreads) beta_w_kernel(BetaParams p) {
  constexpr int T = (KP4 * 4 + 15) / 16;
  constexpr int LD = 16 * T + 4;
  __shared__ float sH[kBetaChunk * LD];    // HT chunk, transposed: sH[c][k]

  int unit, rep;
  if (!beta_unit(p.n_strips * p.splits, p.R, unit, rep)) return;
  if (p.active && p.active[rep] == 0) return;
  const int strip = unit % p.n_strips, split = unit / p.n_strips;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, m = lane & 15;
  const int g = strip * 64 + wave * 16 + m;           // this lane's gene (B/C column)
  const bool g_ok = g < p.G;
  const float* __restrict__ W = p.W + (long long)rep * p.w_rs;
  const float* __restrict__ HT = p.HT + (long long)rep * p.h_rs;
  const int per = (p.N + p.splits - 1) / p.splits;
  const int c_begin = split * per, c_end = min(p.N, c_begin + per);

  float wreg[KP4];  // B operand of P: W[k = q + 4s][g]
#pragma unroll
  for (int s = 0; s < KP4; ++s) {
    const int k = q + 4 * s;
    wreg[s] = (g_ok && k < p.K) ? W[(long long)k * p.ldw + g] : 0.f;
  }
  f32x4 num[T], den[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    num[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    den[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float* __restrict__ xcol = p.X + (g_ok ? g : 0);

  for (int c0 = c_begin; c0 < c_end; c0 += kBetaChunk) {
    const int cc = min(kBetaChunk, c_end - c0);
    __syncthreads();
    for (int e = threadIdx.x; e < 16 * T * kBetaChunk; e += kBetaThreads) {
      const int k = e / kBetaChunk, c = e % kBetaChunk;
      sH[c * LD + k] = (k < p.K && c < cc) ? HT[(long long)k * p.ldh + c0 + c] : 0.f;
    }
    __syncthreads();
    const int nsteps = (cc + 15) >> 4;
#pragma unroll 2
    for (int j = 0; j < nsteps; ++j) {
      const int cl = j * 16;
      f32x4 P = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KP4; ++s) P = mfma4(sH[(cl + m) * LD + q + 4 * s], wreg[s], P);
      float qv[4], dv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = cl + 4 * q + i;                    // row of P held in register i
        const bool ok = g_ok && c < cc;
        const float xv = ok ? xcol[(long long)(c0 + c) * p.ldx] : 0.f;
        beta_terms<MODE>(xv, fmaxf(P[i], p.eps), p.beta, qv[i], dv[i]);
        qv[i] = ok ? qv[i] : 0.f;
        dv[i] = ok ? dv[i] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int t = 0; t < T; ++t) {
          const float a = sH[(cl + 4 * q + i) * LD + m + 16 * t];
          num[t] = mfma4(a, qv[i], num[t]);
          if (MODE != kKL) den[t] = mfma4(a, dv[i], den[t]);
        }
      }
    }
  }
  if (g_ok) {
    const long long base = ((long long)split * p.R + rep) * p.K * p.G;
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 16 * t + 4 * q + i;
        if (k < p.K) {
          p.num[base + (long long)k * p.G + g] = num[t][i];
          if (MODE != kKL && p.den) p.den[base + (long long)k * p.G + g] = den[t][i];
        }
      }
    }
  }
}


// ---------------------------------------------------------------------------------- W update
// One step of the online beta-MU spectra update with anchored sufficient statistics
// (models/nmf.py _online_beta).  Per element, with num/den the chunk's W-side MU
// statistics at the current W (summed over the contraction's split partials):
//   an = W^(1/gamma) num          (the chunk's majoriser, anchored at this W)
//   W' = ((An + an) / (Ad + den + l1 + l2 W))^gamma
// where An/Ad hold the anchored statistics of the chunks already visited this pass.
// an (and den, beta != 1) are written out so the caller can add the final anchor to
// An/Ad.  For KL den is the chunk's per-component usage sum (hsum, (R, K)).  The
// replicate's relative change |W' - W| / (|W| + eps) is reduced by the last-arriving
// workgroup, which clears act[r] below tol and counts the step in iters[r].
struct BetaWUpd {
  float* W;
  long long w_rs, ldw;
  const float* num;     // (splits, R, K, G) contiguous
  const float* den;     // same (beta != 1) or nullptr
  const float* hsum;    // (R, K) (beta == 1)
  const float* An;      // (R, K, G)
  const float* Ad;      // (R, K, G) or (R, K) for beta == 1
  float* an_out;        // (R, K, G)
  float* dn_out;        // (R, K, G) (beta != 1) or nullptr
  int R, K, G, splits, mode;
  float gamma, l1, l2, eps, tol;
  float* part;          // (R, nb, 2)
  int* counter;
  int* act;
  int* iters;
};

__global__ void __launch_bounds__(256) beta_w_update_kernel(BetaWUpd p) {
  const int rep = blockIdx.y;
  if (p.act[rep] == 0) return;
  const int nb = gridDim.x;
  const long long KG = (long long)p.K * p.G;
  const long long rstride = (long long)p.R * KG;
  float d2 = 0.f, o2 = 0.f;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < KG;
       e += (long long)nb * blockDim.x) {
    const int k = (int)(e / p.G), g = (int)(e - (long long)k * p.G);
    float* wp = p.W + rep * p.w_rs + k * p.ldw + g;
    const float w = *wp;
    const long long o = rep * KG + e;
    float nu = 0.f, dn = 0.f;
    for (int s = 0; s < p.splits; ++s) {
      nu += p.num[s * rstride + o];
      if (p.mode != kKL) dn += p.den[s * rstride + o];
    }
    if (p.mode == kKL) dn = p.hsum[rep * p.K + k];
    float wg;                                   // W^(1/gamma)
    if (p.gamma == 1.f) wg = w;
    else if (p.gamma == 0.5f) wg = w * w;
    else wg = __powf(w, 1.f / p.gamma);
    const float an = wg * nu;
    const float A = p.An[o] + an;
    float B = (p.mode == kKL ? p.Ad[rep * p.K + k] : p.Ad[o]) + dn + p.l1 + p.l2 * w;
    if (B == 0.f) B = p.eps;
    float wn = A / B;
    if (p.gamma == 0.5f) wn = sqrtf(wn);
    else if (p.gamma != 1.f) wn = __powf(wn, p.gamma);
    *wp = wn;
    p.an_out[o] = an;
    if (p.mode != kKL) p.dn_out[o] = dn;
    d2 = fmaf(wn - w, wn - w, d2);
    o2 = fmaf(w, w, o2);
  }
  __shared__ float sp[2 * 4];
  __shared__ int s_last;
  block_sum2(d2, o2, sp);
  if (threadIdx.x == 0) {
    float* pp = p.part + ((long long)rep * nb + blockIdx.x) * 2;
    pp[0] = d2;
    pp[1] = o2;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(p.counter + rep, 1, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    s_last = (prev == nb - 1);
  }
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    double td = 0.0, to = 0.0;
    const float* pr = p.part + (long long)rep * nb * 2;
    for (int b = 0; b < nb; ++b) {
      td += __hip_atomic_load(pr + 2 * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      to += __hip_atomic_load(pr + 2 * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (sqrt(td) / (sqrt(to) + (double)p.eps) < (double)p.tol) p.act[rep] = 0;
    if (p.iters) p.iters[rep] += 1;
    p.counter[rep] = 0;
  }
}

template <int KP4, int MODE>
hipError_t launch_beta(int side, const BetaParams& p, hipStream_t s) {
  const int units = side == 0 ? p.n_strips : p.n_strips * p.splits;
  const int per_xcd = (units + 7) / 8;
  const dim3 grid((unsigned)(per_xcd * p.R * 8));
  if (side == 0)
    hipLaunchKernelGGL((beta_h_kernel<KP4, MODE>), grid, dim3(kBetaThreads), 0, s, p);
  else
    hipLaunchKernelGGL((beta_w_kernel<KP4, MODE>), grid, dim3(kBetaThreads), 0, s, p);
  return hipGetLastError();
}

template <int MODE>
hipError_t launch_beta_mode(int side, const BetaParams& p, hipStream_t s) {
  switch ((p.K + 3) / 4) {
    case 1: return launch_beta<1, MODE>(side, p, s);
    case 2: return launch_beta<2, MODE>(side, p, s);
    case 3: return launch_beta<3, MODE>(side, p, s);
    case 4: return launch_beta<4, MODE>(side, p, s);
    case 5: return launch_beta<5, MODE>(side, p, s);
    case 6: return launch_beta<6, MODE>(side, p, s);
    case 7: return launch_beta<7, MODE>(side, p, s);
    case 8: return launch_beta<8, MODE>(side, p, s);
    // K > 32, padded to a multiple of 8 by the engine (models.nmf.native_rank)
    case 10: return launch_beta<10, MODE>(side, p, s);
    case 12: return launch_beta<12, MODE>(side, p, s);
    case 14: return launch_beta<14, MODE>(side, p, s);
    case 16: return launch_beta<16, MODE>(side, p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace cnmf

extern "C" int cnmf_beta_max_k() { return 64; }

// side 0 = H (num/den: (R,K,N), loss partials (R, ceil(N/64))),
// side 1 = W (num/den: (splits,R,K,G)).  mode: 0 KL, 1 IS, 2 general beta.
extern "C" hipError_t cnmf_beta_contract(int side, int mode, const float* X, long long ldx,
                                         const float* HT, long long h_rs, long long ldh,
                                         const float* W, long long w_rs, long long ldw, int N,
                                         int G, int K, int R, float beta, float eps, float* num,
                                         float* den, double* loss, const int* active,
                                         int splits, int upd, const float* den_vec, float l1,
                                         float l2, float gamma, float tol, float* part,
                                         int* counter, int* act, int* iters,
                                         int conv_mode, int check_every, double* hstate,
                                         hipStream_t stream) {
  if (R <= 0 || N <= 0 || G <= 0) return hipSuccess;
  if (K < 1 || K > 64 || (K > 32 && K % 8) || (side != 0 && side != 1))
    return hipErrorInvalidValue;
  if (side == 1 && num == nullptr) return hipErrorInvalidValue;
  if (mode != 0 && num != nullptr && den == nullptr) return hipErrorInvalidValue;
  if (upd && (side != 0 || (mode == 0 && den_vec == nullptr) ||
              (part != nullptr && (counter == nullptr || act == nullptr)) ||
              (part != nullptr && conv_mode == 1 && hstate == nullptr)))
    return hipErrorInvalidValue;
  cnmf::BetaParams p;
  p.X = X; p.ldx = ldx;
  p.HT = HT; p.h_rs = h_rs; p.ldh = ldh;
  p.W = W; p.w_rs = w_rs; p.ldw = ldw;
  p.N = N; p.G = G; p.K = K; p.R = R;
  p.beta = beta; p.eps = eps;
  p.num = num; p.den = mode == 0 ? nullptr : den;
  p.loss = side == 0 ? loss : nullptr;
  p.active = active;
  p.n_strips = side == 0 ? (N + 63) / 64 : (G + 63) / 64;
  p.splits = side == 0 ? 1 : (splits < 1 ? 1 : splits);
  p.upd = upd;
  p.HTw = const_cast<float*>(HT);
  p.den_vec = den_vec;
  p.l1 = l1; p.l2 = l2; p.gamma = gamma; p.tol = tol;
  p.part = upd ? part : nullptr;
  p.counter = counter; p.act = act; p.iters = iters;
  p.conv_mode = conv_mode; p.check_every = check_every; p.hstate = hstate;
  if (upd) p.num = nullptr;
  switch (mode) {
    case 0: return cnmf::launch_beta_mode<cnmf::kKL>(side, p, stream);
    case 1: return cnmf::launch_beta_mode<cnmf::kIS>(side, p, stream);
    case 2: return cnmf::launch_beta_mode<cnmf::kGeneral>(side, p, stream);
    default: return hipErrorInvalidValue;
  }
}

extern "C" int cnmf_beta_w_update_blocks(int K, int G) {
  const long long kg = (long long)K * G;
  long long nb = (kg + 2047) / 2048;
  return (int)(nb < 1 ? 1 : (nb > 64 ? 64 : nb));
}

extern "C" hipError_t cnmf_beta_w_update(int mode, float* W, long long w_rs, long long ldw,
                                         const float* num, const float* den, const float* hsum,
                                         const float* An, const float* Ad, float* an_out,
                                         float* dn_out, int R, int K, int G, int splits,
                                         float gamma, float l1, float l2, float eps, float tol,
                                         float* part, int* counter, int* act, int* iters,
                                         hipStream_t stream) {
  if (R <= 0) return hipSuccess;
  if (K < 1 || G < 1 || splits < 1 || act == nullptr || part == nullptr || counter == nullptr)
    return hipErrorInvalidValue;
  if (mode == cnmf::kKL ? hsum == nullptr : (den == nullptr || dn_out == nullptr))
    return hipErrorInvalidValue;
  cnmf::BetaWUpd p;
  p.W = W; p.w_rs = w_rs; p.ldw = ldw;
  p.num = num; p.den = den; p.hsum = hsum; p.An = An; p.Ad = Ad;
  p.an_out = an_out; p.dn_out = dn_out;
  p.R = R; p.K = K; p.G = G; p.splits = splits; p.mode = mode;
  p.gamma = gamma; p.l1 = l1; p.l2 = l2; p.eps = eps; p.tol = tol;
  p.part = part; p.counter = counter; p.act = act; p.iters = iters;
  const dim3 grid((unsigned)cnmf_beta_w_update_blocks(K, G), (unsigned)R);
  hipLaunchKernelGGL(cnmf::beta_w_update_kernel, grid, dim3(256), 0, stream, p);
  return hipGetLastError();
}
