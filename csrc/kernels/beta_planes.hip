// Fused beta-divergence MU on the bf16 matrix cores: dispatch by rank and the C ABI
// (kernels and launch templates: beta_planes.h; the wide ranks: beta_planes_wide*.hip).
#include "beta_planes.h"

namespace cnmf {

__global__ void __launch_bounds__(256) bp_panel_kernel(const float* __restrict__ F,
                                                       long long f_rs, long long ldf, int K,
                                                       int L, int nchunks, int R, int NP,
                                                       int T, int nt, int kl,
                                                       const float* __restrict__ rowsc,
                                                       unsigned short* __restrict__ out,
                                                       long long out_rs) {
  const long long per = (long long)nchunks * kBpCH;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= per * R) return;
  const int r = (int)(idx / per), l = (int)(idx - (long long)r * per);
  const int PS = bp_ps(NP), CE = bp_chunk(NP, T);
  unsigned short* ch = out + r * out_rs + (long long)(l / kBpCH) * CE;
  const float* rsc = reinterpret_cast<const float*>(out + r * out_rs + (long long)nchunks * CE);
  const int lr = l % kBpCH, o = lr & 31;
  unsigned short* prow = ch + lr * PS;
  unsigned short* np0 = ch + kBpCH * PS;
  unsigned short* np1 = np0 + 16 * T * kBpNS;
  const int pos = (lr & 32) + ((o & 15) >> 2) * 8 + (o >> 4) * 4 + (o & 3);
  const float* f = F + r * f_rs + l;
  for (int k = 0; k < 16 * T; ++k) {
    unsigned short a0 = 0, a1 = 0, a2 = 0, n0 = 0, n1 = 0;
    if (k < K && l < L) {
      const float v = f[(long long)k * ldf];
      bp_split3(rowsc ? v * rowsc[l] : v, a0, a1, a2);   // P panel of S / u (fp16 counts)
      if (kl) {
        const float s = v * rsc[k];
        const _Float16 h0 = (_Float16)s;
        n0 = __builtin_bit_cast(unsigned short, h0);
        n1 = __builtin_bit_cast(unsigned short, (_Float16)(s - (float)h0));
      } else {
        n0 = a0;
        n1 = a1;
      }
    }
    if (k < K)
      for (int t = 0; t < nt; ++t) {
        const int pl = bp_pa(t);
        prow[t * K + k] = pl == 0 ? a0 : (pl == 1 ? a1 : a2);
      }
    np0[k * kBpNS + pos] = n0;
    np1[k * kBpNS + pos] = n1;
  }
  for (int s = nt * K; s < PS; ++s) prow[s] = 0;
}

// KL panel row scales: per replicate r and row k < K, 2^-e_k with max_l |F[r][k][l]| * 2^-e_k
// in [0.5, 1) (1 for an all-zero or non-finite row) and its inverse, into the panel tail.
// One workgroup per replicate.
__global__ void __launch_bounds__(256) bp_rowscale_kernel(const float* __restrict__ F,
                                                          long long f_rs, long long ldf, int K,
                                                          int L, unsigned short* __restrict__ out,
                                                          long long out_rs, long long tail) {
  __shared__ float red[4];
  const int r = blockIdx.x, tid = threadIdx.x;
  const float* f = F + r * f_rs;
  float* dst = reinterpret_cast<float*>(out + r * out_rs + tail);
  for (int k = 0; k < K; ++k) {
    float m = 0.f;
    for (int l = tid; l < L; l += 256) m = fmaxf(m, fabsf(f[(long long)k * ldf + l]));
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    if (tid == 0) {
      const float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      int e = 0;
      if (mx > 0.f && mx <= 3.0e38f) frexpf(mx, &e);
      dst[k] = ldexpf(1.f, -e);
      dst[kBpMaxK + k] = ldexpf(1.f, e);
    }
    __syncthreads();
  }
}

template <int MODE, bool UPD>
hipError_t bp_launch_k(const BpParams& p, hipStream_t s) {
  if constexpr (bp_is_kl(MODE)) {
    const int np = bp_np(p.K, MODE), t = bp_t(p.K);
    if (t >= 3)
      return MODE == kBpKL
                 ? bp_launch_wide_kl(UPD, p.uvec != nullptr || p.fscale != nullptr, np, t, p, s)
                 : bp_launch_wide_klx(UPD, p.uvec != nullptr || p.fscale != nullptr, np, t, p, s);
    if (p.uvec != nullptr || p.fscale != nullptr) {   // fp16 counts
      if (np == 1 && t == 1) return bp_launch<1, 1, MODE, UPD, true>(p, s);
      if (np == 2 && t == 1) return bp_launch<2, 1, MODE, UPD, true>(p, s);
      if (np == 2 && t == 2) return bp_launch<2, 2, MODE, UPD, true>(p, s);
      if (np == 3 && t == 2) return bp_launch<3, 2, MODE, UPD, true>(p, s);
      return hipErrorInvalidValue;
    }
    if (np == 1 && t == 1) return bp_launch<1, 1, MODE, UPD>(p, s);
    if (np == 2 && t == 1) return bp_launch<2, 1, MODE, UPD>(p, s);
    if (np == 2 && t == 2) return bp_launch<2, 2, MODE, UPD>(p, s);
    if (np == 3 && t == 2) return bp_launch<3, 2, MODE, UPD>(p, s);
    return hipErrorInvalidValue;
  } else {
    if (bp_t(p.K) >= 3) return bp_launch_wide_gen(MODE, UPD, bp_np(p.K), bp_t(p.K), p, s);
    switch (bp_np(p.K)) {
      case 1: return bp_launch<1, 1, MODE, UPD>(p, s);
      case 2: return bp_launch<2, 1, MODE, UPD>(p, s);
      case 3: return bp_launch<3, 1, MODE, UPD>(p, s);
      case 4: return bp_launch<4, 2, MODE, UPD>(p, s);
      case 5: return bp_launch<5, 2, MODE, UPD>(p, s);
      case 6: return bp_launch<6, 2, MODE, UPD>(p, s);
      default: return hipErrorInvalidValue;
    }
  }
}

template <bool UPD>
hipError_t bp_launch_mode(int mode, const BpParams& p, hipStream_t s) {
  switch (mode) {
    case kBpKL: return bp_launch_k<kBpKL, UPD>(p, s);
    case kBpIS: return bp_launch_k<kBpIS, UPD>(p, s);
    case kBpGeneral: return bp_launch_k<kBpGeneral, UPD>(p, s);
    case kBpKLX: return bp_launch_k<kBpKLX, UPD>(p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace cnmf

extern "C" int cnmf_bp_max_k() { return cnmf::kBpMaxK; }

// 16-bit elements of one replicate's panel over a streamed axis of length L (layout by
// beta mode: KL panels hold 3-term P slots, fp16 numerator planes and the row-scale tail)
extern "C" long long cnmf_bp_panel_elems(int K, int L, int mode) {
  if (K < 1 || K > cnmf::kBpMaxK || mode < 0 || mode > 3) return -1;
  const int NP = cnmf::bp_np(K, mode), T = cnmf::bp_t(K);
  return (long long)((L + cnmf::kBpCH - 1) / cnmf::kBpCH) * cnmf::bp_chunk(NP, T) +
         (mode == cnmf::kBpKL ? cnmf::kBpTail : 0);
}

// fixed-axis columns per workgroup strip
extern "C" int cnmf_bp_strip_cols(int K, int mode) {
  (void)mode;
  return cnmf::kBpWaves * cnmf::bp_ct(cnmf::bp_t(K)) * 16;
}

extern "C" hipError_t cnmf_bp_panels(const float* F, long long f_rs, long long ldf, int K, int L,
                                     int R, int mode, const float* prow, unsigned short* out,
                                     long long out_rs, hipStream_t stream) {
  if (R <= 0 || L <= 0) return hipSuccess;
  if (K < 1 || K > cnmf::kBpMaxK || mode < 0 || mode > 3) return hipErrorInvalidValue;
  if (out_rs < cnmf_bp_panel_elems(K, L, mode)) return hipErrorInvalidValue;
  // (KLX panels: KL's 3-term P slots with the two bf16 numerator planes of IS / general)
  const int NP = cnmf::bp_np(K, mode), T = cnmf::bp_t(K);
  const int nchunks = (L + cnmf::kBpCH - 1) / cnmf::kBpCH;
  const bool kl = mode == cnmf::kBpKL;
  if (kl)
    hipLaunchKernelGGL(cnmf::bp_rowscale_kernel, dim3((unsigned)R), dim3(256), 0, stream, F,
                       f_rs, ldf, K, L, out, out_rs,
                       (long long)nchunks * cnmf::bp_chunk(NP, T));
  const long long n = (long long)R * nchunks * cnmf::kBpCH;
  const dim3 grid((unsigned)((n + 255) / 256));
  hipLaunchKernelGGL(cnmf::bp_panel_kernel, grid, dim3(256), 0, stream, F, f_rs, ldf, K, L,
                     nchunks, R, NP, T, cnmf::bp_nt(mode), kl ? 1 : 0, prow, out, out_rs);
  return hipGetLastError();
}

// side 0 (H, fused update; nsteps 0 = loss only into `loss`), side 1 (W, num/den partials)
extern "C" hipError_t cnmf_bp_run(
    int side, int mode, const float* X, long long ldx, const unsigned short* panel,
    long long panel_rs, float* F, long long f_rs, long long ldf, int K, int Lf, int Ls, int R,
    int splits, float beta, float eps, float* num, float* den, int nsteps, int loss_entry,
    int loss_exit, const float* den_vec, float l1, float l2, float gamma, float tol,
    int conv_mode, double* hstate, double* part, int* counter, int* act, int* iters,
    const int* active, double* loss, double xsum, int xh, const float* uvec,
    const float* fscale, hipStream_t stream) {
  if (R <= 0 || Lf <= 0) return hipSuccess;
  if (K < 1 || K > cnmf::kBpMaxK || Ls <= 0 || (side != 0 && side != 1)) return hipErrorInvalidValue;
  // fp16 counts: KL only; the H side needs the loss weights, the W side the column scales
  // (the fp32-accurate KL mode reads them on the W side only: its loss has no weights)
  if (xh && (!cnmf::bp_is_kl(mode) || (mode == cnmf::kBpKLX && side == 0) ||
             (side == 0 ? uvec == nullptr : fscale == nullptr)))
    return hipErrorInvalidValue;
  if (mode < 0 || mode > 3 || panel_rs < cnmf_bp_panel_elems(K, Ls, mode))
    return hipErrorInvalidValue;
  cnmf::BpParams p;
  p.X = X; p.ldx = ldx;
  p.xvec = (ldx % 4 == 0) &&
           ((reinterpret_cast<uintptr_t>(X) & (xh ? 7 : 15)) == 0);
  p.uvec = xh ? (side == 0 ? uvec : nullptr) : nullptr;
  p.fscale = xh ? (side == 1 ? fscale : nullptr) : nullptr;
  if (xh && side == 0 && p.uvec == nullptr) return hipErrorInvalidValue;
  p.panel = panel; p.panel_rs = panel_rs;
  p.F = F; p.f_rs = f_rs; p.ldf = ldf;
  p.K = K; p.Lf = Lf; p.Ls = Ls; p.R = R;
  p.n_strips = (Lf + cnmf_bp_strip_cols(K, mode) - 1) / cnmf_bp_strip_cols(K, mode);
  const int nch = (Ls + cnmf::kBpCH - 1) / cnmf::kBpCH;
  if (side == 0) splits = 1;
  splits = splits < 1 ? 1 : (splits > nch ? nch : splits);
  p.chunks_per_split = (nch + splits - 1) / splits;
  p.splits = (nch + p.chunks_per_split - 1) / p.chunks_per_split;
  p.beta = beta; p.eps = eps;
  p.num = num; p.den = den;
  p.nsteps = nsteps; p.loss_entry = loss_entry; p.loss_exit = loss_exit;
  p.den_vec = den_vec;
  p.l1 = l1; p.l2 = l2; p.gamma = gamma; p.tol = tol;
  p.conv_mode = conv_mode; p.hstate = hstate; p.part = part;
  p.counter = counter; p.act = act; p.iters = iters; p.active = active; p.loss = loss;
  p.xsum = xsum;
  if (side == 1) {
    if (num == nullptr || (!cnmf::bp_is_kl(mode) && den == nullptr)) return hipErrorInvalidValue;
    return cnmf::bp_launch_mode<false>(mode, p, stream);
  }
  if (nsteps < 0 || (cnmf::bp_is_kl(mode) && den_vec == nullptr) ||
      (part != nullptr && (counter == nullptr || act == nullptr)) ||
      (part != nullptr && conv_mode == 1 && hstate == nullptr) ||
      (nsteps == 0 && loss == nullptr && part == nullptr))
    return hipErrorInvalidValue;
  return cnmf::bp_launch_mode<true>(mode, p, stream);
}

// splits actually used by a side-1 launch (partials buffer extent)
extern "C" int cnmf_bp_splits(int Ls, int splits) {
  const int nch = (Ls + cnmf::kBpCH - 1) / cnmf::kBpCH;
  splits = splits < 1 ? 1 : (splits > nch ? nch : splits);
  const int per = (nch + splits - 1) / splits;
  return (nch + per - 1) / per;
}
