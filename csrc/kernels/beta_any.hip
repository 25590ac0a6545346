// Rank-general beta-divergence MU terms (KL, IS, general beta) for the ranks beyond the
// split-bf16 panel kernels (beta_planes*.hip: KL K <= 64, IS / general beta K <= 56; the
// reference's -k is unbounded, cnmf.py:1416-1417, and nmf-torch's beta MU is the same at
// every rank, cnmf.py:762, 819).  At those ranks both contractions of a step are real
// GEMMs (P = H^T W and W Q^T / H Q: N G K flops per replicate each) and run as batched
// library GEMMs on the host side; this kernel is the one pass between them: with
// p = max(P, eps) it overwrites P with Q = X p^(beta-2), writes D = p^(beta-1) (not for
// KL, whose denominator is a row sum) and the beta-divergence terms' per-workgroup sums
// in float64 -- the PyTorch sequence it replaces (ops/reference.py beta_terms /
// beta_loss_terms) made 4-8 passes over P with pow / log temporaries.
//
// Layout: P (m, c, G) contiguous float32, replicate e's rows at P + e c G; X (c, G) with
// row stride ldx, shared by every replicate.  Grid (row blocks, m); an inactive replicate
// (act[e] == 0) gets Q = D = 0 and a zero loss partial (the reference skips it).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "common.h"

namespace cnmf {

constexpr int kBaRows = 8;   // rows of P per workgroup

template <int MODE>   // 0 KL, 1 IS, 2 general beta
__global__ __launch_bounds__(256) void beta_any_terms_kernel(
    const float* __restrict__ X, long long ldx, float* __restrict__ P, float* __restrict__ D,
    int c, int G, float beta, float eps, const int* __restrict__ act, int want_q,
    double* __restrict__ part) {
  __shared__ double sc[4];
  const int e = blockIdx.y;
  const int r0 = blockIdx.x * kBaRows, r1 = min(c, r0 + kBaRows);
  const bool live = act == nullptr || act[e] != 0;
  float* Pe = P + (long long)e * c * G;
  float* De = D ? D + (long long)e * c * G : nullptr;
  double loss = 0.0;
  const double db = (double)beta;
  for (int r = r0; r < r1; ++r) {
    const float* xr = X + (long long)r * ldx;
    float* pr = Pe + (long long)r * G;
    float* dr = De ? De + (long long)r * G : nullptr;
    for (int j = threadIdx.x; j < G; j += blockDim.x) {
      if (!live) {
        if (want_q) pr[j] = 0.f;
        if (dr) dr[j] = 0.f;
        continue;
      }
      const float x = xr[j];
      const float p = fmaxf(pr[j], eps);
      float q, d = 0.f;
      if (MODE == 0) {
        q = x / p;
        if (part) {
          const double xd = x, pd = p;
          loss += (x > 0.f ? xd * log(xd / pd) : 0.0) - xd + pd;
        }
      } else if (MODE == 1) {
        const float rp = 1.f / p;
        q = x * rp * rp;
        d = rp;
        if (part) {
          const double dd = fmax((double)x / (double)p, (double)eps);
          loss += dd - log(dd) - 1.0;
        }
      } else {
        q = x * powf(p, beta - 2.f);
        d = powf(p, beta - 1.f);
        if (part) {
          const double xd = x, pd = p;
          loss += (pow(xd, db) + (db - 1.0) * pow(pd, db) - db * xd * pow(pd, db - 1.0)) /
                  (db * (db - 1.0));
        }
      }
      if (want_q) pr[j] = q;
      if (dr) dr[j] = d;
    }
  }
  if (!part) return;
  double a = loss, b = 0.0;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  a = wave_sum(a);
  if (lane == 0) sc[wid] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 0; w < (int)(blockDim.x / kWave); ++w) b += sc[w];
    part[(long long)e * gridDim.x + blockIdx.x] = live ? b : 0.0;
  }
}

}  // namespace cnmf

// mode: 0 KL, 1 IS, 2 general beta.  P (m, c, G) contiguous is overwritten by Q when
// want_q; D (m, c, G) (nullable; unused for KL); part (m, ceil(c / 8)) float64 loss sums
// (nullable: no loss).
extern "C" int cnmf_beta_any_rows() { return cnmf::kBaRows; }

extern "C" hipError_t cnmf_beta_any_terms(int mode, const float* X, long long ldx, float* P,
                                          float* D, int m, int c, int G, float beta, float eps,
                                          const int* act, int want_q, double* part,
                                          hipStream_t stream) {
  if (m <= 0 || c <= 0 || G <= 0) return hipSuccess;
  if (!X || !P || ldx < G || mode < 0 || mode > 2 || (mode == 0 && D)) return hipErrorInvalidValue;
  const dim3 grid((c + cnmf::kBaRows - 1) / cnmf::kBaRows, m);
  const int threads = G >= 256 ? 256 : 64;
  switch (mode) {
    case 0:
      hipLaunchKernelGGL(cnmf::beta_any_terms_kernel<0>, grid, dim3(threads), 0, stream, X, ldx,
                         P, D, c, G, beta, eps, act, want_q, part);
      break;
    case 1:
      hipLaunchKernelGGL(cnmf::beta_any_terms_kernel<1>, grid, dim3(threads), 0, stream, X, ldx,
                         P, D, c, G, beta, eps, act, want_q, part);
      break;
    default:
      hipLaunchKernelGGL(cnmf::beta_any_terms_kernel<2>, grid, dim3(threads), 0, stream, X, ldx,
                         P, D, c, G, beta, eps, act, want_q, part);
  }
  return hipGetLastError();
}
