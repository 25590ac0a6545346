// KL ranks 33..64 of the fused beta-divergence MU kernels (beta_planes.h): K padded to a
// multiple of 8 by the engine (models.nmf.native_rank) -> (panels NP, tiles T) of
// K = 40 (4, 3), 48 (5, 3), 56 / 64 (6, 4); one column tile per wave (bp_ct).  Usage and
// spectra sides, fp32 X or fp16 counts.
#include "beta_planes.h"

namespace cnmf {

template <bool UPD, bool XH>
static hipError_t bp_wide_kl(int np, int t, const BpParams& p, hipStream_t s) {
  if (np == 4 && t == 3) return bp_launch<4, 3, kBpKL, UPD, XH>(p, s);
  if (np == 5 && t == 3) return bp_launch<5, 3, kBpKL, UPD, XH>(p, s);
  if (np == 6 && t == 4) return bp_launch<6, 4, kBpKL, UPD, XH>(p, s);
  return hipErrorInvalidValue;
}

hipError_t bp_launch_wide_kl(bool upd, bool xh, int np, int t, const BpParams& p, hipStream_t s) {
  if (upd) return xh ? bp_wide_kl<true, true>(np, t, p, s) : bp_wide_kl<true, false>(np, t, p, s);
  return xh ? bp_wide_kl<false, true>(np, t, p, s) : bp_wide_kl<false, false>(np, t, p, s);
}

}  // namespace cnmf
