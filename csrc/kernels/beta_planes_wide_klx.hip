// Fp32-accurate KL (kBpKLX, the default KL mode) at ranks 33..64 of the fused
// beta-divergence MU kernels (beta_planes.h): the (panels NP, tiles T) of
// beta_planes_wide.hip, in their own unit so the units compile in parallel.
#include "beta_planes.h"

namespace cnmf {

template <bool UPD, bool XH>
static hipError_t bp_wide_klx(int np, int t, const BpParams& p, hipStream_t s) {
  if (np == 4 && t == 3) return bp_launch<4, 3, kBpKLX, UPD, XH>(p, s);
  if (np == 5 && t == 3) return bp_launch<5, 3, kBpKLX, UPD, XH>(p, s);
  if (np == 6 && t == 4) return bp_launch<6, 4, kBpKLX, UPD, XH>(p, s);
  return hipErrorInvalidValue;
}

hipError_t bp_launch_wide_klx(bool upd, bool xh, int np, int t, const BpParams& p, hipStream_t s) {
  // (fp16 counts only on the spectra side, which does not update in place)
  if (upd) return xh ? hipErrorInvalidValue : bp_wide_klx<true, false>(np, t, p, s);
  return xh ? bp_wide_klx<false, true>(np, t, p, s) : bp_wide_klx<false, false>(np, t, p, s);
}

}  // namespace cnmf
