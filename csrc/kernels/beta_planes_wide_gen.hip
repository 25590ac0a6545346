// Itakura-Saito / general-beta ranks 33..56 of the fused beta-divergence MU kernels
// (beta_planes.h), K padded to a multiple of 8: (NP, T) of K = 40 (8, 3), 48 (9, 3),
// 56 (11, 4).  K = 64 would need 12 panels of P slots -- two panel chunks of it exceed
// the 160 KB LDS -- so those replicates take the eager path (models.nmf.kernel_max_rank).
#include "beta_planes.h"

namespace cnmf {

template <int MODE, bool UPD>
static hipError_t bp_wide_gen(int np, int t, const BpParams& p, hipStream_t s) {
  if (np == 8 && t == 3) return bp_launch<8, 3, MODE, UPD>(p, s);
  if (np == 9 && t == 3) return bp_launch<9, 3, MODE, UPD>(p, s);
  if (np == 11 && t == 4) return bp_launch<11, 4, MODE, UPD>(p, s);
  return hipErrorInvalidValue;
}

hipError_t bp_launch_wide_gen(int mode, bool upd, int np, int t, const BpParams& p,
                              hipStream_t s) {
  if (mode == kBpIS)
    return upd ? bp_wide_gen<kBpIS, true>(np, t, p, s) : bp_wide_gen<kBpIS, false>(np, t, p, s);
  if (mode == kBpGeneral)
    return upd ? bp_wide_gen<kBpGeneral, true>(np, t, p, s)
               : bp_wide_gen<kBpGeneral, false>(np, t, p, s);
  return hipErrorInvalidValue;
}

}  // namespace cnmf
