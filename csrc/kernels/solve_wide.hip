// Wide-rank instantiations (K = 40, 48, 56, 64) of the fused inner solve: the NMF engine
// pads K in (32, 64] to a multiple of 8 with zero components (they stay zero under MU and
// HALS), so four instantiations cover every K <= 64.  Separate unit: long compile.
#include "solve_core.h"

namespace cnmf {
hipError_t launch_solve_wide(int K, int algo, const SolveParams& p, int nblocks, int threads,
                             hipStream_t s) {
  CNMF_SOLVE_WIDE_SWITCH()
}
}  // namespace cnmf
