// Register-resident instantiations of the fused inner solve (see solve_core.h), U = 3..4
// columns per thread (small K only: U * K <= 36).
#include "solve_core.h"

namespace cnmf {
hipError_t launch_solve_resident34(int K, int U, int algo, const SolveParams& p, int nblocks,
                                   int threads, hipStream_t s) {
  if (U == 3) { CNMF_SOLVE_RES_SWITCH(3) }
  if (U == 4) { CNMF_SOLVE_RES_SWITCH(4) }
  return hipErrorInvalidValue;
}
}  // namespace cnmf
