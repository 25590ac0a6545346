// Register-resident instantiations of the fused inner solve (see solve_core.h), U = 1..2
// columns per thread; U = 3..4 live in solve_res34.hip so the sets build in parallel.
#include "solve_core.h"

namespace cnmf {
hipError_t launch_solve_resident(int K, int U, int algo, const SolveParams& p, int nblocks,
                                 int threads, hipStream_t s) {
  if (U == 1) { CNMF_SOLVE_RES_SWITCH(1) }
  if (U == 2) { CNMF_SOLVE_RES_SWITCH(2) }
  return launch_solve_resident34(K, U, algo, p, nblocks, threads, s);
}
}  // namespace cnmf
