// Register-resident instantiations of the fused inner solve (see solve_core.h):
// compiled as a separate unit so the two variant sets build in parallel.
#include "solve_core.h"

namespace cnmf {
hipError_t launch_solve_resident(int K, int algo, const SolveParams& p, int nblocks,
                                 int threads, hipStream_t s) {
  switch (K) {
    case 1: return launch_solve_k<1, 1>(algo, p, nblocks, threads, s);
    case 2: return launch_solve_k<2, 1>(algo, p, nblocks, threads, s);
    case 3: return launch_solve_k<3, 1>(algo, p, nblocks, threads, s);
    case 4: return launch_solve_k<4, 1>(algo, p, nblocks, threads, s);
    case 5: return launch_solve_k<5, 1>(algo, p, nblocks, threads, s);
    case 6: return launch_solve_k<6, 1>(algo, p, nblocks, threads, s);
    case 7: return launch_solve_k<7, 1>(algo, p, nblocks, threads, s);
    case 8: return launch_solve_k<8, 1>(algo, p, nblocks, threads, s);
    case 9: return launch_solve_k<9, 1>(algo, p, nblocks, threads, s);
    case 10: return launch_solve_k<10, 1>(algo, p, nblocks, threads, s);
    case 11: return launch_solve_k<11, 1>(algo, p, nblocks, threads, s);
    case 12: return launch_solve_k<12, 1>(algo, p, nblocks, threads, s);
    case 13: return launch_solve_k<13, 1>(algo, p, nblocks, threads, s);
    case 14: return launch_solve_k<14, 1>(algo, p, nblocks, threads, s);
    case 15: return launch_solve_k<15, 1>(algo, p, nblocks, threads, s);
    case 16: return launch_solve_k<16, 1>(algo, p, nblocks, threads, s);
    default: return hipErrorInvalidValue;   // K > kResidentMaxK: streaming only
  }
}
}  // namespace cnmf
