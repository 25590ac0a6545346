// Pipelined matrix-core MU solve (solve_pipe.h): K = 17..24.
#include "solve_pipe.h"

namespace cnmf {
hipError_t launch_solve_pipe_b2(int K, const SolveParams& p, int nblocks, int T, int pl_n,
                                hipStream_t s) {
  switch (K) {
    case 17: return launch_pipe_k<17>(p, nblocks, T, pl_n, s);
    case 18: return launch_pipe_k<18>(p, nblocks, T, pl_n, s);
    case 19: return launch_pipe_k<19>(p, nblocks, T, pl_n, s);
    case 20: return launch_pipe_k<20>(p, nblocks, T, pl_n, s);
    case 21: return launch_pipe_k<21>(p, nblocks, T, pl_n, s);
    case 22: return launch_pipe_k<22>(p, nblocks, T, pl_n, s);
    case 23: return launch_pipe_k<23>(p, nblocks, T, pl_n, s);
    case 24: return launch_pipe_k<24>(p, nblocks, T, pl_n, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace cnmf
