// Pipelined matrix-core MU solve (solve_pipe.h): K = 25..32.
#include "solve_pipe.h"

namespace cnmf {
hipError_t launch_solve_pipe_b3(int K, const SolveParams& p, int nblocks, int T, int pl_n,
                                hipStream_t s) {
  switch (K) {
    case 25: return launch_pipe_k<25>(p, nblocks, T, pl_n, s);
    case 26: return launch_pipe_k<26>(p, nblocks, T, pl_n, s);
    case 27: return launch_pipe_k<27>(p, nblocks, T, pl_n, s);
    case 28: return launch_pipe_k<28>(p, nblocks, T, pl_n, s);
    case 29: return launch_pipe_k<29>(p, nblocks, T, pl_n, s);
    case 30: return launch_pipe_k<30>(p, nblocks, T, pl_n, s);
    case 31: return launch_pipe_k<31>(p, nblocks, T, pl_n, s);
    case 32: return launch_pipe_k<32>(p, nblocks, T, pl_n, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace cnmf
