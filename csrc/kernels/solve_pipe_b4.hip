// Pipelined matrix-core MU solve (solve_pipe.h): K = 40..64 (the padded wide ranks, models/nmf.py native_rank).
#include "solve_pipe.h"

namespace cnmf {
hipError_t launch_solve_pipe_b4(int K, const SolveParams& p, int nblocks, int T, int pl_n,
                                hipStream_t s) {
  switch (K) {
    case 40: return launch_pipe_k<40>(p, nblocks, T, pl_n, s);
    case 48: return launch_pipe_k<48>(p, nblocks, T, pl_n, s);
    case 56: return launch_pipe_k<56>(p, nblocks, T, pl_n, s);
    case 64: return launch_pipe_k<64>(p, nblocks, T, pl_n, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace cnmf
