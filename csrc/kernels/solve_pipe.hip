// Pipelined matrix-core MU solve (solve_pipe.h): K 1..16 instantiations, the K dispatch
// over the band units (solve_pipe_b2.hip 17..24, solve_pipe_b3.hip 25..32,
// solve_pipe_b4.hip 40..64) and the host-side geometry queries.
#include "solve_pipe.h"

namespace cnmf {
hipError_t launch_solve_pipe_b2(int K, const SolveParams& p, int nblocks, int T, int pl_n,
                                hipStream_t s);
hipError_t launch_solve_pipe_b3(int K, const SolveParams& p, int nblocks, int T, int pl_n,
                                hipStream_t s);
hipError_t launch_solve_pipe_b4(int K, const SolveParams& p, int nblocks, int T, int pl_n,
                                hipStream_t s);

#define CNMF_PIPE_CASE(KK) \
  case KK: return launch_pipe_k<KK>(p, nblocks, T, pl_n, s);
hipError_t launch_solve_pipe(int K, const SolveParams& p, int nblocks, int T, int pl_n,
                             hipStream_t s) {
  if (K < 1 || T < 1 || T > pipe_tile_max(K)) return hipErrorInvalidValue;
  if (K > 32) return launch_solve_pipe_b4(K, p, nblocks, T, pl_n, s);
  if (K > 24) return launch_solve_pipe_b3(K, p, nblocks, T, pl_n, s);
  if (K > 16) return launch_solve_pipe_b2(K, p, nblocks, T, pl_n, s);
  switch (K) {
    CNMF_PIPE_CASE(1) CNMF_PIPE_CASE(2) CNMF_PIPE_CASE(3) CNMF_PIPE_CASE(4)
    CNMF_PIPE_CASE(5) CNMF_PIPE_CASE(6) CNMF_PIPE_CASE(7) CNMF_PIPE_CASE(8)
    CNMF_PIPE_CASE(9) CNMF_PIPE_CASE(10) CNMF_PIPE_CASE(11) CNMF_PIPE_CASE(12)
    CNMF_PIPE_CASE(13) CNMF_PIPE_CASE(14) CNMF_PIPE_CASE(15) CNMF_PIPE_CASE(16)
    default: return hipErrorInvalidValue;
  }
}
#undef CNMF_PIPE_CASE
}  // namespace cnmf

// ranks with a pipelined instantiation: 1..32 and the padded wide ranks 40..64
extern "C" int cnmf_solve_pipe_k(int K) {
  return (K >= 1 && K <= 32) || K == 40 || K == 48 || K == 56 || K == 64;
}

// tile count the pipelined solve runs for `per` columns per slice (0: not covered)
extern "C" int cnmf_solve_pipe_tiles(int K, int per) {
  if (!cnmf_solve_pipe_k(K) || per < 1) return 0;
  const int need = (per + 16 * cnmf::kPipeWaves - 1) / (16 * cnmf::kPipeWaves);
  if (need > cnmf::pipe_tile_max(K)) return 0;
  for (int i = 0; i < cnmf::kPipeTCount; ++i)
    if (cnmf::pipe_t_of(i) >= need) return cnmf::pipe_t_of(i);
  return 0;
}

// columns one workgroup of the pipelined solve can own, and its workgroups per CU
extern "C" int cnmf_solve_pipe_max_cols(int K) {
  return cnmf_solve_pipe_k(K) ? 16 * cnmf::kPipeWaves * cnmf::pipe_tile_max(K) : 0;
}
extern "C" int cnmf_solve_pipe_wg_per_cu(int K) {
  return cnmf_solve_pipe_k(K) ? cnmf::pipe_wg_per_cu(K) : 0;
}
