// Parameter block shared by the streaming (solve.hip) and register-resident
// (solve_reg.hip) fused solve kernels.
#pragma once

namespace cnmf {

struct SolveParams {
  float* x;                 // solution, replicate r at x + r*x_rs, row (component) stride ldx
  long long x_rs, ldx;
  const float* numer;       // numerator, same layout as x
  long long n_rs, ldn;
  const float* gram;        // K x K per replicate
  long long g_rs;
  const int* rep_index;     // blockIdx.x -> replicate (nullptr = identity)
  int ncols, max_iter;
  float tol, l1_num, l1_den, l2, eps;
  float* lin_out;           // optional <numer, x>
  float* quad_out;          // optional sum_j x_j^T Gram x_j
  int* iters_out;           // optional: += steps taken (accumulates across calls)
  const int* active;        // optional per-replicate flag: 0 -> the block returns at once
  int nsplit;               // >1: blockIdx.y splits the columns; single fixed step
  int conv_mode;            // 0: ||dx||/(||x||+eps) < tol each step (cnmf.py:375-378)
                            // 1: block objective every `check_every` steps (nmf-torch online)
  int check_every;
  // Cooperative split (gridDim.y = S > 1 workgroups per replicate, WITH convergence):
  // per-epoch partial sums are exchanged through global memory (deterministic order) as
  // {tag = coop_gen, value} granules (coop_sum2 in solve_core.h), never zeroed between
  // eager launches: coop_gen strictly increases per workspace.
  unsigned long long* coop_slots;   // [R][coop_epochs][S][2] granules
  unsigned coop_gen;
  int coop_epochs;
  int* coop_timeout;        // set to 1 if a spin gave up (residency violated)
  int coop_epochs_split;    // launch-side: S (gridDim.y) for the cooperative split
  // Optional epilogue feeding the split-precision GEMM (gemm_planes.hip): the final x
  // times pl_colmul[col] (optional) split exactly into three bf16 planes at
  // planes + p*pl_plane + rep*pl_rs + k*pl_ld + col, columns [ncols, pl_cols) zeroed.
  unsigned short* planes;
  long long pl_rs, pl_ld, pl_plane;
  const float* pl_colmul;
  int pl_cols;
  int pl_n;                 // planes written (1..3): the consuming GEMM reads only its A planes
  // Optional (matrix-core kernel only): the system matrix is the Gram F F^T of the factor
  // F_r = gsrc + r*gs_rs (K x gs_cols, row stride gs_ld), formed in the prologue on the
  // matrix cores instead of being read from `gram` (W W^T fused into
  // the H-update prologue; no separate Gram launch per online step)
  const float* gsrc;
  long long gs_rs, gs_ld;
  int gs_cols;
};

}  // namespace cnmf
