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
  const int* rep_index;     // rep0 + blockIdx.x -> replicate (nullptr = identity)
  int rep0;                 // first replicate slot of this launch (co-resident rounds)
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
  // Fused operands (solve_pipe.hip only; all off by default).  They let one online step
  // run GEMM -> solve -> GEMM -> solve with no reduction or Gram launches in between:
  //  * numerator = nbase + n_scale[col] * sum_{q < nslab_n} numer[q * nslab_stride + ..]
  //    (the raw split-K slabs of gemm_planes(raw_slab=...), summed in slice order as
  //    gemm_reduce_kernel does), optionally written back to nout (the accumulated B);
  //  * Gram = gram (optional base) + sum_{q < gpart_n} gpart[rep * gpart_rs + q * K * K]
  //    (partial Grams of the producing solve's slices), written by slice 0 to gout;
  //  * gp_out: this slice's partial Gram sum_cols x x^T of the FINAL x, at
  //    gp_out[rep * gp_rs + slice * K * K] -- the next solve's gpart.
  int nslab_n;
  long long nslab_stride;
  const float* n_scale;
  const float* nbase;
  float* nout;
  long long nb_rs, ldnb;
  const float* gpart;
  int gpart_n;
  long long gpart_rs;
  float* gout;
  float* gp_out;
  long long gp_rs;
  // Device-side launch generation for the cooperative granules (solve_pipe.hip): the
  // tag is read from *coop_gen_dev at kernel start instead of the host's coop_gen, and
  // the last workgroup to finish (arrival counter coop_arrive) advances it.  A launch
  // captured in a HIP graph then tags every replay differently without re-zeroing the
  // granules (tags in [2^31, 2^32 - 1); host tags stay below 2^31).
  unsigned* coop_gen_dev;
  unsigned* coop_arrive;
  // Diagnostic (solve_pipe.h only; nullptr in every production launch): per workgroup 8
  // uint64 at stamps[(slice * blocks + block) * 10]: s_memrealtime at start
  // and end, then cycles (s_memtime deltas) of the prologue, the sweep loop, the objective
  // checks inside it (chain + block reduce + cooperative exchange), the epilogue; checks,
  // sweeps.  Written only to this buffer; nothing in the kernel reads it.
  unsigned long long* stamps;
  // solve_pipe.h workgroup order: 0 = grid (replicates, slices); 1 = a 1-D grid in which
  // the S slices of one replicate are consecutive workgroups of ONE XCD (workgroup w runs
  // on XCD w % 8): they start together and exchange through one L2.  pipe_nblocks: the
  // launch's replicate count (set by the launcher).
  int pipe_map;
  int pipe_nblocks;
  // Optional (matrix-core kernel only): the system matrix is the Gram F F^T of the factor
  // F_r = gsrc + r*gs_rs (K x gs_cols, row stride gs_ld), formed in the prologue on the
  // matrix cores instead of being read from `gram` (W W^T fused into
  // the H-update prologue; no separate Gram launch per online step)
  const float* gsrc;
  long long gs_rs, gs_ld;
  int gs_cols;
};

}  // namespace cnmf
