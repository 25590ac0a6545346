// Launcher + C ABI of the fused inner solve (kernels in solve_core.h).  This unit
// instantiates the streaming variant; solve_res.hip the register-resident one.
#include "solve_core.h"

namespace cnmf {
hipError_t launch_solve_stream(int K, int algo, const SolveParams& p, int nblocks, int threads,
                               hipStream_t s) {
  CNMF_SOLVE_K_SWITCH(0)
}
}  // namespace cnmf

extern "C" int cnmf_solve_max_k() { return 128; }
extern "C" int cnmf_solve_mfma_max_cols(int K);
extern "C" int cnmf_solve_pipe_tiles(int K, int per);
extern "C" int cnmf_solve_pipe_k(int K);
extern "C" int cnmf_solve_pipe_wg_per_cu(int K);

// ranks the kernels are instantiated for: 1..32, the padded wide ranks 40..64 (multiples
// of 8) and 80..128 (multiples of 16, MU only: solve_wmfma.hip)
extern "C" int cnmf_solve_native_k(int K) {
  return (K >= 1 && K <= 32) || K == 40 || K == 48 || K == 56 || K == 64 || K == 80 ||
         K == 96 || K == 112 || K == 128;
}

extern "C" int cnmf_solve_max_threads(int K) { return K > 32 ? 256 : 1024; }

extern "C" int cnmf_solve_reg_max_cols(int K) {
  return K <= cnmf::kResidentMaxK ? 1024 * cnmf::res_max_cols(K) : 0;
}

extern "C" hipError_t cnmf_solve(int algo, int K, float* x, long long x_rs, long long ldx,
                                 const float* numer, long long n_rs, long long ldn,
                                 const float* gram, long long g_rs, const int* rep_index,
                                 int nblocks, int ncols, int max_iter, float tol, float l1_num,
                                 float l1_den, float l2, float eps, float* lin_out,
                                 float* quad_out, int* iters_out, int nsplit, int conv_mode,
                                 int check_every, int threads, int variant,
                                 const int* active, int coop_split, float* coop_slots,
                                 unsigned long long* coop_count, unsigned coop_gen,
                                 int coop_epochs, int* coop_timeout,
                                 unsigned short* planes, long long pl_rs, long long pl_ld,
                                 long long pl_plane, const float* pl_colmul, int pl_cols,
                                 int pl_n, const float* gsrc, long long gs_rs, long long gs_ld,
                                 int gs_cols, int nslab_n, long long nslab_stride, const float* n_scale, const float* nbase,
                                 float* nout, long long nb_rs, long long ldnb, const float* gpart,
                                 int gpart_n, long long gpart_rs, float* gout, float* gp_out,
                                 long long gp_rs, unsigned* coop_gen_dev, unsigned* coop_arrive,
                                 int reps_per_launch, unsigned long long* stamps,
                                 hipStream_t stream) {
  if (nblocks <= 0) return hipSuccess;
  // buffer offsets are 32-bit: a replicate's block must span < 2 GiB
  if ((long long)K * (ldx > ldn ? ldx : ldn) * 4 >= 0x7fffffffLL) return hipErrorInvalidValue;
  cnmf::SolveParams p;
  p.x = x; p.x_rs = x_rs; p.ldx = ldx;
  p.numer = numer; p.n_rs = n_rs; p.ldn = ldn;
  p.gram = gram; p.g_rs = g_rs;
  p.rep_index = rep_index;
  p.rep0 = 0;
  p.ncols = ncols; p.max_iter = max_iter;
  p.tol = tol; p.l1_num = l1_num; p.l1_den = l1_den; p.l2 = l2; p.eps = eps;
  p.lin_out = lin_out; p.quad_out = quad_out; p.iters_out = iters_out;
  p.nsplit = nsplit;
  p.conv_mode = conv_mode;
  p.check_every = check_every;
  p.active = active;
  p.coop_slots = coop_split > 1 ? (unsigned long long*)coop_slots : nullptr;
  (void)coop_count;   // unused since the granule exchange (kept in the C ABI)
  p.coop_gen = coop_gen;
  p.coop_epochs = coop_epochs;
  p.coop_timeout = coop_timeout;
  p.coop_epochs_split = coop_split > 1 ? coop_split : 1;
  p.planes = planes; p.pl_rs = pl_rs; p.pl_ld = pl_ld; p.pl_plane = pl_plane;
  p.pl_colmul = pl_colmul; p.pl_cols = pl_cols;
  p.pl_n = pl_n < 1 ? 1 : (pl_n > 3 ? 3 : pl_n);
  p.gsrc = gsrc; p.gs_rs = gs_rs; p.gs_ld = gs_ld; p.gs_cols = gs_cols;
  p.nslab_n = nslab_n < 1 ? 1 : nslab_n; p.nslab_stride = nslab_stride; p.n_scale = n_scale;
  p.nbase = nbase; p.nout = nout; p.nb_rs = nb_rs; p.ldnb = ldnb;
  p.gpart = gpart; p.gpart_n = gpart_n; p.gpart_rs = gpart_rs; p.gout = gout;
  p.gp_out = gp_out; p.gp_rs = gp_rs;
  p.coop_gen_dev = coop_split > 1 ? coop_gen_dev : nullptr;
  p.coop_arrive = coop_arrive;
  p.stamps = stamps;
  {
    // workgroup order of the pipelined kernel (SolveParams.pipe_map); CNMF_PIPE_MAP
    // overrides the default for A/B runs
    static const int map_env = [] {
      const char* e = getenv("CNMF_PIPE_MAP");
      return (e && *e) ? atoi(e) : -1;
    }();
    p.pipe_map = map_env >= 0 ? map_env : -1;     // -1: chosen per launch below
    p.pipe_nblocks = nblocks;
  }
  if (p.coop_gen_dev && !coop_arrive) return hipErrorInvalidValue;
  const bool fused = p.nslab_n > 1 || n_scale || nbase || nout || gpart || gout || gp_out ||
                     (coop_split > 1 && coop_gen_dev);
  if (fused && (p.nslab_n > 1 && p.nslab_stride * 4 * (long long)p.nslab_n >= 0x7fffffffLL))
    return hipErrorInvalidValue;
  if (!gram && !gpart && !gsrc) return hipErrorInvalidValue;
  // the in-prologue Gram is a matrix-core kernel feature (K <= 16)
  if (gsrc && (variant != 3 || K > 16 || gs_cols < 1)) return hipErrorInvalidValue;
  if (planes && pl_cols < ncols) return hipErrorInvalidValue;
  if (coop_split > 1 && nsplit > 1) return hipErrorInvalidValue;
  if (coop_split > cnmf::kCoopMaxSlices) return hipErrorInvalidValue;
  if (!cnmf_solve_native_k(K)) return hipErrorInvalidValue;
  if (variant == 3 || variant == 5) {
    // matrix-core variants, MU, every slice within one workgroup's tiles; the host picks
    // the slicing (ops.solve / _mfma_split / _pipe_plan).  The software-pipelined kernel
    // (solve_pipe.h, K <= 64) takes the unregularised block-objective solves;
    // solve_mfma.hip (K <= 16) the rest (and everything under variant 5 =
    // CNMF_SOLVE_PIPE=0).  reps_per_launch > 0: the pipelined kernel runs the replicates
    // in rounds of that many, each round's S * reps workgroups co-resident (the host's
    // budget) -- the wide ranks' register tiles do not hold every replicate at once
    const int parts = nsplit > 1 ? nsplit : (coop_split > 1 ? coop_split : 1);
    const int per = (ncols + parts - 1) / parts;
    const int T = ((per + 15) / 16 + 3) / 4;
    if (algo != 0) return hipErrorInvalidValue;
    const int Tp = cnmf_solve_pipe_tiles(K, per);
    const bool pipe = variant == 3 && Tp > 0 && conv_mode == 1 && nsplit <= 1 && !gsrc &&
                      l1_num == 0.f && l1_den == 0.f && l2 == 0.f;
    if (pipe) {
      const int rpl = reps_per_launch > 0 ? reps_per_launch : nblocks;
      if (p.pipe_map < 0) {
        // XCD-grouped slices (one L2 for a replicate's exchanges: the objective checks
        // cost ~half) when the launch runs in ONE round and each XCD's share fits its
        // resident budget.  Measured (profiles/r4za_*): headline 13,133-13,198 ->
        // 13,482-13,535 rep/s, K=5..13 grid 18,972 -> 19,677; launches in several rounds
        // (K = 20 / 30 usage side) lost with it (r4g, r4z), so they keep the plain order
        static int n_cu[16] = {0};
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (dev < 0 || dev >= 16) dev = 0;
        if (n_cu[dev] == 0) {
          int v = 0;
          if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
              v <= 0)
            v = 256;
          n_cu[dev] = v;
        }
        const int S = coop_split > 1 ? coop_split : 1;
        const long long per_xcd = (long long)cnmf_solve_pipe_wg_per_cu(K) * n_cu[dev] / 8;
        p.pipe_map = (S > 1 && rpl >= nblocks && (long long)((rpl + 7) / 8) * S <= per_xcd) ? 1 : 0;
      }
      for (int r0 = 0; r0 < nblocks; r0 += rpl) {
        p.rep0 = r0;
        const hipError_t e = cnmf::launch_solve_pipe(K, p, nblocks - r0 < rpl ? nblocks - r0 : rpl,
                                                     Tp, p.pl_n, stream);
        if (e != hipSuccess) return e;
      }
      return hipSuccess;
    }
    if (reps_per_launch > 0 && reps_per_launch < nblocks) return hipErrorInvalidValue;
    if (per > cnmf_solve_mfma_max_cols(K)) return hipErrorInvalidValue;
    // the fused operands exist only in the pipelined kernel: never drop them silently
    if (fused || (!gram && !gsrc)) return hipErrorInvalidValue;
    return cnmf::launch_solve_mfma(K, p, nblocks, T < 1 ? 1 : T, stream);
  }
  if (fused || !gram) return hipErrorInvalidValue;
  // K > 64: the matrix-core wide solve, MU only (HALS is Gauss-Seidel over components).
  // Split-bf16 Gram apply at K = 96 / 128 (whole 32-deep k-blocks); fp32 MFMA at 80 / 112
  // and under variant 1 (streaming): padding those to 96 / 128 inside the kernel cost
  // occupancy and measured slower (profiles/r3af_*)
  if (K > 64)
    return algo == 0 ? cnmf::launch_solve_wmfma(K, p, nblocks, variant != 1 && K % 32 == 0, stream)
                     : hipErrorInvalidValue;
  if (K > 32) return cnmf::launch_solve_wide(K, algo, p, nblocks, threads, stream);
  // variant: 0 auto, 1 streaming, 2 register-resident (3 = mfma above).  Resident needs every slice to
  // fit U <= res_max_cols(K) columns per thread of a <= 1024-thread workgroup; it runs
  // with the smallest such U and just enough threads for the slice.
  const int parts = nsplit > 1 ? nsplit : (coop_split > 1 ? coop_split : 1);
  const int per = (ncols + parts - 1) / parts;
  const int U = per <= 1024 ? 1 : (per + 1023) / 1024;
  const bool fits = K <= cnmf::kResidentMaxK && U <= cnmf::res_max_cols(K);
  if (variant == 2 && !fits) return hipErrorInvalidValue;
  if ((variant == 0 && fits) || variant == 2) {
    int t_res = (((per + U - 1) / U + 63) / 64) * 64;
    if (t_res < 64) t_res = 64;
    return cnmf::launch_solve_resident(K, U, algo, p, nblocks, t_res, stream);
  }
  return cnmf::launch_solve_stream(K, algo, p, nblocks, threads, stream);
}
