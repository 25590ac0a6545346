// pybind11 entry points for the HIP kernels.  No torch headers: the Python ops layer
// (cnmf_torch_amd/ops/__init__.py) validates shapes, dtypes, devices and strides on
// the host and hands raw device pointers plus the current HIP stream here.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "kernels/launchers.h"

namespace py = pybind11;

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
static T* P(uintptr_t v) { return reinterpret_cast<T*>(v); }

PYBIND11_MODULE(_hip, m) {
  m.doc() = "cnmf_torch_amd native HIP kernels (gfx950)";

  m.def("cu_count", [](int dev) {
    int v = 0;
    check(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev),
          "hipDeviceGetAttribute");
    return v;
  });
  m.def("solve_max_k", []() { return cnmf_solve_max_k(); });
  m.def("solve_max_threads", [](int K) { return cnmf_solve_max_threads(K); });
  m.def("solve_native_k", [](int K) { return cnmf_solve_native_k(K); });
  m.def("solve_reg_max_cols", [](int K) { return cnmf_solve_reg_max_cols(K); });
  m.def("solve_mfma_max_cols", [](int K) { return cnmf_solve_mfma_max_cols(K); });
  m.def("solve_pipe_tiles", [](int K, int per) { return cnmf_solve_pipe_tiles(K, per); });
  m.def("solve_pipe_k", [](int K) { return cnmf_solve_pipe_k(K); });
  m.def("exact_moments",
        [](uintptr_t X, int is_f64, long long ld, long long rows, int G, int chunks,
           uintptr_t part, uintptr_t out, uintptr_t bad, uintptr_t stream) {
          check(cnmf_exact_moments(reinterpret_cast<const void*>(X), is_f64, ld, rows, G, chunks,
                                   P<long long>(part), P<long long>(out),
                                   P<unsigned long long>(bad),
                                   reinterpret_cast<hipStream_t>(stream)),
                "cnmf_exact_moments");
        });
  m.def("ridge_seg_tgemm",
        [](uintptr_t Rt, long long ldr, int Kc, uintptr_t X, int x_f64, long long ldx, int F,
           uintptr_t idx, uintptr_t seg, int nseg, uintptr_t out, long long seg_stride,
           long long ldo, uintptr_t stream) {
          check(cnmf_ridge_seg_tgemm(P<const double>(Rt), ldr, Kc, reinterpret_cast<const void*>(X),
                                     x_f64, ldx, F, P<const int>(idx), P<const long long>(seg),
                                     nseg, P<double>(out), seg_stride, ldo,
                                     reinterpret_cast<hipStream_t>(stream)),
                "cnmf_ridge_seg_tgemm");
        });
  m.def("ridge_seg_reduce",
        [](uintptr_t part, uintptr_t cfirst, int nseg, int Kc, int F, uintptr_t out,
           long long seg_stride, long long ldo, uintptr_t stream) {
          check(cnmf_ridge_seg_reduce(P<const double>(part), P<const int>(cfirst), nseg, Kc, F,
                                      P<double>(out), seg_stride, ldo,
                                      reinterpret_cast<hipStream_t>(stream)),
                "cnmf_ridge_seg_reduce");
        });
  m.def("ridge_apply",
        [](uintptr_t Rt, long long ldr, int Kc, uintptr_t X, int x_f64, long long ldx, uintptr_t Y,
           long long ldy, int F, uintptr_t order, uintptr_t blk, int nblk, uintptr_t Wc,
           long long wc_combo, long long ldw, uintptr_t stream) {
          check(cnmf_ridge_apply(P<const double>(Rt), ldr, Kc, reinterpret_cast<const void*>(X),
                                 x_f64, ldx, reinterpret_cast<void*>(Y), ldy, F, P<const int>(order),
                                 P<const int>(blk), nblk, P<const double>(Wc), wc_combo, ldw,
                                 reinterpret_cast<hipStream_t>(stream)),
                "cnmf_ridge_apply");
        });
  m.def("predict_err",
        [](uintptr_t X, long long ldx, uintptr_t U, long long ldu, uintptr_t S, long long lds,
           int N, int G, int K, uintptr_t part, uintptr_t stream) {
          check(cnmf_predict_err(P<const float>(X), ldx, P<const double>(U), ldu,
                                 P<const double>(S), lds, N, G, K, P<double>(part),
                                 reinterpret_cast<hipStream_t>(stream)),
                "cnmf_predict_err");
        });
  m.def("solve_pipe_max_cols", [](int K) { return cnmf_solve_pipe_max_cols(K); });
  m.def("solve_pipe_wg_per_cu", [](int K) { return cnmf_solve_pipe_wg_per_cu(K); });

  m.def("solve",
        [](int algo, int K, uintptr_t x, long long x_rs, long long ldx, uintptr_t numer,
           long long n_rs, long long ldn, uintptr_t gram, long long g_rs, uintptr_t rep_index,
           int nblocks, int ncols, int max_iter, float tol, float l1_num, float l1_den, float l2,
           float eps, uintptr_t lin_out, uintptr_t quad_out, uintptr_t iters_out, int nsplit,
           int conv_mode, int check_every, int threads, int variant, uintptr_t active,
           int coop_split, uintptr_t coop_slots, uintptr_t coop_count, unsigned coop_gen,
           int coop_epochs,
           uintptr_t coop_timeout, uintptr_t planes, long long pl_rs, long long pl_ld,
           long long pl_plane, uintptr_t pl_colmul, int pl_cols, int pl_n, uintptr_t gsrc,
           long long gs_rs, long long gs_ld, int gs_cols, int nslab_n, long long nslab_stride,
           uintptr_t n_scale, uintptr_t nbase, uintptr_t nout, long long nb_rs, long long ldnb,
           uintptr_t gpart, int gpart_n, long long gpart_rs, uintptr_t gout, uintptr_t gp_out,
           long long gp_rs, uintptr_t coop_gen_dev, uintptr_t coop_arrive, int reps_per_launch,
           uintptr_t stamps, uintptr_t stream) {
          check(cnmf_solve(algo, K, P<float>(x), x_rs, ldx, P<const float>(numer), n_rs, ldn,
                           P<const float>(gram), g_rs, P<const int>(rep_index), nblocks, ncols,
                           max_iter, tol, l1_num, l1_den, l2, eps, P<float>(lin_out),
                           P<float>(quad_out), P<int>(iters_out), nsplit, conv_mode,
                           check_every, threads, variant, P<const int>(active), coop_split,
                           P<float>(coop_slots), P<unsigned long long>(coop_count), coop_gen,
                           coop_epochs,
                           P<int>(coop_timeout), P<unsigned short>(planes), pl_rs, pl_ld,
                           pl_plane, P<const float>(pl_colmul), pl_cols, pl_n,
                           P<const float>(gsrc), gs_rs, gs_ld, gs_cols, nslab_n, nslab_stride,
                           P<const float>(n_scale), P<const float>(nbase), P<float>(nout), nb_rs,
                           ldnb, P<const float>(gpart), gpart_n, gpart_rs, P<float>(gout),
                           P<float>(gp_out), gp_rs, P<unsigned>(coop_gen_dev),
                           P<unsigned>(coop_arrive), reps_per_launch,
                           P<unsigned long long>(stamps), reinterpret_cast<hipStream_t>(stream)),
                "cnmf_solve");
        });

  // continuous batching: the swap block in StreamSwap field order (ints, then pointers /
  // strides as 64-bit integers; ops.stream_swap builds the list)
  m.def("stream_swap", [](py::sequence v, int chunks, uintptr_t stream) {
    if (py::len(v) != 41) throw std::runtime_error("stream_swap: 41 fields expected");
    auto I = [&](int i) { return v[i].cast<long long>(); };
    cnmf::StreamSwap p;
    int i = 0;
    p.n = (int)I(i++); p.K = (int)I(i++); p.G = (int)I(i++); p.N = (int)I(i++);
    p.S = (int)I(i++); p.Gp = (int)I(i++);
    p.active = P<const int>(I(i++)); p.occ = P<int>(I(i++)); p.plan = P<int>(I(i++));
    p.sf = P<double>(I(i++)); p.sf_ld = I(i++); p.si = P<int>(I(i++)); p.si_ld = I(i++);
    p.W = P<float>(I(i++)); p.ldw = I(i++); p.HT = P<float>(I(i++)); p.ldh = I(i++);
    p.parts = P<float>(I(i++));
    p.wpl = P<unsigned short>(I(i++)); p.pl_ld = I(i++); p.pl_plane = I(i++);
    p.qc = (int)I(i++); p.head = P<int>(I(i++)); p.tail = P<const int>(I(i++));
    p.ring_id = P<const int>(I(i++)); p.rW = P<const float>(I(i++));
    p.rHT = P<const float>(I(i++)); p.rsf = P<const double>(I(i++));
    p.rsi = P<const int>(I(i++)); p.rparts = P<const float>(I(i++));
    p.rwpl = P<const unsigned short>(I(i++)); p.rpl_plane = I(i++);
    p.offs = P<const long long>(I(i++)); p.oW = P<float>(I(i++)); p.oHT = P<float>(I(i++));
    p.osf = P<double>(I(i++)); p.osf_ld = I(i++); p.osi = P<int>(I(i++)); p.osi_ld = I(i++);
    p.done = P<int>(I(i++)); p.gate = P<int>(I(i++));
    (void)i;
    check(cnmf_stream_swap(&p, chunks, reinterpret_cast<hipStream_t>(stream)),
          "cnmf_stream_swap");
  });

  // in-place compaction swap: pairs ptr, K, [(ptr, ld, plane, cols, esz, planes) x nmat],
  // (sf, sf_ld, nsf), (si, si_ld, nsi)
  m.def("rows_swap", [](uintptr_t pairs, int npairs, int K, py::sequence mats, uintptr_t sf,
                        long long sf_ld, int nsf, uintptr_t si, long long si_ld, int nsi,
                        int chunks, uintptr_t stream) {
    cnmf::RowsSwap p{};
    p.K = K;
    p.pairs = P<const int>(pairs);
    p.nmat = (int)py::len(mats);
    if (p.nmat > 4) throw std::runtime_error("rows_swap: at most 4 matrices");
    for (int m_ = 0; m_ < p.nmat; ++m_) {
      py::sequence q = mats[m_];
      if (py::len(q) != 6) throw std::runtime_error("rows_swap: 6 fields per matrix");
      p.mat[m_].p = reinterpret_cast<void*>(q[0].cast<uintptr_t>());
      p.mat[m_].ld = q[1].cast<long long>();
      p.mat[m_].plane = q[2].cast<long long>();
      p.mat[m_].cols = q[3].cast<int>();
      p.mat[m_].esz = q[4].cast<int>();
      p.mat[m_].planes = q[5].cast<int>();
    }
    p.sf = P<double>(sf); p.sf_ld = sf_ld; p.nsf = nsf;
    p.si = P<int>(si); p.si_ld = si_ld; p.nsi = nsi;
    check(cnmf_rows_swap(&p, npairs, chunks, reinterpret_cast<hipStream_t>(stream)),
          "cnmf_rows_swap");
  });

  m.def("stream_publish", [](uintptr_t ctr, int n, uintptr_t seq, uintptr_t mail, int slots,
                             int width, uintptr_t stream) {
    check(cnmf_stream_publish(P<const int>(ctr), n, P<int>(seq), P<int>(mail), slots, width,
                              reinterpret_cast<hipStream_t>(stream)),
          "cnmf_stream_publish");
  });
  // device address of pinned host memory (kernels write host mailboxes directly)
  m.def("host_dev_ptr", [](uintptr_t host) {
    void* d = nullptr;
    check(hipHostGetDevicePointer(&d, reinterpret_cast<void*>(host), 0), "hipHostGetDevicePointer");
    return reinterpret_cast<uintptr_t>(d);
  });

  m.def("conv_update",
        [](uintptr_t lin, uintptr_t quad, double x_sq, uintptr_t err_init, uintptr_t err_prev,
           uintptr_t err, uintptr_t active, uintptr_t converged, uintptr_t n_pass, int n,
           int pass, double tol, int final_pass, int init, uintptr_t gate, int max_pass,
           uintptr_t hflags, uintptr_t hcnt, uintptr_t stream) {
          check(cnmf_conv_update(P<const float>(lin), P<const float>(quad), x_sq,
                                 P<double>(err_init), P<double>(err_prev), P<double>(err),
                                 P<int>(active), P<int>(converged), P<int>(n_pass), n, pass, tol,
                                 final_pass, init, P<int>(gate), max_pass, P<int>(hflags),
                                 P<int>(hcnt), reinterpret_cast<hipStream_t>(stream)),
                "cnmf_conv_update");
        });

  m.def("beta_max_k", []() { return cnmf_beta_max_k(); });
  m.def("beta_contract",
        [](int side, int mode, uintptr_t X, long long ldx, uintptr_t HT, long long h_rs,
           long long ldh, uintptr_t W, long long w_rs, long long ldw, int N, int G, int K, int R,
           float beta, float eps, uintptr_t num, uintptr_t den, uintptr_t loss, uintptr_t active,
           int splits, int upd, uintptr_t den_vec, float l1, float l2, float gamma, float tol,
           uintptr_t part, uintptr_t counter, uintptr_t act, uintptr_t iters, int conv_mode,
           int check_every, uintptr_t hstate, uintptr_t stream) {
          check(cnmf_beta_contract(side, mode, P<const float>(X), ldx, P<const float>(HT), h_rs,
                                   ldh, P<const float>(W), w_rs, ldw, N, G, K, R, beta, eps,
                                   P<float>(num), P<float>(den), P<double>(loss),
                                   P<const int>(active), splits, upd, P<const float>(den_vec),
                                   l1, l2, gamma, tol, P<float>(part), P<int>(counter),
                                   P<int>(act), P<int>(iters), conv_mode, check_every,
                                   P<double>(hstate), reinterpret_cast<hipStream_t>(stream)),
                "beta_contract");
        });
  m.def("beta_w_update_blocks", [](int K, int G) { return cnmf_beta_w_update_blocks(K, G); });
  m.def("beta_w_update",
        [](int mode, uintptr_t W, long long w_rs, long long ldw, uintptr_t num, uintptr_t den,
           uintptr_t hsum, uintptr_t An, uintptr_t Ad, uintptr_t an_out, uintptr_t dn_out, int R,
           int K, int G, int splits, float gamma, float l1, float l2, float eps, float tol,
           uintptr_t part, uintptr_t counter, uintptr_t act, uintptr_t iters, uintptr_t stream) {
          check(cnmf_beta_w_update(mode, P<float>(W), w_rs, ldw, P<const float>(num),
                                   P<const float>(den), P<const float>(hsum), P<const float>(An),
                                   P<const float>(Ad), P<float>(an_out), P<float>(dn_out), R, K,
                                   G, splits, gamma, l1, l2, eps, tol, P<float>(part),
                                   P<int>(counter), P<int>(act), P<int>(iters),
                                   reinterpret_cast<hipStream_t>(stream)),
                "beta_w_update");
        });

  m.def("bp_max_k", []() { return cnmf_bp_max_k(); });
  m.def("bp_panel_elems",
        [](int K, int L, int mode) { return cnmf_bp_panel_elems(K, L, mode); });
  m.def("bp_strip_cols", [](int K, int mode) { return cnmf_bp_strip_cols(K, mode); });
  m.def("bp_splits", [](int Ls, int splits) { return cnmf_bp_splits(Ls, splits); });
  m.def("bp_panels",
        [](uintptr_t F, long long f_rs, long long ldf, int K, int L, int R, int mode,
           uintptr_t prow, uintptr_t out, long long out_rs, uintptr_t stream) {
          check(cnmf_bp_panels(P<const float>(F), f_rs, ldf, K, L, R, mode, P<const float>(prow),
                               P<unsigned short>(out),
                               out_rs, reinterpret_cast<hipStream_t>(stream)),
                "bp_panels");
        });
  m.def("bp_run",
        [](int side, int mode, uintptr_t X, long long ldx, uintptr_t panel, long long panel_rs,
           uintptr_t F, long long f_rs, long long ldf, int K, int Lf, int Ls, int R, int splits,
           float beta, float eps, uintptr_t num, uintptr_t den, int nsteps, int loss_entry,
           int loss_exit, uintptr_t den_vec, float l1, float l2, float gamma, float tol,
           int conv_mode, uintptr_t hstate, uintptr_t part, uintptr_t counter, uintptr_t act,
           uintptr_t iters, uintptr_t active, uintptr_t loss, double xsum, int xh,
           uintptr_t uvec, uintptr_t fscale, uintptr_t stream) {
          check(cnmf_bp_run(side, mode, P<const float>(X), ldx, P<const unsigned short>(panel),
                            panel_rs, P<float>(F), f_rs, ldf, K, Lf, Ls, R, splits, beta, eps,
                            P<float>(num), P<float>(den), nsteps, loss_entry, loss_exit,
                            P<const float>(den_vec), l1, l2, gamma, tol, conv_mode,
                            P<double>(hstate), P<double>(part), P<int>(counter), P<int>(act),
                            P<int>(iters), P<const int>(active), P<double>(loss), xsum, xh,
                            P<const float>(uvec), P<const float>(fscale),
                            reinterpret_cast<hipStream_t>(stream)),
                "bp_run");
        });
  m.def("sk_k4", [](int K) { return cnmf_sk_k4(K); });
  m.def("sk_groups", [](int Lf, int R, int Ls, int K) { return cnmf_sk_groups(Lf, R, Ls, K); });
  m.def("sk_lds", [](int Ls, int K) { return cnmf_sk_lds(Ls, K); });
  m.def("sk_run",
        [](int side, uintptr_t rowptr, uintptr_t col, uintptr_t val, uintptr_t ST,
           long long st_rs, uintptr_t F, long long f_rs, long long ldf, int K, int Lf, int Ls,
           int R, float eps, uintptr_t num, int nsteps, int loss_entry, int loss_exit,
           uintptr_t den_vec, float l1, float l2, float tol, int conv_mode, uintptr_t hstate,
           uintptr_t part, uintptr_t counter, uintptr_t act, uintptr_t iters, uintptr_t active,
           uintptr_t loss, double xsum, uintptr_t stream) {
          check(cnmf_sk_run(side, P<const int>(rowptr), P<const int>(col), P<const float>(val),
                            P<const float>(ST), st_rs, P<float>(F), f_rs, ldf, K, Lf, Ls, R, eps,
                            P<float>(num), nsteps, loss_entry, loss_exit,
                            P<const float>(den_vec), l1, l2, tol, conv_mode, P<double>(hstate),
                            P<double>(part), P<int>(counter), P<int>(act), P<int>(iters),
                            P<const int>(active), P<double>(loss), xsum,
                            reinterpret_cast<hipStream_t>(stream)),
                "sk_run");
        });

  m.def("pairdist", [](uintptr_t A, long long lda, uintptr_t B, long long ldb, uintptr_t na,
                       uintptr_t nb, int n, int mm, int kdim, uintptr_t D, long long ldd, int same,
                       int squared, uintptr_t stream) {
    check(cnmf_pairdist(P<const double>(A), lda, P<const double>(B), ldb, P<const double>(na),
                        P<const double>(nb), n, mm, kdim, P<double>(D), ldd, same, squared,
                        reinterpret_cast<hipStream_t>(stream)),
          "pairdist");
  });
  m.def("knn_sum", [](uintptr_t D, long long ldd, int n, int mm, int k, uintptr_t out,
                      uintptr_t stream) {
    check(cnmf_knn_sum(P<const double>(D), ldd, n, mm, k, P<double>(out),
                       reinterpret_cast<hipStream_t>(stream)),
          "knn_sum");
  });
  m.def("small_gram", [](uintptr_t A, long long s_i, long long s_a, int n, int K, int esz,
                         int rows_per, uintptr_t part, uintptr_t stream) {
    check(cnmf_small_gram(reinterpret_cast<const void*>(A), s_i, s_a, n, K, esz, rows_per,
                          reinterpret_cast<void*>(part), reinterpret_cast<hipStream_t>(stream)),
          "small_gram");
  });
  m.def("seg_colsum", [](uintptr_t X, long long ldx, int n, int d, uintptr_t lab, long long ldl,
                         int nrest, int k, uintptr_t out, uintptr_t stream) {
    check(cnmf_seg_colsum(P<const double>(X), ldx, n, d, P<const int>(lab), ldl, nrest, k,
                          P<double>(out), reinterpret_cast<hipStream_t>(stream)),
          "seg_colsum");
  });
  m.def("seg_rowsum", [](uintptr_t D, long long ldd, int n, int m_, uintptr_t lab, int k,
                         uintptr_t out, long long ldo, uintptr_t stream) {
    check(cnmf_seg_rowsum(P<const double>(D), ldd, n, m_, P<const int>(lab), k, P<double>(out),
                          ldo, reinterpret_cast<hipStream_t>(stream)),
          "seg_rowsum");
  });
  m.def("seg_argmin", [](uintptr_t D, long long ldd, int n, int nseg, int k, uintptr_t row_add,
                         uintptr_t col_add, uintptr_t labels, uintptr_t mind, uintptr_t stream) {
    check(cnmf_seg_argmin(P<const double>(D), ldd, n, nseg, k, P<const double>(row_add),
                          P<const double>(col_add), P<int>(labels), P<double>(mind),
                          reinterpret_cast<hipStream_t>(stream)),
          "seg_argmin");
  });

  m.def("kmeans_blocks", [](int n) { return cnmf_kmeans_blocks(n); });
  m.def("kmeanspp_blocks", [](int n) { return cnmf_kmeanspp_blocks(n); });
  m.def("kmeanspp_sample_blocks", [](int n) { return cnmf_kmeanspp_sample_blocks(n); });
  m.def("kmeanspp_sample", [](uintptr_t closest, int n, int n_init, uintptr_t u, int trials,
                              uintptr_t bsum, uintptr_t cand, uintptr_t stream) {
    check(cnmf_kmeanspp_sample(P<const double>(closest), n, n_init, P<const double>(u), trials,
                               P<double>(bsum), P<long long>(cand),
                               reinterpret_cast<hipStream_t>(stream)),
          "kmeanspp_sample");
  });
  m.def("kmeanspp_fits", [](int M, int d) { return cnmf_kmeanspp_fits(M, d); });
  m.def("kmeanspp", [](uintptr_t X, long long ldx, int n, int d, uintptr_t C, int M, int trials,
                       uintptr_t closest, int n_init, int mode, uintptr_t pot, uintptr_t stream) {
    check(cnmf_kmeanspp(P<const double>(X), ldx, n, d, P<const double>(C), M, trials,
                        P<double>(closest), n_init, mode, P<double>(pot),
                        reinterpret_cast<hipStream_t>(stream)),
          "kmeanspp");
  });
  m.def("kmeans_fits", [](int k, int d) { return cnmf_kmeans_fits(k, d); });
  m.def("kmeans_step", [](uintptr_t X, long long ldx, int n, int d, uintptr_t C, int k,
                          int n_init, uintptr_t live, uintptr_t labels, uintptr_t mind,
                          uintptr_t psum, uintptr_t pcnt, uintptr_t stream) {
    check(cnmf_kmeans_step(P<const double>(X), ldx, n, d, P<const double>(C), k, n_init,
                           P<const int>(live), P<int>(labels), P<double>(mind), P<double>(psum),
                           P<double>(pcnt), reinterpret_cast<hipStream_t>(stream)),
          "kmeans_step");
  });

  m.def("csr_row_sums", [](uintptr_t indptr, uintptr_t data, int f64, int n, uintptr_t out,
                           uintptr_t stream) {
    check(cnmf_csr_row_sums(P<const long long>(indptr), P<const void>(data), f64, n,
                            P<double>(out), reinterpret_cast<hipStream_t>(stream)),
          "csr_row_sums");
  });
  m.def("csr_stats_blocks", [](int n) { return cnmf_csr_stats_blocks(n); });
  m.def("csr_col_stats",
        [](uintptr_t indptr, uintptr_t indices, uintptr_t data, int f64, int n, int n_out,
           uintptr_t row_scale, uintptr_t col_map, uintptr_t col_div, uintptr_t clip,
           double max_value, int round_mid, uintptr_t center, uintptr_t psum, uintptr_t psq,
           uintptr_t pcnt, uintptr_t stream) {
          check(cnmf_csr_col_stats(P<const long long>(indptr), P<const int>(indices),
                                   P<const void>(data), f64, n, n_out,
                                   P<const double>(row_scale), P<const int>(col_map),
                                   P<const double>(col_div), P<const double>(clip), max_value,
                                   round_mid, P<const double>(center), P<double>(psum),
                                   P<double>(psq), P<double>(pcnt),
                                   reinterpret_cast<hipStream_t>(stream)),
                "csr_col_stats");
        });
  m.def("csr_transform",
        [](uintptr_t indptr, uintptr_t indices, uintptr_t data, int f64, int n,
           uintptr_t row_scale, uintptr_t col_map, uintptr_t col_div, uintptr_t clip,
           double max_value, int round_mid, uintptr_t out, int out_f64, uintptr_t stream) {
          check(cnmf_csr_transform(P<const long long>(indptr), P<const int>(indices),
                                   P<const void>(data), f64, n, P<const double>(row_scale),
                                   P<const int>(col_map), P<const double>(col_div),
                                   P<const double>(clip), max_value, round_mid, P<void>(out),
                                   out_f64, reinterpret_cast<hipStream_t>(stream)),
                "csr_transform");
        });
  m.def("csr_densify",
        [](uintptr_t indptr, uintptr_t indices, uintptr_t data, int f64, int n,
           uintptr_t row_scale, uintptr_t col_map, uintptr_t col_div, uintptr_t clip,
           double max_value, int round_mid, uintptr_t out, int out_f64, long long ldo,
           uintptr_t stream) {
          check(cnmf_csr_densify(P<const long long>(indptr), P<const int>(indices),
                                 P<const void>(data), f64, n, P<const double>(row_scale),
                                 P<const int>(col_map), P<const double>(col_div),
                                 P<const double>(clip), max_value, round_mid, P<void>(out),
                                 out_f64, ldo, reinterpret_cast<hipStream_t>(stream)),
                "csr_densify");
        });
  m.def("csr_spmm",
        [](uintptr_t indptr, uintptr_t indices, uintptr_t data, int f64, int n,
           uintptr_t row_scale, uintptr_t col_map, uintptr_t col_div, uintptr_t clip,
           double max_value, int round_mid, uintptr_t B, int K, uintptr_t out, uintptr_t stream) {
          check(cnmf_csr_spmm(P<const long long>(indptr), P<const int>(indices),
                              P<const void>(data), f64, n, P<const double>(row_scale),
                              P<const int>(col_map), P<const double>(col_div),
                              P<const double>(clip), max_value, round_mid, P<const float>(B), K,
                              P<float>(out), reinterpret_cast<hipStream_t>(stream)),
                "csr_spmm");
        });
  m.def("csr_tspmm_blocks", [](int n) { return cnmf_csr_tspmm_blocks(n); });
  m.def("csr_tspmm",
        [](uintptr_t indptr, uintptr_t indices, uintptr_t data, int f64, int n, int n_out,
           uintptr_t row_scale, uintptr_t col_map, uintptr_t col_div, uintptr_t clip,
           double max_value, int round_mid, uintptr_t B, int b_f64, int K, uintptr_t part,
           uintptr_t stream) {
          check(cnmf_csr_tspmm(P<const long long>(indptr), P<const int>(indices),
                               P<const void>(data), f64, n, n_out, P<const double>(row_scale),
                               P<const int>(col_map), P<const double>(col_div),
                               P<const double>(clip), max_value, round_mid, P<const void>(B),
                               b_f64, K, P<double>(part), reinterpret_cast<hipStream_t>(stream)),
                "csr_tspmm");
        });
  m.def("radix_hist", [](uintptr_t x, long long m, unsigned prefix, unsigned mask, int shift,
                         uintptr_t hist, uintptr_t stream) {
    check(cnmf_radix_hist(P<const float>(x), m, prefix, mask, shift,
                          P<unsigned long long>(hist), reinterpret_cast<hipStream_t>(stream)),
          "radix_hist");
  });

  m.def("harmony_max_kb", []() { return cnmf_harmony_max_kb(); });
  m.def("harmony_block", [](int op, uintptr_t Rt, uintptr_t distT, uintptr_t sigma,
                            uintptr_t cells, uintptr_t bidx, int nb, int N, int K, int B,
                            int nvar, int chunk, uintptr_t E, uintptr_t O, uintptr_t Pr_b,
                            uintptr_t theta, uintptr_t Pen, uintptr_t part, uintptr_t Y,
                            uintptr_t Zt, int d, uintptr_t obj, uintptr_t stream) {
    check(cnmf_harmony_block(op, P<double>(Rt), P<const double>(distT), P<const double>(sigma),
                             P<const int>(cells), P<const int>(bidx), nb, N, K, B, nvar, chunk,
                             P<double>(E), P<double>(O), P<const double>(Pr_b),
                             P<const double>(theta), P<double>(Pen), P<double>(part),
                             P<const double>(Y), P<const double>(Zt), d, P<double>(obj),
                             reinterpret_cast<hipStream_t>(stream)),
          "harmony_block");
  });
  m.def("harmony_centroid_max_d", []() { return cnmf_harmony_centroid_max_d(); });
  m.def("harmony_centroid", [](uintptr_t Zt, uintptr_t Rt, int N, int d, int K, int chunk,
                               uintptr_t part, uintptr_t Y, uintptr_t stream) {
    check(cnmf_harmony_centroid(P<const double>(Zt), P<const double>(Rt), N, d, K, chunk,
                                P<double>(part), P<double>(Y),
                                reinterpret_cast<hipStream_t>(stream)),
          "harmony_centroid");
  });
  m.def("harmony_objective", [](uintptr_t O, uintptr_t E, uintptr_t sigma, uintptr_t theta,
                                int K, int B, uintptr_t obj, uintptr_t out, uintptr_t stream) {
    check(cnmf_harmony_objective(P<const double>(O), P<const double>(E), P<const double>(sigma),
                                 P<const double>(theta), K, B, P<double>(obj), P<double>(out),
                                 reinterpret_cast<hipStream_t>(stream)),
          "harmony_objective");
  });

  m.def("beta_any_rows", []() { return cnmf_beta_any_rows(); });
  m.def("beta_any_terms", [](int mode, uintptr_t X, long long ldx, uintptr_t Pm, uintptr_t D, int m_,
                             int c, int G, float beta, float eps, uintptr_t act, int want_q,
                             uintptr_t part, uintptr_t stream) {
    check(cnmf_beta_any_terms(mode, P<const float>(X), ldx, P<float>(Pm), P<float>(D), m_, c, G,
                              beta, eps, P<const int>(act), want_q, P<double>(part),
                              reinterpret_cast<hipStream_t>(stream)),
          "beta_any_terms");
  });
  m.def("solve_any_hals_max_k", []() { return cnmf_solve_any_hals_max_k(); });
  m.def("solve_any", [](int op, uintptr_t x, long long x_rs, long long ldx, uintptr_t numer,
                        long long n_rs, long long ldn, uintptr_t D, uintptr_t G, long long g_rs,
                        uintptr_t reps, uintptr_t act, int m_, int K, int n, int per,
                        float l1_num, float l1_den, float l2, float eps, uintptr_t part,
                        uintptr_t iters, uintptr_t stream) {
    check(cnmf_solve_any(op, P<float>(x), x_rs, ldx, P<const float>(numer), n_rs, ldn,
                         P<const float>(D), P<const float>(G), g_rs, P<const int>(reps),
                         P<int>(act), m_, K, n, per, l1_num, l1_den, l2, eps, P<double>(part),
                         P<int>(iters), reinterpret_cast<hipStream_t>(stream)),
          "solve_any");
  });
  m.def("solve_any_conv", [](int mode, uintptr_t part, int nblk, int m_, uintptr_t act,
                             uintptr_t act0, uintptr_t reps, uintptr_t f_prev, int have_prev,
                             float tol, float eps, uintptr_t lin_out, uintptr_t quad_out,
                             uintptr_t stream) {
    check(cnmf_solve_any_conv(mode, P<const double>(part), nblk, m_, P<int>(act),
                              P<const int>(act0), P<const int>(reps), P<double>(f_prev),
                              have_prev, tol, eps, P<float>(lin_out), P<float>(quad_out),
                              reinterpret_cast<hipStream_t>(stream)),
          "solve_any_conv");
  });
  m.def("gram", [](uintptr_t X, long long x_rs, long long ldx, int R, int K, int n,
                   uintptr_t out, long long o_rs, int accumulate, uintptr_t active,
                   uintptr_t part, int S, uintptr_t stream) {
    check(cnmf_gram(P<const float>(X), x_rs, ldx, R, K, n, P<float>(out), o_rs, accumulate,
                    P<const int>(active), P<float>(part), S,
                    reinterpret_cast<hipStream_t>(stream)),
          "gram");
  });

  m.def("philox_fill",
        [](uintptr_t out, long long rows, long long cols, long long s_row, long long s_col,
           long long rep_stride, long long row_offset, uintptr_t seeds, uintptr_t scales, int R,
           unsigned stream_id, int mode, uintptr_t stream) {
          check(cnmf_philox_fill(P<float>(out), rows, cols, s_row, s_col, rep_stride, row_offset,
                                 P<const unsigned long long>(seeds), P<const float>(scales), R,
                                 stream_id, mode, reinterpret_cast<hipStream_t>(stream)),
                "cnmf_philox_fill");
        });

  m.def("seg_median_max_rows", []() { return cnmf_seg_median_max_rows(); });
  m.def("seg_median_max_clusters", []() { return cnmf_seg_median_max_clusters(); });
  m.def("seg_median", [](uintptr_t S, long long lds, int n, int G, uintptr_t perm, uintptr_t seg,
                         int k, uintptr_t out, long long ldo, uintptr_t stream) {
    check(cnmf_seg_median(P<const double>(S), lds, n, G, P<const int>(perm), P<const int>(seg),
                          k, P<double>(out), ldo, reinterpret_cast<hipStream_t>(stream)),
          "seg_median");
  });
  m.def("gemm_planes_bk", [](int pb) { return cnmf_gemm_planes_bk(pb); });
  m.def("gemm_planes_tile", [](int v, int which) { return cnmf_gemm_planes_tile(v, which); });
  m.def("gemm_planes",
        [](uintptr_t A, long long lda, long long a_plane, int a_rows, uintptr_t B,
           long long ldb, long long b_plane, int b_rows, uintptr_t C, long long ldc,
           uintptr_t col_scale, int M, int N, int Kd, int pa, int pb, int accumulate,
           int variant, int ksplit, uintptr_t slab, int stages, int kstep, int raw,
           uintptr_t gate, uintptr_t stream) {
          check(cnmf_gemm_planes(P<const unsigned short>(A), lda, a_plane, a_rows,
                                 P<const unsigned short>(B), ldb, b_plane, b_rows, P<float>(C),
                                 ldc, P<const float>(col_scale), M, N, Kd, pa, pb, accumulate,
                                 variant, ksplit, P<float>(slab), stages, kstep, raw,
                                 P<const int>(gate), reinterpret_cast<hipStream_t>(stream)),
                "cnmf_gemm_planes");
        });
  m.def("split_planes",
        [](uintptr_t S, long long lds, int rows, int cols, int cols_pad, uintptr_t col_mul,
           uintptr_t Pl, long long ldp, long long plane, int nplanes, uintptr_t stream) {
          check(cnmf_split_planes(P<const float>(S), lds, rows, cols, cols_pad,
                                  P<const float>(col_mul), P<unsigned short>(Pl), ldp, plane,
                                  nplanes, reinterpret_cast<hipStream_t>(stream)),
                "cnmf_split_planes");
        });

  m.def("colstats_blocks", [](int N) { return cnmf_colstats_blocks(N); });
  m.def("colstats",
        [](uintptr_t X, long long ldx, int N, int G, uintptr_t pmin, uintptr_t psq,
           uintptr_t pneg, uintptr_t mn, uintptr_t sq, uintptr_t neg, uintptr_t stream) {
          check(cnmf_colstats(P<const float>(X), ldx, N, G, P<float>(pmin), P<double>(psq),
                              P<int>(pneg), P<float>(mn), P<double>(sq), P<int>(neg),
                              reinterpret_cast<hipStream_t>(stream)),
                "cnmf_colstats");
        });
  m.def("count_unit_check",
        [](uintptr_t X, long long ldx, int N, int G, uintptr_t mn, uintptr_t bad,
           uintptr_t stream) {
          check(cnmf_count_unit_check(P<const float>(X), ldx, N, G, P<const float>(mn),
                                      P<unsigned>(bad), reinterpret_cast<hipStream_t>(stream)),
                "cnmf_count_unit_check");
        });

  // one-shot xGMI all-reduce (xgmi_allreduce.hip): workspace, IPC handles, launch
  m.def("xgmi_data_offset", []() { return cnmf_xgmi_data_offset(); });
  m.def("xgmi_max_ranks", []() { return cnmf_xgmi_max_ranks(); });
  m.def("xgmi_max_blocks", []() { return cnmf_xgmi_max_blocks(); });
  m.def("xgmi_alloc", [](long long cap) {
    void* p = nullptr;
    unsigned mode = 0;
    check(cnmf_xgmi_alloc(cap, &p, &mode), "cnmf_xgmi_alloc");
    return py::make_tuple(reinterpret_cast<uintptr_t>(p), mode);
  });
  m.def("ptr_alloc_flags", [](uintptr_t p) {
    unsigned f = 0;
    check(cnmf_ptr_alloc_flags(P<const void>(p), &f), "hipPointerGetAttributes");
    return f;
  });
  m.attr("MALLOC_UNCACHED") = (unsigned)hipDeviceMallocUncached;
  m.attr("MALLOC_FINEGRAINED") = (unsigned)hipDeviceMallocFinegrained;
  m.def("xgmi_free", [](uintptr_t p) { check(hipFree(P<void>(p)), "hipFree"); });
  m.def("xgmi_handle", [](uintptr_t p) {
    hipIpcMemHandle_t h;
    check(hipIpcGetMemHandle(&h, P<void>(p)), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  });
  m.def("xgmi_open", [](py::bytes b) {
    std::string s = b;
    hipIpcMemHandle_t h;
    if (s.size() != sizeof(h)) throw std::runtime_error("xgmi_open: bad IPC handle size");
    std::memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    return reinterpret_cast<uintptr_t>(p);
  });
  m.def("xgmi_close", [](uintptr_t p) {
    check(hipIpcCloseMemHandle(P<void>(p)), "hipIpcCloseMemHandle");
  });
  m.def("xgmi_wall_clock_khz", [](int dev) {
    int v = 0;
    check(hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev),
          "hipDeviceGetAttribute");
    return v;
  });
  m.def("xgmi_allreduce",
        [](uintptr_t peers, int world, int rank, uintptr_t in, uintptr_t out, long long n,
           long long cap, unsigned epoch, unsigned long long limit, uintptr_t timeout,
           int blocks, uintptr_t stream) {
          check(cnmf_xgmi_allreduce(P<const unsigned long long>(peers), world, rank,
                                    P<const float>(in), P<float>(out), n, cap, epoch, limit,
                                    P<int>(timeout), blocks,
                                    reinterpret_cast<hipStream_t>(stream)),
                "cnmf_xgmi_allreduce");
        });
  m.def("xgmi_collective",
        [](int mode, uintptr_t peers, int world, int rank, uintptr_t in, uintptr_t out,
           long long m, long long cap, unsigned epoch, uintptr_t ep, uintptr_t arrive,
           unsigned long long limit, uintptr_t timeout, int blocks, uintptr_t stream) {
          check(cnmf_xgmi_collective(mode, P<const unsigned long long>(peers), world, rank,
                                     P<const float>(in), P<float>(out), m, cap, epoch,
                                     P<unsigned>(ep), P<unsigned>(arrive), limit,
                                     P<int>(timeout), blocks,
                                     reinterpret_cast<hipStream_t>(stream)),
                "cnmf_xgmi_collective");
        });
}
