// C ABI of every HIP launcher compiled into cnmf_torch_amd/ops/_hip*.so.
#pragma once
#include <hip/hip_runtime.h>

#include "stream.h"

extern "C" {

int cnmf_solve_max_k();
int cnmf_solve_max_threads(int K);
int cnmf_solve_native_k(int K);
hipError_t cnmf_solve(int algo, int K, float* x, long long x_rs, long long ldx, const float* numer,
                      long long n_rs, long long ldn, const float* gram, long long g_rs,
                      const int* rep_index, int nblocks, int ncols, int max_iter, float tol,
                      float l1_num, float l1_den, float l2, float eps, float* lin_out,
                      float* quad_out, int* iters_out, int nsplit, int conv_mode,
                      int check_every, int threads, int variant, const int* active,
                      int coop_split, float* coop_slots, unsigned long long* coop_count,
                      unsigned coop_gen, int coop_epochs,
                      int* coop_timeout, unsigned short* planes, long long pl_rs,
                      long long pl_ld, long long pl_plane, const float* pl_colmul,
                      int pl_cols, int pl_n, const float* gsrc, long long gs_rs,
                      long long gs_ld, int gs_cols, int nslab_n, long long nslab_stride,
                      const float* n_scale, const float* nbase, float* nout, long long nb_rs,
                      long long ldnb, const float* gpart, int gpart_n, long long gpart_rs,
                      float* gout, float* gp_out, long long gp_rs, unsigned* coop_gen_dev,
                      unsigned* coop_arrive, int reps_per_launch, unsigned long long* stamps,
                      hipStream_t stream);

hipError_t cnmf_stream_swap(const cnmf::StreamSwap* args, int chunks, hipStream_t stream);
hipError_t cnmf_rows_swap(const cnmf::RowsSwap* args, int npairs, int chunks, hipStream_t stream);
hipError_t cnmf_stream_publish(const int* ctr, int n, int* seq, int* mail, int slots, int width,
                               hipStream_t stream);

hipError_t cnmf_conv_update(const float* lin, const float* quad, double x_sq, double* err_init,
                            double* err_prev, double* err, int* active, int* converged,
                            int* n_pass, int n, int pass, double tol, int final_pass,
                            int init, int* gate, int max_pass, int* hflags, int* hcnt,
                            hipStream_t stream);
int cnmf_solve_reg_max_cols(int K);
int cnmf_solve_mfma_max_cols(int K);
int cnmf_solve_pipe_tiles(int K, int per);
int cnmf_solve_pipe_k(int K);
hipError_t cnmf_ridge_seg_tgemm(const double* Rt, long long ldr, int Kc, const void* X, int x_f64,
                                long long ldx, int F, const int* idx, const long long* seg,
                                int nseg, double* out, long long seg_stride, long long ldo,
                                hipStream_t stream);
hipError_t cnmf_ridge_seg_reduce(const double* part, const int* cfirst, int nseg, int Kc, int F,
                                 double* out, long long seg_stride, long long ldo,
                                 hipStream_t stream);
hipError_t cnmf_ridge_apply(const double* Rt, long long ldr, int Kc, const void* X, int x_f64,
                            long long ldx, void* Y, long long ldy, int F, const int* order,
                            const int* blk, int nblk, const double* Wc, long long wc_combo,
                            long long ldw, hipStream_t stream);
hipError_t cnmf_exact_moments(const void* X, int is_f64, long long ld, long long rows, int G,
                              int chunks, long long* part, long long* out,
                              unsigned long long* bad, hipStream_t stream);
hipError_t cnmf_predict_err(const float* X, long long ldx, const double* U, long long ldu,
                            const double* S, long long lds, int N, int G, int K, double* part,
                            hipStream_t stream);
int cnmf_solve_pipe_max_cols(int K);
int cnmf_solve_pipe_wg_per_cu(int K);

int cnmf_beta_max_k();
hipError_t cnmf_beta_contract(int side, int mode, const float* X, long long ldx, const float* HT,
                              long long h_rs, long long ldh, const float* W, long long w_rs,
                              long long ldw, int N, int G, int K, int R, float beta, float eps,
                              float* num, float* den, double* loss, const int* active,
                              int splits, int upd, const float* den_vec, float l1, float l2,
                              float gamma, float tol, float* part, int* counter, int* act,
                              int* iters, int conv_mode, int check_every, double* hstate,
                              hipStream_t stream);
int cnmf_beta_w_update_blocks(int K, int G);
hipError_t cnmf_beta_w_update(int mode, float* W, long long w_rs, long long ldw,
                              const float* num, const float* den, const float* hsum,
                              const float* An, const float* Ad, float* an_out, float* dn_out,
                              int R, int K, int G, int splits, float gamma, float l1, float l2,
                              float eps, float tol, float* part, int* counter, int* act,
                              int* iters, hipStream_t stream);

int cnmf_bp_max_k();
long long cnmf_bp_panel_elems(int K, int L, int mode);
int cnmf_bp_strip_cols(int K, int mode);
int cnmf_bp_splits(int Ls, int splits);
hipError_t cnmf_bp_panels(const float* F, long long f_rs, long long ldf, int K, int L, int R,
                          int mode, const float* prow, unsigned short* out, long long out_rs,
                          hipStream_t stream);
hipError_t cnmf_bp_run(int side, int mode, const float* X, long long ldx,
                       const unsigned short* panel, long long panel_rs, float* F, long long f_rs,
                       long long ldf, int K, int Lf, int Ls, int R, int splits, float beta,
                       float eps, float* num, float* den, int nsteps, int loss_entry,
                       int loss_exit, const float* den_vec, float l1, float l2, float gamma,
                       float tol, int conv_mode, double* hstate, double* part, int* counter,
                       int* act, int* iters, const int* active, double* loss, double xsum,
                       int xh, const float* uvec, const float* fscale, hipStream_t stream);

// sparse_kl.hip: KL MU statistics over a CSR matrix
int cnmf_sk_k4(int K);
int cnmf_sk_lds(int Ls, int K);
int cnmf_sk_cols_per_wg(int Lf, int R, int Ls, int K);
int cnmf_sk_groups(int Lf, int R, int Ls, int K);
hipError_t cnmf_sk_run(int side, const int* rowptr, const int* col, const float* val,
                       const float* ST, long long st_rs, float* F, long long f_rs,
                       long long ldf, int K, int Lf, int Ls, int R, float eps, float* num,
                       int nsteps,
                       int loss_entry, int loss_exit, const float* den_vec, float l1, float l2,
                       float tol, int conv_mode, double* hstate, double* part, int* counter,
                       int* act, int* iters, const int* active, double* loss, double xsum,
                       hipStream_t stream);

hipError_t cnmf_pairdist(const double* A, long long lda, const double* B, long long ldb,
                         const double* na, const double* nb, int n, int m, int kdim, double* D,
                         long long ldd, int same, int squared, hipStream_t stream);
hipError_t cnmf_knn_sum(const double* D, long long ldd, int n, int m, int k, double* out,
                        hipStream_t stream);
hipError_t cnmf_small_gram(const void* A, long long s_i, long long s_a, int n, int K, int esz,
                           int rows_per, void* part, hipStream_t stream);
hipError_t cnmf_seg_colsum(const double* X, long long ldx, int n, int d, const int* lab,
                           long long ldl, int nrest, int k, double* out, hipStream_t stream);
hipError_t cnmf_seg_rowsum(const double* D, long long ldd, int n, int m, const int* lab, int k,
                           double* out, long long ldo, hipStream_t stream);
hipError_t cnmf_seg_argmin(const double* D, long long ldd, int n, int nseg, int k,
                           const double* row_add, const double* col_add, int* labels,
                           double* mind, hipStream_t stream);

int cnmf_harmony_max_kb();
hipError_t cnmf_harmony_block(int op, double* Rt, const double* distT, const double* sigma,
                              const int* cells, const int* bidx, int nb, int N, int K, int B,
                              int nvar, int chunk, double* E, double* O, const double* Pr_b,
                              const double* theta, double* Pen, double* part, const double* Y,
                              const double* Zt, int d, double* obj, hipStream_t stream);
int cnmf_harmony_centroid_max_d();
hipError_t cnmf_harmony_centroid(const double* Zt, const double* Rt, int N, int d, int K,
                                 int chunk, double* part, double* Y, hipStream_t stream);
hipError_t cnmf_harmony_objective(const double* O, const double* E, const double* sigma,
                                  const double* theta, int K, int B, double* obj, double* out,
                                  hipStream_t stream);

int cnmf_beta_any_rows();
hipError_t cnmf_beta_any_terms(int mode, const float* X, long long ldx, float* P, float* D, int m,
                               int c, int G, float beta, float eps, const int* act, int want_q,
                               double* part, hipStream_t stream);
int cnmf_solve_any_hals_max_k();
hipError_t cnmf_solve_any(int op, float* x, long long x_rs, long long ldx, const float* numer,
                          long long n_rs, long long ldn, const float* D, const float* G,
                          long long g_rs, const int* reps, int* act, int m, int K, int n, int per,
                          float l1_num, float l1_den, float l2, float eps, double* part,
                          int* iters, hipStream_t stream);
hipError_t cnmf_solve_any_conv(int mode, const double* part, int nblk, int m, int* act,
                               const int* act0, const int* reps, double* f_prev, int have_prev,
                               float tol, float eps, float* lin_out, float* quad_out,
                               hipStream_t stream);

hipError_t cnmf_gram(const float* X, long long x_rs, long long ldx, int R, int K, int n,
                     float* out, long long o_rs, int accumulate, const int* active,
                     float* part, int S, hipStream_t stream);

int cnmf_kmeans_blocks(int n);
int cnmf_kmeanspp_blocks(int n);
int cnmf_kmeanspp_sample_blocks(int n);
hipError_t cnmf_kmeanspp_sample(const double* closest, int n, int n_init, const double* u,
                                int trials, double* bsum, long long* cand, hipStream_t stream);
int cnmf_kmeanspp_fits(int M, int d);
hipError_t cnmf_kmeanspp(const double* X, long long ldx, int n, int d, const double* C, int M,
                         int trials, double* closest, int n_init, int mode, double* pot,
                         hipStream_t stream);
int cnmf_kmeans_fits(int k, int d);
hipError_t cnmf_kmeans_step(const double* X, long long ldx, int n, int d, const double* C, int k,
                            int n_init, const int* live, int* labels, double* mind, double* psum,
                            double* pcnt, hipStream_t stream);

hipError_t cnmf_csr_row_sums(const long long* indptr, const void* data, int f64, int n,
                             double* out, hipStream_t stream);
int cnmf_csr_stats_blocks(int n);
hipError_t cnmf_csr_col_stats(const long long* indptr, const int* indices, const void* data,
                              int f64, int n, int n_out, const double* row_scale,
                              const int* col_map, const double* col_div, const double* clip,
                              double max_value, int round_mid, const double* center,
                              double* psum, double* psq, double* pcnt, hipStream_t stream);
hipError_t cnmf_csr_transform(const long long* indptr, const int* indices, const void* data,
                              int f64, int n, const double* row_scale, const int* col_map,
                              const double* col_div, const double* clip, double max_value,
                              int round_mid, void* out, int out_f64, hipStream_t stream);
hipError_t cnmf_csr_densify(const long long* indptr, const int* indices, const void* data,
                            int f64, int n, const double* row_scale, const int* col_map,
                            const double* col_div, const double* clip, double max_value,
                            int round_mid, void* out, int out_f64, long long ldo,
                            hipStream_t stream);
hipError_t cnmf_csr_spmm(const long long* indptr, const int* indices, const void* data, int f64,
                         int n, const double* row_scale, const int* col_map,
                         const double* col_div, const double* clip, double max_value,
                         int round_mid, const float* B, int K, float* out, hipStream_t stream);
int cnmf_csr_tspmm_blocks(int n);
hipError_t cnmf_csr_tspmm(const long long* indptr, const int* indices, const void* data, int f64,
                          int n, int n_out, const double* row_scale, const int* col_map,
                          const double* col_div, const double* clip, double max_value,
                          int round_mid, const void* B, int b_f64, int K, double* part,
                          hipStream_t stream);
hipError_t cnmf_radix_hist(const float* x, long long m, unsigned int prefix, unsigned int mask,
                           int shift, unsigned long long* hist, hipStream_t stream);

hipError_t cnmf_philox_fill(float* out, long long rows, long long cols, long long s_row,
                            long long s_col, long long rep_stride, long long row_offset,
                            const unsigned long long* seeds, const float* scales, int R,
                            unsigned int stream_id, int mode, hipStream_t stream);
int cnmf_seg_median_max_rows();
int cnmf_seg_median_max_clusters();
hipError_t cnmf_seg_median(const double* S, long long lds, int n, int G, const int* perm,
                           const int* seg, int k, double* out, long long ldo, hipStream_t stream);
int cnmf_gemm_planes_bk(int pb);
int cnmf_gemm_planes_tile(int v, int which);
hipError_t cnmf_gemm_planes(const unsigned short* A, long long lda, long long a_plane, int a_rows,
                            const unsigned short* B, long long ldb, long long b_plane, int b_rows,
                            float* C, long long ldc, const float* col_scale, int M, int N,
                            int Kd, int pa, int pb, int accumulate, int variant, int ksplit,
                            float* slab, int stages, int kstep, int raw, const int* gate,
                            hipStream_t stream);
hipError_t cnmf_split_planes(const float* S, long long lds, int rows, int cols, int cols_pad,
                             const float* col_mul, unsigned short* P, long long ldp,
                             long long plane, int nplanes, hipStream_t stream);

int cnmf_colstats_blocks(int N);
hipError_t cnmf_colstats(const float* X, long long ldx, int N, int G, float* pmin, double* psq,
                         int* pneg, float* mn, double* sq, int* neg, hipStream_t stream);
hipError_t cnmf_count_unit_check(const float* X, long long ldx, int N, int G, const float* mn,
                                 unsigned* bad, hipStream_t stream);


// xgmi_allreduce.hip: one-shot all-reduce over IPC-mapped peer workspaces
long long cnmf_xgmi_data_offset();
int cnmf_xgmi_max_ranks();
int cnmf_xgmi_max_blocks();
hipError_t cnmf_xgmi_alloc(long long cap, void** ptr, unsigned* mode);
hipError_t cnmf_ptr_alloc_flags(const void* p, unsigned* flags);
hipError_t cnmf_xgmi_allreduce(const unsigned long long* peers, int world, int rank,
                               const float* in, float* out, long long n, long long cap,
                               unsigned epoch, unsigned long long limit, int* timeout,
                               int blocks, hipStream_t stream);
hipError_t cnmf_xgmi_collective(int mode, const unsigned long long* peers, int world, int rank,
                                const float* in, float* out, long long m, long long cap,
                                unsigned epoch, unsigned* ep, unsigned* arrive,
                                unsigned long long limit, int* timeout, int blocks,
                                hipStream_t stream);

}
