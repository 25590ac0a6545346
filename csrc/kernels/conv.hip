// On-device convergence bookkeeping for a replicate batch (one thread per replicate).
//
// Frobenius loss from the W-solve epilogue's sufficient statistics:
//   err = sqrt(max(||X||^2 - 2 <B, W> + <A, W W^T>, 0))  (sklearn square_root=True)
// and the nmf-torch / sklearn stopping rule (prev - cur) / init < tol.
// Keeping this on the device lets the host enqueue pass p+1 before it has read pass p's
// result: the solves skip replicates whose `active` flag dropped, so the host only polls
// the flags one pass behind instead of draining the GPU at every pass boundary.
//
// Pass counting on the device (pass < 0) with a per-replicate pass limit (max_pass > 0):
// a replicate stops after ITS max_pass-th pass, whatever pass the batch is in -- the
// continuous (streaming) solver refills converged slots with new replicates mid-run, so
// replicates of one batch sit at different passes (models/nmf.py NMFBatchSolver.run_stream).
#include <hip/hip_runtime.h>

namespace cnmf {

__global__ void __launch_bounds__(256) conv_update_kernel(
    const float* lin, const float* quad, double x_sq, double* err_init, double* err_prev,
    double* err, int* active, int* converged, int* n_pass, int n, int pass, double tol,
    int final_pass, int init, int* gate, int max_pass, int* hflags, int* hcnt) {
  // one workgroup strides over the replicates, so `gate` (any replicate still active)
  // is a plain block reduction: no atomics, nothing to reset between passes
  const int slot = hflags ? (*hcnt & 1) : 0;   // read before thread 0 advances it below
  int any = 0;
  for (int r = threadIdx.x; r < n; r += blockDim.x) {
    const double e = sqrt(fmax(x_sq - 2.0 * (double)lin[r] + (double)quad[r], 0.0));
    if (init) {  // error of the initial factors
      err_init[r] = e;
      err_prev[r] = e;
      err[r] = e;
      active[r] = 1;
      converged[r] = 0;
      n_pass[r] = 0;
      any = 1;
      continue;
    }
    if (!active[r]) continue;
    err[r] = e;
    const int np = pass >= 0 ? pass : n_pass[r] + 1;   // pass < 0: count on device (graphs)
    n_pass[r] = np;
    const double denom = err_init[r] > 1e-300 ? err_init[r] : 1e-300;
    if ((err_prev[r] - e) / denom < tol) {
      active[r] = 0;
      converged[r] = 1;
    } else if (final_pass || (max_pass > 0 && np >= max_pass)) {
      active[r] = 0;
    } else {
      err_prev[r] = e;
      any = 1;
    }
  }
  any = __syncthreads_or(any);
  if (gate && threadIdx.x == 0) *gate = any;
  // the flags into host-mapped pinned memory, alternating between two slots by this
  // launch's ordinal (*hcnt): the host reads launch c's slot after c's event, while
  // launch c + 1 writes the other one -- no device->host copy launch per pass
  if (hflags) {
    for (int r = threadIdx.x; r < n; r += blockDim.x) hflags[slot * n + r] = active[r];
    if (threadIdx.x == 0) *hcnt = *hcnt + 1;   // every thread has read it (barrier above)
  }
}

}  // namespace cnmf

// gate (optional): set to 1 while any replicate is still active, 0 once none is -- the
// split GEMMs of the next (speculative) pass then return at once (gemm_planes.hip).
// hflags / hcnt (optional, together): host-mapped pinned int32 [2][n] receiving the
// active flags in slot (*hcnt & 1), and the device launch counter advanced per launch.
extern "C" hipError_t cnmf_conv_update(const float* lin, const float* quad, double x_sq,
                                       double* err_init, double* err_prev, double* err,
                                       int* active, int* converged, int* n_pass, int n, int pass,
                                       double tol, int final_pass, int init, int* gate,
                                       int max_pass, int* hflags, int* hcnt,
                                       hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if ((hflags == nullptr) != (hcnt == nullptr)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnmf::conv_update_kernel, dim3(1), dim3(256), 0, stream, lin, quad, x_sq,
                     err_init, err_prev, err, active, converged, n_pass, n, pass, tol, final_pass,
                     init, gate, max_pass, hflags, hcnt);
  return hipGetLastError();
}
