// On-device convergence bookkeeping for a replicate batch (one thread per replicate).
//
// Frobenius loss from the W-solve epilogue's sufficient statistics:
//   err = sqrt(max(||X||^2 - 2 <B, W> + <A, W W^T>, 0))  (sklearn square_root=True)
// and the nmf-torch / sklearn stopping rule (prev - cur) / init < tol.
// Keeping this on the device lets the host enqueue pass p+1 before it has read pass p's
// result: the solves skip replicates whose `active` flag dropped, so the host only polls
// the flags one pass behind instead of draining the GPU at every pass boundary.
#include <hip/hip_runtime.h>

namespace cnmf {

// Device-side ragged batching (optional `slot` block, graph-replayable: no host decision).
// After the flags are updated, the rows of the replicates still active are given compact
// slots: slot_cur[r] = sum of kvec[r'] over active r' < r (batch order), live[1] = the
// live row count; the previous pass's slots / count move to slot_prev / live[0].  The
// fused online step writes the GEMM operands (bf16 planes) and reads the GEMM outputs
// (split-K slabs) at those slots, and the plane GEMMs skip M-tiles past the live count,
// so GEMM work shrinks with every converged replicate (models/nmf.py _fused_pass).
// Optional active list (alist / apos, the pipelined solve's workgroup -> replicate map,
// solve_pipe.h): apos[r] = number of active r' < r (apos[n] = the active count) and
// alist[apos[r]] = r for the active r -- a launch over replicates [p0, p0 + m) walks
// alist[apos[p0] ..< apos[p0 + m]], so its workgroups carry only live replicates.
__device__ void conv_slots(const int* active, const int* kvec, int* slot_cur, int* slot_prev,
                           int* live, int n, int init, int* alist, int* apos) {
  __shared__ int ssum[256];
  __shared__ int scnt[256];
  const int per = (n + 255) / 256;
  const int r0 = threadIdx.x * per, r1 = min(n, r0 + per);
  int tot = 0, cnt = 0;
  for (int r = r0; r < r1; ++r) {
    const bool on = init || active[r];
    tot += on ? kvec[r] : 0;
    cnt += on ? 1 : 0;
  }
  ssum[threadIdx.x] = tot;
  scnt[threadIdx.x] = cnt;
  __syncthreads();
  // inclusive scans of the 256 per-thread sums (Hillis-Steele in LDS)
  for (int d = 1; d < 256; d <<= 1) {
    const int v = threadIdx.x >= d ? ssum[threadIdx.x - d] : 0;
    const int w = threadIdx.x >= d ? scnt[threadIdx.x - d] : 0;
    __syncthreads();
    ssum[threadIdx.x] += v;
    scnt[threadIdx.x] += w;
    __syncthreads();
  }
  int off = ssum[threadIdx.x] - tot;
  int pos = scnt[threadIdx.x] - cnt;
  for (int r = r0; r < r1; ++r) {
    const bool on = init || active[r];
    const int old = slot_cur[r];
    slot_prev[r] = init ? off : old;
    slot_cur[r] = off;
    off += on ? kvec[r] : 0;
    if (apos) {
      apos[r] = pos;
      if (on) alist[pos] = r;
    }
    pos += on ? 1 : 0;
  }
  if (threadIdx.x == 0) {
    const int total = ssum[255];
    live[0] = init ? total : live[1];
    live[1] = total;
    if (apos) apos[n] = scnt[255];
  }
}

__global__ void __launch_bounds__(256) conv_update_kernel(
    const float* lin, const float* quad, double x_sq, double* err_init, double* err_prev,
    double* err, int* active, int* converged, int* n_pass, int n, int pass, double tol,
    int final_pass, int init, int* gate, const int* kvec, int* slot_cur, int* slot_prev,
    int* live, int* alist, int* apos) {
  // one workgroup strides over the replicates, so `gate` (any replicate still active)
  // is a plain block reduction: no atomics, nothing to reset between passes
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
    n_pass[r] = pass >= 0 ? pass : n_pass[r] + 1;   // pass < 0: count on device (graphs)
    const double denom = err_init[r] > 1e-300 ? err_init[r] : 1e-300;
    if ((err_prev[r] - e) / denom < tol) {
      active[r] = 0;
      converged[r] = 1;
    } else if (final_pass) {
      active[r] = 0;
    } else {
      err_prev[r] = e;
      any = 1;
    }
  }
  any = __syncthreads_or(any);
  if (gate && threadIdx.x == 0) *gate = any;
  if (kvec) conv_slots(active, kvec, slot_cur, slot_prev, live, n, init, alist, apos);
}

}  // namespace cnmf

// gate (optional): set to 1 while any replicate is still active, 0 once none is -- the
// split GEMMs of the next (speculative) pass then return at once (gemm_planes.hip)
extern "C" hipError_t cnmf_conv_update(const float* lin, const float* quad, double x_sq,
                                       double* err_init, double* err_prev, double* err,
                                       int* active, int* converged, int* n_pass, int n, int pass,
                                       double tol, int final_pass, int init, int* gate,
                                       const int* kvec, int* slot_cur, int* slot_prev,
                                       int* live, int* alist, int* apos, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (kvec && (!slot_cur || !slot_prev || !live)) return hipErrorInvalidValue;
  if ((alist != nullptr) != (apos != nullptr) || (apos && !kvec)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnmf::conv_update_kernel, dim3(1), dim3(256), 0, stream, lin, quad, x_sq,
                     err_init, err_prev, err, active, converged, n_pass, n, pass, tol, final_pass,
                     init, gate, kvec, slot_cur, slot_prev, live, alist, apos);
  return hipGetLastError();
}
