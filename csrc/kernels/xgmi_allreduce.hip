// One-shot all-reduce over xGMI peer memory (optional custom op).
//
// Every rank of a node owns one IPC-exported workspace:
//
//   [ flags: kMaxRanks x kMaxBlocks uint32 | pad to kDataOff | data parity 0 | data parity 1 ]
//
// and maps every peer's workspace into its address space (hipIpcOpenMemHandle), so a kernel
// on GPU r can load GPU q's HBM directly over the point-to-point xGMI link r<->q.  One launch
// of xgmi_allreduce_kernel per call:
//
//   1. block b copies its slice of the local input into this call's data parity (epoch & 1)
//      of its OWN workspace, releases it at system scope and stores the call's epoch into
//      flags[rank][b] of EVERY peer's workspace (one remote store per peer);
//   2. it waits until flags[q][b] >= epoch in its own workspace for every peer q;
//   3. it sums slice b of every peer's parity buffer, in rank order (bitwise the same result
//      on every rank), into the output.
//
// Block b only ever depends on block b of the peers, so there is no grid-wide barrier: a
// rank's slice moves as soon as the matching peer blocks have staged theirs.  Each rank
// READS all 7 peers at once (one hop on each of its 7 links) and the data crosses each link
// once -- against the 2 x (W-1)/W link volume and 2 x (W-1) latency steps of a ring.  Two
// parities make the next call safe without a closing barrier: a peer can run at most one
// call ahead (its step-2 wait needs this rank's flag of that call), so the parity a rank is
// about to overwrite was last read two calls ago, by kernels that have finished.
//
// A peer that never arrives (crashed rank, mismatched call sequence) would spin the GPU
// forever; the wait is bounded by a wall-clock limit instead.  Past it the block raises
// `timeout` and carries on (its output is then garbage): the host checks the flag and
// fails loudly, and every later call exits at once while the flag is up.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace cnmf {

constexpr int kXgRanks = 16;                       // ranks per node handled
constexpr int kXgBlocks = 128;                     // slices per call (<= CUs: co-resident)
constexpr long long kXgDataOff = 64 * 1024;        // data after the flag page
constexpr int kXgThreads = 256;

__global__ __launch_bounds__(kXgThreads) void xgmi_allreduce_kernel(
    const unsigned long long* __restrict__ peers, int world, int rank, const float* in,
    float* out, long long n, long long cap, unsigned epoch, unsigned long long limit,
    int* timeout) {
  __shared__ int s_abort;
  const int b = blockIdx.x;
  const int nb = gridDim.x;
  const int tid = threadIdx.x;
  if (tid == 0)
    s_abort = __hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_abort) return;

  // slice of this block: a multiple of 4 floats so every interior access is a float4
  const long long per = (((n + nb - 1) / nb) + 3) & ~3LL;
  const long long lo = min(n, (long long)b * per);
  const long long hi = min(n, lo + per);
  const unsigned par = epoch & 1u;
  char* mine = reinterpret_cast<char*>(peers[rank]);
  float* stage = reinterpret_cast<float*>(mine + kXgDataOff) + par * cap;

  // 1. stage the slice, make it visible system-wide, raise this block's flag in every peer
  {
    const long long v0 = lo >> 2, v1 = hi >> 2;    // lo is 4-aligned; tail handled below
    const float4* src = reinterpret_cast<const float4*>(in);
    float4* dst = reinterpret_cast<float4*>(stage);
    const bool aligned = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
    if (aligned) {
      for (long long v = v0 + tid; v < v1; v += kXgThreads) dst[v] = src[v];
      for (long long i = (v1 << 2) + tid; i < hi; i += kXgThreads) stage[i] = in[i];
    } else {
      for (long long i = lo + tid; i < hi; i += kXgThreads) stage[i] = in[i];
    }
  }
  __threadfence_system();
  __syncthreads();
  if (tid < world) {
    unsigned* f = reinterpret_cast<unsigned*>(peers[tid]) + rank * kXgBlocks + b;
    __hip_atomic_store(f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }

  // 2. wait for the matching block of every peer (wrap-safe epoch compare, bounded)
  if (tid < world) {
    unsigned* f = reinterpret_cast<unsigned*>(mine) + tid * kXgBlocks + b;
    const unsigned long long t0 = wall_clock64();
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(4);
      if (wall_clock64() - t0 > limit) {
        atomicExch(timeout, 1);
        break;
      }
    }
  }
  __syncthreads();
  // system-scope acquire: the flag loads above were system-scope acquires by the polling
  // lanes; this fence orders every lane's slice loads after them.  The slices live in
  // uncached / fine-grained memory (cnmf_xgmi_alloc), so the loads read the peer's HBM.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");

  // 3. sum the peers' slices in rank order
  const long long v0 = lo >> 2, v1 = hi >> 2;
  const bool oaligned = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (oaligned) {
    for (long long v = v0 + tid; v < v1; v += kXgThreads) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int q = 0; q < world; ++q) {
        const float4* p = reinterpret_cast<const float4*>(
            reinterpret_cast<const char*>(peers[q]) + kXgDataOff) + (par * cap >> 2);
        const float4 t = p[v];
        acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
      }
      reinterpret_cast<float4*>(out)[v] = acc;
    }
  }
  for (long long i = (oaligned ? (v1 << 2) : lo) + tid; i < hi; i += kXgThreads) {
    float acc = 0.f;
    for (int q = 0; q < world; ++q)
      acc += reinterpret_cast<const float*>(reinterpret_cast<const char*>(peers[q]) +
                                            kXgDataOff)[par * cap + i];
    out[i] = acc;
  }
}

}  // namespace cnmf

extern "C" {

long long cnmf_xgmi_data_offset() { return cnmf::kXgDataOff; }
int cnmf_xgmi_max_ranks() { return cnmf::kXgRanks; }
int cnmf_xgmi_max_blocks() { return cnmf::kXgBlocks; }

// Workspace for `cap` floats per parity; zeroed (flags start below every epoch >= 1).
//
// Memory model.  Peers spin on flags that REMOTE GPUs store into this workspace while the
// kernel runs, and read the peers' staged slices right after.  Plain hipMalloc memory is
// coarse-grained: HIP makes it coherent across devices only at dispatch boundaries (a
// reading GPU may serve a peer's line from its own L2), which is not enough for an
// in-kernel hand-off between GPUs.  The workspace is therefore allocated UNCACHED
// (hipDeviceMallocUncached: every access goes to the owning GPU's memory, never a stale
// cached copy) and, where that flag is refused, FINE-GRAINED (coherent across devices at
// system scope, which is the scope of the flag release/acquire pair below).  Coarse-grained
// memory is never used: `mode` reports which kind was obtained (the allocation flags,
// hipPointerGetAttributes reads them back) and the call fails if neither is available.
hipError_t cnmf_xgmi_alloc(long long cap, void** ptr, unsigned* mode) {
  const size_t bytes = (size_t)cnmf::kXgDataOff + 2 * (size_t)cap * sizeof(float);
  const unsigned kinds[2] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
  hipError_t e = hipErrorOutOfMemory;
  *ptr = nullptr;
  for (unsigned k : kinds) {
    e = hipExtMallocWithFlags(ptr, bytes, k);
    if (e == hipSuccess) {
      *mode = k;
      break;
    }
    (void)hipGetLastError();   // clear the sticky error of the refused flag
    *ptr = nullptr;
  }
  if (e != hipSuccess) return e;
  e = hipMemset(*ptr, 0, bytes);
  if (e != hipSuccess) return e;
  return hipDeviceSynchronize();
}

// allocation flags of a device pointer (0 = coarse-grained hipMalloc)
hipError_t cnmf_ptr_alloc_flags(const void* p, unsigned* flags) {
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) return e;
  *flags = a.allocationFlags;
  return hipSuccess;
}

hipError_t cnmf_xgmi_allreduce(const unsigned long long* peers, int world, int rank,
                               const float* in, float* out, long long n, long long cap,
                               unsigned epoch, unsigned long long limit, int* timeout,
                               int blocks, hipStream_t stream) {
  if (world < 1 || world > cnmf::kXgRanks || rank < 0 || rank >= world || n > cap || n < 0)
    return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  if (blocks < 1) blocks = 1;
  if (blocks > cnmf::kXgBlocks) blocks = cnmf::kXgBlocks;
  hipLaunchKernelGGL(cnmf::xgmi_allreduce_kernel, dim3(blocks), dim3(cnmf::kXgThreads), 0,
                     stream, peers, world, rank, in, out, n, cap, epoch, limit, timeout);
  return hipGetLastError();
}

}  // extern "C"
