// One-shot all-reduce / reduce-scatter / all-gather over xGMI peer memory (SURVEY.md §2.6
// item 4, optional custom ops).
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

// Collectives of one launch each (MODE), over m floats per block-slice index range:
//   kXgAllReduce      in n = m floats, out n: sum over ranks;
//   kXgReduceScatter  in world x m (rank-major chunks), out m: chunk `rank` of the sum --
//                     block b stages slice b of EVERY chunk, so one flag per (peer, block)
//                     still covers everything block b of any rank reads;
//   kXgAllGather      in m, out world x m: every rank's input, no arithmetic.
// The call's epoch is either the host's (`epoch` > 0) or kept on the device (`epoch` == 0:
// read from *ep at start; the last block to finish advances it -- graph replays then
// advance it too, exactly like the host counter would).
constexpr int kXgAllReduce = 0, kXgReduceScatter = 1, kXgAllGather = 2;

template <int MODE>
__global__ __launch_bounds__(kXgThreads) void xgmi_coll_kernel(
    const unsigned long long* __restrict__ peers, int world, int rank, const float* in,
    float* out, long long m, long long cap, unsigned host_epoch, unsigned* ep, unsigned* arrive,
    unsigned long long limit, int* timeout) {
  __shared__ int s_abort;
  __shared__ unsigned s_epoch;
  const int b = blockIdx.x;
  const int nb = gridDim.x;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_abort = __hip_atomic_load(timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_epoch = host_epoch ? host_epoch
                         : __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  }
  __syncthreads();
  const unsigned epoch = s_epoch;
  if (!s_abort) {
    // slice of this block within [0, m): a multiple of 4 floats so interior accesses are
    // float4 (whole chunks stay 16-byte aligned when m % 4 == 0)
    const long long per = (((m + nb - 1) / nb) + 3) & ~3LL;
    const long long lo = min(m, (long long)b * per);
    const long long hi = min(m, lo + per);
    const unsigned par = epoch & 1u;
    char* mine = reinterpret_cast<char*>(peers[rank]);
    float* stage = reinterpret_cast<float*>(mine + kXgDataOff) + par * cap;
    const bool vec = (m & 3) == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(out) & 15) == 0;

    // 1. stage, make visible system-wide, raise this block's flag in every peer
    const int nchunk = MODE == kXgReduceScatter ? world : 1;
    for (int c = 0; c < nchunk; ++c) {
      const long long o = (long long)c * m;
      if (vec) {
        const float4* src = reinterpret_cast<const float4*>(in + o);
        float4* dst = reinterpret_cast<float4*>(stage + o);
        for (long long v = (lo >> 2) + tid; v < (hi >> 2); v += kXgThreads) dst[v] = src[v];
      } else {
        for (long long i = lo + tid; i < hi; i += kXgThreads) stage[o + i] = in[o + i];
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

    // 3. read the peers' slices: sum in rank order, or copy
    auto pstage = [&](int q) {
      return reinterpret_cast<const float*>(reinterpret_cast<const char*>(peers[q]) + kXgDataOff) +
             par * cap;
    };
    if (MODE == kXgAllGather) {
      for (int q = 0; q < world; ++q) {
        const float* p = pstage(q);
        float* o = out + (long long)q * m;
        if (vec) {
          for (long long v = (lo >> 2) + tid; v < (hi >> 2); v += kXgThreads)
            reinterpret_cast<float4*>(o)[v] = reinterpret_cast<const float4*>(p)[v];
        } else {
          for (long long i = lo + tid; i < hi; i += kXgThreads) o[i] = p[i];
        }
      }
    } else {
      const long long src0 = MODE == kXgReduceScatter ? (long long)rank * m : 0;
      if (vec) {
        for (long long v = (lo >> 2) + tid; v < (hi >> 2); v += kXgThreads) {
          float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
          for (int q = 0; q < world; ++q) {
            const float4 t = reinterpret_cast<const float4*>(pstage(q) + src0)[v];
            acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
          }
          reinterpret_cast<float4*>(out)[v] = acc;
        }
      } else {
        for (long long i = lo + tid; i < hi; i += kXgThreads) {
          float acc = 0.f;
          for (int q = 0; q < world; ++q) acc += pstage(q)[src0 + i];
          out[i] = acc;
        }
      }
    }
  }
  // device epoch: the last block of the launch advances it (every block read it above)
  if (!host_epoch) {
    __syncthreads();
    if (tid == 0) {
      const unsigned old = atomicAdd(arrive, 1u);
      if (old + 1 == (unsigned)nb) {
        atomicExch(arrive, 0u);
        __hip_atomic_store(ep, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
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

// mode 0 all-reduce (m = n floats), 1 reduce-scatter (in world x m, out m), 2 all-gather
// (in m, out world x m); epoch > 0: the host's call counter, 0: the device counter at
// `ep` (+ its arrival counter `arrive`) -- capturable in a HIP graph
hipError_t cnmf_xgmi_collective(int mode, const unsigned long long* peers, int world, int rank,
                                const float* in, float* out, long long m, long long cap,
                                unsigned epoch, unsigned* ep, unsigned* arrive,
                                unsigned long long limit, int* timeout, int blocks,
                                hipStream_t stream) {
  if (world < 1 || world > cnmf::kXgRanks || rank < 0 || rank >= world || m < 0 ||
      mode < 0 || mode > 2)
    return hipErrorInvalidValue;
  if ((mode == 1 ? (long long)world * m : m) > cap) return hipErrorInvalidValue;
  if (epoch == 0 && (!ep || !arrive)) return hipErrorInvalidValue;
  if (m == 0) return hipSuccess;
  if (blocks < 1) blocks = 1;
  if (blocks > cnmf::kXgBlocks) blocks = cnmf::kXgBlocks;
  const dim3 g(blocks), t(cnmf::kXgThreads);
  if (mode == 0)
    hipLaunchKernelGGL(cnmf::xgmi_coll_kernel<cnmf::kXgAllReduce>, g, t, 0, stream, peers, world,
                       rank, in, out, m, cap, epoch, ep, arrive, limit, timeout);
  else if (mode == 1)
    hipLaunchKernelGGL(cnmf::xgmi_coll_kernel<cnmf::kXgReduceScatter>, g, t, 0, stream, peers,
                       world, rank, in, out, m, cap, epoch, ep, arrive, limit, timeout);
  else
    hipLaunchKernelGGL(cnmf::xgmi_coll_kernel<cnmf::kXgAllGather>, g, t, 0, stream, peers, world,
                       rank, in, out, m, cap, epoch, ep, arrive, limit, timeout);
  return hipGetLastError();
}

hipError_t cnmf_xgmi_allreduce(const unsigned long long* peers, int world, int rank,
                               const float* in, float* out, long long n, long long cap,
                               unsigned epoch, unsigned long long limit, int* timeout,
                               int blocks, hipStream_t stream) {
  if (epoch == 0) return hipErrorInvalidValue;
  return cnmf_xgmi_collective(0, peers, world, rank, in, out, n, cap, epoch, nullptr, nullptr,
                              limit, timeout, blocks, stream);
}

}  // extern "C"
