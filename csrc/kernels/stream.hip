// Device-side replicate swap of the continuous-batching solver (models/nmf.py
// NMFBatchSolver.run_stream; SURVEY.md §7.4.3 -- the reference factorises replicates one
// after the other, cnmf.py:882-892, with a host sync per inner iteration, cnmf.py:377).
//
// A streaming batch keeps a fixed set of replicate POSITIONS per K group.  At the end of
// every pass (after conv_update), two kernels of the pass's captured graph
//   1. plan (one workgroup): every position whose replicate stopped (active == 0) is
//      harvested, and the free positions are handed the next staged replicates of the
//      group's ring in position order (a block scan: deterministic), advancing the ring's
//      head; the occupant table and the harvested count are updated, and the GEMM gate is
//      raised when anything was placed;
//   2. copy (positions x column slices): the finished occupant's spectra (and usages) go
//      to its rows of the result store, its error / pass / convergence / iteration state
//      to its column; then the staged replicate's factors, state, W W^T partial-Gram block
//      and spectra bf16 planes are copied into the position -- the operands the next pass
//      (the same graph, replayed) reads in place.
// A replicate is therefore replaced in the pass it finished, with no host round trip: the
// host only keeps the ring stocked (staging = Philox init + initial error + operands, in a
// few large launches) and reads the harvested count one pass late to know when to stop.
#include "stream.h"

#include <stdint.h>

namespace cnmf {

__global__ void __launch_bounds__(1024) stream_plan_kernel(StreamSwap p) {
  __shared__ int s_scan[1024];
  __shared__ int s_base, s_nh;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_base = 0;
    s_nh = 0;
  }
  const int h0 = *p.head;
  const int avail = max(0, *p.tail - h0);
  __syncthreads();
  for (int c0 = 0; c0 < p.n; c0 += 1024) {
    const int pos = c0 + tid;
    int fr = 0, oc = -1;
    if (pos < p.n) {
      oc = p.occ[pos];
      fr = p.active[pos] == 0 ? 1 : 0;
    }
    s_scan[tid] = fr;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      const int v = tid >= d ? s_scan[tid - d] : 0;
      __syncthreads();
      s_scan[tid] += v;
      __syncthreads();
    }
    const int rank = s_base + s_scan[tid] - fr;
    if (pos < p.n) {
      const int e = (fr && rank < avail) ? h0 + rank : -1;
      const int hv = (fr && oc >= 0) ? oc : -1;
      p.plan[pos] = e;
      p.plan[p.n + pos] = hv;
      p.occ[pos] = e >= 0 ? p.ring_id[e % p.qc] : (fr ? -1 : oc);
      if (hv >= 0) atomicAdd(&s_nh, 1);
    }
    __syncthreads();
    if (tid == 0) s_base += s_scan[1023];
    __syncthreads();
  }
  if (tid == 0) {
    const int used = min(s_base, avail);
    *p.head = h0 + used;
    *p.done += s_nh;
    if (used > 0) *p.gate = 1;
  }
}

// rows x cols of T from src (row pitch lds) to dst (ldd), slice y of ny of the flattened
// (row, 16-byte vector) index space -- every thread issues 4 independent loads before
// its stores; scalar when a pitch or a base does not allow 16-byte vectors
// ``vec`` (16-byte vectors) is decided ONCE per matrix by the caller from every base the
// harvest and the placement of a position touch: both phases then cut the (rows x cols)
// range into the same slices, so the __syncthreads between them orders every element's
// read-out before its overwrite (per-call decisions could slice the two differently).
template <typename T>
__device__ __forceinline__ bool sw_vec(int cols, long long ld, const void* a, const void* b,
                                       const void* c) {
  constexpr int V = 16 / sizeof(T);
  return ((cols | ld) % V) == 0 &&
         ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
           reinterpret_cast<uintptr_t>(c)) & 15) == 0;
}

template <typename T>
__device__ __forceinline__ void sw_rows(const T* __restrict__ src, long long lds, T* __restrict__ dst,
                                        long long ldd, int rows, int cols, int y, int ny,
                                        bool vec) {
  constexpr int V = 16 / sizeof(T);
  const int bd = blockDim.x;
  if (vec) {
    const int cv = cols / V;
    const long long tot = (long long)rows * cv;
    const long long a = tot * y / ny, b = tot * (y + 1) / ny;
    const long long ldsv = lds / V, lddv = ldd / V;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (long long i0 = a + threadIdx.x; i0 < b; i0 += 4LL * bd) {
      uint4 v[4];
      long long od[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long i = i0 + (long long)u * bd;
        od[u] = -1;
        if (i < b) {
          const long long r = i / cv, c = i - r * cv;
          v[u] = s4[r * ldsv + c];
          od[u] = r * lddv + c;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (od[u] >= 0) d4[od[u]] = v[u];
    }
  } else {
    const long long tot = (long long)rows * cols;
    const long long a = tot * y / ny, b = tot * (y + 1) / ny;
    for (long long i = a + threadIdx.x; i < b; i += bd) {
      const long long r = i / cols, c = i - r * cols;
      dst[r * ldd + c] = src[r * lds + c];
    }
  }
}

// grid (n, chunks): workgroup (pos, y) moves column slice y of the position's rows
__global__ void __launch_bounds__(256) stream_copy_kernel(StreamSwap p) {
  const int pos = blockIdx.x, y = blockIdx.y, ny = gridDim.y;
  const int e = p.plan[pos], h = p.plan[p.n + pos];
  if (e < 0 && h < 0) return;
  const int K = p.K, tid = threadIdx.x;
  const long long r0 = (long long)pos * K;
  const int slot = e >= 0 ? e % p.qc : 0;
  const long long s0 = (long long)slot * K;
  const long long o = h >= 0 ? p.offs[h] : 0;
  float* Wp = p.W + r0 * p.ldw;
  float* Hp = p.HT + r0 * p.ldh;
  const bool vw = sw_vec<float>(p.G, p.ldw, Wp, p.oW + o * p.ldw, p.rW + s0 * p.ldw);
  const bool vh = sw_vec<float>(p.N, p.ldh, Hp, p.oHT ? p.oHT + o * p.ldh : Hp,
                                p.N > 0 ? p.rHT + s0 * p.ldh : Hp);
  if (h >= 0) {
    sw_rows(Wp, p.ldw, p.oW + o * p.ldw, p.ldw, K, p.G, y, ny, vw);
    if (p.oHT) sw_rows(Hp, p.ldh, p.oHT + o * p.ldh, p.ldh, K, p.N, y, ny, vh);
    if (y == 0) {
      if (tid < 3) p.osf[tid * p.osf_ld + h] = p.sf[tid * p.sf_ld + pos];
      else if (tid < 8) p.osi[(tid - 3) * p.osi_ld + h] = p.si[(tid - 3) * p.si_ld + pos];
    }
  }
  if (e < 0) return;
  __syncthreads();     // this slice of the position is read out before it is overwritten
  sw_rows(p.rW + s0 * p.ldw, p.ldw, Wp, p.ldw, K, p.G, y, ny, vw);
  if (p.N > 0) sw_rows(p.rHT + s0 * p.ldh, p.ldh, Hp, p.ldh, K, p.N, y, ny, vh);
  for (int pl = 0; pl < 3; ++pl) {
    const unsigned short* ps = p.rwpl + pl * p.rpl_plane + s0 * p.pl_ld;
    unsigned short* pd = p.wpl + pl * p.pl_plane + r0 * p.pl_ld;
    sw_rows(ps, p.pl_ld, pd, p.pl_ld, K, p.Gp, y, ny, sw_vec<unsigned short>(p.Gp, p.pl_ld, ps, pd, pd));
  }
  if (y == 0) {
    const int blk = p.S * K * K;
    const float* sp = p.rparts + (long long)slot * blk;
    float* dp = p.parts + (long long)pos * blk;
    for (int i = tid; i < blk; i += 256) dp[i] = sp[i];
    if (tid < 3) p.sf[tid * p.sf_ld + pos] = p.rsf[tid * p.qc + slot];
    else if (tid < 8) p.si[(tid - 3) * p.si_ld + pos] = p.rsi[(tid - 3) * p.qc + slot];
  }
}

// The host's view of a pass without a copy launch: one thread writes the pass's sequence
// number and the counter block (harvested count, ring heads) into slot seq % slots of a
// pinned host mailbox (device-mapped), and advances seq.  After the pass's event the host
// reads the slot and checks the sequence number.
__global__ void stream_publish_kernel(const int* __restrict__ ctr, int n, int* __restrict__ seq,
                                      int* __restrict__ mail, int slots, int width) {
  if (threadIdx.x != 0) return;
  const int s = *seq;
  int* row = mail + (long long)(s % slots) * width;
  for (int i = 0; i < n && i + 1 < width; ++i) row[1 + i] = ctr[i];
  row[0] = s;
  *seq = s + 1;
}

// In-place batch compaction by disjoint position swaps (models/nmf_batch.py _Batch.compact,
// single-K batches): pair i exchanges positions pairs[2i] and pairs[2i+1] -- K rows of
// every listed matrix and one column of each per-replicate state table.  The pairs are
// disjoint, so every workgroup owns its rows and nothing is staged: only the replicates
// that change position move (a host gather-and-copy of the whole HT / W moved every row
// twice).  grid (npairs, chunks): workgroup (i, y) swaps column slice y.
template <typename T>
__device__ __forceinline__ void swap_rows(T* __restrict__ a, T* __restrict__ b, long long ld,
                                          int rows, int cols, int y, int ny) {
  constexpr int V = 16 / sizeof(T);
  const int bd = blockDim.x;
  const bool vec = ((cols | ld) % V) == 0 &&
                   ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
  if (vec) {
    const int cv = cols / V;
    const long long tot = (long long)rows * cv, ldv = ld / V;
    const long long lo = tot * y / ny, hi = tot * (y + 1) / ny;
    uint4* a4 = reinterpret_cast<uint4*>(a);
    uint4* b4 = reinterpret_cast<uint4*>(b);
    for (long long i0 = lo + threadIdx.x; i0 < hi; i0 += 2LL * bd) {
      uint4 va[2], vb[2];
      long long o[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const long long i = i0 + (long long)u * bd;
        o[u] = -1;
        if (i < hi) {
          const long long r = i / cv;
          o[u] = r * ldv + (i - r * cv);
          va[u] = a4[o[u]];
          vb[u] = b4[o[u]];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (o[u] >= 0) {
          a4[o[u]] = vb[u];
          b4[o[u]] = va[u];
        }
    }
  } else {
    const long long tot = (long long)rows * cols;
    const long long lo = tot * y / ny, hi = tot * (y + 1) / ny;
    for (long long i = lo + threadIdx.x; i < hi; i += bd) {
      const long long r = i / cols, off = r * ld + (i - r * cols);
      const T t = a[off];
      a[off] = b[off];
      b[off] = t;
    }
  }
}

__global__ void __launch_bounds__(256) rows_swap_kernel(RowsSwap p) {
  const int i = blockIdx.x, y = blockIdx.y, ny = gridDim.y;
  const int pa = p.pairs[2 * i], pb = p.pairs[2 * i + 1];
  const long long ra = (long long)pa * p.K, rb = (long long)pb * p.K;
  for (int m = 0; m < p.nmat; ++m) {
    const SwapMat& q = p.mat[m];
    for (int pl = 0; pl < q.planes; ++pl) {
      if (q.esz == 4) {
        float* base = reinterpret_cast<float*>(q.p) + pl * q.plane;
        swap_rows(base + ra * q.ld, base + rb * q.ld, q.ld, p.K, q.cols, y, ny);
      } else {
        unsigned short* base = reinterpret_cast<unsigned short*>(q.p) + pl * q.plane;
        swap_rows(base + ra * q.ld, base + rb * q.ld, q.ld, p.K, q.cols, y, ny);
      }
    }
  }
  if (y != 0) return;
  const int t = threadIdx.x;
  if (t < p.nsf) {
    double* r = p.sf + t * p.sf_ld;
    const double v = r[pa];
    r[pa] = r[pb];
    r[pb] = v;
  } else if (t >= 64 && t < 64 + p.nsi) {
    int* r = p.si + (t - 64) * p.si_ld;
    const int v = r[pa];
    r[pa] = r[pb];
    r[pb] = v;
  }
}

}  // namespace cnmf

extern "C" hipError_t cnmf_rows_swap(const cnmf::RowsSwap* args, int npairs, int chunks,
                                     hipStream_t stream) {
  const cnmf::RowsSwap& p = *args;
  if (npairs <= 0) return hipSuccess;
  if (p.K < 1 || chunks < 1 || !p.pairs || p.nmat < 0 || p.nmat > 4 || p.nsf < 0 || p.nsf > 8 ||
      p.nsi < 0 || p.nsi > 8 || (p.nsf && !p.sf) || (p.nsi && !p.si))
    return hipErrorInvalidValue;
  for (int m = 0; m < p.nmat; ++m) {
    const cnmf::SwapMat& q = p.mat[m];
    if (!q.p || q.cols < 1 || q.ld < q.cols || (q.esz != 4 && q.esz != 2) || q.planes < 1 ||
        q.planes > 3)
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(cnmf::rows_swap_kernel, dim3((unsigned)npairs, (unsigned)chunks), dim3(256), 0,
                     stream, p);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_stream_publish(const int* ctr, int n, int* seq, int* mail, int slots,
                                          int width, hipStream_t stream) {
  if (n < 1 || slots < 1 || width < 2 || !ctr || !seq || !mail) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnmf::stream_publish_kernel, dim3(1), dim3(64), 0, stream, ctr, n, seq, mail,
                     slots, width);
  return hipGetLastError();
}

extern "C" hipError_t cnmf_stream_swap(const cnmf::StreamSwap* args, int chunks,
                                       hipStream_t stream) {
  const cnmf::StreamSwap& p = *args;
  if (p.n <= 0) return hipSuccess;
  if (p.K < 1 || p.G < 1 || p.qc < 1 || p.S < 1 || chunks < 1 || !p.active || !p.occ ||
      !p.plan || !p.head || !p.tail || !p.ring_id || !p.rW || !p.rsf || !p.rsi ||
      !p.rparts || !p.rwpl || !p.offs || !p.oW || !p.osf || !p.osi || !p.done || !p.gate ||
      (p.N > 0 && (!p.HT || !p.rHT)) || (p.oHT && p.N <= 0))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnmf::stream_plan_kernel, dim3(1), dim3(1024), 0, stream, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(cnmf::stream_copy_kernel, dim3((unsigned)p.n, (unsigned)chunks), dim3(256), 0,
                     stream, p);
  return hipGetLastError();
}
