// Fused Lloyd step for low-dimensional k-means (Harmony's k-means init over cells in PC
// space: harmonypy's KMeans(k ~ N/30 <= 100, n_init=10, max_iter=25) on N x d PCs,
// d <= 64; consensus k-means at K x G spectra keeps the MFMA distance path).
//
// One launch per Lloyd iteration for ALL restarts (grid.y = restart):
//   phase A  assignment on the f64 matrix cores: wave w owns 64 points of the round as 4
//            tiles of 16; the restart's centroids sit in LDS transposed (coordinate-major,
//            A operand), the points are the B operand straight from global memory, and
//            v_mfma_f64_16x16x4f64 forms 16 x 16 blocks of x . c; the score
//            |c|^2 - 2 x . c (sklearn's expanded distance, |x|^2 added only for the
//            distance output) picks the nearest centroid per point (first index on ties,
//            as numpy argmin) with a cross-lane reduction over the 4 lane groups.  The
//            previous thread-per-point form (exact (x - c)^2 sums, broadcast LDS reads of
//            every centroid) ran at ~12 ms per step at 500k x 50 x 100 x 10 restarts
//            (profiles/r5i_*).
//   phase B  the round's points are added to the workgroup's centroid accumulator (its
//            own partial slot of psum, in global memory):
//            a stable counting sort groups them by label, then each thread sums whole
//            (cluster, feature) segments in point order and adds them once (no float
//            atomics; the label histogram uses integer LDS atomics).
//   flush    the workgroup writes its partial sums/counts; the host sums the partials over
//            workgroups with a fixed-order reduction -> bitwise deterministic centroids.
// The (n x n_init*k) distance matrix of the MFMA path (4 GB at 500k cells x 10 x 100) is
// never materialised.
// f64 16x16x4 MFMA: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15];
// D: col = lane&15, row = (lane>>4) + 4*reg.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "common.h"

namespace cnmf {

constexpr int kKmThreads = 256;
constexpr int kKmRounds = 4;   // rounds of 256 points per workgroup

typedef double km_f64x4 __attribute__((ext_vector_type(4)));

// centroid tile pitch of the transposed LDS table: 16 (mod 32) doubles, so the 4 lane
// groups of an A-operand read fall on disjoint bank halves
__host__ __device__ constexpr int km_kps(int k) {
  return ((k + 15) / 16 * 16) % 32 == 16 ? (k + 15) / 16 * 16 : (k + 15) / 16 * 16 + 16;
}

__host__ __device__ constexpr size_t km_lds_bytes(int k, int dp) {
  return ((size_t)dp * km_kps(k) + (size_t)(k + 15) / 16 * 16 + k +
          (size_t)(kKmThreads / 64) * dp) *
             sizeof(double) +
         (2 * kKmThreads + 2 * (size_t)k + kKmThreads / 64 + (kKmThreads / 64) * (size_t)k) *
             sizeof(int);
}

__device__ __forceinline__ void km_take(double v, int c, double& best, int& arg) {
  if (v < best || (v == best && c < arg)) {
    best = v;
    arg = c;
  }
}

// two workgroups per CU (LDS ~65 KB each at k = 100, DP = 64): at most 256 registers
template <int DP>
__global__ void __launch_bounds__(kKmThreads) __attribute__((amdgpu_waves_per_eu(2)))
    kmeans_step_kernel(const double* __restrict__ X, long long ldx, int n, int d,
                       const double* __restrict__ C, int k, const int* __restrict__ live,
                       int* __restrict__ labels, double* __restrict__ mind,
                       double* __restrict__ psum, double* __restrict__ pcnt) {
  extern __shared__ double smem[];
  const int KP = (k + 15) / 16 * 16, KPS = km_kps(k);
  double* sCt = smem;                       // DP x KPS centroids, coordinate-major
  double* sCsq = sCt + (long long)DP * KPS; // KP squared norms (+inf for the padding)
  double* sCnt = sCsq + KP;                 // k counts
  double* sEdge = sCnt + k;                 // [wave][DP] first-run partials (phase B)
  int* sLab = reinterpret_cast<int*>(sEdge + (kKmThreads / 64) * DP);   // 256 round labels
  int* sPerm = sLab + kKmThreads;                   // round's points grouped by label
  int* sHist = sPerm + kKmThreads;                  // k: points per label this round
  int* sOff = sHist + k;                            // k: exclusive prefix of sHist
  int* sEdgeLab = sOff + k;                         // [wave] label of the first run
  int* sWH = sEdgeLab + kKmThreads / 64;            // [wave][k] per-wave label counts
  const int r = blockIdx.y;
  const int n_init = gridDim.y;
  if (live != nullptr && live[r] == 0) return;    // frozen restart: partials unused
  const int tid = threadIdx.x;
  const double* Cr = C + (long long)r * k * d;
  for (int e = tid; e < DP * KPS; e += kKmThreads) {
    const int j = e / KPS, c = e - j * KPS;
    sCt[e] = (c < k && j < d) ? Cr[(long long)c * d + j] : 0.0;
  }
  // the cluster sums accumulate straight in this workgroup's partial slot of psum
  // ([k][d], global memory: only this workgroup touches it) -- in LDS they took 51 KB,
  // which held the kernel to one workgroup (one wave per SIMD) per CU
  double* acc_g = psum != nullptr ? psum + ((long long)blockIdx.x * n_init + r) * k * d : nullptr;
  if (acc_g != nullptr)
    for (int e = tid; e < k * d; e += kKmThreads) acc_g[e] = 0.0;
  for (int c = tid; c < k; c += kKmThreads) sCnt[c] = 0.0;
  __syncthreads();
  // squared norms from the LDS table (independent reads; a walk over the global rows was
  // a chain of dependent loads per centroid)
  for (int c = tid; c < KP; c += kKmThreads) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < DP; ++j) {
      const double v = sCt[j * KPS + c];
      s = fma(v, v, s);
    }
    sCsq[c] = c < k ? s : INFINITY;
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6, col = lane & 15, grp = lane >> 4;
  const int nct = KP >> 4;
  const long long base = (long long)blockIdx.x * (kKmThreads * kKmRounds);
  for (int round = 0; round < kKmRounds; ++round) {
    const long long p0 = base + (long long)round * kKmThreads;
    if (p0 >= n) break;                              // uniform across the workgroup
    // ---- phase A: assignment (MFMA scores)
    // the wave's 4 point tiles are loaded up front (one wave per SIMD: the registers are
    // there, and one memory round trip instead of one per tile)
    double bxa[4][DP / 4];
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const long long i = p0 + 64 * wave + 16 * pt + col;
      const bool ok = i < n;
      const double* xr = X + (ok ? i : 0) * ldx;
#pragma unroll
      for (int ks = 0; ks < DP / 4; ++ks) {
        const int j = 4 * ks + grp;
        bxa[pt][ks] = (ok && j < d) ? xr[j] : 0.0;
      }
    }
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const int slot = 64 * wave + 16 * pt + col;
      const long long i = p0 + slot;
      const bool ok = i < n;
      const double* bx = bxa[pt];
      double xsq = 0.0;
#pragma unroll
      for (int ks = 0; ks < DP / 4; ++ks) xsq = fma(bx[ks], bx[ks], xsq);
      double best = INFINITY;
      int arg = 0x7fffffff;
      for (int ct = 0; ct < nct; ct += 2) {
        const bool two = ct + 1 < nct;                 // uniform
        km_f64x4 a0 = km_f64x4{0.0, 0.0, 0.0, 0.0}, a1 = a0;
        const double* ap = sCt + (long long)grp * KPS + 16 * ct + col;
        // every k-step of the padded DP (the padding is zero on both sides): no branch
        // between the LDS operand loads and their MFMAs, so the loads issue ahead
        double av0[DP / 4], av1[DP / 4];
#pragma unroll
        for (int ks = 0; ks < DP / 4; ++ks) {
          const double* row = ap + (long long)(4 * ks) * KPS;
          av0[ks] = row[0];
          av1[ks] = two ? row[16] : 0.0;
        }
        if (two) {
#pragma unroll
          for (int ks = 0; ks < DP / 4; ++ks) {
            a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av0[ks], bx[ks], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av1[ks], bx[ks], a1, 0, 0, 0);
          }
        } else {              // the odd last tile alone
#pragma unroll
          for (int ks = 0; ks < DP / 4; ++ks)
            a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av0[ks], bx[ks], a0, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = 16 * ct + grp + 4 * q;
          km_take(sCsq[c] - 2.0 * a0[q], c, best, arg);
        }
        if (two) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = 16 * (ct + 1) + grp + 4 * q;
            km_take(sCsq[c] - 2.0 * a1[q], c, best, arg);
          }
        }
      }
      // the point's 4 lane groups hold disjoint centroid subsets: min over them
#pragma unroll
      for (int m = 16; m <= 32; m <<= 1) {
        const double ob = __shfl_xor(best, m);
        const int oa = __shfl_xor(arg, m);
        km_take(ob, oa, best, arg);
        xsq += __shfl_xor(xsq, m);
      }
      if (grp == 0) {
        sLab[slot] = ok ? arg : -1;
        if (ok) {
          labels[(long long)r * n + i] = arg;
          if (mind != nullptr) mind[(long long)r * n + i] = fmax(xsq + best, 0.0);
        }
      }
    }
    __syncthreads();
    // ---- phase B: ordered accumulation (only when partial sums are wanted).  The
    // round's points are grouped by label with a stable counting sort (rank = earlier
    // points with the same label: a broadcast LDS walk); wave w then walks sorted
    // positions [64 w, 64 w + 64) with one lane per coordinate -- coalesced row loads, 16
    // in flight -- keeping a register running sum per run of equal labels.  Every run
    // but the wave's first is a whole cluster of this round and is added to the
    // accumulator directly (no other wave holds that cluster); the first runs may
    // continue a run of the previous wave and are added after a barrier, in wave order.
    // Deterministic: fixed summation order for every (cluster, feature).  (One thread per
    // (cluster, feature) summing its points -- dependent gathered loads -- spent ~4 ms of
    // a 5 ms step at 500k x 50 x 100 x 10 restarts, profiles/r5l_*; d threads walking all
    // 256 points with LDS read-modify-writes took ~11 ms, profiles/r3ae_*.)
    if (psum != nullptr) {
      // stable counting sort of the round's points by label: a point's rank among the
      // earlier points of its label = the same label's count in the earlier waves (per-wave
      // histograms: integer LDS atomics, order-free) + the earlier lanes of its own wave
      // (a v_readlane walk over the 64 labels); cluster offsets by a block scan
      for (int e = tid; e < (kKmThreads / 64) * k; e += kKmThreads) sWH[e] = 0;
      __syncthreads();
      const int lab = sLab[tid];
      int rank = 0;
      for (int j = 0; j < 64; ++j) {
        const int lj = __builtin_amdgcn_readlane(lab, j);
        rank += (j < lane && lj == lab) ? 1 : 0;
      }
      if (lab >= 0) atomicAdd(&sWH[wave * k + lab], 1);
      __syncthreads();
      int tot = 0;
      if (tid < k)
        for (int w = 0; w < kKmThreads / 64; ++w) tot += sWH[w * k + tid];
      int* sScan = sPerm;                        // scratch until the permutation is written
      sScan[tid] = tot;
      __syncthreads();
      for (int dd = 1; dd < kKmThreads; dd <<= 1) {
        const int v = tid >= dd ? sScan[tid - dd] : 0;
        __syncthreads();
        sScan[tid] += v;
        __syncthreads();
      }
      if (tid < k) {
        sOff[tid] = sScan[tid] - tot;
        sHist[tid] = tot;
      }
      __syncthreads();
      if (lab >= 0) {
        for (int w = 0; w < wave; ++w) rank += sWH[w * k + lab];
        sPerm[sOff[lab] + rank] = tid;
      }
      __syncthreads();
      const int nval = (int)min((long long)kKmThreads, (long long)n - p0);
      const int q0 = 64 * wave, q1 = min(q0 + 64, nval);
      const bool jok = lane < d;
      double* edge = sEdge + wave * DP;
      int elab = -1;
      if (q0 < q1) {                                   // uniform
        int cur = sLab[sPerm[q0]];
        double acc = 0.0;
        bool first = true;
        for (int q = q0; q < q1; q += 16) {
          double xv[16];
          int lb[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) {
            const int qq = q + u;
            lb[u] = -2;
            xv[u] = 0.0;
            if (qq < q1) {
              const int pp = sPerm[qq];
              lb[u] = sLab[pp];
              if (jok) xv[u] = X[(p0 + pp) * ldx + lane];
            }
          }
#pragma unroll
          for (int u = 0; u < 16; ++u) {
            if (lb[u] == -2) break;                    // uniform: past the range
            if (lb[u] != cur) {                        // uniform: a run ends
              if (first) {
                if (jok) edge[lane] = acc;
                elab = cur;
                first = false;
              } else if (jok) {
                acc_g[(long long)cur * d + lane] += acc;
              }
              cur = lb[u];
              acc = 0.0;
            }
            acc += xv[u];
          }
        }
        if (first) {
          if (jok) edge[lane] = acc;
          elab = cur;
        } else if (jok) {
          acc_g[(long long)cur * d + lane] += acc;
        }
      }
      if (lane == 0) sEdgeLab[wave] = elab;
      __syncthreads();
      if (tid < d)
        for (int w = 0; w < kKmThreads / 64; ++w) {
          const int c = sEdgeLab[w];
          if (c >= 0) acc_g[(long long)c * d + tid] += sEdge[w * DP + tid];
        }
      for (int c = tid; c < k; c += kKmThreads) sCnt[c] += (double)sHist[c];
    }
    __syncthreads();
  }
  if (psum != nullptr) {
    const long long slot = (long long)blockIdx.x * n_init + r;
    for (int c = tid; c < k; c += kKmThreads) pcnt[slot * k + c] = sCnt[c];
  }
}

template <int DP>
static hipError_t launch_kmeans(const double* X, long long ldx, int n, int d, const double* C,
                                int k, int n_init, const int* live, int* labels, double* mind,
                                double* psum, double* pcnt, hipStream_t stream) {
  const size_t lds = km_lds_bytes(k, DP);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeans_step_kernel<DP>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int per = kKmThreads * kKmRounds;
  const dim3 grid((unsigned)((n + per - 1) / per), (unsigned)n_init);
  hipLaunchKernelGGL(kmeans_step_kernel<DP>, grid, dim3(kKmThreads), lds, stream, X, ldx, n, d, C,
                     k, live, labels, mind, psum, pcnt);
  return hipGetLastError();
}

// ---------------------------------------------------------------------- k-means++ step
// Greedy k-means++ (sklearn _kmeans_plusplus) for every restart at once, low-dimensional
// points (d <= 64): the M = n_init * trials candidates sit in LDS, every thread owns one
// point in registers and, for each candidate m of restart r = m / trials, takes
// min(closest[i][r], |x_i - c_m|^2).
//   mode 0  per-workgroup partial potentials pot[block][m] (summed on the host in block
//           order: deterministic) -- nothing (n x M) is materialised
//   mode 1  the candidates are the chosen centres (trials = 1): closest[i][r] is
//           lowered in place
template <int DP>
__global__ void __launch_bounds__(kKmThreads)
    kmeanspp_kernel(const double* __restrict__ X, long long ldx, int n, int d,
                    const double* __restrict__ C, int M, int trials,
                    double* __restrict__ closest, int n_init, int mode,
                    double* __restrict__ pot) {
  extern __shared__ double smem[];
  double* sC = smem;                      // M * DP candidates (zero padded)
  double* sRed = sC + (long long)M * DP;  // (kKmThreads / 64) * M wave partials
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < M * DP; e += kKmThreads) {
    const int c = e / DP, j = e % DP;
    sC[e] = j < d ? C[(long long)c * d + j] : 0.0;
  }
  __syncthreads();
  const long long i = (long long)blockIdx.x * kKmThreads + tid;
  const bool ok = i < n;
  double x[DP];
  const double* xr = X + (ok ? i : 0) * ldx;
#pragma unroll
  for (int j = 0; j < DP; ++j) x[j] = (ok && j < d) ? xr[j] : 0.0;
  double* cl = closest + (ok ? i : 0) * n_init;
  for (int m = 0; m < M; ++m) {
    const double2* cc = reinterpret_cast<const double2*>(sC + (long long)m * DP);
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < DP / 2; ++j) {
      const double2 v = cc[j];
      const double a = x[2 * j] - v.x, b = x[2 * j + 1] - v.y;
      s0 = fma(a, a, s0);
      s1 = fma(b, b, s1);
    }
    const int r = m / trials;
    const double cur = ok ? cl[r] : 0.0;
    const double v = ok ? fmin(cur, s0 + s1) : 0.0;
    if (mode == 1) {
      if (ok) cl[r] = v;
    } else {
      const double w = wave_sum(v);
      if (lane == 0) sRed[wave * M + m] = w;
    }
  }
  if (mode == 1) return;
  __syncthreads();
  for (int m = tid; m < M; m += kKmThreads) {
    double t = 0.0;
    for (int w = 0; w < kKmThreads / 64; ++w) t += sRed[w * M + m];
    pot[(long long)blockIdx.x * M + m] = t;
  }
}

template <int DP>
static hipError_t launch_kmeanspp(const double* X, long long ldx, int n, int d, const double* C,
                                  int M, int trials, double* closest, int n_init, int mode,
                                  double* pot, hipStream_t stream) {
  const size_t lds = ((size_t)M * DP + (size_t)(kKmThreads / 64) * M) * sizeof(double);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeanspp_kernel<DP>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const dim3 grid((unsigned)((n + kKmThreads - 1) / kKmThreads));
  hipLaunchKernelGGL(kmeanspp_kernel<DP>, grid, dim3(kKmThreads), lds, stream, X, ldx, n, d, C,
                     M, trials, closest, n_init, mode, pot);
  return hipGetLastError();
}

// ------------------------------------------------------------- k-means++ candidate sampling
// Inverse-CDF draw of every restart's candidates from its potential (torch.searchsorted of
// the inclusive prefix sum of closest[:, r], side left): the first point whose running sum
// reaches u * total.  A (n_init x n) cumsum + searchsorted cost ~1.3 ms per centre at 500k
// points (the scan of 10 long rows runs on few workgroups, profiles/r5i_*); here
//   1. ppsum_kernel: block sums of 1024 points per restart (fixed order);
//   2. ppsample_kernel (one workgroup per restart): prefix of the block sums in LDS, a
//      binary search per trial for the block, then a scan of that block's 1024 values.
constexpr int kPpBlock = 1024;

__global__ void __launch_bounds__(256) ppsum_kernel(const double* __restrict__ closest, int n,
                                                    int n_init, double* __restrict__ bsum) {
  __shared__ double red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long p0 = (long long)blockIdx.x * kPpBlock + 4 * tid;
  for (int r = 0; r < n_init; ++r) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (p0 + j < n) s += closest[(p0 + j) * n_init + r];
    s = wave_sum(s);
    if (lane == 0) red[wave] = s;
    __syncthreads();
    if (tid == 0) bsum[(long long)r * gridDim.x + blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
    __syncthreads();
  }
}

// inclusive scan of v over the 1024 threads (Hillis-Steele in LDS)
__device__ __forceinline__ double pp_scan(double v, double* s) {
  const int tid = threadIdx.x;
  s[tid] = v;
  __syncthreads();
  for (int d = 1; d < kPpBlock; d <<= 1) {
    const double a = tid >= d ? s[tid - d] : 0.0;
    __syncthreads();
    s[tid] += a;
    __syncthreads();
  }
  return s[tid];
}

__global__ void __launch_bounds__(kPpBlock) ppsample_kernel(
    const double* __restrict__ closest, int n, int n_init, const double* __restrict__ bsum, int nb,
    const double* __restrict__ u, int trials, long long* __restrict__ cand) {
  extern __shared__ double pre[];          // nb block prefix sums
  __shared__ double sc[kPpBlock];
  __shared__ int s_hit, s_last;
  const int r = blockIdx.x, tid = threadIdx.x;
  double carry = 0.0;
  for (int b0 = 0; b0 < nb; b0 += kPpBlock) {
    const int b = b0 + tid;
    const double v = b < nb ? bsum[(long long)r * nb + b] : 0.0;
    const double inc = pp_scan(v, sc) + carry;
    if (b < nb) pre[b] = inc;
    carry = sc[kPpBlock - 1] + carry;
    __syncthreads();
  }
  const double total = pre[nb - 1];
  for (int t = 0; t < trials; ++t) {
    const double target = u[(long long)r * trials + t] * total;
    // first block whose prefix reaches the target (the last block if none does)
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (pre[mid] >= target) hi = mid; else lo = mid + 1;
    }
    // the block sums' own scan can round a later all-zero block's prefix above the last
    // positive block's: step back to the block holding the last positive weight before it
    // (the target lies past every earlier block's prefix, so the draw is in that block)
    int b = lo;
    while (b > 0 && !(bsum[(long long)r * nb + b] > 0.0)) --b;
    const double base = b > 0 ? pre[b - 1] : 0.0;
    const long long i = (long long)b * kPpBlock + tid;
    const double v = i < n ? closest[i * n_init + r] : 0.0;
    if (tid == 0) {
      s_hit = kPpBlock;
      s_last = -1;
    }
    __syncthreads();
    const double inc = base + pp_scan(v, sc);
    // only points of positive weight can be drawn: the scan's tree order rounds the
    // running sums of different positions differently, and across a stretch of zeros a
    // later (zero-weight) position can reach a target the last positive one missed
    if (inc >= target && i < n && v > 0.0) atomicMin(&s_hit, tid);
    if (v > 0.0 && i < n) atomicMax(&s_last, tid);
    __syncthreads();
    if (tid == 0) {
      // the block sums (ppsum, tree order) and this in-block scan round differently: a
      // target the block's prefix reached may stay just above base + scan.  Then take the
      // block's last point of positive weight (never a zero-potential point: an existing
      // centre or padding), as searchsorted does for a target at the running total
      const int hit = s_hit < kPpBlock ? s_hit : (s_last >= 0 ? s_last : kPpBlock - 1);
      long long idx = (long long)b * kPpBlock + hit;
      if (idx > n - 1) idx = n - 1;
      cand[(long long)r * trials + t] = idx;
    }
    __syncthreads();
  }
}

}  // namespace cnmf

extern "C" int cnmf_kmeanspp_sample_blocks(int n) {
  return (n + cnmf::kPpBlock - 1) / cnmf::kPpBlock;
}

// cand (n_init x trials, int64) from closest (n x n_init, f64) and u (n_init x trials);
// bsum: workspace of n_init * cnmf_kmeanspp_sample_blocks(n) doubles
extern "C" hipError_t cnmf_kmeanspp_sample(const double* closest, int n, int n_init,
                                           const double* u, int trials, double* bsum,
                                           long long* cand, hipStream_t stream) {
  if (n <= 0 || n_init <= 0 || trials <= 0) return hipErrorInvalidValue;
  const int nb = cnmf_kmeanspp_sample_blocks(n);
  const size_t lds = (size_t)nb * sizeof(double);
  if (lds > 120 * 1024) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cnmf::ppsample_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(cnmf::ppsum_kernel, dim3(nb), dim3(256), 0, stream, closest, n, n_init, bsum);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(cnmf::ppsample_kernel, dim3(n_init), dim3(cnmf::kPpBlock), lds, stream,
                     closest, n, n_init, bsum, nb, u, trials, cand);
  return hipGetLastError();
}

extern "C" int cnmf_kmeanspp_blocks(int n) {
  return (n + cnmf::kKmThreads - 1) / cnmf::kKmThreads;
}

extern "C" int cnmf_kmeanspp_fits(int M, int d) {
  if (M < 1 || d < 1 || d > 64) return 0;
  const int dp = (d + 15) / 16 * 16;
  return ((size_t)M * dp + (size_t)(cnmf::kKmThreads / 64) * M) * sizeof(double) <= 150 * 1024;
}

extern "C" hipError_t cnmf_kmeanspp(const double* X, long long ldx, int n, int d,
                                    const double* C, int M, int trials, double* closest,
                                    int n_init, int mode, double* pot, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (!cnmf_kmeanspp_fits(M, d) || trials < 1 || M % trials || M / trials != n_init ||
      (mode == 0 && pot == nullptr) || (mode != 0 && mode != 1))
    return hipErrorInvalidValue;
  const int dp = (d + 15) / 16 * 16;
  switch (dp) {
    case 16: return cnmf::launch_kmeanspp<16>(X, ldx, n, d, C, M, trials, closest, n_init, mode, pot, stream);
    case 32: return cnmf::launch_kmeanspp<32>(X, ldx, n, d, C, M, trials, closest, n_init, mode, pot, stream);
    case 48: return cnmf::launch_kmeanspp<48>(X, ldx, n, d, C, M, trials, closest, n_init, mode, pot, stream);
    default: return cnmf::launch_kmeanspp<64>(X, ldx, n, d, C, M, trials, closest, n_init, mode, pot, stream);
  }
}

extern "C" int cnmf_kmeans_blocks(int n) {
  const int per = cnmf::kKmThreads * cnmf::kKmRounds;
  return (n + per - 1) / per;
}

// padded dimension of the Lloyd kernel: a multiple of 16, or 52 for the common 50 PCs (13
// MFMA k-steps instead of 16)
static int km_dp(int d) { return d <= 48 ? (d + 15) / 16 * 16 : d <= 52 ? 52 : 64; }

// Whether the LDS budget (160 KiB per CU) holds the transposed centroid table, the
// accumulator and the label arrays of (k, d).
extern "C" int cnmf_kmeans_fits(int k, int d) {
  if (k < 1 || k > cnmf::kKmThreads || d < 1 || d > 64) return 0;
  return cnmf::km_lds_bytes(k, km_dp(d)) <= 156 * 1024 ? 1 : 0;
}

extern "C" hipError_t cnmf_kmeans_step(const double* X, long long ldx, int n, int d,
                                       const double* C, int k, int n_init, const int* live,
                                       int* labels, double* mind, double* psum, double* pcnt,
                                       hipStream_t stream) {
  if (n <= 0 || n_init <= 0) return hipSuccess;
  if (!cnmf_kmeans_fits(k, d)) return hipErrorInvalidValue;
  switch (km_dp(d)) {
    case 16: return cnmf::launch_kmeans<16>(X, ldx, n, d, C, k, n_init, live, labels, mind, psum, pcnt, stream);
    case 32: return cnmf::launch_kmeans<32>(X, ldx, n, d, C, k, n_init, live, labels, mind, psum, pcnt, stream);
    case 48: return cnmf::launch_kmeans<48>(X, ldx, n, d, C, k, n_init, live, labels, mind, psum, pcnt, stream);
    case 52: return cnmf::launch_kmeans<52>(X, ldx, n, d, C, k, n_init, live, labels, mind, psum, pcnt, stream);
    default: return cnmf::launch_kmeans<64>(X, ldx, n, d, C, k, n_init, live, labels, mind, psum, pcnt, stream);
  }
}
