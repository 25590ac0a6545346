// Argument block of the continuous-batching swap kernels (stream.hip), shared with the
// pybind layer (bindings.cpp fills it field by field from the Python ops wrapper).
#pragma once
#include <hip/hip_runtime.h>

namespace cnmf {

struct StreamSwap {
  int n, K, G, N, S, Gp;      // positions of the group, rank, spectra / usage columns,
                              // partial-Gram slots, planes k pitch
  const int* active;          // [n] the group's active flags
  int* occ;                   // [n] occupant replicate id, -1 = free
  int* plan;                  // [2n] ring entry placed per position, harvested id per position
  double* sf; long long sf_ld;          // batch state (3 rows) at the group's first column
  int* si; long long si_ld;             // (5 rows)
  float* W; long long ldw;              // group rows (K per position)
  float* HT; long long ldh;
  float* parts;                         // (n, S, K, K)
  unsigned short* wpl; long long pl_ld, pl_plane;   // (3 planes, rows, Gp)
  int qc;                               // ring capacity
  int* head; const int* tail;           // ring entries consumed / published
  const int* ring_id;                   // [qc] replicate id of each ring slot
  const float* rW; const float* rHT;    // (qc K, G), (qc K, N)
  const double* rsf; const int* rsi;    // (3, qc), (5, qc)
  const float* rparts;                  // (qc, S, K, K)
  const unsigned short* rwpl; long long rpl_plane;  // (3, qc K, Gp)
  const long long* offs;                // [R] store row of replicate id
  float* oW; float* oHT;                // (sum K, G), (sum K, N) or null
  double* osf; long long osf_ld;        // (3, R)
  int* osi; long long osi_ld;           // (5, R)
  int* done;                            // harvested replicates
  int* gate;
};

// One matrix of a compaction swap (rows_swap_kernel): `planes` planes `plane` elements
// apart, K rows per position at row pitch `ld`, `cols` columns of `esz`-byte elements.
struct SwapMat {
  void* p; long long ld; long long plane; int cols; int esz; int planes;
};

struct RowsSwap {
  int K;                       // rows per position
  const int* pairs;            // [2 npairs] disjoint position pairs
  int nmat;                    // matrices in `mat` (<= 4)
  SwapMat mat[4];
  double* sf; long long sf_ld; int nsf;   // per-position float64 state rows
  int* si; long long si_ld; int nsi;      // per-position int32 state rows
};

}  // namespace cnmf
