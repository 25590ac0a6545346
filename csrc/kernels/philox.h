// Philox4x32-10 counter-based RNG shared by device kernels and the host oracle.
//
// Replicate initialisation in cnmf_torch_amd is keyed by (nmf_seed, stream, element):
// the same replicate gets the same W/H init on any device, rank or batch position,
// which is what makes replicate-parallel results independent of the ledger sharding
// (SURVEY.md §7.4 item 6).  The numpy twin lives in cnmf_torch_amd/utils/rng.py and
// must stay bit-identical on the uniform stream.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define CNMF_HD __host__ __device__ __forceinline__
#else
#define CNMF_HD inline
#endif

namespace cnmf {

struct u32x4 { uint32_t x, y, z, w; };

CNMF_HD void mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
  const uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  *lo = (uint32_t)p;
}

// 10 rounds, Random123 constants.
CNMF_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c.x, &hi0, &lo0);
    mulhilo32(0xCD9E8D57u, c.z, &hi1, &lo1);
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
  }
  return c;
}

// Uniform in the open interval (0, 1), 32-bit resolution.
CNMF_HD double u32_to_open01(uint32_t v) { return ((double)v + 0.5) * 2.3283064365386963e-10; }

}  // namespace cnmf
