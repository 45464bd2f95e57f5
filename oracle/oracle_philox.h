/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product.
 *
 * Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3",
 * SC'11), the counter-based generator that the HIP kernels use for every
 * in-kernel draw.  Restated here independently of
 * omniisaacgymenvs_loop_amd/csrc/philox.h so the oracle can regenerate the
 * kernel's uniform streams; pinned by the Random123 known-answer vectors in
 * tests/test_oracle_golden.py.
 *
 * The reference draws with torch.rand / torch.rand_like (torch CPU/CUDA
 * generators), whose streams cannot be reproduced; parity against the
 * reference therefore injects the reference's recorded draws (tests/golden).
 */
#ifndef ORACLE_PHILOX_H
#define ORACLE_PHILOX_H
#include <stdint.h>

static inline void oph_round(uint32_t c[4], const uint32_t k[2]) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  const uint32_t n0 = hi1 ^ c[1] ^ k[0];
  const uint32_t n2 = hi0 ^ c[3] ^ k[1];
  c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}

static inline void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  uint32_t k[2] = {key[0], key[1]};
  for (int r = 0; r < 10; ++r) {
    oph_round(c, k);
    if (r < 9) { k[0] += 0x9E3779B9u; k[1] += 0xBB67AE85u; }
  }
  out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = c[3];
}

/* uniform in [0,1) with 24 random mantissa bits (same mapping as torch.rand) */
static inline float oracle_u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

#endif
