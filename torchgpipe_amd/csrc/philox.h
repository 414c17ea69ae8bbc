// Philox4x32-10 counter-based RNG (Salmon et al., SC'11) for gfx950.
//
// Convention used by every framework RNG op (and mirrored bit-for-bit by the
// pure-PyTorch reference in torchgpipe_amd/ops/philox.py):
//   key     = (seed_lo32, seed_hi32 ^ kDomain)
//   counter = (index_lo32, index_hi32, offset_lo32, offset_hi32)
//   uniform = (word >> 8) * 2^-24  in [0, 1)
// `offset` comes from the device generator (reserved per op call, recorded
// on an RngTape for checkpoint replay), `index` enumerates the random draws
// of one op call.  kDomain separates this stream from PyTorch's own Philox
// use of the same generator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tgpipe {

constexpr uint32_t kPhiloxM0 = 0xD2511F53u;
constexpr uint32_t kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u;
constexpr uint32_t kPhiloxW1 = 0xBB67AE85u;
constexpr uint32_t kDomain = 0x7467706Du;  // "tgpm"

struct PhiloxOut {
  uint32_t v[4];
};

__device__ __forceinline__ PhiloxOut philox4x32_10(uint64_t index, uint64_t offset, uint64_t seed) {
  uint32_t c0 = static_cast<uint32_t>(index);
  uint32_t c1 = static_cast<uint32_t>(index >> 32);
  uint32_t c2 = static_cast<uint32_t>(offset);
  uint32_t c3 = static_cast<uint32_t>(offset >> 32);
  uint32_t k0 = static_cast<uint32_t>(seed);
  uint32_t k1 = static_cast<uint32_t>(seed >> 32) ^ kDomain;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = kPhiloxM0 * c0;
    const uint32_t hi0 = __umulhi(kPhiloxM0, c0);
    const uint32_t lo1 = kPhiloxM1 * c2;
    const uint32_t hi1 = __umulhi(kPhiloxM1, c2);
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += kPhiloxW0;
    k1 += kPhiloxW1;
  }
  PhiloxOut o;
  o.v[0] = c0;
  o.v[1] = c1;
  o.v[2] = c2;
  o.v[3] = c3;
  return o;
}

__device__ __forceinline__ float philox_uniform(uint32_t word) {
  return static_cast<float>(word >> 8) * (1.0f / 16777216.0f);
}

}  // namespace tgpipe
