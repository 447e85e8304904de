// chacha_device.hpp — the ChaCha block function on gfx950 lanes, and the
// coefficient stream of dn_m521_split_prng (include/dn_shamir.h).
//
// Block: Bernstein's ChaCha, state words 0-3 "expand 32-byte k", 4-11 key,
// 12-13 a 64-bit block counter, 14-15 a 64-bit nonce; `rounds` in {8,12,20}.
// Coefficient index i = g * (t-1) + (j-1) for global element g, coefficient
// j = 1..t-1: limbs 0..15 = block i; limb 16 (9 bits) = word i % 16 of block
// kTopDomain + i / 16; values >= p - 1 are redrawn from kRetryDomain (the
// reject rule of randint(1, p-1), shamir.py:59-61) and 1 is added.
// Restated on the CPU in oracle/chacha_oracle.c (test infrastructure).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dn {

constexpr uint64_t kTopDomain = 1ull << 62;
constexpr uint64_t kRetryDomain = 1ull << 63;

struct ChachaKey {
  uint32_t k[8];
  uint32_t n0, n1;  // nonce words 14, 15
  int32_t rounds;
  int32_t pad;
};

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }

__device__ __forceinline__ void chacha_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  a += b; d ^= a; d = rotl32(d, 16);
  c += d; b ^= c; b = rotl32(b, 12);
  a += b; d ^= a; d = rotl32(d, 8);
  c += d; b ^= c; b = rotl32(b, 7);
}

// x <- ChaCha block (counter) of key/nonce, in place (16 VGPRs).
__device__ __forceinline__ void chacha_block(uint32_t x[16], const ChachaKey& K, uint64_t counter) {
  const uint32_t c0 = static_cast<uint32_t>(counter), c1 = static_cast<uint32_t>(counter >> 32);
  x[0] = 0x61707865u; x[1] = 0x3320646eu; x[2] = 0x79622d32u; x[3] = 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[4 + i] = K.k[i];
  x[12] = c0; x[13] = c1; x[14] = K.n0; x[15] = K.n1;
#pragma unroll 1
  for (int r = 0; r < K.rounds; r += 2) {
    chacha_qr(x[0], x[4], x[8], x[12]);
    chacha_qr(x[1], x[5], x[9], x[13]);
    chacha_qr(x[2], x[6], x[10], x[14]);
    chacha_qr(x[3], x[7], x[11], x[15]);
    chacha_qr(x[0], x[5], x[10], x[15]);
    chacha_qr(x[1], x[6], x[11], x[12]);
    chacha_qr(x[2], x[7], x[8], x[13]);
    chacha_qr(x[3], x[4], x[9], x[14]);
  }
  x[0] += 0x61707865u; x[1] += 0x3320646eu; x[2] += 0x79622d32u; x[3] += 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[4 + i] += K.k[i];
  x[12] += c0; x[13] += c1; x[14] += K.n0; x[15] += K.n1;
}

// v >= p - 1 (limb 16 already masked to 9 bits).
__device__ __forceinline__ bool prng_rejected(const uint32_t v[17]) {
  uint32_t all = v[1];
#pragma unroll
  for (int i = 2; i < 16; ++i) all &= v[i];
  return v[16] == 0x1FFu && all == 0xFFFFFFFFu && v[0] >= 0xFFFFFFFEu;
}

// Redraw (odds 2^-520 per coefficient; never taken in practice, kept exact).
// Uses v itself as the block buffer: the top-limb block first (keeping word
// 0), then the low block — no extra registers on the hot path.
__device__ __forceinline__ void prng_retry(uint32_t v[17], const ChachaKey& K, uint64_t i) {
#pragma unroll 1
  for (uint32_t attempt = 0;; ++attempt) {
    const uint64_t c = kRetryDomain + (i << 6) + 2ull * (attempt & 31u);
    chacha_block(v, K, c + 1);
    const uint32_t top = v[0] & 0x1FFu;
    chacha_block(v, K, c);
    v[16] = top;
    if (!prng_rejected(v)) return;
  }
}

}  // namespace dn
