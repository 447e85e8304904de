// host_pcg64.cpp — numpy SeedSequence -> PCG64 seeding on the host
// (reference: delta_node/utils/arr.py:21-24 `np.random.default_rng(seed)`).
//
// Restates numpy/random/bit_generator.pyx SeedSequence (hashmix, mix,
// mix_entropy with pool_size 4, generate_state) and _pcg64.pyx / pcg64.h
// seeding: generate_state(4, uint64) -> seed = v0:v1, inc = v2:v3 ->
// pcg_setseq_128_srandom_r (state = 0; inc = 2 inc + 1; step; state += seed; step).
#include <cstring>

#include "dn_internal.hpp"
#include "dn_mask.h"
#include "pcg64_common.hpp"

namespace dn {
namespace {
constexpr uint32_t kInitA = 0x43b0d7e5u, kMultA = 0x931e8875u;
constexpr uint32_t kInitB = 0x8b51f9ddu, kMultB = 0x58f38dedu;
constexpr uint32_t kMixL = 0xca01f9ddu, kMixR = 0x4973f715u;
constexpr int kXShift = 16, kPool = 4;

uint32_t hashmix(uint32_t value, uint32_t& hc) {
  value ^= hc;
  hc *= kMultA;
  value *= hc;
  return value ^ (value >> kXShift);
}

uint32_t mix(uint32_t x, uint32_t y) {
  uint32_t r = kMixL * x - kMixR * y;
  return r ^ (r >> kXShift);
}
}  // namespace
}  // namespace dn

using namespace dn;

extern "C" int dn_pcg64_seed(const uint32_t* entropy, int n_words, dn_pcg64_t* out) {
  if (!out || n_words < 0 || (n_words > 0 && !entropy)) return set_error(DN_ERR_ARG, "dn_pcg64_seed: bad arguments");
  uint32_t pool[kPool];
  uint32_t hc = kInitA;
  for (int i = 0; i < kPool; ++i) pool[i] = hashmix(i < n_words ? entropy[i] : 0u, hc);
  for (int s = 0; s < kPool; ++s)
    for (int d = 0; d < kPool; ++d)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s], hc));
  for (int s = kPool; s < n_words; ++s)
    for (int d = 0; d < kPool; ++d) pool[d] = mix(pool[d], hashmix(entropy[s], hc));
  uint32_t w[8];
  uint32_t hb = kInitB;
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i % kPool] ^ hb;
    hb *= kMultB;
    v *= hb;
    w[i] = v ^ (v >> kXShift);
  }
  uint64_t v64[4];
  for (int i = 0; i < 4; ++i) v64[i] = static_cast<uint64_t>(w[2 * i]) | (static_cast<uint64_t>(w[2 * i + 1]) << 32);
  const u128 seed = to_u128(v64[0], v64[1]);
  const u128 init_inc = to_u128(v64[2], v64[3]);
  const u128 a = pcg64_mult();
  const u128 inc = (init_inc << 1) | 1u;
  u128 state = 0;
  state = state * a + inc;
  state += seed;
  state = state * a + inc;
  out->state_hi = static_cast<uint64_t>(state >> 64);
  out->state_lo = static_cast<uint64_t>(state);
  out->inc_hi = static_cast<uint64_t>(inc >> 64);
  out->inc_lo = static_cast<uint64_t>(inc);
  return DN_OK;
}

extern "C" int dn_pcg64_advance(dn_pcg64_t* g, uint64_t delta) {
  if (!g) return set_error(DN_ERR_ARG, "dn_pcg64_advance: null pointer");
  u128 jA[64], jG[64];
  pcg64_jump_tables(jA, jG);
  u128 A = 1, G = 0;
  for (int k = 0; k < 64; ++k)
    if ((delta >> k) & 1u) {
      G = jA[k] * G + jG[k];
      A = jA[k] * A;
    }
  const u128 inc = to_u128(g->inc_hi, g->inc_lo);
  const u128 s = A * to_u128(g->state_hi, g->state_lo) + inc * G;
  g->state_hi = static_cast<uint64_t>(s >> 64);
  g->state_lo = static_cast<uint64_t>(s);
  return DN_OK;
}
