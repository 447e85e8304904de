/* chacha_oracle.c — CPU restatement of the device-PRNG coefficient stream of
 * dn_m521_split_prng (include/dn_shamir.h).  TEST INFRASTRUCTURE ONLY.
 *
 * Not a reference algorithm: the reference draws coefficients from CPython's
 * MT19937 (delta_node/crypto/shamir/shamir.py:59-61, restated in
 * m521_oracle.c).  This is SURVEY.md §8(b)'s dn_m521_split_prng / §8(d)
 * config 2' — coefficients generated on the device from a keyed stream
 * cipher, with the reference's randint(1, p-1) rejection rule.  The ChaCha
 * block function is Bernstein's ChaCha with 64-bit block counter (words 12-13)
 * and 64-bit nonce (words 14-15); pinned against OpenSSL's `enc -chacha20`
 * keystream (tests/golden/make_golden_chacha.py -> chacha_kat.json).
 */
#include <stdint.h>
#include <string.h>

#define ROTL(x, n) (((x) << (n)) | ((x) >> (32 - (n))))
#define QR(a, b, c, d)                         \
  do {                                         \
    a += b; d ^= a; d = ROTL(d, 16);           \
    c += d; b ^= c; b = ROTL(b, 12);           \
    a += b; d ^= a; d = ROTL(d, 8);            \
    c += d; b ^= c; b = ROTL(b, 7);            \
  } while (0)

void oracle_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t nonce, int rounds, uint32_t out[16]) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  memcpy(in + 4, key, 32);
  in[12] = (uint32_t)counter;
  in[13] = (uint32_t)(counter >> 32);
  in[14] = (uint32_t)nonce;
  in[15] = (uint32_t)(nonce >> 32);
  uint32_t x[16];
  memcpy(x, in, sizeof(x));
  for (int r = 0; r < rounds; r += 2) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

#define TOP_DOMAIN (1ull << 62)
#define RETRY_DOMAIN (1ull << 63)

/* v >= p - 1 = 2^521 - 2 (the values randint's _randbelow(p-1) rejects). */
static int rejected(const uint32_t v[17]) {
  if (v[16] != 0x1FFu) return 0;
  for (int i = 1; i < 16; ++i)
    if (v[i] != 0xFFFFFFFFu) return 0;
  return v[0] >= 0xFFFFFFFEu;
}

/* Coefficient index i (= g * (t-1) + j - 1) -> 17 limbs in [1, p-1]. */
void oracle_prng_coeff(const uint32_t key[8], uint64_t nonce, int rounds, uint64_t i, uint32_t v[17]) {
  uint32_t blk[16];
  oracle_chacha_block(key, i, nonce, rounds, v); /* limbs 0..15 */
  oracle_chacha_block(key, TOP_DOMAIN + i / 16, nonce, rounds, blk);
  v[16] = blk[i % 16] & 0x1FFu;
  for (uint32_t attempt = 0; rejected(v); ++attempt) {
    const uint64_t c = RETRY_DOMAIN + (i << 6) + 2ull * (attempt & 31u);
    oracle_chacha_block(key, c, nonce, rounds, v);
    oracle_chacha_block(key, c + 1, nonce, rounds, blk);
    v[16] = blk[0] & 0x1FFu;
  }
  /* + 1 (no carry out: v < p - 1) */
  for (int k = 0; k < 17; ++k) {
    if (++v[k] != 0) break;
  }
}

/* Coefficients of elements elem_offset .. elem_offset + n - 1: out [n][tm1][17]. */
void oracle_prng_coeffs(const uint32_t key[8], uint64_t nonce, int rounds, uint64_t elem_offset, uint64_t n, int tm1,
                        uint32_t* out) {
  for (uint64_t e = 0; e < n; ++e)
    for (int j = 0; j < tm1; ++j)
      oracle_prng_coeff(key, nonce, rounds, (elem_offset + e) * (uint64_t)tm1 + (uint64_t)j,
                        out + (e * (uint64_t)tm1 + (uint64_t)j) * 17u);
}
