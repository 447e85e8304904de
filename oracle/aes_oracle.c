/* aes_oracle.c — CPU restatement of the share envelope's cipher.  TEST
 * INFRASTRUCTURE ONLY (tests/ and bench.py's cpu_baseline leg).
 *
 * Reference: delta_node/crypto/aes/aes.py:8-23 —
 *   encrypt(key, data) = b64encode(nonce + AES(key).CTR(nonce).update(data)),
 * with key = the 32-byte SHA-256 ECDH digest (crypto/ecdhe/ecdhe.py:23-34),
 * i.e. AES-256.  `cryptography`'s CTR mode (OpenSSL) treats the 16-byte nonce
 * as a 128-bit big-endian counter block incremented once per 16-byte block,
 * wrapping mod 2^128.  `cryptography` is not installed here; this is FIPS-197
 * AES (byte-oriented: S-box from the GF(2^8) inverse and the affine map,
 * 128/192/256-bit keys) with SP 800-38A CTR, pinned by FIPS-197 C.1-C.3,
 * SP 800-38A F.5.1/F.5.5 and `openssl enc -aes-*-ctr` outputs
 * (tests/golden/make_golden_aes.py -> aes_kat.json).
 */
#include <stdint.h>
#include <string.h>

static uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1B : 0)); }

static uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = xtime(a);
    b >>= 1;
  }
  return r;
}

static uint8_t sbox_of(uint8_t x) {
  uint8_t inv = 1, base = x; /* x^254 = x^-1 in GF(2^8), 0 -> 0 */
  for (int e = 254; e; e >>= 1) {
    if (e & 1) inv = gmul(inv, base);
    base = gmul(base, base);
  }
  if (x == 0) inv = 0;
  uint8_t s = 0x63; /* affine map: b_i ^ b_{i+4} ^ b_{i+5} ^ b_{i+6} ^ b_{i+7} ^ c_i */
  for (int i = 0; i < 8; ++i) {
    const int bit = ((inv >> i) ^ (inv >> ((i + 4) & 7)) ^ (inv >> ((i + 5) & 7)) ^ (inv >> ((i + 6) & 7)) ^
                     (inv >> ((i + 7) & 7))) & 1;
    s ^= (uint8_t)(bit << i);
  }
  return s;
}

static uint8_t SBOX[256];
static int sbox_ready = 0;

static void init_sbox(void) {
  if (sbox_ready) return;
  for (int i = 0; i < 256; ++i) SBOX[i] = sbox_of((uint8_t)i);
  sbox_ready = 1;
}

uint8_t oracle_aes_sbox(uint8_t x) {
  init_sbox();
  return SBOX[x];
}

/* Key schedule (FIPS-197 §5.2): nk = 4, 6 or 8 key words, nr = nk + 6
 * rounds; rk = 16 (nr + 1) bytes, round r = bytes 16r..16r+15.  Returns nr. */
int oracle_aes_expand(const uint8_t* key, int key_bytes, uint8_t* rk) {
  init_sbox();
  const int nk = key_bytes / 4, nr = nk + 6, total = 4 * (nr + 1);
  memcpy(rk, key, (size_t)key_bytes);
  uint8_t rcon = 1;
  for (int i = nk; i < total; ++i) {
    uint8_t t[4];
    memcpy(t, rk + 4 * (i - 1), 4);
    if (i % nk == 0) {
      const uint8_t t0 = t[0];
      t[0] = (uint8_t)(SBOX[t[1]] ^ rcon);
      t[1] = SBOX[t[2]];
      t[2] = SBOX[t[3]];
      t[3] = SBOX[t0];
      rcon = xtime(rcon);
    } else if (nk > 6 && i % nk == 4) {
      for (int j = 0; j < 4; ++j) t[j] = SBOX[t[j]];
    }
    for (int j = 0; j < 4; ++j) rk[4 * i + j] = (uint8_t)(rk[4 * (i - nk) + j] ^ t[j]);
  }
  return nr;
}

static void encrypt_block(const uint8_t* rk, int nr, const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16];
  for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(in[i] ^ rk[i]);
  for (int r = 1; r <= nr; ++r) {
    uint8_t u[16];
    for (int c = 0; c < 4; ++c) /* SubBytes + ShiftRows (row q rotates left by q) */
      for (int q = 0; q < 4; ++q) u[4 * c + q] = SBOX[s[4 * ((c + q) & 3) + q]];
    if (r < nr) {
      for (int c = 0; c < 4; ++c) { /* MixColumns */
        const uint8_t a0 = u[4 * c], a1 = u[4 * c + 1], a2 = u[4 * c + 2], a3 = u[4 * c + 3];
        s[4 * c + 0] = (uint8_t)(gmul(a0, 2) ^ gmul(a1, 3) ^ a2 ^ a3);
        s[4 * c + 1] = (uint8_t)(a0 ^ gmul(a1, 2) ^ gmul(a2, 3) ^ a3);
        s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ gmul(a2, 2) ^ gmul(a3, 3));
        s[4 * c + 3] = (uint8_t)(gmul(a0, 3) ^ a1 ^ a2 ^ gmul(a3, 2));
      }
    } else {
      memcpy(s, u, 16);
    }
    for (int i = 0; i < 16; ++i) s[i] ^= rk[16 * r + i];
  }
  memcpy(out, s, 16);
}

void oracle_aes_block(const uint8_t* key, int key_bytes, const uint8_t in[16], uint8_t out[16]) {
  uint8_t rk[240];
  const int nr = oracle_aes_expand(key, key_bytes, rk);
  encrypt_block(rk, nr, in, out);
}

/* out = in XOR keystream; keystream block b = AES(iv + b mod 2^128). */
void oracle_aes_ctr(const uint8_t* key, int key_bytes, const uint8_t iv[16], const uint8_t* in, uint8_t* out,
                    uint64_t n) {
  uint8_t rk[240], ctr[16], ks[16];
  const int nr = oracle_aes_expand(key, key_bytes, rk);
  memcpy(ctr, iv, 16);
  for (uint64_t off = 0; off < n; off += 16) {
    encrypt_block(rk, nr, ctr, ks);
    const uint64_t m = n - off < 16 ? n - off : 16;
    for (uint64_t i = 0; i < m; ++i) out[off + i] = (uint8_t)(in[off + i] ^ ks[i]);
    for (int i = 15; i >= 0; --i)
      if (++ctr[i] != 0) break;
  }
}
