// host_aes.cpp — the share envelope's byte API on the calling core.
//
// Reference: delta_node/crypto/aes/aes.py:8-23 (Cipher(AES(key), CTR(nonce))
// over OpenSSL, then base64), called once per share per peer on ~70-byte
// payloads (runner/horizontal/agg.py:192-196 encrypt, :258 / :265 decrypt).
// A GPU launch and two PCIe copies cost ~100x a 70-byte message's cipher
// work, so `aes.encrypt` / `aes.decrypt` (bytes in, bytes out) run here; the
// vector forms (`encrypt_vec` / `decrypt_vec`, aes_envelope.hip) stay on the
// GPU.  Same key schedule as the device (dn_aes_expand_key, FIPS-197 words),
// the same CTR convention (128-bit big-endian counter block, +1 per 16-byte
// block, mod 2^128), the same text (base64 of nonce || ct, optionally its
// lowercase hex).
//
// Cipher: AES-NI (aesenc / aesenclast, eight counter blocks in flight) when
// the CPU has it (__builtin_cpu_supports), else a table implementation
// (T-tables built from the S-box at first use).  Both are checked against
// FIPS-197, SP 800-38A and the `openssl enc` vectors (tests/test_host_aes.py).
#include <immintrin.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "dn_aes.h"
#include "dn_internal.hpp"

namespace dn {
namespace {

// ---- table cipher (no AES-NI) -----------------------------------------------
struct Tables {
  uint8_t sbox[256];
  uint32_t te[4][256];  // te[k][x] = rotr(te[0][x], 8 k), te[0][x] = (2s, s, s, 3s) big-endian
};

const Tables& tables() {
  static Tables t;
  static std::once_flag once;
  std::call_once(once, [] {
    auto xt = [](uint32_t a) { return ((a << 1) ^ ((a & 0x80u) ? 0x1Bu : 0u)) & 0xFFu; };
    auto mul = [&](uint32_t a, uint32_t b) {
      uint32_t r = 0;
      for (; b; b >>= 1, a = xt(a))
        if (b & 1u) r ^= a;
      return r;
    };
    for (uint32_t x = 0; x < 256; ++x) {
      uint32_t inv = 0;  // multiplicative inverse in GF(2^8) (0 -> 0)
      for (uint32_t y = 1; y < 256 && x; ++y)
        if (mul(x, y) == 1u) {
          inv = y;
          break;
        }
      uint32_t s = inv;
      for (int i = 1; i < 5; ++i) s ^= ((inv << i) | (inv >> (8 - i))) & 0xFFu;
      t.sbox[x] = static_cast<uint8_t>(s ^ 0x63u);
    }
    for (uint32_t x = 0; x < 256; ++x) {
      const uint32_t s = t.sbox[x], s2 = xt(s), s3 = s2 ^ s;
      const uint32_t w = (s2 << 24) | (s << 16) | (s << 8) | s3;
      for (int k = 0; k < 4; ++k) t.te[k][x] = k ? (w >> (8 * k)) | (w << (32 - 8 * k)) : w;
    }
  });
  return t;
}

// ---- schedule ----------------------------------------------------------------
// FIPS-197 §5.2, the same words as dn_aes_expand_key (aes_envelope.hip, whose
// S-box is computed per call: ~6 us a key) with the S-box from the table
// (~0.1 us): the byte API expands the peer's key on every call.
struct Sched {
  uint32_t w[60];      // w[i], big-endian words
  uint8_t bytes[240];  // the same round keys as bytes (AES-NI loads)
  int nr = 0;
};

int schedule(const uint8_t* key, int key_bytes, Sched& s) {
  if (!key) return set_error(DN_ERR_ARG, "AES: null key");
  if (key_bytes != 16 && key_bytes != 24 && key_bytes != 32)
    return set_error(DN_ERR_ARG, "Invalid key size (%d) for AES.", key_bytes * 8);
  const uint8_t* sb = tables().sbox;
  auto sub = [sb](uint32_t t) {
    return (static_cast<uint32_t>(sb[t >> 24]) << 24) | (static_cast<uint32_t>(sb[(t >> 16) & 255]) << 16) |
           (static_cast<uint32_t>(sb[(t >> 8) & 255]) << 8) | sb[t & 255];
  };
  const int nk = key_bytes / 4, nr = nk + 6, total = 4 * (nr + 1);
  for (int i = 0; i < nk; ++i)
    s.w[i] = (static_cast<uint32_t>(key[4 * i]) << 24) | (static_cast<uint32_t>(key[4 * i + 1]) << 16) |
             (static_cast<uint32_t>(key[4 * i + 2]) << 8) | key[4 * i + 3];
  uint32_t rcon = 1u;
  for (int i = nk; i < total; ++i) {
    uint32_t t = s.w[i - 1];
    if (i % nk == 0) {
      t = sub((t << 8) | (t >> 24)) ^ (rcon << 24);
      rcon = ((rcon << 1) ^ ((rcon & 0x80u) ? 0x1Bu : 0u)) & 0xFFu;
    } else if (nk > 6 && i % nk == 4) {
      t = sub(t);
    }
    s.w[i] = s.w[i - nk] ^ t;
  }
  s.nr = nr;
  for (int i = 0; i < total; ++i)
    for (int b = 0; b < 4; ++b) s.bytes[4 * i + b] = static_cast<uint8_t>(s.w[i] >> (24 - 8 * b));
  return DN_OK;
}

// one block, big-endian state words in / out
void block_table(const Sched& s, const uint32_t in[4], uint32_t out[4]) {
  const Tables& T = tables();
  uint32_t a0 = in[0] ^ s.w[0], a1 = in[1] ^ s.w[1], a2 = in[2] ^ s.w[2], a3 = in[3] ^ s.w[3];
  for (int r = 1; r < s.nr; ++r) {
    const uint32_t* k = s.w + 4 * r;
    const uint32_t b0 = T.te[0][a0 >> 24] ^ T.te[1][(a1 >> 16) & 255] ^ T.te[2][(a2 >> 8) & 255] ^ T.te[3][a3 & 255] ^ k[0];
    const uint32_t b1 = T.te[0][a1 >> 24] ^ T.te[1][(a2 >> 16) & 255] ^ T.te[2][(a3 >> 8) & 255] ^ T.te[3][a0 & 255] ^ k[1];
    const uint32_t b2 = T.te[0][a2 >> 24] ^ T.te[1][(a3 >> 16) & 255] ^ T.te[2][(a0 >> 8) & 255] ^ T.te[3][a1 & 255] ^ k[2];
    const uint32_t b3 = T.te[0][a3 >> 24] ^ T.te[1][(a0 >> 16) & 255] ^ T.te[2][(a1 >> 8) & 255] ^ T.te[3][a2 & 255] ^ k[3];
    a0 = b0, a1 = b1, a2 = b2, a3 = b3;
  }
  const uint32_t* k = s.w + 4 * s.nr;
  auto last = [&](uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
    return (static_cast<uint32_t>(T.sbox[x0 >> 24]) << 24) | (static_cast<uint32_t>(T.sbox[(x1 >> 16) & 255]) << 16) |
           (static_cast<uint32_t>(T.sbox[(x2 >> 8) & 255]) << 8) | T.sbox[x3 & 255];
  };
  out[0] = last(a0, a1, a2, a3) ^ k[0];
  out[1] = last(a1, a2, a3, a0) ^ k[1];
  out[2] = last(a2, a3, a0, a1) ^ k[2];
  out[3] = last(a3, a0, a1, a2) ^ k[3];
}

// the counter block as (hi, lo) 64-bit halves of the big-endian 128-bit integer
struct Ctr {
  uint64_t hi, lo;
  void next() {
    if (++lo == 0) ++hi;
  }
};

Ctr load_ctr(const uint8_t* iv) {
  Ctr c{0, 0};
  for (int i = 0; i < 8; ++i) c.hi = (c.hi << 8) | iv[i];
  for (int i = 8; i < 16; ++i) c.lo = (c.lo << 8) | iv[i];
  return c;
}

void ctr_table(const Sched& s, Ctr c, const uint8_t* in, uint8_t* out, uint64_t n) {
  for (uint64_t off = 0; off < n; off += 16, c.next()) {
    const uint32_t blk[4] = {static_cast<uint32_t>(c.hi >> 32), static_cast<uint32_t>(c.hi),
                             static_cast<uint32_t>(c.lo >> 32), static_cast<uint32_t>(c.lo)};
    uint32_t ks[4];
    block_table(s, blk, ks);
    uint8_t kb[16];
    for (int i = 0; i < 16; ++i) kb[i] = static_cast<uint8_t>(ks[i >> 2] >> (24 - 8 * (i & 3)));
    const uint64_t m = n - off < 16 ? n - off : 16;
    for (uint64_t i = 0; i < m; ++i) out[off + i] = in[off + i] ^ kb[i];
  }
}

// ---- AES-NI cipher -----------------------------------------------------------
__attribute__((target("aes,sse4.1"))) inline __m128i ctr_block(const Ctr& c) {
  return _mm_set_epi64x(static_cast<long long>(__builtin_bswap64(c.lo)), static_cast<long long>(__builtin_bswap64(c.hi)));
}

template <int NR>
__attribute__((target("aes,sse4.1"))) void ctr_ni(const Sched& s, Ctr c, const uint8_t* in, uint8_t* out, uint64_t n) {
  __m128i rk[NR + 1];
  for (int r = 0; r <= NR; ++r) rk[r] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s.bytes + 16 * r));
  uint64_t off = 0;
  // eight blocks in flight (aesenc's latency), whole 128-byte pieces
  for (; off + 128 <= n; off += 128) {
    __m128i x[8];
    for (int b = 0; b < 8; ++b, c.next()) x[b] = _mm_xor_si128(ctr_block(c), rk[0]);
    for (int r = 1; r < NR; ++r)
      for (int b = 0; b < 8; ++b) x[b] = _mm_aesenc_si128(x[b], rk[r]);
    for (int b = 0; b < 8; ++b) {
      x[b] = _mm_aesenclast_si128(x[b], rk[NR]);
      const __m128i p = _mm_loadu_si128(reinterpret_cast<const __m128i*>(in + off + 16 * b));
      _mm_storeu_si128(reinterpret_cast<__m128i*>(out + off + 16 * b), _mm_xor_si128(p, x[b]));
    }
  }
  // the tail: up to eight blocks, the last one partial
  if (off < n) {
    const int nb = static_cast<int>((n - off + 15) / 16);
    __m128i x[8];
    for (int b = 0; b < nb; ++b, c.next()) x[b] = _mm_xor_si128(ctr_block(c), rk[0]);
    for (int r = 1; r < NR; ++r)
      for (int b = 0; b < nb; ++b) x[b] = _mm_aesenc_si128(x[b], rk[r]);
    for (int b = 0; b < nb; ++b) {
      alignas(16) uint8_t ks[16];
      _mm_store_si128(reinterpret_cast<__m128i*>(ks), _mm_aesenclast_si128(x[b], rk[NR]));
      const uint64_t o = off + 16u * b, m = n - o < 16 ? n - o : 16;
      for (uint64_t i = 0; i < m; ++i) out[o + i] = in[o + i] ^ ks[i];
    }
  }
}

bool have_aesni() {
  static const bool ok = __builtin_cpu_supports("aes") && __builtin_cpu_supports("sse4.1");
  return ok;
}

// DN_AES_HOST=table (tuning build): the table cipher even where AES-NI exists (tests of both)
bool use_aesni() {
  const char* e = tune_env("DN_AES_HOST");
  if (e && e[0] == 't') return false;
  return have_aesni();
}

void ctr(const Sched& s, const uint8_t* iv, const uint8_t* in, uint8_t* out, uint64_t n) {
  if (n == 0) return;
  const Ctr c = load_ctr(iv);
  if (!use_aesni()) return ctr_table(s, c, in, out, n);
  if (s.nr == 14) ctr_ni<14>(s, c, in, out, n);
  else if (s.nr == 12) ctr_ni<12>(s, c, in, out, n);
  else ctr_ni<10>(s, c, in, out, n);
}

// ---- base64 / hex ------------------------------------------------------------
constexpr char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
constexpr char kHex[] = "0123456789abcdef";

// base64 of src[0..n) (with '=' padding) into dst; hex: each character as two lowercase hex digits
void b64_text(const uint8_t* src, uint64_t n, uint8_t* dst, bool hex) {
  auto put = [&](char ch) {
    const uint8_t c = static_cast<uint8_t>(ch);
    if (hex) {
      *dst++ = static_cast<uint8_t>(kHex[c >> 4]);
      *dst++ = static_cast<uint8_t>(kHex[c & 15]);
    } else {
      *dst++ = c;
    }
  };
  uint64_t i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t v = (static_cast<uint32_t>(src[i]) << 16) | (static_cast<uint32_t>(src[i + 1]) << 8) | src[i + 2];
    put(kB64[v >> 18]), put(kB64[(v >> 12) & 63]), put(kB64[(v >> 6) & 63]), put(kB64[v & 63]);
  }
  if (n - i == 1) {
    const uint32_t v = static_cast<uint32_t>(src[i]) << 16;
    put(kB64[v >> 18]), put(kB64[(v >> 12) & 63]), put('='), put('=');
  } else if (n - i == 2) {
    const uint32_t v = (static_cast<uint32_t>(src[i]) << 16) | (static_cast<uint32_t>(src[i + 1]) << 8);
    put(kB64[v >> 18]), put(kB64[(v >> 12) & 63]), put(kB64[(v >> 6) & 63]), put('=');
  }
}

int b64_value(uint8_t c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

int hex_value(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// Canonical base64 (length a multiple of 4, alphabet only, '=' only as the
// last one or two characters) -> raw bytes; false otherwise.  Bits below a
// final partial group are ignored, as base64.b64decode ignores them.
bool b64_decode(const uint8_t* t, uint64_t n, std::vector<uint8_t>& raw) {
  if (n % 4) return false;
  raw.clear();
  raw.reserve(n / 4 * 3);
  for (uint64_t i = 0; i < n; i += 4) {
    int v[4];
    int pad = 0;
    for (int k = 0; k < 4; ++k) {
      if (t[i + k] == '=') {
        if (i + 4 != n || k < 2) return false;
        v[k] = 0;
        ++pad;
      } else {
        if (pad) return false;  // '=' then a letter
        v[k] = b64_value(t[i + k]);
        if (v[k] < 0) return false;
      }
    }
    const uint32_t w = (static_cast<uint32_t>(v[0]) << 18) | (static_cast<uint32_t>(v[1]) << 12) |
                       (static_cast<uint32_t>(v[2]) << 6) | static_cast<uint32_t>(v[3]);
    raw.push_back(static_cast<uint8_t>(w >> 16));
    if (pad < 2) raw.push_back(static_cast<uint8_t>(w >> 8));
    if (pad < 1) raw.push_back(static_cast<uint8_t>(w));
  }
  return true;
}

}  // namespace
}  // namespace dn

using namespace dn;

extern "C" int dn_aes_ctr_host(const uint8_t* key, int key_bytes, const uint8_t* iv, const void* in, void* out,
                               uint64_t n) {
  Sched s;
  if (int rc = schedule(key, key_bytes, s)) return rc;
  if (!iv) return set_error(DN_ERR_ARG, "dn_aes_ctr_host: null iv");
  if (n && (!in || !out)) return set_error(DN_ERR_ARG, "dn_aes_ctr_host: null buffer");
  ctr(s, iv, static_cast<const uint8_t*>(in), static_cast<uint8_t*>(out), n);
  return DN_OK;
}

extern "C" int dn_aes_encrypt_host(const uint8_t* key, int key_bytes, const uint8_t* nonce, const void* in,
                                   uint64_t n, void* out, int hex) {
  Sched s;
  if (int rc = schedule(key, key_bytes, s)) return rc;
  if (!nonce) return set_error(DN_ERR_ARG, "dn_aes_encrypt_host: null nonce");
  if ((n && !in) || !out) return set_error(DN_ERR_ARG, "dn_aes_encrypt_host: null buffer");
  // nonce || ct in one buffer (a share is ~70 bytes: on the stack)
  uint8_t small[512];
  std::vector<uint8_t> big;
  uint8_t* raw = small;
  if (16 + n > sizeof(small)) {
    big.resize(16 + n);
    raw = big.data();
  }
  std::memcpy(raw, nonce, 16);
  ctr(s, nonce, static_cast<const uint8_t*>(in), raw + 16, n);
  b64_text(raw, 16 + n, static_cast<uint8_t*>(out), hex != 0);
  return DN_OK;
}

extern "C" int dn_aes_decrypt_host(const uint8_t* key, int key_bytes, const void* text, uint64_t n_text, int hex,
                                   void* out, uint64_t capacity, uint64_t* out_len) {
  Sched s;
  if (int rc = schedule(key, key_bytes, s)) return rc;
  const uint64_t cap = dn_aes_decrypt_capacity(n_text, hex);
  if (cap == 0)
    return set_error(DN_ERR_RETRY, "dn_aes_decrypt_host: %llu characters are not canonical %s",
                     static_cast<unsigned long long>(n_text), hex ? "hex of base64" : "base64");
  if (capacity < cap)
    return set_error(DN_ERR_ARG, "dn_aes_decrypt_host: capacity %llu < %llu", static_cast<unsigned long long>(capacity),
                     static_cast<unsigned long long>(cap));
  if (!text || !out || !out_len) return set_error(DN_ERR_ARG, "dn_aes_decrypt_host: null pointer");
  const uint8_t* t = static_cast<const uint8_t*>(text);
  std::vector<uint8_t> b64;
  uint64_t nb = n_text;
  if (hex) {
    nb = n_text / 2;
    b64.resize(nb);
    for (uint64_t i = 0; i < nb; ++i) {
      const int h = hex_value(t[2 * i]), l = hex_value(t[2 * i + 1]);
      if (h < 0 || l < 0) return set_error(DN_ERR_RETRY, "dn_aes_decrypt_host: not hex");
      b64[i] = static_cast<uint8_t>((h << 4) | l);
    }
    t = b64.data();
  }
  std::vector<uint8_t> raw;
  if (!b64_decode(t, nb, raw) || raw.size() < 16)
    return set_error(DN_ERR_RETRY, "dn_aes_decrypt_host: not canonical base64");
  const uint64_t m = raw.size() - 16;
  ctr(s, raw.data(), raw.data() + 16, static_cast<uint8_t*>(out), m);
  *out_len = m;
  return DN_OK;
}

extern "C" int dn_aes_host_impl(void) { return use_aesni() ? 1 : 0; }

extern "C" int dn_aes_expand_key_host(const uint8_t* key, int key_bytes, uint32_t* rk, int32_t* rounds) {
  if (!rk || !rounds) return set_error(DN_ERR_ARG, "dn_aes_expand_key_host: null pointer");
  Sched s;
  if (int rc = schedule(key, key_bytes, s)) return rc;
  for (int i = 0; i < 60; ++i) rk[i] = i < 4 * (s.nr + 1) ? s.w[i] : 0u;
  *rounds = s.nr;
  return DN_OK;
}
