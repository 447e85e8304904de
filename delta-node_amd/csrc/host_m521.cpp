// host_m521.cpp — host side of the native library: errors, layout sizes, the
// CPython-compatible MT19937 coefficient stream, and Lagrange weights.
//
// * dn_mt19937_draw_coeffs restates what `SecretShare.make_shares` asks of
//   `self.random` (delta_node/crypto/shamir/shamir.py:59-61):
//   randint(1, p-1) -> 1 + _randbelow(p-1) -> getrandbits(521) until < p-1.
//   getrandbits(521) takes 17 MT19937 words, little-endian, the last >> 23
//   (CPython Modules/_randommodule.c, random_getrandbits; MT19937 is
//   Matsumoto & Nishimura's published generator with CPython's tempering).
// * dn_m521_lagrange computes the weights of `resolve_shares`
//   (shamir.py:77-89; op.py:4-29 extend_gcd/inverse_mod/div_mod) once per
//   call, on the host, in a form that lets the kernel multiply by small
//   integers: lambda_i = a_i / (d * 2^e).
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "dn_internal.hpp"

namespace dn {

namespace {
thread_local std::string g_err = "";
}

int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// ---------------------------------------------------------------- MT19937
namespace {
constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

// CPython's MT19937 (genrand_uint32), consumed a block at a time: the twist
// of the 624-word state and the tempering of the whole block are two
// branch-free loops the compiler vectorises (AVX2 / AVX-512 clones picked at
// load time), then words are handed out from the tempered block.  `s` / `idx`
// stay exactly CPython's state array and index.
__attribute__((target_clones("avx512f", "avx2", "default")))
void mt_twist_temper(uint32_t* __restrict s, uint32_t* __restrict out) {
  for (int k = 0; k < kN - kM; ++k) {
    const uint32_t y = (s[k] & kUpper) | (s[k + 1] & kLower);
    s[k] = s[k + kM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  }
  for (int k = kN - kM; k < kN - 1; ++k) {
    const uint32_t y = (s[k] & kUpper) | (s[k + 1] & kLower);
    s[k] = s[k + (kM - kN)] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  }
  const uint32_t y = (s[kN - 1] & kUpper) | (s[0] & kLower);
  s[kN - 1] = s[kM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  for (int k = 0; k < kN; ++k) {
    uint32_t v = s[k];
    v ^= (v >> 11);
    v ^= (v << 7) & 0x9d2c5680u;
    v ^= (v << 15) & 0xefc60000u;
    v ^= (v >> 18);
    out[k] = v;
  }
}

struct Mt {
  uint32_t* s;
  int idx;
  uint32_t out[kN];
  Mt(uint32_t* state, int index) : s(state), idx(index) {
    // words idx..623 of the current block were not handed out yet: temper them
    for (int k = idx; k < kN; ++k) {
      uint32_t v = s[k];
      v ^= (v >> 11);
      v ^= (v << 7) & 0x9d2c5680u;
      v ^= (v << 15) & 0xefc60000u;
      v ^= (v >> 18);
      out[k] = v;
    }
  }
  inline uint32_t next() {
    if (idx >= kN) {
      mt_twist_temper(s, out);
      idx = 0;
    }
    return out[idx++];
  }
  // 17 consecutive words (one getrandbits(521) draw, LE 32-bit words)
  inline void next17(uint32_t v[17]) {
    if (idx + 17 <= kN) {
      std::memcpy(v, out + idx, 17 * sizeof(uint32_t));
      idx += 17;
    } else {
      for (int i = 0; i < 17; ++i) v[i] = next();
    }
  }
};
}  // namespace

namespace {
// w >= p - 1 = 2^521 - 2 ?
inline bool ge_p_minus_1(const uint32_t w[17]) {
  if (w[16] != 0x1FFu || w[0] < 0xFFFFFFFEu) return false;
  for (int i = 1; i < 16; ++i)
    if (w[i] != 0xFFFFFFFFu) return false;
  return true;
}
}  // namespace

// ------------------------------------------------- 521-bit host arithmetic
namespace {
struct Fe {
  uint32_t l[17];
};

Fe fe_zero() {
  Fe r;
  std::memset(r.l, 0, sizeof(r.l));
  return r;
}

Fe fe_u128(unsigned __int128 v) {  // v < 2^128 < p
  Fe r = fe_zero();
  for (int i = 0; i < 4; ++i) r.l[i] = static_cast<uint32_t>(v >> (32 * i));
  return r;
}

// canonicalise v (< 2^544) mod p
void fe_reduce(uint32_t v[17]) {
  uint64_t hi = v[16] >> 9;
  v[16] &= 0x1FFu;
  uint64_t c = hi;
  for (int i = 0; i < 17; ++i) {
    c += v[i];
    v[i] = static_cast<uint32_t>(c);
    c >>= 32;
  }
  const uint32_t top = v[16] >> 9;
  bool is_p = v[16] == 0x1FFu;
  for (int i = 0; i < 16 && is_p; ++i) is_p = v[i] == 0xFFFFFFFFu;
  v[16] &= 0x1FFu;
  v[0] += top;
  if (is_p) std::memset(v, 0, 17 * sizeof(uint32_t));
}

Fe fe_mul(const Fe& a, const Fe& b) {
  uint32_t S[34] = {0};
  for (int j = 0; j < 17; ++j) {
    uint64_t carry = 0;
    for (int l = 0; l < 17; ++l) {
      const uint64_t t = static_cast<uint64_t>(a.l[j]) * b.l[l] + S[j + l] + carry;
      S[j + l] = static_cast<uint32_t>(t);
      carry = t >> 32;
    }
    S[j + 17] = static_cast<uint32_t>(carry);
  }
  // fold at bit 521: r = (S mod 2^521) + (S >> 521)  (< 2^522)
  Fe r;
  uint64_t c = 0;
  for (int m = 0; m < 17; ++m) {
    uint32_t h = (S[16 + m] >> 9) | ((16 + m + 1 < 34) ? (S[16 + m + 1] << 23) : 0u);
    const uint32_t lo = (m < 16) ? S[m] : (S[16] & 0x1FFu);
    c += static_cast<uint64_t>(lo) + h;
    r.l[m] = static_cast<uint32_t>(c);
    c >>= 32;
  }
  fe_reduce(r.l);
  return r;
}

Fe fe_sub(const Fe& a, const Fe& b) {  // a - b mod p, canonical in/out
  // a + (p - b); p - b = ~b within 521 bits
  Fe r;
  uint64_t c = 0;
  for (int i = 0; i < 17; ++i) {
    const uint32_t nb = (i < 16) ? ~b.l[i] : ((~b.l[16]) & 0x1FFu);
    c += static_cast<uint64_t>(a.l[i]) + nb;
    r.l[i] = static_cast<uint32_t>(c);
    c >>= 32;
  }
  fe_reduce(r.l);
  return r;
}

Fe fe_pow_pm2(const Fe& a) {  // a^(p-2) = a^{-1} for a != 0
  // p - 2 = 2^521 - 3: bit 1 clear, bits 0 and 2..520 set.
  Fe result = fe_u128(1), base = a;
  for (int bit = 0; bit < 521; ++bit) {
    if (bit != 1) result = fe_mul(result, base);
    base = fe_mul(base, base);
  }
  return result;
}

bool fe_is_zero(const Fe& a) {
  for (int i = 0; i < 17; ++i)
    if (a.l[i]) return false;
  return true;
}

using u128 = unsigned __int128;
using i128 = __int128;

u128 gcd128(u128 a, u128 b) {
  while (b) {
    const u128 t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// a^{-1} mod m for gcd(a, m) == 1, small m (extended Euclid).
uint64_t inv_small(uint64_t a, uint64_t m) {
  int64_t r0 = static_cast<int64_t>(m), r1 = static_cast<int64_t>(a % m), s0 = 0, s1 = 1;
  while (r1) {
    const int64_t q = r0 / r1, r2 = r0 - q * r1, s2 = s0 - q * s1;
    r0 = r1;
    r1 = r2;
    s0 = s1;
    s1 = s2;
  }
  return static_cast<uint64_t>((s0 % static_cast<int64_t>(m) + static_cast<int64_t>(m)) % static_cast<int64_t>(m));
}

// DN_EXACT_DIV=0 forces the full-width inverse (A/B and test hook).
bool exact_div_disabled() {
  const char* s = tune_env("DN_EXACT_DIV");
  return s && s[0] == '0';
}

bool mul_ovf(u128 a, u128 b, u128* out, u128 limit) {
  if (a == 0 || b == 0) {
    *out = 0;
    return false;
  }
  if (a > limit / b) return true;
  *out = a * b;
  return false;
}
}  // namespace

}  // namespace dn

using namespace dn;

extern "C" uint64_t dn_m521_vec_bytes(uint64_t n_elem) {
  const uint64_t tiles = (n_elem + DN_M521_TILE - 1) / DN_M521_TILE;
  return tiles * static_cast<uint64_t>(DN_M521_TILE_BYTES);
}

extern "C" const char* dn_last_error(void) { return g_err.c_str(); }

extern "C" const char* dn_version(void) { return "dn_shamir 0.1 (gfx950, M521)"; }

namespace dn {
namespace {
// Coefficient c (17 words w, w[16] already >> 23, < p - 1) + 1 into element e,
// row j of the tiled block.
inline void put_coeff(uint8_t* base, uint64_t vb, uint64_t e, int j, const uint32_t* w) {
  uint32_t v[17];
  std::memcpy(v, w, sizeof(v));
  for (int i = 0; i < 17; ++i)  // + 1 (randint's lower bound); v < p - 1: no carry out of the top limb
    if (++v[i] != 0u) break;
  const uint64_t tile = e / DN_M521_TILE, lane = e % DN_M521_TILE;
  uint8_t* t = base + static_cast<uint64_t>(j) * vb + tile * DN_M521_TILE_BYTES;
  uint32_t* lo = reinterpret_cast<uint32_t*>(t);
  uint16_t* hi = reinterpret_cast<uint16_t*>(t + 64 * DN_M521_TILE);
  for (int i = 0; i < 16; ++i) lo[i * DN_M521_TILE + lane] = v[i];
  hi[lane] = static_cast<uint16_t>(v[16]);
}

// One draw of randint(1, p - 1)'s getrandbits(521) loop into w[17] (w[16] >> 23).
inline void draw_521(Mt& mt, uint32_t* w) {
  do {
    mt.next17(w);
    w[16] >>= 23;
  } while (ge_p_minus_1(w));
}

}  // namespace
}  // namespace dn

extern "C" int dn_mt19937_draw_coeffs(uint32_t* mt_state, int32_t* mt_index, uint64_t n_elem, int tm1,
                                      void* coeffs) {
  if (!mt_state || !mt_index || (tm1 > 0 && n_elem > 0 && !coeffs))
    return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs: null pointer");
  if (tm1 < 0 || tm1 >= DN_MAX_THRESHOLD)
    return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs: t-1=%d", tm1);
  if (*mt_index < 0 || *mt_index > kN) return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs: bad MT index");
  // Sequential by definition (one MT19937 stream, element-major, coefficient
  // j inner, as n make_shares calls draw).  Scattering the words over worker
  // threads measured slower on the GPU box than this loop (0.57 vs 0.44 s at
  // 2^24, t = 3): the stream itself is the bound.
  Mt mt(mt_state, *mt_index);
  const uint64_t vb = dn_m521_vec_bytes(n_elem);
  uint8_t* base = static_cast<uint8_t*>(coeffs);
  for (uint64_t e = 0; e < n_elem; ++e)
    for (int j = 0; j < tm1; ++j) {
      uint32_t w[17];
      draw_521(mt, w);
      put_coeff(base, vb, e, j, w);
    }
  *mt_index = mt.idx;
  return DN_OK;
}

extern "C" int dn_m521_lagrange(const uint64_t* xs, int k, int threshold, dn_m521_lagrange_t* out) {
  if (!out || (k > 0 && !xs)) return set_error(DN_ERR_ARG, "dn_m521_lagrange: null pointer");
  if (k < 1) return set_error(DN_ERR_ARG, "not enough values to unpack (expected 2, got 0)");
  if (k < threshold) return set_error(DN_ERR_TOO_FEW, "need at least %d shares", threshold);
  for (int i = 0; i < k; ++i)
    for (int j = i + 1; j < k; ++j)
      if (xs[i] == xs[j]) return set_error(DN_ERR_DISTINCT, "shares must be distinct");
  if (k == 1) return set_error(DN_ERR_EMPTY, "reduce() of empty iterable with no initial value");
  if (k > DN_MAX_RESOLVE)
    return set_error(DN_ERR_UNSUPPORTED, "dn_m521_lagrange: %d shares > %d", k, DN_MAX_RESOLVE);
  std::memset(out, 0, sizeof(*out));
  out->k = k;

  // Exact rationals lambda_i = prod_{j!=i} x_j / prod_{j!=i} (x_j - x_i), when they fit 128 bits.
  const u128 kLim = (static_cast<u128>(1) << 126);
  bool exact = true;
  u128 num[DN_MAX_RESOLVE], den[DN_MAX_RESOLVE];
  bool negv[DN_MAX_RESOLVE];
  for (int i = 0; i < k && exact; ++i) {
    u128 n = 1, d = 1;
    bool neg = false;
    for (int j = 0; j < k && exact; ++j) {
      if (j == i) continue;
      u128 diff;
      if (xs[j] > xs[i]) {
        diff = static_cast<u128>(xs[j] - xs[i]);
      } else {
        diff = static_cast<u128>(xs[i] - xs[j]);
        neg = !neg;
      }
      if (mul_ovf(n, xs[j], &n, kLim) || mul_ovf(d, diff, &d, kLim)) exact = false;
    }
    if (!exact) break;
    if (n == 0) {
      d = 1;
      neg = false;
    } else {
      const u128 g = gcd128(n, d);
      n /= g;
      d /= g;
    }
    num[i] = n;
    den[i] = d;
    negv[i] = neg;
  }
  u128 L = 1;
  for (int i = 0; i < k && exact; ++i) {
    const u128 g = gcd128(L, den[i]);
    if (mul_ovf(L / g, den[i], &L, kLim)) exact = false;
  }
  u128 a[DN_MAX_RESOLVE];
  u128 amax = 0;
  for (int i = 0; i < k && exact; ++i) {
    if (mul_ovf(num[i], L / den[i], &a[i], kLim)) exact = false;
    if (a[i] > amax) amax = a[i];
  }
  if (exact && (amax >> 64) == 0) {
    out->a_limbs = (amax >> 32) ? 2 : 1;
    for (int i = 0; i < k; ++i) {
      out->a[i][0] = static_cast<uint32_t>(a[i]);
      out->a[i][1] = static_cast<uint32_t>(a[i] >> 32);
      if (negv[i] && a[i] != 0) out->neg |= (1u << i);
    }
    int e = 0;
    while (((L >> e) & 1) == 0) ++e;
    u128 d = L;
    if (e < 32) {
      d = L >> e;
      out->shift = e;
    }
    if (d != 1) {
      out->d = static_cast<uint32_t>(d);
      if (d < 65536u && (d & 1) && !exact_div_disabled()) {
        // exact division by the small odd d (see dn_shamir.h)
        const uint32_t d32 = static_cast<uint32_t>(d);
        uint32_t inv32 = d32;  // Newton: x <- x (2 - d x), 5 steps from 3 correct bits
        for (int it = 0; it < 5; ++it) inv32 *= 2u - d32 * inv32;
        uint64_t pw = 1;  // 2^521 mod d, then p mod d = 2^521 - 1
        for (int b = 0; b < 521; ++b) pw = (pw * 2) % d32;
        const uint64_t pmod = (pw + d32 - 1) % d32;
        out->has_inv = 2;
        out->d_inv32 = inv32;
        out->p_inv_d = static_cast<uint32_t>(inv_small(pmod, d32));
        out->d_recip = UINT64_MAX / d32;
        uint64_t wv = 1;
        for (int i = 0; i < 17; ++i) {
          out->w[i] = static_cast<uint32_t>(wv);
          wv = (wv << 32) % d32;
        }
      } else {
        out->has_inv = 1;
        const Fe inv = fe_pow_pm2(fe_u128(d));
        std::memcpy(out->inv, inv.l, sizeof(out->inv));
      }
    }
    return DN_OK;
  }

  // Generic: a_i = lambda_i mod p (full width), no final scaling.
  out->a_limbs = 17;
  for (int i = 0; i < k; ++i) {
    Fe n = fe_u128(1), d = fe_u128(1);
    const Fe xi = fe_u128(xs[i]);
    for (int j = 0; j < k; ++j) {
      if (j == i) continue;
      const Fe xj = fe_u128(xs[j]);
      n = fe_mul(n, xj);
      d = fe_mul(d, fe_sub(xj, xi));
    }
    if (fe_is_zero(d)) return set_error(DN_ERR_ARG, "dn_m521_lagrange: singular abscissas");
    const Fe lam = fe_mul(n, fe_pow_pm2(d));
    std::memcpy(out->a[i], lam.l, sizeof(out->a[i]));
  }
  return DN_OK;
}
