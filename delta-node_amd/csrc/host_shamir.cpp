// host_shamir.cpp — the reference's byte API on the host, native (plain C++).
//
// The reference's callers split and resolve ONE 32-byte secret per call
// (runner/horizontal/agg.py:142-153, coord/horizontal/agg.py:296,330,362): a
// GPU launch plus two copies per call (~100-190 us) is a latency regression
// against the reference's ~5-15 us of Python big-int work, so single secrets
// are computed here, with the same arithmetic:
//   make_shares     shamir.py:55-66 with _eval_at :19-25 (Horner from the top,
//                   % p after every step) and _share_to_bytes :28-33;
//   resolve_shares  shamir.py:68-90 with _bytes_to_share :36-45 and op.py:4-29
//                   (nums / dens / den, div_mod by extended Euclid; the same
//                   ZeroDivisionError / assertion failures).
// Any prime (the reference's `prime` keyword, shamir.py:49-51); p = 2^521 - 1
// takes a fixed 9 x 64-bit-limb path (Mersenne folding, small-divisor
// inverses), everything else a small arbitrary-precision integer type.  The
// vector API (the hot path) stays on the GPU.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "dn_internal.hpp"

namespace dn {
namespace {

using u128 = unsigned __int128;
using i128 = __int128;

// ================================================================ M521 path
constexpr int kW = 9;  // 9 x 64 = 576 bits
constexpr uint64_t kTop = (1ull << 9) - 1;  // bits 512..520 in word 8

struct F {
  uint64_t w[kW];
};

// r = v mod p for v < 2^640 given as 10 words; canonical result.
void fold10(const uint64_t v[10], F& r) {
  // lo = v mod 2^521, hi = v >> 521 (< 2^119: words 0..1)
  uint64_t hi0 = (v[8] >> 9) | (v[9] << 55), hi1 = v[9] >> 9;
  u128 c = 0;
  for (int i = 0; i < kW; ++i) {
    uint64_t lo = i < 8 ? v[i] : (v[8] & kTop);
    c += static_cast<u128>(lo) + (i == 0 ? hi0 : i == 1 ? hi1 : 0);
    r.w[i] = static_cast<uint64_t>(c);
    c >>= 64;
  }
  // r < 2^521 + 2^119: fold the carry bit 521 once more
  const uint64_t t = r.w[8] >> 9;
  r.w[8] &= kTop;
  c = t;
  for (int i = 0; i < kW && c; ++i) {
    c += r.w[i];
    r.w[i] = static_cast<uint64_t>(c);
    c >>= 64;
  }
  bool all = r.w[8] == kTop;
  for (int i = 0; i < 8 && all; ++i) all = r.w[i] == ~0ull;
  if (all) std::memset(r.w, 0, sizeof(r.w));  // == p
}

// r = (v * x + c) mod p; v, c canonical, x < 2^64.
void mul_small_add(const F& v, uint64_t x, const F& c, F& r) {
  uint64_t t[10];
  u128 carry = 0;
  for (int i = 0; i < kW; ++i) {
    carry += static_cast<u128>(v.w[i]) * x + c.w[i];
    t[i] = static_cast<uint64_t>(carry);
    carry >>= 64;
  }
  t[9] = static_cast<uint64_t>(carry);
  fold10(t, r);
}

// r = a * b mod p (canonical inputs).
void mul(const F& a, const F& b, F& r) {
  uint64_t t[2 * kW] = {};
  for (int i = 0; i < kW; ++i) {
    u128 carry = 0;
    for (int j = 0; j < kW; ++j) {
      carry += static_cast<u128>(a.w[i]) * b.w[j] + t[i + j];
      t[i + j] = static_cast<uint64_t>(carry);
      carry >>= 64;
    }
    t[i + kW] = static_cast<uint64_t>(carry);
  }
  // t < 2^1042: t = lo + hi * 2^521 == lo + hi (mod p), hi < 2^521
  uint64_t s[10] = {};
  u128 c = 0;
  for (int i = 0; i < kW; ++i) {
    const int bit = 521 + 64 * i, q = bit >> 6, sh = bit & 63;
    uint64_t h = t[q] >> sh;
    if (q + 1 < 2 * kW) h |= sh ? (t[q + 1] << (64 - sh)) : 0;
    if (i == 8) h &= kTop;
    const uint64_t lo = i < 8 ? t[i] : (t[8] & kTop);
    c += static_cast<u128>(lo) + h;
    s[i] = static_cast<uint64_t>(c);
    c >>= 64;
  }
  s[9] = static_cast<uint64_t>(c);
  fold10(s, r);
}

void add(const F& a, const F& b, F& r) { mul_small_add(a, 1, b, r); }

// p - a (a canonical) = complement of the 521 bits; p - 0 = p -> 0.
void neg(const F& a, F& r) {
  bool zero = true;
  for (int i = 0; i < kW; ++i) zero = zero && a.w[i] == 0;
  if (zero) {
    r = a;
    return;
  }
  for (int i = 0; i < 8; ++i) r.w[i] = ~a.w[i];
  r.w[8] = (~a.w[8]) & kTop;
}

// big-endian bytes (any length) -> value mod p, 4 bytes at a time: v = v 2^32 + chunk
void from_be(const uint8_t* b, uint64_t n, F& r) {
  std::memset(r.w, 0, sizeof(r.w));
  uint64_t i = 0;
  const uint64_t head = n % 4;
  F c{};
  if (head) {
    uint64_t x = 0;
    for (; i < head; ++i) x = (x << 8) | b[i];
    c.w[0] = x;
    r = c;
  }
  for (; i < n; i += 4) {
    c.w[0] = (static_cast<uint64_t>(b[i]) << 24) | (static_cast<uint64_t>(b[i + 1]) << 16) |
             (static_cast<uint64_t>(b[i + 2]) << 8) | b[i + 3];
    F t;
    mul_small_add(r, 1ull << 32, c, t);
    r = t;
  }
}

// minimal big-endian bytes of a canonical value (0 -> none); returns the length
uint32_t to_be_min(const F& a, uint8_t* out) {
  uint8_t buf[kW * 8];
  for (int i = 0; i < kW; ++i)
    for (int j = 0; j < 8; ++j) buf[kW * 8 - 1 - (8 * i + j)] = static_cast<uint8_t>(a.w[i] >> (8 * j));
  int s = 0;
  while (s < kW * 8 && buf[s] == 0) ++s;
  std::memcpy(out, buf + s, kW * 8 - s);
  return static_cast<uint32_t>(kW * 8 - s);
}

// d^{-1} mod p for 0 < d < 2^63: u = (m p + 1) / d with m = -p^{-1} mod d.
void inv_small(uint64_t d, F& r) {
  // p mod d = (2^521 mod d) - 1
  u128 pw = 1, base = 2 % d;
  for (int e = 521; e; e >>= 1) {
    if (e & 1) pw = pw * base % d;
    base = base * base % d;
  }
  const uint64_t pm = static_cast<uint64_t>((pw + d - 1) % d);
  // inverse of pm mod d (gcd(p, d) == 1: p is prime and d < p)
  i128 r0 = pm, r1 = d, s0 = 1, s1 = 0;
  while (r1) {
    const i128 q = r0 / r1, r2 = r0 - q * r1, s2 = s0 - q * s1;
    r0 = r1, r1 = r2, s0 = s1, s1 = s2;
  }
  const uint64_t pinv = static_cast<uint64_t>(((s0 % static_cast<i128>(d)) + d) % d);
  const uint64_t m = static_cast<uint64_t>((d - pinv) % d);
  // m p + 1 = m 2^521 - m + 1, then exact division by d, top word first
  uint64_t v[10] = {};
  v[8] = (m & ((1ull << 55) - 1)) << 9;  // m << 521: bits 521.. in words 8, 9
  v[9] = m >> 55;
  // - (m - 1): subtract m - 1 (m >= 1 unless d == 1)
  u128 borrow = m ? m - 1 : 0;
  for (int i = 0; i < 10 && borrow; ++i) {
    const uint64_t x = v[i];
    v[i] = x - static_cast<uint64_t>(borrow);
    borrow = (static_cast<u128>(x) < borrow) ? 1 : 0;
  }
  if (m == 0) v[0] += 1;  // d == 1: u = 1
  u128 rem = 0;
  for (int i = 9; i >= 0; --i) {
    const u128 cur = (rem << 64) | v[i];
    v[i] = static_cast<uint64_t>(cur / d);
    rem = cur % d;
  }
  fold10(v, r);
}

// ================================================================ generic path
// Magnitude in base 2^32, little-endian, no leading zero limbs; sign separate.
struct BN {
  std::vector<uint32_t> m;
  bool neg = false;
  bool zero() const { return m.empty(); }
  void trim() {
    while (!m.empty() && m.back() == 0) m.pop_back();
    if (m.empty()) neg = false;
  }
};

BN bn_from_be(const uint8_t* b, uint64_t n) {
  BN r;
  r.m.assign((n + 3) / 4, 0u);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t k = n - 1 - i;  // byte significance
    r.m[k / 4] |= static_cast<uint32_t>(b[i]) << (8 * (k % 4));
  }
  r.trim();
  return r;
}

BN bn_from_u64(uint64_t v, bool neg = false) {
  BN r;
  if (v) r.m = {static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32)};
  r.neg = neg;
  r.trim();
  return r;
}

int cmp_mag(const BN& a, const BN& b) {
  if (a.m.size() != b.m.size()) return a.m.size() < b.m.size() ? -1 : 1;
  for (size_t i = a.m.size(); i-- > 0;)
    if (a.m[i] != b.m[i]) return a.m[i] < b.m[i] ? -1 : 1;
  return 0;
}

BN add_mag(const BN& a, const BN& b) {
  BN r;
  const size_t n = std::max(a.m.size(), b.m.size());
  r.m.resize(n + 1);
  uint64_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c += static_cast<uint64_t>(i < a.m.size() ? a.m[i] : 0) + (i < b.m.size() ? b.m[i] : 0);
    r.m[i] = static_cast<uint32_t>(c);
    c >>= 32;
  }
  r.m[n] = static_cast<uint32_t>(c);
  r.trim();
  return r;
}

BN sub_mag(const BN& a, const BN& b) {  // |a| >= |b|
  BN r;
  r.m.resize(a.m.size());
  int64_t br = 0;
  for (size_t i = 0; i < a.m.size(); ++i) {
    int64_t d = static_cast<int64_t>(a.m[i]) - (i < b.m.size() ? b.m[i] : 0) - br;
    br = d < 0;
    r.m[i] = static_cast<uint32_t>(d + (br << 32));
  }
  r.trim();
  return r;
}

BN bn_add(const BN& a, const BN& b) {
  if (a.neg == b.neg) {
    BN r = add_mag(a, b);
    r.neg = a.neg && !r.zero();
    return r;
  }
  const int c = cmp_mag(a, b);
  if (c == 0) return BN{};
  BN r = c > 0 ? sub_mag(a, b) : sub_mag(b, a);
  r.neg = (c > 0 ? a.neg : b.neg) && !r.zero();
  return r;
}

BN bn_neg(BN a) {
  if (!a.zero()) a.neg = !a.neg;
  return a;
}

BN bn_mul(const BN& a, const BN& b) {
  BN r;
  if (a.zero() || b.zero()) return r;
  r.m.assign(a.m.size() + b.m.size(), 0u);
  for (size_t i = 0; i < a.m.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < b.m.size(); ++j) {
      c += static_cast<uint64_t>(a.m[i]) * b.m[j] + r.m[i + j];
      r.m[i + j] = static_cast<uint32_t>(c);
      c >>= 32;
    }
    r.m[i + b.m.size()] = static_cast<uint32_t>(c);
  }
  r.neg = a.neg != b.neg;
  r.trim();
  return r;
}

// |a| = q |b| + r (Knuth, TAOCP 4.3.1 algorithm D), b != 0; magnitudes only.
void divmod_mag(const BN& a, const BN& b, BN& q, BN& r) {
  q = BN{};
  r = BN{};
  if (cmp_mag(a, b) < 0) {
    r.m = a.m;
    return;
  }
  const size_t n = b.m.size(), mlen = a.m.size() - n;
  if (n == 1) {
    q.m.assign(a.m.size(), 0u);
    uint64_t rem = 0;
    for (size_t i = a.m.size(); i-- > 0;) {
      const uint64_t cur = (rem << 32) | a.m[i];
      q.m[i] = static_cast<uint32_t>(cur / b.m[0]);
      rem = cur % b.m[0];
    }
    q.trim();
    r = bn_from_u64(rem);
    return;
  }
  const int s = __builtin_clz(b.m.back());
  std::vector<uint32_t> v(n), u(a.m.size() + 1);
  for (size_t i = n; i-- > 0;) v[i] = (b.m[i] << s) | (s && i ? b.m[i - 1] >> (32 - s) : 0);
  u[a.m.size()] = s ? a.m.back() >> (32 - s) : 0;
  for (size_t i = a.m.size(); i-- > 0;) u[i] = (a.m[i] << s) | (s && i ? a.m[i - 1] >> (32 - s) : 0);
  q.m.assign(mlen + 1, 0u);
  for (size_t j = mlen + 1; j-- > 0;) {
    const uint64_t num = (static_cast<uint64_t>(u[j + n]) << 32) | u[j + n - 1];
    uint64_t qh = num / v[n - 1], rh = num % v[n - 1];
    while (qh >= (1ull << 32) || qh * v[n - 2] > ((rh << 32) | u[j + n - 2])) {
      --qh;
      rh += v[n - 1];
      if (rh >= (1ull << 32)) break;
    }
    int64_t borrow = 0;
    uint64_t carry = 0;
    for (size_t i = 0; i < n; ++i) {
      const uint64_t p = qh * v[i] + carry;
      carry = p >> 32;
      const int64_t t = static_cast<int64_t>(u[i + j]) - borrow - static_cast<int64_t>(p & 0xFFFFFFFFu);
      u[i + j] = static_cast<uint32_t>(t);
      borrow = t < 0 ? 1 : 0;
    }
    const int64_t t = static_cast<int64_t>(u[j + n]) - borrow - static_cast<int64_t>(carry);
    u[j + n] = static_cast<uint32_t>(t);
    if (t < 0) {  // add back
      --qh;
      uint64_t c = 0;
      for (size_t i = 0; i < n; ++i) {
        c += static_cast<uint64_t>(u[i + j]) + v[i];
        u[i + j] = static_cast<uint32_t>(c);
        c >>= 32;
      }
      u[j + n] += static_cast<uint32_t>(c);
    }
    q.m[j] = static_cast<uint32_t>(qh);
  }
  q.trim();
  r.m.assign(n, 0u);
  for (size_t i = 0; i < n; ++i) r.m[i] = (u[i] >> s) | (s ? u[i + 1] << (32 - s) : 0);
  r.trim();
}

// Python's a % p (p > 0): the result in [0, p)
BN bn_mod(const BN& a, const BN& p) {
  BN q, r;
  divmod_mag(a, p, q, r);
  if (a.neg && !r.zero()) r = sub_mag(p, r);
  return r;
}

// Python's a // b (floor) for b != 0
BN bn_floordiv(const BN& a, const BN& b) {
  BN q, r;
  divmod_mag(a, b, q, r);
  q.neg = (a.neg != b.neg) && !q.zero();
  if (a.neg != b.neg && !r.zero()) q = bn_add(q, bn_from_u64(1, true));
  return q;
}

// op.inverse_mod(k, p) (op.py:16-25): DN_ERR_ZERODIV for k == 0,
// DN_ERR_ASSERT when gcd(k, p) != 1.  extend_gcd(k, p) with Python floor
// division; its first step turns k into k % p.
int bn_inverse(const BN& k, const BN& p, BN& out) {
  if (k.zero()) return set_error(DN_ERR_ZERODIV, "ZeroDivisionError");
  BN r0 = k, r1 = p, x0 = bn_from_u64(1), x1{};
  while (!r1.zero()) {
    const BN q = bn_floordiv(r0, r1);
    BN r2 = bn_add(r0, bn_neg(bn_mul(q, r1)));
    BN x2 = bn_add(x0, bn_neg(bn_mul(q, x1)));
    r0 = std::move(r1), r1 = std::move(r2);
    x0 = std::move(x1), x1 = std::move(x2);
  }
  if (!(r0.m.size() == 1 && r0.m[0] == 1 && !r0.neg)) return set_error(DN_ERR_ASSERT, "AssertionError");
  out = bn_mod(x0, p);
  return DN_OK;
}

uint32_t bn_to_be_min(const BN& a, uint8_t* out) {
  uint32_t n = 0;
  for (size_t i = a.m.size(); i-- > 0;)
    for (int j = 3; j >= 0; --j) {
      const uint8_t b = static_cast<uint8_t>(a.m[i] >> (8 * j));
      if (n || b) out[n++] = b;
    }
  return n;
}

bool is_m521(const uint8_t* p, uint32_t n) {
  if (!p || !n) return true;
  uint32_t s = 0;
  while (s < n && p[s] == 0) ++s;
  if (n - s != 66 || p[s] != 0x01) return false;
  for (uint32_t i = s + 1; i < n; ++i)
    if (p[i] != 0xFF) return false;
  return true;
}

// share record [len(x)][x minimal BE][y minimal BE] (shamir.py:28-33)
uint64_t put_record(uint64_t x, const uint8_t* yb, uint32_t ylen, uint8_t* out) {
  uint8_t xb[8];
  uint32_t xl = 0;
  for (int j = 7; j >= 0; --j) {
    const uint8_t b = static_cast<uint8_t>(x >> (8 * j));
    if (xl || b) xb[xl++] = b;
  }
  out[0] = static_cast<uint8_t>(xl);
  std::memcpy(out + 1, xb, xl);
  std::memcpy(out + 1 + xl, yb, ylen);
  return 1 + xl + ylen;
}

struct Parsed {
  const uint8_t* x;
  uint32_t xl;
  const uint8_t* y;
  uint64_t yl;
};

// _bytes_to_share (shamir.py:36-45): x = bytes 1 .. 1 + data[0], y = the rest
Parsed parse(const uint8_t* d, uint64_t n) {
  Parsed p{};
  const uint32_t xl = n ? d[0] : 0;
  const uint64_t xe = std::min<uint64_t>(n, 1ull + xl);
  p.x = d + std::min<uint64_t>(n, 1);
  p.xl = static_cast<uint32_t>(xe - std::min<uint64_t>(n, 1));
  p.y = d + xe;
  p.yl = n - xe;
  return p;
}

}  // namespace
}  // namespace dn

using namespace dn;

extern "C" int dn_shamir_make_shares_host(const uint8_t* value, uint64_t value_len, const uint8_t* coeffs_be,
                                          uint32_t coeff_bytes, int threshold, const uint8_t* prime_be,
                                          uint32_t prime_len, uint64_t n_shares, uint8_t* out, uint64_t out_cap,
                                          uint64_t* offsets) {
  if (threshold > 0 && static_cast<uint64_t>(threshold) > n_shares)
    return set_error(DN_ERR_THRESHOLD, "threshold should be little equal than shares");
  if (n_shares == 0) {
    if (offsets) offsets[0] = 0;
    return DN_OK;
  }
  if ((value_len && !value) || (threshold > 1 && !coeffs_be) || !out || !offsets)
    return set_error(DN_ERR_ARG, "dn_shamir_make_shares_host: null pointer");
  const int t = threshold > 0 ? threshold : 1;
  const uint32_t plen = is_m521(prime_be, prime_len) ? 66u : prime_len;
  if (out_cap < n_shares * (9ull + plen))
    return set_error(DN_ERR_ARG, "dn_shamir_make_shares_host: output capacity < n * (9 + len(p))");
  uint64_t o = 0;
  offsets[0] = 0;
  if (is_m521(prime_be, prime_len)) {
    // Horner from the top with % p each step == canonical residue of f(x);
    // the secret (coefficient 0) is reduced first: (v x + c0) % p == (v x + c0 % p) % p
    std::vector<F> c(t);
    from_be(value, value_len, c[0]);
    for (int j = 1; j < t; ++j) from_be(coeffs_be + static_cast<uint64_t>(j - 1) * coeff_bytes, coeff_bytes, c[j]);
    uint8_t yb[kW * 8];
    for (uint64_t x = 1; x <= n_shares; ++x) {
      F v{};
      for (int j = t - 1; j >= 0; --j) {
        F nv;
        mul_small_add(v, x, c[j], nv);
        v = nv;
      }
      o += put_record(x, yb, to_be_min(v, yb), out + o);
      offsets[x] = o;
    }
    return DN_OK;
  }
  const BN p = bn_from_be(prime_be, prime_len);
  if (p.zero()) return set_error(DN_ERR_ZERODIV, "ZeroDivisionError");
  std::vector<BN> c(t);
  c[0] = bn_from_be(value, value_len);
  for (int j = 1; j < t; ++j) c[j] = bn_from_be(coeffs_be + static_cast<uint64_t>(j - 1) * coeff_bytes, coeff_bytes);
  std::vector<uint8_t> yb(plen + 8);
  for (uint64_t x = 1; x <= n_shares; ++x) {
    const BN bx = bn_from_u64(x);
    BN v{};
    for (int j = t - 1; j >= 0; --j) v = bn_mod(bn_add(bn_mul(v, bx), c[j]), p);
    o += put_record(x, yb.data(), bn_to_be_min(v, yb.data()), out + o);
    offsets[x] = o;
  }
  return DN_OK;
}

// _eval_at (shamir.py:19-25) for any integers: Horner from the top with
// `value %= prime` after each step, Python's signed % (the result takes the
// sign of the modulus).  Signed values travel as magnitude BE + sign flag.
extern "C" int dn_shamir_eval_at_host(const uint8_t* coeffs_be, const uint64_t* coeff_offsets,
                                      const uint8_t* coeff_neg, int n_coeffs, const uint8_t* x_be, uint32_t x_len,
                                      int x_neg, const uint8_t* prime_be, uint32_t prime_len, int prime_neg,
                                      uint8_t* out, uint64_t out_cap, uint64_t* out_len, int* out_neg) {
  if (n_coeffs < 0 || !out_len || !out_neg || (n_coeffs && (!coeffs_be || !coeff_offsets)) ||
      (x_len && !x_be) || (prime_len && !prime_be))
    return set_error(DN_ERR_ARG, "dn_shamir_eval_at_host: bad arguments");
  *out_len = 0;
  *out_neg = 0;
  if (n_coeffs == 0) return DN_OK;  // the loop never runs: value = 0
  BN p = bn_from_be(prime_be, prime_len);
  if (p.zero()) return set_error(DN_ERR_ZERODIV, "integer division or modulo by zero");
  BN x = bn_from_be(x_be, x_len);
  x.neg = x_neg && !x.zero();
  BN v{};
  for (int j = n_coeffs - 1; j >= 0; --j) {
    BN c = bn_from_be(coeffs_be + coeff_offsets[j], coeff_offsets[j + 1] - coeff_offsets[j]);
    c.neg = coeff_neg && coeff_neg[j] && !c.zero();
    v = bn_mod(bn_add(bn_mul(v, x), c), p);  // in [0, |p|)
    if (prime_neg && !v.zero()) {            // Python: (a % -m) == (a % m) - m when nonzero
      v = sub_mag(p, v);
      v.neg = true;
    }
  }
  if (out_cap < v.m.size() * 4) return set_error(DN_ERR_ARG, "dn_shamir_eval_at_host: output capacity too small");
  *out_len = bn_to_be_min(v, out);
  *out_neg = v.neg ? 1 : 0;
  return DN_OK;
}

extern "C" int dn_shamir_resolve_shares_host(const uint8_t* shares, const uint64_t* offsets, int k, int threshold,
                                             const uint8_t* prime_be, uint32_t prime_len, uint8_t* out,
                                             uint64_t out_cap, uint64_t* out_len) {
  if (k < 0 || !offsets || !out || !out_len || (k && !shares))
    return set_error(DN_ERR_ARG, "dn_shamir_resolve_shares_host: bad arguments");
  if (k < threshold) return set_error(DN_ERR_TOO_FEW, "need at least %d shares", threshold);
  std::vector<Parsed> sh(k);
  for (int i = 0; i < k; ++i) sh[i] = parse(shares + offsets[i], offsets[i + 1] - offsets[i]);
  // x values compared as integers (leading zero bytes do not count)
  std::vector<BN> xs(k);
  for (int i = 0; i < k; ++i) xs[i] = bn_from_be(sh[i].x, sh[i].xl);
  for (int i = 0; i < k; ++i)
    for (int j = i + 1; j < k; ++j)
      if (cmp_mag(xs[i], xs[j]) == 0) return set_error(DN_ERR_DISTINCT, "shares must be distinct");
  if (k == 1) return set_error(DN_ERR_EMPTY, "reduce() of empty iterable with no initial value");
  const bool m521 = is_m521(prime_be, prime_len);
  const uint32_t plen = m521 ? 66u : prime_len;
  if (out_cap < plen) return set_error(DN_ERR_ARG, "dn_shamir_resolve_shares_host: output capacity < len(p)");
  if (m521) {
    // fast form: every |num_i|, |den_i| < 2^63 (small abscissas): the secret is
    // sum_i y_i num_i / den_i mod p, the same field value the reference's
    // num * den ... / den sequence computes
    bool small = true;
    std::vector<int64_t> x(k);
    for (int i = 0; i < k && small; ++i) {
      small = xs[i].m.size() <= 1;
      x[i] = small ? (xs[i].zero() ? 0 : xs[i].m[0]) : 0;
    }
    std::vector<i128> num(k, 1), den(k, 1);
    const i128 lim = static_cast<i128>(1) << 63;
    for (int i = 0; i < k && small; ++i)
      for (int j = 0; j < k && small; ++j) {
        if (i == j) continue;
        num[i] *= -x[j];
        den[i] *= x[i] - x[j];
        small = num[i] < lim && num[i] > -lim && den[i] < lim && den[i] > -lim;
      }
    if (small) {
      F acc{};
      for (int i = 0; i < k; ++i) {
        F y, yn, inv, term, zero{};
        from_be(sh[i].y, sh[i].yl, y);
        const bool nneg = num[i] < 0, dneg = den[i] < 0;
        mul_small_add(y, static_cast<uint64_t>(nneg ? -num[i] : num[i]), zero, yn);
        inv_small(static_cast<uint64_t>(dneg ? -den[i] : den[i]), inv);
        mul(yn, inv, term);
        if (nneg != dneg) neg(term, term);
        F s;
        add(acc, term, s);
        acc = s;
      }
      *out_len = to_be_min(acc, out);
      return DN_OK;
    }
  }
  // the reference's sequence verbatim (shamir.py:77-90, op.py:28-29)
  BN P;
  if (m521) {
    std::vector<uint8_t> pb(66, 0xFF);
    pb[0] = 0x01;
    P = bn_from_be(pb.data(), 66);
  } else {
    P = bn_from_be(prime_be, prime_len);
  }
  if (P.zero()) return set_error(DN_ERR_ZERODIV, "ZeroDivisionError");
  std::vector<BN> nums(k), dens(k);
  for (int i = 0; i < k; ++i) {
    BN a = bn_from_u64(1), b = bn_from_u64(1);
    for (int j = 0; j < k; ++j) {
      if (i == j) continue;
      a = bn_mul(a, bn_neg(xs[j]));
      b = bn_mul(b, bn_add(xs[i], bn_neg(xs[j])));
    }
    nums[i] = a, dens[i] = b;
  }
  BN den = bn_from_u64(1);
  for (int i = 0; i < k; ++i) den = bn_mul(den, dens[i]);
  BN num{};
  for (int i = 0; i < k; ++i) {
    const BN y = bn_from_be(sh[i].y, sh[i].yl);
    const BN a = bn_mod(bn_mul(bn_mul(nums[i], den), y), P);
    BN inv;
    const int rc = bn_inverse(dens[i], P, inv);
    if (rc != DN_OK) return rc;
    num = bn_add(num, bn_mod(bn_mul(a, inv), P));
  }
  BN inv;
  const int rc = bn_inverse(den, P, inv);
  if (rc != DN_OK) return rc;
  const BN res = bn_mod(bn_mul(num, inv), P);
  std::vector<uint8_t> buf(res.m.size() * 4 + 1);
  const uint32_t n = bn_to_be_min(res, buf.data());
  if (n > out_cap) return set_error(DN_ERR_ARG, "dn_shamir_resolve_shares_host: output capacity");
  std::memcpy(out, buf.data(), n);
  *out_len = n;
  return DN_OK;
}
