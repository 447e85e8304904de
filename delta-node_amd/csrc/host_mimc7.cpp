// host_mimc7.cpp — calc_weight_commitment's MiMC7 chain on a host core
// (SURVEY.md §8(f) row 4), plus the field parameters of utils/constant.py.
//
// Reference: delta_node/utils/mimc7.py:18-60 (mimc7_hash, mimc7_hash_arr,
// _float2mpz, calc_weight_commitment) over the BN254 scalar field q with the
// 13 round constants of utils/constant.py:6-30.
//
// Why the host: the weight commitment is ONE chain — every step's hash is
// keyed by the previous step's result, each hash is 13 rounds of t^7 (4
// dependent field products), so a weight costs 52 strictly dependent 254-bit
// Montgomery products and nothing can run beside them.  A GPU lane runs such a
// chain at its dependent-instruction latency (measured on one gfx950 lane:
// 67.7 us per weight with 8x32-bit CIOS, 33 us with the 29-bit separated-operand
// product of mimc7_bn254.hip); a host core with 64x64->128-bit
// multiplies does a 4-limb CIOS product in tens of ns.  The parallel parts of
// the row (calc_data_commitment's row hashes and Merkle blocks) stay on the
// GPU (mimc7_bn254.hip).  The weights are host data in the reference's caller
// (coord/hlr/manager.py:68-69), so no transfer is involved either.
//
// Arithmetic: Montgomery with R = 2^256, 4 x 64-bit limbs (CIOS, unsigned
// __int128 products); values stay in Montgomery form through the chain (sums
// commute with the form).  _float2mpz is exact for every finite double (the
// device row pass stops at |v 10^p| < 2^253).
#include <cmath>
#include <cstdint>
#include <cstring>

#include "dn_internal.hpp"
#include "dn_mimc7.h"
#include "mimc7_consts.hpp"

namespace dn {
namespace mimc {
namespace {

typedef unsigned __int128 u128;

struct F {
  uint64_t w[4];
};

struct Host {
  F q;
  uint64_t qinv;  // -q^{-1} mod 2^64
  F r2;           // R^2 mod q
  F half_q;       // floor(q / 2)
  F cts[kRounds]; // Montgomery form
};

inline bool geq(const F& a, const F& b) {
  for (int i = 3; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] > b.w[i];
  return true;
}

inline void sub_in(F& a, const F& b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 d = static_cast<u128>(a.w[i]) - b.w[i] - br;
    a.w[i] = static_cast<uint64_t>(d);
    br = static_cast<uint64_t>(d >> 64) & 1u;
  }
}

// a + b mod q for a, b < q (q < 2^254: the sum never carries out of 256 bits)
inline F addmod(const F& a, const F& b, const F& q) {
  F r;
  uint64_t c = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 s = static_cast<u128>(a.w[i]) + b.w[i] + c;
    r.w[i] = static_cast<uint64_t>(s);
    c = static_cast<uint64_t>(s >> 64);
  }
  if (geq(r, q)) sub_in(r, q);
  return r;
}

// CIOS Montgomery product a b R^{-1} mod q (inputs < q, output < q).  With
// q < 2^254 the running value stays below 2q < 2^255, so one spare limb holds
// every carry and a single conditional subtraction finishes.
inline F mont_mul(const F& a, const F& b, const Host& h) {
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
  for (int i = 0; i < 4; ++i) {
    const uint64_t bi = b.w[i];
    u128 s = static_cast<u128>(a.w[0]) * bi + t0;
    t0 = static_cast<uint64_t>(s);
    s = static_cast<u128>(a.w[1]) * bi + t1 + (s >> 64);
    t1 = static_cast<uint64_t>(s);
    s = static_cast<u128>(a.w[2]) * bi + t2 + (s >> 64);
    t2 = static_cast<uint64_t>(s);
    s = static_cast<u128>(a.w[3]) * bi + t3 + (s >> 64);
    t3 = static_cast<uint64_t>(s);
    t4 += static_cast<uint64_t>(s >> 64);
    const uint64_t m = t0 * h.qinv;
    s = static_cast<u128>(m) * h.q.w[0] + t0;
    s = static_cast<u128>(m) * h.q.w[1] + t1 + (s >> 64);
    t0 = static_cast<uint64_t>(s);
    s = static_cast<u128>(m) * h.q.w[2] + t2 + (s >> 64);
    t1 = static_cast<uint64_t>(s);
    s = static_cast<u128>(m) * h.q.w[3] + t3 + (s >> 64);
    t2 = static_cast<uint64_t>(s);
    s = static_cast<u128>(t4) + (s >> 64);
    t3 = static_cast<uint64_t>(s);
    t4 = static_cast<uint64_t>(s >> 64);
  }
  F r = {{t0, t1, t2, t3}};
  if (t4 || geq(r, h.q)) sub_in(r, h.q);
  return r;
}

F from_limbs32(const uint32_t v[8]) {
  F r;
  for (int i = 0; i < 4; ++i) r.w[i] = static_cast<uint64_t>(v[2 * i]) | (static_cast<uint64_t>(v[2 * i + 1]) << 32);
  return r;
}

void to_limbs32(const F& a, uint32_t v[8]) {
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = static_cast<uint32_t>(a.w[i]);
    v[2 * i + 1] = static_cast<uint32_t>(a.w[i] >> 32);
  }
}

inline F to_mont(const F& a, const Host& h) { return mont_mul(a, h.r2, h); }
inline F from_mont(const F& a, const Host& h) {
  const F one = {{1, 0, 0, 0}};
  return mont_mul(a, one, h);
}

void make_host(Host& h) {
  h.q = from_limbs32(kQ32);
  uint64_t inv = h.q.w[0];  // Newton: inv = q^{-1} mod 2^64
  for (int i = 0; i < 6; ++i) inv *= 2u - h.q.w[0] * inv;
  h.qinv = 0u - inv;
  F v = {{1, 0, 0, 0}};
  for (int it = 0; it < 512; ++it) v = addmod(v, v, h.q);  // 2^512 mod q
  h.r2 = v;
  for (int i = 0; i < 4; ++i) h.half_q.w[i] = (h.q.w[i] >> 1) | (i < 3 ? (h.q.w[i + 1] << 63) : 0u);
  for (int c = 0; c < kRounds; ++c) {
    uint32_t plain[8];
    dec_to_limbs(kCtsDec[c], plain);
    h.cts[c] = to_mont(from_limbs32(plain), h);
  }
}

// mimc7_hash(x, key) (mimc7.py:18-27) in Montgomery form, reduced mod q
inline F hash_m(const F& x, const F& key, const Host& h) {
  F r = x;
  for (int c = 0; c < kRounds; ++c) {
    const F t = addmod(addmod(r, key, h.q), h.cts[c], h.q);
    const F t2 = mont_mul(t, t, h);
    const F t3 = mont_mul(t2, t, h);
    const F t6 = mont_mul(t3, t3, h);
    r = mont_mul(t6, t, h);
  }
  return addmod(r, key, h.q);
}

// _float2mpz(v, p) (mimc7.py:39-44) as a plain field element: a = int(v 10^p)
// exactly (the reference's float multiply, then truncation toward zero), then
// min(a, q - a) mod q.  Negative a stays a (field q - |a|); a > q/2 becomes
// q - a (field -a, also when a >= q).  Returns false for inf / NaN.
bool float_to_field(double v, double scale, const Host& h, F& out) {
  const double y = v * scale;
  out = F{{0, 0, 0, 0}};
  if (!std::isfinite(y)) return false;
  const double ay = std::fabs(y);
  int e;
  const double m = std::frexp(ay, &e);  // ay = m 2^e, m in [0.5, 1)
  if (e <= 0) return true;              // |a| = 0
  uint64_t mant = static_cast<uint64_t>(std::ldexp(m, 53));
  int sh = e - 53;
  if (sh < 0) {
    mant >>= -sh;
    sh = 0;
  }
  bool above_half;  // |a| > floor(q / 2)
  F mag;            // |a| mod q
  if (sh <= 256 - 53) {  // |a| = mant 2^sh < 2^256: exact limbs
    const int limb = sh / 64, bit = sh % 64;
    mag.w[0] = mag.w[1] = mag.w[2] = mag.w[3] = 0;
    mag.w[limb] = mant << bit;
    if (bit && limb + 1 < 4) mag.w[limb + 1] = mant >> (64 - bit);
    above_half = !geq(h.half_q, mag);
    while (geq(mag, h.q)) sub_in(mag, h.q);
  } else {  // |a| >= 2^52 2^204 > q: doubling mod q
    above_half = true;
    mag = F{{mant, 0, 0, 0}};
    for (int i = 0; i < sh; ++i) mag = addmod(mag, mag, h.q);
  }
  const bool zero = !(mag.w[0] | mag.w[1] | mag.w[2] | mag.w[3]);
  if ((y < 0 || above_half) && !zero) {
    out = h.q;
    sub_in(out, mag);
  } else {
    out = mag;
  }
  return true;
}

}  // namespace
}  // namespace mimc
}  // namespace dn

using namespace dn;
using namespace dn::mimc;

extern "C" int dn_mimc7_params(uint32_t* q, uint32_t* cts) {
  if (!q || !cts) return set_error(DN_ERR_ARG, "dn_mimc7_params: null pointer");
  std::memcpy(q, kQ32, sizeof(kQ32));
  for (int c = 0; c < kRounds; ++c) dec_to_limbs(kCtsDec[c], cts + 8 * c);
  return DN_OK;
}

extern "C" int dn_mimc7_weight_commitment_host(const double* w, uint64_t n, int precision, uint32_t* out) {
  if ((!w && n) || !out) return set_error(DN_ERR_ARG, "dn_mimc7_weight_commitment_host: null pointer");
  if (precision < 0 || precision > 22)
    return set_error(DN_ERR_ARG, "dn_mimc7_weight_commitment_host: precision 0..22");
  Host h;
  make_host(h);
  const double scale = pow10d(precision);
  F r = to_mont(F{{2, 0, 0, 0}}, h);  // mimc7_hash_arr(..., 2)
  for (uint64_t i = 0; i < n; ++i) {
    F x;
    if (!float_to_field(w[i], scale, h, x)) {  // int(inf): OverflowError, int(nan): ValueError
      if (std::isnan(w[i])) return set_error(DN_ERR_ARG, "cannot convert float NaN to integer");
      return set_error(DN_ERR_OVERFLOW, "cannot convert float infinity to integer");
    }
    x = to_mont(x, h);
    const F hx = hash_m(x, r, h);
    r = addmod(addmod(r, x, h.q), hx, h.q);  // mimc7.py:35
  }
  to_limbs32(from_mont(r, h), out);
  return DN_OK;
}
