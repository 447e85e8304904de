// host_gf2poly.cpp — MT19937 jump polynomials computed on the host at run time
// (plain C++; mt19937_device.hip uses them).
//
// The device draw reaches substream window s by jumps g(f) W with
// g = x^J mod P (P the characteristic polynomial of the one-word transition,
// degree 19937; tools/gen_mt_jump.py).  For the largest draws it can take one
// direct level instead of the radix-64 levels A then B if it has
// D_s = x^(L - 624 + (s - 1) L) mod P for s up to ~2048 (L = 17 * 2^14): too
// many rows to tabulate in source (5 MB), so they are computed here as
// D_{s+1} = D_s * x^L mod P from the tabulated D_1 and x^L = B_1, one GF(2)[x]
// product and one Barrett reduction per row (carry-less multiplies), and
// checked against the 63 tabulated direct rows D_2..D_64.
//
// Computing the 1024 rows a 2^24 draw needs took ~0.13 s of a process's first
// make_shares_vec, so the build computes all kMtRtRows
// once (csrc/gen_mt_rt_rows.cpp -> lib/mt_rt_rows14.bin) and embeds them in
// the library (csrc/mt_rt_rows14.S, .incbin); at first use the embedded rows
// are checked — the generator's 128-bit checksum of the whole table (two
// trailing words: a blob damaged after generation), D_1..D_64 against the
// tabulated rows, and 16 rows spread over the table against the recurrence
// D_s = D_{s-1} x^L (a wrong computation) — and used as they are.  A library
// built without the blob (the build host had no carry-less multiply: the
// Makefile embeds an empty one), or a blob that fails the check, falls back to
// computing rows at run time.
#include <immintrin.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "dn_internal.hpp"

namespace dn {
namespace {

#include "mt19937_charpoly.inc"
#include "mt19937_jump.inc"
#include "mt19937_jump_direct.inc"

constexpr int kW = kMtPolyWords;  // 312 words: degree < 19937
constexpr int kDeg = 19937;
static_assert(kW * 64 > kDeg && (kW - 1) * 64 <= kDeg, "poly words");

const uint64_t kP[1][kW] = DN_MT_CHAR_POLY;
const uint64_t kJump14[kMtJumpRows][kW] = DN_MT_JUMP_POLYS;
const uint64_t kDirect14[kMtDirectRows][kW] = DN_MT_JUMP_DIRECT_L14;

// r[0 .. na + nb) = a * b (carry-less), column by column: the 128-bit
// products of word pairs (i, k - i) XOR into one register, two output words
// per column, so the inner loop has no memory traffic
__attribute__((target("pclmul,sse4.1"))) void clmul_poly(const uint64_t* a, int na, const uint64_t* b, int nb,
                                                          uint64_t* r) {
  std::memset(r, 0, sizeof(uint64_t) * (na + nb));
  for (int k = 0; k < na + nb - 1; ++k) {
    const int i0 = k - nb + 1 > 0 ? k - nb + 1 : 0, i1 = k < na - 1 ? k : na - 1;
    __m128i acc = _mm_setzero_si128(), acc2 = _mm_setzero_si128();
    int i = i0;
    for (; i + 1 <= i1; i += 2) {  // two independent chains; b[k - i - 1], b[k - i] as one load
      const __m128i av = _mm_loadu_si128(reinterpret_cast<const __m128i*>(a + i));
      const __m128i bv = _mm_loadu_si128(reinterpret_cast<const __m128i*>(b + k - i - 1));
      acc = _mm_xor_si128(acc, _mm_clmulepi64_si128(av, bv, 0x10));   // a[i] * b[k - i]
      acc2 = _mm_xor_si128(acc2, _mm_clmulepi64_si128(av, bv, 0x01));  // a[i + 1] * b[k - i - 1]
    }
    if (i <= i1)
      acc = _mm_xor_si128(acc, _mm_clmulepi64_si128(_mm_loadl_epi64(reinterpret_cast<const __m128i*>(a + i)),
                                                     _mm_loadl_epi64(reinterpret_cast<const __m128i*>(b + k - i)), 0x00));
    acc = _mm_xor_si128(acc, acc2);
    r[k] ^= static_cast<uint64_t>(_mm_cvtsi128_si64(acc));
    r[k + 1] ^= static_cast<uint64_t>(_mm_extract_epi64(acc, 1));
  }
}

// out[0 .. n) = words of (a >> sh bits), a of na words
void shr_bits(const uint64_t* a, int na, int sh, uint64_t* out, int n) {
  const int ws = sh / 64, bs = sh % 64;
  for (int i = 0; i < n; ++i) {
    const int k = i + ws;
    const uint64_t lo = k < na ? a[k] : 0u;
    const uint64_t hi = k + 1 < na ? a[k + 1] : 0u;
    out[i] = bs ? (lo >> bs) | (hi << (64 - bs)) : lo;
  }
}

bool bit(const uint64_t* a, int i) { return (a[i / 64] >> (i % 64)) & 1u; }

struct Barrett {
  std::vector<uint64_t> mu;  // floor(x^(2 deg) / P): degree deg, kW words
  Barrett() : mu(kW, 0) {
    // long division of x^(2 deg) by P, one quotient bit at a time
    std::vector<uint64_t> r(2 * kW + 1, 0);
    r[(2 * kDeg) / 64] |= 1ull << ((2 * kDeg) % 64);
    for (int i = 2 * kDeg; i >= kDeg; --i) {
      if (!bit(r.data(), i)) continue;
      mu[(i - kDeg) / 64] |= 1ull << ((i - kDeg) % 64);
      const int sh = i - kDeg, ws = sh / 64, bs = sh % 64;  // r ^= P << sh
      for (int k = 0; k < kW; ++k) {
        const uint64_t w = kP[0][k];
        r[k + ws] ^= w << bs;
        if (bs) r[k + ws + 1] ^= w >> (64 - bs);
      }
    }
  }
  // out = a * b mod P (a, b of degree < deg)
  void mulmod(const uint64_t* a, const uint64_t* b, uint64_t* out) const {
    std::vector<uint64_t> c(2 * kW), hi(kW), t(2 * kW), q(kW), qp(2 * kW);
    clmul_poly(a, kW, b, kW, c.data());
    shr_bits(c.data(), 2 * kW, kDeg, hi.data(), kW);  // c / x^deg
    clmul_poly(hi.data(), kW, mu.data(), kW, t.data());
    shr_bits(t.data(), 2 * kW, kDeg, q.data(), kW);  // quotient
    clmul_poly(q.data(), kW, kP[0], kW, qp.data());
    for (int k = 0; k < kW; ++k) out[k] = c[k] ^ qp[k];
    out[kW - 1] &= (1ull << (kDeg % 64)) - 1u;  // bits >= deg are zero in c ^ qP
  }
};

struct Rows {
  std::mutex m;
  std::vector<uint64_t> rows;  // row s - 1 = D_s; allocated once (pointers stay valid)
  std::vector<uint8_t> have;   // row computed
  uint64_t odd_top = 0;        // D_1, D_3, .., D_odd_top computed in sequence
  uint64_t version = 0;        // rows computed so far (changes when any row is added)
  bool ok = true;
  Barrett* br = nullptr;
};

Rows& rows14() {
  static Rows* r = new Rows;  // never destroyed
  return *r;
}

bool set_row(Rows& R, uint64_t s, const uint64_t* prev, const uint64_t* mul) {
  uint64_t* out = R.rows.data() + (s - 1) * kW;
  R.br->mulmod(prev, mul, out);
  R.have[s - 1] = 1;
  ++R.version;
  // the tabulated direct rows D_2 .. D_64 check the arithmetic
  if (s <= static_cast<uint64_t>(kMtDirectRows) && std::memcmp(out, kDirect14[s - 1], sizeof(uint64_t) * kW)) {
    R.ok = false;
    return false;
  }
  return true;
}

// The embedded table (csrc/mt_rt_rows14.S): kMtRtRows rows, or none.
extern "C" const uint64_t dn_mt_rt_rows14_blob[] __attribute__((weak, visibility("hidden")));
extern "C" const uint64_t dn_mt_rt_rows14_blob_end[] __attribute__((weak, visibility("hidden")));

// The embedded rows once checked (nullptr: absent or wrong).
const uint64_t* embedded_rows() {
  static const uint64_t* checked = [] () -> const uint64_t* {
    const uint64_t* b = dn_mt_rt_rows14_blob;
    const uint64_t nw = kMtRtRows * static_cast<uint64_t>(kW);
    if (!b || !dn_mt_rt_rows14_blob_end || static_cast<uint64_t>(dn_mt_rt_rows14_blob_end - b) != nw + 2)
      return nullptr;
    uint64_t h[2];
    mt_rt_rows_checksum(b, nw, h);
    if (h[0] != b[nw] || h[1] != b[nw + 1]) return nullptr;
    for (int s = 1; s <= kMtDirectRows; ++s)
      if (std::memcmp(b + (s - 1) * kW, kDirect14[s - 1], sizeof(uint64_t) * kW)) return nullptr;
    Barrett br;
    std::vector<uint64_t> r(kW);
    for (uint64_t s = kMtRtRows; s > kMtRtRows - 16 * 127; s -= 127) {  // 16 rows, the last one included
      br.mulmod(b + (s - 2) * kW, kJump14[kMtRowB + 1], r.data());
      if (std::memcmp(r.data(), b + (s - 1) * kW, sizeof(uint64_t) * kW)) return nullptr;
    }
    return b;
  }();
  return checked;
}

}  // namespace

void mt_rt_rows_checksum(const uint64_t* w, uint64_t n, uint64_t out[2]) {
  // two independent multiply-rotate chains over the words (not a MAC: it
  // catches a blob damaged between the generator and the library)
  uint64_t a = 0x9E3779B97F4A7C15ull ^ n, c = 0xC2B2AE3D27D4EB4Full;
  for (uint64_t i = 0; i < n; ++i) {
    a = ((a ^ w[i]) * 0xFF51AFD7ED558CCDull);
    a ^= a >> 29;
    c = ((c + w[i]) * 0xC4CEB9FE1A85EC53ull) ^ (c >> 31) ^ i;
  }
  out[0] = a;
  out[1] = c;
}

// x^e mod P by square-and-multiply (Barrett squarings; a multiply by x is a
// shift and at most one XOR of P): the jump polynomial of e words, for the
// speculated next call's W_idx (mt19937_device.hip, DN_MT_SPEC beside the
// generation).  ~30 products: a few ms, once per draw size.
bool mt_xpow_mod(uint64_t e, uint64_t* out) {
  if (!__builtin_cpu_supports("pclmul")) return false;
  static Barrett* br = new Barrett;  // (never destroyed; built once: ~20 ms)
  std::vector<uint64_t> r(kW, 0), t(kW);
  r[0] = 1;
  for (int b = e ? 63 - __builtin_clzll(e) : -1; b >= 0; --b) {
    br->mulmod(r.data(), r.data(), t.data());
    r.swap(t);
    if ((e >> b) & 1u) {
      uint64_t carry = 0;
      for (int k = 0; k < kW; ++k) {
        const uint64_t w = r[k];
        r[k] = (w << 1) | carry;
        carry = w >> 63;
      }
      if (bit(r.data(), kDeg)) {
        for (int k = 0; k < kW; ++k) r[k] ^= kP[0][k];
      }
    }
  }
  std::memcpy(out, r.data(), sizeof(uint64_t) * kW);
  return true;
}

bool mt_rt_rows_compute(uint64_t* out, uint64_t nrows) {
  if (!__builtin_cpu_supports("pclmul") || nrows == 0) return false;
  Barrett br;
  std::memcpy(out, kDirect14[0], sizeof(uint64_t) * kW);  // D_1
  for (uint64_t s = 2; s <= nrows; ++s) {
    br.mulmod(out + (s - 2) * kW, kJump14[kMtRowB + 1], out + (s - 1) * kW);
    if (s <= static_cast<uint64_t>(kMtDirectRows) &&
        std::memcmp(out + (s - 1) * kW, kDirect14[s - 1], sizeof(uint64_t) * kW))
      return false;
  }
  return true;
}

const uint64_t* mt_direct_rows_l14(uint64_t S, uint64_t* version) {
  if (S < 2 || S - 1 > kMtRtRows) return nullptr;
  if (const uint64_t* e = embedded_rows()) {
    if (version) *version = ~0ull;  // every row, never changes
    return e;
  }
  if (!__builtin_cpu_supports("pclmul")) return nullptr;
  Rows& R = rows14();
  std::lock_guard<std::mutex> g(R.m);
  if (!R.ok) return nullptr;
  if (R.rows.empty()) {
    R.rows.assign(static_cast<size_t>(kMtRtRows) * kW, 0u);
    R.have.assign(kMtRtRows, 0u);
    R.br = new Barrett;
    std::memcpy(R.rows.data(), kDirect14[0], sizeof(uint64_t) * kW);  // D_1
    R.have[0] = 1;
    R.odd_top = 1;
    if (!set_row(R, 2, R.rows.data(), kJump14[kMtRowB + 1])) return nullptr;  // D_2 = D_1 x^L, checked
  }
  // the windows a backward-generating draw of S substreams starts from: odd
  // s < S (D_{s+2} = D_s x^(2L), B_2 = x^(2L)) and the last, S - 1
  const uint64_t last = S - 1;
  for (uint64_t s = R.odd_top + 2; s <= last; s += 2, R.odd_top += 2)
    if (!set_row(R, s, R.rows.data() + (s - 3) * kW, kJump14[kMtRowB + 2])) return nullptr;
  if (!R.have[last - 1] && !set_row(R, last, R.rows.data() + (last - 2) * kW, kJump14[kMtRowB + 1]))
    return nullptr;
  if (version) *version = R.version;
  return R.rows.data();
}

}  // namespace dn

extern "C" int dn_mt19937_rt_rows_embedded(void) { return dn::embedded_rows() ? 1 : 0; }
