// host_mt_jump.cpp — MT19937 jump-ahead on the host (plain C++; see
// mt19937_device.hip for how the device draw uses it).
//
// MT19937's one-word transition f (window (x_T .. x_T+623) -> (x_T+1 ..
// x_T+624), x_{T+624} = x_{T+397} ^ twist(x_T, x_{T+1})) is F2-linear on 19937
// state bits; jumping J words is g(f) with g = x^J mod P, P its characteristic
// polynomial (tools/gen_mt_jump.py -> mt19937_jump.inc), evaluated by Horner
// (Haramoto et al., INFORMS J. Computing 20(3), 2008).
#include <cstdint>
#include <cstring>
#include <vector>

#include "dn_internal.hpp"

namespace dn {
namespace {

#include "mt19937_jump.inc"

alignas(64) static const uint64_t kMtJumpPolys[kMtJumpRows][kMtPolyWords] = DN_MT_JUMP_POLYS;

constexpr int kMtN = 624, kMtM = 397;
constexpr uint32_t kMtA = 0x9908b0dfu, kMtUp = 0x80000000u, kMtLo = 0x7fffffffu;

inline uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
  const uint32_t y = (a & kMtUp) | (b & kMtLo);
  return m ^ (y >> 1) ^ ((0u - (y & 1u)) & kMtA);
}

// Windows are advanced in a linear buffer: buf[p .. p+623] is the window at
// time T + p and a step appends buf[p + 624] = mix(buf[p], buf[p+1],
// buf[p+397]).  Up to 227 consecutive steps read only words already in the
// buffer, so they are one branch-free (vectorised) loop.
__attribute__((target_clones("avx512f", "avx2", "default")))
void mt_extend(uint32_t* __restrict buf, uint64_t p, int steps) {  // steps <= 227
  const uint32_t* src = buf + p;
  uint32_t* dst = buf + p + kMtN;
  for (int i = 0; i < steps; ++i) dst[i] = mt_mix(src[i], src[i + 1], src[i + kMtM]);
}

__attribute__((target_clones("avx512f", "avx2", "default")))
void xor_words(uint32_t* __restrict d, const uint32_t* __restrict s, int n) {
  for (int i = 0; i < n; ++i) d[i] ^= s[i];
}

void mt_advance(const uint32_t* win, uint64_t steps, uint32_t* out) {
  std::vector<uint32_t> buf(kMtN + steps);
  std::memcpy(buf.data(), win, kMtN * sizeof(uint32_t));
  for (uint64_t p = 0; p < steps;) {
    const int n = steps - p < 227 ? static_cast<int>(steps - p) : 227;
    mt_extend(buf.data(), p, n);
    p += n;
  }
  std::memcpy(out, buf.data() + steps, kMtN * sizeof(uint32_t));
}

// out = g(f)(win): the window jumped by J words.  The low 31 bits of out[0]
// are not determined (they reach neither an output nor the dynamics).
// Horner over 8-bit chunks of g: r = f^8(r) ^ T[chunk], T[b] = sum_j b_j f^j(win)
// (256 precomputed windows): one 624-word XOR per 8 coefficients.
void mt_jump(const uint32_t* win, const uint64_t* g, uint32_t* out) {
  constexpr int kQ = 8;
  std::vector<uint32_t> T(static_cast<size_t>(1 << kQ) * kMtN, 0u);
  {
    std::vector<uint32_t> w(kMtN + kQ);
    std::memcpy(w.data(), win, kMtN * sizeof(uint32_t));
    mt_extend(w.data(), 0, kQ);  // f^j(win) = w[j .. j+623]
    for (int j = 0; j < kQ; ++j) {  // T[2^j + b] = T[b] ^ f^j(win)
      const int bit = 1 << j;
      for (int b = 0; b < bit; ++b) {
        uint32_t* d = T.data() + static_cast<size_t>(bit + b) * kMtN;
        std::memcpy(d, T.data() + static_cast<size_t>(b) * kMtN, kMtN * sizeof(uint32_t));
        xor_words(d, w.data() + j, kMtN);
      }
    }
  }
  int top = kMtPolyWords * 64 - 1;
  while (top >= 0 && !((g[top >> 6] >> (top & 63)) & 1u)) --top;
  const int chunks = top / kQ + 1;
  std::vector<uint32_t> buf(kMtN + static_cast<size_t>(chunks) * kQ, 0u);
  uint64_t p = 0;
  for (int c = chunks - 1; c >= 0; --c) {
    mt_extend(buf.data(), p, kQ);
    p += kQ;
    const int bit0 = c * kQ;
    const uint32_t chunk = static_cast<uint32_t>((g[bit0 >> 6] >> (bit0 & 63)) & ((1u << kQ) - 1u));
    if (chunk) xor_words(buf.data() + p, T.data() + static_cast<size_t>(chunk) * kMtN, kMtN);
  }
  std::memcpy(out, buf.data() + p, kMtN * sizeof(uint32_t));
}

// The window of substream s >= 1: buffer positions idx + s L - 624 ..
// idx + s L - 1, counted from the caller's array (position 0) — s L stream
// words after the caller's next output, minus one array.  With
// s - 1 = 4096 c + 64 a + b: A_a, then C_c (c > 0), then B_b (b > 0).
void mt_window_at(const uint32_t* state, int idx, uint64_t s, uint32_t* out) {
  std::vector<uint32_t> cur(kMtN), nxt(kMtN);
  mt_advance(state, static_cast<uint64_t>(idx), cur.data());  // W_idx
  const uint64_t d = s - 1;
  const int b = static_cast<int>(d % kMtJumpRadix), a = static_cast<int>((d / kMtJumpRadix) % kMtJumpRadix),
            c = static_cast<int>(d / (kMtJumpRadix * kMtJumpRadix));
  mt_jump(cur.data(), kMtJumpPolys[kMtRowA + a], nxt.data());
  cur.swap(nxt);
  if (c) {
    mt_jump(cur.data(), kMtJumpPolys[kMtRowC + c], nxt.data());
    cur.swap(nxt);
  }
  if (b) {
    mt_jump(cur.data(), kMtJumpPolys[kMtRowB + b], nxt.data());
    cur.swap(nxt);
  }
  std::memcpy(out, cur.data(), kMtN * sizeof(uint32_t));
}

}  // namespace

uint64_t mt_jump_words() { return kMtJumpL; }
uint64_t mt_jump_max_subs() { return 1ull + static_cast<uint64_t>(kMtJumpRadix) * kMtJumpRadix * kMtJumpRadix; }

// CPython's state after `words` more outputs: the array at buffer position
// 624 q (q = ceil((words - h) / 624) twists, h = 624 - idx) with index
// words - h - 624 (q - 1), stepped from the last substream window strictly
// before it (the windows' first word is exact only in its top bit, so at
// least one step).
bool mt_final_state(const uint32_t* state, int idx, uint64_t words, uint32_t* fin, int32_t* fidx) {
  const uint64_t h = static_cast<uint64_t>(kMtN - idx);
  if (words <= h) {
    std::memcpy(fin, state, kMtN * sizeof(uint32_t));
    *fidx = idx + static_cast<int32_t>(words);
    return true;
  }
  const uint64_t m_end = words - h, q = (m_end + kMtN - 1) / kMtN, tf = kMtN * q;  // buffer position
  // substream s >= 1 starts at position idx + s L - 624 (mt_window_at)
  const uint64_t sig = (tf + kMtN - 1 - static_cast<uint64_t>(idx)) / kMtJumpL;  // idx + sig L - 624 < tf
  if (sig >= mt_jump_max_subs()) return false;  // beyond the jump table (> 1.4e11 words)
  std::vector<uint32_t> w(kMtN);
  uint64_t t_sig = 0;
  if (sig == 0) {
    std::memcpy(w.data(), state, kMtN * sizeof(uint32_t));
  } else {
    mt_window_at(state, idx, sig, w.data());
    t_sig = static_cast<uint64_t>(idx) + sig * kMtJumpL - kMtN;
  }
  mt_advance(w.data(), tf - t_sig, fin);
  *fidx = static_cast<int32_t>(m_end - kMtN * (q - 1));
  return true;
}

void mt_advance_window(const uint32_t* win, uint64_t steps, uint32_t* out) { mt_advance(win, steps, out); }

}  // namespace dn

using namespace dn;

extern "C" int dn_mt19937_skip(uint32_t* mt_state, int32_t* mt_index, uint64_t words) {
  if (!mt_state || !mt_index) return set_error(DN_ERR_ARG, "dn_mt19937_skip: null pointer");
  const int32_t idx = *mt_index;
  if (idx < 0 || idx > kMtN) return set_error(DN_ERR_ARG, "dn_mt19937_skip: bad MT index");
  std::vector<uint32_t> fin(kMtN);
  int32_t fidx = 0;
  if (!mt_final_state(mt_state, idx, words, fin.data(), &fidx))
    return set_error(DN_ERR_UNSUPPORTED, "dn_mt19937_skip: %llu words exceed the jump table",
                     static_cast<unsigned long long>(words));
  std::memcpy(mt_state, fin.data(), kMtN * sizeof(uint32_t));
  *mt_index = fidx;
  return DN_OK;
}

// x^words mod P (host_gf2poly.cpp's mt_xpow_mod): dn_shamir.h
extern "C" int dn_mt19937_jump_poly(uint64_t words, uint64_t* out) {
  if (!out) return dn::set_error(DN_ERR_ARG, "dn_mt19937_jump_poly: null pointer");
  if (!dn::mt_xpow_mod(words, out))
    return dn::set_error(DN_ERR_UNSUPPORTED, "dn_mt19937_jump_poly: no carry-less multiply");
  return DN_OK;
}
