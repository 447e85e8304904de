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
#include <thread>
#include <vector>

#include "dn_internal.hpp"

namespace dn {
namespace {

#include "mt19937_jump.inc"

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

// Window 1 + d (time B + (1 + d) L - h) from window 1 by the binary
// decomposition of d (jumps of 2^k L; beyond the table, repeated top jumps).
void mt_window_from1(const uint32_t* w1, uint64_t d, uint32_t* out) {
  std::vector<uint32_t> cur(w1, w1 + kMtN), nxt(kMtN);
  for (int lev = 0; d; ++lev, d >>= 1) {
    if (lev == kMtJumpLevels - 1) {  // the rest: d times 2^lev L
      for (uint64_t r = 0; r < d; ++r) {
        mt_jump(cur.data(), kMtJumpPolys[1 + lev], nxt.data());
        cur.swap(nxt);
      }
      break;
    }
    if (d & 1u) {
      mt_jump(cur.data(), kMtJumpPolys[1 + lev], nxt.data());
      cur.swap(nxt);
    }
  }
  std::memcpy(out, cur.data(), kMtN * sizeof(uint32_t));
}

// window 1 (time B + L - h): B's window stepped idx words, then L - 624 more
void mt_window1(const uint32_t* state, int idx, uint32_t* out) {
  std::vector<uint32_t> adv(kMtN);
  mt_advance(state, static_cast<uint64_t>(idx), adv.data());
  mt_jump(adv.data(), kMtJumpPolys[0], out);
}

}  // namespace

uint64_t mt_jump_words() { return kMtJumpL; }
uint64_t mt_jump_max_subs() { return 1ull << kMtJumpLevels; }

// Stream words are numbered from CPython's current position: words 0 .. h-1
// (h = 624 - idx) are the rest of the current array, word w >= h is output
// w - h of the window at time B (the current array).  Substream s >= 1 starts
// at word s L, i.e. at the window of time B + s L - h.
void mt_build_windows(const uint32_t* state, int idx, uint64_t subs, uint32_t* wins) {
  std::memcpy(wins, state, kMtN * sizeof(uint32_t));
  if (subs < 2) return;
  mt_window1(state, idx, wins + kMtN);
  // window 1 + d for d in [2^lev, 2^(lev+1)) = window 1 + d - 2^lev jumped 2^lev L
  const unsigned hw = std::thread::hardware_concurrency();
  const unsigned nthr = hw ? (hw < 16 ? hw : 16) : 1;
  for (int lev = 0; (1ull << lev) < subs - 1; ++lev) {
    const uint64_t d0 = 1ull << lev, d1 = (2ull << lev) < subs - 1 ? (2ull << lev) : subs - 1;
    const uint64_t cnt = d1 - d0;
    auto work = [&](unsigned t) {
      for (uint64_t i = t; i < cnt; i += nthr) {
        const uint64_t d = d0 + i;
        mt_jump(wins + (1 + d - d0) * kMtN, kMtJumpPolys[1 + lev], wins + (1 + d) * kMtN);
      }
    };
    if (cnt < 4 || nthr == 1) {
      for (unsigned t = 0; t < nthr; ++t) work(t);
    } else {
      std::vector<std::thread> th;
      for (unsigned t = 0; t < nthr; ++t) th.emplace_back(work, t);
      for (auto& x : th) x.join();
    }
  }
}

// CPython's state after `words` more outputs: the window at time B + 624 q
// (q = ceil((words - h) / 624) twists) with index words - h - 624 (q - 1),
// stepped from the last substream window strictly before it (from `wins` when
// given — their first word's low bits are not exact, so at least one step).
void mt_final_state(const uint32_t* state, int idx, uint64_t words, const uint32_t* wins, uint64_t subs,
                    uint32_t* fin, int32_t* fidx) {
  const uint64_t h = static_cast<uint64_t>(kMtN - idx);
  if (words <= h) {
    std::memcpy(fin, state, kMtN * sizeof(uint32_t));
    *fidx = idx + static_cast<int32_t>(words);
    return;
  }
  const uint64_t m_end = words - h, q = (m_end + kMtN - 1) / kMtN, tf = kMtN * q + h;
  uint64_t sig = (tf - 1) / kMtJumpL;
  if (wins && sig > subs - 1) sig = subs - 1;
  std::vector<uint32_t> w(kMtN);
  uint64_t t_sig = h;
  if (sig == 0) {
    std::memcpy(w.data(), state, kMtN * sizeof(uint32_t));
  } else if (wins) {
    std::memcpy(w.data(), wins + sig * kMtN, kMtN * sizeof(uint32_t));
    t_sig = sig * kMtJumpL;
  } else {
    std::vector<uint32_t> w1(kMtN);
    mt_window1(state, idx, w1.data());
    mt_window_from1(w1.data(), sig - 1, w.data());
    t_sig = sig * kMtJumpL;
  }
  mt_advance(w.data(), tf - t_sig, fin);
  *fidx = static_cast<int32_t>(m_end - kMtN * (q - 1));
}

}  // namespace dn

using namespace dn;

extern "C" int dn_mt19937_skip(uint32_t* mt_state, int32_t* mt_index, uint64_t words) {
  if (!mt_state || !mt_index) return set_error(DN_ERR_ARG, "dn_mt19937_skip: null pointer");
  const int32_t idx = *mt_index;
  if (idx < 0 || idx > kMtN) return set_error(DN_ERR_ARG, "dn_mt19937_skip: bad MT index");
  std::vector<uint32_t> fin(kMtN);
  int32_t fidx = 0;
  mt_final_state(mt_state, idx, words, nullptr, 0, fin.data(), &fidx);
  std::memcpy(mt_state, fin.data(), kMtN * sizeof(uint32_t));
  *mt_index = fidx;
  return DN_OK;
}
