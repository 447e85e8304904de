// m521_device.hpp — in-lane multi-limb arithmetic mod p = 2^521 - 1 (gfx950).
//
// One field element per lane, 17 little-endian u32 limbs held in VGPRs.
// Values are kept "lazy" (any integer < 2^544 that fits the 17 limbs) between
// operations and brought to the canonical residue in [0, p) only before a
// store, using the Mersenne identity 2^521 == 1 (mod p): reduction is a
// shift + add (fold), never a division.  This restates the `% prime` steps of
// the reference's `_eval_at` (delta_node/crypto/shamir/shamir.py:19-25) and
// the `% self.prime` / `div_mod` of `resolve_shares` (shamir.py:86-90).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dn {

constexpr int kLimbs = 17;
constexpr uint32_t kTopMask = 0x1FFu;  // bits 512..520 live in limb 16
constexpr int kTile = 256;             // elements per layout tile
constexpr uint64_t kTileBytes = 66ull * kTile;
constexpr uint64_t kHiOffset = 64ull * kTile;  // byte offset of the u16 plane

// ---- tiled-layout addressing (see include/dn_shamir.h) --------------------
// Every wave works on one tile at a time, so the tile base is wave-uniform
// (SGPRs) and each lane only adds a 32-bit offset: the loads/stores below
// compile to the saddr form `global_load_dword v, v_off, s[base:base+1] offset:imm`,
// which keeps per-limb 64-bit addresses out of the VGPR budget.
__device__ __forceinline__ const uint8_t* tile_base(const uint8_t* vec, uint32_t tile) {
  return vec + static_cast<uint64_t>(tile) * kTileBytes;
}
__device__ __forceinline__ uint8_t* tile_base(uint8_t* vec, uint32_t tile) {
  return vec + static_cast<uint64_t>(tile) * kTileBytes;
}

// Byte offsets are formed as u32 (w < 256) and added to a uniform per-limb
// pointer so that the compiler can use SGPR-base + VGPR-offset addressing.
template <typename T>
__device__ __forceinline__ const T* at(const uint8_t* base, uint32_t byte_off) {
  return reinterpret_cast<const T*>(base + byte_off);
}
template <typename T>
__device__ __forceinline__ T* at(uint8_t* base, uint32_t byte_off) {
  return reinterpret_cast<T*>(base + byte_off);
}

// Load element w (0..255) of the tile at `tb`.  The top limb is masked to 9 bits.
__device__ __forceinline__ void load_fe(const uint8_t* __restrict__ tb, uint32_t w, uint32_t v[kLimbs]) {
  const uint32_t o4 = w * 4u, o2 = w * 2u;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = __builtin_nontemporal_load(at<uint32_t>(tb + i * 4 * kTile, o4));
  v[16] = static_cast<uint32_t>(__builtin_nontemporal_load(at<uint16_t>(tb + kHiOffset, o2))) & kTopMask;
}

// Same, through the caches (data re-read by the generic split kernel).
__device__ __forceinline__ void load_fe_cached(const uint8_t* __restrict__ tb, uint32_t w, uint32_t v[kLimbs]) {
  const uint32_t o4 = w * 4u, o2 = w * 2u;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = *at<uint32_t>(tb + i * 4 * kTile, o4);
  v[16] = static_cast<uint32_t>(*at<uint16_t>(tb + kHiOffset, o2)) & kTopMask;
}

// Store a canonical element (write-once data: non-temporal stores).
__device__ __forceinline__ void store_fe(uint8_t* __restrict__ tb, uint32_t w, const uint32_t v[kLimbs]) {
  const uint32_t o4 = w * 4u, o2 = w * 2u;
#pragma unroll
  for (int i = 0; i < 16; ++i) __builtin_nontemporal_store(v[i], at<uint32_t>(tb + i * 4 * kTile, o4));
  __builtin_nontemporal_store(static_cast<uint16_t>(v[16]), at<uint16_t>(tb + kHiOffset, o2));
}

// ---- buffer-resource addressing (cdna guide T8/T20) --------------------------
// One 128-bit descriptor per (vector, tile), built from wave-uniform values in
// SGPRs; each lane then needs a single 32-bit VGPR offset (w * 4) for all 17
// limb accesses, the limb's byte offset riding in soffset.  aux = 2: nt.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int kNt = 2;

__device__ __forceinline__ rsrc_t tile_rsrc(const uint8_t* tb) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(tb), 0, static_cast<int>(kTileBytes), 0x00020000);
}

__device__ __forceinline__ void load_fe_b(rsrc_t r, uint32_t w, uint32_t v[kLimbs]) {
  const uint32_t o4 = w * 4u, o2 = w * 2u;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b32(r, o4, i * 4 * kTile, kNt);
  v[16] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b16(r, o2, static_cast<int>(kHiOffset), kNt)) &
          kTopMask;
}

template <int AUX = kNt>
__device__ __forceinline__ void store_fe_b(rsrc_t r, uint32_t w, const uint32_t v[kLimbs]) {
  const uint32_t o4 = w * 4u, o2 = w * 2u;
#pragma unroll
  for (int i = 0; i < 16; ++i) __builtin_amdgcn_raw_buffer_store_b32(v[i], r, o4, i * 4 * kTile, AUX);
  __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(v[16]), r, o2, static_cast<int>(kHiOffset), AUX);
}

// ---- carry chains ----------------------------------------------------------
// v += s (s a small u32), ripple through all limbs.
__device__ __forceinline__ void add_small(uint32_t v[kLimbs], uint32_t s) {
  unsigned c;
  v[0] = __builtin_addc(v[0], s, 0u, &c);
#pragma unroll
  for (int i = 1; i < kLimbs; ++i) v[i] = __builtin_addc(v[i], 0u, c, &c);
}

// v (< 2^521 + 2^23) -> canonical residue in [0, p).
//   top bit 521 set  => v - p = (v - 2^521) + 1, and v - 2^521 < 2^23 sits in limb 0;
//   v == p (all 521 bits set) => 0 (a branch no lane takes in practice).
__device__ __forceinline__ void canon(uint32_t v[kLimbs]) {
  const uint32_t top = v[16] >> 9;
  uint32_t a = v[0];
#pragma unroll
  for (int i = 1; i < 16; ++i) a &= v[i];
  const bool is_p = (a == 0xFFFFFFFFu) && (v[16] == kTopMask);
  v[16] &= kTopMask;
  v[0] += top;
  if (__builtin_expect(is_p, 0)) {
#pragma unroll
    for (int i = 0; i < kLimbs; ++i) v[i] = 0u;
  }
}

// Lazy v (< 2^544) -> canonical.  One fold (bits >= 521 added back at bit 0)
// leaves v < 2^521 + 2^23, then canon().  The fold's carry leaves limb 0 with
// probability < 2^-9 and canon() has work only when limb 16 >= 0x1FF (same
// odds), so both run behind branches that a wave skips unless one of its
// lanes needs them (s_cbranch_execz): ~4 VALU ops in the common case.
__device__ __forceinline__ void reduce(uint32_t v[kLimbs]) {
  const uint32_t hi = v[16] >> 9;
  v[16] &= kTopMask;
  unsigned c;
  v[0] = __builtin_addc(v[0], hi, 0u, &c);
  if (__builtin_expect(c != 0u, 0)) {
#pragma unroll
    for (int i = 1; i < kLimbs; ++i) v[i] = __builtin_addc(v[i], 0u, c, &c);
  }
  if (__builtin_expect(v[16] >= kTopMask, 0)) canon(v);
}

// Lazy fold only: v (< 2^544) -> v' == v (mod p), v' < 2^521 + 2^23.
__device__ __forceinline__ void fold(uint32_t v[kLimbs]) {
  const uint32_t hi = v[16] >> 9;
  v[16] &= kTopMask;
  add_small(v, hi);
}

// v += u (17-limb add; caller guarantees no carry out of limb 16).
__device__ __forceinline__ void add_fe(uint32_t v[kLimbs], const uint32_t u[kLimbs]) {
  unsigned c = 0u;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) v[i] = __builtin_addc(v[i], u[i], c, &c);
}

// D[k] += D[k+1] for k = 0..T-2 (one step of a forward-difference table),
// the T-1 carry chains interleaved limb by limb.  Each chain's carry lives in
// its own SGPR pair, so consecutive v_addc no longer depend on the carry the
// previous VALU wrote (gfx950 needs 2 wait states for that: `s_nop 1` per limb
// in a lone chain).  D[k+1] limb i is read before it is updated in the same
// limb step, so the interleaving preserves the semantics.
template <int T>
__device__ __forceinline__ void fd_step(uint32_t D[T][kLimbs]) {
  unsigned c[T > 1 ? T - 1 : 1];
#pragma unroll
  for (int k = 0; k + 1 < T; ++k) c[k] = 0u;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) {
#pragma unroll
    for (int k = 0; k + 1 < T; ++k) D[k][i] = __builtin_addc(D[k][i], D[k + 1][i], c[k], &c[k]);
  }
}

// Store f = D (lazy, < 2^544) as its canonical residue.  Common case (no
// carry out of limb 0 after the fold, limb 16 < 0x1FF): the residue is D with
// limb 0 += D >> 521 and limb 16 masked — stored straight from D's registers.
// If any lane of the wave needs more (odds ~2^-9 per lane), the whole wave
// reduces D IN PLACE (same residue, smaller value: later forward differences
// stay exact and within bounds) and stores it — no copy, no extra registers.
template <int AUX = kNt>
__device__ __forceinline__ void store_reduced(rsrc_t r, uint32_t w, uint32_t D[kLimbs]) {
  const uint32_t hi = D[16] >> 9;
  const uint32_t top = D[16] & kTopMask;
  unsigned c;
  const uint32_t l0 = __builtin_addc(D[0], hi, 0u, &c);
  const bool rare = (c != 0u) || (top == kTopMask);
  if (__builtin_expect(__ballot(rare) != 0ull, 0)) {
    reduce(D);
    store_fe_b<AUX>(r, w, D);
  } else {
    const uint32_t o4 = w * 4u, o2 = w * 2u;
    __builtin_amdgcn_raw_buffer_store_b32(l0, r, o4, 0, AUX);
#pragma unroll
    for (int i = 1; i < 16; ++i) __builtin_amdgcn_raw_buffer_store_b32(D[i], r, o4, i * 4 * kTile, AUX);
    __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(top), r, o2, static_cast<int>(kHiOffset), AUX);
  }
}

// v = src * x + c   (x < 2^16, caller guarantees the result < 2^544).
// Product limbs come from a v_mad_u64_u32 chain whose 64-bit addend carries
// only the previous high word; c is added by a separate v_addc chain.  (Folding
// c into the mad addend makes hipcc hoist 17 zero-extended {c_i, 0} pairs out
// of the share loop and doubles the register footprint.)
__device__ __forceinline__ void mul_small_add(uint32_t v[kLimbs], const uint32_t src[kLimbs], uint32_t x,
                                              const uint32_t c[kLimbs]) {
  uint32_t hi = 0u;
  unsigned cc = 0u;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) {
    const uint64_t t = static_cast<uint64_t>(src[i]) * x + hi;
    hi = static_cast<uint32_t>(t >> 32);
    v[i] = __builtin_addc(static_cast<uint32_t>(t), c[i], cc, &cc);
  }
}
__device__ __forceinline__ void mul_small_add(uint32_t v[kLimbs], uint32_t x, const uint32_t c[kLimbs]) {
  mul_small_add(v, v, x, c);
}

// ---- forward differences (split) -------------------------------------------
// D = 2 * c (a one-bit left shift across limbs; c < 2^543 so no overflow).
// D may alias c: limb i reads c[i] and c[i-1] before either is overwritten.
__device__ __forceinline__ void twice(uint32_t D[kLimbs], const uint32_t c[kLimbs]) {
#pragma unroll
  for (int i = kLimbs - 1; i > 0; --i) D[i] = __builtin_amdgcn_alignbit(c[i], c[i - 1], 31);
  D[0] = c[0] << 1;
}

constexpr int64_t fd_factorial(int k) { return k <= 1 ? 1 : k * fd_factorial(k - 1); }

// In place, c becomes the forward-difference table of f at x = 1:
// synthetic division by (x - z) for z = 1..T-1 turns the monomial
// coefficients into Newton coefficients b_k on nodes 1, 2, ...
// (f = b0 + b1 (x-1) + b2 (x-1)(x-2) + ...), and Delta^k f(1) = k! b_k.
// Every step is c[j] += z * c[j+1] with a small constant z.
template <int T>
__device__ __forceinline__ void fd_init(uint32_t c[T][kLimbs]) {
  if constexpr (T == 3) {
    // hand-ordered for the headline t = 3 (58 VGPRs, 8 waves/SIMD):
    // D2 = 2 c2; c2 <- c1 + c2; c1 <- c2 + D2 (= c1 + 3 c2); c2 <- c2 + c0.
    // (c0 is added last: an int64 secret is 2 live limbs until then.)
    uint32_t d2[kLimbs];
    twice(d2, c[2]);
    add_fe(c[2], c[1]);
#pragma unroll
    for (int i = 0; i < kLimbs; ++i) c[1][i] = c[2][i];
    add_fe(c[1], d2);
    add_fe(c[2], c[0]);
#pragma unroll
    for (int i = 0; i < kLimbs; ++i) {
      c[0][i] = c[2][i];
      c[2][i] = d2[i];
    }
  } else {
#pragma unroll
    for (int k = 0; k + 1 < T; ++k) {
#pragma unroll
      for (int j = T - 2; j >= k; --j) {
        if (k == 0) add_fe(c[j], c[j + 1]);
        else mul_small_add(c[j], c[j + 1], static_cast<uint32_t>(k + 1), c[j]);
      }
    }
    if constexpr (T >= 3) {
#pragma unroll
      for (int k = 2; k < T; ++k) {
        uint32_t zero[kLimbs];
#pragma unroll
        for (int i = 0; i < kLimbs; ++i) zero[i] = 0u;
        mul_small_add(c[k], c[k], static_cast<uint32_t>(fd_factorial(k)), zero);
      }
    }
  }
}

// ---- wide accumulators (reconstruct) --------------------------------------
// S[0..N) += a[0..A) * y[0..17)   (schoolbook).  FRESH: S was zero before the
// call, so limb j+17 is still untouched when row j ends and takes the carry
// directly; otherwise each row's carry ripples to the top limb.
template <int N, int A, bool FRESH = false>
__device__ __forceinline__ void mac_wide(uint32_t S[N], const uint32_t* a, const uint32_t y[kLimbs]) {
#pragma unroll
  for (int j = 0; j < A; ++j) {
    const uint32_t aj = a[j];
    uint64_t carry = 0;
#pragma unroll
    for (int l = 0; l < kLimbs; ++l) {
      const uint64_t t = static_cast<uint64_t>(aj) * y[l] + (static_cast<uint64_t>(S[j + l]) + carry);
      S[j + l] = static_cast<uint32_t>(t);
      carry = t >> 32;
    }
    if constexpr (FRESH) {
      if (j + kLimbs < N) S[j + kLimbs] = static_cast<uint32_t>(carry);
    } else {
      unsigned c;
      S[j + kLimbs] = __builtin_addc(S[j + kLimbs], static_cast<uint32_t>(carry), 0u, &c);
#pragma unroll
      for (int m = j + kLimbs + 1; m < N; ++m) S[m] = __builtin_addc(S[m], 0u, c, &c);
    }
  }
}

// N-limb S holding a value < 2^VALUE_BITS -> canonical 17-limb residue.
// One fold r = (S mod 2^521) + (S >> 521); VALUE_BITS <= 1064 keeps S >> 521
// below 2^543, so r < 2^544 fits 17 limbs (the limbs of S >> 521 beyond 17
// are zero by the value bound), then reduce().
template <int N, int VALUE_BITS>
__device__ __forceinline__ void reduce_wide(const uint32_t S[N], uint32_t r[kLimbs]) {
  static_assert(N > kLimbs && VALUE_BITS <= 32 * N && VALUE_BITS <= 1064, "reduce_wide bound");
  constexpr int H = (VALUE_BITS - 521 + 31) / 32;  // limbs of S >> 521 that can be non-zero
  static_assert(H <= kLimbs, "reduce_wide: high part wider than 17 limbs");
  unsigned c = 0;
#pragma unroll
  for (int m = 0; m < kLimbs; ++m) {
    uint32_t h = 0u;
    if (m < H) {
      h = S[16 + m] >> 9;
      if (16 + m + 1 < N) h |= S[16 + m + 1] << 23;
    }
    const uint32_t lo = (m < 16) ? S[m] : (S[16] & kTopMask);
    r[m] = __builtin_addc(lo, h, c, &c);
  }
  reduce(r);
}

// r = x * c mod p (c full width, uniform), canonical in and out.
__device__ __forceinline__ void mulmod(uint32_t r[kLimbs], const uint32_t x[kLimbs], const uint32_t* c) {
  uint32_t S[2 * kLimbs];
#pragma unroll
  for (int i = 0; i < 2 * kLimbs; ++i) S[i] = 0u;
  mac_wide<2 * kLimbs, kLimbs, true>(S, c, x);
  reduce_wide<2 * kLimbs, 1042>(S, r);
}

// x / 2^e mod p for canonical x, 1 <= e <= 31: a right rotation of the
// 521-bit string (2^521 == 1), which keeps the result canonical.
__device__ __forceinline__ void rotr521(uint32_t v[kLimbs], uint32_t e) {
  const uint32_t low = v[0] & ((1u << e) - 1u);
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = __builtin_amdgcn_alignbit(v[i + 1], v[i], e);
  v[16] >>= e;
  if (e <= 9) {
    v[16] |= low << (9u - e);
  } else {
    v[15] |= low << (41u - e);
    v[16] |= low >> (e - 9u);
  }
}

// x mod d for x < 2^64 and d < 2^32, with recip = floor((2^64-1)/d)
// (Barrett: the quotient estimate is low by at most one).
__device__ __forceinline__ uint32_t mod_small(uint64_t x, uint32_t d, uint64_t recip) {
  const uint64_t q = __umul64hi(x, recip);
  uint64_t r = x - q * d;
  if (r >= d) r -= d;
  return static_cast<uint32_t>(r);
}

// r / d mod p for canonical r and a small odd d (3 <= d < 2^16).
//   m = -r * p^{-1} mod d makes u = r + m*p divisible by d, and
//   u / d <= (d p - 1) / d < p, so the quotient is already canonical.
// u = r - m + m*2^521; the division runs LSB first (exact division, as in
// GMP's divexact_1): q_i = (u_i - borrow) * d^{-1} mod 2^32, borrow = hi(q_i d).
__device__ __forceinline__ void exact_div_small(uint32_t r[kLimbs], uint32_t d, uint32_t d_inv32, uint32_t p_inv_d,
                                                uint64_t recip, const uint32_t* w) {
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) acc += static_cast<uint64_t>(r[i]) * w[i];  // < 17 * 2^48
  const uint32_t rm = mod_small(acc, d, recip);
  const uint32_t neg_r = rm ? d - rm : 0u;
  const uint32_t m = mod_small(static_cast<uint64_t>(neg_r) * p_inv_d, d, recip);
  r[16] += m << 9;  // + m * 2^521
  unsigned b;
  r[0] = __builtin_subc(r[0], m, 0u, &b);  // - m
#pragma unroll
  for (int i = 1; i < kLimbs; ++i) r[i] = __builtin_subc(r[i], 0u, b, &b);
  uint32_t c = 0u;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) {
    const uint32_t s = r[i];
    const uint32_t x = s - c;
    const uint32_t q = x * d_inv32;
    c = __umulhi(q, d) + (x > s ? 1u : 0u);
    r[i] = q;
  }
}

}  // namespace dn
