// shamir_m521.hip — split / reconstruct kernels for gfx950 and their C-ABI.
//
// Split (reference: SecretShare.make_shares, delta_node/crypto/shamir/shamir.py:55-66,
// with _eval_at :19-25): per element, Horner evaluation of
//   f(x) = c0 + c1 x + ... + c_{t-1} x^{t-1}  at x = 1..n, mod p = 2^521 - 1.
// Reconstruct (reference: SecretShare.resolve_shares, shamir.py:68-90):
//   f(0) = sum_i lambda_i y_i mod p over ALL k given shares.
//
// Mapping: one wave owns one 256-element layout tile at a time (grid-stride
// over tiles); lane l handles tile elements l, l+64, l+128, l+192 in turn,
// one element per lane, all 17 limbs in VGPRs.  Every global access of a
// wave-instruction is one contiguous 256-byte (u32 plane) or 128-byte (u16
// plane) run.  Inputs are read once and shares written once, so loads and
// stores are non-temporal.  The path is HBM-bound: no MFMA (this is not a
// contraction), only v_mad_u64_u32 / v_add_co chains in the VALU.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "chacha_device.hpp"
#include "dn_internal.hpp"
#include "m521_device.hpp"

namespace dn {

struct SplitArgs {
  const int64_t* sec_u64;  // int64 secrets (u64 two's-complement view), or null
  const uint8_t* sec_fe;   // tiled field-element secrets, or null
  const uint8_t* coeffs;   // block of t-1 tiled vectors
  uint8_t* shares;         // block of n tiled vectors
  uint64_t n_elem;
  uint64_t ntiles;
  uint64_t vec_bytes;
  uint64_t coeff_stride;  // bytes between coefficient rows (>= vec_bytes)
  uint64_t share_stride;  // bytes between share rows (>= vec_bytes)
  uint32_t tile_map;      // wave_sched mode (0 cyclic, 1 XCD, 2 blocked, 3 coop)
  int32_t n_shares;
  int32_t threshold;  // runtime t (generic kernel only)
  uint64_t elem_offset;  // PRNG coefficients: global index of element 0 (multiple of 256)
  ChachaKey key;         // PRNG coefficients: key, nonce, rounds
};

constexpr int kBlock = 256;  // 4 waves
constexpr int kWavesPerBlock = kBlock / 64;
constexpr uint32_t kXcds = 8;

// Which tiles (and which 64-element quarters q of each tile) a wave works.
// Workgroups are dispatched to the 8 XCDs round-robin (XCD = blockIdx % 8).
//   0 cyclic:  wave w takes tiles w, w + W, w + 2W, ... (W waves), all 4 quarters;
//   1 XCD:     as 0, renumbered so that XCD x works the x-th contiguous eighth
//              of each grid-stride pass (8x smaller footprint per XCD L2);
//   2 blocked: wave w takes the contiguous run of tiles [w P, (w + 1) P);
//   3 coop:    workgroup b takes tiles b, b + G, ...; its wave i quarter i, so
//              the 4 waves write each 1-KB plane row of a tile together.
struct WaveSched {
  uint32_t first, step, end, q0, q1;
};

__device__ __forceinline__ WaveSched wave_sched(uint32_t map, uint64_t ntiles64) {
  const uint32_t ntiles = static_cast<uint32_t>(ntiles64);
  const uint32_t wib = threadIdx.x >> 6;
  uint32_t b = blockIdx.x;
  WaveSched s{0u, 1u, ntiles, 0u, 4u};
  if (map == 3u) {
    s.first = b;
    s.step = gridDim.x;
    s.q0 = wib;
    s.q1 = wib + 1u;
  } else if (map == 2u) {
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    const uint32_t per = (ntiles + nw - 1u) / nw;
    const uint32_t w = b * kWavesPerBlock + wib;
    s.first = w * per;
    s.end = s.first + per < ntiles ? s.first + per : ntiles;
  } else {
    if (map == 1u) b = (b % kXcds) * (gridDim.x / kXcds) + b / kXcds;
    s.first = b * kWavesPerBlock + wib;
    s.step = gridDim.x * kWavesPerBlock;
  }
  s.first = __builtin_amdgcn_readfirstlane(s.first);
  s.step = __builtin_amdgcn_readfirstlane(s.step);
  s.end = __builtin_amdgcn_readfirstlane(s.end);
  s.q0 = __builtin_amdgcn_readfirstlane(s.q0);
  s.q1 = __builtin_amdgcn_readfirstlane(s.q1);
  return s;
}

template <bool FE_SECRET>
__device__ __forceinline__ void load_secret(const SplitArgs& a, uint32_t tile, uint32_t w, uint32_t c0[kLimbs]) {
  if constexpr (FE_SECRET) {
    load_fe_b(tile_rsrc(tile_base(a.sec_fe, tile)), w, c0);
  } else {
    const int64_t* sec = a.sec_u64 + static_cast<uint64_t>(tile) * kTile;  // uniform base
    const uint64_t s = static_cast<uint64_t>(__builtin_nontemporal_load(sec + w));
    c0[0] = static_cast<uint32_t>(s);
    c0[1] = static_cast<uint32_t>(s >> 32);
#pragma unroll
    for (int i = 2; i < kLimbs; ++i) c0[i] = 0u;
  }
}


// T = compile-time threshold (1..8).
// FOLD == false: f(x) for x = 1..n by forward differences — the table
// D_k = Delta^k f(x) (built in place from the coefficients, below) advances
// with D_k += D_{k+1}: t-1 17-limb additions per share, no multiplies.  Every D_k stays a non-negative integer below
// 2^521 * sum_{j<t} (n+t)^j < 2^544 (checked on the host), so only the emitted
// f(x) is reduced.
// FOLD == true (large n or t): Horner per share (as _eval_at, shamir.py:19-25)
// with a Mersenne fold after every step.
//
// PRNG == true: coefficients are not read but generated (dn_m521_split_prng,
// chacha_device.hpp): per tile, the wave first computes the 16 (T-1) blocks
// holding the tile's top limbs (one block per lane) into its LDS slice, then
// each lane generates its element's T-1 low blocks in place in c[1..T-1].
// Tiles whose top-limb blocks one pass computes: 16 (T-1) blocks per tile,
// one per lane, so T = 2 and 3 take four and two tiles per pass (every lane
// busy) instead of leaving 48 or 32 lanes idle.  DN_PRNG_TP=0 (variant
// build): one tile per pass.
#ifndef DN_PRNG_TP
#define DN_PRNG_TP 1
#endif
__host__ __device__ constexpr int prng_tiles_per_pass(int t) {
  return (DN_PRNG_TP && 16 * (t - 1) < 64) ? 64 / (16 * (t - 1)) : 1;
}

// Top-limb blocks of tiles tile0, tile0 + step, ... (TP of them, those below
// end) into the wave's LDS slice: tile k's at tops + 256 (T-1) k.
template <int T, int TP>
__device__ __forceinline__ void prng_tile_tops(const SplitArgs& a, uint32_t tile0, uint32_t step, uint32_t end,
                                               uint32_t lane, uint32_t* tops) {
  constexpr uint32_t kBlocks = 16u * (T - 1);  // 256 (T-1) top words per tile
  __builtin_amdgcn_wave_barrier();  // previous tiles' reads are done
#pragma unroll 1
  for (uint32_t b = lane; b < kBlocks * TP; b += 64u) {
    const uint32_t k = b / kBlocks, bb = b - k * kBlocks;
    const uint32_t tile = tile0 + k * step;
    if (tile >= end) continue;
    const uint64_t g0 = a.elem_offset + static_cast<uint64_t>(tile) * kTile;
    uint32_t x[16];
    chacha_block(x, a.key, kTopDomain + g0 * (T - 1) / 16u + bb);
#pragma unroll
    for (int i = 0; i < 16; ++i) tops[b * 16u + i] = x[i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int T>
__device__ __forceinline__ void prng_coeffs_of(const SplitArgs& a, uint32_t tile, uint32_t w, const uint32_t* tops,
                                               uint32_t c[T][kLimbs]) {
  const uint64_t g = a.elem_offset + static_cast<uint64_t>(tile) * kTile + w;
#pragma unroll
  for (int j = 1; j < T; ++j) {
    const uint64_t i = g * (T - 1) + (j - 1);
    chacha_block(c[j], a.key, i);
    c[j][16] = tops[w * (T - 1) + (j - 1)] & kTopMask;
    if (__builtin_expect(prng_rejected(c[j]), 0)) prng_retry(c[j], a.key, i);
    add_small(c[j], 1u);
  }
}

constexpr int kMaxPrngT = 8;

// DN_SPLIT_PF (variant builds): the next quarter's loads ahead of the current
// quarter's stores (explicit coefficients, difference table) — neutral to
// 1 % slower on the headline (9.06-9.13 vs 9.10-9.18e9 elements/s,
// profiles/r05/aj/): the split already runs at ~0.97 of its ceiling
#ifndef DN_SPLIT_PF
#define DN_SPLIT_PF 0
#endif
template <int T, bool FE_SECRET, bool FOLD, bool PRNG, int SAUX>
__device__ __forceinline__ void split_body(const SplitArgs& a) {
  const uint32_t lane = threadIdx.x & 63u;
  const WaveSched ws = wave_sched(a.tile_map, a.ntiles);
  static_assert(!PRNG || (T >= 2 && !FE_SECRET), "PRNG coefficients: u64 secrets, t >= 2");
  // PRNG: per-wave slice of the top-limb words of TP tiles
  constexpr int TP = PRNG ? prng_tiles_per_pass(T) : 1;
  __shared__ uint32_t s_tops[PRNG ? kWavesPerBlock : 1][PRNG ? 256 * (T - 1) * TP : 1];
  uint32_t* tops = s_tops[PRNG ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0];
  for (uint32_t tile0 = ws.first; tile0 < ws.end; tile0 += ws.step * TP) {
    if constexpr (PRNG) prng_tile_tops<T, TP>(a, tile0, ws.step, ws.end, lane, tops);
#pragma unroll 1
    for (int k = 0; k < TP; ++k) {
    const uint32_t tile = tile0 + static_cast<uint32_t>(k) * ws.step;
    if (tile >= ws.end) break;
#if DN_SPLIT_PF
    if constexpr (!PRNG && !FOLD) {
      // a whole tile's four quarters: quarter q + 1's coefficients and secret
      // loaded before quarter q's share stores
      if (ws.q0 == 0u && ws.q1 == 4u && (static_cast<uint64_t>(tile) + 1u) * kTile <= a.n_elem) {
        uint32_t cq[2][T][kLimbs];
        auto load_q = [&](uint32_t w, uint32_t (&cc)[T][kLimbs]) {
#pragma unroll
          for (int j = 1; j < T; ++j)
            load_fe_b(tile_rsrc(tile_base(a.coeffs + static_cast<uint64_t>(j - 1) * a.coeff_stride, tile)), w, cc[j]);
          load_secret<FE_SECRET>(a, tile, w, cc[0]);
        };
        load_q(lane, cq[0]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (q < 3) load_q(lane + 64u * static_cast<uint32_t>(q + 1), cq[(q + 1) & 1]);
          const uint32_t w = lane + 64u * static_cast<uint32_t>(q);
          uint32_t (&D)[T][kLimbs] = cq[q & 1];
          fd_init<T>(D);
#pragma unroll 1
          for (int32_t xi = 1; xi <= a.n_shares; ++xi) {
            store_reduced<SAUX>(tile_rsrc(tile_base(a.shares + static_cast<uint64_t>(xi - 1) * a.share_stride, tile)),
                                w, D[0]);
            fd_step<T>(D);
          }
        }
        continue;
      }
    }
#endif
#pragma unroll 1
    for (uint32_t q = ws.q0; q < ws.q1; ++q) {
      const uint32_t w = lane + 64u * q;
      const uint64_t e = static_cast<uint64_t>(tile) * kTile + w;
      if (e >= a.n_elem) break;
      uint32_t c[T][kLimbs];
      if constexpr (PRNG) {
        prng_coeffs_of<T>(a, tile, w, tops + 256u * (T - 1) * static_cast<uint32_t>(k), c);
      } else {
#pragma unroll
        for (int j = 1; j < T; ++j)
          load_fe_b(tile_rsrc(tile_base(a.coeffs + static_cast<uint64_t>(j - 1) * a.coeff_stride, tile)), w, c[j]);
      }
      load_secret<FE_SECRET>(a, tile, w, c[0]);
      if constexpr (!FOLD) {
        fd_init<T>(c);
        uint32_t (&D)[T][kLimbs] = c;
#pragma unroll 1
        for (int32_t xi = 1; xi <= a.n_shares; ++xi) {
          store_reduced<SAUX>(tile_rsrc(tile_base(a.shares + static_cast<uint64_t>(xi - 1) * a.share_stride, tile)), w,
                              D[0]);
          fd_step<T>(D);
        }
      } else {
#pragma unroll 1
        for (int32_t xi = 1; xi <= a.n_shares; ++xi) {
          const uint32_t x = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(xi));
          uint32_t v[kLimbs];
          if constexpr (T == 1) {
#pragma unroll
            for (int i = 0; i < kLimbs; ++i) v[i] = c[0][i];
          } else {
            mul_small_add(v, c[T - 1], x, c[T - 2]);
            if constexpr (T > 2) fold(v);
#pragma unroll
            for (int j = T - 3; j >= 0; --j) {
              mul_small_add(v, x, c[j]);
              if (j > 0) fold(v);
            }
          }
          reduce(v);
          store_fe_b(tile_rsrc(tile_base(a.shares + static_cast<uint64_t>(xi - 1) * a.share_stride, tile)), w, v);
        }
      }
    }
    }
  }
}

template <int T, bool FE_SECRET, bool FOLD, bool PRNG = false, int SAUX = kNt>
__global__ void __launch_bounds__(kBlock) split_kernel(const SplitArgs a) {
  split_body<T, FE_SECRET, FOLD, PRNG, SAUX>(a);
}

// The device-PRNG split, register-limited to DN_PRNG_WAVES waves per SIMD
// (80 VGPRs at 6): its ChaCha rounds are dependent VALU chains that need the
// waves to hide their latency.
#ifndef DN_PRNG_WAVES
#define DN_PRNG_WAVES 6
#endif
template <int T, bool FOLD>
__global__ void __launch_bounds__(kBlock, DN_PRNG_WAVES) split_prng_kernel(const SplitArgs a) {
  split_body<T, false, FOLD, true, kNt>(a);
}

// ---- wide-access difference-table split ------------------------------------
// E consecutive elements per lane (E = 2 or 4): lane l of a wave holds tile
// elements w0 .. w0 + E - 1 with w0 = 64 E g + E l for group g of the tile, so
// every limb-plane access is one E*4-byte vector per lane and one contiguous
// 256 E-byte run per wave-instruction (E = 4: a whole 1-KB plane row of the
// tile, b128; the u16 top plane b64).  A share of a tile is 17 store
// instructions instead of 68.  The arithmetic is split_kernel<T, false,
// false>'s, per element.  A partial last tile takes the one-element path.
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int E>
__device__ __forceinline__ void load_planes_wide(rsrc_t r, uint32_t o4, uint32_t c[E][kLimbs]) {
  static_assert(E == 2 || E == 4, "E");
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if constexpr (E == 4) {
      const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, o4, i * 4 * kTile, kNt);
      c[0][i] = v.x, c[1][i] = v.y, c[2][i] = v.z, c[3][i] = v.w;
    } else {
      const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, o4, i * 4 * kTile, kNt);
      c[0][i] = v.x, c[1][i] = v.y;
    }
  }
  const int ho = static_cast<int>(kHiOffset);
  if constexpr (E == 4) {
    const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, o4 >> 1, ho, kNt);
    c[0][16] = v.x & kTopMask, c[1][16] = (v.x >> 16) & kTopMask;
    c[2][16] = v.y & kTopMask, c[3][16] = (v.y >> 16) & kTopMask;
  } else {
    const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(r, o4 >> 1, ho, kNt);
    c[0][16] = v & kTopMask, c[1][16] = (v >> 16) & kTopMask;
  }
}

// Store f = D (lazy, < 2^544) of E elements as canonical residues (as
// store_reduced, for E elements at once: if any lane of the wave needs more
// than the one-limb fold, the whole wave reduces its D in place).
template <int T, int E>
__device__ __forceinline__ void store_reduced_wide(rsrc_t r, uint32_t o4, uint32_t D[E][T][kLimbs]) {
  uint32_t l0[E], top[E];
  bool rare = false;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    unsigned c;
    top[e] = D[e][0][16] & kTopMask;
    l0[e] = __builtin_addc(D[e][0][0], D[e][0][16] >> 9, 0u, &c);
    rare |= (c != 0u) || (top[e] == kTopMask);
  }
  if (__builtin_expect(__ballot(rare) != 0ull, 0)) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      reduce(D[e][0]);
      l0[e] = D[e][0][0];
      top[e] = D[e][0][16];
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if constexpr (E == 4) {
      u32x4_t v;
      v.x = i ? D[0][0][i] : l0[0], v.y = i ? D[1][0][i] : l0[1];
      v.z = i ? D[2][0][i] : l0[2], v.w = i ? D[3][0][i] : l0[3];
      __builtin_amdgcn_raw_buffer_store_b128(v, r, o4, i * 4 * kTile, kNt);
    } else {
      u32x2_t v;
      v.x = i ? D[0][0][i] : l0[0], v.y = i ? D[1][0][i] : l0[1];
      __builtin_amdgcn_raw_buffer_store_b64(v, r, o4, i * 4 * kTile, kNt);
    }
  }
  const int ho = static_cast<int>(kHiOffset);
  if constexpr (E == 4) {
    u32x2_t v;
    v.x = top[0] | (top[1] << 16), v.y = top[2] | (top[3] << 16);
    __builtin_amdgcn_raw_buffer_store_b64(v, r, o4 >> 1, ho, kNt);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(top[0] | (top[1] << 16), r, o4 >> 1, ho, kNt);
  }
}

template <int T, int E>
__global__ void __launch_bounds__(kBlock) split_wide_kernel(const SplitArgs a) {
  static_assert(T >= 2 && (E == 2 || E == 4), "wide split: t >= 2, E = 2 or 4");
  constexpr uint32_t kGroups = kTile / (64 * E);
  const uint32_t lane = threadIdx.x & 63u;
  const WaveSched ws = wave_sched(a.tile_map == 3u ? 0u : a.tile_map, a.ntiles);
  for (uint32_t tile = ws.first; tile < ws.end; tile += ws.step) {
    if (static_cast<uint64_t>(tile + 1) * kTile > a.n_elem) {
      // partial last tile: one element per lane (split_kernel's path)
#pragma unroll 1
      for (uint32_t q = 0; q < 4u; ++q) {
        const uint32_t w = lane + 64u * q;
        if (static_cast<uint64_t>(tile) * kTile + w >= a.n_elem) break;
        uint32_t c[T][kLimbs];
#pragma unroll
        for (int j = 1; j < T; ++j)
          load_fe_b(tile_rsrc(tile_base(a.coeffs + static_cast<uint64_t>(j - 1) * a.coeff_stride, tile)), w, c[j]);
        load_secret<false>(a, tile, w, c[0]);
        fd_init<T>(c);
#pragma unroll 1
        for (int32_t xi = 1; xi <= a.n_shares; ++xi) {
          store_reduced(tile_rsrc(tile_base(a.shares + static_cast<uint64_t>(xi - 1) * a.share_stride, tile)), w, c[0]);
          fd_step<T>(c);
        }
      }
      continue;
    }
#pragma unroll 1
    for (uint32_t g = 0; g < kGroups; ++g) {
      const uint32_t w0 = 64u * E * g + E * lane;
      const uint32_t o4 = 4u * w0;
      uint32_t c[E][T][kLimbs];
#pragma unroll
      for (int j = 1; j < T; ++j) {
        uint32_t cj[E][kLimbs];
        load_planes_wide<E>(tile_rsrc(tile_base(a.coeffs + static_cast<uint64_t>(j - 1) * a.coeff_stride, tile)), o4,
                            cj);
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
          for (int i = 0; i < kLimbs; ++i) c[e][j][i] = cj[e][i];
      }
      {
        const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<int64_t*>(a.sec_u64 + static_cast<uint64_t>(tile) * kTile), 0, kTile * 8, 0x00020000);
#pragma unroll
        for (int h = 0; h < E / 2; ++h) {
          const u32x4_t s = __builtin_amdgcn_raw_buffer_load_b128(rs, 8u * w0 + 16u * h, 0, kNt);
          c[2 * h][0][0] = s.x, c[2 * h][0][1] = s.y;
          c[2 * h + 1][0][0] = s.z, c[2 * h + 1][0][1] = s.w;
        }
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
          for (int i = 2; i < kLimbs; ++i) c[e][0][i] = 0u;
      }
#pragma unroll
      for (int e = 0; e < E; ++e) fd_init<T>(c[e]);
#pragma unroll 1
      for (int32_t xi = 1; xi <= a.n_shares; ++xi) {
        store_reduced_wide<T, E>(
            tile_rsrc(tile_base(a.shares + static_cast<uint64_t>(xi - 1) * a.share_stride, tile)), o4, c);
#pragma unroll
        for (int e = 0; e < E; ++e) fd_step<T>(c[e]);
      }
    }
  }
}

// Generic threshold (any t <= 64): coefficients are re-read per share through
// the caches instead of being held in registers; always folds.
template <bool FE_SECRET>
__global__ void __launch_bounds__(kBlock) split_kernel_generic(const SplitArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const WaveSched ws = wave_sched(a.tile_map, a.ntiles);
  for (uint32_t tile = ws.first; tile < ws.end; tile += ws.step) {
#pragma unroll 1
    for (uint32_t q = ws.q0; q < ws.q1; ++q) {
      const uint32_t w = lane + 64u * q;
      const uint64_t e = static_cast<uint64_t>(tile) * kTile + w;
      if (e >= a.n_elem) break;
      uint32_t c0[kLimbs];
      load_secret<FE_SECRET>(a, tile, w, c0);
#pragma unroll 1
      for (int32_t xi = 1; xi <= a.n_shares; ++xi) {
        const uint32_t x = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(xi));
        uint32_t v[kLimbs];
        load_fe_cached(tile_base(a.coeffs + static_cast<uint64_t>(a.threshold - 2) * a.coeff_stride, tile), w, v);
#pragma unroll 1
        for (int j = a.threshold - 3; j >= 0; --j) {
          uint32_t cj[kLimbs];
          load_fe_cached(tile_base(a.coeffs + static_cast<uint64_t>(j) * a.coeff_stride, tile), w, cj);
          mul_small_add(v, x, cj);
          fold(v);
        }
        mul_small_add(v, x, c0);
        reduce(v);
        store_fe(tile_base(a.shares + static_cast<uint64_t>(xi - 1) * a.share_stride, tile), w, v);
      }
    }
  }
}

// The PRNG coefficient stream written out as the tiled block a.coeffs
// (dn_m521_prng_coeffs): rows j-1 = coefficient j, same values split_prng uses.
template <int T>
__global__ void __launch_bounds__(kBlock) prng_coeffs_kernel(const SplitArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const WaveSched ws = wave_sched(a.tile_map, a.ntiles);
  constexpr int TP = prng_tiles_per_pass(T);
  __shared__ uint32_t s_tops[kWavesPerBlock][256 * (T - 1) * TP];
  uint32_t* tops = s_tops[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
  for (uint32_t tile0 = ws.first; tile0 < ws.end; tile0 += ws.step * TP) {
    prng_tile_tops<T, TP>(a, tile0, ws.step, ws.end, lane, tops);
#pragma unroll 1
    for (int k = 0; k < TP; ++k) {
      const uint32_t tile = tile0 + static_cast<uint32_t>(k) * ws.step;
      if (tile >= ws.end) break;
#pragma unroll 1
      for (uint32_t q = ws.q0; q < ws.q1; ++q) {
        const uint32_t w = lane + 64u * q;
        if (static_cast<uint64_t>(tile) * kTile + w >= a.n_elem) break;
        uint32_t c[T][kLimbs];
        prng_coeffs_of<T>(a, tile, w, tops + 256u * (T - 1) * static_cast<uint32_t>(k), c);
#pragma unroll
        for (int j = 1; j < T; ++j)
          store_fe_b(tile_rsrc(tile_base(const_cast<uint8_t*>(a.coeffs) + static_cast<uint64_t>(j - 1) * a.coeff_stride,
                                         tile)), w, c[j]);
      }
    }
  }
}

struct ReconArgs {
  const uint8_t* shares[DN_MAX_RESOLVE];
  uint8_t* out_fe;
  int64_t* out_u64;
  uint32_t* overflow;
  uint64_t n_elem;
  uint64_t ntiles;
  uint32_t tile_map;
  int32_t k;
  uint32_t neg;
  uint32_t shift;
  int32_t pad;
  uint32_t a[DN_MAX_RESOLVE][kLimbs];
  uint32_t inv[kLimbs];
  uint32_t d, d_inv32, p_inv_d, pad2;
  uint64_t d_recip;
  uint32_t w[kLimbs];
};

// A = limbs of |a_i| (1, 2 or 17).  S = sum_i |a_i| * (y_i or p - y_i) is
// accumulated unreduced in A + 17 limbs (value < 2^(521 + 32A + 4) for k <= 16;
// for A = 17, a_i < p so < 2^1046), reduced once, then divided by d
// (INV = 1: times d^{-1} mod p, a full product; INV = 2: exact division by a
// small odd d) and by 2^shift (a 521-bit rotation).
// K > 0: compile-time share count — all K*17 loads of an element are issued
// before the first multiply; K == 0: runtime count, one share at a time.
// S reduced, divided and stored for element w of the tile; returns whether
// the result is >= 2^64 (the overflow count).
template <int A, int INV>
__device__ __forceinline__ bool recon_finish(const ReconArgs& a, uint32_t tile, uint32_t w,
                                             uint32_t (&S)[A + kLimbs]) {
  constexpr int N = A + kLimbs;
  constexpr int VB = (A == kLimbs) ? 1046 : (521 + 32 * A + 4);
  uint32_t r[kLimbs];
  reduce_wide<N, VB>(S, r);
  if constexpr (INV == 1) {
    uint32_t t[kLimbs];
    mulmod(t, r, a.inv);
#pragma unroll
    for (int l = 0; l < kLimbs; ++l) r[l] = t[l];
  } else if constexpr (INV == 2) {
    exact_div_small(r, a.d, a.d_inv32, a.p_inv_d, a.d_recip, a.w);
  }
  if (a.shift != 0u) rotr521(r, a.shift);
  if (a.out_fe) store_fe(tile_base(a.out_fe, tile), w, r);
  if (a.out_u64) {
    const uint64_t lo = static_cast<uint64_t>(r[0]) | (static_cast<uint64_t>(r[1]) << 32);
    __builtin_nontemporal_store(static_cast<int64_t>(lo), a.out_u64 + static_cast<uint64_t>(tile) * kTile + w);
  }
  uint32_t hi_or = 0u;
#pragma unroll
  for (int l = 2; l < kLimbs; ++l) hi_or |= r[l];
  return hi_or != 0u;
}

// One element's S from its K loaded rows (K > 0), then recon_finish.
template <int A, int INV, int K>
__device__ __forceinline__ bool recon_rows(const ReconArgs& a, uint32_t tile, uint32_t w, uint32_t (&y)[K][kLimbs]) {
  uint32_t S[A + kLimbs];
#pragma unroll
  for (int i = 0; i < A + kLimbs; ++i) S[i] = 0u;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    if ((a.neg >> i) & 1u) {  // -y == p - y == ~y within 521 bits
#pragma unroll
      for (int l = 0; l < 16; ++l) y[i][l] = ~y[i][l];
      y[i][16] = (~y[i][16]) & kTopMask;
    }
    mac_wide<A + kLimbs, A>(S, a.a[i], y[i]);
  }
  return recon_finish<A, INV>(a, tile, w, S);
}

// DN_RECON_PF (default 1): a wave working a whole tile's four quarters loads
// quarter q + DN_RECON_PF's K rows before quarter q's arithmetic (164 VGPRs for K = 3,
// 3 waves per SIMD; capping it at 4 or 5 spills): the headline reconstruct
// 0.599-0.603 vs 0.611-0.616 ms (profiles/r05/ai/); two quarters ahead (212
// VGPRs) the same, 0.585-0.589 vs 0.564-0.591 ms (profiles/r05/an/).
#ifndef DN_RECON_PF
#define DN_RECON_PF 1
#endif

template <int A, int INV, int K>
__global__ void __launch_bounds__(kBlock) reconstruct_kernel(const ReconArgs a) {
  constexpr int N = A + kLimbs;
  const uint32_t lane = threadIdx.x & 63u;
  const WaveSched ws = wave_sched(a.tile_map, a.ntiles);
  for (uint32_t tile = ws.first; tile < ws.end; tile += ws.step) {
#if DN_RECON_PF
    if constexpr (K > 0) {
      if (ws.q0 == 0u && ws.q1 == 4u && (static_cast<uint64_t>(tile) + 1u) * kTile <= a.n_elem) {
        constexpr int D = DN_RECON_PF, B = D + 1;  // quarters loaded ahead, buffers
        uint32_t y[B][K][kLimbs];
#pragma unroll
        for (int p = 0; p < D; ++p)
#pragma unroll
          for (int i = 0; i < K; ++i) load_fe(tile_base(a.shares[i], tile), lane + 64u * p, y[p % B][i]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (q + D < 4) {
#pragma unroll
            for (int i = 0; i < K; ++i)
              load_fe(tile_base(a.shares[i], tile), lane + 64u * (q + D), y[(q + D) % B][i]);
          }
          const bool over = recon_rows<A, INV, K>(a, tile, lane + 64u * q, y[q % B]);
          if (a.overflow) {
            const uint64_t m = __ballot(over);
            if (lane == 0 && m) atomicAdd(a.overflow, static_cast<uint32_t>(__popcll(m)));
          }
        }
        continue;
      }
    }
#endif
#pragma unroll 1
    for (uint32_t q = ws.q0; q < ws.q1; ++q) {
      const uint32_t w = lane + 64u * q;
      const uint64_t e = static_cast<uint64_t>(tile) * kTile + w;
      const bool valid = e < a.n_elem;
      bool over = false;
      if (valid) {
        if constexpr (K > 0) {
          uint32_t y[K][kLimbs];
#pragma unroll
          for (int i = 0; i < K; ++i) load_fe(tile_base(a.shares[i], tile), w, y[i]);
          over = recon_rows<A, INV, K>(a, tile, w, y);
        } else {
          uint32_t S[N];
#pragma unroll
          for (int i = 0; i < N; ++i) S[i] = 0u;
#pragma unroll 1
          for (int32_t i = 0; i < a.k; ++i) {
            uint32_t y[kLimbs];
            load_fe(tile_base(a.shares[i], tile), w, y);
            if ((a.neg >> i) & 1u) {
#pragma unroll
              for (int l = 0; l < 16; ++l) y[l] = ~y[l];
              y[16] = (~y[16]) & kTopMask;
            }
            mac_wide<N, A>(S, a.a[i], y);
          }
          over = recon_finish<A, INV>(a, tile, w, S);
        }
      }
      if (a.overflow) {
        const uint64_t m = __ballot(over);
        if (lane == 0 && m) atomicAdd(a.overflow, static_cast<uint32_t>(__popcll(m)));
      }
      if (!valid) break;
    }
  }
}

// DN_RECON_UNROLL=0 selects the runtime-k kernel (A/B hook, read per call).
static bool recon_unroll() {
  const char* e = tune_env("DN_RECON_UNROLL");
  return !(e && e[0] == '0');
}

template <int A, int INV>
static void launch_recon_k(int k, dim3 g, hipStream_t s, const ReconArgs& a) {
  if constexpr (A == 1) {  // the unrolled share counts exist for one-limb weights only
    if (recon_unroll()) {
      switch (k) {
        case 2: hipLaunchKernelGGL((reconstruct_kernel<A, INV, 2>), g, dim3(kBlock), 0, s, a); return;
        case 3: hipLaunchKernelGGL((reconstruct_kernel<A, INV, 3>), g, dim3(kBlock), 0, s, a); return;
        case 4: hipLaunchKernelGGL((reconstruct_kernel<A, INV, 4>), g, dim3(kBlock), 0, s, a); return;
        case 5: hipLaunchKernelGGL((reconstruct_kernel<A, INV, 5>), g, dim3(kBlock), 0, s, a); return;
        default: break;
      }
    }
  }
  hipLaunchKernelGGL((reconstruct_kernel<A, INV, 0>), g, dim3(kBlock), 0, s, a);
}

// Compute units of the current device (cached per device id).
static int cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int v = cache[dev].load(std::memory_order_relaxed);
  if (v > 0) return v;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
  cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

// Workgroups per launch: each 4-wave workgroup strides over tiles.
// Default (reconstruct, compute-heavier splits): up to 16384 workgroups
// (2^24 elements: one tile per wave; 1-3 % ahead of 4096 on reconstruct,
// profiles/r01/tune_gridcap*.jsonl).  The write-dominated difference-table
// split uses one workgroup per CU (one wave per SIMD, 64 tiles per wave at
// 2^24): same time as the full grid where the share buffer's placement is
// fast, 4-5 % faster where it is slow (fewer writes in flight through the
// L2 / EA path; DESIGN.md §5.1, profiles/r01/placement/).
// DN_GRID_CAP overrides both (read per call; used by the tuning scripts).
static int grid_for(uint64_t ntiles, bool per_cu = false) {
  const char* s = tune_env("DN_GRID_CAP");
  const int v = s ? std::atoi(s) : 0;
  const uint64_t cap = v > 0 ? static_cast<uint64_t>(v) : per_cu ? static_cast<uint64_t>(cu_count()) : 16384u;
  const uint64_t blocks = (ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
  return static_cast<int>(blocks < cap ? blocks : cap);
}

// DN_TILE_MAP=0..3 selects the wave_sched mode (A/B hook, read per call);
// default 0.  Mode 1 needs grid % 8 == 0; the PRNG kernels (one wave per tile
// for the shared top-limb blocks) cannot use mode 3.
static uint32_t tile_map_for(int grid, bool allow_coop = true) {
  const char* s = tune_env("DN_TILE_MAP");
  const uint32_t m = (s && s[0] >= '0' && s[0] <= '3') ? static_cast<uint32_t>(s[0] - '0') : 0u;
  if (m == 1u && grid % static_cast<int>(kXcds) != 0) return 0u;
  if (m == 3u && !allow_coop) return 0u;
  return m;
}

static int check_launch(const char* what) {
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "%s: launch failed: %s", what, hipGetErrorString(err));
  return DN_OK;
}

template <bool FE_SECRET, bool FOLD>
static void launch_split_t(int t, dim3 g, hipStream_t s, const SplitArgs& a) {
  switch (t) {
    case 1: hipLaunchKernelGGL((split_kernel<1, FE_SECRET, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 2: hipLaunchKernelGGL((split_kernel<2, FE_SECRET, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 3: {
#ifdef DN_TUNING
      // DN_STORE_AUX (tuning build): cache policy bits of the share stores, headline kernel only
      const char* sa = (!FE_SECRET && !FOLD) ? tune_env("DN_STORE_AUX") : nullptr;
      const int aux = sa ? std::atoi(sa) : kNt;
      if (aux == 0) hipLaunchKernelGGL((split_kernel<3, FE_SECRET, FOLD, false, 0>), g, dim3(kBlock), 0, s, a);
      else if (aux == 1) hipLaunchKernelGGL((split_kernel<3, FE_SECRET, FOLD, false, 1>), g, dim3(kBlock), 0, s, a);
      else if (aux == 3) hipLaunchKernelGGL((split_kernel<3, FE_SECRET, FOLD, false, 3>), g, dim3(kBlock), 0, s, a);
      else if (aux == 16) hipLaunchKernelGGL((split_kernel<3, FE_SECRET, FOLD, false, 16>), g, dim3(kBlock), 0, s, a);
      else if (aux == 17) hipLaunchKernelGGL((split_kernel<3, FE_SECRET, FOLD, false, 17>), g, dim3(kBlock), 0, s, a);
      else if (aux == 18) hipLaunchKernelGGL((split_kernel<3, FE_SECRET, FOLD, false, 18>), g, dim3(kBlock), 0, s, a);
      else if (aux == 19) hipLaunchKernelGGL((split_kernel<3, FE_SECRET, FOLD, false, 19>), g, dim3(kBlock), 0, s, a);
      else
#endif
      hipLaunchKernelGGL((split_kernel<3, FE_SECRET, FOLD>), g, dim3(kBlock), 0, s, a);
      break;
    }
    case 4: hipLaunchKernelGGL((split_kernel<4, FE_SECRET, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 5: hipLaunchKernelGGL((split_kernel<5, FE_SECRET, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 6: hipLaunchKernelGGL((split_kernel<6, FE_SECRET, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 7: hipLaunchKernelGGL((split_kernel<7, FE_SECRET, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 8: hipLaunchKernelGGL((split_kernel<8, FE_SECRET, FOLD>), g, dim3(kBlock), 0, s, a); break;
    default: hipLaunchKernelGGL((split_kernel_generic<FE_SECRET>), g, dim3(kBlock), 0, s, a); break;
  }
}

// Elements per lane of the difference-table split with int64 secrets
// (0: the one-element split_kernel).  DN_SPLIT_E (tuning build) overrides.
// Measured (scripts/split_wide_probe.py, profiles/r02/split_wide.jsonl; the
// same three share allocations each): t = 3, n = 5 — one element per lane is
// fastest (1.48-1.49 ms at 2^24 vs 1.51-1.57 for E = 2 / 4, every grid cap),
// already at 98-101 % of the same-buffer 16-B streaming ceiling; t = 5, n = 9
// — E = 2 is 4.7 % faster where the share buffer's placement is fast (2.42 vs
// 2.54 ms) and within 1 % where it is slow.
static int split_wide_e(int t) {
  const char* e = tune_env("DN_SPLIT_E");
  if (e) return std::atoi(e);
  return t == 5 ? 2 : 0;
}

static bool launch_split_wide(int t, dim3 g, hipStream_t s, const SplitArgs& a) {
  const int E = split_wide_e(t);
  if (E == 4 && t == 3) hipLaunchKernelGGL((split_wide_kernel<3, 4>), g, dim3(kBlock), 0, s, a);
  else if (E == 2 && t == 3) hipLaunchKernelGGL((split_wide_kernel<3, 2>), g, dim3(kBlock), 0, s, a);
  else if (E == 2 && t == 5) hipLaunchKernelGGL((split_wide_kernel<5, 2>), g, dim3(kBlock), 0, s, a);
  else return false;
  return true;
}

template <bool FOLD>
static void launch_split_prng(int t, dim3 g, hipStream_t s, const SplitArgs& a) {
  switch (t) {
    case 2: hipLaunchKernelGGL((split_prng_kernel<2, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 3: hipLaunchKernelGGL((split_prng_kernel<3, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 4: hipLaunchKernelGGL((split_prng_kernel<4, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 5: hipLaunchKernelGGL((split_prng_kernel<5, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 6: hipLaunchKernelGGL((split_prng_kernel<6, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 7: hipLaunchKernelGGL((split_prng_kernel<7, FOLD>), g, dim3(kBlock), 0, s, a); break;
    case 8: hipLaunchKernelGGL((split_prng_kernel<8, FOLD>), g, dim3(kBlock), 0, s, a); break;
    default: break;
  }
}

static void launch_prng_coeffs(int t, dim3 g, hipStream_t s, const SplitArgs& a) {
  switch (t) {
    case 2: hipLaunchKernelGGL((prng_coeffs_kernel<2>), g, dim3(kBlock), 0, s, a); break;
    case 3: hipLaunchKernelGGL((prng_coeffs_kernel<3>), g, dim3(kBlock), 0, s, a); break;
    case 4: hipLaunchKernelGGL((prng_coeffs_kernel<4>), g, dim3(kBlock), 0, s, a); break;
    case 5: hipLaunchKernelGGL((prng_coeffs_kernel<5>), g, dim3(kBlock), 0, s, a); break;
    case 6: hipLaunchKernelGGL((prng_coeffs_kernel<6>), g, dim3(kBlock), 0, s, a); break;
    case 7: hipLaunchKernelGGL((prng_coeffs_kernel<7>), g, dim3(kBlock), 0, s, a); break;
    case 8: hipLaunchKernelGGL((prng_coeffs_kernel<8>), g, dim3(kBlock), 0, s, a); break;
    default: break;
  }
}

static int set_prng_key(SplitArgs& a, const uint32_t* key, uint64_t nonce, int rounds, uint64_t elem_offset,
                        const char* name) {
  if (!key) return set_error(DN_ERR_ARG, "%s: null key", name);
  if (!(rounds == 8 || rounds == 12 || rounds == 20))
    return set_error(DN_ERR_ARG, "%s: rounds must be 8, 12 or 20 (got %d)", name, rounds);
  if (elem_offset % kTile) return set_error(DN_ERR_ARG, "%s: elem_offset must be a multiple of %d", name, kTile);
  std::memcpy(a.key.k, key, sizeof(a.key.k));
  a.key.n0 = static_cast<uint32_t>(nonce);
  a.key.n1 = static_cast<uint32_t>(nonce >> 32);
  a.key.rounds = rounds;
  a.elem_offset = elem_offset;
  return DN_OK;
}

static int split_common(SplitArgs a, int threshold, int n_shares, void* stream, bool fe, const char* name,
                        bool prng = false) {
  if (threshold < 1 || threshold > DN_MAX_THRESHOLD)
    return set_error(DN_ERR_UNSUPPORTED, "%s: threshold %d outside 1..%d", name, threshold, DN_MAX_THRESHOLD);
  if (threshold > n_shares) return set_error(DN_ERR_THRESHOLD, "threshold should be little equal than shares");
  if (n_shares > DN_MAX_SHARES)
    return set_error(DN_ERR_UNSUPPORTED, "%s: %d shares > %d", name, n_shares, DN_MAX_SHARES);
  if (a.n_elem == 0) return DN_OK;
  if (prng && threshold > kMaxPrngT)
    return set_error(DN_ERR_UNSUPPORTED, "%s: threshold %d > %d", name, threshold, kMaxPrngT);
  if (!a.shares || (threshold > 1 && !prng && !a.coeffs) || (fe ? !a.sec_fe : !a.sec_u64))
    return set_error(DN_ERR_ARG, "%s: null pointer", name);
  a.ntiles = (a.n_elem + kTile - 1) / kTile;
  a.vec_bytes = a.ntiles * kTileBytes;
  // rows of the caller's [t-1, vec_bytes] / [n, vec_bytes] blocks are dense
  a.coeff_stride = a.vec_bytes;
  a.share_stride = a.vec_bytes;
  a.n_shares = n_shares;
  a.threshold = threshold;
  // DN_SPLIT_HORNER=1 forces the Horner kernel (A/B hook, read per call).
  const char* hz = tune_env("DN_SPLIT_HORNER");
  const bool fold_each = fd_needs_fold(threshold, n_shares) || (hz && hz[0] == '1');
  const bool per_cu = !prng && !fold_each && threshold <= 8;  // the memory-bound difference-table kernels
  // a PRNG wave takes its tiles prng_tiles_per_pass at a time
  const uint64_t tp = prng ? static_cast<uint64_t>(prng_tiles_per_pass(threshold)) : 1u;
  const dim3 g(grid_for((a.ntiles + tp - 1) / tp, per_cu));
  a.tile_map = tile_map_for(static_cast<int>(g.x), !prng);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (prng && threshold > 1) {
    if (fold_each) launch_split_prng<true>(threshold, g, s, a);
    else launch_split_prng<false>(threshold, g, s, a);
  } else if (fe) {
    if (fold_each) launch_split_t<true, true>(threshold, g, s, a);
    else launch_split_t<true, false>(threshold, g, s, a);
  } else if (!fold_each && launch_split_wide(threshold, g, s, a)) {
  } else {
    if (fold_each) launch_split_t<false, true>(threshold, g, s, a);
    else launch_split_t<false, false>(threshold, g, s, a);
  }
  return check_launch(name);
}

int device_cu_count() { return cu_count(); }

}  // namespace dn

using namespace dn;

extern "C" int dn_m521_split_u64(const int64_t* secrets, const void* coeffs, void* shares, uint64_t n_elem,
                                 int threshold, int n_shares, void* stream) {
  SplitArgs a{};
  a.sec_u64 = secrets;
  a.coeffs = static_cast<const uint8_t*>(coeffs);
  a.shares = static_cast<uint8_t*>(shares);
  a.n_elem = n_elem;
  return split_common(a, threshold, n_shares, stream, false, "dn_m521_split_u64");
}

extern "C" int dn_m521_split_prng(const int64_t* secrets, const uint32_t* key, uint64_t nonce, int rounds,
                                  uint64_t elem_offset, void* shares, uint64_t n_elem, int threshold, int n_shares,
                                  void* stream) {
  SplitArgs a{};
  const int rc = set_prng_key(a, key, nonce, rounds, elem_offset, "dn_m521_split_prng");
  if (rc != DN_OK) return rc;
  a.sec_u64 = secrets;
  a.shares = static_cast<uint8_t*>(shares);
  a.n_elem = n_elem;
  return split_common(a, threshold, n_shares, stream, false, "dn_m521_split_prng", true);
}

extern "C" int dn_m521_prng_coeffs(const uint32_t* key, uint64_t nonce, int rounds, uint64_t elem_offset,
                                   void* coeffs, uint64_t n_elem, int tm1, void* stream) {
  SplitArgs a{};
  const int rc = set_prng_key(a, key, nonce, rounds, elem_offset, "dn_m521_prng_coeffs");
  if (rc != DN_OK) return rc;
  if (tm1 < 1 || tm1 + 1 > kMaxPrngT)
    return set_error(DN_ERR_UNSUPPORTED, "dn_m521_prng_coeffs: %d coefficients outside 1..%d", tm1, kMaxPrngT - 1);
  if (n_elem == 0) return DN_OK;
  if (!coeffs) return set_error(DN_ERR_ARG, "dn_m521_prng_coeffs: null pointer");
  a.coeffs = static_cast<const uint8_t*>(coeffs);
  a.n_elem = n_elem;
  a.ntiles = (n_elem + kTile - 1) / kTile;
  a.vec_bytes = a.ntiles * kTileBytes;
  a.coeff_stride = a.vec_bytes;
  const uint64_t tp = static_cast<uint64_t>(prng_tiles_per_pass(tm1 + 1));
  const dim3 g(grid_for((a.ntiles + tp - 1) / tp));
  a.tile_map = tile_map_for(static_cast<int>(g.x), false);
  launch_prng_coeffs(tm1 + 1, g, static_cast<hipStream_t>(stream), a);
  return check_launch("dn_m521_prng_coeffs");
}

extern "C" int dn_m521_split_fe(const void* secrets_fe, const void* coeffs, void* shares, uint64_t n_elem,
                                int threshold, int n_shares, void* stream) {
  SplitArgs a{};
  a.sec_fe = static_cast<const uint8_t*>(secrets_fe);
  a.coeffs = static_cast<const uint8_t*>(coeffs);
  a.shares = static_cast<uint8_t*>(shares);
  a.n_elem = n_elem;
  return split_common(a, threshold, n_shares, stream, true, "dn_m521_split_fe");
}

extern "C" int dn_m521_reconstruct(const void* const* share_vecs, const dn_m521_lagrange_t* w, void* out_fe,
                                   int64_t* out_u64, uint32_t* overflow_count, uint64_t n_elem, void* stream) {
  if (!w || !share_vecs) return set_error(DN_ERR_ARG, "dn_m521_reconstruct: null pointer");
  if (w->k < 1 || w->k > DN_MAX_RESOLVE)
    return set_error(DN_ERR_UNSUPPORTED, "dn_m521_reconstruct: k=%d outside 1..%d", w->k, DN_MAX_RESOLVE);
  if (!(w->a_limbs == 1 || w->a_limbs == 2 || w->a_limbs == 17) || w->shift < 0 || w->shift > 31)
    return set_error(DN_ERR_ARG, "dn_m521_reconstruct: malformed weights");
  if (n_elem == 0) return DN_OK;
  if (!out_fe && !out_u64) return set_error(DN_ERR_ARG, "dn_m521_reconstruct: no output");
  ReconArgs a{};
  for (int i = 0; i < w->k; ++i) {
    if (!share_vecs[i]) return set_error(DN_ERR_ARG, "dn_m521_reconstruct: null share vector %d", i);
    a.shares[i] = static_cast<const uint8_t*>(share_vecs[i]);
  }
  a.out_fe = static_cast<uint8_t*>(out_fe);
  a.out_u64 = out_u64;
  a.overflow = overflow_count;
  a.n_elem = n_elem;
  a.ntiles = (n_elem + kTile - 1) / kTile;
  a.k = w->k;
  a.neg = w->neg;
  a.shift = static_cast<uint32_t>(w->shift);
  std::memcpy(a.a, w->a, sizeof(a.a));
  std::memcpy(a.inv, w->inv, sizeof(a.inv));
  const dim3 g(grid_for(a.ntiles));
  a.tile_map = tile_map_for(static_cast<int>(g.x));
  hipStream_t s = static_cast<hipStream_t>(stream);
  a.d = w->d;
  a.d_inv32 = w->d_inv32;
  a.p_inv_d = w->p_inv_d;
  a.d_recip = w->d_recip;
  std::memcpy(a.w, w->w, sizeof(a.w));
  const int inv = w->has_inv;
  if (inv < 0 || inv > 2 || (inv == 2 && (w->d < 3 || w->d >= 65536 || !(w->d & 1))))
    return set_error(DN_ERR_ARG, "dn_m521_reconstruct: malformed divisor");
#define DN_RECON(AL, IV) launch_recon_k<AL, IV>(w->k, g, s, a)
  switch (w->a_limbs * 4 + inv) {
    case 1 * 4 + 0: DN_RECON(1, 0); break;
    case 1 * 4 + 1: DN_RECON(1, 1); break;
    case 1 * 4 + 2: DN_RECON(1, 2); break;
    case 2 * 4 + 0: DN_RECON(2, 0); break;
    case 2 * 4 + 1: DN_RECON(2, 1); break;
    case 2 * 4 + 2: DN_RECON(2, 2); break;
    case 17 * 4 + 0: DN_RECON(17, 0); break;
    case 17 * 4 + 1: DN_RECON(17, 1); break;
    default: DN_RECON(17, 2); break;
  }
#undef DN_RECON
  return check_launch("dn_m521_reconstruct");
}
