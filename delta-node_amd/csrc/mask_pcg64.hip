// mask_pcg64.hip — secure-aggregation masks on gfx950: numpy's PCG64 stream
// and bounded-int64 (Lemire) draws, fused with fixed-point conversion and the
// signed sum over masks (reference: delta_node/utils/arr.py:20-28,
// utils/precision.py:5-15, runner/horizontal/agg.py:284-318).
//
// A raw draw r of a PCG64 generator is a pure function of (state, r): the
// LCG s' = a s + inc jumps ahead in closed form, s_r = A_r s_0 + inc G_r with
// A_r = a^r, G_r = 1 + a + ... + a^(r-1) (mod 2^128).  So lanes generate
// their elements independently: lane l of a wave owns elements
// e0 + l + 64 i and steps by 64 with the constant map (A_64, inc G_64).  A
// wave tile's start states cost ONE jump: lane g jumps generator g (all
// generators at once), each lane then applies its fixed T^lane.  Generators
// are sorted by sign on the host and drawn in pairs (two independent LCG
// chains per lane); make_mask's Lemire range 2^47 - 1 takes the product
// x (2^47 - 1) as a shift and a subtraction.  Consecutive lanes write
// consecutive int64s (512 B per wave store).  The output equals numpy's
// whenever no raw draw in the range is rejected by Lemire's test (odds 2^-47
// per draw for make_mask); every draw is tested and rejections are counted per
// generator, and the caller then replays that generator exactly with
// per-segment raw offsets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "dn_internal.hpp"
#include "dn_mask.h"
#include "pcg64_common.hpp"

namespace dn {

constexpr int kMaskBlock = 256;
constexpr int kDrawsPerLane = 8;                 // per chunk
constexpr int kChunkElems = 64 * kDrawsPerLane;  // 512
constexpr int kChunks = 8;
constexpr uint64_t kTileElems = kChunkElems * kChunks;  // 4096 per wave tile
constexpr int kMersK = 47;  // make_mask's integers(0, 2**47 - 1): Lemire range 2^47 - 1

struct AccArgs {
  int64_t* out;
  const int64_t* base_i64;
  const double* base_f64;
  double scale;
  uint64_t elem_begin, elem_end;
  uint64_t excl, threshold;
  uint64_t low_total;  // sum_g sign_g * low (mod 2^64), added once per element
  int32_t mers_k;      // excl == 2^mers_k - 1 (make_mask: 47), else 0 (general multiply)
  int32_t ngen;
  int32_t npos;                   // generators [0, npos) add, [npos, ngen) subtract
  int32_t orig[DN_MASK_MAX_GENS]; // caller's index of each (sign-sorted) generator
  uint64_t raw_off[DN_MASK_MAX_GENS];
  u128 state0[DN_MASK_MAX_GENS];  // state before raw draw 0 (draw r uses T^(r+1))
  u128 inc[DN_MASK_MAX_GENS];
  u128 c64[DN_MASK_MAX_GENS];     // inc * G_64
  u128 jA[64], jG[64];            // T^(2^k) = (A, G)
  u128 A64;
  uint32_t* rejects;
  u128 strideA, strideG;  // T^(nwaves * kChunkElems): a wave's step from one tile to its next (small tiles)
};

__device__ __forceinline__ uint64_t xsl_rr(u128 s) {
  const uint64_t hi = static_cast<uint64_t>(s >> 64), lo = static_cast<uint64_t>(s);
  const uint64_t x = hi ^ lo;
  const uint32_t rot = static_cast<uint32_t>(hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

// numpy's x86 float64 -> int64 cast: truncation, NaN / out of range -> INT64_MIN.
__device__ __forceinline__ int64_t f64_to_i64_x86(double x) {
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
  return static_cast<int64_t>(x);
}

__device__ __forceinline__ u128 bcast_u128(u128 v, int src) {  // v of lane `src` (wave-uniform src)
  const uint64_t lo = static_cast<uint64_t>(v), hi = static_cast<uint64_t>(v >> 64);
  const uint32_t w0 = __builtin_amdgcn_readlane(static_cast<uint32_t>(lo), src);
  const uint32_t w1 = __builtin_amdgcn_readlane(static_cast<uint32_t>(lo >> 32), src);
  const uint32_t w2 = __builtin_amdgcn_readlane(static_cast<uint32_t>(hi), src);
  const uint32_t w3 = __builtin_amdgcn_readlane(static_cast<uint32_t>(hi >> 32), src);
  return to_u128((static_cast<uint64_t>(w3) << 32) | w2, (static_cast<uint64_t>(w1) << 32) | w0);
}

// kDrawsPerLane draws of K generators (same sign) at stride 64 (lane-strided
// elements), accumulated into acc.  K = 2 interleaves two independent LCG
// chains for latency hiding.  Lemire's value is the high word of x * excl; for
// excl = 2^k - 1 that is x 2^k - x (shifts, no multiply).  The rejection test
// (low word < threshold) also covers draws past elem_end: a spurious hit (odds
// 2^-47 per draw) only sends the generator down the exact replay path.
// Returns bit j set if generator j saw a rejected draw.
template <bool MERS>
__device__ __forceinline__ uint64_t lemire_hi(const uint64_t x, const uint64_t excl, const uint64_t thr, bool& rj) {
  uint64_t lo, hi;
  if (MERS) {
    const uint64_t xs = x << kMersK;
    lo = xs - x;
    hi = (x >> (64 - kMersK)) - (xs < x ? 1u : 0u);
  } else {
    const u128 m = static_cast<u128>(x) * excl;
    lo = static_cast<uint64_t>(m);
    hi = static_cast<uint64_t>(m >> 64);
  }
  rj |= lo < thr;
  return hi;
}

template <bool MERS, bool NEG, int K>
__device__ __forceinline__ uint32_t draws_chunk(u128 (&st)[K], uint64_t (&acc)[kDrawsPerLane], const u128 A64,
                                                const u128 (&c64)[K], const uint64_t excl, const uint64_t thr) {
  bool rj[K];
#pragma unroll
  for (int j = 0; j < K; ++j) rj[j] = false;
#pragma unroll
  for (int i = 0; i < kDrawsPerLane; ++i) {
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      sum += lemire_hi<MERS>(xsl_rr(st[j]), excl, thr, rj[j]);
      st[j] = A64 * st[j] + c64[j];
    }
    acc[i] = NEG ? acc[i] - sum : acc[i] + sum;
  }
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) m |= rj[j] ? (1u << j) : 0u;
  return m;
}

// One step of the generator loop: generators [g, g + K) of one sign.
template <bool MERS, bool NEG, int K>
__device__ __forceinline__ uint32_t gens_step(const AccArgs& a, u128* s_state, const uint32_t tid, const int g,
                                              uint64_t (&acc)[kDrawsPerLane]) {
  u128 st[K], c[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    st[j] = s_state[(g + j) * kMaskBlock + tid];
    c[j] = a.c64[g + j];
  }
  const uint32_t m = draws_chunk<MERS, NEG, K>(st, acc, a.A64, c, a.excl, a.threshold);
#pragma unroll
  for (int j = 0; j < K; ++j) s_state[(g + j) * kMaskBlock + tid] = st[j];
  return m << g;
}

// Each lane keeps one PCG64 state per generator in LDS between chunks (16 B
// per lane per generator, wave-private slots, no barrier; dynamic LDS sized by
// ngen).  A tile's start states come from ONE lane-parallel jump: lane g < ngen
// jumps generator g to the tile start (all generators' jumps in the time of
// one), each lane then offsets itself by its fixed T^lane.
template <bool MERS>
__global__ void __launch_bounds__(kMaskBlock) bounded_acc_kernel(const AccArgs a) {
  extern __shared__ u128 s_state[];  // [ngen][kMaskBlock]
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint64_t n = a.elem_end - a.elem_begin;
  const uint64_t ntiles = (n + kTileElems - 1) / kTileElems;
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kMaskBlock / 64);
  const uint64_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * (kMaskBlock / 64) + (tid >> 6));
  uint32_t rejmask = 0u;  // bit g: this lane saw a rejected draw of generator g
  for (uint64_t tile = wave0; tile < ntiles; tile += nwaves) {
    const uint64_t e0 = a.elem_begin + tile * kTileElems;  // wave-uniform
    if (a.ngen > 0) {
      // (recomputed per tile rather than held in registers across the draw loops)
      // this lane's generator for the tile-start jump (lanes >= ngen idle there)
      uint64_t my_off = 0;
      u128 my_s0 = 0, my_inc = 0;
#pragma unroll 1
      for (int g = 0; g < a.ngen; ++g) {
        if (lane == static_cast<uint32_t>(g)) {
          my_off = a.raw_off[g];
          my_s0 = a.state0[g];
          my_inc = a.inc[g];
        }
      }
      const uint64_t r = my_off + e0 + 1;  // raw draw r needs T^(r+1) from state0
      u128 A = 1, G = 0;
#pragma unroll 1
      for (int k = 0; k < 64; ++k) {
        const uint64_t rk = r >> k;
        if (!__any(rk != 0)) break;
        if (rk & 1u) {
          G = a.jA[k] * G + a.jG[k];
          A = a.jA[k] * A;
        }
      }
      const u128 s_tile = A * my_s0 + my_inc * G;
      // T^lane = (A_l, G_l)
      u128 Al = 1, Gl = 0;
#pragma unroll 1
      for (int k = 0; k < 6; ++k) {
        if ((lane >> k) & 1u) {
          Gl = a.jA[k] * Gl + a.jG[k];
          Al = a.jA[k] * Al;
        }
      }
#pragma unroll 1
      for (int g = 0; g < a.ngen; ++g)
        s_state[g * kMaskBlock + tid] = Al * bcast_u128(s_tile, g) + a.inc[g] * Gl;
    }
    const bool full = e0 + kTileElems <= a.elem_end;
#pragma unroll 1
    for (int c = 0; c < kChunks; ++c) {
      const uint64_t ec = e0 + static_cast<uint64_t>(c) * kChunkElems + lane;
      uint64_t acc[kDrawsPerLane];
      if (a.base_i64) {  // base kind and tile fullness are wave-uniform: no per-element branches
#pragma unroll
        for (int i = 0; i < kDrawsPerLane; ++i) {
          const uint64_t e = ec + 64u * i;
          acc[i] = (full || e < a.elem_end) ? static_cast<uint64_t>(a.base_i64[e]) : 0u;
        }
      } else if (a.base_f64) {
#pragma unroll
        for (int i = 0; i < kDrawsPerLane; ++i) {
          const uint64_t e = ec + 64u * i;
          acc[i] = (full || e < a.elem_end) ? static_cast<uint64_t>(f64_to_i64_x86(a.base_f64[e] * a.scale)) : 0u;
        }
      } else {
#pragma unroll
        for (int i = 0; i < kDrawsPerLane; ++i) acc[i] = 0;
      }
#pragma unroll
      for (int i = 0; i < kDrawsPerLane; ++i) acc[i] += a.low_total;
      // generators are sorted by sign on the host (positives first), so pairs share a sign
      int g = 0;
#pragma unroll 1
      for (; g + 1 < a.npos; g += 2) rejmask |= gens_step<MERS, false, 2>(a, s_state, tid, g, acc);
      if (g < a.npos) rejmask |= gens_step<MERS, false, 1>(a, s_state, tid, g++, acc);
#pragma unroll 1
      for (; g + 1 < a.ngen; g += 2) rejmask |= gens_step<MERS, true, 2>(a, s_state, tid, g, acc);
      if (g < a.ngen) rejmask |= gens_step<MERS, true, 1>(a, s_state, tid, g, acc);
#pragma unroll
      for (int i = 0; i < kDrawsPerLane; ++i) {
        const uint64_t e = ec + 64u * i;
        if (full || e < a.elem_end) __builtin_nontemporal_store(static_cast<int64_t>(acc[i]), a.out + e);
      }
    }
  }
  if (a.rejects) {
#pragma unroll 1
    for (int g = 0; g < a.ngen; ++g) {
      if (__ballot((rejmask >> g) & 1u) && lane == 0) atomicAdd(a.rejects + a.orig[g], 1u);
    }
  }
}


// DN_MASK_SMALL: tiles of one chunk (512 elements per wave) and no LDS.  A
// wave's lane g keeps generator g's state at the wave's tile start in
// registers and steps it to the wave's next tile by one constant map
// (strideA, strideG: T^(nwaves 512), from the host) instead of a binary
// jump per tile; each lane offsets it by T^lane per generator.  No generator
// state crosses a tile, so nothing lives in LDS and occupancy is set by the
// registers alone (the 4096-element tiles keep 16 B per lane per generator in
// LDS between chunks: 40 KB per workgroup at 10 generators, 4 waves per SIMD).
#ifndef DN_MASK_SMALL
#define DN_MASK_SMALL 0
#endif
#ifndef DN_MASK_WAVES
#define DN_MASK_WAVES 5  // launch bound: waves per SIMD the small-tile kernel is compiled for
#endif

template <bool MERS, bool NEG, int K>
__device__ __forceinline__ uint32_t gens_step_small(const AccArgs& a, const u128 sg, const u128 Al, const u128 Gl,
                                                    const int g, uint64_t (&acc)[kDrawsPerLane]) {
  u128 st[K], c[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    // generator g + j's tile-start state, from lane g + j, offset by T^lane
    st[j] = Al * bcast_u128(sg, g + j) + a.inc[g + j] * Gl;
    c[j] = a.c64[g + j];
  }
  return draws_chunk<MERS, NEG, K>(st, acc, a.A64, c, a.excl, a.threshold) << g;
}

template <bool MERS>
__global__ void __launch_bounds__(kMaskBlock, DN_MASK_WAVES) bounded_acc_small_kernel(const AccArgs a) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint64_t n = a.elem_end - a.elem_begin;
  const uint64_t ntiles = (n + kChunkElems - 1) / kChunkElems;
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kMaskBlock / 64);
  const uint64_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * (kMaskBlock / 64) + (tid >> 6));
  if (wave0 >= ntiles) return;
  uint32_t rejmask = 0u;
  // T^lane = (Al, Gl), once
  u128 Al = 1, Gl = 0;
#pragma unroll 1
  for (int k = 0; k < 6; ++k) {
    if ((lane >> k) & 1u) {
      Gl = a.jA[k] * Gl + a.jG[k];
      Al = a.jA[k] * Al;
    }
  }
  // lane g: generator g before the wave's first tile (raw draw r uses T^(r+1)), one binary jump
  u128 sg = 0, cs = 0;
  if (a.ngen > 0) {
    uint64_t my_off = 0;
    u128 my_s0 = 0, my_inc = 0;
#pragma unroll 1
    for (int g = 0; g < a.ngen; ++g) {
      if (lane == static_cast<uint32_t>(g)) {
        my_off = a.raw_off[g];
        my_s0 = a.state0[g];
        my_inc = a.inc[g];
      }
    }
    const uint64_t r = my_off + a.elem_begin + wave0 * kChunkElems + 1;
    u128 A = 1, G = 0;
#pragma unroll 1
    for (int k = 0; k < 64; ++k) {
      const uint64_t rk = r >> k;
      if (!__any(rk != 0)) break;
      if (rk & 1u) {
        G = a.jA[k] * G + a.jG[k];
        A = a.jA[k] * A;
      }
    }
    sg = A * my_s0 + my_inc * G;
    cs = my_inc * a.strideG;  // this lane's generator: the tile-to-tile step's additive term
  }
#pragma unroll 1
  for (uint64_t tile = wave0; tile < ntiles; tile += nwaves) {
    const uint64_t ec = a.elem_begin + tile * kChunkElems + lane;
    const bool full = a.elem_begin + (tile + 1) * kChunkElems <= a.elem_end;
    uint64_t acc[kDrawsPerLane];
    if (a.base_i64) {
#pragma unroll
      for (int i = 0; i < kDrawsPerLane; ++i) {
        const uint64_t e = ec + 64u * i;
        acc[i] = (full || e < a.elem_end) ? static_cast<uint64_t>(a.base_i64[e]) : 0u;
      }
    } else if (a.base_f64) {
#pragma unroll
      for (int i = 0; i < kDrawsPerLane; ++i) {
        const uint64_t e = ec + 64u * i;
        acc[i] = (full || e < a.elem_end) ? static_cast<uint64_t>(f64_to_i64_x86(a.base_f64[e] * a.scale)) : 0u;
      }
    } else {
#pragma unroll
      for (int i = 0; i < kDrawsPerLane; ++i) acc[i] = 0;
    }
#pragma unroll
    for (int i = 0; i < kDrawsPerLane; ++i) acc[i] += a.low_total;
    int g = 0;
#pragma unroll 1
    for (; g + 1 < a.npos; g += 2) rejmask |= gens_step_small<MERS, false, 2>(a, sg, Al, Gl, g, acc);
    if (g < a.npos) rejmask |= gens_step_small<MERS, false, 1>(a, sg, Al, Gl, g++, acc);
#pragma unroll 1
    for (; g + 1 < a.ngen; g += 2) rejmask |= gens_step_small<MERS, true, 2>(a, sg, Al, Gl, g, acc);
    if (g < a.ngen) rejmask |= gens_step_small<MERS, true, 1>(a, sg, Al, Gl, g, acc);
#pragma unroll
    for (int i = 0; i < kDrawsPerLane; ++i) {
      const uint64_t e = ec + 64u * i;
      if (full || e < a.elem_end) __builtin_nontemporal_store(static_cast<int64_t>(acc[i]), a.out + e);
    }
    sg = a.strideA * sg + cs;  // lane g: generator g to the wave's next tile
  }
  if (a.rejects) {
#pragma unroll 1
    for (int g = 0; g < a.ngen; ++g) {
      if (__ballot((rejmask >> g) & 1u) && lane == 0) atomicAdd(a.rejects + a.orig[g], 1u);
    }
  }
}

struct RejArgs {
  u128 state0, inc, c64;
  u128 jA[64], jG[64];
  u128 A64;
  uint64_t raw_begin, raw_end, excl, threshold;
  uint64_t* out_idx;
  uint32_t* count;
  uint32_t capacity;
};

__global__ void __launch_bounds__(kMaskBlock) rejects_kernel(const RejArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t n = a.raw_end - a.raw_begin;
  const uint64_t ntiles = (n + kChunkElems - 1) / kChunkElems;
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kMaskBlock / 64);
  const uint64_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * (kMaskBlock / 64) + (threadIdx.x >> 6));
  for (uint64_t tile = wave0; tile < ntiles; tile += nwaves) {
    const uint64_t r0 = a.raw_begin + tile * kChunkElems;
    u128 A = 1, G = 0;
    const uint64_t ru = r0 + 1;
    for (int k = 0; k < 64 && (ru >> k); ++k)
      if ((ru >> k) & 1u) {
        G = a.jA[k] * G + a.jG[k];
        A = a.jA[k] * A;
      }
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if ((lane >> k) & 1u) {
        G = a.jA[k] * G + a.jG[k];
        A = a.jA[k] * A;
      }
    u128 st = A * a.state0 + a.inc * G;
    for (int i = 0; i < kDrawsPerLane; ++i) {
      const uint64_t r = r0 + lane + 64u * i;
      const u128 m = static_cast<u128>(xsl_rr(st)) * a.excl;
      if (r < a.raw_end && static_cast<uint64_t>(m) < a.threshold) {
        const uint32_t slot = atomicAdd(a.count, 1u);
        if (slot < a.capacity) a.out_idx[slot] = r;
      }
      st = a.A64 * st + a.c64;
    }
  }
}

__global__ void unfix_kernel(const int64_t* __restrict__ in, double* __restrict__ out, uint64_t n, double scale) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    out[i] = static_cast<double>(in[i]) / scale;
}

static double pow10_exact(int p) {
  double s = 1.0;
  for (int i = 0; i < p; ++i) s *= 10.0;  // exact for p <= 22 (as numpy's float64(10**p))
  return s;
}

// T^m = (A, G) from the power-of-two table (host)
static void pcg64_jump(uint64_t m, const u128* jA, const u128* jG, u128* A, u128* G) {
  u128 a = 1, g = 0;
  for (int k = 0; k < 64 && (m >> k); ++k)
    if ((m >> k) & 1u) {
      g = jA[k] * g + jG[k];
      a = jA[k] * a;
    }
  *A = a;
  *G = g;
}

static int grid_for_tiles(uint64_t tiles) {
  const uint64_t blocks = (tiles + 3) / 4;
  return static_cast<int>(blocks < 8192 ? (blocks ? blocks : 1) : 8192);
}

}  // namespace dn

using namespace dn;

extern "C" int dn_bounded_i64_accumulate(const dn_pcg64_t* gens, const int32_t* signs, const uint64_t* raw_offsets,
                                         int ngen, int64_t low, uint64_t rng, const int64_t* base_i64,
                                         const double* base_f64, int precision, int64_t* out, uint64_t elem_begin,
                                         uint64_t elem_end, uint32_t* reject_count, void* stream) {
  if (ngen < 0 || ngen > DN_MASK_MAX_GENS)
    return set_error(DN_ERR_UNSUPPORTED, "dn_bounded_i64_accumulate: %d generators (max %d)", ngen, DN_MASK_MAX_GENS);
  if (rng <= 0xFFFFFFFFull || rng == ~0ull)
    return set_error(DN_ERR_UNSUPPORTED, "dn_bounded_i64_accumulate: range %llu outside the 64-bit Lemire path",
                     static_cast<unsigned long long>(rng));
  if (precision < 0 || precision > 22) return set_error(DN_ERR_ARG, "dn_bounded_i64_accumulate: precision 0..22");
  if (elem_end <= elem_begin) return DN_OK;
  if (!out || (ngen > 0 && (!gens || !signs))) return set_error(DN_ERR_ARG, "dn_bounded_i64_accumulate: null pointer");
  AccArgs a;
  std::memset(&a, 0, sizeof(a));
  a.out = out;
  a.base_i64 = base_i64;
  a.base_f64 = base_i64 ? nullptr : base_f64;
  a.scale = pow10_exact(precision);
  a.elem_begin = elem_begin;
  a.elem_end = elem_end;
  a.excl = rng + 1;
  a.threshold = (~0ull - rng) % a.excl;
  a.ngen = ngen;
  a.rejects = reject_count;
  pcg64_jump_tables(a.jA, a.jG);
  a.A64 = a.jA[6];
  for (int g = 0; g < ngen; ++g)
    if (signs[g] != 1 && signs[g] != -1) return set_error(DN_ERR_ARG, "dn_bounded_i64_accumulate: sign must be +-1");
  int slot = 0;
  for (int pass = 0; pass < 2; ++pass) {  // positives first, then negatives (the sum commutes)
    for (int g = 0; g < ngen; ++g) {
      if ((signs[g] < 0) != (pass == 1)) continue;
      a.orig[slot] = g;
      a.low_total += signs[g] < 0 ? 0ull - static_cast<uint64_t>(low) : static_cast<uint64_t>(low);
      a.raw_off[slot] = raw_offsets ? raw_offsets[g] : 0;
      a.state0[slot] = to_u128(gens[g].state_hi, gens[g].state_lo);
      a.inc[slot] = to_u128(gens[g].inc_hi, gens[g].inc_lo);
      a.c64[slot] = a.inc[slot] * a.jG[6];
      ++slot;
    }
    if (pass == 0) a.npos = slot;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a.excl == (1ull << kMersK) - 1) a.mers_k = kMersK;  // Lemire by shifts (make_mask's range)
  const char* sm = tune_env("DN_MASK_SMALL");
  if (sm ? sm[0] == '1' : DN_MASK_SMALL) {
    // small tiles: a resident grid (DN_MASK_GRID workgroups per CU), each wave
    // stepping through its tiles by the constant map T^(nwaves 512)
    const uint64_t tiles = (elem_end - elem_begin + kChunkElems - 1) / kChunkElems;
    const char* gc = tune_env("DN_MASK_GRID");
    const uint64_t per_cu = gc ? static_cast<uint64_t>(std::atoi(gc)) : static_cast<uint64_t>(DN_MASK_WAVES);
    const uint64_t cap = static_cast<uint64_t>(device_cu_count()) * (per_cu ? per_cu : 1);
    const uint64_t blocks = std::min<uint64_t>((tiles + 3) / 4, cap);
    pcg64_jump(4ull * blocks * kChunkElems, a.jA, a.jG, &a.strideA, &a.strideG);
    if (a.mers_k) hipLaunchKernelGGL(bounded_acc_small_kernel<true>, dim3(blocks), dim3(kMaskBlock), 0, s, a);
    else hipLaunchKernelGGL(bounded_acc_small_kernel<false>, dim3(blocks), dim3(kMaskBlock), 0, s, a);
  } else {
    const uint64_t tiles = (elem_end - elem_begin + kTileElems - 1) / kTileElems;
    const dim3 grid(grid_for_tiles(tiles)), block(kMaskBlock);
    const size_t lds = static_cast<size_t>(ngen) * kMaskBlock * sizeof(u128);
    if (a.mers_k) hipLaunchKernelGGL(bounded_acc_kernel<true>, grid, block, lds, s, a);
    else hipLaunchKernelGGL(bounded_acc_kernel<false>, grid, block, lds, s, a);
  }
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_bounded_i64_accumulate: %s", hipGetErrorString(err));
  return DN_OK;
}

extern "C" int dn_bounded_i64_rejects(const dn_pcg64_t* gen, uint64_t rng, uint64_t raw_begin, uint64_t raw_end,
                                      uint64_t* out_idx, uint32_t* count, uint32_t capacity, void* stream) {
  if (!gen || !count || (capacity && !out_idx)) return set_error(DN_ERR_ARG, "dn_bounded_i64_rejects: null pointer");
  if (rng <= 0xFFFFFFFFull || rng == ~0ull) return set_error(DN_ERR_UNSUPPORTED, "dn_bounded_i64_rejects: range");
  if (raw_end <= raw_begin) return DN_OK;
  RejArgs a;
  std::memset(&a, 0, sizeof(a));
  pcg64_jump_tables(a.jA, a.jG);
  a.A64 = a.jA[6];
  a.state0 = to_u128(gen->state_hi, gen->state_lo);
  a.inc = to_u128(gen->inc_hi, gen->inc_lo);
  a.c64 = a.inc * a.jG[6];
  a.raw_begin = raw_begin;
  a.raw_end = raw_end;
  a.excl = rng + 1;
  a.threshold = (~0ull - rng) % a.excl;
  a.out_idx = out_idx;
  a.count = count;
  a.capacity = capacity;
  const uint64_t tiles = (raw_end - raw_begin + kChunkElems - 1) / kChunkElems;
  hipLaunchKernelGGL(rejects_kernel, dim3(grid_for_tiles(tiles)), dim3(kMaskBlock), 0, static_cast<hipStream_t>(stream),
                     a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_bounded_i64_rejects: %s", hipGetErrorString(err));
  return DN_OK;
}

extern "C" int dn_unfix_precision(const int64_t* in, double* out, uint64_t n, int precision, void* stream) {
  if (precision < 0 || precision > 22) return set_error(DN_ERR_ARG, "dn_unfix_precision: precision 0..22");
  if (n == 0) return DN_OK;
  if (!in || !out) return set_error(DN_ERR_ARG, "dn_unfix_precision: null pointer");
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(unfix_kernel, dim3(blocks < 8192 ? blocks : 8192), dim3(256), 0,
                     static_cast<hipStream_t>(stream), in, out, n, pow10_exact(precision));
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_unfix_precision: %s", hipGetErrorString(err));
  return DN_OK;
}
