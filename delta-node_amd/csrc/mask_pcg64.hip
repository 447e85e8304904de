// mask_pcg64.hip — secure-aggregation masks on gfx950: numpy's PCG64 stream
// and bounded-int64 (Lemire) draws, fused with fixed-point conversion and the
// signed sum over masks (reference: delta_node/utils/arr.py:20-28,
// utils/precision.py:5-15, runner/horizontal/agg.py:284-318).
//
// A raw draw r of a PCG64 generator is a pure function of (state, r): the
// LCG s' = a s + inc jumps ahead in closed form, s_r = A_r s_0 + inc G_r with
// A_r = a^r, G_r = 1 + a + ... + a^(r-1) (mod 2^128).  So lanes generate
// their elements independently: lane l of a wave owns elements
// e0 + l + 64 i; it jumps once to raw e0 + l and then steps by 64 with the
// constant map (A_64, inc G_64).  Consecutive lanes write consecutive int64s
// (512 B per wave store).  The output equals numpy's whenever no raw draw in
// the range is rejected by Lemire's test (odds 2^-47 per draw for make_mask);
// every draw is tested and rejections are counted per generator, and the
// caller then replays that generator exactly with per-segment raw offsets.
#include <hip/hip_runtime.h>

#include <cstring>

#include "dn_internal.hpp"
#include "dn_mask.h"
#include "pcg64_common.hpp"

namespace dn {

constexpr int kMaskBlock = 256;
constexpr int kDrawsPerLane = 16;                // per chunk
constexpr int kChunkElems = 64 * kDrawsPerLane;  // 1024
constexpr int kChunks = 4;
constexpr uint64_t kTileElems = kChunkElems * kChunks;  // 4096 per wave tile

struct AccArgs {
  int64_t* out;
  const int64_t* base_i64;
  const double* base_f64;
  double scale;
  uint64_t elem_begin, elem_end;
  uint64_t excl, threshold;
  int64_t low;
  int32_t ngen;
  int32_t sign[DN_MASK_MAX_GENS];
  uint64_t raw_off[DN_MASK_MAX_GENS];
  u128 state0[DN_MASK_MAX_GENS];  // state before raw draw 0 (draw r uses T^(r+1))
  u128 inc[DN_MASK_MAX_GENS];
  u128 c64[DN_MASK_MAX_GENS];     // inc * G_64
  u128 jA[64], jG[64];            // T^(2^k) = (A, G)
  u128 A64;
  uint32_t* rejects;
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

// (A, G) of T^r for a wave-uniform r: product of the set bits' tables.
__device__ __forceinline__ void jump_uniform(const AccArgs& a, uint64_t r, u128& A, u128& G) {
  A = 1;
  G = 0;
  for (int k = 0; k < 64 && (r >> k); ++k) {
    if ((r >> k) & 1u) {
      G = a.jA[k] * G + a.jG[k];
      A = a.jA[k] * A;
    }
  }
}

// ... composed with T^l for the lane offset l < 64 (6 predicated steps).
__device__ __forceinline__ void jump_lane(const AccArgs& a, uint32_t l, u128& A, u128& G) {
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    if ((l >> k) & 1u) {
      G = a.jA[k] * G + a.jG[k];
      A = a.jA[k] * A;
    }
  }
}

// Each lane keeps one PCG64 state per generator; they live in LDS between
// chunks (16 B per lane per generator, wave-private slots, no barrier) so
// that the generator loop can stay a runtime loop at ~60 VGPRs.
__global__ void __launch_bounds__(kMaskBlock) bounded_acc_kernel(const AccArgs a) {
  __shared__ u128 s_state[DN_MASK_MAX_GENS][kMaskBlock];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint64_t n = a.elem_end - a.elem_begin;
  const uint64_t ntiles = (n + kTileElems - 1) / kTileElems;
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kMaskBlock / 64);
  const uint64_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * (kMaskBlock / 64) + (tid >> 6));
  uint32_t rejmask = 0u;  // bit g: this lane saw a rejected draw of generator g
  for (uint64_t tile = wave0; tile < ntiles; tile += nwaves) {
    const uint64_t e0 = a.elem_begin + tile * kTileElems;  // wave-uniform
#pragma unroll 1
    for (int g = 0; g < a.ngen; ++g) {
      u128 A, G;
      jump_uniform(a, a.raw_off[g] + e0 + 1, A, G);  // raw r needs T^(r+1) from state0
      jump_lane(a, lane, A, G);
      s_state[g][tid] = A * a.state0[g] + a.inc[g] * G;
    }
#pragma unroll 1
    for (int c = 0; c < kChunks; ++c) {
      const uint64_t ec = e0 + static_cast<uint64_t>(c) * kChunkElems + lane;
      uint64_t acc[kDrawsPerLane];
#pragma unroll
      for (int i = 0; i < kDrawsPerLane; ++i) {
        const uint64_t e = ec + 64u * i;
        uint64_t v = 0;
        if (e < a.elem_end) {
          if (a.base_i64) v = static_cast<uint64_t>(a.base_i64[e]);
          else if (a.base_f64) v = static_cast<uint64_t>(f64_to_i64_x86(a.base_f64[e] * a.scale));
        }
        acc[i] = v;
      }
#pragma unroll 1
      for (int g = 0; g < a.ngen; ++g) {
        const bool neg = a.sign[g] < 0;
        const u128 c64 = a.c64[g];
        u128 st = s_state[g][tid];
        bool rj = false;
#pragma unroll
        for (int i = 0; i < kDrawsPerLane; ++i) {
          const uint64_t x = xsl_rr(st);
          const u128 m = static_cast<u128>(x) * a.excl;
          const uint64_t val = static_cast<uint64_t>(a.low) + static_cast<uint64_t>(m >> 64);
          rj |= ((ec + 64u * i) < a.elem_end) && (static_cast<uint64_t>(m) < a.threshold);
          acc[i] = neg ? acc[i] - val : acc[i] + val;
          st = a.A64 * st + c64;
        }
        s_state[g][tid] = st;
        if (rj) rejmask |= 1u << g;
      }
#pragma unroll
      for (int i = 0; i < kDrawsPerLane; ++i) {
        const uint64_t e = ec + 64u * i;
        if (e < a.elem_end) __builtin_nontemporal_store(static_cast<int64_t>(acc[i]), a.out + e);
      }
    }
  }
  if (a.rejects) {
#pragma unroll 1
    for (int g = 0; g < a.ngen; ++g) {
      if (__ballot((rejmask >> g) & 1u) && lane == 0) atomicAdd(a.rejects + g, 1u);
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
  a.low = low;
  a.ngen = ngen;
  a.rejects = reject_count;
  pcg64_jump_tables(a.jA, a.jG);
  a.A64 = a.jA[6];
  for (int g = 0; g < ngen; ++g) {
    if (signs[g] != 1 && signs[g] != -1) return set_error(DN_ERR_ARG, "dn_bounded_i64_accumulate: sign must be +-1");
    a.sign[g] = signs[g];
    a.raw_off[g] = raw_offsets ? raw_offsets[g] : 0;
    a.state0[g] = to_u128(gens[g].state_hi, gens[g].state_lo);
    a.inc[g] = to_u128(gens[g].inc_hi, gens[g].inc_lo);
    a.c64[g] = a.inc[g] * a.jG[6];
  }
  const uint64_t tiles = (elem_end - elem_begin + kTileElems - 1) / kTileElems;
  const dim3 grid(grid_for_tiles(tiles)), block(kMaskBlock);
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(bounded_acc_kernel, grid, block, 0, s, a);
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
