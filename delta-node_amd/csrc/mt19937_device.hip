// mt19937_device.hip — CPython's MT19937 coefficient draw on the GPU, bit-exact.
//
// Reference: SecretShare.make_shares draws its t-1 coefficients per element
// with self.random.randint(1, p-1) (delta_node/crypto/shamir/shamir.py:59-61):
// 1 + getrandbits(521), redrawn while >= p-1; getrandbits(521) is 17 MT19937
// words, little-endian, the last >> 23.  dn_mt19937_draw_coeffs (host_m521.cpp)
// restates that stream sequentially; this file produces the same values on the
// device by cutting the word stream into S substreams of L = 17 * 2^k words
// (2^k whole draws each; k = 14 from 2^24 coefficients, 12 from 2^21, else
// 10), all on the GPU:
//
//  * jump kernel: the MT window at the start of every substream by
//    jump-ahead, g(f)(W) with g = x^J mod P (P the characteristic polynomial
//    of the one-word transition f; tools/gen_mt_jump.py), evaluated by Horner
//    over 64-bit chunks of g: r <- f^64(r) ^ sum of table rows, the table E the
//    64 combinations of six consecutive shifts of W, in LDS.  A wave holds r
//    (624 words + 80 free slots) in 11 VGPRs; f^64 appends 64 words (three
//    ds_bpermute + the twist per lane).  Windows are at most three jumps
//    (radix-64 digits of s - 1, mt19937_jump.inc) from the caller's window:
//    one launch per level, every jump of a level independent;
//  * generation kernel: one wave per substream keeps its window in the same
//    register ring, appends 64 words at a time, tempers them into an LDS ring
//    and turns every 17-word group into one coefficient (+1, rejection test):
//    stored in the tiled layout (T = 0) or consumed at once by the split of
//    the element it belongs to (T = t, the fused draw + split); one extra
//    wave steps the last window before CPython's final array to it, so
//    self.random continues exactly as after n sequential make_shares calls.
// A rejected draw (probability ~2^-520 per coefficient) shifts every later
// word; the device flags it and the caller redoes the draw on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

#include "dn_internal.hpp"
#include "m521_device.hpp"

namespace dn {
namespace {

#include "mt19937_jump.inc"
#include "mt19937_jump_short.inc"
#include "mt19937_jump_direct.inc"

// Substream lengths: L_k = 17 * 2^k words (2^k whole draws), k = 10, 12, 14,
// one jump table each (rows A, C, B as in mt19937_jump.inc).  A draw of ncoef
// coefficients uses one k for all its substreams (mt_sub_len): long
// substreams for big draws (fewer jumps), short ones for small draws (a
// substream's generation is one wave's sequential run: ~48 ns per draw, so
// 2^14 draws cost ~0.8 ms whatever the vector size).
// Index 3 (2^8 draws) serves only draws of at most 65 substreams, whose
// windows are all one jump from the caller's (direct rows D_s, below): it has
// no A / C / B rows.
constexpr int kMtLens = 4;
constexpr int kMtLenLog2[kMtLens] = {10, 12, 14, 8};
constexpr int kMtTabLens = 3;  // lengths with A / C / B rows
__device__ const uint64_t kMtPolysDev[kMtTabLens][kMtJumpRows][kMtPolyWords] = {
    DN_MT_JUMP_POLYS_L10, DN_MT_JUMP_POLYS_L12, DN_MT_JUMP_POLYS};
static_assert(kMtJumpL10 == 17ull << 10 && kMtJumpL12 == 17ull << 12 && kMtJumpL == 17ull << 14, "table lengths");
// Direct rows (tools/gen_mt_jump.py --direct): D_s = x^(L - 624 + (s - 1) L),
// W(s) = D_s(W_idx), s = 1..64, per length in kMtLenLog2's order.  A draw of
// S <= 65 substreams takes ONE jump level from the caller's window instead of
// A then B (one launch, one combine and one level's latency less).  Job poly
// indices from kMtDirectBase address this table.
__device__ const uint64_t kMtDirectDev[kMtLens][kMtDirectRows][kMtPolyWords] = {
    DN_MT_JUMP_DIRECT_L10, DN_MT_JUMP_DIRECT_L12, DN_MT_JUMP_DIRECT_L14, DN_MT_JUMP_DIRECT_L8};
static_assert(kMtJumpL8 == 17ull << 8, "table lengths");
constexpr int32_t kMtDirectBase = kMtTabLens * kMtJumpRows;
// Runtime direct rows (host_gf2poly.cpp, kMtRtRows of them for L = 17 * 2^14,
// uploaded once per device): job poly indices from kMtRtBase address them.
constexpr int32_t kMtRtBase = kMtDirectBase + kMtLens * kMtDirectRows;

typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kMtN = 624, kMtM = 397;
constexpr uint32_t kMtA = 0x9908b0dfu, kMtUp = 0x80000000u, kMtLo = 0x7fffffffu;

// table index of the substream length of a draw of ncoef coefficients:
// 2^14 draws from 2^24 coefficients, 2^12 from 2^21, 2^10 down to 65 * 2^8
// + 1, else 2^8 (at least ~2048 substreams for the big draws; a few hundred
// jumps and a short generation run below; the smallest draws: at most 65
// substreams of 2^8 draws, one direct jump level and a ~4352-word run)
inline int mt_sub_len(uint64_t ncoef) {
  if (ncoef <= static_cast<uint64_t>(kMtDirectRows + 1) << 8) return 3;
  return ncoef >= (1ull << 24) ? 2 : ncoef >= (1ull << 21) ? 1 : 0;
}
inline uint64_t mt_sub_draws(int ki) { return 1ull << kMtLenLog2[ki]; }

__host__ __device__ inline uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

__host__ __device__ inline uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
  const uint32_t y = (a & kMtUp) | (b & kMtLo);
  return m ^ (y >> 1) ^ ((0u - (y & 1u)) & kMtA);
}

// A workgroup's waves work independently; LDS traffic between the lanes of
// one wave needs ordering, not a hardware barrier (a wavefront-scope fence
// keeps the compiler from moving LDS accesses across it; the LDS executes a
// wave's accesses in order).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The producer / consumer handoff: the ring half one wave wrote (ds_write)
// or read (ds_read) in this step is complete before the other wave touches it
// in the next, so a step ends with the LDS counter drained and s_barrier —
// not __syncthreads(), whose workgroup-scope release also drains the global
// stores: the consumer's 85 share stores per group would have to land before
// every barrier (emission alone 1.18 vs 1.04 ms at 2^24, profiles/r04/s/).
__device__ __forceinline__ void pc_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ------------------------------------------------------------------ jumps
#ifndef DN_JUMP_TABLE_POS
#define DN_JUMP_TABLE_POS 1  // jump table built per stream position (1) or per table word (0; A/B builds)
#endif

struct JumpJob {
  int32_t src, poly, dst;  // window indices (dst < 0: padding), jump-table row
  int32_t span;            // words [lo, hi) of g this job evaluates: lo | hi << 16
};

// The runtime direct level (build_levels' rt; DN_MT_RT=0 in the tuning
// build turns it off for A/B).
#ifndef DN_MT_RT_DIRECT
#define DN_MT_RT_DIRECT 1
#endif

// DN_MT_SPLIT2: the 2^24 draw's direct level in two halves; the first half's
// generation (substreams [0, S/2), on a side stream) runs while the second
// half's jumps do (their 85 KB tables beside the generation's rings), then the
// second half's generation (round 6; the tuning build's env knob of the same
// name A/Bs it).
#ifndef DN_MT_SPLIT2
#define DN_MT_SPLIT2 0
#endif

// A latency-bound level (few jobs: one Horner chain of ~312 steps per jump)
// splits every jump into P parts over word ranges [lo, hi) of g.  Since
// g(f) W = sum_k f^(64 k) g_k(f) W, part [lo, hi) evaluates
// sum_{k in [lo, hi)} f^(64 (k - lo)) g_k(f) (f^(64 lo) W) by Horner over its
// own words from the window 64 lo words further down W's stream, and the
// parts' windows XOR to the jump (mt_combine_kernel).
struct CombineJob {
  int32_t dst, first, parts, pad;  // dst = XOR of window rows first .. first + parts - 1
};

struct JumpArgs {
  uint32_t* wins;  // window s at row s (row 0 the caller's array), the caller's window advanced idx words at row -1
  const JumpJob* jobs;
  uint32_t njobs;
  uint32_t probe;  // tuning build only (DN_MT_JUMP_PROBE): 1 = no Horner steps, 2 = no stream stepping (timing only)
  const uint64_t* rt;  // runtime direct rows on the device (poly >= kMtRtBase), or null
};

// Jump and generation waves keep a 624-word MT window in registers: Q[11] a
// 704-slot ring (slot 64 r + lane), the window's word i at slot 16 + i of the
// current frame.  One append = the next 64 words of the stream
// (mix(word l, word l + 1, word l + 397), operands by ds_bpermute), written
// to the frame's free register; the frame then moves by one register.
// APPEND<K> is append number K mod 11 of an unrolled run: logical register r
// is Q[(r + K) % 11], so no register moves.
struct Lanes {
  int pa, pb, pm;  // ds_bpermute byte addresses of lanes l + 16, l + 17, l + 29 (mod 64)
  bool la, lb, lm;  // lane < 16, < 17, < 29
};

template <int K>
__device__ __forceinline__ uint32_t append64(uint32_t (&Q)[11], const Lanes& L) {
  const uint32_t xa = static_cast<uint32_t>(
      __builtin_amdgcn_ds_bpermute(L.pa, static_cast<int>(L.la ? Q[(1 + K) % 11] : Q[K % 11])));
  const uint32_t xb = static_cast<uint32_t>(
      __builtin_amdgcn_ds_bpermute(L.pb, static_cast<int>(L.lb ? Q[(1 + K) % 11] : Q[K % 11])));
  const uint32_t xm = static_cast<uint32_t>(
      __builtin_amdgcn_ds_bpermute(L.pm, static_cast<int>(L.lm ? Q[(7 + K) % 11] : Q[(6 + K) % 11])));
  Q[(10 + K) % 11] = mt_mix(xa, xb, xm);
  return Q[(10 + K) % 11];
}

// Jump table of one source window W, E[v] = words 0..683 of the stream of
// T[v] = sum over bits j of v of f^j(W), laid out for ds_read_b64.  The ten
// words a lane XORs into its window registers for one chunk are E[v][64 k +
// m - 16] for k = 0..9 (main half) or k = 1..10 (wrap half, lanes whose row
// index wraps); they are stored as five 8-B pairs, pair i of (v, m) at
//   half * kEWrap + i * kEPair + (64 v + m) * 2
// so one chunk is five ds_read_b64 at immediate offsets from one address.
// Banking (64 x 4-B banks, a b64 lane group = 32 lanes = 64 banks): a lane
// group reads 32 consecutive rows m (mod 64) of one pair plane -> 32
// distinct bank pairs, and kEWrap is a multiple of 64 words, so wrapped lanes
// keep their pairs: conflict-free (SQ_LDS_BANK_CONFLICT ~0), 160 LDS cycles
// per 16 chunks.  kEPair is 8 B off a multiple of 512 B so the compiler cannot
// fuse the five reads into ds_read2(st64)_b64 (half-rate, banks mod 32).
// A/B at 2^24 (profiles/r02/mt_jump_layout.md): the earlier 28-word rows
// (two b128 + one b64, wrap copy at +12 words) took 252 cycles by the bank
// model, SQ_LDS_BANK_CONFLICT +54 % of the array cycles, and the level of
// 2016 jumps 0.37-0.41 ms; this layout 0.29-0.31 ms; 12-word rows read as
// three b128 (conflict-free by the model, 192 cycles) 0.34-0.37 ms.
constexpr int kEVWords = 64 * 2;                      // words per chunk value v in one pair plane
constexpr int kEPair = 16 * kEVWords + 2;              // 2050 words
constexpr int kEWrap = ((5 * kEPair + 63) / 64) * 64;  // 10304 words
constexpr int kEWords = kEWrap + 5 * kEPair;           // 82 KB
constexpr int kJumpWaves = 16;  // at most this many jumps (waves) per workgroup, all from one source and part
// 32: small levels (the direct level of a small draw, level A) split into
// parts of ~10 Horner steps (make_shares_vec 2^12 -1.5 us, level A 26.5 vs
// 29.1 us at 2^24; profiles/r04/e/)
#ifndef DN_MT_MAX_PARTS
#define DN_MT_MAX_PARTS 32
#endif
constexpr int kMaxParts = DN_MT_MAX_PARTS;  // at most this many parts per jump

// a ^ b ^ c in one VALU instruction (gfx950 v_bitop3_b32, truth table 0x96;
// hipcc keeps two v_xor_b32 otherwise).  Inline asm on purpose in the jump
// kernel's Horner step: with the compiler builtin the scheduler hoists the
// table reads further and the kernel spills ~1,300 scratch accesses (the
// generation kernels' bitop3 below are builtins: no spill there, fewer s_nop).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// the ten table words of chunk t (value c) for this lane: off = the lane's row offset for t
__device__ __forceinline__ void table_words(const uint32_t* E, uint32_t off, uint32_t c, uint32_t (&x)[10]) {
  const uint32_t* p = E + c * kEVWords + off;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const u32x2_t d = *reinterpret_cast<const u32x2_t*>(p + i * kEPair);
    x[2 * i] = d.x, x[2 * i + 1] = d.y;
  }
}

// One Horner step over the 64-bit word gw of g in frame K (logical register
// r is Q[(r + K) % 11]): f^64 into the frame's free register, then the 16
// table windows XORed (two per instruction) into the 624 window words, which
// now sit at slots 80 .. 703 of the frame (registers 1 .. 10).
template <int K>
__device__ __forceinline__ void jump_mega(uint32_t (&Q)[11], const Lanes& L, const uint32_t* E,
                                          const uint32_t (&off)[16], uint64_t gw) {
  // the table reads of chunk pair p + 1 are issued before the XORs of pair p
  // (f^64's ds_bpermute first: LDS results return in issue order)
  uint32_t x[2][2][10];
  append64<K>(Q, L);
  table_words(E, off[0], static_cast<uint32_t>(gw >> 60) & 15u, x[0][0]);
  table_words(E, off[1], static_cast<uint32_t>(gw >> 56) & 15u, x[0][1]);
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    if (p < 7) {
      table_words(E, off[2 * p + 2], static_cast<uint32_t>(gw >> (52 - 8 * p)) & 15u, x[(p + 1) & 1][0]);
      table_words(E, off[2 * p + 3], static_cast<uint32_t>(gw >> (48 - 8 * p)) & 15u, x[(p + 1) & 1][1]);
    }
#pragma unroll
    for (int r = 1; r < 11; ++r)
      Q[(r + K) % 11] = xor3(Q[(r + K) % 11], x[p & 1][0][r - 1], x[p & 1][1][r - 1]);
  }
}

// DN_MT_JUMP_SMEM (default 1): a run's 11 words of g are read up front by
// scalar loads (g is read-only for the kernel's lifetime: the constant
// address space) — one wait per run, the chunk values extracted on the scalar
// unit (~70 fewer VALU per step) — instead of a vector load per step whose
// vmcnt(0) opened every step: the 2^24 level 171.6 vs 180.0 us on average,
// make_shares_vec 2^20 -2 % (profiles/r05/y/).
#ifndef DN_MT_JUMP_SMEM
#define DN_MT_JUMP_SMEM 1
#endif
typedef __attribute__((address_space(4))) const uint64_t const_u64_t;

template <int... ks>
__device__ __forceinline__ void jump_run(uint32_t (&Q)[11], const Lanes& L, const uint32_t* E,
                                         const uint32_t (&off)[16], const uint64_t* g, int wi, int top,
                                         std::integer_sequence<int, ks...>) {
#if DN_MT_JUMP_SMEM
  const_u64_t* gc = (const_u64_t*)(g);
  const int tu = __builtin_amdgcn_readfirstlane(top);
  uint64_t gws[sizeof...(ks)];
  ((void)(gws[ks] = gc[__builtin_amdgcn_readfirstlane(wi - ks <= tu ? wi - ks : tu)]), ...);  // in range
  ((void)(gws[ks] = (wi - ks) <= tu ? gws[ks] : 0ull), ...);
  ((void)jump_mega<ks>(Q, L, E, off, gws[ks]), ...);
#else
  ((void)[&] {
     const int w = wi - ks;
     const uint64_t gw = w <= top ? g[w] : 0ull;
     jump_mega<ks>(Q, L, E, off, gw);
   }(),
   ...);
#endif
}

// One workgroup = up to W jumps (or parts of jumps, words [lo, hi) of g)
// from the same source window W and the same lo (the host groups them;
// padding jobs have dst < 0).  Horner over 4-bit chunks of g,
// 16 chunks (one 64-bit word of g) per step: r <- f^64(r) ^ sum_t
// f^(4 (15 - t))(T[c_t]); f^m(T[v]) is the window at offset m of T[v]'s own
// stream, which the workgroup tables once (E, 82 KB of LDS), so a step is
//   * f^64(r): 64 new words mix(r[l], r[l+1], r[l+397]), l = 0..63 — one
//     register, its operands gathered by 3 ds_bpermute;
//   * the XOR of 16 table windows into the 624 window words (10 registers;
//     80 ds_read_b64 and 80 v_bitop3 per lane).
template <int W>  // waves per workgroup (8 or 16)
__global__ void __launch_bounds__(64 * W) mt_jump_kernel(const JumpArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t E[kEWords];
  __shared__ uint32_t ext[kMtN + 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  const uint32_t j0 = blockIdx.x * W;
  const JumpJob* jp = a.jobs + __builtin_amdgcn_readfirstlane(j0 + wid < a.njobs ? j0 + wid : j0);
  const int32_t poly = __builtin_amdgcn_readfirstlane(jp->poly), dsti = __builtin_amdgcn_readfirstlane(jp->dst);
  // the workgroup's jobs share the source and lo (one table; job j0 is never padding)
  const int32_t lo = __builtin_amdgcn_readfirstlane(a.jobs[j0].span) & 0xffff;
  const int32_t hi = __builtin_amdgcn_readfirstlane(jp->span) >> 16;
  const uint32_t* src = a.wins + static_cast<int64_t>(__builtin_amdgcn_readfirstlane(a.jobs[j0].src)) * kMtN;
  if (lo == 0) {
    // the source stream: words 0..623 of W, then 63 more (each from words <= 459 of W)
    for (uint32_t i = tid; i < kMtN; i += 64u * W) ext[i] = src[i];
    __syncthreads();
    if (tid < 63u) ext[kMtN + tid] = mt_mix(ext[tid], ext[tid + 1], ext[tid + kMtM]);
    __syncthreads();
  } else {
    // words 64 lo .. 64 lo + 686 of W's stream: step the stream in a 1024-word
    // LDS ring (the table's space, not yet built), 227 words per step (word
    // 624 + i needs words i, i + 1, i + 397).  A step writes ring slots
    // 624..850 past its base and reads 0..623, so one barrier per step.
    uint32_t* ring = E;
    for (uint32_t i = tid; i < kMtN; i += 64u * W) ring[i] = src[i];
    __syncthreads();
    const uint32_t need = a.probe == 2u ? 687u : 64u * static_cast<uint32_t>(lo) + 687u;
    for (uint32_t base = 0; base + kMtN < need; base += kMtN - kMtM) {
      if (tid < static_cast<uint32_t>(kMtN - kMtM)) {
        const uint32_t i = base + tid;
        ring[(i + kMtN) & 1023u] = mt_mix(ring[i & 1023u], ring[(i + 1u) & 1023u], ring[(i + kMtM) & 1023u]);
      }
      __syncthreads();
    }
    for (uint32_t i = tid; i < 687u; i += 64u * W) ext[i] = ring[(64u * static_cast<uint32_t>(lo) + i) & 1023u];
    __syncthreads();
  }
#if DN_JUMP_TABLE_POS
  // One thread per stream position q = 64 k + m (row k = 0..10 of the frame,
  // m = 0..63; T-stream word j = q - 16, zero outside 0..683): the 16
  // combinations of words j..j+3 from four LDS reads, stored to the main half
  // (row k = 2 i + parity, k <= 9) and the wrap half (k = 2 i + parity + 1,
  // k >= 1) of pair plane i.  The gap before the wrap half and the planes'
  // pad words are never read.
  for (uint32_t q = tid; q < 704u; q += 64u * W) {
    const int j = static_cast<int>(q) - 16;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (j >= 0 && j < 684) {
#pragma unroll
      for (int b = 0; b < 4; ++b) w[b] = ext[j + b];
    }
    const uint32_t k = q >> 6, m = q & 63u;
    uint32_t* em = k <= 9u ? E + (k >> 1) * kEPair + 2u * m + (k & 1u) : nullptr;
    uint32_t* ew = k >= 1u ? E + kEWrap + ((k - 1u) >> 1) * kEPair + 2u * m + ((k - 1u) & 1u) : nullptr;
    uint32_t c[16];
    c[0] = 0u;
#pragma unroll
    for (int v = 1; v < 16; ++v) c[v] = c[v & (v - 1)] ^ w[__builtin_ctz(v)];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      if (em) em[v * kEVWords] = c[v];
      if (ew) ew[v * kEVWords] = c[v];
    }
  }
#else
  for (uint32_t e = tid; e < static_cast<uint32_t>(kEWords); e += 64u * W) {
    const uint32_t wrap = e >= static_cast<uint32_t>(kEWrap) ? 1u : 0u, re = e - wrap * kEWrap;
    const uint32_t i = re / kEPair, rem = re - i * kEPair;  // pair plane, position in it
    const uint32_t v = rem / kEVWords, mw = rem - v * kEVWords, m = mw >> 1;
    // T-stream word; -1 in the gap before the wrap half and the 2 pad words of a plane
    const int j = (i < 5u && v < 16u) ? 64 * static_cast<int>(2 * i + (mw & 1u) + wrap) + static_cast<int>(m) - 16 : -1;
    uint32_t x = 0u;
    if (j >= 0 && j < 684) {
#pragma unroll
      for (int b = 0; b < 4; ++b) x ^= ext[j + b] & (0u - ((v >> b) & 1u));
    }
    E[e] = x;
  }
#endif
  __syncthreads();
  if (j0 + wid >= a.njobs || dsti < 0) return;

  // poly = table * rows + row, kMtDirectBase + length * 64 + s - 1, or
  // kMtRtBase + s - 1 (wave-uniform)
  const uint64_t* g = poly < kMtDirectBase ? &kMtPolysDev[0][0][0] + static_cast<uint64_t>(poly) * kMtPolyWords
                      : poly < kMtRtBase
                          ? &kMtDirectDev[0][0][0] + static_cast<uint64_t>(poly - kMtDirectBase) * kMtPolyWords
                          : a.rt + static_cast<uint64_t>(poly - kMtRtBase) * kMtPolyWords;
  uint32_t Q[11];
#pragma unroll
  for (int r = 0; r < 11; ++r) Q[r] = 0u;
  Lanes L;
  L.pa = static_cast<int>(((lane + 16u) & 63u) * 4u);
  L.pb = static_cast<int>(((lane + 17u) & 63u) * 4u);
  L.pm = static_cast<int>(((lane + 29u) & 63u) * 4u);
  L.la = lane < 16u, L.lb = lane < 17u, L.lm = lane < 29u;
  // chunk t's words for register r (1..10): table index 64 (r - 1) + lane + 60 - 4 t
  uint32_t off[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const uint32_t u = lane + 60u - 4u * t;
    off[t] = (u & 63u) * 2u + (u >> 6) * static_cast<uint32_t>(kEWrap);
  }
  int top = hi - 1;
  while (top > lo && g[top] == 0ull) --top;  // steps above it leave r = 0
  top = __builtin_amdgcn_readfirstlane(top);
  // runs of 11 steps (the frame returns to Q[0] after 11) ending at word lo;
  // r = 0 before the first nonzero word, so a run starts with zero words above it
  if (a.probe != 1u)
    for (int wi = lo + 11 * ((top - lo) / 11) + 10; wi >= lo + 10; wi -= 11)
      jump_run(Q, L, E, off, g, wi, top, std::make_integer_sequence<int, 11>{});
  uint32_t* dst = a.wins + static_cast<uint64_t>(dsti) * kMtN;
#pragma unroll
  for (int r = 0; r < 11; ++r) {
    const int i = 64 * r + static_cast<int>(lane) - 16;
    if (i >= 0 && i < kMtN) dst[i] = Q[r];
  }
}

// ---- jumps with a contiguous table: the two-bit kernel that sits beside the
// generation, and a four-bit variant
// mt_jump_kernel's Horner over CB-bit chunks of g (64 / CB per word of g)
// with the table T[v] = sum over bits j of v of f^j(W), v < 2^CB, stored as
// the 704 consecutive stream positions q = 64 k + m of each value (T-stream
// word q - 16; zero outside the used range): chunk t of a step reads, for
// window register r = 1..10, position 64 (r - 1) + lane + 64 - CB - CB t of
// T[c_t] — ten ds_read_b32 from one address (immediate offsets 256 B apart,
// 64 consecutive words per instruction: conflict-free, no wrapped copy), two
// chunks XORed per v_bitop3 as in mt_jump_kernel.
//  * CB = 2, W = 4 (mt_jumpc_kernel<4, 2>): 4 values, 11 KB — a workgroup fits
//    on a CU beside the generation's eight 17.7 KB rings (160 KB), at twice
//    the table bytes and XORs per word of g; the speculated levels that run
//    beside the generation (DN_MT_SPEC_BESIDE).
//  * CB = 4 (DN_MT_JUMP4B, tuning build): 16 values, 45 KB instead of
//    mt_jump_kernel's 83 (no wrapped copy), so two 16-wave workgroups share
//    a CU (<= 64 VGPRs): twice the waves per CU at twice the LDS
//    instructions (b32, same bytes) — an A/B of the direct level.
constexpr int kE2Val = 704;  // words per table value
// CB = 3: 21 three-bit chunks and bit 0 alone (22 per word of g, offsets 61 - 3 t
// and 0); T[0] = 0 is not stored (7 values, 19.3 KB: it still fits beside the
// rings) — a zero chunk's read goes to T[1] and its XOR is skipped (the chunk
// values are wave-uniform: a scalar branch per pair)
template <int CB>
constexpr int kNVal = CB == 3 ? 7 : (1 << CB);
template <int CB>
constexpr int kECWords = kNVal<CB> * kE2Val;  // 11 KB at CB = 2, 19.3 KB at 3, 45 KB at 4
template <int CB>
constexpr int kNChunks = CB == 3 ? 22 : 64 / CB;
static_assert(kECWords<2> >= 1024 + kMtN + 63, "the stepping ring and the source stream fit in the table's space");

template <int CB>
__device__ __forceinline__ uint32_t chunk_val(uint64_t gw, int t) {
  if constexpr (CB == 3) return t < 21 ? static_cast<uint32_t>(gw >> (61 - 3 * t)) & 7u : static_cast<uint32_t>(gw) & 1u;
  else return static_cast<uint32_t>(gw >> (64 - CB * (t + 1))) & ((1u << CB) - 1u);
}
template <int CB>
constexpr int chunk_off(int t) { return CB == 3 ? (t < 21 ? 61 - 3 * t : 0) : 64 - CB - CB * t; }
template <int CB>
__device__ __forceinline__ uint32_t chunk_row(uint32_t c) { return CB == 3 ? (c ? c - 1u : 0u) : c; }

template <int CB>
__device__ __forceinline__ void table_words_c(const uint32_t* E, uint32_t c, int t, uint32_t lane, uint32_t (&x)[10]) {
  const uint32_t* p = E + chunk_row<CB>(c) * static_cast<uint32_t>(kE2Val) + lane + static_cast<uint32_t>(chunk_off<CB>(t));
#pragma unroll
  for (int i = 0; i < 10; ++i) x[i] = p[64 * i];
}

template <int CB, int K>
__device__ __forceinline__ void jump_mega_c(uint32_t (&Q)[11], const Lanes& L, const uint32_t* E, uint32_t lane,
                                            uint64_t gw) {
  constexpr int NC = kNChunks<CB>;
  uint32_t x[2][2][10];
  append64<K>(Q, L);
  table_words_c<CB>(E, chunk_val<CB>(gw, 0), 0, lane, x[0][0]);
  table_words_c<CB>(E, chunk_val<CB>(gw, 1), 1, lane, x[0][1]);
#pragma unroll
  for (int p = 0; p < NC / 2; ++p) {
    if (p < NC / 2 - 1) {
      table_words_c<CB>(E, chunk_val<CB>(gw, 2 * p + 2), 2 * p + 2, lane, x[(p + 1) & 1][0]);
      table_words_c<CB>(E, chunk_val<CB>(gw, 2 * p + 3), 2 * p + 3, lane, x[(p + 1) & 1][1]);
    }
    if constexpr (CB == 3) {
      const bool n0 = chunk_val<CB>(gw, 2 * p) != 0u, n1 = chunk_val<CB>(gw, 2 * p + 1) != 0u;
      if (n0 && n1) {
#pragma unroll
        for (int r = 1; r < 11; ++r)
          Q[(r + K) % 11] = xor3(Q[(r + K) % 11], x[p & 1][0][r - 1], x[p & 1][1][r - 1]);
      } else if (n0 || n1) {
#pragma unroll
        for (int r = 1; r < 11; ++r) Q[(r + K) % 11] ^= n0 ? x[p & 1][0][r - 1] : x[p & 1][1][r - 1];
      }
    } else {
#pragma unroll
      for (int r = 1; r < 11; ++r)
        Q[(r + K) % 11] = xor3(Q[(r + K) % 11], x[p & 1][0][r - 1], x[p & 1][1][r - 1]);
    }
  }
}

template <int CB, int... ks>
__device__ __forceinline__ void jump_run_c(uint32_t (&Q)[11], const Lanes& L, const uint32_t* E, uint32_t lane,
                                           const uint64_t* g, int wi, int top, std::integer_sequence<int, ks...>) {
  const_u64_t* gc = (const_u64_t*)(g);
  const int tu = __builtin_amdgcn_readfirstlane(top);
  uint64_t gws[sizeof...(ks)];
  ((void)(gws[ks] = gc[__builtin_amdgcn_readfirstlane(wi - ks <= tu ? wi - ks : tu)]), ...);  // in range
  ((void)(gws[ks] = (wi - ks) <= tu ? gws[ks] : 0ull), ...);
  ((void)jump_mega_c<CB, ks>(Q, L, E, lane, gws[ks]), ...);
}

// Jobs as mt_jump_kernel's (W jumps or parts of one source and lo per
// workgroup); the source stream is staged in the table's space and read into
// registers before the table overwrites it.
template <int W, int CB>
__global__ void __launch_bounds__(64 * W, CB == 4 ? 8 : 1) mt_jumpc_kernel(const JumpArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t E[kECWords<CB>];
  uint32_t* ext = E + 1024;  // words 0 .. 686 of the source stream, until the table is built
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  const uint32_t j0 = blockIdx.x * W;
  const JumpJob* jp = a.jobs + __builtin_amdgcn_readfirstlane(j0 + wid < a.njobs ? j0 + wid : j0);
  const int32_t poly = __builtin_amdgcn_readfirstlane(jp->poly), dsti = __builtin_amdgcn_readfirstlane(jp->dst);
  const int32_t lo = __builtin_amdgcn_readfirstlane(a.jobs[j0].span) & 0xffff;
  const int32_t hi = __builtin_amdgcn_readfirstlane(jp->span) >> 16;
  const uint32_t* src = a.wins + static_cast<int64_t>(__builtin_amdgcn_readfirstlane(a.jobs[j0].src)) * kMtN;
  if (lo == 0) {
    for (uint32_t i = tid; i < kMtN; i += 64u * W) ext[i] = src[i];
    __syncthreads();
    if (tid < 63u) ext[kMtN + tid] = mt_mix(ext[tid], ext[tid + 1], ext[tid + kMtM]);
    __syncthreads();
  } else {
    // words 64 lo .. 64 lo + 686 of the stream, stepped in a 1024-word ring (E[0, 1024))
    uint32_t* ring = E;
    for (uint32_t i = tid; i < kMtN; i += 64u * W) ring[i] = src[i];
    __syncthreads();
    const uint32_t need = 64u * static_cast<uint32_t>(lo) + 687u;
    for (uint32_t base = 0; base + kMtN < need; base += kMtN - kMtM) {
      for (uint32_t tt = tid; tt < static_cast<uint32_t>(kMtN - kMtM); tt += 64u * W) {
        const uint32_t i = base + tt;
        ring[(i + kMtN) & 1023u] = mt_mix(ring[i & 1023u], ring[(i + 1u) & 1023u], ring[(i + kMtM) & 1023u]);
      }
      __syncthreads();
    }
    for (uint32_t i = tid; i < 687u; i += 64u * W) ext[i] = ring[(64u * static_cast<uint32_t>(lo) + i) & 1023u];
    __syncthreads();
  }
  // the table: position q holds T[v] word j = q - 16 = XOR of s_{j+b} over bits b of v
  constexpr int kQ = (kE2Val + 64 * W - 1) / (64 * W);
  constexpr int kJEnd = 687 - (CB - 1);  // j + CB - 1 <= 686
  uint32_t w[kQ][CB];
#pragma unroll
  for (int k = 0; k < kQ; ++k) {
    const int q = static_cast<int>(tid) + 64 * W * k, j = q - 16;
    const bool in = q < kE2Val && j >= 0 && j < kJEnd;
#pragma unroll
    for (int b = 0; b < CB; ++b) w[k][b] = in ? ext[j + b] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kQ; ++k) {
    const int q = static_cast<int>(tid) + 64 * W * k;
    if (q < kE2Val) {
      uint32_t c[1 << CB];
      c[0] = 0u;
#pragma unroll
      for (int v = 1; v < (1 << CB); ++v) c[v] = c[v & (v - 1)] ^ w[k][__builtin_ctz(v)];
#pragma unroll
      for (int v = CB == 3 ? 1 : 0; v < (1 << CB); ++v) E[(CB == 3 ? v - 1 : v) * kE2Val + q] = c[v];
    }
  }
  __syncthreads();
  if (j0 + wid >= a.njobs || dsti < 0) return;

  const uint64_t* g = poly < kMtDirectBase ? &kMtPolysDev[0][0][0] + static_cast<uint64_t>(poly) * kMtPolyWords
                      : poly < kMtRtBase
                          ? &kMtDirectDev[0][0][0] + static_cast<uint64_t>(poly - kMtDirectBase) * kMtPolyWords
                          : a.rt + static_cast<uint64_t>(poly - kMtRtBase) * kMtPolyWords;
  uint32_t Q[11];
#pragma unroll
  for (int r = 0; r < 11; ++r) Q[r] = 0u;
  Lanes L;
  L.pa = static_cast<int>(((lane + 16u) & 63u) * 4u);
  L.pb = static_cast<int>(((lane + 17u) & 63u) * 4u);
  L.pm = static_cast<int>(((lane + 29u) & 63u) * 4u);
  L.la = lane < 16u, L.lb = lane < 17u, L.lm = lane < 29u;
  int top = hi - 1;
  while (top > lo && g[top] == 0ull) --top;
  top = __builtin_amdgcn_readfirstlane(top);
  if (a.probe != 1u)
    for (int wi = lo + 11 * ((top - lo) / 11) + 10; wi >= lo + 10; wi -= 11)
      jump_run_c<CB>(Q, L, E, lane, g, wi, top, std::make_integer_sequence<int, 11>{});
  uint32_t* dst = a.wins + static_cast<int64_t>(dsti) * kMtN;
#pragma unroll
  for (int r = 0; r < 11; ++r) {
    const int i = 64 * r + static_cast<int>(lane) - 16;
    if (i >= 0 && i < kMtN) dst[i] = Q[r];
  }
}

// The chunk width of the kernel beside the generation (DN_MT_BESIDE_CB, 2 or
// 3; tuning build: the env variable of that name)
#ifndef DN_MT_BESIDE_CB
#define DN_MT_BESIDE_CB 2
#endif
int beside_cb() {
  const char* e = tune_env("DN_MT_BESIDE_CB");
  return e ? (e[0] == '2' ? 2 : 3) : DN_MT_BESIDE_CB;
}
void launch_jumpc4(dim3 grid, hipStream_t s, const JumpArgs& ja) {
  if (beside_cb() == 2) hipLaunchKernelGGL((mt_jumpc_kernel<4, 2>), grid, dim3(256), 0, s, ja);
  else hipLaunchKernelGGL((mt_jumpc_kernel<4, 3>), grid, dim3(256), 0, s, ja);
}

// The parts of a split level XORed into their jumps' windows: one thread per
// window word, the (at most 16) part loads issued together.
__global__ void __launch_bounds__(640) mt_combine_kernel(uint32_t* wins, const CombineJob* cj) {
  const CombineJob c = cj[blockIdx.x];
  const uint32_t i = threadIdx.x;
  if (i >= static_cast<uint32_t>(kMtN)) return;
  const uint32_t* p = wins + static_cast<uint64_t>(c.first) * kMtN + i;
  uint32_t x = 0u;
#pragma unroll
  for (int32_t j = 0; j < kMaxParts; ++j)
    if (j < c.parts) x ^= p[static_cast<uint64_t>(j) * kMtN];
  wins[static_cast<int64_t>(c.dst) * kMtN + i] = x;  // (dst -1: the W_idx row)
}

// ------------------------------------------------------------------ generation
struct GenArgs {
  const uint32_t* wins;  // [S + 1][624]
  uint8_t* coeffs;       // tm1 tiled vectors
  uint32_t* flag;        // != 0: a draw was rejected
  uint32_t* fin;         // CPython's final array (the final-state wave)
  uint64_t ncoef, vb;
  uint64_t sub_draws;    // draws per substream (2^k)
  uint64_t tm1_magic;    // ceil(2^32 / tm1): x / tm1 = (x * magic) >> 32 for x < 2^16
  uint32_t S;            // substreams
  uint32_t idx;          // CPython index: stream words 0..623-idx are temper(window0[idx..])
  int32_t tm1;
  int32_t final_sig;     // window the final-state wave starts from (-1: no such wave)
  uint64_t final_pos;    // position of that window's first word (0: the caller's array)
  uint64_t final_tf;     // position of CPython's final array
  // fused split (mt_gen_kernel<T>, T > 0): int64 secrets in, n share vectors out
  const int64_t* secrets;
  uint8_t* shares;
  uint64_t n_elem;
  int32_t n_shares;
  uint32_t ring;         // ring slots of one wave (2 emission groups; GenRing)
  uint32_t back;         // even substreams 2 .. S-2 run backward from the next window
  uint32_t probe;        // tuning build only (DN_MT_PROBE): 1 skip emissions, 2 skip generation
  uint32_t sub_lo;       // substream of workgroup 0 (a launch over substreams sub_lo ..: DN_MT_SPLIT2)
  uint32_t sub_n;        // workgroups of the launch (0: S + 1, every substream and the final-state wave)
  uint32_t* next_win;    // the next call's W_idx (null: not wanted), written with the final state
  uint64_t next_pos;     // its position idx + 17 ncoef (final-state wave)
  // tail_fin: the last substream writes the final state (and next_win) itself
  // after its generation, at positions fin_lo / next_lo of its own frame
  // (position 0 its first output); no final-state wave is launched
  uint32_t tail_fin;
  int32_t fin_lo, next_lo;  // (fin_lo < 0: words of the substream's window, still in the ring)
};

// DN_MT_PROBE (tuning build): time the generation and the emission apart.
#ifdef DN_TUNING
#define DN_PROBE_SKIP(a, bit) if (!((a).probe & (bit)))
#else
#define DN_PROBE_SKIP(a, bit)
#endif

// Substream s runs forward from W(s) unless backward generation is on
// (back = 1) and s is even, not 0 and not the last (then backward from
// W(s + 1)).  back = 2 (tuning build, DN_MT_BACK=2: a probe of the backward
// generation rate) runs every substream but the first and the last backward.
__host__ __device__ inline bool mt_sub_forward(uint32_t s, uint64_t S, int back) {
  if (back == 2) return s == 0u || s + 1u >= S;
  return !back || s == 0u || (s & 1u) || s + 1u >= S;
}

// W(s) is jumped to when substream s starts from it or substream s - 1 ends on it.
__host__ __device__ inline bool mt_window_needed(uint32_t s, uint64_t S, int back) {
  return mt_sub_forward(s, S, back) || !mt_sub_forward(s - 1u, S, back);
}

// Raw (untempered) words of a substream pass through an LDS ring of M words
// (M = two emission groups): stream word p sits at slot (p + delta) mod M,
// physical word o + slot, and physical words [o + M, o + M + 64) mirror slots
// [0, 64).
//  * An append writes the 64 words p0 .. p0 + 63 (p0 + delta a multiple of
//    64, so its slots never wrap), word p = mix(word p - 624, word p - 623,
//    word p - 227): one address plus immediates, except in the first 688
//    slots of the ring, where the three operands' slots wrap per lane (a
//    wave-uniform branch, 11 of 68 appends at t = 3).
//  * An emission group [g G, (g + 1) G) reads physical o + delta + (g % 2) G
//    onwards, below o + M + 64: the mirror holds the slots past M.
// delta is 0 except in substream 0, whose stream starts with the caller's
// 624 - idx words; o = delta & 1 keeps every group's first word 8-byte aligned
// (the emission's b64 reads).  Tempering happens when a group is emitted.
// Per 64 words an append is one address add, three ds_read_b32, the mix
// (5 VALU) and one ds_write — against three ds_bpermute, their operand
// selects, the mix, the temper and the ring address arithmetic of a
// register-resident window.
struct GenRing {
  uint32_t M, delta, o;
};

__device__ __forceinline__ uint32_t ring_wrap(uint32_t s, uint32_t M) { return s >= M ? s - M : s; }

// mt_mix in five VALU: y = bfi(UP, a, b); m ^ (y >> 1) ^ (-(b & 1) & A), the
// last two terms by v_bitop3 ((S0 & S1) ^ S2, table 0x6a; S0 the index MSB).
__device__ __forceinline__ uint32_t mt_mix5(uint32_t a, uint32_t b, uint32_t m) {
  const uint32_t y = (kMtUp & a) | (~kMtUp & b);  // v_bfi_b32
  const uint32_t u = (y >> 1) ^ m;
  const uint32_t mk = static_cast<uint32_t>(static_cast<int32_t>(b << 31) >> 31);
  return __builtin_amdgcn_bitop3_b32(mk, kMtA, u, 0x6a);  // (mk & A) ^ u
}

// B appends (B <= 3: the appends of a batch read no word another one of the
// batch writes: word p + 64 i - 227 < p for i < 3), reads first, one wait.
// WRAP: some operand slots of the batch lie below 0 (the batch starts in the
// ring's first 688 slots, or the batch itself wraps) and are wrapped per lane.
// vals: the raw words (the final-state wave keeps them).
template <int B, bool WRAP>
__device__ __forceinline__ void ring_appends(uint32_t* Rg, const GenRing& g, uint32_t slot, uint32_t lane,
                                             uint32_t (&vals)[3]) {
  uint32_t s[B], xa[B], xb[B], xm[B];
#pragma unroll
  for (int i = 0; i < B; ++i) {
    if constexpr (WRAP) {
      s[i] = ring_wrap(slot + 64u * i, g.M);
      const uint32_t q = s[i] + lane;
      const uint32_t qa = q < 624u ? q + g.M - 624u : q - 624u;
      const uint32_t qb = qa + 1u == g.M ? 0u : qa + 1u;
      const uint32_t qm = q < 227u ? q + g.M - 227u : q - 227u;
      xa[i] = Rg[g.o + qa];
      xb[i] = Rg[g.o + qb];
      xm[i] = Rg[g.o + qm];
    } else {
      s[i] = slot + 64u * i;
      const uint32_t* p = Rg + (g.o + s[i] - 624u) + lane;
      xa[i] = p[0];
      xb[i] = p[1];
      xm[i] = p[kMtM];
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // every read of the batch issued before the first mix waits
#pragma unroll
  for (int i = 0; i < B; ++i) {
    const uint32_t v = mt_mix5(xa[i], xb[i], xm[i]);
    vals[i] = v;
    Rg[g.o + s[i] + lane] = v;
    if (WRAP && s[i] == 0u) Rg[g.o + g.M + lane] = v;  // mirror of slots 0 .. 63
  }
}

template <int B>
__device__ __forceinline__ void ring_batch(uint32_t* Rg, const GenRing& g, uint32_t& slot, uint32_t lane,
                                           uint32_t (&vals)[3]) {
  const uint32_t s0 = __builtin_amdgcn_readfirstlane(slot);
  if (s0 >= 688u && s0 + 64u * B <= g.M) ring_appends<B, false>(Rg, g, s0, lane, vals);
  else ring_appends<B, true>(Rg, g, s0, lane, vals);
  slot = __builtin_amdgcn_readfirstlane(ring_wrap(s0 + 64u * B, g.M));
}

// NA appends as batches of three (one of one or two last).
// The final-state wave: CPython's final array (stream positions tf .. tf +
// 623) into a.fin, from the window at position P = a.final_pos (its word 0)
// onwards, and — when the call speculates on its successor (a.next_win,
// DN_MT_SPEC) — the window at position a.next_pos (>= tf): the next call's
// W_idx, the source of its jump levels.
__device__ __forceinline__ void final_state_wave(uint32_t* R, const GenRing& g, uint32_t slot, uint32_t lane,
                                                 const uint32_t* win, const GenArgs& a) {
  const uint64_t P = a.final_pos, tf = a.final_tf, nx = a.next_pos;
  uint32_t* nw = a.next_win;
  const uint64_t end = nw ? nx + kMtN : tf + kMtN;
  for (uint32_t i = lane; i < static_cast<uint32_t>(kMtN); i += 64u) {
    const uint64_t x = P + i;
    if (x >= tf && x < tf + kMtN) a.fin[x - tf] = win[i];
    if (nw && x >= nx && x < nx + kMtN) nw[x - nx] = win[i];
  }
  uint64_t np = P + kMtN;  // position of the next append's word 0
  while (np < end) {
    uint32_t v[3];
    ring_batch<3>(R, g, slot, lane, v);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint64_t x = np + 64u * k + lane;
      if (x >= tf && x < tf + kMtN) a.fin[x - tf] = v[k];
      if (nw && x >= nx && x < nx + kMtN) nw[x - nx] = v[k];
    }
    np += 192u;
  }
}

// The last substream's tail (tail_fin): CPython's final array (positions
// fin_lo .. fin_lo + 623 of the substream's frame) and, when the call
// speculates, the next call's W_idx (next_lo .., next_lo >= fin_lo), from the
// ring — which holds the substream's last M words, `end` being the position
// of the next append — and at most ten more appends.  The draw ends at
// next_lo, at most 624 words past fin_lo and at most a group before `end`, so
// every word needed is either still in the ring or appended here.
__device__ __forceinline__ void last_sub_tail(uint32_t* R, const GenRing& g, uint32_t slot, uint32_t lane, uint32_t end,
                                              const GenArgs& a) {
  const int32_t f0 = a.fin_lo, n0 = a.next_lo, e = static_cast<int32_t>(end);
  const int32_t off = static_cast<int32_t>(g.delta + g.M);  // slot of position x: (x + off) % M, x >= -624
  uint32_t* nw = a.next_win;
  for (int32_t i = static_cast<int32_t>(lane); i < kMtN; i += 64) {
    const int32_t x = f0 + i, y = n0 + i;
    if (x < e) a.fin[i] = R[g.o + static_cast<uint32_t>(x + off) % g.M];
    if (nw && y < e) nw[i] = R[g.o + static_cast<uint32_t>(y + off) % g.M];
  }
  const int32_t stop = (nw ? n0 : f0) + kMtN;
  for (int32_t p = e; p < stop; p += 64) {
    uint32_t v[3];
    ring_batch<1>(R, g, slot, lane, v);
    const int32_t x = p + static_cast<int32_t>(lane);
    if (x >= f0 && x < f0 + kMtN) a.fin[x - f0] = v[0];
    if (nw && x >= n0 && x < n0 + kMtN) nw[x - n0] = v[0];
  }
}

template <int NA>
__device__ __forceinline__ void ring_run(uint32_t* Rg, const GenRing& g, uint32_t& slot, uint32_t lane) {
  uint32_t v[3];
#pragma unroll
  for (int k = 0; k + 3 <= NA; k += 3) ring_batch<3>(Rg, g, slot, lane, v);
  if constexpr (NA % 3) ring_batch<NA % 3>(Rg, g, slot, lane, v);
}

// n appends, n known at run time (batches of three, then one or two).
__device__ __forceinline__ void ring_run_rt(uint32_t* Rg, const GenRing& g, uint32_t& slot, uint32_t lane,
                                            uint32_t n) {
  uint32_t v[3];
  uint32_t k = 0;
  for (; k + 3u <= n; k += 3u) ring_batch<3>(Rg, g, slot, lane, v);
  if (n - k == 2u) ring_batch<2>(Rg, g, slot, lane, v);
  else if (n - k == 1u) ring_batch<1>(Rg, g, slot, lane, v);
}

// The window (624 raw words at stream positions [p_start - 624, p_start))
// into the ring, with the mirror.
__device__ __forceinline__ void ring_init(uint32_t* Rg, const GenRing& g, const uint32_t* win, uint32_t p_start,
                                          uint32_t lane) {
  for (uint32_t i = lane; i < static_cast<uint32_t>(kMtN); i += 64u) {
    // slot of position p_start - 624 + i, in [0, M)
    const uint32_t s = (p_start + g.delta + g.M - static_cast<uint32_t>(kMtN) + i) % g.M;
    const uint32_t v = win[i];
    Rg[g.o + s] = v;
    if (s < 64u) Rg[g.o + g.M + s] = v;
  }
}

// ---- backward generation ----------------------------------------------------
// The word transition is invertible, so one jump window serves two
// substreams: substream s + 1 forward from W(s + 1) and substream s backward
// from it (W(s + 1) is the last 624 raw words of substream s).  Only windows
// of odd s (and of the last substream) are jumped to — half of level B.
// From word p + 624 = mix(x_p, x_{p+1}, x_{p+397}) with t_p = x_{p+624} ^
// x_{p+397} = (y >> 1) ^ (y odd ? A : 0), y = (x_p & UP) | (x_{p+1} & LO):
// A's top bit is set and y >> 1's is clear, so y's low bit is t_p's top bit and
// y = ((t_p ^ (that bit ? A : 0)) << 1) | bit.  x_p takes its top bit from y_p
// (bit 30 of t_p, A's bit 30 being clear) and its low 31 bits from y_{p-1}:
//   x_p = alignbit(bfi(2^30, t_p, t_{p-1} ^ (A & -(t_{p-1} >> 31))), t_{p-1}, 31)
// — six VALU over words p + 396, p + 397, p + 623 and p + 624.  A word needs
// none of the 395 words below it, so six 64-word blocks are independent.
__device__ __forceinline__ uint32_t mt_unmix(uint32_t x396, uint32_t x397, uint32_t x623, uint32_t x624) {
  const uint32_t t1 = x624 ^ x397, t0 = x623 ^ x396;
  const uint32_t m0 = static_cast<uint32_t>(static_cast<int32_t>(t0) >> 31);
  const uint32_t u0 = __builtin_amdgcn_bitop3_b32(m0, kMtA, t0, 0x6a);  // (m0 & A) ^ t0
  const uint32_t up = (0x40000000u & t1) | (~0x40000000u & u0);        // v_bfi_b32
  return __builtin_amdgcn_alignbit(up, t0, 31);
}

// B blocks below ring slot `top` (block i: slots [top - 64 (i + 1), top - 64 i),
// lane = word), reads first.  Backward substreams use delta = 0 (slot =
// position mod M).  WRAP: operand slots at or past M wrap (top > M - 624).
// PART: only slots below `lim` are written (the first block under the window).
template <int B, bool WRAP, bool PART>
__device__ __forceinline__ void back_blocks(uint32_t* Rg, uint32_t M, uint32_t top, uint32_t lane, uint32_t lim) {
  uint32_t q[B], x396[B], x397[B], x623[B], x624[B];
#pragma unroll
  for (int i = 0; i < B; ++i) {
    q[i] = top - 64u * (i + 1) + lane;
    if constexpr (WRAP) {
      auto w = [&](uint32_t s) { return Rg[s >= M ? s - M : s]; };
      x396[i] = w(q[i] + 396u);
      x397[i] = w(q[i] + 397u);
      x623[i] = w(q[i] + 623u);
      x624[i] = w(q[i] + 624u);
    } else {
      const uint32_t* p = Rg + q[i] + 396u;
      x396[i] = p[0];
      x397[i] = p[1];
      x623[i] = p[227];
      x624[i] = p[228];
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // every read issued before the first unmix waits
#pragma unroll
  for (int i = 0; i < B; ++i) {
    const uint32_t v = mt_unmix(x396[i], x397[i], x623[i], x624[i]);
    if (!PART || q[i] < lim) Rg[q[i]] = v;
  }
}

template <int B>
__device__ __forceinline__ void back_batch(uint32_t* Rg, uint32_t M, uint32_t& top, uint32_t lane) {
  const uint32_t t0 = __builtin_amdgcn_readfirstlane(top);
  if (t0 + 624u <= M) back_blocks<B, false, false>(Rg, M, t0, lane, 0u);
  else back_blocks<B, true, false>(Rg, M, t0, lane, 0u);
  top = t0 - 64u * B;
}

// NB blocks down from `top`, as batches of six (one shorter last); a run that
// ended at slot 0 continues from slot M.
template <int NB>
__device__ __forceinline__ void back_run(uint32_t* Rg, uint32_t M, uint32_t& top, uint32_t lane) {
  if (top == 0u) top = M;
#pragma unroll
  for (int k = 0; k + 6 <= NB; k += 6) back_batch<6>(Rg, M, top, lane);
  if constexpr (NB % 6) back_batch<NB % 6>(Rg, M, top, lane);
}

// A rejected draw: every writer stores the same nonzero word, so a plain
// store serves (no atomic: the flag may live in pinned host memory, where a
// device atomic would be a PCIe atomic).
__device__ __forceinline__ void mt_flag(const GenArgs& a) { __hip_atomic_store(a.flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

// 64 draws of one group (lane = draw c of this substream, raw words 17 c ..
// 17 c + 16 of the group at `rb`): temper, +1, rejection test, tiled store.
__device__ __forceinline__ void emit_group(const GenArgs& a, const uint32_t* rb, uint64_t qb, uint32_t rbm,
                                          uint32_t c, uint32_t nloc, uint32_t lane, bool mid = false) {
  if (c >= nloc) return;
  uint32_t v[kLimbs];  // (the group's ring slice is 64 draws of 17 words)
  const uint32_t* w = rb + 17u * lane;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) v[i] = w[i];
  if (mid) pc_barrier();  // mt_gen_pc_kernel: the producer may now overwrite this group's slots
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) v[i] = mt_temper(v[i]);
  v[16] >>= 23;
  uint32_t all = v[1];
#pragma unroll
  for (int i = 2; i < 16; ++i) all &= v[i];
  if (v[16] == 0x1FFu && v[0] >= 0xFFFFFFFEu && all == 0xFFFFFFFFu) mt_flag(a);  // >= p - 1: rejected
  uint32_t cy = 1u;  // + 1 (randint's lower bound); v < p - 1: no carry out of limb 16
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) v[i] = __builtin_addc(v[i], 0u, cy, &cy);
  // draw number of the whole stream = S0 + c with S0 = qb tm1 + rbm: element, row
  const uint32_t x = rbm + c;
  const uint32_t ex = static_cast<uint32_t>((static_cast<uint64_t>(x) * a.tm1_magic) >> 32);
  const uint32_t j = x - ex * static_cast<uint32_t>(a.tm1);
  const uint64_t e = qb + ex;
  uint8_t* tb = a.coeffs + j * a.vb + (e >> 8) * kTileBytes;
  const uint32_t wl = static_cast<uint32_t>(e & 255u);
#pragma unroll
  for (int i = 0; i < 16; ++i) __builtin_nontemporal_store(v[i], reinterpret_cast<uint32_t*>(tb) + i * kTile + wl);
  __builtin_nontemporal_store(static_cast<uint16_t>(v[16]), reinterpret_cast<uint16_t*>(tb + kHiOffset) + wl);
}

// Fused split (T = t): the 64 elements of one group (lane = element, 64 (t-1)
// consecutive draws of this substream, element-major as make_shares draws
// them: raw words 17 ((t-1) lane + j - 1) .. + 16 of the group for
// coefficient j), their int64 secrets, and the split of split_kernel<T,
// false, false>: the forward-difference table stored share by share.
// The group's coefficients (ring words of this lane's element, tempered, +1,
// rejection flagged) and secret s into the difference table c (fd_init).
template <int T>
__device__ __forceinline__ void emit_prepare(const GenArgs& a, const uint32_t* rb, uint32_t lane, uint64_t s,
                                             uint32_t (&c)[T][kLimbs], bool mid) {
  constexpr int TM1 = T - 1;
  const uint32_t* w = rb + 17u * TM1 * lane;
  if constexpr (TM1 % 2 == 0) {
    // an element's 17 (t-1) words start at an even word: 8-B reads, and with
    // a lane stride of 34 words (t = 3) the 32 lanes of a b64 group hit 32
    // distinct bank pairs (b32 reads at that stride are 2-way conflicted)
    uint32_t ww[17 * TM1];
#pragma unroll
    for (int k = 0; k < 17 * TM1 / 2; ++k) {
      const u32x2_t d = *reinterpret_cast<const u32x2_t*>(w + 2 * k);
      ww[2 * k] = d.x, ww[2 * k + 1] = d.y;
    }
    if (mid) pc_barrier();  // mt_gen_pc_kernel: the producer may now overwrite this group's slots
#pragma unroll
    for (int j = 1; j < T; ++j)
#pragma unroll
      for (int i = 0; i < kLimbs; ++i) c[j][i] = mt_temper(ww[17 * (j - 1) + i]);
  } else {
#pragma unroll
    for (int j = 1; j < T; ++j)
#pragma unroll
      for (int i = 0; i < kLimbs; ++i) c[j][i] = w[17 * (j - 1) + i];
    if (mid) pc_barrier();
#pragma unroll
    for (int j = 1; j < T; ++j)
#pragma unroll
      for (int i = 0; i < kLimbs; ++i) c[j][i] = mt_temper(c[j][i]);
  }
#pragma unroll
  for (int j = 1; j < T; ++j) {
    c[j][16] >>= 23;
    uint32_t all = c[j][1];
#pragma unroll
    for (int i = 2; i < 16; ++i) all &= c[j][i];
    if (c[j][16] == 0x1FFu && c[j][0] >= 0xFFFFFFFEu && all == 0xFFFFFFFFu) mt_flag(a);
    uint32_t cy = 1u;  // randint(1, p-1) = 1 + getrandbits(521)
#pragma unroll
    for (int i = 0; i < kLimbs; ++i) c[j][i] = __builtin_addc(c[j][i], 0u, cy, &cy);
  }
  c[0][0] = static_cast<uint32_t>(s);
  c[0][1] = static_cast<uint32_t>(s >> 32);
#pragma unroll
  for (int i = 2; i < kLimbs; ++i) c[0][i] = 0u;
  fd_init<T>(c);
}

template <int T, int SAUX, int NS, bool WHOLE>
__device__ __forceinline__ void emit_split(const GenArgs& a, const uint32_t* rb, uint64_t ebase, uint32_t lane,
                                           uint64_t s, bool mid = false) {
  // ebase (the group's first element) is wave-uniform and a multiple of 64, so
  // the group's 64 elements share one tile: its index is a scalar and every
  // share store takes the tile's buffer descriptor from SGPRs (no per-lane
  // descriptor, no waterfall loop around the stores)
  const uint32_t tile = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(ebase >> 8));
  const uint64_t e = ebase + lane;
  if (!WHOLE && e >= a.n_elem) return;  // WHOLE: every element of the group is in the vector
  uint32_t c[T][kLimbs];
  emit_prepare<T>(a, rb, lane, s, c, mid);
  const uint32_t wl = static_cast<uint32_t>(e & 255u);
  if constexpr (NS > 0) {
#pragma unroll
    for (int xi = 1; xi <= NS; ++xi) {
      store_reduced<SAUX>(tile_rsrc(tile_base(a.shares + static_cast<uint64_t>(xi - 1) * a.vb, tile)), wl, c[0]);
      if (xi < NS) fd_step<T>(c);
    }
  } else {
#pragma unroll 1
    for (int32_t xi = 1; xi <= a.n_shares; ++xi) {
      store_reduced<SAUX>(tile_rsrc(tile_base(a.shares + static_cast<uint64_t>(xi - 1) * a.vb, tile)), wl, c[0]);
      fd_step<T>(c);
    }
  }
}

// One 64-thread workgroup per substream (one extra for CPython's final state):
// T == 0 stores the coefficients (groups of 64 draws), T > 0 splits the
// substream's elements (groups of 64 elements) with them as they are drawn.
// Dynamic LDS: 1 + ring + 64 words (GenRing).
template <int T, int SAUX = kNt, int NS = 0>
__global__ void __launch_bounds__(64) mt_gen_kernel(const GenArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t sub = blockIdx.x + a.sub_lo;
  if (sub > a.S || (sub == a.S && a.final_sig < 0)) return;
  const bool fin_wave = sub == a.S;
  const bool fwd = fin_wave || mt_sub_forward(sub, a.S, static_cast<int>(a.back));
  const uint32_t sub_words = 17u * static_cast<uint32_t>(a.sub_draws);
  const uint32_t wsel = fin_wave ? static_cast<uint32_t>(a.final_sig) : fwd ? sub : sub + 1u;
  const uint32_t* win = a.wins + static_cast<uint64_t>(wsel) * kMtN;
  // positions of this substream: word 0 is its first output; the window holds
  // [p_start - 624, p_start) (substream 0: the caller's array, whose words
  // idx .. 623 are outputs 0 .. 623 - idx; a backward substream: its last 624
  // words, slots M - 624 .. M - 1 since the substream is a whole number of
  // ring lengths)
  const uint32_t p_start = (sub == 0 && !fin_wave) ? kMtN - a.idx : fwd ? 0u : sub_words;
  GenRing g;
  g.M = a.ring;
  g.delta = (64u - (p_start & 63u)) & 63u;
  g.o = g.delta & 1u;
  uint32_t* R = s_ring;
  ring_init(R, g, win, p_start, lane);
  uint32_t slot = __builtin_amdgcn_readfirstlane((p_start + g.delta) % g.M);  // slot of the next append
  wave_sync();
  if (fin_wave) {
    final_state_wave(R, g, slot, lane, win, a);
    return;
  }
  const uint32_t group = a.ring / 2u;                            // words per emission group
  const uint64_t k0 = static_cast<uint64_t>(sub) * a.sub_draws;  // first draw of this substream
  const uint32_t nloc = static_cast<uint32_t>(a.ncoef - k0 < a.sub_draws ? a.ncoef - k0 : a.sub_draws);
  const uint32_t gdraws = T ? 64u * (T - 1) : 64u;  // draws per group
  const uint32_t ngroups = (nloc + gdraws - 1u) / gdraws;
  const uint64_t qb = k0 / static_cast<uint64_t>(a.tm1);
  const uint32_t rbm = static_cast<uint32_t>(k0 - qb * static_cast<uint64_t>(a.tm1));
  constexpr int kRun = 17 * (T ? T - 1 : 1);  // appends per run = one group's words / 64
  static_assert(kRun > 10, "a group holds the 640 words under the window");
  if (!fwd) {
    // Backward: whole groups, all inside the vector (never the last
    // substream), last group first; group gi sits in ring half gi % 2
    // (ngroups is even, so the window is the top of half 1).  First the 16
    // words under the window (one block, masked), then the group's other
    // kRun - 10 blocks, then per group: emit it, generate the one below.
    const uint32_t M = a.ring;
    back_blocks<1, true, true>(R, M, M - 576u, lane, M - 624u);
    uint32_t top = M - 640u;
    back_run<kRun - 10>(R, M, top, lane);
    wave_sync();
    if constexpr (T == 0) {
      for (uint32_t gi = ngroups - 1u;; --gi) {
        emit_group(a, R + (gi & 1u) * group, qb, rbm, 64u * gi + lane, nloc, lane);
        if (gi == 0u) break;
        wave_sync();
        back_run<kRun>(R, M, top, lane);
        wave_sync();
      }
    } else {
      // the next (lower) group's secrets loaded before this group's share
      // stores, into one of two registers by parity (as the forward loop)
      const uint64_t e0 = qb + lane;
      auto secret_of = [&](uint32_t gi) {
        return static_cast<uint64_t>(__builtin_nontemporal_load(a.secrets + e0 + 64u * gi));
      };
      auto bstep = [&](uint32_t gi, uint64_t cur, uint64_t& nxt) {
        DN_PROBE_SKIP(a, 2u) back_run<kRun>(R, M, top, lane);
        wave_sync();
        nxt = secret_of(gi ? gi - 1u : 0u);
        DN_PROBE_SKIP(a, 1u)
        emit_split<T, SAUX, NS, true>(a, R + (gi & 1u) * group, qb + 64u * gi, lane, cur);
        wave_sync();
      };
      uint64_t secA = secret_of(ngroups - 1u), secB = secret_of(ngroups - 2u);
      DN_PROBE_SKIP(a, 1u)
      emit_split<T, SAUX, NS, true>(a, R + group, qb + 64u * (ngroups - 1u), lane, secA);
      wave_sync();
      for (uint32_t gi = ngroups - 2u;; gi -= 2u) {
        bstep(gi, secB, secA);
        if (gi == 0u) break;
        bstep(gi - 1u, secA, secB);
        if (gi == 1u) break;
      }
      asm volatile("" : : "v"(secA ^ secB));  // no load left in flight at the end
    }
    return;
  }
  // Every run appends exactly one group's words (have = p_start + runs * group
  // with p_start < group), so each run is followed by exactly one emission.
  if constexpr (T == 0) {
    for (uint32_t done = 0; done < ngroups; ++done) {
      DN_PROBE_SKIP(a, 2u) ring_run<kRun>(R, g, slot, lane);
      wave_sync();
      DN_PROBE_SKIP(a, 1u)
      emit_group(a, R + g.o + g.delta + (done & 1u) * group, qb, rbm, 64u * done + lane, nloc, lane);
      wave_sync();
    }
    if (a.tail_fin && sub + 1u == a.S) last_sub_tail(R, g, slot, lane, p_start + ngroups * group, a);
  } else {
    // The int64 secret of this lane's element in the next group is loaded a
    // group ahead — before the current group's share stores, since loads and
    // stores retire in issue order and a load issued after them would wait for
    // them — into one of two registers by group parity (no copy of a pending
    // load), from an index clamped to the vector (the last prefetch is unused).
    // With the share count a template argument (NS) and only whole groups
    // (all 64 elements in the vector) in the loop, the share stores are
    // straight-line code on every path and the wait before a prefetched
    // secret's use leaves them in flight (vmcnt(63)); a runtime share loop or a
    // lane-masked emission gets vmcnt(<= 1).  A last partial group is emitted
    // after the loop, with a secret loaded at that point.
    const uint64_t e0 = qb + lane;  // k0 / (t-1) = the substream's first element
    const uint64_t elast = a.n_elem - 1u;
    auto secret_of = [&](uint32_t gi) {
      const uint64_t e = e0 + 64u * gi;
      return static_cast<uint64_t>(__builtin_nontemporal_load(a.secrets + (e < elast ? e : elast)));
    };
    const uint64_t rem = a.n_elem - qb;  // elements from this substream's first one to the vector's end
    const uint32_t nfull = rem >= 64ull * ngroups ? ngroups : static_cast<uint32_t>(rem / 64u);
    auto step = [&](uint32_t gi, uint64_t cur, uint64_t& nxt) {
      DN_PROBE_SKIP(a, 2u) ring_run<kRun>(R, g, slot, lane);
      wave_sync();
      nxt = secret_of(gi + 1u);
      DN_PROBE_SKIP(a, 1u)
      emit_split<T, SAUX, NS, true>(a, R + g.o + g.delta + (gi & 1u) * group, qb + 64u * gi, lane, cur);
      wave_sync();
    };
    uint64_t secA = secret_of(0), secB = 0;
    uint32_t gi = 0;
    if (nfull > 0u) {
      step(0u, secA, secB);
      gi = 1u;
      for (; gi + 1u < nfull; gi += 2u) {
        step(gi, secB, secA);
        step(gi + 1u, secA, secB);
      }
      if (gi < nfull) {
        step(gi, secB, secA);
        ++gi;
      }
    }
    if (gi < ngroups) {  // the vector's last, partial group
      ring_run<kRun>(R, g, slot, lane);
      wave_sync();
      emit_split<T, SAUX, NS, false>(a, R + g.o + g.delta + (gi & 1u) * group, qb + 64u * gi, lane, secret_of(gi));
    }
    asm volatile("" : : "v"(secA ^ secB));  // no load left in flight at the end
    if (a.tail_fin && sub + 1u == a.S) {
      wave_sync();
      last_sub_tail(R, g, slot, lane, p_start + ngroups * group, a);
    }
  }
}

// The fused draw + split with generation and emission on separate waves: a
// 128-thread workgroup per substream, wave 1 (producer) appends group i + 1
// to the LDS ring while wave 0 (consumer) emits group i (temper, split, the
// share stores), one workgroup barrier per group.  A group's words depend on
// the 624 words before it only (a group is 2176 words or more), so the
// producer writes the ring half the consumer emitted one step earlier while
// both read the other: the emission (at the share block's write rate) no
// longer waits for the generation, which in mt_gen_kernel's one wave per
// substream runs between two emissions (r04i: full 1.02 ms, emission alone
// 0.93, generation alone 0.50 at 2^24 3-of-5 on a share block).  Backward
// substreams the same way downwards.  Same output and final state as
// mt_gen_kernel<T> (T = 2, 3, 5; T = 0 the coefficient draw, whose consumer
// stores the tempered draws instead of splitting).
// Dynamic LDS as mt_gen_kernel; registers for 4 waves per SIMD (8 workgroups
// per CU, the most the rings' LDS allows at t <= 3), 2 at t = 5 (4 fit).
template <int T, int SAUX = kNt, int NS = 0>
__global__ void __launch_bounds__(128, T == 5 ? 2 : 4) mt_gen_pc_kernel(const GenArgs a) {
  static_assert(T == 0 || T >= 2, "coefficient draw or fused split");
  extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
  const uint32_t lane = threadIdx.x & 63u;
  // (roles alternating with the workgroup's parity: no faster, profiles/r04/l/)
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // 0 consumer, 1 producer
  const uint32_t sub = blockIdx.x + a.sub_lo;
  if (sub > a.S || (sub == a.S && a.final_sig < 0)) return;
  const bool fin_wave = sub == a.S;
  const bool fwd = fin_wave || mt_sub_forward(sub, a.S, static_cast<int>(a.back));
  const uint32_t sub_words = 17u * static_cast<uint32_t>(a.sub_draws);
  const uint32_t wsel = fin_wave ? static_cast<uint32_t>(a.final_sig) : fwd ? sub : sub + 1u;
  const uint32_t* win = a.wins + static_cast<uint64_t>(wsel) * kMtN;
  const uint32_t p_start = (sub == 0 && !fin_wave) ? kMtN - a.idx : fwd ? 0u : sub_words;
  GenRing g;
  g.M = a.ring;
  g.delta = (64u - (p_start & 63u)) & 63u;
  g.o = g.delta & 1u;
  uint32_t* R = s_ring;
  uint32_t slot = __builtin_amdgcn_readfirstlane((p_start + g.delta) % g.M);  // producer: slot of the next append
  if (fin_wave) {
    if (wid != 0u) return;  // one wave steps to CPython's final array (as mt_gen_kernel)
    ring_init(R, g, win, p_start, lane);
    wave_sync();
    final_state_wave(R, g, slot, lane, win, a);
    return;
  }
  const uint32_t group = a.ring / 2u;
  const uint64_t k0 = static_cast<uint64_t>(sub) * a.sub_draws;
  const uint32_t nloc = static_cast<uint32_t>(a.ncoef - k0 < a.sub_draws ? a.ncoef - k0 : a.sub_draws);
  constexpr uint32_t gdraws = T ? 64u * (T - 1) : 64u;
  const uint32_t ngroups = (nloc + gdraws - 1u) / gdraws;
  const uint64_t qb = k0 / static_cast<uint64_t>(a.tm1);
  const uint32_t rbm = static_cast<uint32_t>(k0 - qb * static_cast<uint64_t>(a.tm1));
  constexpr int kRun = 17 * (T ? T - 1 : 1);
  static_assert(kRun > 10, "a group holds the 640 words under the window");
  const bool prod = wid == 1u;
  // The two waves run separate loops with the same number of barriers (one
  // per step, ngroups + 1 steps), so the consumer's secrets stay in two
  // registers by group parity as in mt_gen_kernel: no copy of a pending load
  // (a copy waits vmcnt(0), i.e. for every share store in flight).
  if (!fwd) {
    // backward (whole groups, ngroups even; group gi in ring half gi % 2):
    // the producer fills the top group under the window, then per step
    // generates group gi - 1 while the consumer emits group gi
    const uint32_t M = a.ring;
    if (prod) {
      uint32_t top = M - 640u;
      ring_init(R, g, win, p_start, lane);
      wave_sync();
      back_blocks<1, true, true>(R, M, M - 576u, lane, M - 624u);
      back_run<kRun - 10>(R, M, top, lane);
      pc_barrier();
      for (uint32_t gi = ngroups - 1u; gi > 0u; --gi) {
        DN_PROBE_SKIP(a, 2u) back_run<kRun>(R, M, top, lane);
        pc_barrier();
      }
      pc_barrier();
      return;
    }
    if constexpr (T == 0) {
      pc_barrier();  // the top group is in the ring
      for (uint32_t gi = ngroups - 1u;; --gi) {
        DN_PROBE_SKIP(a, 1u) emit_group(a, R + (gi & 1u) * group, qb, rbm, 64u * gi + lane, nloc, lane);
        pc_barrier();
        if (gi == 0u) break;
      }
    } else {
    const uint64_t e0 = qb + lane;
    auto secret_of = [&](uint32_t gi) {
      return static_cast<uint64_t>(__builtin_nontemporal_load(a.secrets + e0 + 64u * gi));
    };
    auto bstep = [&](uint32_t gi, uint64_t cur, uint64_t& nxt) {
      nxt = secret_of(gi ? gi - 1u : 0u);
      DN_PROBE_SKIP(a, 1u)
      emit_split<T, SAUX, NS, true>(a, R + (gi & 1u) * group, qb + 64u * gi, lane, cur);
      pc_barrier();
    };
    uint64_t secA = secret_of(ngroups - 1u), secB = 0;
    pc_barrier();  // the top group is in the ring
    for (uint32_t gi = ngroups - 1u;; gi -= 2u) {
      bstep(gi, secA, secB);
      bstep(gi - 1u, secB, secA);
      if (gi == 1u) break;
    }
    asm volatile("" : : "v"(secA ^ secB));  // no load left in flight at the end
    }
    return;
  }
  // forward: step i generates group i (producer) and emits group i - 1 (consumer).
  // Substream 0 starting inside the caller's array (p_start > 0) is the one
  // place a run reaches past its group: run i ends with the first p_start
  // words of group i + 1, whose ring slots are group i - 1's, which the
  // consumer is emitting.  There each step has a second barrier: the consumer
  // passes it once group i - 1's words are in its registers, the producer
  // before the blocks from `kstar` on (the first one holding a word of group i
  // + 1).
  const bool mid = sub == 0u && p_start > 0u;
  const uint32_t kstar = mid ? (group - p_start) / 64u : static_cast<uint32_t>(kRun);
#ifdef DN_TUNING
  const bool skip_emit = (a.probe & 1u) != 0u, skip_gen = (a.probe & 2u) != 0u;
#else
  constexpr bool skip_emit = false, skip_gen = false;
#endif
  if (prod) {
    ring_init(R, g, win, p_start, lane);
    wave_sync();
    for (uint32_t i = 0; i < ngroups; ++i) {
      if (mid) {
        if (!skip_gen) ring_run_rt(R, g, slot, lane, kstar);
        pc_barrier();
        if (!skip_gen) ring_run_rt(R, g, slot, lane, static_cast<uint32_t>(kRun) - kstar);
      } else if (!skip_gen) {
        ring_run<kRun>(R, g, slot, lane);
      }
      pc_barrier();
    }
    if (mid) pc_barrier();
    pc_barrier();  // the consumer has read its last group: the ring is the producer's
    if (a.tail_fin && sub + 1u == a.S) last_sub_tail(R, g, slot, lane, p_start + ngroups * group, a);
    return;
  }
  if constexpr (T == 0) {
    if (mid) pc_barrier();
    pc_barrier();  // group 0 is in the ring
    for (uint32_t gi = 0; gi < ngroups; ++gi) {
      if (!skip_emit) emit_group(a, R + g.o + g.delta + (gi & 1u) * group, qb, rbm, 64u * gi + lane, nloc, lane, mid);
      else if (mid) pc_barrier();
      pc_barrier();
    }
  } else {
  const uint64_t e0 = qb + lane;
  const uint64_t elast = a.n_elem - 1u;
  auto secret_of = [&](uint32_t gi) {
    const uint64_t e = e0 + 64u * gi;
    return static_cast<uint64_t>(__builtin_nontemporal_load(a.secrets + (e < elast ? e : elast)));
  };
  const uint64_t rem = a.n_elem - qb;
  const uint32_t nfull = rem >= 64ull * ngroups ? ngroups : static_cast<uint32_t>(rem / 64u);
  auto cstep = [&](uint32_t gi, uint64_t cur, uint64_t& nxt) {
    nxt = secret_of(gi + 1u);
    if (!skip_emit)
      emit_split<T, SAUX, NS, true>(a, R + g.o + g.delta + (gi & 1u) * group, qb + 64u * gi, lane, cur, mid);
    else if (mid)
      pc_barrier();
    pc_barrier();
  };
  uint64_t secA = secret_of(0), secB = 0;
  if (mid) pc_barrier();
  pc_barrier();  // group 0 is in the ring
  uint32_t gi = 0;
  for (; gi + 1u < nfull; gi += 2u) {
    cstep(gi, secA, secB);
    cstep(gi + 1u, secB, secA);
  }
  if (gi < nfull) {
    cstep(gi, secA, secB);
    ++gi;
  }
  if (gi < ngroups) {  // the vector's last, partial group
    emit_split<T, SAUX, NS, false>(a, R + g.o + g.delta + (gi & 1u) * group, qb + 64u * gi, lane, secret_of(gi),
                                   mid);
    pc_barrier();
  }
  asm volatile("" : : "v"(secA ^ secB));
  }
}

uint64_t mt_subs(uint64_t ncoef) {
  const uint64_t d = mt_sub_draws(mt_sub_len(ncoef));
  return (ncoef + d - 1) / d;
}

constexpr int32_t kFullSpan = kMtPolyWords << 16;  // words [0, 312)
constexpr uint64_t kPartRows = 4096;  // part windows of one split level (jumps x parts <= 4096)

// The jobs of one level: W waves per workgroup (one job each; padding jobs
// have dst -1), grouped by source window and part (one table per workgroup).
struct Level {
  int W = 8;
  std::vector<JumpJob> jobs;
  std::vector<CombineJob> comb;
};

void push_group(Level& L, int32_t src, const std::vector<std::pair<int32_t, int32_t>>& pd, int32_t span) {
  for (size_t i = 0; i < pd.size(); ++i) L.jobs.push_back({src, pd[i].first, pd[i].second, span});
  while (L.jobs.size() % static_cast<size_t>(L.W)) L.jobs.push_back({src, 0, -1, span});
}

// a source's jobs in groups of at most `per`
void push_groups(Level& L, int32_t src, const std::vector<std::pair<int32_t, int32_t>>& pd, size_t per,
                 int32_t span = kFullSpan) {
  for (size_t i = 0; i < pd.size(); i += per)
    push_group(L, src, std::vector<std::pair<int32_t, int32_t>>(pd.begin() + i, pd.begin() + std::min(pd.size(), i + per)),
               span);
}

// One level: (source, [(poly, dst)]) lists of n jumps in all.  A jump's
// Horner chain is ~312 dependent steps of LDS-table reads, so the level is
// latency-bound unless every CU holds many waves.  The level therefore splits
// each jump into P = min(16, 4096 / n) parts over word ranges of g (n P part
// jobs, each ~312 / P steps, written to part rows prow0 .. and XORed into the
// jump's window by mt_combine_kernel) and groups per = clamp(n P / 256, 2,
// 16) part jobs of one source and part per workgroup (one table): ~256
// workgroups, one per CU (82 KB of LDS each), 2..16 waves.  Large levels
// (n >= 4096) stay whole, 16 jumps per workgroup.
// Word ranges [cut[j], cut[j + 1]) of g for at most P parts.  A part costs
// its Horner steps — whole runs of 11 words (jump_run), the words above g's
// top included — plus the stepping of its source stream to word 64 lo, about
// r runs' worth per word of lo (r ~ 0.053 / 11 for 8-wave workgroups, ~0.014 / 11
// for 16-wave ones: profiles/r03/ab/jump_probe/).  Parts nearer the top of g
// start further down the stream, so they get fewer runs: the smallest cost
// bound T (in steps) the greedy split meets with at most P parts.
std::vector<int32_t> part_cuts(int P, int W) {
  const double r = W >= 16 ? 0.014 : 0.053;  // stepping cost per word of lo, in Horner steps
  const int runs_total = (kMtPolyWords + 10) / 11;
  for (int T = 11; ; T += 1) {
    std::vector<int32_t> cut{0};
    while (cut.back() < kMtPolyWords && static_cast<int>(cut.size()) <= P) {
      const int lo = cut.back();
      const int runs = static_cast<int>((T - r * lo) / 11.0);
      if (runs < 1) break;
      cut.push_back(std::min(kMtPolyWords, lo + 11 * runs));
    }
    if (cut.back() >= kMtPolyWords && static_cast<int>(cut.size()) - 1 <= P) return cut;
    if (T > 11 * runs_total + 1000) break;
  }
  std::vector<int32_t> cut;  // unreachable: one part of all the words
  for (int j = 0; j <= P; ++j) cut.push_back(kMtPolyWords * j / P);
  return cut;
}

void push_level(Level& L, const std::vector<std::pair<int32_t, std::vector<std::pair<int32_t, int32_t>>>>& srcs,
                int32_t prow0, int p_force = 0, int w_force = 0) {
  size_t n = 0, most = 0;  // jumps, and the most of one source
  for (auto& sp : srcs) n += sp.second.size(), most = std::max(most, sp.second.size());
  if (n == 0) return;
  int P = static_cast<int>(std::max<size_t>(1, std::min<size_t>(kMaxParts, kPartRows / n)));
  if (p_force > 0) P = std::min(p_force, kMaxParts);
  // DN_MT_PARTS_B (tuning build): the part count of levels of 256 jumps or more
  const char* pb = n >= 256 ? tune_env("DN_MT_PARTS_B") : nullptr;
  if (pb && std::atoi(pb) >= 1) P = std::min(kMaxParts, std::atoi(pb));
  size_t per = std::min<size_t>(kJumpWaves, std::max<size_t>(2, (n * P + 255) / 256));
  L.W = std::min(per, most) > 8 ? 16 : 8;
  if (w_force > 0) L.W = w_force, per = static_cast<size_t>(w_force);  // (mt_jumpc_kernel's workgroups)
  if (P == 1) {
    for (auto& sp : srcs) push_groups(L, sp.first, sp.second, per);
    return;
  }
  const std::vector<int32_t> cut = part_cuts(P, L.W);
  P = static_cast<int>(cut.size()) - 1;
  int32_t row = prow0;
  for (auto& sp : srcs)
    for (auto& pd : sp.second) {
      L.comb.push_back({pd.second, row, P, 0});
      row += P;
    }
  for (int j = 0; j < P; ++j) {
    const int32_t lo = cut[j], hi = cut[j + 1];
    row = prow0 + j;
    for (auto& sp : srcs) {
      std::vector<std::pair<int32_t, int32_t>> pd;
      for (auto& q : sp.second) {
        pd.push_back({q.first, row});
        row += P;
      }
      push_groups(L, sp.first, pd, per, lo | hi << 16);
    }
  }
}

// Levels for windows 1 .. S-1 (s - 1 = 4096 c + 64 a + b; row S holds W_idx;
// part rows from S + 1) with the jump table of substream length ki:
// A: W(1 + 64 a) = A_a(W_idx); C: W(1 + 4096 c + 64 a) = C_c(W(1 + 64 a));
// B: W(base + b) = B_b(W(base)).  back: only the windows a generation wave
// starts from (mt_sub_forward: odd s, the last one) — A and C windows are odd.
// rt: one direct level through the runtime rows (host_gf2poly.cpp) for the
// draws of up to kMtRtRows + 1 substreams of 2^14 draws that generate
// backward: the 1024 windows of a 2^24-element 3-of-5 draw in one level of
// ~150 us instead of level A (~28 us), its combine and level B (~148 us).
// The first substream of split2's second half: even, so the first half's
// last substream (odd) runs forward from a window of the first half, and every
// even substream runs backward from a window of its own half.
inline uint64_t mt_split_half(uint64_t S) { return (S / 2 + 1) & ~1ull; }

// split2 (DN_MT_SPLIT2): the runtime direct level as two levels, the windows
// of substreams [0, S/2) and of [S/2, S), at the whole level's part count, so
// the first half's generation can start while the second half's jumps run.
void build_levels(uint64_t S, int ki, int back, bool rt, Level lv[3], bool split2 = false) {
  const uint64_t R = kMtJumpRadix;
  if (S < 2) return;
  const uint64_t last = S - 2;  // largest s - 1
  const int32_t prow0 = static_cast<int32_t>(S + 1);
  if (rt && split2) {
    const uint64_t half = mt_split_half(S);
    std::vector<std::pair<int32_t, int32_t>> pd1, pd2;
    for (uint64_t s = 1; s < S; ++s)
      if (mt_window_needed(static_cast<uint32_t>(s), S, back))
        (s < half ? pd1 : pd2).push_back({kMtRtBase + static_cast<int32_t>(s - 1), static_cast<int32_t>(s)});
    const int P = static_cast<int>(std::max<size_t>(1, std::min<size_t>(kMaxParts, kPartRows / (pd1.size() + pd2.size()))));
    push_level(lv[0], {{-1, pd1}}, prow0, P);
    int32_t prow1 = prow0;
    for (auto& c : lv[0].comb) prow1 = std::max(prow1, c.first + c.parts);
    push_level(lv[1], {{-1, pd2}}, prow1, P);
    return;
  }
  if (rt) {
    std::vector<std::pair<int32_t, int32_t>> pd;
    for (uint64_t s = 1; s < S; ++s)
      if (mt_window_needed(static_cast<uint32_t>(s), S, back))
        pd.push_back({kMtRtBase + static_cast<int32_t>(s - 1), static_cast<int32_t>(s)});
    push_level(lv[0], {{-1, pd}}, prow0);
    return;
  }
  if (last < static_cast<uint64_t>(kMtDirectRows)) {
    // every window one jump from W_idx: W(s) = D_s(W_idx), one level
    std::vector<std::pair<int32_t, int32_t>> pd;
    for (uint64_t s = 1; s < S; ++s)
      if (mt_window_needed(static_cast<uint32_t>(s), S, back))
        pd.push_back({kMtDirectBase + ki * kMtDirectRows + static_cast<int32_t>(s - 1), static_cast<int32_t>(s)});
    push_level(lv[0], {{-1, pd}}, prow0);
    return;
  }
  const int32_t t0 = ki * kMtJumpRows;  // the table's first row
  {
    std::vector<std::pair<int32_t, int32_t>> pd;
    for (uint64_t a = 0; a <= last / R && a < R; ++a)
      pd.push_back({t0 + kMtRowA + static_cast<int32_t>(a), static_cast<int32_t>(1 + R * a)});
    push_level(lv[0], {{-1, pd}}, prow0);  // source: W_idx, the row before row 0
  }
  {
    std::vector<std::pair<int32_t, std::vector<std::pair<int32_t, int32_t>>>> srcs;
    for (uint64_t a = 0; a < R && R * a <= last; ++a) {  // C: per source W(1 + 64 a), its c digits
      std::vector<std::pair<int32_t, int32_t>> pd;
      for (uint64_t c = 1; c < R && R * R * c + R * a <= last; ++c)
        pd.push_back({t0 + kMtRowC + static_cast<int32_t>(c), static_cast<int32_t>(1 + R * R * c + R * a)});
      if (!pd.empty()) srcs.push_back({static_cast<int32_t>(1 + R * a), pd});
    }
    push_level(lv[1], srcs, prow0);
  }
  {
    std::vector<std::pair<int32_t, std::vector<std::pair<int32_t, int32_t>>>> srcs;
    for (uint64_t base = 0; base <= last; base += R) {  // B: per source W(1 + base)
      std::vector<std::pair<int32_t, int32_t>> pd;
      for (uint64_t b = 1; b < R && base + b <= last; ++b)
        if (mt_window_needed(static_cast<uint32_t>(1 + base + b), S, back))
          pd.push_back({t0 + kMtRowB + static_cast<int32_t>(b), static_cast<int32_t>(1 + base + b)});
      if (!pd.empty()) srcs.push_back({static_cast<int32_t>(1 + base), pd});
    }
    push_level(lv[2], srcs, prow0);
  }
}

// Per-thread host side of a draw: the job tables of the last substream count
// and length (they depend on S and ki only; plain host memory, freed with the
// thread).
struct MtHost {
  uint64_t S = ~0ull;
  int ki = -1;
  int back = 0;
  int parts_b = 0;  // tuning build: DN_MT_PARTS_B the levels were built with
  bool rt = false;  // one direct level through the runtime rows
  bool split2 = false;  // that level in two halves (DN_MT_SPLIT2)
  Level lv[3];
  Level beside;  // rt: the direct level for mt_jumpc_kernel<4, 2> (whole jumps, 4 per workgroup)
  Level j0;      // rt: one jump, row S -> row -1 by x^(17 ncoef) (the rt pointer), in parts, mt_jumpc_kernel<4, 2>
  std::vector<uint32_t> jobs;  // the levels' jobs, their combine jobs, beside's jobs, j0's jobs and combine job
  uint64_t beside_off = 0, j0_off = 0, j0_comb_off = 0;  // word offsets in `jobs`
  uint64_t part_rows = 0;      // part windows the largest split level writes (levels reuse them)
};
thread_local MtHost tls_mt;

// Backward generation of the even substreams (on; DN_MT_BACK=0 in the tuning
// build turns it off for A/B).
int mt_back() {
  const char* e = tune_env("DN_MT_BACK");
  return e ? (e[0] == '0' ? 0 : e[0] == '2' ? 2 : 1) : 1;
}

MtHost& mt_levels(uint64_t S, int ki) {
  MtHost& H = tls_mt;
  // 2^8-draw substreams run forward only: at t = 5 one holds a single
  // emission group, and backward generation needs an even count (its window
  // is the top of ring half 1); their one direct level takes the extra jumps
  const int back = ki == 3 ? 0 : mt_back();
  const char* pb = tune_env("DN_MT_PARTS_B");
  const int parts_b = pb ? std::atoi(pb) : 0;
  // the runtime direct level: 2^14-draw substreams generating backward, more
  // than the tabulated direct rows cover, at most kMtRtRows + 1 of them, and
  // rows available on this host (DN_MT_RT=0, tuning build: off)
  const char* rte = tune_env("DN_MT_RT");
  const bool rt = DN_MT_RT_DIRECT && !(rte && rte[0] == '0') && ki == 2 && back == 1 &&
                  S - 1 > static_cast<uint64_t>(kMtDirectRows) && S - 1 <= kMtRtRows &&
                  mt_direct_rows_l14(S, nullptr) != nullptr;
  const char* sp = tune_env("DN_MT_SPLIT2");
  const bool split2 = rt && (sp ? sp[0] == '1' : DN_MT_SPLIT2 != 0) && S >= 4;
  if (H.S != S || H.ki != ki || H.back != back || H.parts_b != parts_b || H.rt != rt || H.split2 != split2) {
    for (auto& l : H.lv) l = Level();
    build_levels(S, ki, back, rt, H.lv, split2);
    H.beside = Level();
    H.j0 = Level();
    if (rt && !split2) {
      std::vector<std::pair<int32_t, int32_t>> pd;
      for (uint64_t s = 1; s < S; ++s)
        if (mt_window_needed(static_cast<uint32_t>(s), S, back))
          pd.push_back({kMtRtBase + static_cast<int32_t>(s - 1), static_cast<int32_t>(s)});
      push_level(H.beside, {{-1, pd}}, static_cast<int32_t>(S + 1), 1, 4);
    }
    // the next call's W_idx for a speculation beside the generation (any
    // shape with jump levels: the levels of a small generation run beside it
    // as they are, mt_device_run)
    if (!split2 && S >= 2)
      push_level(H.j0, {{static_cast<int32_t>(S), {{kMtRtBase, -1}}}}, static_cast<int32_t>(S + 1), kMaxParts, 4);
    uint64_t nj = 0, nc = 0;
    for (auto& l : H.lv) nj += l.jobs.size(), nc += l.comb.size();
    nj += H.beside.jobs.size() + H.j0.jobs.size();
    nc += H.j0.comb.size();
    H.part_rows = 0;
    for (auto& l : H.lv)
      for (auto& c : l.comb) H.part_rows = std::max<uint64_t>(H.part_rows, c.first + c.parts - (S + 1));
    for (auto& c : H.j0.comb) H.part_rows = std::max<uint64_t>(H.part_rows, c.first + c.parts - (S + 1));
    H.jobs.assign((nj * sizeof(JumpJob) + nc * sizeof(CombineJob)) / 4, 0u);
    uint64_t o = 0;
    for (auto& l : H.lv) {
      std::memcpy(H.jobs.data() + o, l.jobs.data(), l.jobs.size() * sizeof(JumpJob));
      o += l.jobs.size() * sizeof(JumpJob) / 4;
    }
    for (auto& l : H.lv) {
      std::memcpy(H.jobs.data() + o, l.comb.data(), l.comb.size() * sizeof(CombineJob));
      o += l.comb.size() * sizeof(CombineJob) / 4;
    }
    H.beside_off = o;
    std::memcpy(H.jobs.data() + o, H.beside.jobs.data(), H.beside.jobs.size() * sizeof(JumpJob));
    o += H.beside.jobs.size() * sizeof(JumpJob) / 4;
    H.j0_off = o;
    std::memcpy(H.jobs.data() + o, H.j0.jobs.data(), H.j0.jobs.size() * sizeof(JumpJob));
    o += H.j0.jobs.size() * sizeof(JumpJob) / 4;
    H.j0_comb_off = o;
    std::memcpy(H.jobs.data() + o, H.j0.comb.data(), H.j0.comb.size() * sizeof(CombineJob));
    H.S = S;
    H.ki = ki;
    H.back = back;
    H.parts_b = parts_b;
    H.rt = rt;
    H.split2 = split2;
  }
  return H;
}

// Pinned staging buffers for a draw's small copies (from pageable memory HIP
// stages every copy through a buffer of its own and the host waits for it).
// A process-wide pool: a call leases one for its duration — every call
// synchronises its stream before it returns, so the buffer is idle again —
// and gives it back, so the pool holds as many buffers as calls ever ran at
// once, whatever number of threads made them.  The pool is never destroyed
// (the HIP runtime may be torn down before static destructors run).
struct PinPool {
  std::mutex m;
  std::vector<std::pair<uint32_t*, size_t>> idle;
};
PinPool& pin_pool() {
  static PinPool* pool = new PinPool;
  return *pool;
}

struct PinLease {
  uint32_t* p = nullptr;
  size_t words = 0;
  explicit PinLease(size_t need) {
    PinPool& pool = pin_pool();
    {
      std::lock_guard<std::mutex> g(pool.m);
      if (!pool.idle.empty()) {
        auto it = std::max_element(pool.idle.begin(), pool.idle.end(),
                                   [](const auto& a, const auto& b) { return a.second < b.second; });
        p = it->first;
        words = it->second;
        pool.idle.erase(it);
      }
    }
    if (words < need) {
      if (p) (void)hipHostFree(p);
      void* q = nullptr;
      p = hipHostMalloc(&q, need * 4, hipHostMallocDefault) == hipSuccess ? static_cast<uint32_t*>(q) : nullptr;
      words = p ? need : 0;
    }
  }
  ~PinLease() {
    if (!p) return;
    PinPool& pool = pin_pool();
    std::lock_guard<std::mutex> g(pool.m);
    pool.idle.push_back({p, words});
  }
  PinLease(const PinLease&) = delete;
  PinLease& operator=(const PinLease&) = delete;
};

constexpr uint64_t kHead = 2816;  // flag (4 B at 0), final array (2496 B at 256), pad to 256 B

// DN_MT_HOST_HEAD = 1: the generation writes the flag and CPython's final
// array straight into the call's pinned staging buffer (mapped host memory,
// visible once the stream has synchronised) instead of the scratch head and
// a device-to-host copy after it.
// (make_shares_vec 2^12 -1.5 us: no read-back copy; profiles/r04/e/)
#ifndef DN_MT_HOST_HEAD
#define DN_MT_HOST_HEAD 1
#endif

// The levels' job tables on the device, one upload per (device, shape): they
// depend on (S, ki, back, parts) only, so a call copies just its own state
// (head, W_idx, row 0: ~7.8 KB — a blit, where the job tables of a large draw
// went by SDMA and the first jump waited ~11-14 us on its completion signal;
// profiles/r04/c/msv_timeline.json).  Library-owned, never freed (a few KB to
// ~100 KB per shape; the runtime may be torn down before static destructors).
struct DevJobs {
  int dev;
  uint64_t S;
  int ki, back, parts_b;
  bool rt, split2;
  void* p;
};

const void* device_jobs(const MtHost& H, int* err) {
  static std::mutex* m = new std::mutex;
  static auto* cache = new std::vector<DevJobs>;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    *err = 1;
    return nullptr;
  }
  std::lock_guard<std::mutex> g(*m);
  for (const DevJobs& d : *cache)
    if (d.dev == dev && d.S == H.S && d.ki == H.ki && d.back == H.back && d.parts_b == H.parts_b && d.rt == H.rt &&
        d.split2 == H.split2)
      return d.p;
  void* p = nullptr;
  const size_t bytes = std::max<size_t>(H.jobs.size() * 4, 16);
  if (hipMalloc(&p, bytes) != hipSuccess ||
      (!H.jobs.empty() && hipMemcpy(p, H.jobs.data(), H.jobs.size() * 4, hipMemcpyHostToDevice) != hipSuccess)) {
    if (p) (void)hipFree(p);
    *err = 1;
    return nullptr;
  }
  cache->push_back({dev, H.S, H.ki, H.back, H.parts_b, H.rt, H.split2, p});
  return p;
}

// The runtime direct rows on the device: one kMtRtRows-row buffer per device,
// rows copied when the host has computed rows the device copy lacks (rows are
// only ever added, never changed).  Library-owned, never freed (5.1 MB).
struct DevRt {
  int dev;
  uint64_t* p;
  uint64_t version, rows;
};

const uint64_t* device_rt(uint64_t S, int* err) {
  static std::mutex* m = new std::mutex;
  static auto* cache = new std::vector<DevRt>;
  uint64_t version = 0;
  const uint64_t* host = mt_direct_rows_l14(S, &version);
  int dev = 0;
  if (!host || hipGetDevice(&dev) != hipSuccess) {
    *err = 1;
    return nullptr;
  }
  std::lock_guard<std::mutex> g(*m);
  DevRt* d = nullptr;
  for (DevRt& c : *cache)
    if (c.dev == dev) d = &c;
  if (!d) {
    void* p = nullptr;
    if (hipMalloc(&p, kMtRtRows * kMtPolyWords * sizeof(uint64_t)) != hipSuccess) {
      *err = 1;
      return nullptr;
    }
    cache->push_back({dev, static_cast<uint64_t*>(p), 0, 0});
    d = &cache->back();
  }
  const uint64_t need = S - 1;
  if (d->version != version || d->rows < need) {
    const uint64_t n = std::max(d->rows, need);
    if (hipMemcpy(d->p, host, n * kMtPolyWords * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess) {
      *err = 1;
      return nullptr;
    }
    d->version = version;
    d->rows = n;
  }
  return d->p;
}

// The call's end: DN_MT_SPIN_SYNC = 1 records an event behind the last
// launch and polls it (the thread spins instead of blocking in the runtime:
// a shorter wake-up for a call whose GPU work is tens of microseconds);
// otherwise hipStreamSynchronize.  One event per thread, created once.
#ifndef DN_MT_SPIN_SYNC
#define DN_MT_SPIN_SYNC 0
#endif
// DN_MT_SPLIT2's side stream and its two events, per thread and device
// (created once, never destroyed: the runtime may be torn down first).
struct SideStream {
  int dev = -1;
  hipStream_t s = nullptr;
  hipEvent_t levels = nullptr, gen = nullptr;
  // DN_MT_SPEC_PROBE: the prefix copied, the side levels done (pending: a
  // wait owed by the next call), the side levels' own buffer
  hipEvent_t copy = nullptr, spec = nullptr;
  bool pending = false;
  void* buf = nullptr;
  uint64_t buf_bytes = 0;
};
SideStream* side_stream() {
  thread_local SideStream side[16];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  SideStream& x = side[dev];
  if (!x.s) {
    if (hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking) != hipSuccess) return x.s = nullptr, nullptr;
    if (hipEventCreateWithFlags(&x.levels, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x.gen, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x.copy, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x.spec, hipEventDisableTiming) != hipSuccess)
      return nullptr;
    x.dev = dev;
  }
  return &x;
}

// DN_MT_SPEC (default 1; tuning build: DN_MT_SPEC=0 off): a call speculates
// that the next draw on this device has the same size and starts where this
// one ends — the loop `for x in batch: make_shares_vec(x)` — and computes the
// next call's windows while its own host side finishes: the generation's last
// substream also writes the next call's W_idx (the window at stream position
// idx + 17 ncoef) into a buffer of the device's speculation state, then the
// shape's jump levels from it run on a side stream into that buffer.  The
// next call uses the buffer in place of its jump levels when its draw size,
// CPython index and 624-word array equal the ones this call left (anything
// else — another size, random.Random touched in between, a rejected draw —
// is a miss: the call jumps itself).  A call speculates only when it
// continues the previous call (same size, starting where that one ended), so
// a lone call, or equal calls on fresh random.Random states, launch nothing
// extra.  Two buffers alternate (one the generation reads, one the side
// stream fills); the side stream's work is always awaited by the call stream
// before a buffer is reused.  One state per device, process-wide; a call that
// finds it busy (another thread's call) neither speculates nor hits.
#ifndef DN_MT_SPEC
#define DN_MT_SPEC 1
#endif
// The final state by the last substream (tail_fin, last_sub_tail) rather than
// a final-state wave: that wave stepped the whole last substream again, one
// wave alone, and finished ~100 us after the other substreams at 2^24
// (profiles/r06/g/timeline_spec.json: substreams 0.88-0.91 ms, the wave
// 0.93-1.09 ms).
#ifndef DN_MT_TAIL_FIN
#define DN_MT_TAIL_FIN 1
#endif
// The speculated levels of a runtime-direct-level draw (2^24 scale) beside
// the generation rather than after it (mt_jumpc_kernel<4, 2>; tuning build:
// DN_MT_SPEC_BESIDE=0 off)
#ifndef DN_MT_SPEC_BESIDE
#define DN_MT_SPEC_BESIDE 1
#endif
// draws of fewer coefficients than this do not speculate after the
// generation (tuning build: DN_MT_SPEC_MIN), nor beside it below
// DN_MT_BESIDE_MIN (the levels of a small generation beside it, round 6)
#ifndef DN_MT_SPEC_MIN
#define DN_MT_SPEC_MIN (1ull << 23)
#endif
#ifndef DN_MT_BESIDE_MIN
#define DN_MT_BESIDE_MIN (1ull << 16)
#endif
struct SpecState {
  std::mutex m;
  hipStream_t side = nullptr, side2 = nullptr;
  hipEvent_t win = nullptr, done = nullptr;  // this call's windows in place (call stream), the side streams done
  hipEvent_t j0ev = nullptr, done2 = nullptr;
  bool widx2 = false;  // beside: buf[next ^ 1]'s row -1 holds the W_idx of the call after the armed one
  void* buf[2] = {nullptr, nullptr};
  uint64_t bytes = 0;  // of each buffer
  bool armed = false;  // buf[next] holds (at `done`) the windows of a call starting as below
  int next = 0;
  uint64_t ncoef = 0;
  int32_t idx = -1;
  uint32_t state[kMtN];
  bool have_end = false;  // ncoef, idx, state: where the previous call ended
  uint64_t hits = 0, misses = 0, launched = 0;
  uint64_t* xpow = nullptr;  // device: x^xpow_words mod P (the next call's W_idx from this one's)
  uint64_t xpow_words = 0;
  bool xpow_failed = false;  // no carry-less multiply here, or the upload failed: no beside levels
};

std::mutex& spec_table_mutex() {
  static std::mutex* m = new std::mutex;
  return *m;
}
SpecState* spec_slot(int dev) {  // created once per device, never destroyed (the runtime may go first)
  static SpecState* table[16] = {};
  if (dev < 0 || dev >= 16) return nullptr;
  std::lock_guard<std::mutex> g(spec_table_mutex());
  if (!table[dev]) {
    auto* x = new SpecState;
    if (hipStreamCreateWithFlags(&x->side, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&x->side2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&x->j0ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->done2, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->win, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->done, hipEventDisableTiming) != hipSuccess)
      return nullptr;  // (leaks the half-made state: a runtime that cannot make a stream has bigger problems)
    table[dev] = x;
  }
  return table[dev];
}

// x^words mod P on the device for the beside chain's first jump (computed on
// the host once per draw size: ~30 Barrett products, a few ms)
bool spec_xpow(SpecState& sp, uint64_t words) {
  if (sp.xpow_failed) return false;
  if (sp.xpow && sp.xpow_words == words) return true;
  std::vector<uint64_t> g(kMtPolyWords);
  if (!mt_xpow_mod(words, g.data()) ||
      (!sp.xpow && hipMalloc(reinterpret_cast<void**>(&sp.xpow), kMtPolyWords * sizeof(uint64_t)) != hipSuccess)) {
    sp.xpow_failed = true;
    return false;
  }
  (void)hipStreamSynchronize(sp.side);  // the previous size's polynomial may still be read
  (void)hipStreamSynchronize(sp.side2);
  if (hipMemcpy(sp.xpow, g.data(), kMtPolyWords * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess) {
    sp.xpow_failed = true;
    return false;
  }
  sp.xpow_words = words;
  return true;
}

// both buffers at least `need` bytes (false: allocation failed; no speculation)
bool spec_buffers(SpecState& sp, uint64_t need) {
  if (sp.bytes >= need && sp.buf[0] && sp.buf[1]) return true;
  (void)hipStreamSynchronize(sp.side);  // nothing of ours uses them once the side streams are idle
  (void)hipStreamSynchronize(sp.side2);
  sp.armed = false;
  sp.widx2 = false;
  for (void*& b : sp.buf)
    if (b) (void)hipFree(b), b = nullptr;
  sp.bytes = 0;
  for (void*& b : sp.buf)
    if (hipMalloc(&b, need) != hipSuccess) {
      for (void*& c : sp.buf)
        if (c) (void)hipFree(c), c = nullptr;
      return false;
    }
  sp.bytes = need;
  return true;
}

hipError_t mt_wait(hipStream_t s) {
#if DN_MT_SPIN_SYNC
  thread_local hipEvent_t ev = nullptr;
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    ev = nullptr;
    return hipStreamSynchronize(s);
  }
  hipError_t e = hipEventRecord(ev, s);
  if (e != hipSuccess) return e;
  while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
  }
  return e;
#else
  return hipStreamSynchronize(s);
#endif
}

}  // namespace
}  // namespace dn

using namespace dn;

extern "C" uint64_t dn_mt19937_device_scratch_bytes(uint64_t n_elem, int tm1) {
  const uint64_t ncoef = tm1 > 0 ? n_elem * static_cast<uint64_t>(tm1) : 0;
  const uint64_t S = ncoef ? mt_subs(ncoef) : 0;
  if (!S) return kHead + kMtN * 4;
  const MtHost& H = mt_levels(S, mt_sub_len(ncoef));
  return kHead + (1 + S + 1 + H.part_rows) * kMtN * 4;
}

namespace dn {
namespace {

// The device draw of n_elem * tm1 coefficients from CPython state
// (mt_state, *mt_index): jump levels, then `launch_gen(ga, S)` (the
// generation kernel: coefficients or fused split), then CPython's final state.
constexpr uint64_t kCus = 256, kLdsPerCu = 160 * 1024;  // MI355X: CUs, LDS bytes per CU

template <typename F>
int mt_device_run(const char* name, uint32_t* mt_state, int32_t* mt_index, uint64_t n_elem, int tm1, void* scratch,
                  uint64_t scratch_bytes, void* stream, int ring_units, F launch_gen) {
  if (!mt_state || !mt_index) return set_error(DN_ERR_ARG, "%s: null pointer", name);
  if (tm1 < 0 || tm1 >= DN_MAX_THRESHOLD) return set_error(DN_ERR_ARG, "%s: t-1=%d", name, tm1);
  const int32_t idx = *mt_index;
  if (idx < 0 || idx > kMtN) return set_error(DN_ERR_ARG, "%s: bad MT index", name);
  const uint64_t ncoef = n_elem * static_cast<uint64_t>(tm1);
  if (ncoef == 0) return DN_OK;
  if (!scratch) return set_error(DN_ERR_ARG, "%s: null pointer", name);
  const uint64_t S = mt_subs(ncoef);
  if (S > mt_jump_max_subs() - 1)
    return set_error(DN_ERR_UNSUPPORTED, "%s: %llu words exceed the jump table", name,
                     static_cast<unsigned long long>(17 * ncoef));
  if (scratch_bytes < dn_mt19937_device_scratch_bytes(n_elem, tm1)) return set_error(DN_ERR_ARG, "%s: scratch too small", name);

  // CPython's state after the draw: the array at buffer position tf = 624 q,
  // stepped by the final-state wave from window `sig` (position P_sig < tf)
  const uint64_t words = 17 * ncoef, h = static_cast<uint64_t>(kMtN - idx);
  int32_t sig = -1, fidx = idx + static_cast<int32_t>(words <= h ? words : 0);
  uint64_t fpos = 0, ftf = 0;
  if (words > h) {
    const uint64_t m_end = words - h, q = (m_end + kMtN - 1) / kMtN, tf = kMtN * q;
    const uint64_t Lk = 17 * mt_sub_draws(mt_sub_len(ncoef));  // words per substream
    uint64_t sg = (tf + kMtN - 1 - static_cast<uint64_t>(idx)) / Lk;  // idx + sg L - 624 < tf
    if (sg > S - 1) sg = S - 1;
    sig = static_cast<int32_t>(sg);
    fpos = sg ? static_cast<uint64_t>(idx) + sg * Lk - kMtN : 0;
    ftf = tf;
    fidx = static_cast<int32_t>(m_end - kMtN * (q - 1));
  }

  // scratch: head (flag at 0, final array at 256) | W_idx (the caller's
  // array advanced idx words: window "-1", the level-A source) | windows 0..S
  // (row 0 the caller's array; row S unused) | part rows (split levels).  The
  // job tables are the device copy of this shape's (device_jobs).  What the
  // GPU needs from the host is the prefix head .. row 0: ONE copy from the
  // pinned staging buffer, which holds that prefix and, in its tail, the head
  // read back at the end.
  const int ki = mt_sub_len(ncoef);
  MtHost& H = mt_levels(S, ki);
  const Level* lv = H.lv;
  const uint64_t njobs = lv[0].jobs.size() + lv[1].jobs.size() + lv[2].jobs.size();
  int jerr = 0;
  const void* jobs_dev = device_jobs(H, &jerr);
  if (jerr) return set_error(DN_ERR_HIP, "%s: job tables on the device", name);
  const uint64_t* rt_dev = H.rt ? device_rt(S, &jerr) : nullptr;
  if (jerr) return set_error(DN_ERR_HIP, "%s: runtime jump rows on the device", name);
  const size_t wpre = kHead / 4 + 2 * kMtN, wh = 256 / 4 + kMtN;
  PinLease lease(wpre + wh);  // idle again once this call has synchronised its stream
  uint32_t* pin = lease.p;
  if (!pin) return set_error(DN_ERR_HIP, "%s: pinned staging buffer", name);
  uint32_t *stw = pin + kHead / 4, *head = pin + wpre;
  std::memset(pin, 0, 256);  // the flag (the final array is written by the device)
  mt_advance_window(mt_state, static_cast<uint64_t>(idx), stw);  // W_idx
  std::memcpy(stw + kMtN, mt_state, kMtN * 4);                    // row 0
  hipStream_t s = static_cast<hipStream_t>(stream);
  // DN_MT_SPEC_PROBE (tuning build, timing probe only: the output is wrong):
  // 1 = the call's jump levels skipped (the generation reads stale windows);
  // 2 = skipped, and the same levels run on the side stream into a buffer of
  // their own, launched before the generation and awaited by the next call's
  // generation — the cost of a next call's speculative levels beside this
  // call's generation; 3 = as 2, launched after the generation; 4 = as 2 with
  // the runtime direct level by mt_jumpc_kernel<4, 2> (beside the generation);
  // 5 = the call's own levels by mt_jumpc_kernel<4, 2> (its time alone).
  const char* spp = tune_env("DN_MT_SPEC_PROBE");
  const int spec_probe = spp ? std::atoi(spp) : 0;
  // the speculation state (DN_MT_SPEC): this call's draw may have been
  // speculated (hit), and it may speculate on the next one (spec_next)
  const char* spe = tune_env("DN_MT_SPEC");
  // DN_MT_TAIL_FIN (default 1; tuning build: 0 = the final-state wave)
  const char* tfe = tune_env("DN_MT_TAIL_FIN");
  const bool tail_fin = sig >= 0 && (tfe ? tfe[0] != '0' : DN_MT_TAIL_FIN != 0);
  const char* spm = tune_env("DN_MT_SPEC_MIN");
  const uint64_t spec_min = spm ? std::strtoull(spm, nullptr, 10) : DN_MT_SPEC_MIN;
  const char* bmn = tune_env("DN_MT_BESIDE_MIN");
  const uint64_t beside_min = bmn ? std::strtoull(bmn, nullptr, 10) : DN_MT_BESIDE_MIN;
  const bool spec_on = (spe ? spe[0] != '0' : DN_MT_SPEC != 0) && spec_probe == 0 && !H.split2 && tail_fin &&
                       njobs > 0 && ncoef >= std::min(spec_min, beside_min);
  SpecState* sp = nullptr;
  std::unique_lock<std::mutex> spl;
  if (spec_on) {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && (sp = spec_slot(dev))) {
      spl = std::unique_lock<std::mutex>(sp->m, std::try_to_lock);
      if (!spl.owns_lock()) sp = nullptr;
    }
  }
  bool hit = false, spec_next = false, widx2 = false;
  if (sp) {
    // this call continues the previous one (same size, starting where it
    // ended): a hit if that call speculated, and a reason to speculate again
    const bool cont = sp->have_end && sp->ncoef == ncoef && sp->idx == idx &&
                      !std::memcmp(sp->state, mt_state, kMtN * 4);
    hit = cont && sp->armed;
    if (sp->armed && !hit) ++sp->misses;
    widx2 = hit && sp->widx2;
    sp->armed = false;
    sp->widx2 = false;
    sp->have_end = false;
    spec_next = cont && spec_buffers(*sp, dn_mt19937_device_scratch_bytes(n_elem, tm1));
  }
  // beside (DN_MT_SPEC_BESIDE, runtime direct level only): the next call's
  // W_idx by one jump from this call's, then its level, both by
  // mt_jumpc_kernel<4, 2> on the side stream beside this call's generation
  // Other shapes: the levels as they are (mt_jump_kernel, 83 KB workgroups)
  // when the generation's rings leave a CU that much LDS (a generation of at
  // most ~1000 3-of-5 substreams: 2^22 coefficients and less), and when the
  // generation outlasts them: substreams of 2^12 draws, or of 2^10 and at most
  // 256 of them (loops of 2^20 / 2^16 elements -15 / -10 %; 512 substreams
  // of 2^10 draws, 2^18 elements, +2.5 %: profiles/r06/y/).
  const char* sbe = tune_env("DN_MT_SPEC_BESIDE");
  const uint64_t gen_lds = (1u + 2u * 17u * 64u * static_cast<uint32_t>(ring_units) + 64u) * 4u;
  const bool levels_fit = (S + kCus - 1) / kCus * gen_lds + (kEWords + kMtN + 64) * 4u <= kLdsPerCu;
  const bool beside = spec_next && (sbe ? sbe[0] != '0' : DN_MT_SPEC_BESIDE != 0) && ncoef >= beside_min &&
                      (H.rt ? !H.beside.jobs.empty() : levels_fit && (mt_sub_draws(ki) >= 4096 || S <= 256)) &&
                      !H.j0.jobs.empty() && spec_xpow(*sp, words);
  if (!beside && ncoef < spec_min) spec_next = false;  // (no speculation after the generation this small)
  const int spec_dst = sp ? sp->next ^ 1 : 0;  // the buffer the next call's windows go to
  // a hit generates from its speculated buffer; a beside call runs in the
  // other library buffer too (the side stream reads its W_idx from there)
  uint8_t* sc = hit || beside ? static_cast<uint8_t*>(sp->buf[sp->next]) : static_cast<uint8_t*>(scratch);
  const JumpJob* djobs = static_cast<const JumpJob*>(jobs_dev);
  const CombineJob* dcomb = reinterpret_cast<const CombineJob*>(djobs + njobs);
  uint32_t* dwin = reinterpret_cast<uint32_t*>(sc + kHead) + kMtN;  // row 0
  // the side stream's last work (the speculated levels) is done before this
  // call writes a speculation buffer or reads one (a wait on the device only
  // if it is still running)
  hipError_t err = (spec_next || hit) && hipEventQuery(sp->done) != hipSuccess ? hipStreamWaitEvent(s, sp->done, 0)
                                                                              : hipSuccess;
  if (err == hipSuccess && (spec_next || hit) && hipEventQuery(sp->done2) != hipSuccess)
    err = hipStreamWaitEvent(s, sp->done2, 0);
  if (err == hipSuccess) err = hipMemcpyAsync(sc, pin, wpre * 4, hipMemcpyHostToDevice, s);
  if (err != hipSuccess) {
    (void)hipStreamSynchronize(s);  // the staging buffer is reused by the next call
    return set_error(DN_ERR_HIP, "%s: %s", name, hipGetErrorString(err));
  }
  SideStream* side = H.split2 || spec_probe >= 2 ? side_stream() : nullptr;
  if ((H.split2 || spec_probe >= 2) && !side) {
    (void)hipStreamSynchronize(s);
    return set_error(DN_ERR_HIP, "%s: side stream", name);
  }
  auto launch_levels = [&](hipStream_t ls, uint32_t* wins) {
    uint64_t off = 0, coff = 0;
    for (int k = 0; k < 3; ++k) {
      const Level& l = lv[k];
      if (!l.jobs.empty()) {
        const char* jpr = tune_env("DN_MT_JUMP_PROBE");
        const JumpArgs ja{wins, djobs + off, static_cast<uint32_t>(l.jobs.size()),
                          jpr ? static_cast<uint32_t>(std::atoi(jpr)) : 0u, rt_dev};
        const dim3 grid(static_cast<uint32_t>(l.jobs.size() / static_cast<size_t>(l.W)));
        const char* j4 = tune_env("DN_MT_JUMP4B");  // tuning build: 16-wave levels by mt_jumpc_kernel<16, 4>
        if (l.W == 16 && j4 && j4[0] == '1') hipLaunchKernelGGL((mt_jumpc_kernel<16, 4>), grid, dim3(64 * 16), 0, ls, ja);
        else if (l.W == 16) hipLaunchKernelGGL(mt_jump_kernel<16>, grid, dim3(64 * 16), 0, ls, ja);
        else hipLaunchKernelGGL(mt_jump_kernel<8>, grid, dim3(64 * 8), 0, ls, ja);
      }
      if (!l.comb.empty())
        hipLaunchKernelGGL(mt_combine_kernel, dim3(static_cast<uint32_t>(l.comb.size())), dim3(640), 0, ls, wins,
                           dcomb + coff);
      off += l.jobs.size();
      coff += l.comb.size();
      // split2: the first half's windows are complete after level 0
      if (H.split2 && k == 0) err = hipEventRecord(side->levels, ls);
    }
  };
  auto probe_beside = [&](hipStream_t ls, uint32_t* wins) {  // DN_MT_SPEC_PROBE=4: the rt level by mt_jumpc_kernel<4, 2>
    const Level& l = H.beside;
    if (l.jobs.empty()) return;
    const JumpJob* bj = reinterpret_cast<const JumpJob*>(static_cast<const uint32_t*>(jobs_dev) + H.beside_off);
    const JumpArgs ja{wins, bj, static_cast<uint32_t>(l.jobs.size()), 0u, rt_dev};
    launch_jumpc4(dim3(static_cast<uint32_t>(l.jobs.size() / 4)), ls, ja);
  };
  auto probe_levels = [&]() {
    if (!side->buf || side->buf_bytes < scratch_bytes) {
      if (side->buf) (void)hipFree(side->buf);
      side->buf = nullptr;
      side->buf_bytes = 0;
      if (hipMalloc(&side->buf, scratch_bytes) != hipSuccess) return hipErrorOutOfMemory;
      side->buf_bytes = scratch_bytes;
    }
    hipError_t e = hipStreamWaitEvent(side->s, side->copy, 0);
    uint32_t* pw = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(side->buf) + kHead) + kMtN;
    if (spec_probe == 4) probe_beside(side->s, pw);
    else launch_levels(side->s, pw);
    if (e == hipSuccess) e = hipEventRecord(side->spec, side->s);
    side->pending = true;
    return e;
  };
  if (spec_probe == 5) {
    probe_beside(s, dwin);
  } else if (spec_probe == 0) {
    if (!hit) launch_levels(s, dwin);  // (a hit's windows are in place)
  } else if (spec_probe >= 2) {
    err = hipEventRecord(side->copy, s);
    if (err == hipSuccess && side->pending) err = hipStreamWaitEvent(s, side->spec, 0);
    if (err == hipSuccess && (spec_probe == 2 || spec_probe == 4)) err = probe_levels();
  }
  GenArgs ga{};
  ga.wins = dwin;
#if DN_MT_HOST_HEAD
  head[0] = 0u;  // the flag; the final-state wave writes the final array at head + 64
  void* dhead = nullptr;
  if (hipHostGetDevicePointer(&dhead, head, 0) != hipSuccess || !dhead) {
    (void)hipStreamSynchronize(s);
    return set_error(DN_ERR_HIP, "%s: staging buffer not mapped", name);
  }
  ga.flag = static_cast<uint32_t*>(dhead);
  ga.fin = static_cast<uint32_t*>(dhead) + 64;
#else
  ga.flag = reinterpret_cast<uint32_t*>(sc);
  ga.fin = reinterpret_cast<uint32_t*>(sc + 256);
#endif
  ga.ncoef = ncoef;
  ga.sub_draws = mt_sub_draws(ki);
  ga.vb = dn_m521_vec_bytes(n_elem);
  ga.tm1_magic = ((1ull << 32) + static_cast<uint64_t>(tm1) - 1) / static_cast<uint64_t>(tm1);
  ga.S = static_cast<uint32_t>(S);
  ga.idx = static_cast<uint32_t>(idx);
  ga.tm1 = tm1;
  ga.final_sig = sig;
  ga.final_pos = fpos;
  ga.final_tf = ftf;
  ga.n_elem = n_elem;
  ga.back = static_cast<uint32_t>(H.back);
  const char* pr = tune_env("DN_MT_PROBE");
  ga.probe = pr ? static_cast<uint32_t>(std::atoi(pr)) : 0u;
  if (tail_fin) {
    // the last substream's frame: position 0 = stream position idx + (S - 1) L
    const uint64_t base = static_cast<uint64_t>(idx) + (S - 1) * (17 * mt_sub_draws(ki));
    ga.tail_fin = 1u;
    ga.fin_lo = static_cast<int32_t>(static_cast<int64_t>(ftf) - static_cast<int64_t>(base));
    ga.next_lo = static_cast<int32_t>(static_cast<int64_t>(idx + words) - static_cast<int64_t>(base));
  }
  const uint32_t nwg = static_cast<uint32_t>(S) + (tail_fin ? 0u : 1u);  // + the final-state wave
  ga.sub_n = nwg;
  bool side_used = false;  // work of this call on the speculation side stream
  if (H.split2) {
    // substreams [0, S/2) on the side stream once level 0 is done (beside
    // level 1's jumps), then [S/2, S] and the final-state wave on the call's
    // stream after level 1; the call's stream then waits for the side stream
    const uint32_t half = static_cast<uint32_t>(mt_split_half(S));
    if (err == hipSuccess) err = hipStreamWaitEvent(side->s, side->levels, 0);
    GenArgs g1 = ga;
    g1.sub_lo = 0u;
    g1.sub_n = half;
    launch_gen(g1, side->s);
    if (err == hipSuccess) err = hipEventRecord(side->gen, side->s);
    ga.sub_lo = half;
    ga.sub_n = nwg - half;
    launch_gen(ga, s);
    if (err == hipSuccess) err = hipStreamWaitEvent(s, side->gen, 0);
  } else if (beside) {
    // Once this call's windows are in place, in workgroups of 11 KB that fit
    // on a CU beside the generation's rings: on the side stream the next
    // call's level into the other buffer from its W_idx (row -1 there) — which
    // the previous call computed (widx2) or, first, one jump by x^(17 ncoef)
    // from this call's W_idx computes (copied to row S, 32 parts + combine);
    // on the second side stream the W_idx of the call after that, jumped from
    // the next call's into this call's buffer (rows S, part rows and -1: none
    // of them read by this call's generation).
    uint8_t* nb = static_cast<uint8_t*>(sp->buf[spec_dst]);
    uint32_t* nw = reinterpret_cast<uint32_t*>(nb + kHead) + kMtN;  // the next call's row 0
    const uint32_t* hj = static_cast<const uint32_t*>(jobs_dev);
    auto jump0 = [&](hipStream_t ls, uint32_t* w) {  // row S -> row -1 of w by x^(17 ncoef)
      const JumpArgs j0{w, reinterpret_cast<const JumpJob*>(hj + H.j0_off), static_cast<uint32_t>(H.j0.jobs.size()), 0u,
                        sp->xpow};
      launch_jumpc4(dim3(static_cast<uint32_t>(H.j0.jobs.size() / 4)), ls, j0);
      hipLaunchKernelGGL(mt_combine_kernel, dim3(static_cast<uint32_t>(H.j0.comb.size())), dim3(640), 0, ls, w,
                         reinterpret_cast<const CombineJob*>(hj + H.j0_comb_off));
    };
    err = hipEventRecord(sp->win, s);
    launch_gen(ga, s);
    side_used = true;
    if (err == hipSuccess) err = hipStreamWaitEvent(sp->side, sp->win, 0);
    if (err == hipSuccess) err = hipStreamWaitEvent(sp->side2, sp->win, 0);
    if (!widx2) {
      if (err == hipSuccess)
        err = hipMemcpyAsync(nw + S * kMtN, dwin - kMtN, kMtN * 4, hipMemcpyDeviceToDevice, sp->side);
      jump0(sp->side, nw);
      if (err == hipSuccess) err = hipEventRecord(sp->j0ev, sp->side);
      if (err == hipSuccess) err = hipStreamWaitEvent(sp->side2, sp->j0ev, 0);
    }
    if (H.rt) {
      const JumpArgs bl{nw, reinterpret_cast<const JumpJob*>(hj + H.beside_off),
                        static_cast<uint32_t>(H.beside.jobs.size()), 0u, rt_dev};
      launch_jumpc4(dim3(static_cast<uint32_t>(H.beside.jobs.size() / 4)), sp->side, bl);
    } else {
      launch_levels(sp->side, nw);
    }
    if (err == hipSuccess) err = hipEventRecord(sp->done, sp->side);
    if (err == hipSuccess)
      err = hipMemcpyAsync(dwin + S * kMtN, nw - kMtN, kMtN * 4, hipMemcpyDeviceToDevice, sp->side2);
    jump0(sp->side2, dwin);
    if (err == hipSuccess) err = hipEventRecord(sp->done2, sp->side2);
    ++sp->launched;
  } else if (spec_next) {
    // the generation, whose last substream also writes the next call's W_idx
    // into row -1 of the other buffer; then on the side stream the next
    // call's jump levels from it, while this call's host side finishes and
    // the next call's begins
    uint8_t* nb = static_cast<uint8_t*>(sp->buf[spec_dst]);
    ga.next_win = reinterpret_cast<uint32_t*>(nb + kHead);
    launch_gen(ga, s);
    err = hipEventRecord(sp->win, s);
    if (err == hipSuccess) err = hipStreamWaitEvent(sp->side, sp->win, 0);
    side_used = true;
    launch_levels(sp->side, reinterpret_cast<uint32_t*>(nb + kHead) + kMtN);
    if (err == hipSuccess) err = hipEventRecord(sp->done, sp->side);
    ++sp->launched;
  } else {
    launch_gen(ga, s);
    if (err == hipSuccess && spec_probe == 3) err = probe_levels();
  }
  // an early exit waits for this call's side work too (it writes the staging buffer)
  auto drain = [&]() {
    (void)hipStreamSynchronize(s);
    if (side_used) (void)hipStreamSynchronize(sp->side), (void)hipStreamSynchronize(sp->side2);
  };
  if (err != hipSuccess) {
    drain();
    return set_error(DN_ERR_HIP, "%s: side stream: %s", name, hipGetErrorString(err));
  }
  err = hipGetLastError();
  if (err != hipSuccess) {
    drain();
    return set_error(DN_ERR_HIP, "%s: launch: %s", name, hipGetErrorString(err));
  }

#if !DN_MT_HOST_HEAD
  err = hipMemcpyAsync(head, sc, wh * 4, hipMemcpyDeviceToHost, s);  // flag .. final array
#endif
  const hipError_t serr = mt_wait(s);
  if (err == hipSuccess) err = serr;
  if (err != hipSuccess) {
    if (side_used) (void)hipStreamSynchronize(sp->side), (void)hipStreamSynchronize(sp->side2);
    return set_error(DN_ERR_HIP, "%s: %s", name, hipGetErrorString(err));
  }
  if (hit) ++sp->hits;
  // DN_MT_FORCE_RETRY=1 (tuning build) takes the rejected-draw exit so the
  // caller's host fallback can be exercised.
  const char* fr = tune_env("DN_MT_FORCE_RETRY");
  if (head[0] || (fr && fr[0] == '1')) return set_error(DN_ERR_RETRY, "%s: a draw was rejected; redo on the host", name);
  if (sig >= 0) std::memcpy(mt_state, head + 256 / 4, kMtN * 4);
  *mt_index = fidx;
  if (sp) {
    // where this call ended; the next call, if it starts here, uses the
    // speculated windows (spec_next) or speculates itself
    sp->have_end = true;
    sp->ncoef = ncoef;
    sp->idx = fidx;
    std::memcpy(sp->state, mt_state, kMtN * 4);
    sp->armed = spec_next;
    sp->widx2 = beside;  // this call's buffer now holds the W_idx after the next call's
    if (spec_next) sp->next = spec_dst;
  }
  return DN_OK;
}

#ifndef DN_MT_SAUX
#define DN_MT_SAUX 16
#endif
constexpr int kSc1 = DN_MT_SAUX;
// the fused split's generation and emission on two waves per substream for
// draws of few substreams (mt_gen_pc_kernel; 0: always one wave, mt_gen_kernel)
#ifndef DN_MT_PC
#define DN_MT_PC 1
#endif  // buffer-store cache policy of the 3-of-5 share stores: sc1 (16)

template <int T>
void launch_gen(GenArgs& ga, hipStream_t s) {
  ga.ring = 2u * 17u * 64u * (T ? T - 1 : 1);
  const uint32_t lds_words = 1u + ga.ring + 64u;  // GenRing: alignment word, ring, mirror
#ifdef DN_TUNING
  // DN_MT_STORE_AUX (tuning build): cache policy bits of the fused split's share stores (3-of-5)
  const char* sa = T == 3 ? tune_env("DN_MT_STORE_AUX") : nullptr;
  if (sa && T == 3 && ga.n_shares == 5) {
    const int aux = std::atoi(sa);
    constexpr int NS = T == 3 ? 5 : 0;
    const dim3 g(ga.S + 1), b(64);
    if (aux == 0) hipLaunchKernelGGL((mt_gen_kernel<T, 0, NS>), g, b, lds_words * 4u, s, ga);
    else if (aux == 1) hipLaunchKernelGGL((mt_gen_kernel<T, 1, NS>), g, b, lds_words * 4u, s, ga);
    else if (aux == 2) hipLaunchKernelGGL((mt_gen_kernel<T, 2, NS>), g, b, lds_words * 4u, s, ga);
    else if (aux == 16) hipLaunchKernelGGL((mt_gen_kernel<T, 16, NS>), g, b, lds_words * 4u, s, ga);
    else hipLaunchKernelGGL((mt_gen_kernel<T, 18, NS>), g, b, lds_words * 4u, s, ga);
    return;
  }
#endif
  // the headline 3-of-5: straight-line share stores (see mt_gen_kernel), sc1
  // rather than non-temporal: 2.2 % faster on two buffers of one process
  // (profiles/r03/ab/mt_store_aux_ns5.json)
  // Generation and emission on two waves per substream (mt_gen_pc_kernel):
  // at 2^24 the kernel runs at its emission-only time (0.92 vs 1.01 ms for
  // the one-wave kernel on a share block, profiles/r04/t/), at 2^20 / 2^16 /
  // 2^12 make_shares_vec -12 / -8 / -3 % (profiles/r04/l/).
  if constexpr (DN_MT_PC) {
    // DN_MT_PC_FORCE (tuning build): 0 = the one-wave kernel (A/B)
    const char* pf = tune_env("DN_MT_PC_FORCE");
    const bool pc = !(pf && pf[0] == '0');
    // DN_MT_GEN_SUBS (tuning build, timing probe only: the output is partial and
    // CPython's final state is not computed): launch only the first K substream
    // workgroups — how the generation's time scales with the substreams in flight
    uint32_t grid = ga.sub_n ? ga.sub_n : ga.S + 1;
    if (const char* gs = tune_env("DN_MT_GEN_SUBS")) grid = std::min<uint32_t>(grid, std::max(1, std::atoi(gs)));
    if (pc) {
      if (T == 3 && ga.n_shares == 5)
        hipLaunchKernelGGL((mt_gen_pc_kernel<T, kSc1, T == 3 ? 5 : 0>), dim3(grid), dim3(128), lds_words * 4u, s, ga);
      else
        hipLaunchKernelGGL((mt_gen_pc_kernel<T>), dim3(grid), dim3(128), lds_words * 4u, s, ga);
      return;
    }
  }
  const dim3 g1(ga.sub_n ? ga.sub_n : ga.S + 1);
  if (T == 3 && ga.n_shares == 5)
    hipLaunchKernelGGL((mt_gen_kernel<T, kSc1, T == 3 ? 5 : 0>), g1, dim3(64), lds_words * 4u, s, ga);
  else
    hipLaunchKernelGGL((mt_gen_kernel<T>), g1, dim3(64), lds_words * 4u, s, ga);
}

}  // namespace
}  // namespace dn

extern "C" int dn_mt19937_draw_coeffs_device(uint32_t* mt_state, int32_t* mt_index, uint64_t n_elem, int tm1,
                                             void* coeffs, void* scratch, uint64_t scratch_bytes, void* stream) {
  if (n_elem && tm1 > 0 && !coeffs) return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs_device: null pointer");
  return mt_device_run("dn_mt19937_draw_coeffs_device", mt_state, mt_index, n_elem, tm1, scratch, scratch_bytes, stream, 1,
                       [&](GenArgs& ga, hipStream_t s) {
                         ga.coeffs = static_cast<uint8_t*>(coeffs);
                         launch_gen<0>(ga, s);
                       });
}

extern "C" int dn_mt19937_split_supported(uint64_t n_elem, int threshold, int n_shares) {
  if (!(threshold == 2 || threshold == 3 || threshold == 5) || threshold > n_shares || n_shares > DN_MAX_SHARES ||
      fd_needs_fold(threshold, n_shares))
    return 0;
  const uint64_t ncoef = n_elem * static_cast<uint64_t>(threshold - 1);
  return !ncoef || mt_subs(ncoef) <= mt_jump_max_subs() - 1;
}

extern "C" int dn_mt19937_split_device(uint32_t* mt_state, int32_t* mt_index, const int64_t* secrets, void* shares,
                                       uint64_t n_elem, int threshold, int n_shares, void* scratch,
                                       uint64_t scratch_bytes, void* stream) {
  const char* name = "dn_mt19937_split_device";
  if (threshold < 1 || threshold > DN_MAX_THRESHOLD)
    return set_error(DN_ERR_UNSUPPORTED, "%s: threshold %d outside 1..%d", name, threshold, DN_MAX_THRESHOLD);
  if (threshold > n_shares) return set_error(DN_ERR_THRESHOLD, "threshold should be little equal than shares");
  if (!(threshold == 2 || threshold == 3 || threshold == 5) || fd_needs_fold(threshold, n_shares) ||
      n_shares > DN_MAX_SHARES)
    return set_error(DN_ERR_UNSUPPORTED, "%s: fused form needs t in {2, 3, 5} and forward differences (t=%d, n=%d)",
                     name, threshold, n_shares);
  if (n_elem && (!secrets || !shares)) return set_error(DN_ERR_ARG, "%s: null pointer", name);
  return mt_device_run(name, mt_state, mt_index, n_elem, threshold - 1, scratch, scratch_bytes, stream, threshold - 1,
                       [&](GenArgs& ga, hipStream_t s) {
                         ga.secrets = secrets;
                         ga.shares = static_cast<uint8_t*>(shares);
                         ga.n_shares = n_shares;
                         if (threshold == 2) launch_gen<2>(ga, s);
                         else if (threshold == 3) launch_gen<3>(ga, s);
                         else launch_gen<5>(ga, s);
                       });
}

// The current device's speculation counters (DN_MT_SPEC): out[0] calls that
// used speculated windows, out[1] speculations a call did not match, out[2]
// speculations launched, out[3] 1 if one is armed now (the device's state is
// made here if no draw has made it yet: all zero).
extern "C" int dn_mt19937_spec_stats(uint64_t* out) {
  if (!out) return set_error(DN_ERR_ARG, "dn_mt19937_spec_stats: null pointer");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return set_error(DN_ERR_HIP, "dn_mt19937_spec_stats: no device");
  SpecState* sp = spec_slot(dev);
  if (!sp) return set_error(DN_ERR_HIP, "dn_mt19937_spec_stats: speculation state");
  std::lock_guard<std::mutex> g(sp->m);
  out[0] = sp->hits;
  out[1] = sp->misses;
  out[2] = sp->launched;
  out[3] = sp->armed ? 1u : 0u;
  return DN_OK;
}
