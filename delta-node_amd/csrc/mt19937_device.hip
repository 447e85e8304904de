// mt19937_device.hip — CPython's MT19937 coefficient draw on the GPU, bit-exact.
//
// Reference: SecretShare.make_shares draws its t-1 coefficients per element
// with self.random.randint(1, p-1) (delta_node/crypto/shamir/shamir.py:59-61):
// 1 + getrandbits(521), redrawn while >= p-1; getrandbits(521) is 17 MT19937
// words, little-endian, the last >> 23.  dn_mt19937_draw_coeffs (host_m521.cpp)
// restates that stream sequentially; this file produces the same values on the
// device by cutting the word stream into S substreams of L = 17 * 2^15 words
// (2^15 whole draws each), all on the GPU:
//
//  * jump kernels: the MT window at the start of every substream by
//    jump-ahead, g(f)(W) with g = x^J mod P (P the characteristic polynomial
//    of the one-word transition f; tools/gen_mt_jump.py), evaluated by
//    Horner over 4-bit chunks of g: r <- f^4(r) ^ T[chunk], T the 16
//    combinations of f^0..f^3(W) in LDS.  A wave holds r (624 words + 16 free
//    slots) in 10 VGPRs; f^4 appends 4 words (readlane -> scalar twist ->
//    writelane).  Windows are at most three jumps (radix-64 digits of s - 1,
//    mt19937_jump.inc) from the caller's window: one launch per level, every
//    jump of a level independent;
//  * generation kernel: one wave per substream keeps its window in LDS,
//    twists it (CPython's three dependency phases, up to 4 words per lane),
//    tempers into an LDS ring and turns every 17-word group into one
//    coefficient (+1, rejection test) stored in the tiled layout; one extra
//    wave steps the last window before CPython's final array to it, so
//    self.random continues exactly as after n sequential make_shares calls.
// A rejected draw (probability ~2^-520 per coefficient) shifts every later
// word; the device flags it and the caller redoes the draw on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "dn_internal.hpp"
#include "m521_device.hpp"

namespace dn {
namespace {

#include "mt19937_jump.inc"

__device__ const uint64_t kMtPolysDev[kMtJumpRows][kMtPolyWords] = DN_MT_JUMP_POLYS;

constexpr int kMtN = 624, kMtM = 397;
constexpr uint32_t kMtA = 0x9908b0dfu, kMtUp = 0x80000000u, kMtLo = 0x7fffffffu;
constexpr uint64_t kCoefPerSub = kMtJumpL / 17;            // 2^14 draws per substream
constexpr int kGroup = 64 * 17;                            // words of one emission group (64 draws)
constexpr int kRingG = 2 * kGroup;                         // tempered-word ring of the generation wave
static_assert(kMtJumpL % 17 == 0, "substreams hold whole 17-word draws");

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

// ------------------------------------------------------------------ jumps
struct JumpJob {
  int32_t src, poly, dst, pad;  // window indices (dst < 0: padding), jump-table row
};

struct JumpArgs {
  uint32_t* wins;  // [S + 1][624]: window s at row s, the caller's window advanced idx words at row S
  const JumpJob* jobs;
  uint32_t njobs;
};

constexpr int kERow = 704;  // E row: 16 zero words, then 684 words of a T stream (+4 pad)

// One workgroup = 4 jumps from the same source window W (the host groups
// them).  Horner over 4-bit chunks of g, 16 chunks (one 64-bit word of g) per
// step: r <- f^64(r) ^ sum_t f^(4 (15 - t))(T[c_t]), T[v] = sum over bits j of
// v of f^j(W).  f^m(T[v]) is the window at offset m of T[v]'s own stream, so
// the workgroup stores those streams once, E[v] = words 0..683 of T[v]'s
// stream (LDS, 45 KB), and a step is
//   * f^64(r): 64 new words mix(r[l], r[l+1], r[l+397]), l = 0..63 — one
//     register, its operands gathered by 3 ds_bpermute;
//   * the XOR of 16 E windows into the 624 window words (10 registers, 160
//     LDS reads and XORs per lane).
// Registers: Q[11] is a 704-slot ring (slot 64 r + lane); at the start of a
// step word i of r sits at slot 16 + i, the new words land in Q[10] (slots
// 640..703), and afterwards the frame moves by one register.
__global__ void __launch_bounds__(256) mt_jump_kernel(const JumpArgs a) {
  __shared__ uint32_t E[16 * kERow];
  __shared__ uint32_t ext[kMtN + 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  const uint32_t j0 = blockIdx.x * 4u;
  const JumpJob* jp = a.jobs + __builtin_amdgcn_readfirstlane(j0 + wid < a.njobs ? j0 + wid : j0);
  const int32_t poly = __builtin_amdgcn_readfirstlane(jp->poly), dsti = __builtin_amdgcn_readfirstlane(jp->dst);
  const uint32_t* src = a.wins + static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(a.jobs[j0].src)) * kMtN;
  // the source stream: words 0..623 of W, then 63 more (each from words <= 459 of W)
  for (uint32_t i = tid; i < kMtN; i += 256u) ext[i] = src[i];
  __syncthreads();
  if (tid < 63u) ext[kMtN + tid] = mt_mix(ext[tid], ext[tid + 1], ext[tid + kMtM]);
  __syncthreads();
  for (uint32_t e = tid; e < 16u * kERow; e += 256u) {
    const uint32_t v = e / kERow, i = e - v * kERow;
    uint32_t x = 0u;
    if (i >= 16u && i < 16u + 684u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) x ^= ext[i - 16u + j] & (0u - ((v >> j) & 1u));
    }
    E[e] = x;
  }
  __syncthreads();
  if (j0 + wid >= a.njobs || dsti < 0) return;

  const uint64_t* g = kMtPolysDev[poly];
  uint32_t Q[11];
#pragma unroll
  for (int r = 0; r < 11; ++r) Q[r] = 0u;
  // ds_bpermute byte addresses: lane (l + 16), (l + 17), (l + 29) mod 64
  const int pa = static_cast<int>(((lane + 16u) & 63u) * 4u), pb = static_cast<int>(((lane + 17u) & 63u) * 4u),
            pm = static_cast<int>(((lane + 29u) & 63u) * 4u);
  const uint32_t* El = E + lane;
  int top = kMtPolyWords - 1;
  while (top > 0 && g[top] == 0ull) --top;  // steps above it leave r = 0
#pragma unroll 1
  for (int wi = top; wi >= 0; --wi) {
    const uint64_t gw = g[wi];
    // f^64: word l at slot 16 + l, word l + 1 at 17 + l, word l + 397 at 413 + l
    const uint32_t xa = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(pa, static_cast<int>(lane < 16u ? Q[1] : Q[0])));
    const uint32_t xb = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(pb, static_cast<int>(lane < 17u ? Q[1] : Q[0])));
    const uint32_t xm = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(pm, static_cast<int>(lane < 29u ? Q[7] : Q[6])));
    Q[10] = mt_mix(xa, xb, xm);
    // new word i (old stream word 64 + i) sits at slot 80 + i: XOR E[c_t][16 + 4 (15 - t) + i]
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint32_t c = static_cast<uint32_t>(gw >> (60 - 4 * t)) & 15u;
      const uint32_t* Ec = El + c * kERow + (60 - 4 * t);
#pragma unroll
      for (int r = 1; r < 11; ++r) Q[r] ^= Ec[64 * (r - 1)];
    }
    const uint32_t q0 = Q[0];
#pragma unroll
    for (int r = 0; r < 10; ++r) Q[r] = Q[r + 1];
    Q[10] = q0;
  }
  uint32_t* dst = a.wins + static_cast<uint64_t>(dsti) * kMtN;
#pragma unroll
  for (int r = 0; r < 11; ++r) {
    const int i = 64 * r + static_cast<int>(lane) - 16;
    if (i >= 0 && i < kMtN) dst[i] = Q[r];
  }
}

// ------------------------------------------------------------------ generation
struct GenArgs {
  const uint32_t* wins;  // [S + 1][624]
  uint8_t* coeffs;       // tm1 tiled vectors
  uint32_t* flag;        // != 0: a draw was rejected
  uint32_t* fin;         // CPython's final array (the final-state wave)
  uint64_t ncoef, vb;
  uint64_t tm1_magic;    // ceil(2^32 / tm1): x / tm1 = (x * magic) >> 32 for x < 2^16
  uint32_t S;            // substreams
  uint32_t idx;          // CPython index: stream words 0..623-idx are temper(window0[idx..])
  int32_t tm1;
  int32_t final_sig;     // window the final-state wave starts from (-1: no such wave)
  uint64_t final_pos;    // position of that window's first word (0: the caller's array)
  uint64_t final_tf;     // position of CPython's final array
};

// The generation wave keeps the MT stream in registers exactly as a jump
// wave keeps r: Q[11] a 704-slot ring, the window's word i at slot 16 + i
// of the current frame.  One append = the next 64 words of the stream
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

// 64 draws of one group (lane = draw c of this substream, words 17 c .. 17 c +
// 16 of the ring at `rb` words): +1, rejection test, tiled store.
__device__ __forceinline__ void emit_group(const GenArgs& a, const uint32_t* rb, uint64_t qb, uint32_t rbm,
                                          uint32_t c, uint32_t nloc, uint32_t lane) {
  if (c >= nloc) return;
  uint32_t v[kLimbs];
  const uint32_t* w = rb + 17u * lane;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) v[i] = w[i];
  v[16] >>= 23;
  uint32_t all = v[1];
#pragma unroll
  for (int i = 2; i < 16; ++i) all &= v[i];
  if (v[16] == 0x1FFu && v[0] >= 0xFFFFFFFEu && all == 0xFFFFFFFFu) atomicOr(a.flag, 1u);  // >= p - 1: rejected
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

template <int... ks>
__device__ __forceinline__ void gen_run(uint32_t (&Q)[11], const Lanes& L, uint32_t* R, uint32_t& wpos,
                                        std::integer_sequence<int, ks...>) {
  // each append: temper the 64 new words into the ring at stream word wpos
  ((void)[&] {
     const uint32_t t = mt_temper(append64<ks>(Q, L));
     uint32_t pos = wpos + (threadIdx.x & 63u);
     pos = pos >= static_cast<uint32_t>(kRingG) ? pos - kRingG : pos;
     R[pos] = t;
     wpos = wpos + 64u >= static_cast<uint32_t>(kRingG) ? wpos + 64u - kRingG : wpos + 64u;
   }(),
   ...);
}

template <int... ks>
__device__ __forceinline__ void final_run(uint32_t (&Q)[11], const Lanes& L, uint64_t& np, uint64_t tf,
                                          uint32_t* fin, std::integer_sequence<int, ks...>) {
  ((void)[&] {
     const uint32_t v = append64<ks>(Q, L);
     const uint64_t x = np + (threadIdx.x & 63u);
     if (x >= tf && x < tf + kMtN) fin[x - tf] = v;
     np += 64u;
   }(),
   ...);
}

__global__ void __launch_bounds__(256) mt_gen_kernel(const GenArgs a) {
  __shared__ uint32_t s_ring[4][kRingG];
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  const uint32_t sub = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + wid);
  if (sub > a.S || (sub == a.S && a.final_sig < 0)) return;
  const bool fin_wave = sub == a.S;
  const uint32_t wsel = fin_wave ? static_cast<uint32_t>(a.final_sig) : sub;
  const uint32_t* win = a.wins + static_cast<uint64_t>(wsel) * kMtN;
  Lanes L;
  L.pa = static_cast<int>(((lane + 16u) & 63u) * 4u);
  L.pb = static_cast<int>(((lane + 17u) & 63u) * 4u);
  L.pm = static_cast<int>(((lane + 29u) & 63u) * 4u);
  L.la = lane < 16u, L.lb = lane < 17u, L.lm = lane < 29u;
  uint32_t Q[11];
#pragma unroll
  for (int r = 0; r < 11; ++r) {
    const int i = 64 * r + static_cast<int>(lane) - 16;
    Q[r] = (i >= 0 && i < kMtN) ? win[i] : 0u;
  }
  const auto run11 = std::make_integer_sequence<int, 11>{};
  if (fin_wave) {
    // step from the window at final_pos until positions tf .. tf + 623 are produced
    const uint64_t P = a.final_pos, tf = a.final_tf;
    for (uint32_t i = lane; i < static_cast<uint32_t>(kMtN); i += 64u)
      if (P + i >= tf && P + i < tf + kMtN) a.fin[P + i - tf] = win[i];
    uint64_t np = P + kMtN;
    while (np < tf + kMtN) final_run(Q, L, np, tf, a.fin, run11);
    return;
  }
  uint32_t* R = s_ring[wid];
  const uint64_t k0 = static_cast<uint64_t>(sub) * kCoefPerSub;  // first draw of this substream
  const uint32_t nloc = static_cast<uint32_t>(a.ncoef - k0 < kCoefPerSub ? a.ncoef - k0 : kCoefPerSub);
  const uint32_t ngroups = (nloc + 63u) / 64u;
  const uint64_t qb = k0 / static_cast<uint64_t>(a.tm1);
  const uint32_t rbm = static_cast<uint32_t>(k0 - qb * static_cast<uint64_t>(a.tm1));
  uint32_t wpos = 0;  // ring position of the next stream word of this substream
  if (sub == 0) {     // the rest of the caller's array comes first
    const uint32_t h = kMtN - a.idx;
    for (uint32_t j = lane; j < h; j += 64u) R[j] = mt_temper(win[a.idx + j]);
    wpos = h;
  }
  uint32_t done = 0, have = wpos;  // groups emitted, stream words produced
  while (done < ngroups) {
    gen_run(Q, L, R, wpos, run11);
    have += 11u * 64u;
    wave_sync();
    while (done < ngroups && have >= (done + 1u) * static_cast<uint32_t>(kGroup)) {
      emit_group(a, R + (done & 1u) * kGroup, qb, rbm, 64u * done + lane, nloc, lane);
      ++done;
    }
    wave_sync();
  }
}

uint64_t mt_subs(uint64_t ncoef) { return (ncoef + kCoefPerSub - 1) / kCoefPerSub; }

// Jump jobs of one level, grouped by source window in fours (padding: dst -1).
void push_group(std::vector<JumpJob>& jobs, int32_t src, const std::vector<std::pair<int32_t, int32_t>>& pd) {
  for (size_t i = 0; i < pd.size(); ++i) jobs.push_back({src, pd[i].first, pd[i].second, 0});
  while (jobs.size() % 4) jobs.push_back({src, 0, -1, 0});
}

// Levels for windows 1 .. S-1 (s - 1 = 4096 c + 64 a + b; row S holds W_idx):
// A: W(1 + 64 a) = A_a(W_idx); C: W(1 + 4096 c + 64 a) = C_c(W(1 + 64 a));
// B: W(base + b) = B_b(W(base)).
void build_levels(uint64_t S, std::vector<JumpJob> lv[3]) {
  const uint64_t R = kMtJumpRadix;
  if (S < 2) return;
  const uint64_t last = S - 2;  // largest s - 1
  {
    std::vector<std::pair<int32_t, int32_t>> pd;
    for (uint64_t a = 0; a <= last / R && a < R; ++a)
      pd.push_back({kMtRowA + static_cast<int32_t>(a), static_cast<int32_t>(1 + R * a)});
    for (size_t i = 0; i < pd.size(); i += 4)
      push_group(lv[0], static_cast<int32_t>(S),
                 std::vector<std::pair<int32_t, int32_t>>(pd.begin() + i, pd.begin() + std::min(pd.size(), i + 4)));
  }
  for (uint64_t a = 0; a < R && R * a <= last; ++a) {  // C: per source W(1 + 64 a), its c digits
    std::vector<std::pair<int32_t, int32_t>> pd;
    for (uint64_t c = 1; c < R && R * R * c + R * a <= last; ++c)
      pd.push_back({kMtRowC + static_cast<int32_t>(c), static_cast<int32_t>(1 + R * R * c + R * a)});
    for (size_t i = 0; i < pd.size(); i += 4)
      push_group(lv[1], static_cast<int32_t>(1 + R * a),
                 std::vector<std::pair<int32_t, int32_t>>(pd.begin() + i, pd.begin() + std::min(pd.size(), i + 4)));
  }
  for (uint64_t base = 0; base <= last; base += R) {  // B: per source W(1 + base)
    std::vector<std::pair<int32_t, int32_t>> pd;
    for (uint64_t b = 1; b < R && base + b <= last; ++b)
      pd.push_back({kMtRowB + static_cast<int32_t>(b), static_cast<int32_t>(1 + base + b)});
    for (size_t i = 0; i < pd.size(); i += 4)
      push_group(lv[2], static_cast<int32_t>(1 + base),
                 std::vector<std::pair<int32_t, int32_t>>(pd.begin() + i, pd.begin() + std::min(pd.size(), i + 4)));
  }
}

uint64_t jobs_cap(uint64_t S) { return 2 * S + 1024; }  // >= the three levels with padding

constexpr uint64_t kHead = 4096;  // flag (4 B at 0), final array (2496 B at 256)

}  // namespace
}  // namespace dn

using namespace dn;

extern "C" uint64_t dn_mt19937_device_scratch_bytes(uint64_t n_elem, int tm1) {
  const uint64_t S = tm1 > 0 ? mt_subs(n_elem * static_cast<uint64_t>(tm1)) : 0;
  return kHead + (S + 1) * kMtN * 4 + jobs_cap(S) * sizeof(JumpJob);
}

extern "C" int dn_mt19937_draw_coeffs_device(uint32_t* mt_state, int32_t* mt_index, uint64_t n_elem, int tm1,
                                             void* coeffs, void* scratch, uint64_t scratch_bytes, void* stream) {
  if (!mt_state || !mt_index) return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs_device: null pointer");
  if (tm1 < 0 || tm1 >= DN_MAX_THRESHOLD)
    return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs_device: t-1=%d", tm1);
  const int32_t idx = *mt_index;
  if (idx < 0 || idx > kMtN) return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs_device: bad MT index");
  const uint64_t ncoef = n_elem * static_cast<uint64_t>(tm1);
  if (ncoef == 0) return DN_OK;
  if (!coeffs || !scratch) return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs_device: null pointer");
  const uint64_t S = mt_subs(ncoef);
  if (S > mt_jump_max_subs() - 1)
    return set_error(DN_ERR_UNSUPPORTED, "dn_mt19937_draw_coeffs_device: %llu words exceed the jump table",
                     static_cast<unsigned long long>(17 * ncoef));
  if (scratch_bytes < dn_mt19937_device_scratch_bytes(n_elem, tm1))
    return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs_device: scratch too small");

  // CPython's state after the draw: the array at buffer position tf = 624 q,
  // stepped by the final-state wave from window `sig` (position P_sig < tf)
  const uint64_t words = 17 * ncoef, h = static_cast<uint64_t>(kMtN - idx);
  int32_t sig = -1, fidx = idx + static_cast<int32_t>(words <= h ? words : 0);
  uint64_t fpos = 0, ftf = 0;
  if (words > h) {
    const uint64_t m_end = words - h, q = (m_end + kMtN - 1) / kMtN, tf = kMtN * q;
    uint64_t s = (tf + kMtN - 1 - static_cast<uint64_t>(idx)) / kMtJumpL;  // idx + s L - 624 < tf
    if (s > S - 1) s = S - 1;
    sig = static_cast<int32_t>(s);
    fpos = s ? static_cast<uint64_t>(idx) + s * kMtJumpL - kMtN : 0;
    ftf = tf;
    fidx = static_cast<int32_t>(m_end - kMtN * (q - 1));
  }

  // host staging: window 0 = the caller's array, row S = it advanced idx words; the jump jobs
  std::vector<JumpJob> lv[3];
  build_levels(S, lv);
  const uint64_t njobs = lv[0].size() + lv[1].size() + lv[2].size();
  if (njobs > jobs_cap(S)) return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs_device: job table overflow");
  std::vector<uint32_t> w_idx(kMtN);
  mt_advance_window(mt_state, static_cast<uint64_t>(idx), w_idx.data());

  hipStream_t s = static_cast<hipStream_t>(stream);
  uint8_t* sc = static_cast<uint8_t*>(scratch);
  uint32_t* flag = reinterpret_cast<uint32_t*>(sc);
  uint32_t* fin = reinterpret_cast<uint32_t*>(sc + 256);
  uint32_t* dwin = reinterpret_cast<uint32_t*>(sc + kHead);
  JumpJob* djobs = reinterpret_cast<JumpJob*>(sc + kHead + (S + 1) * kMtN * 4);
  std::vector<JumpJob> all;
  all.reserve(njobs);
  for (auto& l : lv) all.insert(all.end(), l.begin(), l.end());
  hipError_t err = hipMemsetAsync(flag, 0, 4, s);
  if (err == hipSuccess) err = hipMemcpyAsync(dwin, mt_state, kMtN * 4, hipMemcpyHostToDevice, s);
  if (err == hipSuccess) err = hipMemcpyAsync(dwin + S * kMtN, w_idx.data(), kMtN * 4, hipMemcpyHostToDevice, s);
  if (err == hipSuccess && njobs)
    err = hipMemcpyAsync(djobs, all.data(), njobs * sizeof(JumpJob), hipMemcpyHostToDevice, s);
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mt19937_draw_coeffs_device: %s", hipGetErrorString(err));
  uint64_t off = 0;
  for (auto& l : lv) {
    if (!l.empty()) {
      const JumpArgs ja{dwin, djobs + off, static_cast<uint32_t>(l.size())};
      hipLaunchKernelGGL(mt_jump_kernel, dim3(static_cast<uint32_t>(l.size() / 4)), dim3(256), 0, s, ja);
    }
    off += l.size();
  }
  GenArgs ga{dwin, static_cast<uint8_t*>(coeffs), flag, fin, ncoef, dn_m521_vec_bytes(n_elem),
             ((1ull << 32) + static_cast<uint64_t>(tm1) - 1) / static_cast<uint64_t>(tm1), static_cast<uint32_t>(S),
             static_cast<uint32_t>(idx), tm1, sig, fpos, ftf};
  hipLaunchKernelGGL(mt_gen_kernel, dim3(static_cast<uint32_t>((S + 1 + 3) / 4)), dim3(256), 0, s, ga);
  err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mt19937_draw_coeffs_device: launch: %s", hipGetErrorString(err));

  std::vector<uint32_t> head(256 / 4 + kMtN);  // flag .. final array
  err = hipMemcpyAsync(head.data(), sc, head.size() * 4, hipMemcpyDeviceToHost, s);
  if (err == hipSuccess) err = hipStreamSynchronize(s);
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mt19937_draw_coeffs_device: %s", hipGetErrorString(err));
  // DN_MT_FORCE_RETRY=1 (tuning build) takes the rejected-draw exit so the
  // caller's host fallback can be exercised.
  const char* fr = tune_env("DN_MT_FORCE_RETRY");
  if (head[0] || (fr && fr[0] == '1'))
    return set_error(DN_ERR_RETRY, "dn_mt19937_draw_coeffs_device: a draw was rejected; redo on the host");
  if (sig >= 0) std::memcpy(mt_state, head.data() + 256 / 4, kMtN * 4);
  *mt_index = fidx;
  return DN_OK;
}
