// mt19937_device.hip — CPython's MT19937 coefficient draw on the GPU, bit-exact.
//
// Reference: SecretShare.make_shares draws its t-1 coefficients per element
// with self.random.randint(1, p-1) (delta_node/crypto/shamir/shamir.py:59-61):
// 1 + getrandbits(521), redrawn while >= p-1; getrandbits(521) is 17 MT19937
// words, little-endian, the last >> 23.  dn_mt19937_draw_coeffs (host_m521.cpp)
// restates that stream sequentially; this file produces the same values on the
// device by cutting the word stream into substreams of kMtJumpL words:
//
//  * host: the MT state at the start of each substream by jump-ahead — Horner
//    evaluation of g(f) on the 624-word window with g = x^J mod P, P the
//    characteristic polynomial of the one-word transition f (polynomials for
//    J = kMtJumpL - 624 and 2^k kMtJumpL precomputed by tools/gen_mt_jump.py);
//    substream windows are built by doubling (each from an earlier one by one
//    jump), the jumps of a doubling level spread over host threads;
//  * device: one wave per substream keeps its window in LDS, twists it block
//    by block (the three dependency phases of the 624-word twist, 64 lanes
//    wide), tempers into an LDS ring and turns every complete 17-word group
//    that starts in its substream into one coefficient (+1, rejection test)
//    stored in the tiled layout;
//  * host: the final CPython state (array + index) by stepping the nearest
//    substream window forward, so self.random continues exactly as after n
//    sequential make_shares calls.
// A rejected draw (probability ~2^-520 per coefficient) shifts every later
// word; the device flags it and the caller redoes the draw on the host.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "dn_internal.hpp"
#include "m521_device.hpp"

namespace dn {
namespace {

constexpr int kMtN = 624, kMtM = 397;
constexpr uint32_t kMtA = 0x9908b0dfu, kMtUp = 0x80000000u, kMtLo = 0x7fffffffu;
constexpr int kMtRing = 1024;  // tempered-word ring (>= 624 + 16)

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

// ----------------------------------------------------------------- device
struct MtArgs {
  const uint32_t* windows;  // [subs][624]; window 0 = CPython's array at time B
  uint8_t* coeffs;          // tm1 tiled vectors
  uint32_t* flag;           // != 0: a draw was rejected
  uint64_t n_elem, ncoef, vb;
  uint64_t L;               // words per substream
  uint32_t idx;             // CPython index: stream words 0..623-idx are temper(window0[idx..])
  int32_t tm1;
};

// The workgroup is one wave: LDS traffic between its lanes needs ordering,
// not a hardware barrier (a wavefront-scope fence keeps the compiler from
// moving LDS accesses across it; the LDS executes a wave's accesses in order).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ void __launch_bounds__(64) mt_coeffs_kernel(const MtArgs a) {
  __shared__ uint32_t S[kMtN];
  __shared__ uint32_t R[kMtRing];
  const uint32_t lane = threadIdx.x;
  const uint64_t sub = blockIdx.x;
  const uint64_t lo = sub * a.L, hi = lo + a.L;
  uint64_t k = (lo + 16) / 17;                                   // first coefficient starting here
  const uint64_t k_end = (hi + 16) / 17 < a.ncoef ? (hi + 16) / 17 : a.ncoef;
  if (k >= k_end) return;
  const uint32_t* win = a.windows + sub * kMtN;
  for (int j = lane; j < kMtN; j += 64) S[j] = win[j];
  uint64_t re;  // stream position one past the last word in the ring
  if (sub == 0) {
    const uint32_t h = kMtN - a.idx;
    for (uint32_t j = lane; j < h; j += 64) R[j] = mt_temper(S[a.idx + j]);
    re = h;
  } else {
    re = lo;
  }
  wave_sync();
  while (k < k_end) {
    if (re < 17 * k + 17) {
      // twist S in place (CPython order: three phases, reads before writes in each round)
      for (int r = 0; r < 4; ++r) {  // k in [0, 227): reads S[k + 1], S[k + 397] (old)
        const int kk = r * 64 + static_cast<int>(lane);
        uint32_t v = 0;
        if (kk < kMtN - kMtM) v = mt_mix(S[kk], S[kk + 1], S[kk + kMtM]);
        wave_sync();
        if (kk < kMtN - kMtM) S[kk] = v;
        wave_sync();
      }
      for (int r = 0; r < 4; ++r) {  // k in [227, 454): S[k - 227] new (phase 1)
        const int kk = kMtN - kMtM + r * 64 + static_cast<int>(lane);
        uint32_t v = 0;
        if (kk < 2 * (kMtN - kMtM)) v = mt_mix(S[kk], S[kk + 1], S[kk - (kMtN - kMtM)]);
        wave_sync();
        if (kk < 2 * (kMtN - kMtM)) S[kk] = v;
        wave_sync();
      }
      for (int r = 0; r < 3; ++r) {  // k in [454, 623): S[k - 227] new (previous phase)
        const int kk = 2 * (kMtN - kMtM) + r * 64 + static_cast<int>(lane);
        uint32_t v = 0;
        if (kk < kMtN - 1) v = mt_mix(S[kk], S[kk + 1], S[kk - (kMtN - kMtM)]);
        wave_sync();
        if (kk < kMtN - 1) S[kk] = v;
        wave_sync();
      }
      if (lane == 0) S[kMtN - 1] = mt_mix(S[kMtN - 1], S[0], S[kMtM - 1]);
      wave_sync();
      for (int j = lane; j < kMtN; j += 64) R[(re + j) & (kMtRing - 1)] = mt_temper(S[j]);
      re += kMtN;
      wave_sync();
    }
    const uint64_t kav = re / 17 < k_end ? re / 17 : k_end;  // coefficients complete in the ring
    for (uint64_t base = k; base < kav; base += 64) {
      const uint64_t kk = base + lane;
      if (kk < kav) {
        uint32_t v[kLimbs];
        const uint64_t w0 = 17 * kk;
#pragma unroll
        for (int i = 0; i < kLimbs; ++i) v[i] = R[(w0 + i) & (kMtRing - 1)];
        v[16] >>= 23;
        bool rej = v[16] == 0x1FFu && v[0] >= 0xFFFFFFFEu;
#pragma unroll
        for (int i = 1; i < 16; ++i) rej = rej && v[i] == 0xFFFFFFFFu;
        if (rej) atomicOr(a.flag, 1u);
        uint32_t c = 1u;  // + 1 (randint's lower bound); v < p - 1: no carry out of limb 16
#pragma unroll
        for (int i = 0; i < kLimbs; ++i) {
          const uint64_t s = static_cast<uint64_t>(v[i]) + c;
          v[i] = static_cast<uint32_t>(s);
          c = static_cast<uint32_t>(s >> 32);
        }
        const uint64_t e = kk / static_cast<uint64_t>(a.tm1);
        const uint64_t j = kk - e * static_cast<uint64_t>(a.tm1);
        uint8_t* tb = a.coeffs + j * a.vb + (e / kTile) * kTileBytes;
        const uint32_t w = static_cast<uint32_t>(e % kTile);
#pragma unroll
        for (int i = 0; i < 16; ++i) reinterpret_cast<uint32_t*>(tb)[i * kTile + w] = v[i];
        reinterpret_cast<uint16_t*>(tb + kHiOffset)[w] = static_cast<uint16_t>(v[16]);
      }
    }
    k = kav;
    wave_sync();
  }
}

uint64_t mt_subs(uint64_t ncoef) {
  const uint64_t words = 17 * ncoef;
  const uint64_t L = mt_jump_words();
  return words ? (words + L - 1) / L : 0;
}

}  // namespace
}  // namespace dn

using namespace dn;

extern "C" uint64_t dn_mt19937_device_scratch_bytes(uint64_t n_elem, int tm1) {
  const uint64_t subs = tm1 > 0 ? mt_subs(n_elem * static_cast<uint64_t>(tm1)) : 0;
  return 256 + subs * kMtN * 4;
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
  const uint64_t subs = mt_subs(ncoef);
  if (subs > mt_jump_max_subs())
    return set_error(DN_ERR_UNSUPPORTED, "dn_mt19937_draw_coeffs_device: %llu words exceed the jump table",
                     static_cast<unsigned long long>(17 * ncoef));
  if (scratch_bytes < dn_mt19937_device_scratch_bytes(n_elem, tm1))
    return set_error(DN_ERR_ARG, "dn_mt19937_draw_coeffs_device: scratch too small");

  // substream windows (host jump-ahead, host_mt_jump.cpp)
  std::vector<uint32_t> wins(subs * kMtN);
  mt_build_windows(mt_state, idx, subs, wins.data());

  hipStream_t s = static_cast<hipStream_t>(stream);
  uint8_t* sc = static_cast<uint8_t*>(scratch);
  uint32_t* flag = reinterpret_cast<uint32_t*>(sc);
  uint32_t* dwin = reinterpret_cast<uint32_t*>(sc + 256);
  hipError_t err = hipMemsetAsync(flag, 0, 4, s);
  if (err == hipSuccess) err = hipMemcpyAsync(dwin, wins.data(), wins.size() * 4, hipMemcpyHostToDevice, s);
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mt19937_draw_coeffs_device: %s", hipGetErrorString(err));
  MtArgs a{dwin, static_cast<uint8_t*>(coeffs), flag, n_elem, ncoef, dn_m521_vec_bytes(n_elem), mt_jump_words(),
           static_cast<uint32_t>(idx), tm1};
  hipLaunchKernelGGL(mt_coeffs_kernel, dim3(static_cast<uint32_t>(subs)), dim3(64), 0, s, a);
  err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mt19937_draw_coeffs_device: launch: %s", hipGetErrorString(err));

  // final CPython state while the device works
  std::vector<uint32_t> fin(kMtN);
  int32_t fidx = 0;
  mt_final_state(mt_state, idx, 17 * ncoef, wins.data(), subs, fin.data(), &fidx);
  uint32_t hflag = 0;
  err = hipMemcpyAsync(&hflag, flag, 4, hipMemcpyDeviceToHost, s);
  if (err == hipSuccess) err = hipStreamSynchronize(s);
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mt19937_draw_coeffs_device: %s", hipGetErrorString(err));
  // DN_MT_FORCE_RETRY=1 (test hook) takes the rejected-draw exit so the
  // caller's host fallback can be exercised.
  const char* fr = tune_env("DN_MT_FORCE_RETRY");
  if (hflag || (fr && fr[0] == '1'))
    return set_error(DN_ERR_RETRY, "dn_mt19937_draw_coeffs_device: a draw was rejected; redo on the host");
  std::memcpy(mt_state, fin.data(), kMtN * 4);
  *mt_index = fidx;
  return DN_OK;
}
