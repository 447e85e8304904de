// mimc7_bn254.hip — MiMC7 data / weight commitments on gfx950.
//
// Reference: delta_node/utils/mimc7.py:18-92 over the BN254 scalar field
// q = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001
// (utils/constant.py:6-7) with 13 round constants (constant.py:14-30):
//   mimc7_hash(x, k)      = r_13 + k,  r_0 = x,  r_{i+1} = ((r_i + k + c_i) mod q)^7 mod q
//   mimc7_hash_arr(xs, k) = fold r <- (r + x + mimc7_hash(x, r)) mod q, r_0 = k
//   _float2mpz(v, p)      = min(a, q - a),  a = int(v * 10^p)
//   data commitment: rows -> field ints (features 10^8, label 10^21), zero
//   rows padded to a multiple of 128, hash_arr(row, 2) per row, then a
//   binary Merkle tree of hash_arr([left, right], 2) per 128-row block.
//
// Arithmetic: Montgomery over 9 x 29-bit limbs (R = 2^261, one element per
// lane), separated operand scanning: the 81 limb products of a b and the 81 of
// m q go into 64-bit column accumulators (29-bit limbs leave room for 18
// products per column), so every v_mad_u64_u32 takes its addend straight from
// the accumulator pair — no carry chain per product, no register moves to
// build zero-extended addends (the 8 x 32-bit CIOS form compiled to ~750 VALU
// per product, this one to ~250) and short dependency chains.  R > 170 q, so
// products of operands below 3 q still leave a result below 2 q: the round
// sums r + k + c are carry-normalized but not reduced.  Everything stays in
// Montgomery form between rounds (sums commute with the form);
// t^7 = t^4 t^3: 2 squares (45 limb products) and 2 products per round.  Field values cross memory as
// 8 x 32-bit plain limbs.  The row pass
// is one lane per row (rows are independent chains); the Merkle pass is one
// 64-lane workgroup per 128-leaf block, levels handed over through LDS.
// The weight commitment is one sequential chain by definition (each step
// keys the next hash): one lane, latency-bound.
#include <hip/hip_runtime.h>

#include <cstring>

#include "dn_internal.hpp"
#include "dn_mimc7.h"
#include "mimc7_consts.hpp"

namespace dn {
namespace mimc {

constexpr int L = 8;

constexpr int N = 9;                 // 29-bit limbs of the Montgomery form
constexpr uint32_t kM29 = (1u << 29) - 1;

struct Consts {
  uint32_t q[L];             // 32-bit limbs (float_to_field)
  uint32_t half_q[L];        // floor(q / 2), 32-bit limbs
  uint32_t q29[N];           // q, 29-bit limbs
  uint32_t qinv;             // -q^{-1} mod 2^29
  uint32_t r2[N];            // R^2 mod q, R = 2^261
  uint32_t cts[kRounds][N];  // round constants, Montgomery form
};

// ---- 256-bit helpers (host + device) ----
__host__ __device__ inline bool geq(const uint32_t a[L], const uint32_t b[L]) {
  for (int i = L - 1; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return true;
}

__host__ __device__ inline uint32_t sub_in(uint32_t a[L], const uint32_t b[L]) {  // a -= b, returns borrow
  uint64_t br = 0;
  for (int i = 0; i < L; ++i) {
    const uint64_t d = static_cast<uint64_t>(a[i]) - b[i] - br;
    a[i] = static_cast<uint32_t>(d);
    br = (d >> 63) & 1u;
  }
  return static_cast<uint32_t>(br);
}

__host__ __device__ inline uint32_t add_in(uint32_t a[L], const uint32_t b[L]) {  // a += b, returns carry
  uint64_t c = 0;
  for (int i = 0; i < L; ++i) {
    c += static_cast<uint64_t>(a[i]) + b[i];
    a[i] = static_cast<uint32_t>(c);
    c >>= 32;
  }
  return static_cast<uint32_t>(c);
}

// a = (a + b) mod q for a, b < q (q < 2^254 so a + b < 2^255: no carry out).
__host__ __device__ inline void addmod(uint32_t a[L], const uint32_t b[L], const uint32_t q[L]) {
  add_in(a, b);
  if (geq(a, q)) sub_in(a, q);
}

// ---- 29-bit limb form (host + device) ----
__host__ __device__ inline void to29(const uint32_t a[L], uint32_t o[N]) {
  for (int i = 0; i < N; ++i) {
    const int bit = 29 * i, w = bit / 32, sh = bit % 32;
    const uint64_t lo = a[w], hi = w + 1 < L ? a[w + 1] : 0u;
    o[i] = static_cast<uint32_t>(((hi << 32) | lo) >> sh) & kM29;
  }
}

__host__ __device__ inline void from29(const uint32_t o[N], uint32_t a[L]) {
  uint64_t acc = 0;
  int nb = 0, w = 0;
  for (int i = 0; i < N; ++i) {
    acc |= static_cast<uint64_t>(o[i]) << nb;
    nb += 29;
    while (nb >= 32 && w < L) {
      a[w++] = static_cast<uint32_t>(acc);
      acc >>= 32;
      nb -= 32;
    }
  }
  while (w < L) {
    a[w++] = static_cast<uint32_t>(acc);
    acc >>= 32;
  }
}

__host__ __device__ inline bool geq29(const uint32_t a[N], const uint32_t b[N]) {
  for (int i = N - 1; i >= 0; --i)
    if (a[i] != b[i]) return a[i] > b[i];
  return true;
}

__host__ __device__ inline void sub29_in(uint32_t a[N], const uint32_t b[N]) {  // a -= b (a >= b)
  uint32_t br = 0;
  for (int i = 0; i < N; ++i) {
    const uint32_t d = a[i] - b[i] - br;  // in (-2^30, 2^29)
    br = d >> 31;
    a[i] = d & kM29;
  }
}

// carries of limbs up to 2^32 - 1 into their neighbours (the value fits 9 limbs)
__host__ __device__ inline void norm29(uint32_t a[N]) {
  uint32_t c = 0;
  for (int i = 0; i < N; ++i) {
    const uint32_t v = a[i] + c;
    a[i] = v & kM29;
    c = v >> 29;
  }
}

// a = (a + b) mod q for a, b < q
__host__ __device__ inline void addmod29(uint32_t a[N], const uint32_t b[N], const uint32_t q[N]) {
  for (int i = 0; i < N; ++i) a[i] += b[i];
  norm29(a);
  if (geq29(a, q)) sub29_in(a, q);
}

// Montgomery product r = a b R^{-1} mod q for a, b < 3 q (normalized limbs),
// r < q.  Columns T[i + j] accumulate a_i b_j and m_i q_j (at most 18 products
// of < 2^58 plus a carry < 2^35: below 2^63).
__host__ __device__ inline void mont_mul(uint32_t r[N], const uint32_t a[N], const uint32_t b[N], const Consts& k) {
  uint64_t T[2 * N];
#pragma unroll
  for (int i = 0; i < 2 * N; ++i) T[i] = 0;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) T[i + j] += static_cast<uint64_t>(a[i]) * b[j];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t m = (static_cast<uint32_t>(T[i]) * k.qinv) & kM29;
#pragma unroll
    for (int j = 0; j < N; ++j) T[i + j] += static_cast<uint64_t>(m) * k.q29[j];
    T[i + 1] += T[i] >> 29;  // the low 29 bits of T[i] are now zero
  }
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t v = T[N + i] + c;
    r[i] = static_cast<uint32_t>(v) & kM29;
    c = v >> 29;
  }
  if (geq29(r, k.q29)) sub29_in(r, k.q29);
}

// Montgomery square r = a^2 R^{-1} mod q (same bounds as mont_mul): the 36
// off-diagonal products once, against the doubled limb 2 a_j < 2^30 (each
// column still sums at most 9 products' worth, < 2^59 apiece for the doubled
// ones), plus the 9 squares — 45 instead of 81 multiply-adds before the
// reduction.
__host__ __device__ inline void mont_sqr(uint32_t r[N], const uint32_t a[N], const Consts& k) {
  uint64_t T[2 * N];
  uint32_t a2[N];
#pragma unroll
  for (int i = 0; i < N; ++i) a2[i] = a[i] << 1;
#pragma unroll
  for (int i = 0; i < 2 * N; ++i) T[i] = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    T[2 * i] += static_cast<uint64_t>(a[i]) * a[i];
#pragma unroll
    for (int j = i + 1; j < N; ++j) T[i + j] += static_cast<uint64_t>(a[i]) * a2[j];
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t m = (static_cast<uint32_t>(T[i]) * k.qinv) & kM29;
#pragma unroll
    for (int j = 0; j < N; ++j) T[i + j] += static_cast<uint64_t>(m) * k.q29[j];
    T[i + 1] += T[i] >> 29;
  }
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t v = T[N + i] + c;
    r[i] = static_cast<uint32_t>(v) & kM29;
    c = v >> 29;
  }
  if (geq29(r, k.q29)) sub29_in(r, k.q29);
}

// plain 32-bit limbs (< q) -> Montgomery form, and back (canonical)
__host__ __device__ inline void to_mont(uint32_t r[N], const uint32_t a[L], const Consts& k) {
  uint32_t a29[N];
  to29(a, a29);
  mont_mul(r, a29, k.r2, k);
}

__host__ __device__ inline void from_mont(uint32_t r[L], const uint32_t a[N], const Consts& k) {
  uint32_t one[N] = {1, 0, 0, 0, 0, 0, 0, 0, 0}, t[N];
  mont_mul(t, a, one, k);
  from29(t, r);
}

// mimc7_hash in Montgomery form: (r_13 + k) mod q in `out` (Montgomery).
__host__ __device__ inline void hash_m(uint32_t out[N], const uint32_t x[N], const uint32_t key[N], const Consts& k) {
  uint32_t r[N];
  for (int i = 0; i < N; ++i) r[i] = x[i];
  for (int c = 0; c < kRounds; ++c) {
    uint32_t t[N];
    for (int i = 0; i < N; ++i) t[i] = r[i] + key[i] + k.cts[c][i];  // < 3 q: not reduced
    norm29(t);
    // t^7 = t^4 t^3: depth 3 (t^2; t^4 and t^3 independent; their product)
    uint32_t t2[N], t3[N], t4[N];
    mont_sqr(t2, t, k);
    mont_sqr(t4, t2, k);
    mont_mul(t3, t2, t, k);
    mont_mul(r, t4, t3, k);
  }
  for (int i = 0; i < N; ++i) out[i] = r[i];
  addmod29(out, key, k.q29);
}

// One chain step of mimc7_hash_arr: r <- (r + x + mimc7_hash(x, r)) mod q.
__host__ __device__ inline void arr_step(uint32_t r[N], const uint32_t x[N], const Consts& k) {
  uint32_t h[N];
  hash_m(h, x, r, k);
  addmod29(r, x, k.q29);
  addmod29(r, h, k.q29);
}

// _float2mpz: field value (plain, < q) of min(a, q - a), a = int(v * 10^p);
// returns false if |v * 10^p| >= 2^253 (not handled on the device).
__device__ inline bool float_to_field(double v, double scale, uint32_t out[L], const Consts& k) {
  const double y = v * scale;  // the reference's float multiply
  for (int i = 0; i < L; ++i) out[i] = 0;
  if (y != y) return false;
  const double ay = y < 0 ? -y : y;
  if (!(ay < 14474011154664524427946373126085988481658748083205070504932198000989141204992.0))  // 2^253
    return false;
  // exact integer part of |y| as 8 limbs: mantissa * 2^e
  int e;
  const double m = frexp(ay, &e);  // ay = m 2^e, m in [0.5, 1)
  if (e <= 0) return true;         // |a| = 0
  uint64_t mant = static_cast<uint64_t>(ldexp(m, 53));  // 53-bit integer, ay = mant 2^(e-53)
  int sh = e - 53;
  if (sh < 0) {
    mant >>= -sh;  // truncation toward zero (int())
    sh = 0;
  }
  const int limb = sh / 32, bit = sh % 32;
  const unsigned __int128 wide = static_cast<unsigned __int128>(mant) << bit;  // < 2^117
  // out[limb + d] = word d of wide (d < 4), by select: a dynamic index into
  // out would put the array in scratch memory
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int d = i - limb;
    out[i] = d >= 0 && d < 4 ? static_cast<uint32_t>(wide >> (32 * d)) : 0u;
  }
  const bool neg = y < 0;
  // a = +-out.  min(a, q - a): negative a -> a (value q - |a|); a > q/2 -> q - a.
  if (neg) {
    bool zero = true;
    for (int i = 0; i < L; ++i) zero &= out[i] == 0;
    if (!zero) {
      uint32_t t[L];
      for (int i = 0; i < L; ++i) t[i] = k.q[i];
      sub_in(t, out);
      for (int i = 0; i < L; ++i) out[i] = t[i];
    }
  } else if (!geq(k.half_q, out)) {  // a > floor(q/2)  <=>  a > q - a
    uint32_t t[L];
    for (int i = 0; i < L; ++i) t[i] = k.q[i];
    sub_in(t, out);
    for (int i = 0; i < L; ++i) out[i] = t[i];
  }
  return true;
}

struct RowArgs {
  Consts k;
  const double* data;  // [rows][cols], row-major
  uint64_t rows, rows_pad;
  int32_t cols;
  double scale_feat, scale_label;
  uint32_t* out;  // [rows_pad][8] plain canonical hashes
  uint32_t* bad;
};

__global__ void __launch_bounds__(256) rows_kernel(const RowArgs a) {
  const uint64_t row = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (row >= a.rows_pad) return;
  uint32_t r[N];
  {  // key 2 in Montgomery form
    const uint32_t two[L] = {2, 0, 0, 0, 0, 0, 0, 0};
    to_mont(r, two, a.k);
  }
  bool ok = true;
  for (int c = 0; c < a.cols; ++c) {
    uint32_t x[L], xm[N];
    if (row < a.rows) {
      const double v = a.data[row * a.cols + c];
      ok &= float_to_field(v, c == a.cols - 1 ? a.scale_label : a.scale_feat, x, a.k);
    } else {
      for (int i = 0; i < L; ++i) x[i] = 0;  // padding rows: [0] * cols
    }
    to_mont(xm, x, a.k);
    arr_step(r, xm, a.k);
  }
  uint32_t h[L];
  from_mont(h, r, a.k);
  for (int i = 0; i < L; ++i) a.out[row * L + i] = h[i];
  if (!ok) atomicAdd(a.bad, 1u);
}

struct MerkleArgs {
  Consts k;
  const uint32_t* leaves;  // [blocks * 128][8] plain
  uint32_t* roots;         // [blocks][8] plain
};

// BPW 128-leaf blocks per workgroup of 64 BPW lanes; level sizes 64, 32,
// ..., 1 nodes per block.  The nodes of a level are packed onto the first
// lanes (thread t -> block t / w, node t % w), so every active wave is full
// until a level has fewer than 64 nodes in the workgroup: 33 wave-levels per
// 16 blocks instead of 7 per block (many blocks); BPW = 1 when there are few
// blocks (each level is then one hash-pair latency per wave either way).
template <int BPW>
__global__ void __launch_bounds__(64 * BPW) merkle_kernel(const MerkleArgs a, uint64_t blocks) {
  __shared__ uint32_t s[64 * BPW][N];
  const uint32_t t = threadIdx.x;
  const uint64_t b0 = static_cast<uint64_t>(blockIdx.x) * BPW;
  uint32_t key[N];
  {
    const uint32_t two[L] = {2, 0, 0, 0, 0, 0, 0, 0};
    to_mont(key, two, a.k);
  }
  if (b0 + t / 64 < blocks) {
    const uint32_t* lv = a.leaves + (b0 + t / 64) * 128 * L;
    const uint32_t j = t % 64;
    uint32_t l[L], r[L], lm[N], rm[N], acc[N];
    for (int i = 0; i < L; ++i) {
      l[i] = lv[(2 * j) * L + i];
      r[i] = lv[(2 * j + 1) * L + i];
    }
    to_mont(lm, l, a.k);
    to_mont(rm, r, a.k);
    for (int i = 0; i < N; ++i) acc[i] = key[i];
    arr_step(acc, lm, a.k);
    arr_step(acc, rm, a.k);
    for (int i = 0; i < N; ++i) s[t][i] = acc[i];  // Montgomery form from here on; block b at s[64 b ..]
  }
  __syncthreads();
  for (uint32_t width = 32; width >= 1; width >>= 1) {
    uint32_t nxt[N];
    const uint32_t b = t / width, j = t % width;
    const bool act = t < BPW * width && b0 + b < blocks;
    if (act) {
      for (int i = 0; i < N; ++i) nxt[i] = key[i];
      arr_step(nxt, s[64 * b + 2 * j], a.k);
      arr_step(nxt, s[64 * b + 2 * j + 1], a.k);
    }
    __syncthreads();
    if (act)
      for (int i = 0; i < N; ++i) s[64 * b + j][i] = nxt[i];
    __syncthreads();
  }
  if (t < BPW && b0 + t < blocks) {
    uint32_t out[L];
    from_mont(out, s[64 * t], a.k);
    for (int i = 0; i < L; ++i) a.roots[(b0 + t) * L + i] = out[i];
  }
}

struct ChainArgs {
  Consts k;
  const double* w;
  uint64_t n;
  double scale;
  uint32_t key[L];  // plain
  uint32_t* out;    // [8] plain
  uint32_t* bad;
};

__global__ void chain_kernel(const ChainArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t r[N];
  to_mont(r, a.key, a.k);
  // keep the chain on the VALU: every value here is wave-uniform, and the
  // compiler would otherwise run the products on the scalar unit (slower:
  // DESIGN.md 4.6); an asm-defined VGPR value counts as divergent
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(r[i]));
  bool ok = true;
  for (uint64_t i = 0; i < a.n; ++i) {
    uint32_t x[L], xm[N];
    ok &= float_to_field(a.w[i], a.scale, x, a.k);
    to_mont(xm, x, a.k);
    arr_step(r, xm, a.k);
  }
  uint32_t h[L];
  from_mont(h, r, a.k);
  for (int i = 0; i < L; ++i) a.out[i] = h[i];
  if (!ok) atomicAdd(a.bad, 1u);
}

struct HashArgs {
  Consts k;
  const uint32_t* x;    // [n][8] plain, < q
  const uint32_t* key;  // [n][8] plain, < q
  uint32_t* out;        // [n][9] plain unreduced r + k (< 2q < 2^255; 9th limb 0)
  uint64_t n;
};

__global__ void __launch_bounds__(256) hash_kernel(const HashArgs a) {
  const uint64_t e = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= a.n) return;
  uint32_t x[L], k[L], xm[N], km[N];
  for (int i = 0; i < L; ++i) {
    x[i] = a.x[e * L + i];
    k[i] = a.key[e * L + i];
  }
  to_mont(xm, x, a.k);
  to_mont(km, k, a.k);
  uint32_t r[N];
  for (int i = 0; i < N; ++i) r[i] = xm[i];
  for (int c = 0; c < kRounds; ++c) {
    uint32_t t[N];
    for (int i = 0; i < N; ++i) t[i] = r[i] + km[i] + a.k.cts[c][i];  // < 3 q
    norm29(t);
    uint32_t t2[N], t3[N], t6[N];
    mont_mul(t2, t, t, a.k);
    mont_mul(t3, t2, t, a.k);
    mont_mul(t6, t3, t3, a.k);
    mont_mul(r, t6, t, a.k);
  }
  uint32_t rp[L];
  from_mont(rp, r, a.k);
  const uint32_t carry = add_in(rp, k);  // r + k, unreduced (mimc7.py:26)
  for (int i = 0; i < L; ++i) a.out[e * 9 + i] = rp[i];
  a.out[e * 9 + 8] = carry;
}

// ---- host: constants ----
void make_consts(Consts& k) {
  const uint32_t* q = kQ32;
  std::memcpy(k.q, q, sizeof(k.q));
  to29(q, k.q29);
  // qinv = -q^{-1} mod 2^29 (Newton mod 2^32, then the low 29 bits)
  uint32_t inv = q[0];
  for (int i = 0; i < 5; ++i) inv *= 2u - q[0] * inv;
  k.qinv = (0u - inv) & kM29;
  // R^2 mod q, R = 2^261: double 1 (mod q) 522 times
  uint32_t v[L] = {1, 0, 0, 0, 0, 0, 0, 0};
  for (int it = 0; it < 2 * 29 * N; ++it) {
    uint32_t t[L];
    std::memcpy(t, v, sizeof(t));
    addmod(v, t, q);
  }
  to29(v, k.r2);
  // floor(q / 2)
  for (int i = 0; i < L; ++i) k.half_q[i] = (q[i] >> 1) | (i + 1 < L ? (q[i + 1] << 31) : 0u);
}

}  // namespace mimc
}  // namespace dn

using namespace dn;
using namespace dn::mimc;

namespace {
void consts(Consts& k) {
  std::memset(&k, 0, sizeof(k));
  make_consts(k);
  for (int c = 0; c < kRounds; ++c) {
    uint32_t plain[L];
    dec_to_limbs(kCtsDec[c], plain);
    to_mont(k.cts[c], plain, k);
  }
}

}  // namespace

extern "C" int dn_mimc7_data_rows(const double* data, uint64_t rows, int cols, uint32_t* row_hashes,
                                  uint32_t* bad_count, void* stream) {
  if (cols < 1 || rows == 0) return set_error(DN_ERR_ARG, "dn_mimc7_data_rows: empty data");
  if (!data || !row_hashes || !bad_count) return set_error(DN_ERR_ARG, "dn_mimc7_data_rows: null pointer");
  RowArgs a;
  std::memset(&a, 0, sizeof(a));
  consts(a.k);
  a.data = data;
  a.rows = rows;
  a.rows_pad = (rows + 127) / 128 * 128;
  a.cols = cols;
  a.scale_feat = pow10d(8);
  a.scale_label = pow10d(21);
  a.out = row_hashes;
  a.bad = bad_count;
  hipLaunchKernelGGL(rows_kernel, dim3(static_cast<uint32_t>((a.rows_pad + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mimc7_data_rows: %s", hipGetErrorString(err));
  return DN_OK;
}

extern "C" int dn_mimc7_merkle_blocks(const uint32_t* leaves, uint64_t blocks, uint32_t* roots, void* stream) {
  if (blocks == 0) return DN_OK;
  if (!leaves || !roots) return set_error(DN_ERR_ARG, "dn_mimc7_merkle_blocks: null pointer");
  MerkleArgs a;
  std::memset(&a, 0, sizeof(a));
  consts(a.k);
  a.leaves = leaves;
  a.roots = roots;
  // blocks per workgroup: pack levels across blocks once there are >= 512 workgroups' worth
  const hipStream_t s = static_cast<hipStream_t>(stream);
  if (blocks >= 16 * 512)
    hipLaunchKernelGGL(merkle_kernel<16>, dim3(static_cast<uint32_t>((blocks + 15) / 16)), dim3(64 * 16), 0, s, a, blocks);
  else if (blocks >= 4 * 512)
    hipLaunchKernelGGL(merkle_kernel<4>, dim3(static_cast<uint32_t>((blocks + 3) / 4)), dim3(64 * 4), 0, s, a, blocks);
  else
    hipLaunchKernelGGL(merkle_kernel<1>, dim3(static_cast<uint32_t>(blocks)), dim3(64), 0, s, a, blocks);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mimc7_merkle_blocks: %s", hipGetErrorString(err));
  return DN_OK;
}

extern "C" int dn_mimc7_weight_chain(const double* w, uint64_t n, int precision, uint32_t* out, uint32_t* bad_count,
                                    void* stream) {
  if (!w || !out || !bad_count) return set_error(DN_ERR_ARG, "dn_mimc7_weight_chain: null pointer");
  if (precision < 0 || precision > 22) return set_error(DN_ERR_ARG, "dn_mimc7_weight_chain: precision 0..22");
  ChainArgs a;
  std::memset(&a, 0, sizeof(a));
  consts(a.k);
  a.w = w;
  a.n = n;
  a.scale = pow10d(precision);
  a.key[0] = 2;
  a.out = out;
  a.bad = bad_count;
  hipLaunchKernelGGL(chain_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mimc7_weight_chain: %s", hipGetErrorString(err));
  return DN_OK;
}

extern "C" int dn_mimc7_hash(const uint32_t* xs, const uint32_t* keys, uint64_t n, uint32_t* out, void* stream) {
  if (n == 0) return DN_OK;
  if (!xs || !keys || !out) return set_error(DN_ERR_ARG, "dn_mimc7_hash: null pointer");
  HashArgs a;
  std::memset(&a, 0, sizeof(a));
  consts(a.k);
  a.x = xs;
  a.key = keys;
  a.out = out;
  a.n = n;
  hipLaunchKernelGGL(hash_kernel, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_mimc7_hash: %s", hipGetErrorString(err));
  return DN_OK;
}
