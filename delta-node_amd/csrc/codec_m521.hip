// codec_m521.hip — the share wire codec over whole vectors.
//
// Reference (delta_node/crypto/shamir/shamir.py:28-45, serialize/hex.py:44-50):
//   _share_to_bytes((x, y)) = bytes([len(xb)]) + xb + yb,
//   xb / yb = minimal big-endian bytes (0 -> b"").
// The vector form encodes share x of every element into one packed byte
// stream (records back to back) plus int64 offsets[n + 1]; record e is
// exactly the reference's bytes for (x, y_e).  Decoding parses records back
// into a tiled vector (and each record's x).
//
// Encode = three launches: (1) per 1024-element block: record lengths and
// their in-block exclusive scan, block total; (2) scan of the block totals;
// (3) per wave: records assembled in LDS at their final byte positions
// (mod 4 aligned like the destination), then written out as aligned dwords
// plus a few head/tail bytes, so global writes stay contiguous and wide.
#include <hip/hip_runtime.h>

#include <cstring>

#include "dn_internal.hpp"
#include "m521_device.hpp"

namespace dn {

constexpr int kCodecBlock = 256;
constexpr int kScanElems = 1024;       // elements per scan block (4 per thread)
constexpr int kMaxRecord = 1 + 8 + 66;  // [len][x up to 8 bytes][y up to 66 bytes]

struct XBytes {
  uint32_t len;
  uint8_t b[8];  // big-endian minimal bytes of x
};

// Minimal big-endian byte length of a canonical 17-limb value (0 -> 0).
__device__ __forceinline__ uint32_t y_len(const uint32_t v[kLimbs]) {
  uint32_t len = 0;
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) {
    if (v[i]) len = 4u * i + (32u - __builtin_clz(v[i]) + 7u) / 8u;
  }
  return len;
}

// y length of element w of a tile from limbs 15 .. 0 (the top limb was zero)
__device__ __noinline__ uint32_t y_len_low(const uint8_t* tb, uint32_t w) {
  for (int i = 15; i >= 0; --i) {
    const uint32_t l = reinterpret_cast<const uint32_t*>(tb)[i * kTile + w];
    if (l) return 4u * i + (32u - __builtin_clz(l) + 7u) / 8u;
  }
  return 0u;
}

// Per 1024-element block: record lengths of 4 consecutive elements per thread
// (one 8-B load of their top-limb u16s: the only read unless a top limb is
// zero, odds 2^-9), their in-block exclusive prefix (wave scans by shuffles,
// then across the 4 waves) as one 16-B store per thread, and the block total.
__global__ void __launch_bounds__(kCodecBlock) lengths_scan_kernel(const uint8_t* __restrict__ vec, uint64_t n,
                                                                    uint32_t xlen, uint32_t* __restrict__ local,
                                                                    uint64_t* __restrict__ block_tot) {
  __shared__ uint32_t s_w[kCodecBlock / 64];
  const uint64_t b = blockIdx.x;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint64_t e0 = b * kScanElems + t * 4;  // 4 consecutive elements, one tile (256 % 4 == 0)
  uint32_t len[4] = {0u, 0u, 0u, 0u};
  if (e0 < n) {
    const uint8_t* tb = tile_base(vec, static_cast<uint32_t>(e0 / kTile));
    const uint32_t w0 = static_cast<uint32_t>(e0 % kTile);
    uint16_t top[4];
    if (e0 + 4 <= n) {
      const uint64_t q = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(tb + kHiOffset) + w0 / 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) top[j] = static_cast<uint16_t>(q >> (16 * j));
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) top[j] = e0 + j < n ? reinterpret_cast<const uint16_t*>(tb + kHiOffset)[w0 + j] : 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (e0 + j < n) {
        const uint32_t tp = top[j] & kTopMask;
        len[j] = 1u + xlen + (tp ? 64u + (32u - __builtin_clz(tp) + 7u) / 8u : y_len_low(tb, w0 + j));
      }
    }
  }
  const uint32_t sum = len[0] + len[1] + len[2] + len[3];
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += v;
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kCodecBlock / 64; ++w) {
    wbase += (w < static_cast<int>(wv)) ? s_w[w] : 0u;
    tot += s_w[w];
  }
  uint32_t run = wbase + inc - sum;  // exclusive prefix of this thread's 4 elements
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 o;
  o.x = run;
  o.y = run + len[0];
  o.z = run + len[0] + len[1];
  o.w = run + len[0] + len[1] + len[2];
  if (e0 + 4 <= n) {
    __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(local + e0));
  } else {
    const uint32_t ov[4] = {o.x, o.y, o.z, o.w};
    for (int j = 0; j < 4; ++j)
      if (e0 + j < n) local[e0 + j] = ov[j];
  }
  if (t == 0) block_tot[b] = tot;
}

// Exclusive scan of the block totals in one workgroup: the totals
// are staged in LDS as 32-bit words (a block's total is at most 1024 * 76
// bytes) with coalesced loads, each thread scans a contiguous run of them
// (padded rows: no bank conflicts), the run sums are scanned across threads.
constexpr int kScanThreads = 1024;
constexpr int kScanStage = 8192;  // totals staged per pass (34 KB of LDS)

__global__ void __launch_bounds__(kScanThreads) scan_blocks_kernel(uint64_t* __restrict__ tot, uint64_t nb,
                                                                   uint64_t* __restrict__ total_out) {
  __shared__ uint32_t s[kScanStage + kScanStage / 8];  // row of 8 + 1 pad per thread
  __shared__ uint64_t s_w[kScanThreads / 64];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  uint64_t carry = 0;  // total of the previous passes
  for (uint64_t base = 0; base < nb; base += kScanStage) {
    const uint32_t m = static_cast<uint32_t>(nb - base < kScanStage ? nb - base : kScanStage);
    for (uint32_t i = t; i < m; i += kScanThreads) s[i + i / 8] = static_cast<uint32_t>(tot[base + i]);
    __syncthreads();
    // thread t: totals 8 t .. 8 t + 7 of this pass
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = 8u * t + j;
      sum += i < m ? s[i + i / 8] : 0u;
    }
    uint64_t inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t v = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += v;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint64_t wbase = 0, ptot = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
      wbase += (w < static_cast<int>(wv)) ? s_w[w] : 0u;
      ptot += s_w[w];
    }
    uint64_t run = carry + wbase + inc - sum;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = 8u * t + j;
      if (i < m) {
        const uint32_t v = s[i + i / 8];
        tot[base + i] = run;
        run += v;
      }
    }
    carry += ptot;
    __syncthreads();
  }
  if (t == 0) *total_out = carry;
}

// One wave = 64 consecutive elements = one contiguous run of records.
// Each lane lays its record into the wave's LDS window at its final byte
// position (mod 4 like the destination): the 1 + xlen header bytes one by
// one, then y.  y's minimal big-endian bytes are the tail of the 68-byte
// big-endian image W_0..W_16 (W_m = bswap(limb 16 - m)) ending at the record
// end E, so with r = (68 - E) mod 4 every destination dword is one
// v_alignbyte of two neighbouring W words (static indices): dwords wholly
// inside [y start, E) go out as ds_write_b32, the two partial edge dwords
// byte by byte.  The window is then written to HBM as aligned dwords.
__device__ __forceinline__ void lds_put_bytes(uint8_t* sb, int32_t lo, int32_t hi, int32_t pos, uint32_t word) {
  // bytes of `word` (LE at LDS position pos) that fall inside [lo, hi)
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (pos + i >= lo && pos + i < hi) sb[pos + i] = static_cast<uint8_t>(word >> (8 * i));
}

// W16: `out` is 16-B aligned, so the window is laid out from the 16-B boundary
// at or below its start and the body goes out as 16-B stores (else 4-B ones).
template <bool W16>
__global__ void __launch_bounds__(kCodecBlock) encode_kernel(const uint8_t* __restrict__ vec, uint64_t n, XBytes xb,
                                                             const uint32_t* __restrict__ local,
                                                             const uint64_t* __restrict__ block_pre,
                                                             uint64_t* __restrict__ offsets, uint8_t* __restrict__ out) {
  constexpr int kRowWords = ((64 * kMaxRecord + 8 + 16) / 4 + 2 + 3) & ~3;  // 16-B aligned rows
  __shared__ __attribute__((aligned(16))) uint32_t s_buf[kCodecBlock / 64][kRowWords];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t e = (static_cast<uint64_t>(blockIdx.x) * kCodecBlock) + threadIdx.x;
  const bool valid = e < n;
  const uint64_t vmask = __ballot(valid);
  if (!vmask) return;  // wave-uniform: the whole wave is past the end
  uint32_t v[kLimbs];
  uint64_t off = 0;
  uint32_t ylen = 0;
  if (valid) {
    load_fe(tile_base(vec, static_cast<uint32_t>(e / kTile)), static_cast<uint32_t>(e % kTile), v);
    ylen = y_len(v);
    off = block_pre[e / kScanElems] + local[e];
    offsets[e] = off;
    if (e == n - 1) offsets[n] = off + 1 + xb.len + ylen;
  }
  // the wave's byte range [A, B)
  const uint64_t A = __shfl(off, 0);
  const uint32_t last = static_cast<uint32_t>(63 - __builtin_clzll(vmask));
  const uint64_t endl = off + (valid ? 1 + xb.len + ylen : 0);
  const uint64_t B = __shfl(endl, last);
  const uint64_t A4 = W16 ? (A & ~15ull) : (A & ~3ull);  // LDS byte 0 of the window
  uint8_t* sb = reinterpret_cast<uint8_t*>(s_buf[wv]);
  uint32_t* sw4 = s_buf[wv];
  if (valid) {
    const int32_t p = static_cast<int32_t>(off - A4);
    const int32_t ys = p + 1 + static_cast<int32_t>(xb.len);
    const int32_t E = ys + static_cast<int32_t>(ylen);
    sb[p] = static_cast<uint8_t>(xb.len);
    for (uint32_t i = 0; i < xb.len; ++i) sb[p + 1 + i] = xb.b[i];
    if (ylen) {
      uint32_t W[kLimbs + 1];
#pragma unroll
      for (int m = 0; m < kLimbs; ++m) W[m] = __builtin_bswap32(v[kLimbs - 1 - m]);
      W[kLimbs] = 0u;
      const int32_t base = E - 4 * kLimbs;           // LDS position of image byte 0
      const uint32_t r = static_cast<uint32_t>(-base) & 3u;
      const int32_t d0 = (base + static_cast<int32_t>(r)) >> 2;  // dword holding image bytes r..r+3
      // dword d0 - 1: image bytes 0..r-1 at its top (r > 0)
      if (r) lds_put_bytes(sb, ys, E, 4 * (d0 - 1), __builtin_amdgcn_alignbyte(W[0], 0u, r));
#pragma unroll
      for (int m = 0; m < kLimbs; ++m) {
        const uint32_t u = __builtin_amdgcn_alignbyte(W[m + 1], W[m], r);
        const int32_t pos = 4 * (d0 + m);
        if (pos >= ys && pos + 4 <= E) sw4[d0 + m] = u;
        else if (pos + 4 > ys && pos < E) lds_put_bytes(sb, ys, E, pos, u);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // head bytes [A, a4), aligned body [a4, b4), tail [b4, B)
  constexpr uint64_t kAl = W16 ? 16u : 4u;
  const uint64_t a4 = (A + kAl - 1) & ~(kAl - 1), b4 = B & ~(kAl - 1);
  if (a4 > b4) {  // the whole range sits inside one aligned chunk
    for (uint64_t q = A + lane; q < B; q += 64) out[q] = sb[q - A4];
    return;
  }
  if (lane < a4 - A) out[A + lane] = sb[A + lane - A4];
  if (lane < B - b4) out[b4 + lane] = sb[b4 + lane - A4];
  if constexpr (W16) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* sq = reinterpret_cast<const u32x4*>(s_buf[wv]);
    u32x4* oq = reinterpret_cast<u32x4*>(out + a4);
    const uint32_t base_q = static_cast<uint32_t>((a4 - A4) / 16);
    const uint32_t nq = static_cast<uint32_t>((b4 - a4) / 16);
    for (uint32_t q = lane; q < nq; q += 64) __builtin_nontemporal_store(sq[base_q + q], oq + q);
  } else {
    const uint32_t* sw = s_buf[wv];
    uint32_t* ow = reinterpret_cast<uint32_t*>(out + a4);
    const uint32_t base_w = static_cast<uint32_t>((a4 - A4) / 4);
    const uint32_t nw = static_cast<uint32_t>((b4 - a4) / 4);
    for (uint32_t q = lane; q < nw; q += 64) __builtin_nontemporal_store(sw[base_w + q], ow + q);
  }
}

// Decode record e -> element e of a tiled vector (+ its x).  y is reduced
// mod p (resolve_shares reduces ys the same way, shamir.py:86-88).  Records
// whose y has more than 68 significant bytes, or whose x is longer than
// 8 bytes, are counted in *bad and stored as 0 (the caller re-decodes them).
//
// One wave = 64 consecutive records = one contiguous byte window: the wave
// stages the window in LDS with dword loads, then each lane rebuilds its limbs
// from the record's tail: LE limb i is the big-endian dword ending 4i bytes
// before the record end, i.e. bswap of one v_alignbyte of two LDS dwords,
// masked to the bytes after the y start.  Windows larger than the LDS slice
// (records padded with leading zero bytes) take the byte-serial path.
__device__ __forceinline__ bool parse_record_global(const uint8_t* __restrict__ in, uint64_t o, uint64_t end,
                                                    uint64_t& x, uint32_t v[kLimbs]) {
  bool ok = end > o;
  const uint32_t xlen = ok ? in[o] : 0u;
  x = 0;
  ok = ok && xlen <= 8 && o + 1 + xlen <= end;
  if (ok)
    for (uint32_t i = 0; i < xlen; ++i) x = (x << 8) | in[o + 1 + i];
#pragma unroll
  for (int i = 0; i < kLimbs; ++i) v[i] = 0u;
  if (ok) {
    const uint64_t y0 = o + 1 + xlen;
    uint64_t skip = 0;  // leading zero bytes are allowed (bytes_to_int ignores them)
    while (y0 + skip < end && in[y0 + skip] == 0) ++skip;
    const uint64_t sig = end - y0 - skip;
    ok = sig <= 68;
    if (ok) {
      for (uint64_t i = 0; i < sig; ++i) {
        const uint32_t byte = in[end - 1 - i];
        v[i >> 2] |= byte << (8 * (i & 3));
      }
    }
  }
  return ok;
}

constexpr int kDecPad = 16;  // LDS bytes before / after each wave's window
constexpr int kDecWindow = 64 * kMaxRecord + 8;

// W16: the input is 16-B aligned, so the window is staged with 16-B loads and
// LDS stores from the 16-B boundary at or below its start (else 4-B ones).
template <bool W16>
__global__ void __launch_bounds__(kCodecBlock) decode_kernel(const uint8_t* __restrict__ in, uint64_t in_bytes,
                                                             const uint64_t* __restrict__ offsets, uint64_t n,
                                                             uint8_t* __restrict__ vec, uint64_t* __restrict__ xs,
                                                             uint32_t* __restrict__ bad) {
  constexpr int kRowWords = ((kDecWindow + 16 + 2 * kDecPad) / 4 + 3) & ~3;  // 16-B aligned rows
  __shared__ __attribute__((aligned(16))) uint32_t s_win[kCodecBlock / 64][kRowWords];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t e0 = (static_cast<uint64_t>(blockIdx.x) * kCodecBlock) + (threadIdx.x & ~63u);
  if (e0 >= n) return;  // wave-uniform
  const uint64_t e = e0 + lane;
  const bool valid = e < n;
  const uint64_t eN = e0 + 64 < n ? e0 + 64 : n;
  const uint64_t A = offsets[e0], Bend = offsets[eN];
  const uint64_t A4 = W16 ? (A & ~15ull) : (A & ~3ull);  // window base (all positions below are from it)
  uint64_t x = 0;
  uint32_t v[kLimbs];
  bool ok;
  if (Bend >= A && Bend <= in_bytes && Bend - A4 <= static_cast<uint64_t>(kDecWindow) + 12u) {
    uint32_t* S = s_win[wv] + kDecPad / 4;  // S[k] = dword at window byte 4k
    uint8_t* sb = reinterpret_cast<uint8_t*>(S);
    if constexpr (W16) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const uint64_t B16 = Bend & ~15ull;
      const uint32_t nq = static_cast<uint32_t>((B16 - A4) / 16);
      const u32x4* inq = reinterpret_cast<const u32x4*>(in + A4);
      u32x4* Sq = reinterpret_cast<u32x4*>(S);
      for (uint32_t q = lane; q < nq; q += 64) Sq[q] = __builtin_nontemporal_load(inq + q);
      if (lane < Bend - B16) sb[B16 - A4 + lane] = in[B16 + lane];
    } else {
      const uint64_t B4 = Bend & ~3ull;
      const uint32_t nw = static_cast<uint32_t>((B4 - A4) / 4);
      const uint32_t* inw = reinterpret_cast<const uint32_t*>(in + A4);
      for (uint32_t q = lane; q < nw; q += 64) S[q] = __builtin_nontemporal_load(inw + q);
      if (lane < Bend - B4) sb[B4 - A4 + lane] = in[B4 + lane];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    ok = false;
#pragma unroll
    for (int i = 0; i < kLimbs; ++i) v[i] = 0u;
    if (valid) {
      const uint64_t oe = offsets[e], ee = offsets[e + 1];
      // untrusted offsets: the record must lie inside this wave's window
      ok = oe >= A && ee > oe && ee <= Bend;
      const int32_t o = static_cast<int32_t>(oe - A4), end = static_cast<int32_t>(ee - A4);
      const uint32_t xlen = ok ? sb[o] : 0u;
      ok = ok && xlen <= 8 && o + 1 + static_cast<int32_t>(xlen) <= end;
      if (ok) {
        for (uint32_t i = 0; i < xlen; ++i) x = (x << 8) | sb[o + 1 + i];
        int32_t ys = o + 1 + static_cast<int32_t>(xlen);
        for (; end - ys > 68; ++ys)  // leading zero bytes beyond 68 (rare)
          if (sb[ys]) {
            ok = false;
            break;
          }
        if (ok) {
#pragma unroll
          for (int i = 0; i < kLimbs; ++i) {
            const int32_t q = end - 4 * (i + 1);        // window position of limb i's top byte
            const int32_t nv = end - ys - 4 * i;         // bytes of limb i inside y
            const int32_t qa = q < -4 ? -4 : q;          // stay inside the padded slice
            const uint32_t lo = S[qa >> 2], hi = S[(qa >> 2) + 1];
            uint32_t w = __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, lo, static_cast<uint32_t>(qa) & 3u));
            w = nv >= 4 ? w : (nv <= 0 ? 0u : (w & ((1u << (8 * nv)) - 1u)));
            v[i] = w;
          }
        }
      }
    }
  } else if (valid) {
    const uint64_t oe = offsets[e], ee = offsets[e + 1];
    ok = oe < ee && ee <= in_bytes && parse_record_global(in, oe, ee, x, v);
    if (!ok) {
#pragma unroll
      for (int i = 0; i < kLimbs; ++i) v[i] = 0u;
    }
  } else {
    ok = false;
  }
  if (!valid) return;
  if (ok) {
    reduce(v);
  } else {
#pragma unroll
    for (int i = 0; i < kLimbs; ++i) v[i] = 0u;
    atomicAdd(bad, 1u);
  }
  store_fe(tile_base(vec, static_cast<uint32_t>(e / kTile)), static_cast<uint32_t>(e % kTile), v);
  if (xs) xs[e] = x;
}

}  // namespace dn

using namespace dn;

extern "C" uint64_t dn_m521_codec_scratch_bytes(uint64_t n_elem) {
  const uint64_t nb = (n_elem + kScanElems - 1) / kScanElems;
  return n_elem * 4 + nb * 8 + 8 + 256;
}

extern "C" uint64_t dn_m521_encoded_capacity(uint64_t n_elem, uint64_t x) {
  uint32_t xl = 0;
  while (xl < 8 && (x >> (8 * xl))) ++xl;
  return n_elem * (1 + xl + 66);
}

extern "C" int dn_m521_encode_shares(const void* vec, uint64_t n_elem, uint64_t x, uint64_t* offsets, uint8_t* out,
                                     uint64_t capacity, void* scratch, uint64_t scratch_bytes, void* stream) {
  if (n_elem == 0) return DN_OK;
  if (!vec || !offsets || !out || !scratch) return set_error(DN_ERR_ARG, "dn_m521_encode_shares: null pointer");
  if (capacity < dn_m521_encoded_capacity(n_elem, x))
    return set_error(DN_ERR_ARG, "dn_m521_encode_shares: capacity %llu < %llu", (unsigned long long)capacity,
                     (unsigned long long)dn_m521_encoded_capacity(n_elem, x));
  if (scratch_bytes < dn_m521_codec_scratch_bytes(n_elem))
    return set_error(DN_ERR_ARG, "dn_m521_encode_shares: scratch too small");
  XBytes xb;
  std::memset(&xb, 0, sizeof(xb));
  while (xb.len < 8 && (x >> (8 * xb.len))) ++xb.len;
  for (uint32_t i = 0; i < xb.len; ++i) xb.b[i] = static_cast<uint8_t>(x >> (8 * (xb.len - 1 - i)));
  const uint64_t nb = (n_elem + kScanElems - 1) / kScanElems;
  uint32_t* local = static_cast<uint32_t*>(scratch);
  uint64_t* tot = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(scratch) + ((n_elem * 4 + 15) & ~15ull));
  uint64_t* total = tot + nb;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint8_t* v = static_cast<const uint8_t*>(vec);
  hipLaunchKernelGGL(lengths_scan_kernel, dim3(static_cast<uint32_t>(nb)), dim3(kCodecBlock), 0, s, v, n_elem,
                     xb.len, local, tot);
  hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(1024), 0, s, tot, nb, total);
  const uint64_t blocks = (n_elem + kCodecBlock - 1) / kCodecBlock;
  bool w16 = (reinterpret_cast<uintptr_t>(out) & 15u) == 0;
#ifdef DN_TUNING
  if (tune_env("DN_ENCODE_W4") && tune_env("DN_ENCODE_W4")[0] == '1') w16 = false;  // A/B: 4-B stores
#endif
  if (w16)
    hipLaunchKernelGGL(encode_kernel<true>, dim3(static_cast<uint32_t>(blocks)), dim3(kCodecBlock), 0, s, v, n_elem,
                       xb, local, tot, offsets, out);
  else
    hipLaunchKernelGGL(encode_kernel<false>, dim3(static_cast<uint32_t>(blocks)), dim3(kCodecBlock), 0, s, v, n_elem,
                       xb, local, tot, offsets, out);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_m521_encode_shares: %s", hipGetErrorString(err));
  return DN_OK;
}

extern "C" int dn_m521_decode_shares(const uint8_t* in, uint64_t in_bytes, const uint64_t* offsets, uint64_t n_elem,
                                     void* vec, uint64_t* xs, uint32_t* bad_count, void* stream) {
  if (n_elem == 0) return DN_OK;
  if (!in || !offsets || !vec || !bad_count) return set_error(DN_ERR_ARG, "dn_m521_decode_shares: null pointer");
  const uint64_t blocks = (n_elem + kCodecBlock - 1) / kCodecBlock;
  bool w16 = (reinterpret_cast<uintptr_t>(in) & 15u) == 0;
#ifdef DN_TUNING
  if (tune_env("DN_DECODE_W4") && tune_env("DN_DECODE_W4")[0] == '1') w16 = false;  // A/B: 4-B staging
#endif
  if (w16)
    hipLaunchKernelGGL(decode_kernel<true>, dim3(static_cast<uint32_t>(blocks)), dim3(kCodecBlock), 0,
                       static_cast<hipStream_t>(stream), in, in_bytes, offsets, n_elem, static_cast<uint8_t*>(vec), xs,
                       bad_count);
  else
    hipLaunchKernelGGL(decode_kernel<false>, dim3(static_cast<uint32_t>(blocks)), dim3(kCodecBlock), 0,
                       static_cast<hipStream_t>(stream), in, in_bytes, offsets, n_elem, static_cast<uint8_t*>(vec), xs,
                       bad_count);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_m521_decode_shares: %s", hipGetErrorString(err));
  return DN_OK;
}
