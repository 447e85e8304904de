// aes_envelope.hip — the share envelope on gfx950 (SURVEY.md §8(f) row 2,
// second half): AES-CTR + base64 (+ hex) over whole messages.
//
// Reference (delta-mpc/delta-node):
//   aes.encrypt(key, data) = b64encode(nonce || AES-CTR(key, nonce)(data)),
//                            nonce = os.urandom(16)      crypto/aes/aes.py:8-14
//   aes.decrypt(key, text) = AES-CTR(key, raw[:16])(raw[16:]),
//                            raw = b64decode(text)       crypto/aes/aes.py:17-23
// `cryptography`'s CTR (OpenSSL): the nonce is a 128-bit big-endian counter
// block, +1 per 16-byte block, mod 2^128.  The runner seals each share for its
// receiver (runner/horizontal/agg.py:191-196) and hex-encodes the envelope into
// the coordinator's JSON (serialize.bytes_to_hex, serialize/hex.py:11-26;
// runner/horizontal/commu.py:23-49; app/v1/coord.py:93-94 accepts
// "0x[0-9a-fA-F]+"); the receiver undoes both (agg.py:258-266).  For a vector
// share — the packed _share_to_bytes records of codec_m521.hip — that message
// is megabytes to gigabytes per receiver.
//
// AES: T-table rounds.  Te_k (Te0 rotated right by 8k) live in LDS, each
// replicated 32 times and interleaved so that lane l reads replica l % 32:
// every ds_read_b32 of a 32-lane half hits 32 distinct banks (conflict-free
// for any indices).  A table row is 256 B (two tables x 32 replicas), so the
// LDS address of Te_k[byte j of s] is ONE v_perm_b32 of s and a per-lane word
// (replica in byte 0, table pair in byte 2); the second table of a pair is the
// instruction's +128 offset.  NTAB = 4 keeps all four tables (128 KB, one
// 1024-thread workgroup per CU); NTAB = 2 keeps Te0/Te1 (64 KB) and rotates by
// 16 for Te2/Te3.  Round keys are kernel arguments (SGPRs).  CDNA4 has no AES
// instructions: this is LDS + VALU work, not HBM-bound.
//
// encrypt fuses base64 (and hex): one thread unit = 48 bytes of the base64
// input nonce || ct — keystream blocks 3g-1, 3g, 3g+1, block -1 being the
// nonce — -> 64 base64 characters -> 128 hex digits; decrypt runs the units
// backwards.  Units 0 and last (nonce, '=' padding, ragged end) go byte-wise.
// Inputs may start at any byte (e.g. after "0x"): data = base + skew with a
// 16-byte aligned base, read as aligned vectors and funnel-shifted
// (v_alignbyte); outputs are 16-byte aligned.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "dn_aes.h"
#include "dn_internal.hpp"

// DN_AES_SDWA (default 1): round lookups address LDS through SDWA byte moves
// (aes_block); 0 builds the v_perm form (the A/B baseline, `make variant`).
#ifndef DN_AES_SDWA
#define DN_AES_SDWA 1
#endif
// DN_AES_HEX_LDS (default 1): the encrypt-to-hex kernel turns base64 sextets
// into hex digit pairs by LDS lookups (hex_lds_word) instead of the SWAR
// base64 + hex arithmetic; 0 builds the SWAR form (A/B baseline).
#ifndef DN_AES_HEX_LDS
#define DN_AES_HEX_LDS 1
#endif
// DN_AES_HEX_COAL (default 1, with DN_AES_HEX_LDS): a wave whose 64 lanes all
// hold whole units stores its 8 KB of hex text line by line (hex_coalesce:
// cross-lane transpose, each store instruction one contiguous KB) instead of
// each lane its own 128 bytes (16 B in each of 64 lines per instruction).
// 2 (default): two transpose stages instead of three (hex_coalesce_half: no
// selects), each store writing the 64-B halves of 16 lines: 1.339-1.342 vs
// 1.364-1.382 ms (profiles/r05/r/).
#ifndef DN_AES_HEX_COAL
#define DN_AES_HEX_COAL 2
#endif
// DN_AES_DEC_SPLIT: 2 (default) = one pass with decode_kernel's coalesced,
// transposed text reads (decrypt_fused_kernel): 1.67-1.70 vs 1.95-1.96 ms for
// the two passes (profiles/r05/x/); 1 = two passes, decode then CTR in place
// (decode_kernel, ctr_text_kernel); 0 = the one-pass decrypt_kernel with
// per-lane text reads.
#ifndef DN_AES_DEC_SPLIT
#define DN_AES_DEC_SPLIT 2
#endif
// DN_AES_DEC_COAL: the decrypt kernels read a wave's hex text line by line
// and transpose it (as the encrypt kernel's text stores).  2 (default since
// round 6): half lines, transposed by hex_coalesce_half (two permlane-swap
// stages, no selects or DPP) — in the VALU-heavy one-pass decrypt
// (decrypt_fused_kernel) 1.593-1.611 vs 1.615-1.646 ms, 4 of 4 alternating
// pairs (profiles/r06/v/); the two-pass decode_kernel of round 5 was the
// other way round (1.98-2.01 vs 1.94-1.96 ms, profiles/r05/s/).  1: whole
// lines, three stages (hex_coalesce).
#ifndef DN_AES_DEC_COAL
#define DN_AES_DEC_COAL 2
#endif
// DN_AES_NB (default 3): keystream blocks of an encrypt unit whose rounds run
// interleaved (aes_blocks); 2 = two interleaved + one alone, 1 = one at a time.
#ifndef DN_AES_NB
#define DN_AES_NB 3
#endif

namespace dn {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kPadChar = 0x3Du;  // '='
constexpr uint32_t kDecPad = 0x40u;   // base64 decode table: '='
constexpr uint32_t kDecBad = 0x80u;   // base64 decode table: outside the alphabet

struct AesArgs {
  uint32_t rk[60];    // round keys, big-endian words (FIPS-197 w[i])
  uint32_t iv[4];     // initial counter block, big-endian words (encrypt / ctr)
  const uint8_t* in;  // 16-byte aligned; the data starts at in + skew
  uint8_t* out;       // 16-byte aligned
  uint64_t n;         // encrypt / ctr: plaintext bytes; decrypt: base64 characters
  uint64_t units;     // thread units (ctr: 16-byte blocks)
  uint64_t* out_len;  // decrypt: plaintext bytes (device)
  uint32_t* bad;      // decrypt: non-canonical text seen (device)
  uint32_t skew;      // 0..15
  uint32_t plain;     // encrypt text stores without the nt hint (default; DN_AES_STORE=nt to A/B)
};

template <int NTAB>
struct AesLds {
  uint32_t tab[NTAB / 2][256][64];  // [pair][byte][32 x Te_{2 pair} | 32 x Te_{2 pair + 1}]
  uint32_t te0[256];
  uint8_t dec[256];  // base64 character -> sextet / kDecPad / kDecBad
};

// ---- GF(2^8), S-box, tables -------------------------------------------------
__host__ __device__ inline uint32_t gf_x2(uint32_t a) { return ((a << 1) ^ (0x1Bu & (0u - ((a >> 7) & 1u)))) & 0xFFu; }

__host__ __device__ inline uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t r = 0u;
  for (int i = 0; i < 8; ++i) {
    r ^= a & (0u - ((b >> i) & 1u));
    a = gf_x2(a);
  }
  return r;
}

// S(x) = affine(x^254) (FIPS-197 §5.1.1); x^254 = x^(2+4+...+128), 0 -> 0.
__host__ __device__ inline uint32_t aes_sbox(uint32_t x) {
  uint32_t p = gf_mul(x, x), inv = p;
  for (int i = 0; i < 6; ++i) {
    p = gf_mul(p, p);
    inv = gf_mul(inv, p);
  }
  const uint32_t r = inv | (inv << 8);  // rotl8(inv, k) = (r >> (8 - k)) & 0xFF
  return (inv ^ (r >> 7) ^ (r >> 6) ^ (r >> 5) ^ (r >> 4) ^ 0x63u) & 0xFFu;
}

template <int NTAB>
__device__ void build_tables(AesLds<NTAB>& L) {
  constexpr uint32_t TH = NTAB == 4 ? 1024u : 512u;
  for (uint32_t e = threadIdx.x; e < 256u; e += TH) {
    const uint32_t s = aes_sbox(e), s2 = gf_x2(s);
    L.te0[e] = (s2 << 24) | (s << 16) | (s << 8) | (s2 ^ s);  // (2S, S, S, 3S)
    uint32_t d = kDecBad;
    if (e >= 'A' && e <= 'Z') d = e - 'A';
    else if (e >= 'a' && e <= 'z') d = e - 'a' + 26u;
    else if (e >= '0' && e <= '9') d = e - '0' + 52u;
    else if (e == '+') d = 62u;
    else if (e == '/') d = 63u;
    else if (e == '=') d = kDecPad;
    L.dec[e] = static_cast<uint8_t>(d);
  }
  __syncthreads();
  uint32_t* flat = &L.tab[0][0][0];
  for (uint32_t w = threadIdx.x; w < (NTAB / 2) * 256u * 64u; w += TH) {
    const uint32_t k = 2u * (w >> 14) + ((w >> 5) & 1u);  // which Te_k this word holds
    const uint32_t v = L.te0[(w >> 6) & 255u];
    flat[w] = __builtin_amdgcn_alignbit(v, v, 8u * k);
  }
  __syncthreads();
}

// Te_T[byte K of s] from this lane's replica; lw[p] = (lane % 32) * 4 | p << 16.
template <int NTAB, int K, int T>
__device__ __forceinline__ uint32_t te(const AesLds<NTAB>& L, uint32_t s, const uint32_t lw[2]) {
  constexpr int P = NTAB == 4 ? T / 2 : 0;  // table pair (LDS region)
  constexpr int H = T & 1;                  // first or second table of the pair
  const uint32_t addr = __builtin_amdgcn_perm(s, lw[P], 0x0C020000u | ((4u + K) << 8));
  uint32_t v = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(&L.tab[0][0][0]) + addr + 128 * H);
  if constexpr (NTAB == 2 && T >= 2) v = __builtin_amdgcn_alignbit(v, v, 16);
  return v;
}

// One column of SubBytes + ShiftRows + MixColumns + AddRoundKey (big-endian words).
template <int NTAB>
__device__ __forceinline__ uint32_t mix_col(const AesLds<NTAB>& L, const uint32_t lw[2], uint32_t a, uint32_t b,
                                            uint32_t c, uint32_t d, uint32_t k) {
  return te<NTAB, 3, 0>(L, a, lw) ^ te<NTAB, 2, 1>(L, b, lw) ^ te<NTAB, 1, 2>(L, c, lw) ^ te<NTAB, 0, 3>(L, d, lw) ^ k;
}

// Final round: the S-box bytes, taken out of Te0 = (2S, S, S, 3S) by v_perm.
template <int NTAB>
__device__ __forceinline__ uint32_t sub_col(const AesLds<NTAB>& L, const uint32_t lw[2], uint32_t a, uint32_t b,
                                            uint32_t c, uint32_t d, uint32_t k) {
  const uint32_t hi = __builtin_amdgcn_perm(te<NTAB, 3, 0>(L, a, lw), te<NTAB, 2, 0>(L, b, lw), 0x06020C0Cu);
  const uint32_t lo = __builtin_amdgcn_perm(te<NTAB, 1, 0>(L, c, lw), te<NTAB, 0, 0>(L, d, lw), 0x0C0C0602u);
  return hi ^ lo ^ k;
}

// Te_T[byte K of s] with the LDS address built by one SDWA v_mov (VOP1, a
// full-rate slot) instead of a v_perm (VOP3): byte 1 of this lookup's own
// address register ar — its lane and table-pair bits set once — is
// overwritten with byte K of s (dst_unused:UNUSED_PRESERVE keeps the rest).
// Each of a round's 16 lookups has its own register, so a register is
// rewritten a whole round after the read that used it.
template <int K>
__device__ __forceinline__ void addr_byte(uint32_t& ar, uint32_t s) {
  if constexpr (K == 0) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(ar) : "v"(s));
  else if constexpr (K == 1) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(ar) : "v"(s));
  else if constexpr (K == 2) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(ar) : "v"(s));
  else asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(ar) : "v"(s));
}

// a ^ b ^ c in one v_bitop3 (table 0x96); the compiler leaves the round's
// five-term XORs as four v_xor_b32 otherwise.  xor3s takes a wave-uniform
// third operand (a round key).  The builtin, not inline asm: the compiler
// then knows the instruction and schedules around it (inline asm blocks got
// an s_nop between dependent ones).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t xor3s(uint32_t a, uint32_t b, uint32_t k) {
  return __builtin_amdgcn_bitop3_b32(a, b, k, 0x96);
}

// DN_AES_B1 (default 1): a byte-1 lookup's address is (s & 0xFF00) | ar, one
// full-rate v_bitop3 (ar keeps its lane and table bits, byte 1 zero), instead
// of the half-rate SDWA move the other three byte positions need.
#ifndef DN_AES_B1
#define DN_AES_B1 1
#endif

template <int K, int T>
__device__ __forceinline__ uint32_t te_sdwa(const AesLds<4>& L, uint32_t s, uint32_t& ar) {
  const uint8_t* base = reinterpret_cast<const uint8_t*>(&L.tab[0][0][0]) + 128 * (T & 1);
  if constexpr (K == 1 && DN_AES_B1)
    return *reinterpret_cast<const uint32_t*>(base + __builtin_amdgcn_bitop3_b32(s, 0xFF00u, ar, 0xEA));
  addr_byte<K>(ar, s);
  return *reinterpret_cast<const uint32_t*>(base + ar);
}

// Final round (SubBytes + ShiftRows + AddRoundKey) through the same address
// registers as the middle rounds: x_t = Te_t[byte 3 - t of column c + t]
// holds S at byte 2 (Te0), 1 (Te1), 0 (Te2), 2 (Te3); two v_perm place the
// four S bytes, one v_bitop3 adds the round key.
__device__ __forceinline__ void final_round_sdwa(const AesLds<4>& L, const uint32_t st[4], uint32_t (&ar)[4][4],
                                                 const uint32_t* rk, uint32_t out[4]) {
  uint32_t x[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    x[c][0] = te_sdwa<3, 0>(L, st[c], ar[c][0]);
    x[c][1] = te_sdwa<2, 1>(L, st[(c + 1) & 3], ar[c][1]);
    x[c][2] = te_sdwa<1, 2>(L, st[(c + 2) & 3], ar[c][2]);
    x[c][3] = te_sdwa<0, 3>(L, st[(c + 3) & 3], ar[c][3]);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < 4; ++c)
    out[c] = xor3s(__builtin_amdgcn_perm(x[c][0], x[c][1], 0x06010C0Cu),
                   __builtin_amdgcn_perm(x[c][2], x[c][3], 0x0C0C0402u), rk[c]);
}

template <int NR, int NTAB>
__device__ __forceinline__ void aes_block(const AesLds<NTAB>& L, const uint32_t lw[2], const AesArgs& a,
                                          uint32_t s[4]) {
  uint32_t s0 = s[0] ^ a.rk[0], s1 = s[1] ^ a.rk[1], s2 = s[2] ^ a.rk[2], s3 = s[3] ^ a.rk[3];
#if DN_AES_SDWA
  if constexpr (NTAB == 4) {
    uint32_t ar[4][4];  // [column][table]: lane bits | table pair (T / 2) << 16
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < 4; ++t) ar[c][t] = lw[t >> 1];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
      // the round's 16 lookups issued back to back, then the XORs
      uint32_t x[4][4];
      const uint32_t st[4] = {s0, s1, s2, s3};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        x[c][0] = te_sdwa<3, 0>(L, st[c], ar[c][0]);
        x[c][1] = te_sdwa<2, 1>(L, st[(c + 1) & 3], ar[c][1]);
        x[c][2] = te_sdwa<1, 2>(L, st[(c + 2) & 3], ar[c][2]);
        x[c][3] = te_sdwa<0, 3>(L, st[(c + 3) & 3], ar[c][3]);
      }
      __builtin_amdgcn_sched_barrier(0);
      s0 = xor3s(xor3(x[0][0], x[0][1], x[0][2]), x[0][3], a.rk[4 * r]);
      s1 = xor3s(xor3(x[1][0], x[1][1], x[1][2]), x[1][3], a.rk[4 * r + 1]);
      s2 = xor3s(xor3(x[2][0], x[2][1], x[2][2]), x[2][3], a.rk[4 * r + 2]);
      s3 = xor3s(xor3(x[3][0], x[3][1], x[3][2]), x[3][3], a.rk[4 * r + 3]);
    }
    const uint32_t st[4] = {s0, s1, s2, s3};
    final_round_sdwa(L, st, ar, a.rk + 4 * NR, s);
    return;
  }
#endif
#pragma unroll
  for (int r = 1; r < NR; ++r) {
    const uint32_t t0 = mix_col(L, lw, s0, s1, s2, s3, a.rk[4 * r]);
    const uint32_t t1 = mix_col(L, lw, s1, s2, s3, s0, a.rk[4 * r + 1]);
    const uint32_t t2 = mix_col(L, lw, s2, s3, s0, s1, a.rk[4 * r + 2]);
    const uint32_t t3 = mix_col(L, lw, s3, s0, s1, s2, a.rk[4 * r + 3]);
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  s[0] = sub_col(L, lw, s0, s1, s2, s3, a.rk[4 * NR]);
  s[1] = sub_col(L, lw, s1, s2, s3, s0, a.rk[4 * NR + 1]);
  s[2] = sub_col(L, lw, s2, s3, s0, s1, a.rk[4 * NR + 2]);
  s[3] = sub_col(L, lw, s3, s0, s1, s2, a.rk[4 * NR + 3]);
}

// NB independent blocks (NTAB == 4, SDWA addressing) with their rounds
// interleaved: each round issues the 16 lookups of every block back to back,
// then the XORs, so a wave has 16 NB LDS reads in flight per round instead of
// 16 (4 waves per SIMD at one 1024-thread workgroup per CU hide too little of
// one block's read latency).  The 16 address registers are shared by the
// blocks: a lookup's register is rewritten for the next block after the read
// that used it has been issued (in order).
template <int NR, int NB>
__device__ __forceinline__ void aes_blocks(const AesLds<4>& L, const uint32_t lw[2], const AesArgs& a,
                                           uint32_t s[NB][4]) {
#if DN_AES_SDWA
  uint32_t st[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) st[b][i] = s[b][i] ^ a.rk[i];
  uint32_t ar[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int t = 0; t < 4; ++t) ar[c][t] = lw[t >> 1];
#pragma unroll
  for (int r = 1; r < NR; ++r) {
    uint32_t x[NB][4][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        x[b][c][0] = te_sdwa<3, 0>(L, st[b][c], ar[c][0]);
        x[b][c][1] = te_sdwa<2, 1>(L, st[b][(c + 1) & 3], ar[c][1]);
        x[b][c][2] = te_sdwa<1, 2>(L, st[b][(c + 2) & 3], ar[c][2]);
        x[b][c][3] = te_sdwa<0, 3>(L, st[b][(c + 3) & 3], ar[c][3]);
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) st[b][c] = xor3s(xor3(x[b][c][0], x[b][c][1], x[b][c][2]), x[b][c][3], a.rk[4 * r + c]);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) final_round_sdwa(L, st[b], ar, a.rk + 4 * NR, s[b]);
#else
#pragma unroll
  for (int b = 0; b < NB; ++b) aes_block<NR>(L, lw, a, s[b]);
#endif
}

// Counter block iv + b (mod 2^128) as big-endian words.
__device__ __forceinline__ void ctr_block(const uint32_t iv[4], uint64_t b, uint32_t w[4]) {
  const uint64_t lo0 = (static_cast<uint64_t>(iv[2]) << 32) | iv[3];
  const uint64_t lo = lo0 + b;
  const uint64_t hi = ((static_cast<uint64_t>(iv[0]) << 32) | iv[1]) + (lo < lo0 ? 1ull : 0ull);
  w[0] = static_cast<uint32_t>(hi >> 32);
  w[1] = static_cast<uint32_t>(hi);
  w[2] = static_cast<uint32_t>(lo >> 32);
  w[3] = static_cast<uint32_t>(lo);
}

// ---- loads / stores -----------------------------------------------------------
template <int Q, int NV>
__device__ __forceinline__ void shift_words(const uint32_t* r, uint32_t sb, uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 4 * NV; ++i) w[i] = __builtin_amdgcn_alignbyte(r[i + Q + 1], r[i + Q], sb);
}

// 16 NV bytes of the stream at byte `off` (a multiple of 16) of data = base + skew,
// as little-endian words: load_raw issues the aligned vector loads (NV, or NV + 1
// with skew != 0 — all hold wanted bytes, none is read past the 16-byte chunk of
// the last one), shift_raw funnel-shifts them into place.  Split so that a loop
// can issue the next unit's loads before this unit's stores: loads and stores
// retire in issue order (one vmcnt), so a load issued after a store waits for it.
template <int NV>
__device__ __forceinline__ void load_raw(const uint8_t* base, uint32_t skew, uint64_t off, uint32_t (&r)[4 * NV + 4]) {
  const u32x4* p = reinterpret_cast<const u32x4*>(base + off);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const u32x4 x = __builtin_nontemporal_load(p + v);
    r[4 * v] = x.x;
    r[4 * v + 1] = x.y;
    r[4 * v + 2] = x.z;
    r[4 * v + 3] = x.w;
  }
  if (skew != 0u) {
    const u32x4 x = __builtin_nontemporal_load(p + NV);
    r[4 * NV] = x.x;
    r[4 * NV + 1] = x.y;
    r[4 * NV + 2] = x.z;
    r[4 * NV + 3] = x.w;
  }
}

template <int NV>
__device__ __forceinline__ void shift_raw(const uint32_t (&r)[4 * NV + 4], uint32_t skew, uint32_t* w) {
  if (skew == 0u) {
#pragma unroll
    for (int i = 0; i < 4 * NV; ++i) w[i] = r[i];
    return;
  }
  const uint32_t sb = skew & 3u;
  switch (skew >> 2) {
    case 0: shift_words<0, NV>(r, sb, w); break;
    case 1: shift_words<1, NV>(r, sb, w); break;
    case 2: shift_words<2, NV>(r, sb, w); break;
    default: shift_words<3, NV>(r, sb, w); break;
  }
}

template <int NV>
__device__ __forceinline__ void load_stream(const uint8_t* base, uint32_t skew, uint64_t off, uint32_t* w) {
  uint32_t r[4 * NV + 4];
  load_raw<NV>(base, skew, off, r);
  shift_raw<NV>(r, skew, w);
}

__device__ __forceinline__ void store4(uint8_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                       bool plain = false) {
  u32x4 v;
  v.x = a;
  v.y = b;
  v.z = c;
  v.w = d;
  if (plain) *reinterpret_cast<u32x4*>(p) = v;
  else __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

// ---- base64 / hex, 4 characters per word (SWAR) ---------------------------------
// 24-bit group -> its 4 sextets, first character in byte 0.
__device__ __forceinline__ uint32_t spread24(uint32_t x) {
  return (x >> 18) | ((x >> 4) & 0x3F00u) | ((x << 10) & 0x3F0000u) | ((x << 24) & 0x3F000000u);
}

// per byte: 1 if the sextet (< 64) is >= k
__device__ __forceinline__ uint32_t ge_bytes(uint32_t d, uint32_t k) {
  return ((d + (128u - k) * 0x01010101u) >> 7) & 0x01010101u;
}

// sextets -> RFC 4648 characters: + the offset of the sextet's class
// (A-Z +65, a-z +71, 0-9 -4, '+' -19, '/' -16), looked up by v_perm
// (split in a positive and a negative part so that no byte carries).
__device__ __forceinline__ uint32_t b64_chars(uint32_t d) {
  const uint32_t cls = ge_bytes(d, 26) + ge_bytes(d, 52) + ge_bytes(d, 62) + ge_bytes(d, 63);
  return d + __builtin_amdgcn_perm(0u, 0x00004741u, cls) - __builtin_amdgcn_perm(0x10u, 0x13040000u, cls);
}

// 48 bytes (12 big-endian words) -> 64 base64 characters (16 words)
__device__ __forceinline__ void b64_unit(const uint32_t W[12], uint32_t C[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t w0 = W[3 * q], w1 = W[3 * q + 1], w2 = W[3 * q + 2];
    C[4 * q + 0] = b64_chars(spread24(w0 >> 8));
    C[4 * q + 1] = b64_chars(spread24(__builtin_amdgcn_alignbit(w0, w1, 16) & 0xFFFFFFu));
    C[4 * q + 2] = b64_chars(spread24(__builtin_amdgcn_alignbit(w1, w2, 24) & 0xFFFFFFu));
    C[4 * q + 3] = b64_chars(spread24(w2 & 0xFFFFFFu));
  }
}

// nibble per byte -> lowercase hex digit
__device__ __forceinline__ uint32_t hex_digits(uint32_t x) {
  const uint32_t m = (x + 0x76767676u) & 0x80808080u;  // bytes >= 10
  return x + 0x30303030u + ((m - (m >> 7)) & 0x27272727u);
}

__device__ __forceinline__ uint32_t hex_digit(uint32_t v) { return v < 10u ? 0x30u + v : 0x57u + v; }

// ---- base64 + hex by LDS lookup (DN_AES_HEX_LDS) ---------------------------------
// The hex digits of the base64 character of a sextet, as two tables in one
// 256-B row per sextet (the AES tables' layout): words 0..31 hold the digit
// pair in bytes 0-1, words 32..63 in bytes 2-3, each 32 times (lane l reads
// replica l % 32: conflict-free).  The LDS byte address of sextet s, table t,
// is s << 8 | (lane % 32) << 2 | t << 7: a sextet already at bits 8..13 of a
// register is ONE full-rate v_bitop3 from its address.  Per 48-byte unit this
// replaces ~45 VALU per 24-bit group (spread, class offsets, hex nibbles) by
// about a dozen plus four lookups: the kernel is VALU-issue-bound with the LDS
// ~half busy (profiles/r04/pmc/summary.json), so moving work to the LDS pays.
struct HexLds {
  uint32_t row[64][64];
};

__device__ __forceinline__ uint32_t b64_char(uint32_t s) {
  return s < 26u ? 0x41u + s : s < 52u ? 0x61u + s - 26u : s < 62u ? 0x30u + s - 52u : s == 62u ? 0x2Bu : 0x2Fu;
}

__device__ void build_hex(HexLds& H, uint32_t TH) {
  uint32_t* flat = &H.row[0][0];
  for (uint32_t w = threadIdx.x; w < 64u * 64u; w += TH) {
    const uint32_t c = b64_char(w >> 6), pair = hex_digit(c >> 4) | (hex_digit(c & 15u) << 8);
    flat[w] = (w & 32u) ? pair << 16 : pair;
  }
}

// the table word of a sextet held at bits 8..13 of v (higher and lower bits
// ignored): LDS address (v & 0x3F00) | lbx by one v_bitop3, where lbx = the
// lane bits | the table's own LDS address (DN_AES_HEX_BASE: the table is
// 16 KB-aligned, so its address has no bit in 8..13 and ORs in — no add per
// lookup; table t at the read's immediate offset)
#ifndef DN_AES_HEX_BASE
#define DN_AES_HEX_BASE 1
#endif
typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;

template <int T>
__device__ __forceinline__ uint32_t hex_lookup(const HexLds& H, uint32_t v, uint32_t lb) {
  const uint32_t a = __builtin_amdgcn_bitop3_b32(v, 0x3F00u, lb, 0xea);  // (v & m) | lb
#if DN_AES_HEX_BASE
  (void)H;
  return *(reinterpret_cast<lds_u32_t*>(static_cast<uintptr_t>(a)) + 32 * T);
#else
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(&H.row[0][0]) + a + 128 * T);
#endif
}

// lb | the LDS address of H (DN_AES_HEX_BASE), else lb
__device__ __forceinline__ uint32_t hex_lane_bits(const HexLds& H, uint32_t lb) {
#if DN_AES_HEX_BASE
  return lb | static_cast<uint32_t>(reinterpret_cast<uintptr_t>(&H.row[0][0]));
#else
  (void)H;
  return lb;
#endif
}

// The wave's 64 x 8 16-byte chunks (lane s holds the 128 text bytes of unit
// g0 + s, chunk c = h[4c .. 4c + 3]) transposed so that chunk register v of
// lane l is chunk l >> 3 of lane 8 v + (l & 7): store v then writes the
// contiguous KB [1024 v, 1024 v + 1024) of the wave's text.  Three butterfly
// stages each swap one lane bit with one chunk-index bit: lane bit 5 <-> bit 2
// (v_permlane32_swap), 4 <-> 1 (v_permlane16_swap), 3 <-> 0 (a DPP row
// rotation by 8 and selects).  All 64 lanes must be active.
__device__ __forceinline__ void hex_coalesce(uint32_t h[32], uint32_t lane) {
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const auto r = __builtin_amdgcn_permlane32_swap(h[4 * c + w], h[4 * (c + 4) + w], false, false);
      h[4 * c + w] = r[0];
      h[4 * (c + 4) + w] = r[1];
    }
#pragma unroll
  for (int c : {0, 1, 4, 5})
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const auto r = __builtin_amdgcn_permlane16_swap(h[4 * c + w], h[4 * (c + 2) + w], false, false);
      h[4 * c + w] = r[0];
      h[4 * (c + 2) + w] = r[1];
    }
  const bool b3 = (lane & 8u) != 0u;
#pragma unroll
  for (int c : {0, 2, 4, 6})
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t A = h[4 * c + w], B = h[4 * (c + 1) + w];
      const uint32_t x = b3 ? A : B;
      const uint32_t y = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x128, 0xF, 0xF, false));
      h[4 * c + w] = b3 ? y : A;
      h[4 * (c + 1) + w] = b3 ? B : y;
    }
}

// Two stages only (DN_AES_HEX_COAL == 2): lane bit 5 <-> chunk bit 1
// (v_permlane32_swap), 4 <-> 0 (v_permlane16_swap), no selects: chunk register
// v of lane l is chunk 4 (v >> 2) + (l >> 4) of lane (l & 15) + 16 (v & 3),
// so store v writes the 64-B halves (v >> 2) of 16 consecutive lines.
__device__ __forceinline__ void hex_coalesce_half(uint32_t h[32]) {
#pragma unroll
  for (int c : {0, 1, 4, 5})
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const auto r = __builtin_amdgcn_permlane32_swap(h[4 * c + w], h[4 * (c + 2) + w], false, false);
      h[4 * c + w] = r[0];
      h[4 * (c + 2) + w] = r[1];
    }
#pragma unroll
  for (int c : {0, 2, 4, 6})
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const auto r = __builtin_amdgcn_permlane16_swap(h[4 * c + w], h[4 * (c + 1) + w], false, false);
      h[4 * c + w] = r[0];
      h[4 * (c + 1) + w] = r[1];
    }
}

// The same for 4 chunks per lane (64 base64 characters): chunk register v of
// lane l is chunk l >> 4 of lane 16 v + (l & 15) — lane bit 4 <-> chunk bit
// 0 (v_permlane16_swap), 5 <-> 1 (v_permlane32_swap); also its own inverse.
__device__ __forceinline__ void b64_coalesce(uint32_t h[16]) {
#pragma unroll
  for (int c : {0, 2})
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const auto r = __builtin_amdgcn_permlane16_swap(h[4 * c + w], h[4 * (c + 1) + w], false, false);
      h[4 * c + w] = r[0];
      h[4 * (c + 1) + w] = r[1];
    }
#pragma unroll
  for (int c : {0, 1})
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const auto r = __builtin_amdgcn_permlane32_swap(h[4 * c + w], h[4 * (c + 2) + w], false, false);
      h[4 * c + w] = r[0];
      h[4 * (c + 2) + w] = r[1];
    }
}

// 12 big-endian words (48 bytes) -> 32 hex words (64 base64 characters): sextet
// j of a word triple (w0, w1, w2) is moved to bits 8..13 by one shift or
// funnel shift (sextet 3 sits there already), looked up, and two lookups are
// ORed into each output word (hex of characters 2i, 2i + 1)
__device__ __forceinline__ void hex_lds_unit(const HexLds& H, const uint32_t W[12], uint32_t lb, uint32_t h[32]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t w0 = W[3 * q], w1 = W[3 * q + 1], w2 = W[3 * q + 2];
    const uint32_t v[16] = {w0 >> 18, w0 >> 12, w0 >> 6, w0, w0 << 6, __builtin_amdgcn_alignbit(w0, w1, 20),
                            w1 >> 14, w1 >> 8, w1 >> 2, w1 << 4, __builtin_amdgcn_alignbit(w1, w2, 22),
                            w2 >> 16, w2 >> 10, w2 >> 4, w2 << 2, w2 << 8};
    uint32_t x[16];
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      x[j] = hex_lookup<0>(H, v[j], lb);
      x[j + 1] = hex_lookup<1>(H, v[j + 1], lb);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) h[8 * q + i] = x[2 * i] | x[2 * i + 1];
  }
}

// 4 characters -> 8 hex digits (2 words, each character's high digit first)
__device__ __forceinline__ void hex_word(uint32_t c, uint32_t& h0, uint32_t& h1) {
  const uint32_t hi = (c >> 4) & 0x0F0F0F0Fu, lo = c & 0x0F0F0F0Fu;
  h0 = hex_digits(__builtin_amdgcn_perm(hi, lo, 0x01050004u));
  h1 = hex_digits(__builtin_amdgcn_perm(hi, lo, 0x03070206u));
}

// hex_word for base64 characters only (A-Z a-z 0-9 + /, all in 0x2B..0x7A):
// every high nibble is 2..7, a decimal digit, so only the low nibbles take
// the letter test
__device__ __forceinline__ void hex_word_b64(uint32_t c, uint32_t& h0, uint32_t& h1) {
  // (c >> 4) & 0x0F0F0F0F | 0x30303030 in one v_bitop3 ((S0 & S1) | S2: table 0xea)
  const uint32_t hi = __builtin_amdgcn_bitop3_b32(c >> 4, 0x0F0F0F0Fu, 0x30303030u, 0xea);
  const uint32_t lo = hex_digits(c & 0x0F0F0F0Fu);
  h0 = __builtin_amdgcn_perm(hi, lo, 0x01050004u);
  h1 = __builtin_amdgcn_perm(hi, lo, 0x03070206u);
}

// 4 hex digits (one per byte) -> 4 nibble values; bad |= non-hex bytes
__device__ __forceinline__ uint32_t unhex4(uint32_t c, uint32_t& bad) {
  const uint32_t c7 = c & 0x7F7F7F7Fu, l7 = c7 | 0x20202020u;
  const uint32_t dig = (c7 + 0x50505050u) & ~(c7 + 0x46464646u);  // '0' <= c <= '9'
  const uint32_t alp = (l7 + 0x1F1F1F1Fu) & ~(l7 + 0x19191919u);  // 'a' <= c | 0x20 <= 'f'
  bad |= (~(dig | alp) | c) & 0x80808080u;
  const uint32_t letter = (c >> 6) & 0x01010101u;
  return (c & 0x0F0F0F0Fu) + (letter << 3) + letter;
}

// 8 nibbles (two words) -> 4 bytes
__device__ __forceinline__ uint32_t pack_nibbles(uint32_t v0, uint32_t v1) {
  const uint32_t hi = __builtin_amdgcn_perm(v1, v0, 0x06040200u), lo = __builtin_amdgcn_perm(v1, v0, 0x07050301u);
  return (hi << 4) | lo;
}

// 4 base64 characters -> 24-bit group; acc collects the table flags
__device__ __forceinline__ uint32_t unb64_word(const uint8_t* dec, uint32_t d, uint32_t& acc) {
  const uint32_t s0 = dec[d & 0xFFu], s1 = dec[(d >> 8) & 0xFFu], s2 = dec[(d >> 16) & 0xFFu], s3 = dec[d >> 24];
  acc |= s0 | s1 | s2 | s3;
  return (s0 << 18) | (s1 << 12) | (s2 << 6) | s3;
}

// 16 groups -> 12 big-endian words
__device__ __forceinline__ void join24(const uint32_t x[16], uint32_t W[12]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    W[3 * q] = (x[4 * q] << 8) | (x[4 * q + 1] >> 16);
    W[3 * q + 1] = (x[4 * q + 1] << 16) | (x[4 * q + 2] >> 8);
    W[3 * q + 2] = (x[4 * q + 2] << 24) | x[4 * q + 3];
  }
}

__device__ __forceinline__ uint32_t hex_val(uint32_t c, uint32_t& bad) {
  const uint32_t l = c | 0x20u;
  if (c - 0x30u < 10u) return c - 0x30u;
  if (l - 0x61u < 6u) return l - 0x57u;
  bad = 1u;
  return 0u;
}

// ---- kernels ----------------------------------------------------------------------
#define DN_AES_PROLOGUE                                                 \
  __shared__ AesLds<NTAB> L;                                            \
  build_tables<NTAB>(L);                                                \
  const uint32_t lb = (threadIdx.x & 31u) << 2;                         \
  const uint32_t lw[2] = {lb, lb | 0x10000u};                           \
  constexpr uint32_t TH = NTAB == 4 ? 1024u : 512u;                     \
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * TH;        \
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * TH + threadIdx.x

// out = in ^ keystream, one 16-byte block per thread and step.
template <int NR, int NTAB>
__global__ void __launch_bounds__(NTAB == 4 ? 1024 : 512) ctr_kernel(const AesArgs a) {
  DN_AES_PROLOGUE;
  const uint8_t* in = a.in + a.skew;
  uint32_t R[8];  // raw loads of the next whole block, issued before this block's store
  if (first < a.units && 16 * (first + 1) <= a.n) load_raw<1>(a.in, a.skew, 16 * first, R);
  for (uint64_t b = first; b < a.units; b += stride) {
    uint32_t ks[4];
    ctr_block(a.iv, b, ks);
    aes_block<NR>(L, lw, a, ks);
    if (16 * (b + 1) <= a.n) {
      uint32_t p[4];
      shift_raw<1>(R, a.skew, p);
      const uint64_t bn = b + stride;
      if (bn < a.units && 16 * (bn + 1) <= a.n) load_raw<1>(a.in, a.skew, 16 * bn, R);
      store4(a.out + 16 * b, p[0] ^ __builtin_bswap32(ks[0]), p[1] ^ __builtin_bswap32(ks[1]),
             p[2] ^ __builtin_bswap32(ks[2]), p[3] ^ __builtin_bswap32(ks[3]));
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint64_t o = 16 * b + k;
        if (o < a.n) a.out[o] = static_cast<uint8_t>(in[o] ^ (ks[k >> 2] >> (24 - 8 * (k & 3))));
      }
    }
  }
}

// Unit g byte-wise (g == 0: the nonce block; the last unit: ragged end, '=').
template <int NR, int NTAB, bool HEX>
__device__ void encrypt_unit_slow(const AesLds<NTAB>& L, const uint32_t lw[2], const AesArgs& a, uint64_t g) {
  const uint64_t m = a.n + 16;
  const uint8_t* in = a.in + a.skew;
  uint32_t W[12];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int64_t kb = 3 * static_cast<int64_t>(g) - 1 + j;
    if (kb < 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) W[4 * j + i] = a.iv[i];
      continue;
    }
    const uint64_t b0 = 16ull * static_cast<uint64_t>(kb);
    uint32_t ks[4] = {0u, 0u, 0u, 0u};
    if (b0 < a.n) {
      ctr_block(a.iv, static_cast<uint64_t>(kb), ks);
      aes_block<NR>(L, lw, a, ks);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t v = 0u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t o = b0 + 4 * i + k;
        const uint32_t byte = o < a.n ? ((in[o] ^ (ks[i] >> (24 - 8 * k))) & 0xFFu) : 0u;
        v |= byte << (24 - 8 * k);
      }
      W[4 * j + i] = v;
    }
  }
  uint32_t C[16];
  b64_unit(W, C);
  const uint64_t len = 4 * ((m + 2) / 3), pad = (3 - m % 3) % 3;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t pos = 64 * g + 4 * w + k;
      if (pos < len) {
        const uint32_t ch = pos >= len - pad ? kPadChar : (C[w] >> (8 * k)) & 0xFFu;
        if constexpr (HEX) {
          a.out[2 * pos] = static_cast<uint8_t>(hex_digit(ch >> 4));
          a.out[2 * pos + 1] = static_cast<uint8_t>(hex_digit(ch & 15u));
        } else {
          a.out[pos] = static_cast<uint8_t>(ch);
        }
      }
    }
  }
}

// The plaintext of unit g (blocks 3g - 1 .. 3g + 1) into R.  (Loading the
// wave's 3 KB lane-contiguous instead was slower: 1.40-1.42 vs 1.37 ms,
// profiles/r05/l/; the per-lane 48-B loads are issued a unit ahead.)
__device__ __forceinline__ void load_unit(const AesArgs& a, uint64_t g, uint32_t (&R)[16]) {
  load_raw<3>(a.in, a.skew, 48 * g - 16, R);
}

template <int NR, int NTAB, bool HEX>
__global__ void __launch_bounds__(NTAB == 4 ? 1024 : 512) encrypt_kernel(const AesArgs a) {
  DN_AES_PROLOGUE;
#if DN_AES_HEX_LDS
  constexpr bool kHexLds = HEX && NTAB == 4;
  __shared__ __attribute__((aligned(16384))) HexLds HX;  // 16 KB-aligned: hex_lookup
  if constexpr (kHexLds) {
    build_hex(HX, TH);
    __syncthreads();
  }
#else
  constexpr bool kHexLds = false;
#endif
  const uint64_t m = a.n + 16;
  // plaintext of blocks 3g-1 .. 3g+1 of the next whole unit, loaded before this unit's stores
  uint32_t R[16];
  if (first < a.units && first != 0 && 48 * (first + 1) <= m) load_unit(a, first, R);
  for (uint64_t g = first; g < a.units; g += stride) {
    const uint64_t gn = g + stride;
    const bool next_whole = gn < a.units && 48 * (gn + 1) <= m;
    if (g == 0 || 48 * (g + 1) > m) {
      encrypt_unit_slow<NR, NTAB, HEX>(L, lw, a, g);
      if (next_whole) load_unit(a, gn, R);
      continue;
    }
    uint32_t W[12];
    shift_raw<3>(R, a.skew, W);
    if (next_whole) load_unit(a, gn, R);
    if constexpr (NTAB == 4 && DN_AES_NB > 1) {
      uint32_t ks[3][4];
#pragma unroll
      for (int j = 0; j < 3; ++j) ctr_block(a.iv, 3 * g - 1 + j, ks[j]);
      if constexpr (DN_AES_NB == 3) {
        aes_blocks<NR, 3>(L, lw, a, ks);
      } else {
        aes_blocks<NR, 2>(L, lw, a, ks);
        aes_block<NR>(L, lw, a, ks[2]);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) W[4 * j + i] = __builtin_bswap32(W[4 * j + i]) ^ ks[j][i];
    } else {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        uint32_t ks[4];
        ctr_block(a.iv, 3 * g - 1 + j, ks);
        aes_block<NR>(L, lw, a, ks);
#pragma unroll
        for (int i = 0; i < 4; ++i) W[4 * j + i] = __builtin_bswap32(W[4 * j + i]) ^ ks[i];
      }
    }
#if DN_AES_HEX_LDS
    if constexpr (kHexLds) {
      uint32_t h[32];
      hex_lds_unit(HX, W, hex_lane_bits(HX, lb), h);
#if DN_AES_HEX_COAL
      if (__ballot(1) == ~0ull) {  // all 64 lanes here, each with a whole unit (units g0 .. g0 + 63)
        const uint32_t lane = threadIdx.x & 63u;
#if DN_AES_HEX_COAL == 2
        hex_coalesce_half(h);
        uint8_t* o = a.out + 128 * (g - lane) + 128 * (lane & 15u) + 16 * (lane >> 4);
#pragma unroll
        for (int v = 0; v < 8; ++v)
          store4(o + 2048 * (v & 1) + 4096 * ((v >> 1) & 1) + 64 * (v >> 2), h[4 * v], h[4 * v + 1], h[4 * v + 2],
                 h[4 * v + 3], a.plain != 0u);
#else
        hex_coalesce(h, lane);
        uint8_t* o = a.out + 128 * (g - lane) + 128 * (lane & 7u) + 16 * (lane >> 3);
#pragma unroll
        for (int v = 0; v < 8; ++v)
          store4(o + 1024 * v, h[4 * v], h[4 * v + 1], h[4 * v + 2], h[4 * v + 3], a.plain != 0u);
#endif
        continue;
      }
#endif
      uint8_t* o = a.out + 128 * g;
#pragma unroll
      for (int v = 0; v < 8; ++v) store4(o + 16 * v, h[4 * v], h[4 * v + 1], h[4 * v + 2], h[4 * v + 3], a.plain != 0u);
      continue;
    }
#endif
    uint32_t C[16];
    b64_unit(W, C);
    if constexpr (HEX) {
      uint8_t* o = a.out + 128 * g;
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        uint32_t h0, h1, h2, h3;
        hex_word_b64(C[2 * v], h0, h1);
        hex_word_b64(C[2 * v + 1], h2, h3);
#ifdef DN_AES_DIAG_COALESCED  // timing diagnostic only: lane-contiguous stores, output permuted
        const uint64_t g0 = g - (threadIdx.x & 63u);  // the wave's first unit
        if (g0 + 64u < a.units)
          store4(a.out + 128 * g0 + 1024 * v + 16 * (threadIdx.x & 63u), h0, h1, h2, h3, a.plain != 0u);
        else
          store4(o + 16 * v, h0, h1, h2, h3, a.plain != 0u);
#else
        store4(o + 16 * v, h0, h1, h2, h3, a.plain != 0u);
#endif
      }
    } else {
#if DN_AES_HEX_COAL
      if (__ballot(1) == ~0ull) {  // all 64 lanes, whole units: one contiguous KB per store
        const uint32_t lane = threadIdx.x & 63u;
        b64_coalesce(C);
        uint8_t* o = a.out + 64 * (g - lane) + 64 * (lane & 15u) + 16 * (lane >> 4);
#pragma unroll
        for (int v = 0; v < 4; ++v)
          store4(o + 1024 * v, C[4 * v], C[4 * v + 1], C[4 * v + 2], C[4 * v + 3], a.plain != 0u);
        continue;
      }
#endif
      uint8_t* o = a.out + 64 * g;
#pragma unroll
      for (int v = 0; v < 4; ++v)
        store4(o + 16 * v, C[4 * v], C[4 * v + 1], C[4 * v + 2], C[4 * v + 3], a.plain != 0u);
    }
  }
}

template <bool HEX>
__device__ __forceinline__ uint32_t text_char(const AesArgs& a, uint64_t pos, uint32_t& bad) {
  const uint8_t* t = a.in + a.skew;
  if constexpr (HEX) return (hex_val(t[2 * pos], bad) << 4) | hex_val(t[2 * pos + 1], bad);
  else return t[pos];
}

// Unit g byte-wise: validates every character ('=' only in the final pad positions).
template <int NR, int NTAB, bool HEX>
__device__ void decrypt_unit_slow(const AesLds<NTAB>& L, const uint32_t lw[2], const AesArgs& a,
                                  const uint32_t iv[4], uint64_t g, uint64_t pad, uint64_t nout) {
  uint32_t bad = 0u, x[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    uint32_t v = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t pos = 64 * g + 4 * q + k;
      uint32_t s = 0u;
      if (pos < a.n) {
        s = L.dec[text_char<HEX>(a, pos, bad)];
        if (pos >= a.n - pad) {
          bad |= s != kDecPad ? 1u : 0u;
          s = 0u;
        } else if (s & (kDecPad | kDecBad)) {
          bad = 1u;
          s = 0u;
        }
      }
      v = (v << 6) | s;
    }
    x[q] = v;
  }
  if (bad) atomicOr(a.bad, 1u);
  uint32_t W[12];
  join24(x, W);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int64_t kb = 3 * static_cast<int64_t>(g) - 1 + j;
    if (kb < 0) continue;
    const uint64_t b0 = 16ull * static_cast<uint64_t>(kb);
    if (b0 >= nout) continue;
    uint32_t ks[4];
    ctr_block(iv, static_cast<uint64_t>(kb), ks);
    aes_block<NR>(L, lw, a, ks);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t o = b0 + 4 * i + k;
        if (o < nout) a.out[o] = static_cast<uint8_t>((W[4 * j + i] ^ ks[i]) >> (24 - 8 * k));
      }
    }
  }
}

// The nonce (first 24 characters) and the padding (last two) of the text,
// through a base64 decode table `dec` (LDS): every thread of a kernel reads
// them (cached lines), the units that hold them validate them again.
template <bool HEX>
__device__ __forceinline__ void text_header(const AesArgs& a, const uint8_t* dec, uint32_t iv[4], uint64_t& pad) {
  uint32_t ignore = 0u, x[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    uint32_t v = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) v = (v << 6) | (dec[text_char<HEX>(a, 4 * q + k, ignore)] & 63u);
    x[q] = v;
  }
  iv[0] = (x[0] << 8) | (x[1] >> 16);
  iv[1] = (x[1] << 16) | (x[2] >> 8);
  iv[2] = (x[2] << 24) | x[3];
  iv[3] = (x[4] << 8) | (x[5] >> 16);
  const uint32_t c1 = text_char<HEX>(a, a.n - 2, ignore), c2 = text_char<HEX>(a, a.n - 1, ignore);
  pad = c2 == kPadChar ? (c1 == kPadChar ? 2u : 1u) : 0u;
}

__device__ void build_dec(uint8_t* dec, uint32_t TH) {
  for (uint32_t e = threadIdx.x; e < 256u; e += TH) {
    uint32_t d = kDecBad;
    if (e >= 'A' && e <= 'Z') d = e - 'A';
    else if (e >= 'a' && e <= 'z') d = e - 'a' + 26u;
    else if (e >= '0' && e <= '9') d = e - '0' + 52u;
    else if (e == '+') d = 62u;
    else if (e == '/') d = 63u;
    else if (e == '=') d = kDecPad;
    dec[e] = static_cast<uint8_t>(d);
  }
  __syncthreads();
}

// ---- decrypt in two passes (DN_AES_DEC_SPLIT) --------------------------------------
// decode_kernel: text -> ciphertext bytes (hex and base64 validated as the
// one-pass kernel does), a streaming pass with a 256-B table, high occupancy
// and the next unit's text loaded before this unit's stores; then
// ctr_text_kernel XORs the keystream in place (the nonce and the length read
// from the text by every workgroup).  The one-pass decrypt_kernel held 122
// VGPRs for the AES and loaded each unit's 128 text bytes just before using
// them (2.62 ms for 1.13 GB, profiles/r05/m/).
template <bool HEX>
__device__ void decode_unit_slow(const uint8_t* dec, const AesArgs& a, uint64_t g, uint64_t pad, uint64_t nout) {
  uint32_t bad = 0u, x[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    uint32_t v = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t pos = 64 * g + 4 * q + k;
      uint32_t s = 0u;
      if (pos < a.n) {
        s = dec[text_char<HEX>(a, pos, bad)];
        if (pos >= a.n - pad) {
          bad |= s != kDecPad ? 1u : 0u;
          s = 0u;
        } else if (s & (kDecPad | kDecBad)) {
          bad = 1u;
          s = 0u;
        }
      }
      v = (v << 6) | s;
    }
    x[q] = v;
  }
  if (bad) atomicOr(a.bad, 1u);
  uint32_t W[12];
  join24(x, W);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int64_t kb = 3 * static_cast<int64_t>(g) - 1 + j;
    if (kb < 0) continue;
    const uint64_t b0 = 16ull * static_cast<uint64_t>(kb);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t o = b0 + 4 * i + k;
        if (o < nout) a.out[o] = static_cast<uint8_t>(W[4 * j + i] >> (24 - 8 * k));
      }
  }
}

// Unit gq's text into R (decode_kernel, decrypt_fused_kernel): a wave whose
// 64 lanes all load whole units reads its text line by line and transposes
// (hex_coalesce: load v of lane l is chunk l >> 3 of lane 8 v + (l & 7); base64:
// b64_coalesce), the chunk after a unit (skew) from the next lane (the next
// wave's first chunk for lane 63); otherwise each lane its own unit.
// Split in two (round 6): issue_unit_text issues the loads and returns the
// mode (1: coalesced, wave-uniform), finish_unit_text transposes once they have
// arrived — so a loop can keep the next unit's loads in flight across this
// unit's AES.  (With the transpose inside the load, the loads were waited for
// at once: every unit's text latency was exposed.)
// WHOLE: the caller guarantees all 64 lanes are active (no ballot, always coalesced)
template <bool HEX, bool WHOLE = false>
__device__ __forceinline__ uint32_t issue_unit_text(const AesArgs& a, uint64_t gq, uint32_t lane,
                                                    uint32_t (&R)[HEX ? 36 : 20]) {
  constexpr int NV = HEX ? 8 : 4;      // 16-B vectors of one unit's text
  const uint64_t tb = HEX ? 128 : 64;  // text bytes per unit
  if constexpr (!HEX && DN_AES_DEC_COAL) {
    if (WHOLE || __ballot(1) == ~0ull) {  // base64 text: 4 chunks per lane, as the encrypt stores
      const uint64_t w0 = tb * (gq - lane);
      const u32x4* p = reinterpret_cast<const u32x4*>(a.in + w0 + 64 * (lane & 15u) + 16 * (lane >> 4));
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const u32x4 x = __builtin_nontemporal_load(p + 64 * v);
        R[4 * v] = x.x, R[4 * v + 1] = x.y, R[4 * v + 2] = x.z, R[4 * v + 3] = x.w;
      }
      if (a.skew != 0u) {  // the next wave's first chunk (lane 63's; every lane loads the line)
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.in + w0 + 4096));
        R[16] = x.x, R[17] = x.y, R[18] = x.z, R[19] = x.w;
      }
      return 1u;
    }
  }
  if constexpr (HEX && DN_AES_DEC_COAL) {
    if (WHOLE || __ballot(1) == ~0ull) {
      const uint64_t w0 = tb * (gq - lane);
#if DN_AES_DEC_COAL == 2
      // half lines (hex_coalesce_half, the encrypt's default transpose, also its own inverse)
      const u32x4* p = reinterpret_cast<const u32x4*>(a.in + w0 + 128 * (lane & 15u) + 16 * (lane >> 4));
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const u32x4 x = __builtin_nontemporal_load(p + 128 * (v & 1) + 256 * ((v >> 1) & 1) + 4 * (v >> 2));
        R[4 * v] = x.x, R[4 * v + 1] = x.y, R[4 * v + 2] = x.z, R[4 * v + 3] = x.w;
      }
#else
      const u32x4* p = reinterpret_cast<const u32x4*>(a.in + w0 + 128 * (lane & 7u) + 16 * (lane >> 3));
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const u32x4 x = __builtin_nontemporal_load(p + 64 * v);
        R[4 * v] = x.x, R[4 * v + 1] = x.y, R[4 * v + 2] = x.z, R[4 * v + 3] = x.w;
      }
#endif
      if (a.skew != 0u) {  // lane 63's next chunk: every lane loads it (one line; no exec-masked load,
                           // whose conditional count made the loop's first wait vmcnt(0))
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.in + w0 + 8192));
        R[32] = x.x, R[33] = x.y, R[34] = x.z, R[35] = x.w;
      }
      return 1u;
    }
  }
  load_raw<NV>(a.in, a.skew, tb * gq, R);
  return 0u;
}

template <bool HEX>
__device__ __forceinline__ void finish_unit_text(const AesArgs& a, uint32_t lane, uint32_t mode,
                                                 uint32_t (&R)[HEX ? 36 : 20]) {
  if (!mode) return;  // each lane loaded its own unit (shift_raw aligns it)
  constexpr int NV = HEX ? 8 : 4;
  if constexpr (HEX) {
#if DN_AES_DEC_COAL == 2
    hex_coalesce_half(R);
#else
    hex_coalesce(R, lane);
#endif
  } else {
    b64_coalesce(R);
  }
  if (a.skew != 0u) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t nx = static_cast<uint32_t>(__shfl_down(static_cast<int>(R[i]), 1));
      R[4 * NV + i] = lane == 63u ? R[4 * NV + i] : nx;
    }
  }
}

template <bool HEX>
__device__ __forceinline__ void load_unit_text(const AesArgs& a, uint64_t gq, uint32_t lane,
                                             uint32_t (&R)[HEX ? 36 : 20]) {
  const uint32_t mode = issue_unit_text<HEX>(a, gq, lane, R);
  finish_unit_text<HEX>(a, lane, mode, R);
}

template <bool HEX>
__global__ void __launch_bounds__(256) decode_kernel(const AesArgs a) {
  __shared__ uint8_t dec[256];
  build_dec(dec, 256u);
  uint32_t iv[4];
  uint64_t pad;
  text_header<HEX>(a, dec, iv, pad);
  const uint64_t nout = a.n / 4 * 3 - pad - 16;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256u;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
  if (first == 0) *a.out_len = nout;
  constexpr int NV = HEX ? 8 : 4;  // 16-B vectors of one unit's text
  uint32_t R[4 * NV + 4];
  auto whole = [&](uint64_t g) { return g != 0 && g + 1 < a.units; };
  const uint32_t lane = threadIdx.x & 63u;
  auto load_text = [&](uint64_t gq) { load_unit_text<HEX>(a, gq, lane, R); };
  if (first < a.units && whole(first)) load_text(first);
  for (uint64_t g = first; g < a.units; g += stride) {
    const uint64_t gn = g + stride;
    if (!whole(g)) {
      decode_unit_slow<HEX>(dec, a, g, pad, nout);
      if (gn < a.units && whole(gn)) load_text(gn);
      continue;
    }
    uint32_t T[16], bad = 0u;
    {
      uint32_t tx[4 * NV];
      shift_raw<NV>(R, a.skew, tx);
      if constexpr (HEX) {
#pragma unroll
        for (int k = 0; k < 16; ++k) T[k] = pack_nibbles(unhex4(tx[2 * k], bad), unhex4(tx[2 * k + 1], bad));
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) T[k] = tx[k];
      }
    }
    if (gn < a.units && whole(gn)) load_text(gn);  // next unit's text before the stores
    uint32_t x[16], acc = 0u;
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = unb64_word(dec, T[k], acc);
    if ((acc & (kDecPad | kDecBad)) | bad) atomicOr(a.bad, 1u);
    uint32_t W[12];
    join24(x, W);
    uint8_t* o = a.out + 48 * g - 16;  // raw bytes 48 g .. 48 g + 47 = ciphertext from 48 g - 16
#pragma unroll
    for (int j = 0; j < 3; ++j)
      store4(o + 16 * j, __builtin_bswap32(W[4 * j]), __builtin_bswap32(W[4 * j + 1]), __builtin_bswap32(W[4 * j + 2]),
             __builtin_bswap32(W[4 * j + 3]));
  }
}

// out[0 .. nout) ^= keystream(nonce), in place; nonce and nout from the text
template <int NR, int NTAB, bool HEX>
__global__ void __launch_bounds__(NTAB == 4 ? 1024 : 512) ctr_text_kernel(const AesArgs a) {
  __shared__ AesLds<NTAB> L;
  build_tables<NTAB>(L);
  const uint32_t lb = (threadIdx.x & 31u) << 2;
  const uint32_t lw[2] = {lb, lb | 0x10000u};
  constexpr uint32_t TH = NTAB == 4 ? 1024u : 512u;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * TH;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * TH + threadIdx.x;
  uint32_t iv[4];
  uint64_t pad;
  text_header<HEX>(a, L.dec, iv, pad);
  const uint64_t nout = a.n / 4 * 3 - pad - 16;
  const uint64_t blocks = (nout + 15) / 16;
  uint32_t R[8];
  if (first < blocks && 16 * (first + 1) <= nout) load_raw<1>(a.out, 0u, 16 * first, R);
  for (uint64_t b = first; b < blocks; b += stride) {
    uint32_t ks[4];
    ctr_block(iv, b, ks);
    aes_block<NR>(L, lw, a, ks);
    if (16 * (b + 1) <= nout) {
      const uint32_t p0 = R[0], p1 = R[1], p2 = R[2], p3 = R[3];
      const uint64_t bn = b + stride;
      if (bn < blocks && 16 * (bn + 1) <= nout) load_raw<1>(a.out, 0u, 16 * bn, R);
      store4(a.out + 16 * b, p0 ^ __builtin_bswap32(ks[0]), p1 ^ __builtin_bswap32(ks[1]),
             p2 ^ __builtin_bswap32(ks[2]), p3 ^ __builtin_bswap32(ks[3]));
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint64_t o = 16 * b + k;
        if (o < nout) a.out[o] = static_cast<uint8_t>(a.out[o] ^ (ks[k >> 2] >> (24 - 8 * (k & 3))));
      }
    }
  }
}

// One pass (DN_AES_DEC_SPLIT == 2): decode_kernel's coalesced, transposed
// text reads and its decode, then the unit's three keystream blocks, each
// block's plaintext stored as soon as its keystream is done — no ciphertext
// round trip through HBM.  Round 6: units 0 and last (the nonce, the
// padding: byte-wise) go to the first two threads, so the loop covers only
// whole units 1 .. units - 2 (32-bit indices: the host keeps units < 2^32);
// the nonce and padding, identical in every lane, are scalars; the next
// unit's text loads are issued before this unit's AES and transposed only when
// the next iteration needs them (issue_unit_text / finish_unit_text).  Round
// 5's kernel spilled three 64-bit values whose reloads' vmcnt(0), and the
// transpose inside the load, waited for those loads at once, exposing every
// unit's text latency; this one carries no spill (118 VGPRs).
template <int NR, bool HEX>
__global__ void __launch_bounds__(1024) decrypt_fused_kernel(const AesArgs a) {
  __shared__ AesLds<4> L;
  build_tables<4>(L);
  const uint32_t lb = (threadIdx.x & 31u) << 2;
  const uint32_t lw[2] = {lb, lb | 0x10000u};
  uint32_t iv[4];
  uint64_t pad;
  text_header<HEX>(a, L.dec, iv, pad);
#pragma unroll
  for (int k = 0; k < 4; ++k) iv[k] = __builtin_amdgcn_readfirstlane(iv[k]);
  pad = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(pad));
  const uint64_t nout = a.n / 4 * 3 - pad - 16;
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.out_len = nout;
  constexpr int NV = HEX ? 8 : 4;
  uint32_t R[4 * NV + 4];
  const uint32_t lane = threadIdx.x & 63u;
  if (blockIdx.x == 0 && threadIdx.x < 2u) {
    const uint64_t gs = threadIdx.x ? a.units - 1 : 0;
    if (threadIdx.x == 0u || a.units > 1) decrypt_unit_slow<NR, 4, HEX>(L, lw, a, iv, gs, pad, nout);
  }
  const uint32_t last = static_cast<uint32_t>(a.units) - 1u;  // whole units: 1 .. last - 1
  const uint32_t stride = gridDim.x * 1024u;
  const uint32_t first = 1u + blockIdx.x * 1024u + threadIdx.x;
  uint32_t mode = 0u;  // how R's loads were issued (finish_unit_text)
  if (a.units >= 3 && first < last) mode = issue_unit_text<HEX>(a, first, lane, R);
  for (uint32_t g = first; a.units >= 3 && g < last; g += stride) {
    const uint32_t gn = g + stride;
    uint32_t T[16], bad = 0u;
    {
      finish_unit_text<HEX>(a, lane, mode, R);  // this unit's text, loaded one unit ago
      uint32_t tx[4 * NV];
      shift_raw<NV>(R, a.skew, tx);
      if constexpr (HEX) {
#pragma unroll
        for (int k = 0; k < 16; ++k) T[k] = pack_nibbles(unhex4(tx[2 * k], bad), unhex4(tx[2 * k + 1], bad));
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) T[k] = tx[k];
      }
    }
    if (gn < last) mode = issue_unit_text<HEX>(a, gn, lane, R);  // in flight across the AES
    uint32_t x[16], acc = 0u;
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = unb64_word(L.dec, T[k], acc);
    if ((acc & (kDecPad | kDecBad)) | bad) atomicOr(a.bad, 1u);
    uint32_t W[12];
    join24(x, W);
    uint8_t* o = a.out + 48 * static_cast<uint64_t>(g) - 16;  // plaintext of keystream blocks 3g-1 .. 3g+1
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // each block stored as soon as its keystream is done
      uint32_t ks[4];
      ctr_block(iv, 3 * static_cast<uint64_t>(g) - 1 + j, ks);
      aes_block<NR>(L, lw, a, ks);
      store4(o + 16 * j, __builtin_bswap32(W[4 * j] ^ ks[0]), __builtin_bswap32(W[4 * j + 1] ^ ks[1]),
             __builtin_bswap32(W[4 * j + 2] ^ ks[2]), __builtin_bswap32(W[4 * j + 3] ^ ks[3]));
    }
  }
}

template <int NR, int NTAB, bool HEX>
__global__ void __launch_bounds__(NTAB == 4 ? 1024 : 512) decrypt_kernel(const AesArgs a) {
  DN_AES_PROLOGUE;
  // the nonce (first 24 characters) and the padding (last two); unit 0 and the
  // last unit validate those characters again
  uint32_t iv[4];
  uint64_t pad;
  {
    uint32_t ignore = 0u, x[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      uint32_t v = 0u;
#pragma unroll
      for (int k = 0; k < 4; ++k) v = (v << 6) | (L.dec[text_char<HEX>(a, 4 * q + k, ignore)] & 63u);
      x[q] = v;
    }
    iv[0] = (x[0] << 8) | (x[1] >> 16);
    iv[1] = (x[1] << 16) | (x[2] >> 8);
    iv[2] = (x[2] << 24) | x[3];
    iv[3] = (x[4] << 8) | (x[5] >> 16);
    const uint32_t c1 = text_char<HEX>(a, a.n - 2, ignore), c2 = text_char<HEX>(a, a.n - 1, ignore);
    pad = c2 == kPadChar ? (c1 == kPadChar ? 2u : 1u) : 0u;
  }
  const uint64_t nout = a.n / 4 * 3 - pad - 16;
  if (first == 0) *a.out_len = nout;
  for (uint64_t g = first; g < a.units; g += stride) {
    if (g == 0 || g + 1 == a.units) {
      decrypt_unit_slow<NR, NTAB, HEX>(L, lw, a, iv, g, pad, nout);
      continue;
    }
    uint32_t T[16], bad = 0u;
    if constexpr (HEX) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // two 64-digit halves keep the kernel within 128 VGPRs
        uint32_t hx[16];
        load_stream<4>(a.in, a.skew, 128 * g + 64 * h, hx);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          T[8 * h + k] = pack_nibbles(unhex4(hx[2 * k], bad), unhex4(hx[2 * k + 1], bad));
      }
    } else {
      load_stream<4>(a.in, a.skew, 64 * g, T);
    }
    uint32_t x[16], acc = 0u;
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = unb64_word(L.dec, T[k], acc);
    if ((acc & (kDecPad | kDecBad)) | bad) atomicOr(a.bad, 1u);
    uint32_t W[12];
    join24(x, W);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const uint64_t kb = 3 * g - 1 + j;
      uint32_t ks[4];
      ctr_block(iv, kb, ks);
      aes_block<NR>(L, lw, a, ks);
      store4(a.out + 16 * kb, __builtin_bswap32(W[4 * j] ^ ks[0]), __builtin_bswap32(W[4 * j + 1] ^ ks[1]),
             __builtin_bswap32(W[4 * j + 2] ^ ks[2]), __builtin_bswap32(W[4 * j + 3] ^ ks[3]));
    }
  }
}

#undef DN_AES_PROLOGUE

// ---- host ---------------------------------------------------------------------------
static int expand_key(const uint8_t* key, int key_bytes, uint32_t rk[60], int* nr) {
  if (!key) return set_error(DN_ERR_ARG, "AES: null key");
  if (key_bytes != 16 && key_bytes != 24 && key_bytes != 32)
    return set_error(DN_ERR_ARG, "Invalid key size (%d) for AES.", key_bytes * 8);
  auto sub = [](uint32_t t) {
    return (aes_sbox(t >> 24) << 24) | (aes_sbox((t >> 16) & 0xFFu) << 16) | (aes_sbox((t >> 8) & 0xFFu) << 8) |
           aes_sbox(t & 0xFFu);
  };
  const int nk = key_bytes / 4, rounds = nk + 6, total = 4 * (rounds + 1);
  for (int i = 0; i < nk; ++i)
    rk[i] = (static_cast<uint32_t>(key[4 * i]) << 24) | (static_cast<uint32_t>(key[4 * i + 1]) << 16) |
            (static_cast<uint32_t>(key[4 * i + 2]) << 8) | key[4 * i + 3];
  uint32_t rcon = 1u;
  for (int i = nk; i < total; ++i) {
    uint32_t t = rk[i - 1];
    if (i % nk == 0) {
      t = sub((t << 8) | (t >> 24)) ^ (rcon << 24);
      rcon = gf_x2(rcon);
    } else if (nk > 6 && i % nk == 4) {
      t = sub(t);
    }
    rk[i] = rk[i - nk] ^ t;
  }
  for (int i = total; i < 60; ++i) rk[i] = 0u;
  *nr = rounds;
  return DN_OK;
}

// DN_AES_TABLES=2 selects the 64-KB two-table layout for AES-256 (A/B hook, read per call).
static int aes_tables() {
  const char* e = tune_env("DN_AES_TABLES");
  return (e && e[0] == '2') ? 2 : 4;
}

enum { kCtr = 0, kEncrypt = 1, kDecrypt = 2 };

template <int NR, int NTAB>
static void launch(int kind, bool hex, uint64_t units, hipStream_t s, const AesArgs& a) {
  constexpr int TH = NTAB == 4 ? 1024 : 512;
  const uint64_t want = (units + TH - 1) / TH;
  const uint64_t cap = static_cast<uint64_t>(device_cu_count()) * (NTAB == 4 ? 1u : 2u);  // LDS-limited residency
  const dim3 g(static_cast<uint32_t>(want < cap ? (want ? want : 1) : cap)), b(TH);
  if (kind == kCtr) {
    hipLaunchKernelGGL((ctr_kernel<NR, NTAB>), g, b, 0, s, a);
  } else if (kind == kEncrypt) {
    if (hex) hipLaunchKernelGGL((encrypt_kernel<NR, NTAB, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((encrypt_kernel<NR, NTAB, false>), g, b, 0, s, a);
  } else if (DN_AES_DEC_SPLIT == 2 && NTAB == 4) {
    if (hex) hipLaunchKernelGGL((decrypt_fused_kernel<NR, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((decrypt_fused_kernel<NR, false>), g, b, 0, s, a);
  } else if (DN_AES_DEC_SPLIT) {
    // pass 1: decode, 256-thread workgroups; pass 2: CTR in place over the
    // ciphertext's 16-B blocks (at most units * 3 of them)
    const uint64_t dw = (units + 255) / 256, dcap = static_cast<uint64_t>(device_cu_count()) * 8u;
    const dim3 dg(static_cast<uint32_t>(dw < dcap ? (dw ? dw : 1) : dcap));
    if (hex) hipLaunchKernelGGL((decode_kernel<true>), dg, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((decode_kernel<false>), dg, dim3(256), 0, s, a);
    const uint64_t cw = (3 * units + TH - 1) / TH;
    const dim3 cg(static_cast<uint32_t>(cw < cap ? (cw ? cw : 1) : cap));
    if (hex) hipLaunchKernelGGL((ctr_text_kernel<NR, NTAB, true>), cg, b, 0, s, a);
    else hipLaunchKernelGGL((ctr_text_kernel<NR, NTAB, false>), cg, b, 0, s, a);
  } else {
    if (hex) hipLaunchKernelGGL((decrypt_kernel<NR, NTAB, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((decrypt_kernel<NR, NTAB, false>), g, b, 0, s, a);
  }
}

static int dispatch(int nr, int kind, bool hex, uint64_t units, void* stream, const AesArgs& a, const char* name) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nr == 14) {
    if (aes_tables() == 2) launch<14, 2>(kind, hex, units, s, a);
    else launch<14, 4>(kind, hex, units, s, a);
  } else if (nr == 12) {
    launch<12, 4>(kind, hex, units, s, a);
  } else {
    launch<10, 4>(kind, hex, units, s, a);
  }
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "%s: launch failed: %s", name, hipGetErrorString(err));
  return DN_OK;
}

// Key schedule, input base / skew, output alignment.
static int prepare(AesArgs& a, int& nr, const uint8_t* key, int key_bytes, const void* in, void* out,
                   const char* name) {
  const int rc = expand_key(key, key_bytes, a.rk, &nr);
  if (rc != DN_OK) return rc;
  if (!out) return set_error(DN_ERR_ARG, "%s: null output", name);
  if (reinterpret_cast<uintptr_t>(out) & 15) return set_error(DN_ERR_ARG, "%s: out must be 16-byte aligned", name);
  a.skew = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(in) & 15);
  a.in = static_cast<const uint8_t*>(in) - a.skew;
  a.out = static_cast<uint8_t*>(out);
  return DN_OK;
}

static void set_iv(AesArgs& a, const uint8_t* iv) {
  for (int i = 0; i < 4; ++i)
    a.iv[i] = (static_cast<uint32_t>(iv[4 * i]) << 24) | (static_cast<uint32_t>(iv[4 * i + 1]) << 16) |
              (static_cast<uint32_t>(iv[4 * i + 2]) << 8) | iv[4 * i + 3];
}

}  // namespace dn

using namespace dn;

extern "C" int dn_aes_expand_key(const uint8_t* key, int key_bytes, uint32_t* rk, int32_t* rounds) {
  if (!rk || !rounds) return set_error(DN_ERR_ARG, "dn_aes_expand_key: null pointer");
  int nr = 0;
  const int rc = expand_key(key, key_bytes, rk, &nr);
  if (rc == DN_OK) *rounds = nr;
  return rc;
}

extern "C" int dn_aes_ctr(const uint8_t* key, int key_bytes, const uint8_t* iv, const void* in, void* out, uint64_t n,
                          void* stream) {
  AesArgs a{};
  int nr = 0;
  if (!iv) return set_error(DN_ERR_ARG, "dn_aes_ctr: null iv");
  if (n == 0) return expand_key(key, key_bytes, a.rk, &nr);
  if (!in) return set_error(DN_ERR_ARG, "dn_aes_ctr: null input");
  const int rc = prepare(a, nr, key, key_bytes, in, out, "dn_aes_ctr");
  if (rc != DN_OK) return rc;
  set_iv(a, iv);
  a.n = n;
  a.units = (n + 15) / 16;
  return dispatch(nr, kCtr, false, a.units, stream, a, "dn_aes_ctr");
}

extern "C" uint64_t dn_aes_encrypt_len(uint64_t n, int hex) {
  const uint64_t len = 4 * ((n + 16 + 2) / 3);
  return hex ? 2 * len : len;
}

extern "C" int dn_aes_encrypt(const uint8_t* key, int key_bytes, const uint8_t* nonce, const void* in, uint64_t n,
                              void* out, int hex, void* stream) {
  AesArgs a{};
  int nr = 0;
  if (!nonce) return set_error(DN_ERR_ARG, "dn_aes_encrypt: null nonce");
  if (n && !in) return set_error(DN_ERR_ARG, "dn_aes_encrypt: null input");
  const int rc = prepare(a, nr, key, key_bytes, in, out, "dn_aes_encrypt");
  if (rc != DN_OK) return rc;
  set_iv(a, nonce);
  a.n = n;
  a.units = (n + 16 + 47) / 48;
  const char* st = tune_env("DN_AES_STORE");
  a.plain = (st && st[0] == 'n') ? 0u : 1u;  // plain vs nt: within a few % either way (profiles/r01/aes/)
  return dispatch(nr, kEncrypt, hex != 0, a.units, stream, a, "dn_aes_encrypt");
}

extern "C" uint64_t dn_aes_decrypt_capacity(uint64_t n_text, int hex) {
  if (hex) {
    if (n_text & 1) return 0;
    n_text /= 2;
  }
  if (n_text < 24 || (n_text & 3)) return 0;
  return n_text / 4 * 3 - 16;
}

extern "C" int dn_aes_decrypt(const uint8_t* key, int key_bytes, const void* text, uint64_t n_text, int hex,
                              void* out, uint64_t capacity, uint64_t* out_len, uint32_t* bad, void* stream) {
  AesArgs a{};
  int nr = 0;
  const uint64_t cap = dn_aes_decrypt_capacity(n_text, hex);
  if (cap == 0) {
    const int rc = expand_key(key, key_bytes, a.rk, &nr);
    if (rc != DN_OK) return rc;
    return set_error(DN_ERR_RETRY, "dn_aes_decrypt: %llu characters are not canonical %s",
                     static_cast<unsigned long long>(n_text), hex ? "hex of base64" : "base64");
  }
  if (capacity < cap) return set_error(DN_ERR_ARG, "dn_aes_decrypt: capacity %llu < %llu",
                                       static_cast<unsigned long long>(capacity), static_cast<unsigned long long>(cap));
  if (!text || !out_len || !bad) return set_error(DN_ERR_ARG, "dn_aes_decrypt: null pointer");
  const int rc = prepare(a, nr, key, key_bytes, text, out, "dn_aes_decrypt");
  if (rc != DN_OK) return rc;
  a.n = hex ? n_text / 2 : n_text;
  a.units = (a.n + 63) / 64;
  if (a.units >= (1ull << 32))  // decrypt_fused_kernel's 32-bit unit indices (256 GB of base64)
    return set_error(DN_ERR_UNSUPPORTED, "dn_aes_decrypt: %llu characters exceed one launch",
                     static_cast<unsigned long long>(n_text));
  a.out_len = out_len;
  a.bad = bad;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemsetAsync(bad, 0, sizeof(uint32_t), s) != hipSuccess)
    return set_error(DN_ERR_HIP, "dn_aes_decrypt: hipMemsetAsync failed");
  return dispatch(nr, kDecrypt, hex != 0, a.units, stream, a, "dn_aes_decrypt");
}
