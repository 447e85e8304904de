/*
 * dn_shamir.h — C-ABI of the MI355X Shamir secret-sharing hot path
 * (split = polynomial evaluation at x = 1..n, reconstruct = Lagrange
 * interpolation at 0) over the Mersenne field GF(p), p = 2^521 - 1.
 *
 * Reference interface replaced (delta-mpc/delta-node, pure Python):
 *   PRIME                            delta_node/crypto/shamir/shamir.py:16
 *   _eval_at(coeffs, x, prime)       delta_node/crypto/shamir/shamir.py:19-25
 *   SecretShare.make_shares          delta_node/crypto/shamir/shamir.py:55-66
 *   SecretShare.resolve_shares       delta_node/crypto/shamir/shamir.py:68-90
 *   op.extend_gcd/inverse_mod/div_mod delta_node/crypto/shamir/op.py:4-29
 *   random.Random.randint (MT19937)  stdlib, drawn at shamir.py:59-61
 * The reference has no FFI of its own; its boundary is the Python module
 * `delta_node.crypto.shamir`, which this library backs (see INTEGRATION.md
 * for the ctypes binding).
 *
 * Conventions
 *   - Plain pointers and sizes only.  Device pointers are HIP device memory
 *     owned by the caller; the library allocates nothing per call.
 *   - Device entry points are asynchronous on `stream` (a hipStream_t, passed
 *     as void*; NULL = the legacy default stream) and never synchronise.
 *   - Return 0 (DN_OK) or a negative DN_ERR_* code; dn_last_error() returns a
 *     thread-local message for the last failure on the calling thread.
 *   - Re-entrant: no global mutable state besides that thread-local message.
 *
 * Field-element vector layout ("M521 tiled vector")
 *   A vector of n field elements is cut into tiles of DN_M521_TILE (256)
 *   elements; the last tile is padded.  Each tile is 16896 bytes:
 *       uint32_t lo[16][256];   limb i (bits 32i..32i+31) of element w at lo[i][w]
 *       uint16_t hi[256];       bits 512..520 of element w (bits 9..15 zero)
 *   i.e. exactly 66 bytes per element (ceil(521/8)), struct-of-arrays inside
 *   a tile so every wave access is a contiguous, coalesced run.  A vector
 *   occupies dn_m521_vec_bytes(n) bytes; a "block" of S vectors is S such
 *   vectors back to back (vector s at byte offset s * dn_m521_vec_bytes(n)).
 *   Values are canonical residues in [0, p) on output; inputs must be < 2^521.
 */
#ifndef DN_SHAMIR_H
#define DN_SHAMIR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DN_M521_LIMBS 17
#define DN_M521_TILE 256
#define DN_M521_TILE_BYTES 16896
#define DN_MAX_THRESHOLD 64
#define DN_MAX_SHARES 65535
#define DN_MAX_RESOLVE 16

enum {
  DN_OK = 0,
  DN_ERR_ARG = -1,         /* bad pointer / size / parameter                      */
  DN_ERR_THRESHOLD = -2,   /* shamir.py:56-57  "threshold should be little equal than shares" */
  DN_ERR_TOO_FEW = -3,     /* shamir.py:72-73  "need at least {t} shares"          */
  DN_ERR_DISTINCT = -4,    /* shamir.py:74-75  "shares must be distinct"           */
  DN_ERR_HIP = -5,         /* HIP runtime error (launch failure)                   */
  DN_ERR_UNSUPPORTED = -6, /* outside the limits above                             */
  DN_ERR_EMPTY = -7,       /* shamir.py:78-83  k == 1: reduce() of empty iterable  */
  DN_ERR_RETRY = -8,       /* device MT draw hit a rejected draw: redo on the host */
  DN_ERR_ZERODIV = -9,     /* op.py:17-18      inverse_mod(0, p): ZeroDivisionError */
  DN_ERR_ASSERT = -10,     /* op.py:22-23      gcd(k, p) != 1: AssertionError      */
  DN_ERR_OVERFLOW = -11    /* mimc7.py:41      int(inf): OverflowError              */
};

/* Bytes of one tiled field-element vector of n elements (66 * round_up(n, 256)). */
uint64_t dn_m521_vec_bytes(uint64_t n_elem);

/*
 * Split, int64 secrets (the vector path).  Element e behaves exactly like the
 * reference `SecretShare(t).make_shares(v_e.to_bytes(8, "big", signed=True), n)`
 * given that call's coefficients: share x (1..n) of element e is
 *     y = (u64(v_e) + c_1 x + ... + c_{t-1} x^{t-1}) mod p
 * (Horner as in `_eval_at`, shamir.py:19-25).
 *   secrets  device int64[n_elem] (two's complement view = the reference's
 *            big-endian 8-byte secret)
 *   coeffs   device block of t-1 tiled vectors: vector j-1 holds c_j, each
 *            in [1, p-1] as drawn at shamir.py:59-61 (may be NULL iff t == 1)
 *   shares   device block of n_shares tiled vectors: vector x-1 = share x
 * Replaces shamir.py:55-66 (+ _eval_at :19-25).  1 <= t <= 64, t <= n <= 65535.
 */
int dn_m521_split_u64(const int64_t* secrets, const void* coeffs, void* shares,
                      uint64_t n_elem, int threshold, int n_shares, void* stream);

/* Split with full field-element secrets (the byte API: c0 = bytes_to_int(value)
 * mod p, a tiled vector).  Same contract as dn_m521_split_u64 otherwise. */
int dn_m521_split_fe(const void* secrets_fe, const void* coeffs, void* shares,
                     uint64_t n_elem, int threshold, int n_shares, void* stream);

/* Split with coefficients generated on the device (SURVEY.md §8(b)
 * dn_m521_split_prng, §8(d) config 2'): no coefficient input, 8 + 66 n bytes
 * of HBM traffic per element.  Replaces make_shares' coefficient source —
 * self.random (CPython MT19937, shamir.py:59-61) — by a keyed stream cipher:
 * coefficient j (1..t-1) of GLOBAL element g = elem_offset + e has index
 * i = g (t-1) + j - 1; its limbs 0..15 are ChaCha block i (64-bit counter,
 * 64-bit nonce, `rounds` in {8, 12, 20}; key = 8 host words), limb 16 is the
 * low 9 bits of word i % 16 of block 2^62 + i / 16; a value >= p - 1 is
 * redrawn from blocks 2^63 + (i << 6) + 2a, +1 (attempt a) — randint's
 * reject rule — and 1 is added, so every coefficient is uniform in [1, p-1].
 * The stream depends only on (key, nonce, g): sharded calls (elem_offset a
 * multiple of 256) produce exactly the unsharded result.  u64 secrets,
 * 2 <= t <= 8 (t = 1 needs no coefficients).  Restated on the CPU in
 * oracle/chacha_oracle.c. */
int dn_m521_split_prng(const int64_t* secrets, const uint32_t* key, uint64_t nonce, int rounds, uint64_t elem_offset,
                       void* shares, uint64_t n_elem, int threshold, int n_shares, void* stream);

/* The same coefficient stream written out as a tiled block of tm1 vectors
 * (row j-1 = coefficient j), e.g. for dn_m521_split_fe; 1 <= tm1 <= 7. */
int dn_m521_prng_coeffs(const uint32_t* key, uint64_t nonce, int rounds, uint64_t elem_offset, void* coeffs,
                        uint64_t n_elem, int tm1, void* stream);

/*
 * Lagrange-at-0 weights for share abscissas xs[0..k-1], in the form the
 * reconstruct kernel consumes:  lambda_i = a_i / (d * 2^shift)  (mod p), with
 * |a_i| held in a_limbs little-endian u32 limbs and the sign in bit i of `neg`.
 * The division by d is
 *   has_inv == 0: none (d == 1);
 *   has_inv == 1: a multiplication by inv = d^{-1} mod p (full width);
 *   has_inv == 2: an exact division by the small odd d (3 <= d < 2^16): the
 *                 kernel adds m*p (m = -r * p^{-1} mod d, from r mod d via the
 *                 residues w[i] = 2^(32 i) mod d and the reciprocal d_recip =
 *                 floor((2^64-1)/d)) and divides limb by limb with d_inv32 =
 *                 d^{-1} mod 2^32 — about a fifth of the full product's work.
 * When the exact rationals do not fit, the generic form is used:
 * a_i = lambda_i mod p (a_limbs = 17), has_inv = 0, shift = 0.
 */
typedef struct dn_m521_lagrange {
  int32_t k;                             /* number of shares, 1..16            */
  int32_t a_limbs;                       /* 1, 2 or 17                         */
  uint32_t neg;                          /* bit i set: a_i is negative         */
  int32_t shift;                         /* 0..31: final division by 2^shift   */
  int32_t has_inv;                       /* 0, 1 (multiply by inv), 2 (exact /d) */
  uint32_t d;                            /* odd part of the denominator        */
  uint32_t a[DN_MAX_RESOLVE][DN_M521_LIMBS];
  uint32_t inv[DN_M521_LIMBS];           /* has_inv == 1: d^{-1} mod p         */
  uint32_t d_inv32;                      /* has_inv == 2: d^{-1} mod 2^32      */
  uint32_t p_inv_d;                      /* has_inv == 2: p^{-1} mod d         */
  uint64_t d_recip;                      /* has_inv == 2: floor((2^64-1)/d)    */
  uint32_t w[DN_M521_LIMBS];             /* has_inv == 2: 2^(32 i) mod d       */
  uint32_t reserved;
} dn_m521_lagrange_t;

/* Host.  Validates like shamir.py:70-75 (k < threshold -> DN_ERR_TOO_FEW,
 * duplicate x -> DN_ERR_DISTINCT, k == 1 -> DN_ERR_EMPTY) and fills *out.
 * Replaces the weight computation of shamir.py:77-89 and op.py:4-29. */
int dn_m521_lagrange(const uint64_t* xs, int k, int threshold, dn_m521_lagrange_t* out);

/*
 * Reconstruct: out_e = sum_i lambda_i * y_{i,e} mod p, canonical — the value
 * `resolve_shares` returns (shamir.py:90) as an integer; ALL k shares are used
 * (shamir.py:76-89), so inconsistent shares give the degree-(k-1) interpolant.
 *   share_vecs    host array of k device pointers, each a tiled vector
 *   out_fe        device tiled vector, or NULL
 *   out_u64       device int64[n_elem] (low 64 bits of the result), or NULL
 *   overflow_count device uint32 counter, incremented (atomically) once per
 *                 element whose result is >= 2^64; may be NULL
 * Replaces shamir.py:68-90.
 */
int dn_m521_reconstruct(const void* const* share_vecs, const dn_m521_lagrange_t* w,
                        void* out_fe, int64_t* out_u64, uint32_t* overflow_count,
                        uint64_t n_elem, void* stream);

/*
 * Host.  Draw the reference's coefficients with CPython's MT19937 semantics:
 * for each element e (in order) and j = 1..t-1, c = randint(1, p-1) =
 * 1 + getrandbits(521) rejected while >= p-1 (17 MT words, little-endian, last
 * word >> 23) — exactly the calls shamir.py:59-61 makes on `self.random`.
 *   mt_state  624 MT words (random.getstate()[1][:624]), updated in place
 *   mt_index  the position (getstate()[1][624]), updated in place
 *   coeffs    HOST block of t-1 tiled vectors (t-1 == tm1), written
 */
int dn_mt19937_draw_coeffs(uint32_t* mt_state, int32_t* mt_index, uint64_t n_elem,
                           int tm1, void* coeffs);

/*
 * The same draw, bit-exact, entirely on the GPU (csrc/mt19937_device.hip):
 * the MT window at the start of every 17*2^14-word substream by jump-ahead
 * kernels (at most three levels of independent jumps), then one wave per
 * substream runs MT19937 from its window.  `coeffs` is a DEVICE block of t-1
 * tiled vectors, `scratch` device memory of
 * dn_mt19937_device_scratch_bytes(n, t-1) bytes.  Synchronises `stream`.  On
 * DN_OK the state is advanced exactly as the host draw advances it.
 * DN_ERR_RETRY (a draw >= p-1 was seen: later words shift, odds ~2^-520 per
 * coefficient) and DN_ERR_UNSUPPORTED (more than 262144 substreams) leave the
 * state untouched: draw on the host instead.
 */
uint64_t dn_mt19937_device_scratch_bytes(uint64_t n_elem, int tm1);
int dn_mt19937_draw_coeffs_device(uint32_t* mt_state, int32_t* mt_index, uint64_t n_elem, int tm1,
                                  void* coeffs, void* scratch, uint64_t scratch_bytes, void* stream);

/*
 * make_shares over a vector with the reference's own coefficients, fused:
 * the device draw above feeding dn_m521_split_u64 in registers — each
 * substream's wave draws the coefficients of 64 consecutive elements at a
 * time and writes their n shares, so the coefficient block never reaches
 * memory (8 + 66 n bytes of HBM per element instead of 8 + 66 n + 4 * 66
 * (t - 1)).  Same results and final MT state as dn_mt19937_draw_coeffs_device
 * followed by dn_m521_split_u64.  Scratch: dn_mt19937_device_scratch_bytes(n, t-1).
 * DN_ERR_UNSUPPORTED: t not in {2, 3, 5} or n too large for forward
 * differences (use the draw and the split); DN_ERR_RETRY as above (the shares
 * are then incomplete: redo the draw on the host and split).
 * Replaces per element: shamir.py:55-66 (make_shares) with :59-61's draws.
 *
 * Both device draws speculate on a loop of equal draws (DN_MT_SPEC, on by
 * default): from the second of two calls of one size a call also computes,
 * on a library-owned side stream and buffer, the jump windows of a next draw
 * of the same size starting where this one ends, and a next call whose size,
 * index and 624-word array match uses them instead of jumping (no visible
 * difference but time; any mismatch is a miss).  The side work holds two
 * library-owned buffers of dn_mt19937_device_scratch_bytes per device.
 */
int dn_mt19937_split_device(uint32_t* mt_state, int32_t* mt_index, const int64_t* secrets, void* shares,
                            uint64_t n_elem, int threshold, int n_shares, void* scratch, uint64_t scratch_bytes,
                            void* stream);

/*
 * 1 when dn_mt19937_split_device takes (n_elem, threshold, n_shares) — t in
 * {2, 3, 5}, t <= n_shares, forward differences without folding, the stream
 * within the jump table — else 0 (draw, then split).  No allocation, no
 * device call: lets a caller skip the fused form's scratch allocation when
 * the call would return DN_ERR_UNSUPPORTED.
 */
int dn_mt19937_split_supported(uint64_t n_elem, int threshold, int n_shares);

/*
 * Host.  The byte API for one secret per call (csrc/host_shamir.cpp), the way
 * the reference's callers use it (runner/horizontal/agg.py:142-153,
 * coord/horizontal/agg.py:296,330,362), in any prime field (shamir.py:49-51).
 *   prime_be / prime_len  big-endian p; NULL or 2^521 - 1 takes the fixed
 *                         9 x 64-bit Mersenne path
 *
 * make_shares (shamir.py:55-66, _eval_at :19-25, _share_to_bytes :28-33):
 *   value / value_len     coefficient 0 as the caller's bytes (bytes_to_int)
 *   coeffs_be             t-1 coefficients, coeff_bytes big-endian bytes each
 *   out, out_cap          records [len(x)][x][y] back to back, capacity
 *                         >= n_shares * (9 + len(p)); offsets[n_shares + 1]
 * DN_ERR_THRESHOLD if t > n_shares.
 *
 * resolve_shares (shamir.py:68-90, _bytes_to_share :36-45, op.py:4-29):
 *   shares, offsets       k records back to back, offsets[k + 1]
 *   out, out_cap, out_len the secret, minimal big-endian
 * DN_ERR_TOO_FEW / DN_ERR_DISTINCT / DN_ERR_EMPTY as dn_m521_lagrange;
 * DN_ERR_ZERODIV / DN_ERR_ASSERT where op.inverse_mod raises.
 */
int dn_shamir_make_shares_host(const uint8_t* value, uint64_t value_len, const uint8_t* coeffs_be,
                               uint32_t coeff_bytes, int threshold, const uint8_t* prime_be, uint32_t prime_len,
                               uint64_t n_shares, uint8_t* out, uint64_t out_cap, uint64_t* offsets);
int dn_shamir_resolve_shares_host(const uint8_t* shares, const uint64_t* offsets, int k, int threshold,
                                  const uint8_t* prime_be, uint32_t prime_len, uint8_t* out, uint64_t out_cap,
                                  uint64_t* out_len);

/*
 * Host.  `_eval_at(coeffs, x, prime)` (shamir.py:19-25) for any integers, the
 * general case the device split does not take (another prime, x outside
 * 1..65535, more than 64 coefficients, negative operands): Horner from the
 * top with Python's `value %= prime` after every step.  Coefficient j is
 * bytes coeff_offsets[j] .. coeff_offsets[j+1] of coeffs_be (magnitude, big
 * endian) with sign coeff_neg[j] (NULL: all non-negative); x and prime are
 * magnitude + sign likewise.  The result (sign of the modulus, as Python) is
 * written minimal big-endian to out, its sign to *out_neg.  n_coeffs == 0
 * gives 0 (the reference's loop never runs); prime == 0 with coefficients is
 * DN_ERR_ZERODIV, as Python's `%`.
 */
int dn_shamir_eval_at_host(const uint8_t* coeffs_be, const uint64_t* coeff_offsets, const uint8_t* coeff_neg,
                           int n_coeffs, const uint8_t* x_be, uint32_t x_len, int x_neg, const uint8_t* prime_be,
                           uint32_t prime_len, int prime_neg, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
                           int* out_neg);

/*
 * Host.  Opt-in share-block allocator (csrc/vmm_block.cpp): `bytes` of device
 * memory on `device` built from physical chunks of chunk_bytes (rounded up to
 * the allocation granularity; 0 = 2 MiB) mapped back to back into one
 * reserved virtual range.  The split's rate depends on the physical pages of
 * its share block; this lets a caller choose the block's
 * composition.  dn_block_free waits for the events the block's uses recorded
 * (dn_block_record; a block with none recorded: everything queued on its own
 * device), then unmaps and releases every chunk; the block's virtual range
 * stays reserved for the life of the process (a new block mapped at a freed
 * block's address had its bytes change under later allocations: DESIGN.md
 * §5.2).  Every other entry point keeps taking caller-owned memory from any
 * allocator.  The returned shares belong to the caller
 * (delta_node/crypto/shamir/shamir.py:62-66), so a pooled block is handed to
 * a new owner only once its last owner's work is ordered before the new
 * owner's:
 *   dn_block_record   record an event on `stream` for the block (call it for
 *                     every stream that used the block, when the block goes idle)
 *   dn_block_ready    *ready = 1 when every recorded event is on `stream` or
 *                     has completed (the block may be used on `stream` now)
 *   dn_block_acquire  hand the block to work on `stream`: wait = 0 fails with
 *                     DN_ERR_RETRY while another stream's event is pending
 *                     (and then changes nothing); wait = 1 makes `stream` wait
 *                     for those events (no host wait)
 *   dn_block_retired_bytes  virtual address space retired so far by frees and
 *                     failed allocations (the caller's budget for new blocks)
 */
int dn_block_granularity(int device, uint64_t* bytes);
int dn_block_alloc(uint64_t bytes, uint64_t chunk_bytes, int device, void** ptr);
int dn_block_free(void* ptr);
int dn_block_record(void* ptr, void* stream);
int dn_block_ready(void* ptr, void* stream, int* ready);
int dn_block_acquire(void* ptr, void* stream, int wait);
int dn_block_retired_bytes(uint64_t* bytes);

/*
 * Device, async on `stream`.  Zero `rows` rows of `row_bytes` (whole
 * 16896-byte tiles) at `ptr` in the order a split writes a share block (per
 * tile, every row's slice): the allocator times it to judge a new block's
 * placement (memory.share_block).
 */
int dn_block_probe_rows(void* ptr, uint32_t rows, uint64_t row_bytes, void* stream);

/*
 * Host.  Advance a CPython MT19937 state by `words` 32-bit outputs (as
 * `words` getrandbits(32) calls would) by jump-ahead instead of stepping.
 */
int dn_mt19937_skip(uint32_t* mt_state, int32_t* mt_index, uint64_t words);

/*
 * Host, diagnostic.  1 when the library's build-time table of MT19937 jump
 * rows (the 2^24-draw direct level) is present and passes its checks —
 * checksum, tabulated rows, recurrence — so a first draw uses it; 0 when the
 * rows would be computed at run time instead.
 */
int dn_mt19937_rt_rows_embedded(void);

/*
 * The current device's draw speculation counters: out[0] calls that used
 * speculated windows, out[1] speculations the next call did not match,
 * out[2] speculations launched, out[3] 1 while one is armed.  (Diagnostics for
 * tests and the bench; no reference counterpart.)
 */
int dn_mt19937_spec_stats(uint64_t* out);

/*
 * The MT19937 jump polynomial of `words` words: out[312] = x^words mod P (P
 * the characteristic polynomial of the one-word transition; the window after
 * `words` words is out(f) applied to the window).  The speculated next draw's
 * start window is jumped to by it.  DN_ERR_UNSUPPORTED on a host without
 * carry-less multiply.  (No reference counterpart: random.Random advances word
 * by word.)
 */
int dn_mt19937_jump_poly(uint64_t words, uint64_t* out);

/*
 * Share wire codec over whole vectors (shamir.py:28-45 `_share_to_bytes` /
 * `_bytes_to_share`, serialize/hex.py:44-50).  Record e of the packed stream
 * is exactly the reference's bytes for share (x, y_e):
 *     [len(xb)][xb][yb],  xb / yb minimal big-endian (0 -> empty)
 * and records are back to back: record e = out[offsets[e] : offsets[e+1]].
 */
/* Device scratch bytes dn_m521_encode_shares needs for n elements. */
uint64_t dn_m521_codec_scratch_bytes(uint64_t n_elem);
/* Upper bound of the packed size (n * (1 + len(xb) + 66)): size `out` to this. */
uint64_t dn_m521_encoded_capacity(uint64_t n_elem, uint64_t x);
/* Encode share x of a tiled vector: device uint64 offsets[n+1], device out
 * (capacity >= dn_m521_encoded_capacity), device scratch. */
int dn_m521_encode_shares(const void* vec, uint64_t n_elem, uint64_t x, uint64_t* offsets, uint8_t* out,
                          uint64_t capacity, void* scratch, uint64_t scratch_bytes, void* stream);
/* Decode records (device in[in_bytes], offsets[n+1]) into a tiled vector, y
 * reduced mod p as resolve_shares does; xs (device uint64[n], may be NULL)
 * receives each record's x.  Records with x longer than 8 bytes or y longer
 * than 68 significant bytes, and records whose offsets are decreasing or run
 * past in_bytes (offsets come from the wire), are counted in *bad_count
 * (device) and decoded as 0; nothing outside in[0, in_bytes) is read. */
int dn_m521_decode_shares(const uint8_t* in, uint64_t in_bytes, const uint64_t* offsets, uint64_t n_elem, void* vec,
                          uint64_t* xs, uint32_t* bad_count, void* stream);

/* Thread-local message of the last failure (never NULL). */
const char* dn_last_error(void);

/* Library version string. */
const char* dn_version(void);

#ifdef __cplusplus
}
#endif

#endif /* DN_SHAMIR_H */
