/*
 * dn_mask.h — C-ABI of the mask-PRG row: the
 * reference's secure-aggregation masks and fixed-point masking on MI355X.
 *
 * Reference interface replaced (delta-mpc/delta-node):
 *   utils.make_mask(seed, shape)          delta_node/utils/arr.py:20-28
 *       np.random.default_rng(seed or list(seed_bytes))
 *         .integers(0, 2**47 - 1, size=shape, dtype=np.int64)
 *   utils.fix_precision / unfix_precision delta_node/utils/precision.py:5-15
 *   ClientAggregator.mask_result          runner/horizontal/agg.py:284-318
 *       fix_precision(val) + seed_mask + sum(+-mask(shared_key))
 *   unmask loop                           coord/horizontal/agg.py:381-404
 * The generator is numpy's (requirements.txt pins numpy): SeedSequence
 * (bit_generator.pyx) -> PCG64 (pcg64.h, XSL-RR 128/64) -> Generator.integers
 * int64 path (_bounded_integers.pyx -> distributions.c bounded_lemire_uint64).
 *
 * Same conventions as dn_shamir.h: plain pointers, caller-owned device
 * buffers, asynchronous on `stream`, 0 or a negative DN_ERR_* code.
 */
#ifndef DN_MASK_H
#define DN_MASK_H

#include <stddef.h>
#include <stdint.h>

#include "dn_shamir.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DN_MASK_MAX_GENS 16

/* A PCG64 generator: 128-bit state and increment (numpy's PCG64.state). */
typedef struct dn_pcg64 {
  uint64_t state_hi, state_lo;
  uint64_t inc_hi, inc_lo;
} dn_pcg64_t;

/* Host.  numpy `PCG64(SeedSequence(entropy))`: entropy as uint32 words
 * (a bytes seed contributes one word per byte, an int seed its 32-bit words,
 * little-endian — SeedSequence's _coerce_to_uint32_array).  Replaces the
 * `np.random.default_rng(...)` of arr.py:21-24. */
int dn_pcg64_seed(const uint32_t* entropy, int n_words, dn_pcg64_t* out);

/* Host.  Advance a generator by `delta` draws (numpy PCG64.advance). */
int dn_pcg64_advance(dn_pcg64_t* g, uint64_t delta);

/*
 * Fused bounded-integer accumulation (the masking hot loop):
 *   out[e] = base[e] + sum_g sign_g * (low + L_g(e + raw_offset_g))
 * for e in [elem_begin, elem_end), int64 arithmetic modulo 2^64 (numpy's
 * wrap-around), where L_g(r) is the Lemire bounded value numpy draws from
 * generator g's r-th raw 64-bit output:  high 64 bits of x * (rng + 1).
 *   rng       high - 1 - low, must be > 2^32 - 1 (numpy's 64-bit path;
 *             make_mask: low 0, rng 2^47 - 2)
 *   base      int64 base_i64, or float64 base_f64 converted like
 *             fix_precision (x * 10^precision, truncated, NaN/out of range ->
 *             INT64_MIN as numpy's x86 cast), or neither (zero)
 *   signs     +1 / -1 per generator
 *   reject_count  device uint32[ngen] (zeroed by the caller): becomes non-zero
 *             iff some raw draw of generator g in the range is REJECTED by
 *             Lemire's test (low word < threshold; odds 2^-47 per draw for
 *             make_mask).  The value above equals numpy's only when it stays
 *             0; otherwise the caller replays that generator exactly with
 *             per-segment raw offsets (dn_bounded_i64_rejects) — the Python
 *             layer does this automatically.
 * Replaces arr.py:26 (and the mask sums of agg.py:284-318 / 381-404).
 */
int dn_bounded_i64_accumulate(const dn_pcg64_t* gens, const int32_t* signs, const uint64_t* raw_offsets,
                              int ngen, int64_t low, uint64_t rng, const int64_t* base_i64,
                              const double* base_f64, int precision, int64_t* out, uint64_t elem_begin,
                              uint64_t elem_end, uint32_t* reject_count, void* stream);

/* List the rejected raw draws of one generator in [raw_begin, raw_end):
 * device uint64 out_idx[capacity], device uint32 *count (atomically
 * incremented; entries past `capacity` are counted but not written). */
int dn_bounded_i64_rejects(const dn_pcg64_t* gen, uint64_t rng, uint64_t raw_begin, uint64_t raw_end,
                           uint64_t* out_idx, uint32_t* count, uint32_t capacity, void* stream);

/* Masked-result sum over members (reference
 * coord/horizontal/agg.py:227-251 make_masked_results: result += val):
 * out[e] = sum_j inputs[j][e], int64 modulo 2^64.  1 <= k <= 16 device
 * pointers (16-byte aligned); out may alias inputs[0]. */
int dn_i64_sum(const int64_t* const* inputs, int k, int64_t* out, uint64_t n, void* stream);

/* unfix_precision: out[e] = (double)in[e] / 10^precision (precision.py:12-15). */
int dn_unfix_precision(const int64_t* in, double* out, uint64_t n, int precision, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DN_MASK_H */
