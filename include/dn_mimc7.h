/*
 * dn_mimc7.h — C-ABI of the MiMC7 commitment row:
 * the hlr verify path's data / weight commitments over the BN254 scalar field.
 *
 * Reference interface replaced (delta-mpc/delta-node):
 *   mimc7_hash(x, key)               delta_node/utils/mimc7.py:18-27
 *   mimc7_hash_arr(xs, key)          mimc7.py:30-36
 *   _float2mpz(x, precision)         mimc7.py:39-44
 *   merkle_mimc7_hash_arr            mimc7.py:47-55
 *   calc_weight_commitment(weight)   mimc7.py:58-60
 *   calc_data_commitment(data)       mimc7.py:63-92
 *   q, cts, data_block_size          utils/constant.py:6-30
 * Field elements are 8 little-endian u32 limbs (plain integers, not
 * Montgomery form).  Same conventions as dn_shamir.h.
 */
#ifndef DN_MIMC7_H
#define DN_MIMC7_H

#include <stdint.h>

#include "dn_shamir.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Row hashes of calc_data_commitment: data is device float64 [rows][cols]
 * (last column the label, converted at 10^21, the others at 10^8); rows are
 * padded with zero rows to a multiple of 128.  row_hashes: device
 * uint32 [round_up(rows,128)][8] = mimc7_hash_arr(row, 2) (mod q).  Values
 * with |v * 10^p| >= 2^253 are counted in *bad_count (device) — not handled. */
int dn_mimc7_data_rows(const double* data, uint64_t rows, int cols, uint32_t* row_hashes, uint32_t* bad_count,
                       void* stream);

/* Merkle root of each block of 128 leaves (merkle_mimc7_hash_arr(block, 2)):
 * leaves device uint32 [blocks*128][8], roots device uint32 [blocks][8]. */
int dn_mimc7_merkle_blocks(const uint32_t* leaves, uint64_t blocks, uint32_t* roots, void* stream);

/* calc_weight_commitment's chain mimc7_hash_arr([_float2mpz(w, p) ...], 2) of
 * device float64 w[n]; out: device uint32[8].  One sequential chain (each
 * hash is keyed by the previous result): a single lane, latency-bound. */
int dn_mimc7_weight_chain(const double* w, uint64_t n, int precision, uint32_t* out, uint32_t* bad_count,
                          void* stream);

/* calc_weight_commitment (mimc7.py:58-60) on the calling host core: w is
 * HOST float64 [n]; out: host uint32[8] = the commitment as a plain field
 * element.  The chain is strictly sequential (52 dependent field products
 * per weight), so it runs where a dependent product is cheapest; exact
 * _float2mpz for every finite double; NaN -> DN_ERR_ARG (ValueError),
 * +-inf -> DN_ERR_OVERFLOW (OverflowError), as int() raises in mimc7.py:41.
 * This is the path calc_weight_commitment takes; dn_mimc7_weight_chain is the
 * single-lane device form of the same chain (kept for device-resident data). */
int dn_mimc7_weight_commitment_host(const double* w, uint64_t n, int precision, uint32_t* out);

/* Field parameters of utils/constant.py:6-30 as plain 8-limb integers:
 * q[8] and cts[13][8] (host memory). */
int dn_mimc7_params(uint32_t* q, uint32_t* cts);

/* Batched mimc7_hash(x_i, key_i) for plain field elements (< q): out is
 * device uint32 [n][9] holding the unreduced r + key (< 2q), as mimc7.py:26. */
int dn_mimc7_hash(const uint32_t* xs, const uint32_t* keys, uint64_t n, uint32_t* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DN_MIMC7_H */
