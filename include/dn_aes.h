/*
 * dn_aes.h — C-ABI of the share envelope (second
 * half): AES-CTR + base64 (+ hex) of whole messages on MI355X.
 *
 * Reference interface replaced (delta-mpc/delta-node):
 *   aes.encrypt(key, data)       delta_node/crypto/aes/aes.py:8-14
 *       b64encode(nonce + Cipher(AES(key), CTR(nonce)).encryptor().update(data)),
 *       nonce = os.urandom(16)
 *   aes.decrypt(key, data)       delta_node/crypto/aes/aes.py:17-23
 *   serialize.bytes_to_hex / hex_to_bytes   delta_node/serialize/hex.py:11-41,
 *       the JSON form of upload_secret_shares (runner/horizontal/commu.py:23-49,
 *       app/v1/coord.py:93-94 "0x[0-9a-fA-F]+")
 * `cryptography`'s CTR mode (OpenSSL): the nonce is a 128-bit big-endian
 * counter block, incremented per 16-byte block modulo 2^128.  Keys of 16, 24
 * or 32 bytes (AES-128/192/256; the runner's ECDH keys are 32,
 * crypto/ecdhe/ecdhe.py:23-34).
 *
 * Same conventions as dn_shamir.h, except that `key`, `iv` / `nonce` are HOST
 * pointers (a few bytes).  Data pointers are caller-owned device buffers;
 * inputs may start at any byte, outputs must be 16-byte aligned.
 */
#ifndef DN_AES_H
#define DN_AES_H

#include <stddef.h>
#include <stdint.h>

#include "dn_shamir.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Host.  FIPS-197 key expansion: 4 (rounds + 1) big-endian words into rk[60],
 * *rounds = 10 / 12 / 14.  Other key sizes: DN_ERR_ARG, "Invalid key size
 * (<bits>) for AES." (cryptography's message). */
int dn_aes_expand_key(const uint8_t* key, int key_bytes, uint32_t* rk, int32_t* rounds);

/* out[i] = in[i] ^ keystream[i], keystream block b = AES(key, iv + b):
 * Cipher(AES(key), CTR(iv)).encryptor().update(in) (aes.py:10-12), either
 * direction.  out may equal in. */
int dn_aes_ctr(const uint8_t* key, int key_bytes, const uint8_t* iv, const void* in, void* out, uint64_t n,
               void* stream);

/* Length of encrypt's text: base64 of 16 + n bytes, doubled when hex != 0. */
uint64_t dn_aes_encrypt_len(uint64_t n, int hex);

/* aes.encrypt(key, in[0..n)) with the given 16-byte nonce: out = base64 of
 * nonce || ct, or (hex != 0) its lowercase hex — serialize.bytes_to_hex
 * without the "0x", which the caller writes in front.  out holds
 * dn_aes_encrypt_len(n, hex) bytes. */
int dn_aes_encrypt(const uint8_t* key, int key_bytes, const uint8_t* nonce, const void* in, uint64_t n, void* out,
                   int hex, void* stream);

/* Largest plaintext dn_aes_decrypt can produce from n_text characters; 0 when
 * the length is not canonical (base64 length not a multiple of 4, odd hex,
 * or shorter than the 24 characters of a nonce) — such text is parsed on the
 * host with the reference's calls. */
uint64_t dn_aes_decrypt_capacity(uint64_t n_text, int hex);

/* aes.decrypt of canonical base64 text (hex != 0: of its hex digits, without
 * "0x"; upper or lower case).  Device outputs: *out_len = plaintext bytes;
 * *bad (zeroed here) != 0 when a character is outside the alphabet or '=' is
 * misplaced — out is then invalid and the caller parses the text on the host.
 * DN_ERR_RETRY when dn_aes_decrypt_capacity(n_text, hex) == 0. */
int dn_aes_decrypt(const uint8_t* key, int key_bytes, const void* text, uint64_t n_text, int hex, void* out,
                   uint64_t capacity, uint64_t* out_len, uint32_t* bad, void* stream);

/* ---- host (the byte API: aes.encrypt / aes.decrypt of one share) ----------
 * The reference seals each ~70-byte share with its own call
 * (runner/horizontal/agg.py:192-196, decrypt at :258 / :265); these run on the
 * calling core (AES-NI when the CPU has it, else T-tables) with the same
 * schedule, counter convention and text as the device entry points above.
 * All pointers are HOST pointers. */

/* dn_aes_ctr on the host: out[i] = in[i] ^ keystream[i] (aes.py:10-12). */
int dn_aes_ctr_host(const uint8_t* key, int key_bytes, const uint8_t* iv, const void* in, void* out, uint64_t n);

/* dn_aes_encrypt on the host (aes.py:8-14 with the given nonce): out holds
 * dn_aes_encrypt_len(n, hex) bytes. */
int dn_aes_encrypt_host(const uint8_t* key, int key_bytes, const uint8_t* nonce, const void* in, uint64_t n,
                        void* out, int hex);

/* dn_aes_decrypt on the host (aes.py:17-23) of canonical base64 (hex != 0: of
 * its hex digits, without "0x"): *out_len = plaintext bytes.  DN_ERR_RETRY
 * when the text is not canonical (the caller parses it with the reference's
 * own calls and uses dn_aes_ctr_host). */
int dn_aes_decrypt_host(const uint8_t* key, int key_bytes, const void* text, uint64_t n_text, int hex, void* out,
                        uint64_t capacity, uint64_t* out_len);

/* dn_aes_expand_key with a tabulated S-box (the byte API expands the peer's
 * key on every call): the same words. */
int dn_aes_expand_key_host(const uint8_t* key, int key_bytes, uint32_t* rk, int32_t* rounds);

/* 1 when the host cipher uses AES-NI, 0 for the table cipher. */
int dn_aes_host_impl(void);

#ifdef __cplusplus
}
#endif

#endif /* DN_AES_H */
