"""Device-PRNG coefficient stream (dn_m521_split_prng): the C restatement
oracle/chacha_oracle.c against OpenSSL's ChaCha20 keystream
(tests/golden/chacha_kat.json, make_golden_chacha.py) and against the
coefficient definition restated in plain Python."""
import json
import os

import numpy as np

from golden.fixtures import HERE, P
from oracle import c_oracle

KAT = json.load(open(os.path.join(HERE, "chacha_kat.json")))


def test_chacha_block_matches_openssl():
    assert any(c.get("rfc8439_2_3_2") for c in KAT["cases"])
    for c in KAT["cases"]:
        key = bytes.fromhex(c["key"])
        words = np.array(c["words"], dtype=np.uint32)
        for b in range(len(words) // 16):
            got = c_oracle.chacha_block(key, c["counter"] + b, c["nonce"])
            assert np.array_equal(got, words[16 * b:16 * b + 16]), (c["counter"], b)


def _py_coeff(key, nonce, i):
    low = c_oracle.chacha_block(key, i, nonce)
    top = int(c_oracle.chacha_block(key, (1 << 62) + i // 16, nonce)[i % 16]) & 0x1FF
    v = sum(int(w) << (32 * k) for k, w in enumerate(low)) | (top << 512)
    assert v < P - 1  # the retry domain is taken with odds 2^-520
    return v + 1


def test_prng_coeffs_definition_and_offsets():
    key = bytes((5 * i + 1) & 0xFF for i in range(32))
    tm1, n, off = 2, 40, 1000
    co = c_oracle.prng_coeffs(key, 9, off, n, tm1)
    for e in range(n):
        for j in range(tm1):
            v = sum(int(w) << (32 * k) for k, w in enumerate(co[e, j]))
            assert v == _py_coeff(key, 9, (off + e) * tm1 + j)
            assert 1 <= v <= P - 1
    # shard independence: the stream of element g does not depend on where a call starts
    assert np.array_equal(c_oracle.prng_coeffs(key, 9, off + 7, 5, tm1), co[7:12])
    # different nonces / rounds give different streams
    assert not np.array_equal(c_oracle.prng_coeffs(key, 10, off, n, tm1), co)
    assert not np.array_equal(c_oracle.prng_coeffs(key, 9, off, n, tm1, rounds=12), co)
