#!/usr/bin/env python3
"""Known-answer keystreams for the ChaCha20 block function of dn_m521_split_prng.

Generated with OpenSSL's `enc -chacha20` (an implementation independent of this
repo): encrypting zeros yields the keystream.  OpenSSL's 16-byte IV is the
state's words 12..15 (block counter word 12, then three nonce words); the
device stream uses words 12-13 as a 64-bit counter and 14-15 as a 64-bit
nonce, so IV = le64(counter) || le64(nonce) as long as the low counter word
does not wrap inside one request.  Output: chacha_kat.json.
"""
import json
import os
import struct
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def keystream(key: bytes, counter: int, nonce: int, nblocks: int) -> bytes:
    iv = struct.pack("<QQ", counter, nonce)
    r = subprocess.run(["openssl", "enc", "-chacha20", "-K", key.hex(), "-iv", iv.hex(), "-nosalt"],
                       input=bytes(64 * nblocks), capture_output=True, check=True)
    return r.stdout


def main():
    cases = []
    keys = [bytes(range(32)), bytes(32), bytes([0xFF] * 32), bytes((7 * i + 3) & 0xFF for i in range(32))]
    for ki, key in enumerate(keys):
        for counter, nonce in [(0, 0), (1, 0x4a00000009000000), (0x1234, 0xDEADBEEFCAFEF00D),
                               ((1 << 62) + 5, 77), ((1 << 63) + (9 << 6), 1), (0xFFFFFFF0 - 4, 3)]:
            ks = keystream(key, counter, nonce, 4)
            cases.append({"key": key.hex(), "counter": counter, "nonce": nonce,
                          "words": list(struct.unpack("<64I", ks))})
    # RFC 8439 §2.3.2's block: key 00..1f, block count 1, nonce 00000009 0000004a 00000000
    # (words 13, 14, 15) -> serialized output begins 10 f1 e7 e4.
    rfc_counter, rfc_nonce = 1 | (0x09000000 << 32), 0x4a000000
    ks = keystream(bytes(range(32)), rfc_counter, rfc_nonce, 1)
    assert ks[:4] == bytes.fromhex("10f1e7e4"), ks[:4].hex()
    cases.append({"key": bytes(range(32)).hex(), "counter": rfc_counter, "nonce": rfc_nonce,
                  "words": list(struct.unpack("<16I", ks)), "rfc8439_2_3_2": True})
    with open(os.path.join(HERE, "chacha_kat.json"), "w") as f:
        json.dump({"source": "openssl enc -chacha20 (OpenSSL 3.0.2), 4 blocks per case", "cases": cases}, f)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
