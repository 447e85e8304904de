#!/usr/bin/env python3
"""Known-answer AES-CTR vectors for the share envelope (crypto/aes/aes.py:8-23).

Generated with OpenSSL's `enc -aes-{128,192,256}-ctr` — the library the
reference's `cryptography` package wraps (absent here), independent of this
repo: ciphertexts of seeded random plaintexts for several keys, counter
blocks (among them ones whose low 64 bits or all 128 bits wrap inside the
message) and lengths (0..3 blocks and ragged sizes).  Output: aes_kat.json.
"""
import json
import os
import random
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def ctr(key: bytes, iv: bytes, pt: bytes) -> bytes:
    r = subprocess.run(["openssl", "enc", f"-aes-{8 * len(key)}-ctr", "-K", key.hex(), "-iv", iv.hex(), "-nosalt"],
                       input=pt, capture_output=True, check=True)
    return r.stdout


def main():
    rng = random.Random(2024)
    ivs = [bytes(16), bytes(range(0xF0, 0x100)), bytes(8) + b"\xff" * 7 + b"\xfe", b"\xff" * 16,
           b"\xff" * 15 + b"\xfd", bytes(rng.randrange(256) for _ in range(16))]
    cases = []
    for kb in (16, 24, 32):
        for ki in range(2):
            key = bytes(rng.randrange(256) for _ in range(kb)) if ki else bytes(range(kb))
            for iv in ivs:
                for n in (0, 1, 16, 17, 48, 100, 257):
                    pt = bytes(rng.randrange(256) for _ in range(n))
                    cases.append({"key": key.hex(), "iv": iv.hex(), "pt": pt.hex(), "ct": ctr(key, iv, pt).hex()})
    ver = subprocess.run(["openssl", "version"], capture_output=True, text=True, check=True).stdout.strip()
    with open(os.path.join(HERE, "aes_kat.json"), "w") as f:
        json.dump({"source": f"openssl enc -aes-*-ctr ({ver})", "cases": cases}, f)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
