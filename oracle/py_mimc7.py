"""Pure-Python restatement of the reference MiMC7 commitments — TEST INFRASTRUCTURE ONLY.

Reference: delta_node/utils/mimc7.py:18-92 (gmpy2 arithmetic; gmpy2 is not
installed here, so this restatement uses Python ints) with the field and
round constants of delta_node/utils/constant.py:6-30 (the BN254 scalar field
and 13 MiMC7 round constants, the first 0 — circomlib's mimc7 constants).
Pinned by the reference's own known-answer tests (tests/mimc7_test.py:5-97,
values in tests/golden/mimc7_kat.json): tests/test_mimc7.py.
"""
from __future__ import annotations

import math
from typing import Iterable, List

Q = 21888242871839275222246405745257275088548364400416034343698204186575808495617
CTS = [
    0,
    20888961410941983456478427210666206549300505294776164667214940546594746570981,
    15265126113435022738560151911929040668591755459209400716467504685752745317193,
    8334177627492981984476504167502758309043212251641796197711684499645635709656,
    1374324219480165500871639364801692115397519265181803854177629327624133579404,
    11442588683664344394633565859260176446561886575962616332903193988751292992472,
    2558901189096558760448896669327086721003508630712968559048179091037845349145,
    11189978595292752354820141775598510151189959177917284797737745690127318076389,
    3262966573163560839685415914157855077211340576201936620532175028036746741754,
    17029914891543225301403832095880481731551830725367286980611178737703889171730,
    4614037031668406927330683909387957156531244689520944789503628527855167665518,
    19647356996769918391113967168615123299113119185942498194367262335168397100658,
    5040699236106090655289931820723926657076483236860546282406111821875672148900,
]
DATA_BLOCK = 128


def mimc7_hash(x: int, key: int) -> int:
    """mimc7.py:18-27 — NB the result r + k is not reduced."""
    r = x
    for c in CTS:
        r = pow((r + key + c) % Q, 7, Q)
    return r + key


def mimc7_hash_arr(xs: List[int], key: int) -> int:
    """mimc7.py:30-36."""
    r = key
    for x in xs:
        r = (r + x + mimc7_hash(x, r)) % Q
    return r


def float2int(x: float, precision: int = 8) -> int:
    """mimc7.py:39-44: min(a, q - a) with a = int(x * 10^precision)."""
    a = int(x * (10 ** precision))
    return min(a, Q - a)


def merkle(xs: List[int], key: int, min_size: int = 2) -> int:
    """mimc7.py:47-55."""
    n = len(xs)
    assert n % 2 == 0
    if n == min_size:
        return mimc7_hash_arr(xs, key)
    return mimc7_hash_arr([merkle(xs[: n // 2], key, min_size), merkle(xs[n // 2:], key, min_size)], key)


def int_to_bytes(v: int) -> bytes:
    return v.to_bytes((v.bit_length() + 7) // 8, "big")


def weight_commitment(weight: Iterable[float]) -> bytes:
    """mimc7.py:58-60."""
    return int_to_bytes(mimc7_hash_arr([float2int(w, 8) for w in weight], 2))


def data_row_hashes(data) -> List[int]:
    """mimc7.py:63-85: rows -> field ints (features at 10^8, label at 10^21),
    padded with zero rows to a multiple of 128, each row chained with key 2."""
    rows = []
    for row in data:
        row = list(row)
        rows.append([float2int(v, 8) for v in row[:-1]] + [float2int(row[-1], 21)])
    cols = len(rows[0])
    pad = math.ceil(len(rows) / DATA_BLOCK) * DATA_BLOCK - len(rows)
    rows += [[0] * cols] * pad
    return [mimc7_hash_arr(r, 2) for r in rows]


def data_commitment(data) -> List[bytes]:
    """mimc7.py:63-92."""
    h = data_row_hashes(data)
    return [int_to_bytes(merkle(h[s:s + DATA_BLOCK], 2)) for s in range(0, len(h), DATA_BLOCK)]
